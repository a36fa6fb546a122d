#!/usr/bin/env python3
"""Per-site SQ counters of ss_score_main from tools/ablate_pmc.sh output."""
import collections
import csv
import re
import sys

run, masks = sys.argv[1], [int(x) for x in sys.argv[2].split(",")]
S = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 22
rows = list(csv.DictReader(open(f"{run}/pmc/run_counter_collection.csv")))
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if re.search(r"ss_score_main[<(]", r["Kernel_Name"]):
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ks = sorted(d)
for i, m in enumerate(masks):
    c = d[ks[3 * i + 2]]
    print(f"mask {m:3d}: " + "  ".join(f"{k.replace('SQ_', '').lower()} {v / S:7.1f}" for k, v in sorted(c.items())))
