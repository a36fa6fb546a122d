#!/usr/bin/env python3
"""Per-kernel mean counters (per dispatch, and per site when --sites is given)
from a rocprofv3 --pmc run directory (run_counter_collection.csv)."""
import argparse
import collections
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--sites", type=float, default=0)
ap.add_argument("--match", default="ss_score")
a = ap.parse_args()
path = a.csv if a.csv.endswith(".csv") else os.path.join(a.csv, "run_counter_collection.csv")
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"]
    if a.match not in k:
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, c in acc.items():
    n = len(disp[k])
    per = f" per site" if a.sites else " per dispatch"
    print(f"{k[:60]:60s} dispatches {n}{per}: " +
          "  ".join(f"{x.replace('SQ_', '').lower()} {v / n / (a.sites or 1):.1f}" for x, v in sorted(c.items())))
