#!/bin/bash
# One rocprofv3 --pmc pass per argument (a space-separated counter list) over a
# short shard-workload bench; per-kernel sums into gpurun_out/pmc/<i>.txt
#   bash tools/pmc_probe.sh "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_IFETCH"
#   PMC_SITES=262144 PMC_ARGS="--lt 500 --ln 500" bash tools/pmc_probe.sh ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$O/p$i" -o run -- \
      python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 3 --warmup 1 --sites ${PMC_SITES:-4194304} ${PMC_ARGS:-} \
      > "$O/p$i.log" 2>&1 || { echo "pass $i ($ctrs) failed"; tail -5 "$O/p$i.log"; exit 1; }
  python3 - "$O/p$i" "$ctrs" > "$O/$i.txt" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"][:40], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); cnt[k] += 1
for (kn, c), v in sorted(tot.items()):
    if "ss_score" in kn:
        print(f"{kn:40s} {c:28s} {v:16.4e}  per-dispatch-row mean {v / cnt[(kn, c)]:.4e}")
PY
  echo "== $ctrs"; cat "$O/$i.txt"
done
