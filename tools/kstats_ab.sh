#!/bin/bash
# Per-kernel average durations (rocprofv3 kernel trace) of bench.py for each
# variant library build/libsniper_amd_<V>.so; LT/LN select the depth config.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  O=$R/gpurun_out/kstats/$V
  mkdir -p "$O"
  SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_$V.so timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run -- \
    python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 5 --warmup 2 --lt ${LT:-500} --ln ${LN:-500} --sites ${SITES:-262144} \
    > "$O/bench.log" 2>&1 || { echo "$V failed"; exit 1; }
  S=$(find "$O" -name '*kernel_stats.csv' | head -1)
  echo "== $V $(grep '^{"metric"' $O/bench.log | python3 -c 'import json,sys; print("%.3e sites/s" % json.loads(sys.stdin.read())["value"])')"
  python3 - "$S" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "ss_" in r["Name"]:
        print(f'  {r["Name"][:40]:40s} calls {r["Calls"]:>4s}  avg {float(r["AverageNs"])/1e3:9.1f} us  total {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
done
