#!/bin/bash
# Round-3 measurement pass on the GPU box (through gpurun):
#   1. the default bench line (C4 workload) with its live PMC passes and CPU baselines
#   2. rocprofv3 --kernel-trace --stats of a short run of the same workload
#   3. per-phase cycle stamps of the main kernel (SS_STAMP variant library)
set -euo pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"
tail -c 600 "$O/bench.json"
if [ -f somatic-sniper_amd/build/libsniper_amd_stamp.so ]; then
  SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_stamp.so timeout -k 10 120 python tools/stamps.py \
      > "$O/stamps.txt" 2>&1
  cat "$O/stamps.txt"
fi
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-pmc > "$O/kt.log" 2>&1
echo done
