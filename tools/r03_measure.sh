#!/bin/bash
# Round-3 measurement pass on the GPU box (through gpurun):
#   1. the default bench line (C4 workload) with its live PMC passes and CPU baselines
#   2. rocprofv3 --kernel-trace --stats of a short run of the same workload
set -euo pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"
tail -c 600 "$O/bench.json"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-pmc --weak-sites 0 > "$O/kt.log" 2>&1
echo done
