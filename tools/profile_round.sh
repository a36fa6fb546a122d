#!/bin/bash
# Collects the round's measurements on the GPU box (run through gpurun):
#   1. the default bench line (its own live PMC passes: traffic, VALU)  -> gpurun_out/<tag>/bench.json
#   2. rocprofv3 --kernel-trace --stats of a short bench                 -> gpurun_out/<tag>/kt/
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=${1:-r02}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-pmc --no-host-fed --strong-steps 0 "$@" > "$O/kt.log" 2>&1
echo done
