#!/bin/bash
# Collects the round's measurements on the GPU box (run through gpurun):
#   1. the default bench line                           -> gpurun_out/<tag>/bench.json
#   2. rocprofv3 --kernel-trace --stats of a short bench -> gpurun_out/<tag>/kt/
#   3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE)  -> gpurun_out/<tag>/pmc_*/
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 420 python bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu > "$O/kt.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o run -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$O/pmc_$c.log" 2>&1
done
echo done
