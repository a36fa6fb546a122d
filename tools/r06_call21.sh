#!/bin/bash
# Round 6: the full GPU suite and smoke() on the current tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c21
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
    > "$O/pytest_gpu.log" 2>&1; rc=$?
tail -25 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
tail -3 "$O/smoke.log"
exit $rc
