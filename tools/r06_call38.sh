#!/bin/bash
# Round 6 close: the full GPU suite and smoke() on the shipped tree, then a
# same-box A/B of the static-first-chunk patch (build/libsniper_amd_sfc.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c38
mkdir -p "$O"
cd "$R"
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 \
    > "$O/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest_gpu.log" | head; exit $rc; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
tail -2 "$O/smoke.log"
[ $rc -eq 0 ] || exit $rc
LIBS="base sfc" CFGS="c5:500:500:1048576 d1200:1200:1000:262144" bash tools/r06_ab.sh
