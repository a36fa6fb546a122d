#!/bin/bash
# Round 6: group / deep kernels without per-wave first atomics -- parity of the
# kernels that changed, then a same-box A/B against the previous commit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c37
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "deep or group or wide or near_exit_deep or routing or mixed" > "$O/pytest.log" 2>&1; rc=$?
tail -3 "$O/pytest.log"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest.log" | head; exit $rc; }
LIBS="base prev" CFGS="c5:500:500:1048576 d1200:1200:1000:262144 d3000:3000:3000:262144 c3:100:60:33554432" bash tools/r06_ab.sh
