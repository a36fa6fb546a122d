#!/bin/bash
# round 6, call 14: deep kernel with run lists in an L2-resident global buffer, 16 waves per CU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c14
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    "$R/tests/test_gpu_parity.py" -k "quirk_parity or giant or deep or wide_sample or routing or unit_boundaries" > "$O/pytest_deep.log" 2>&1; rc=$?; tail -n 2 "$O/pytest_deep.log"
[ $rc -eq 0 ] || exit 1
SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_alldeep.so timeout -k 10 300 python3 -u "$R/tools/quick_parity.py" > "$O/qp_alldeep.log" 2>&1 || exit 1; tail -n 1 "$O/qp_alldeep.log"
bash "$R/tools/r06_abdeep.sh" r06c14 alldeep
