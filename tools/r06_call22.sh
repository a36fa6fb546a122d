#!/bin/bash
# Round 6: A/B of triage-kernel variants at C4 (default c4 workload), quick parity of each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c22
mkdir -p "$O"
cd "$R"
for v in ${AB:-cur}; do
  [ $v = cur ] && continue
  SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -k "near_exit or synthetic_parity" > "$O/pytest_$v.log" 2>&1 || { echo "parity $v FAILED"; tail -5 "$O/pytest_$v.log"; }
  echo "parity $v: $(tail -1 "$O/pytest_$v.log")"
done
timeout -k 10 900 bash tools/ab_libs.sh "$O/ab" ${AB:-cur}
