#!/bin/bash
# quick_parity for several variant libraries (build/libsniper_amd_<V>.so)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/qp"
for V in "$@"; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  SNIPER_AMD_LIB=$L timeout -k 10 200 python "$R/tools/quick_parity.py" > "$R/gpurun_out/qp/$V.log" 2>&1 || { echo "$V run failed"; exit 1; }
  echo "$V $(tail -n 1 $R/gpurun_out/qp/$V.log)"
done
