#!/bin/bash
# VALU instructions per site of ss_score_main for each variant library (one
# rocprofv3 --pmc pass each, SQ_INSTS_VALU + SQ_INSTS_SALU + SQ_INSTS_LDS + SQ_WAVE_CYCLES):
#   bash tools/sq_variants.sh V1 V2 ...        (through gpurun)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sqv
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
for V in "$@"; do
  SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_$V.so timeout -s KILL 120 rocprofv3 \
      --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d "$O/$V" -o run -- \
      python3 "$R/bench.py" --pmc-child --workload shard --sites 16777216 > "$O/$V.log" 2>&1 || { echo "$V failed"; exit 1; }
  echo "$V $(python3 "$R/tools/pmc_kernels.py" "$O/$V" --sites 16777216 --match ss_score_main)"
done
