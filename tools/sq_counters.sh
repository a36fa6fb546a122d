#!/bin/bash
# SQ instruction-mix / stall counters of ss_score_main (one PMC pass per group).
set -euo pipefail
TAG=${1:-sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$O/counters_list.txt" 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$O/pass$i" -o run -- \
      python3 "$R/tools/ablate.py" --masks 0 --reps 2 > "$O/pass$i.log" 2>&1
done
echo done
