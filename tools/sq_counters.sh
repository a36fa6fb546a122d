#!/bin/bash
# SQ instruction-mix / stall counters of the scoring kernels (one PMC pass per
# group) on bench.py's own batch (--pmc-child: the bench's batch 0 scored 3x).
#   bash tools/sq_counters.sh [TAG] [LT] [LN] [SITES]      (through gpurun)
set -euo pipefail
TAG=${1:-sq}; LT=${2:-60}; LN=${3:-30}; SITES=${4:-16777216}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$O/pass$i" -o run -- \
      python3 "$R/bench.py" --pmc-child --workload shard --sites "$SITES" --lt "$LT" --ln "$LN" > "$O/pass$i.log" 2>&1
  python3 "$R/tools/pmc_kernels.py" "$O/pass$i" --sites "$SITES"
done
