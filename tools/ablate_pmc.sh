#!/bin/bash
# Instruction counts per ablation mask (SS_DIAG) of ss_score_main.
set -euo pipefail
TAG=${1:-abl}
MASKS=${2:-0,1,2,4,8,16,32,64,128,255}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    --output-format csv -d "$O/pmc" -o run -- \
    python3 "$R/tools/ablate.py" --masks "$MASKS" --reps 1 > "$O/ablate.log" 2>&1
timeout -k 10 300 python3 "$R/tools/ablate.py" --masks "$MASKS" --reps 5 > "$O/ablate_time.log" 2>&1
echo done
