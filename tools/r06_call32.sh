#!/bin/bash
# Round 6: what bounds the deep triage at 500x/500x -- instruction mix, wait
# and busy counters, texture address / data units.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
PMC_SITES=1048576 PMC_ARGS="--lt 500 --ln 500" timeout -k 10 600 bash tools/pmc_probe.sh \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
  "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
  "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
  "TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum" 2>&1 | grep -v "ss_score_main\|ss_score_group\|ss_score_deep(\|ss_score_wild"
