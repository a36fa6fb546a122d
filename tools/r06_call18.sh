#!/bin/bash
# Round 6: where the triage kernel waits -- the address / L1 / L2 counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c18
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$O/list.txt" 2>&1
grep -oE "\b(TA|TD|TCP|TCC)_[A-Z0-9_]+" "$O/list.txt" | sort -u > "$O/names.txt"
wc -l "$O/names.txt"
cd "$R"
PMC_SITES=16777216 timeout -k 10 600 bash tools/pmc_probe.sh \
  "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
  "TCC_HIT_sum TCC_MISS_sum" \
  "TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum"
