#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C4 bench's own launches only (no host-fed sub-line), so
# the summary's ss_score_main average is the same launch mix as the bench line's HIP-event average
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05kt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_c4" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-pmc --no-host-fed --strong-steps 0 > "$O/kt_c4.log" 2>&1 || exit 1
echo done
