#!/bin/bash
# round 6 measurements: the default C4 bench line (driver's command) with its
# rocprofv3 kernel-trace summary, then the per-configuration lines (C2, C3, C5,
# 1200x/1000x, 3000x/3000x, 2100x/100x) with theirs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06final}
O=$R/gpurun_out/$TAG
mkdir -p "$O/c4"
export TMPDIR=/tmp
# a heartbeat under gpurun_out/ (the long bench steps print only at their end)
(while true; do date >> "$O/heartbeat"; sleep 50; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/c4/bench.json" 2> "$O/c4/bench.err" || exit 1
tail -n 1 "$O/c4/bench.json" | cut -c1-300
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c4/kt" -o run -- \
    python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu --no-host-fed --strong-steps 0 > "$O/c4/kt.log" 2>&1) || exit 1
bash "$R/tools/r06_cfg.sh" $TAG/configs "c2 30 30 67108864 cpu" "c3 100 60 33554432 cpu" "c5 500 500 1048576 cpu" \
    "d1200 1200 1000 262144 nocpu" "d3000 3000 3000 262144 nocpu" "d2100 2100 100 262144 nocpu"
