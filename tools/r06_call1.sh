#!/bin/bash
# round 6, call 1: quick parity of the fixed tree, the early-exit / host-path
# tests, the deep kernel on record (3000x/3000x, 2100x/100x) and C5 with its
# kernel trace (timer reconciliation), plus a C4 shard timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06c1"
O=$R/gpurun_out/r06c1
timeout -k 10 300 python3 -u "$R/tools/quick_parity.py" > "$O/qp.log" 2>&1 && tail -n 1 "$O/qp.log" &&
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    "$R/tests/test_gpu_parity.py" -k "all_reference or early_exit or host" > "$O/pytest_subset.log" 2>&1 && tail -n 2 "$O/pytest_subset.log" &&
bash "$R/tools/r06_cfg.sh" r06c1/deep "d3000 3000 3000 262144 cpu" "d2100 2100 100 262144 cpu" "c5 500 500 1048576 nocpu" &&
timeout -k 10 200 python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --no-host-fed --steps 10 --warmup 2 --sites 67108864 > "$O/c4shard.json" 2>&1 && tail -n 1 "$O/c4shard.json" | cut -c1-400
