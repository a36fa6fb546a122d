#!/bin/bash
# round 6, call 11: main kernel routes samples past SS_ROUTE_DEEP reads to the deep kernel;
# parity of the shipped build, then the routing threshold A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c11
mkdir -p "$O"
timeout -k 10 300 python3 -u "$R/tools/quick_parity.py" > "$O/qp.log" 2>&1 || exit 1; tail -n 1 "$O/qp.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    "$R/tests/test_gpu_parity.py" > "$O/pytest_parity.log" 2>&1; rc=$?; tail -n 2 "$O/pytest_parity.log"
[ $rc -eq 0 ] || exit 1
bash "$R/tools/r06_route_ab.sh" r06c11 base route640 route800 route2048
