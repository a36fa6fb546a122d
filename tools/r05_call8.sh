#!/bin/bash
# depth-ordered tiles: parity, then A/B against the round-5 baseline build
set -o pipefail
O=gpurun_out/dsort; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -3 $O/pytest_parity.log
bash tools/ab_libs.sh $O base5 dsort || exit 1
bash tools/ab_cfgs.sh $O/cfg "base5 dsort" "30:30:67108864 100:60:33554432 500:500:1048576" || exit 1
