#!/bin/bash
# the main kernel's early exit for shallow blocks (ee72: blocks of <= 72 reads per site on average):
# parity (scores with and without glf), then A/B against the committed kernels (r5a) across depths
set -o pipefail
O=gpurun_out/ee72; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_ee72.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
bash tools/ab_libs.sh $O/c4 r5a ee72 || exit 1
bash tools/ab_cfgs.sh $O/cfg "r5a ee72" "30:30:67108864 40:30:67108864 45:25:67108864 100:60:33554432" || exit 1
