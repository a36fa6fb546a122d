#!/bin/bash
# round 5, GPU call 7: refill-round early exit -- parity, then A/B against round 4's main kernel
O=gpurun_out/r05c7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_multi_rank.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_cfgs.sh $O "rf1 r04main"
