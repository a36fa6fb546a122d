#!/bin/bash
# round-5 closing measurements, part 1: the full GPU suite on the tree, then the default bench
# line (PMC, CPU baselines, host-fed) and its rocprofv3 kernel-trace summary
set -o pipefail
O=gpurun_out/r05final4; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
bash tools/profile_round.sh r05final4
