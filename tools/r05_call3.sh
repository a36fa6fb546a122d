#!/bin/bash
# round 5, GPU call 3: the whole GPU suite on this tree
O=gpurun_out/r05c3; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
exit $rc
