#!/bin/bash
# compiler scheduling strategies for the kernels: gcn-max-ilp (ilp) and latency-weighted
# (schedule-metric-bias 0, bias0) vs the shipped build (r5c): C4, then C5 (group kernel)
set -o pipefail
O=gpurun_out/sched; mkdir -p $O
bash tools/ab_libs.sh $O/c4 r5c ilp bias0 > /dev/null 2>&1 || exit 1
cat $O/c4/ab.txt
bash tools/ab_cfgs.sh $O/c5 "r5c ilp bias0" "500:500:1048576" > /dev/null 2>&1 || exit 1
cat $O/c5/ab.txt
