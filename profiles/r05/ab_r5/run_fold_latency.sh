#!/bin/bash
# timing ablations: the fold's float chains split in two (fdep: main kernel, C4; gfdep: group
# kernel, C5) vs the shipped build -- does the fold wait on its own serial f64 latency?
set -o pipefail
O=gpurun_out/fdep; mkdir -p $O
bash tools/ab_libs.sh $O/c4 cur fdep > /dev/null 2>&1 || exit 1
cat $O/c4/ab.txt
bash tools/ab_cfgs.sh $O/c5 "cur gfdep" "500:500:1048576" > /dev/null 2>&1 || exit 1
cat $O/c5/ab.txt
