#!/bin/bash
# main kernel: the long chains' full steps as a guarded do-while (the wave-uniform step
# counter in an SGPR, no loop-carried copies) with idle lanes parked in fk's zeroed upper
# half (dw) vs the shipped build: quick parity, then C4 and C2-like A/B
set -o pipefail
O=gpurun_out/dw; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_dw.so timeout -k 10 300 python -u tools/quick_parity.py > $O/qp.txt 2>&1 || { tail -20 $O/qp.txt; exit 1; }
tail -3 $O/qp.txt
bash tools/ab_libs.sh $O/c4 cur dw > /dev/null 2>&1 || exit 1
cat $O/c4/ab.txt
bash tools/ab_cfgs.sh $O/cfg "cur dw" "30:30:67108864 100:60:33554432" > /dev/null 2>&1 || exit 1
cat $O/cfg/ab.txt
