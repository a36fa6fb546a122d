#!/bin/bash
# main kernel records: every register converted and every row written, without the per-register /
# per-row wave-uniform skips (rc) vs the shipped build: quick parity, C4, C2 / C3
set -o pipefail
O=gpurun_out/rc; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_rc.so timeout -k 10 300 python -u tools/quick_parity.py > $O/qp.txt 2>&1 || { tail -20 $O/qp.txt; exit 1; }
tail -1 $O/qp.txt
bash tools/ab_libs.sh $O/c4 cur rc > /dev/null 2>&1 || exit 1
cat $O/c4/ab.txt
bash tools/ab_cfgs.sh $O/cfg "cur rc" "30:30:67108864 100:60:33554432" > /dev/null 2>&1 || exit 1
cat $O/cfg/ab.txt
