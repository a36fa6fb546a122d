#!/bin/bash
# bar_e: the near-integer test as one |fr - 0.5| compare whose mask is the ballot, and bar_e
# computed for every lane (no branch on c2) -- "be" vs the shipped build: quick parity, C4, C5
set -o pipefail
O=gpurun_out/be; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_be.so timeout -k 10 300 python -u tools/quick_parity.py > $O/qp.txt 2>&1 || { tail -20 $O/qp.txt; exit 1; }
tail -2 $O/qp.txt
bash tools/ab_libs.sh $O/c4 cur be > /dev/null 2>&1 || exit 1
cat $O/c4/ab.txt
bash tools/ab_cfgs.sh $O/cfg "cur be" "500:500:1048576 30:30:67108864" > /dev/null 2>&1 || exit 1
cat $O/cfg/ab.txt
