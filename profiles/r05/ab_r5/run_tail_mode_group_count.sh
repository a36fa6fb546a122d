#!/bin/bash
# the per-tail-mode instantiation extended to the group kernel's key build and the early exit's
# count pass (tg) vs the shipped build: quick parity, C5 / 1200x1000 / C2, C4
set -o pipefail
O=gpurun_out/tg; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_tg.so timeout -k 10 300 python -u tools/quick_parity.py > $O/qp.txt 2>&1 || { tail -20 $O/qp.txt; exit 1; }
tail -1 $O/qp.txt
bash tools/ab_cfgs.sh $O/cfg "cur tg" "500:500:1048576 1200:1000:262144 30:30:67108864" > /dev/null 2>&1 || exit 1
cat $O/cfg/ab.txt
bash tools/ab_libs.sh $O/c4 cur tg > /dev/null 2>&1 || exit 1
cat $O/c4/ab.txt
