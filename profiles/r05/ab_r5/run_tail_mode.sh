#!/bin/bash
# key build: the tail flag as an SGPR integer (tl), and the key build instantiated per tail mode so
# the common path's chunk loads carry no per-load test (tk) vs the shipped build
set -o pipefail
O=gpurun_out/tk; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_tk.so timeout -k 10 300 python -u tools/quick_parity.py > $O/qp.txt 2>&1 || { tail -20 $O/qp.txt; exit 1; }
tail -1 $O/qp.txt
bash tools/ab_libs.sh $O/c4 cur tl tk > /dev/null 2>&1 || exit 1
cat $O/c4/ab.txt
bash tools/ab_cfgs.sh $O/cfg "cur tk" "30:30:67108864 100:60:33554432" > /dev/null 2>&1 || exit 1
cat $O/cfg/ab.txt
