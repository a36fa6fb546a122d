#!/bin/bash
# A/B of library builds across depth configurations (GPU): tools/ab_cfgs.sh OUTDIR "V1 V2 .." [CFGS]
# V = name of somatic-sniper_amd/build/libsniper_amd_V.so or "cur"; CFGS = "lt:ln:sites ..."
O=$1; VS=$2; CFGS=${3:-"60:30:67108864 30:30:67108864 100:60:33554432"}
mkdir -p $O
for rep in 1 2; do
 for c in $CFGS; do
  IFS=: read lt ln n <<< "$c"
  for v in $VS; do
    if [ $v = cur ]; then L=somatic-sniper_amd/libsniper_amd.so; else L=somatic-sniper_amd/build/libsniper_amd_$v.so; fi
    SNIPER_AMD_LIB=$L timeout -k 10 300 python -u bench.py --workload shard --lt $lt --ln $ln --sites $n --steps 10 \
      --warmup 2 --no-pmc --no-cpu --no-host-fed > $O/r_${v}_${lt}_${ln}.json 2> $O/r_${v}_${lt}_${ln}.err \
      || { tail -20 $O/r_${v}_${lt}_${ln}.err; exit 1; }
    python -c "import json;r=json.load(open('$O/r_${v}_${lt}_${ln}.json'));print('$v ${lt}x${ln}', r['value'], r['roofline']['avg_ms_by_kernel']['main'])" | tee -a $O/ab.txt
  done
 done
done
