#!/bin/bash
# A/B of library builds on one box (GPU): tools/ab_libs.sh OUTDIR V1 V2 ... ; V = a name of
# somatic-sniper_amd/build/libsniper_amd_V.so, or "cur" for somatic-sniper_amd/libsniper_amd.so.
# Default C4 bench (20 steps, no PMC / CPU / host-fed), each variant twice, interleaved.
O=$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = cur ]; then L=somatic-sniper_amd/libsniper_amd.so; else L=somatic-sniper_amd/build/libsniper_amd_$v.so; fi
    SNIPER_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-pmc --no-cpu --no-host-fed \
      --strong-steps 0 > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { tail -20 $O/ab_${v}_$rep.err; exit 1; }
    python -c "import json;r=json.load(open('$O/ab_${v}_$rep.json'));print('$v', r['value'], r['roofline']['avg_ms_by_kernel'])" | tee -a $O/ab.txt
  done
done
