#!/bin/bash
# group kernel: own-reads-only loads (gclamp); units of ceil(n/128) lanes packed densely, bpermute merges
# (dense); + chunks dealt round-robin over a unit's lanes (ilv); main kernel: the three small fold chains walked together (fold3; g3 = gclamp + fold3,
# dense3 = dense + fold3).  Parity of dense3, then A/B lines.
set -o pipefail
O=gpurun_out/dense; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_dense3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity_dense3.log 2>&1 || { tail -30 $O/pytest_parity_dense3.log; exit 1; }
tail -2 $O/pytest_parity_dense3.log
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_ilv.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "group or wide or routing or deep" > $O/pytest_parity_ilv.log 2>&1 || { tail -30 $O/pytest_parity_ilv.log; exit 1; }
tail -2 $O/pytest_parity_ilv.log
for v in base5 dense ilv; do
  L=somatic-sniper_amd/build/libsniper_amd_$v.so
  for c in "500 500 1048576" "1200 1000 262144"; do
    set -- $c
    SNIPER_AMD_LIB=$L timeout -k 10 400 python -u bench.py --workload shard --lt $1 --ln $2 --sites $3 --steps 10 --warmup 2 \
      --no-cpu --no-host-fed --strong-steps 0 > $O/b_${v}_$1.json 2> $O/b_${v}_$1.err || { tail -20 $O/b_${v}_$1.err; exit 1; }
    python3 -c "import json;r=json.load(open('$O/b_${v}_$1.json'));f=r['roofline'];print('$v $1', '%.4g'%r['value'], f['avg_ms_by_kernel'], f.get('traffic_over_algorithmic'), f.get('traffic_bytes_per_site'), f.get('valu',{}).get('insts_per_site'))" | tee -a $O/ab.txt
  done
done
bash tools/ab_libs.sh $O/c4 base5 g3 || exit 1
bash tools/ab_cfgs.sh $O/cfg "base5 g3" "30:30:67108864" || exit 1
