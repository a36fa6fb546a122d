#!/bin/bash
# separate-mode tumor pass no longer over-fetches the normal's reads (solo) vs the committed
# kernels (r5b): parity, C3 with PMC traffic, C4 A/B
set -o pipefail
O=gpurun_out/solo; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_solo.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
for v in r5b solo; do
  SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_$v.so timeout -k 10 400 python -u bench.py --workload shard --lt 100 --ln 60 --sites 33554432 --steps 10 --warmup 2 \
    --no-cpu --no-host-fed --strong-steps 0 > $O/b_${v}_c3.json 2> $O/b_${v}_c3.err || { tail -20 $O/b_${v}_c3.err; exit 1; }
  python3 -c "import json;r=json.load(open('$O/b_${v}_c3.json'));f=r['roofline'];print('$v c3', '%.4g'%r['value'], f['avg_ms_by_kernel'], f.get('traffic_over_algorithmic'), f.get('traffic_bytes_per_site'), f.get('valu',{}).get('insts_per_site'))" | tee -a $O/ab.txt
done
bash tools/ab_libs.sh $O/c4 r5b solo || exit 1
bash tools/ab_cfgs.sh $O/cfg "r5b solo" "100:60:33554432" || exit 1
