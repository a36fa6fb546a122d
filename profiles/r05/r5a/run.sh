#!/bin/bash
# the adopted round-5 kernels (fold3 + dense interleaved group units): full GPU suite, then the
# deep configurations with PMC traffic, base5 (round-5 start) vs the tree
set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
for v in base5 cur; do
  if [ $v = cur ]; then L=somatic-sniper_amd/libsniper_amd.so; else L=somatic-sniper_amd/build/libsniper_amd_$v.so; fi
  for c in "500 500 1048576" "1200 1000 262144"; do
    set -- $c
    SNIPER_AMD_LIB=$L timeout -k 10 400 python -u bench.py --workload shard --lt $1 --ln $2 --sites $3 --steps 10 --warmup 2 \
      --no-cpu --no-host-fed --strong-steps 0 > $O/b_${v}_$1.json 2> $O/b_${v}_$1.err || { tail -20 $O/b_${v}_$1.err; exit 1; }
    python3 -c "import json;r=json.load(open('$O/b_${v}_$1.json'));f=r['roofline'];print('$v $1', '%.4g'%r['value'], f['avg_ms_by_kernel'], f.get('traffic_over_algorithmic'), f.get('traffic_bytes_per_site'), f.get('valu',{}).get('insts_per_site'))" | tee -a $O/ab.txt
  done
done
