#!/bin/bash
# experiment: group kernel with mirror stages without the pad substitution when no unit of the batch has virtual lanes vs the
# closing round-5 kernels (r5c): group-path parity, then C5 / 1200x1000 lines
set -o pipefail
O=gpurun_out/nopad; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_nopad.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "group or wide or routing or deep" > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
for rep in 1 2; do
for v in r5c nopad; do
  for c in "500 500 1048576" "1200 1000 262144"; do
    set -- $c
    SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_$v.so timeout -k 10 400 python -u bench.py --workload shard --lt $1 --ln $2 --sites $3 --steps 10 --warmup 2 \
      --no-cpu --no-host-fed --no-pmc --strong-steps 0 > $O/b_${v}_$1_$rep.json 2> $O/b_${v}_$1_$rep.err || { tail -20 $O/b_${v}_$1_$rep.err; exit 1; }
    python3 -c "import json;r=json.load(open('$O/b_${v}_$1_$rep.json'));f=r['roofline'];print('$v $1', '%.4g'%r['value'], f['avg_ms_by_kernel'])" | tee -a $O/ab.txt
  done
done
done
