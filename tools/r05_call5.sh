#!/bin/bash
# round 5, GPU call 5: the lane path's early exit -- parity suite, then A/B bench against round 4's main kernel
O=gpurun_out/r05c5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
for v in new old new old; do
  if [ $v = old ]; then L=somatic-sniper_amd/build/libsniper_amd_r04main.so; else L=somatic-sniper_amd/libsniper_amd.so; fi
  SNIPER_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-pmc --no-cpu --no-host-fed \
    --strong-steps 0 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json;r=json.load(open('$O/ab_$v.json'));print('$v', r['value'], r['roofline']['avg_ms_by_kernel'])" | tee -a $O/ab.txt
done
for cfg in "500 500 1048576" "1200 1000 262144" "30 30 67108864" "100 60 33554432"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload shard --lt $1 --ln $2 --sites $3 --steps 10 --warmup 2 --no-pmc \
    --no-cpu --no-host-fed > $O/cfg_$1_$2.json 2> $O/cfg_$1_$2.err || { tail -20 $O/cfg_$1_$2.err; exit 1; }
  python -c "import json;r=json.load(open('$O/cfg_$1_$2.json'));print('$1x$2', r['value'], r['roofline']['avg_ms_by_kernel'])" | tee -a $O/ab.txt
done
