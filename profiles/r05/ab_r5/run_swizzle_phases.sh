#!/bin/bash
# LUT rows XOR-swizzled (swz) vs the committed kernels (r5a): parity, C4 A/B, deep configs with
# PMC; then group-kernel phase ablations at C5 on the swz source (timing only)
set -o pipefail
O=gpurun_out/swz; mkdir -p $O
SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_swz.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "synthetic or group or routing" > $O/pytest_parity_swz.log 2>&1 || { tail -30 $O/pytest_parity_swz.log; exit 1; }
tail -n 1 $O/pytest_parity_swz.log
bash tools/ab_libs.sh $O/c4 r5a swz || exit 1
for c in "500 500 1048576" "1200 1000 262144"; do
  set -- $c
  SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_swz.so timeout -k 10 400 python -u bench.py --workload shard --lt $1 --ln $2 --sites $3 --steps 10 --warmup 2 \
    --no-cpu --no-host-fed --strong-steps 0 > $O/b_swz_$1.json 2> $O/b_swz_$1.err || { tail -20 $O/b_swz_$1.err; exit 1; }
  python3 -c "import json;r=json.load(open('$O/b_swz_$1.json'));f=r['roofline'];print('swz $1', '%.4g'%r['value'], f['avg_ms_by_kernel'], f.get('traffic_over_algorithmic'), f.get('traffic_bytes_per_site'), f.get('valu',{}).get('insts_per_site'))" | tee -a $O/ab.txt
done
bash tools/c5_phases.sh swz a_gnosort a_gnomerge a_gnorec a_gnofold a_gnofin a_noload > $O/c5_phases.txt 2>&1 || { cat $O/c5_phases.txt; exit 1; }
cat $O/c5_phases.txt
