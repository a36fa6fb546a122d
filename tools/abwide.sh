#!/bin/bash
# Wide-kernel timing A/B: sites/s at high depth for each build/libsniper_amd_<V>.so
# (DEPTHS="lt/ln ..." default "450/450 500/500"), no parity (run tools/ab.sh for that).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/ab"
for V in "$@"; do
  line="$V"
  for D in ${DEPTHS:-450/450 500/500}; do
    L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
    SNIPER_AMD_LIB=$L timeout -k 10 200 python "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 5 --warmup 2 \
      --lt ${D%/*} --ln ${D#*/} --sites 262144 > "$R/gpurun_out/ab/w_${V}_${D%/*}.log" 2>&1 || { echo "$V $D timing failed"; exit 1; }
    line="$line | $D $(python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=r['roofline']['avg_ms_by_kernel']; print('%.3e sites/s (wide %.3f deep %.3f ms)' % (r['value'], k['wide'], k['deep']))" $R/gpurun_out/ab/w_${V}_${D%/*}.log)"
  done
  echo "$line"
done
