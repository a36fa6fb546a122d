#!/bin/bash
# Timing A/B of the deep kernel: ss_score_deep time per launch for each
# build/libsniper_amd_<V>.so at two deep-panel depths (all sites > 2048 slots).
#   bash tools/abdeep.sh V1 V2 ...      (through gpurun)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/ab"
for V in "$@"; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  for cfg in "1200 1000 65536" "3000 3000 16384"; do
    set -- $cfg
    out=$R/gpurun_out/ab/deep_${V}_$1.log
    SNIPER_AMD_LIB=$L timeout -k 10 200 python "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 10 --warmup 2 \
        --lt "$1" --ln "$2" --sites "$3" > "$out" 2>&1 || { echo "$V $1 timing failed"; exit 1; }
    echo "$V ${1}x/${2}x $3 sites: $(python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e sites/s, deep %.3f ms' % (r['value'], r['roofline']['avg_ms_by_kernel']['deep']))" "$out")"
  done
done
