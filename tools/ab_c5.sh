#!/bin/bash
# Same-box C5 A/B at the profile size (500x/500x, 2^20 sites): each library twice, alternating.
#   bash tools/ab_c5.sh LIB_A LIB_B     (through gpurun; paths relative to the repo root)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/ab"
for rep in 1 2; do
  for L in "$@"; do
    SNIPER_AMD_LIB=$R/$L timeout -k 10 200 python "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 10 --warmup 2 --lt 500 --ln 500 --sites 1048576 \
        > "$R/gpurun_out/ab/c5_${rep}_$(basename $L).log" 2>&1 || { echo "$L failed"; exit 1; }
    echo "$L rep $rep $(python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.4e sites/s, wide %.3f ms' % (r['value'], r['roofline']['avg_ms_by_kernel']['wide']))" "$R/gpurun_out/ab/c5_${rep}_$(basename $L).log")"
  done
done
