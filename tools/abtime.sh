#!/bin/bash
# Timing-only A/B (ablation builds whose results are deliberately wrong):
# main-kernel time at 60x/30x for each build/libsniper_amd_<V>.so, no parity.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/ab"
for V in "$@"; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  SNIPER_AMD_LIB=$L timeout -k 10 200 python "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 10 --warmup 2 --sites 16777216 > "$R/gpurun_out/ab/tt_$V.log" 2>&1 || { echo "$V timing failed"; exit 1; }
  echo "$V main $(python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e sites/s, %.3f ms' % (r['value'], r['roofline']['avg_ms_by_kernel']['main']))" $R/gpurun_out/ab/tt_$V.log)"
done
