#!/bin/bash
# A/B: quick parity + main-kernel time for each variant library build/libsniper_amd_<V>.so
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/ab"
for V in "$@"; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  if [ -n "${AB_NOPARITY:-}" ]; then echo "(ablation: no parity)" > "$R/gpurun_out/ab/qp_$V.log"; else
  SNIPER_AMD_LIB=$L timeout -k 10 200 python "$R/tools/quick_parity.py" > "$R/gpurun_out/ab/qp_$V.log" 2>&1 || { echo "$V parity run failed"; exit 1; }
  fi
  if [ -n "${AB_NOMAIN:-}" ]; then echo '{"value": 0, "roofline": {"avg_ms_by_kernel": {"main": 0}}}' > "$R/gpurun_out/ab/t_$V.log"; else
  SNIPER_AMD_LIB=$L timeout -k 10 200 python "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 10 --warmup 2 --sites 16777216 > "$R/gpurun_out/ab/t_$V.log" 2>&1 || { echo "$V timing failed"; exit 1; }
  fi
  if [ -n "${AB_NOC5:-}" ]; then echo '{"value": 0}' > "$R/gpurun_out/ab/t5_$V.log"; else
  SNIPER_AMD_LIB=$L timeout -k 10 200 python "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 5 --warmup 2 --lt ${C5_LT:-500} --ln ${C5_LN:-500} --sites 262144 > "$R/gpurun_out/ab/t5_$V.log" 2>&1 || { echo "$V C5 timing failed"; exit 1; }
  fi
  echo "$V $(tail -n 1 $R/gpurun_out/ab/qp_$V.log) main $(python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e sites/s, %.3f ms' % (r['value'], r['roofline']['avg_ms_by_kernel']['main']))" $R/gpurun_out/ab/t_$V.log) | C5 $(python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e' % r['value'], r.get('roofline', {}).get('avg_ms_by_kernel', ''))" $R/gpurun_out/ab/t5_$V.log) sites/s"
done
