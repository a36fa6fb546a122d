#!/bin/bash
# Full-size A/B: the default bench (2^24 sites, 60x/30x, no CPU leg) with each
# variant library build/libsniper_amd_<V>.so, in the order given (alternate them):
#   bash tools/abbench.sh a b a b      (through gpurun)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/abb"
i=0
for v in "$@"; do
  i=$((i + 1))
  SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_$v.so timeout -k 10 120 \
      python "$R/bench.py" --workload shard --no-cpu --steps 20 --warmup 3 > "$R/gpurun_out/abb/${i}_$v.json" 2>/dev/null
  echo "$v $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%.4e'%d['value'], d['roofline']['avg_kernel_ms'])" "$R/gpurun_out/abb/${i}_$v.json")"
done
