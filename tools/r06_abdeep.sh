#!/bin/bash
# timing A/B of deep-kernel variants (build/libsniper_amd_<V>.so, all listed
# sites on the deep kernel): C5 500x/500x (2^20 sites) and 3000x/3000x (2^18)
#   bash tools/r06_abdeep.sh TAG V1 V2 ...      (through gpurun)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
for V in "$@"; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  for cfg in "500 500 1048576" "3000 3000 262144"; do
    set -- $cfg
    SNIPER_AMD_LIB=$L timeout -k 10 200 python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --no-host-fed --steps 10 --warmup 2 \
        --lt $1 --ln $2 --sites $3 > "$O/ab_${V}_$1.json" 2>&1 || { echo "$V $1 failed"; exit 1; }
    echo "$V $1x/$2x $(python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e sites/s' % r['value'], r['roofline']['avg_ms_by_kernel'])" "$O/ab_${V}_$1.json")"
  done
done
