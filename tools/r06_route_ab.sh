#!/bin/bash
# timing A/B of the deep-routing threshold (build/libsniper_amd_<V>.so; "" = the
# shipped library) at panel depths between C5 and 1200x/1000x
#   bash tools/r06_route_ab.sh TAG V1 V2 ...      (through gpurun)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
for V in "$@"; do
  L=""; [ "$V" != base ] && L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  for cfg in "500 500 1048576" "750 750 524288" "900 900 524288" "1200 1000 262144"; do
    set -- $cfg
    SNIPER_AMD_LIB=$L timeout -k 10 200 python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --no-host-fed --steps 10 --warmup 2 \
        --lt $1 --ln $2 --sites $3 > "$O/ab_${V}_$1.json" 2>&1 || { echo "$V $1 failed"; exit 1; }
    echo "$V $1x/$2x $(python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e sites/s' % r['value'], r['roofline']['avg_ms_by_kernel'])" "$O/ab_${V}_$1.json")"
  done
done
