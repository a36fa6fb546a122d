#!/bin/bash
# Round 6: A/B of kernel variants (SNIPER_AMD_LIB) on shard benches.
#   LIBS="base e1" CFGS="c4:60:30:67108864 c5:500:500:1048576" bash tools/r06_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ab
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
for lib in ${LIBS:-base}; do
  for cfg in ${CFGS:-c4:60:30:67108864 c5:500:500:1048576}; do
    IFS=: read n lt ln sites <<< "$cfg"
    L=""; [ "$lib" != base ] && L=somatic-sniper_amd/build/libsniper_amd_$lib.so
    SNIPER_AMD_LIB=$L timeout -k 10 200 python3 bench.py --workload shard --no-cpu --no-host-fed --no-pmc --steps 20 --warmup 3 \
        --lt "$lt" --ln "$ln" --sites "$sites" > "$O/b_${lib}_$n.json" 2> "$O/b_${lib}_$n.err" || { tail -5 "$O/b_${lib}_$n.err"; exit 1; }
    echo "$rep $lib $n $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('%.4e' % d['value'], r['avg_ms_by_kernel'])" "$O/b_${lib}_$n.json")"
  done
done
done
