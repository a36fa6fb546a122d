#!/bin/bash
# Round 6: deep-triage load pipelining A/B at 500x/500x and 1200x/1000x.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c31
mkdir -p "$O"
cd "$R"
for lib in "" trd_pipe8 trd_p16 trd_pipe4; do
  for cfg in "c5 500 500 1048576" "d1200 1200 1000 262144"; do
    set -- $cfg
    L=${lib:+somatic-sniper_amd/build/libsniper_amd_$lib.so}
    SNIPER_AMD_LIB=$L timeout -k 10 200 python3 bench.py --workload shard --no-cpu --no-host-fed --no-pmc --steps 20 --warmup 3 \
        --lt "$2" --ln "$3" --sites "$4" > "$O/b_${lib:-base}_$1.json" 2> "$O/b_${lib:-base}_$1.err" || { tail -5 "$O/b_${lib:-base}_$1.err"; exit 1; }
    echo "${lib:-base} $1 $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('%.3e' % d['value'], r['avg_ms_by_kernel'])" "$O/b_${lib:-base}_$1.json")"
  done
done
