#!/bin/bash
# round 6, call 7: deep-kernel phase ablations (timing only) and the C5 counters of the all-deep build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/r06_abdeep.sh" r06c7 alldeep ab_nofold ab_noatom ab_nofoldruns || exit 1
SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_alldeep.so timeout -k 10 400 python3 "$R/bench.py" --workload shard --no-cpu --no-host-fed --steps 10 --warmup 2 \
    --lt 500 --ln 500 --sites 1048576 > "$R/gpurun_out/r06c7/pmc_alldeep_c5.json" 2>&1 || exit 1
python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['roofline']; print(r['kernel'], r['traffic_bytes_per_site'], r['valu'])" "$R/gpurun_out/r06c7/pmc_alldeep_c5.json" | cut -c1-600
