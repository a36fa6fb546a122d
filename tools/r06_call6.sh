#!/bin/bash
# round 6, call 6: deep kernel with read prefetch (next chunk entry, next batch)
# quirk parity first (it faulted in call 2), then the parity file, deep lines, C5 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c6
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    "$R/tests/test_gpu_parity.py" -k "quirk_parity or giant" > "$O/pytest_quirk.log" 2>&1; rc=$?; tail -n 2 "$O/pytest_quirk.log"
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    "$R/tests/test_gpu_parity.py" > "$O/pytest_parity.log" 2>&1; rc=$?; tail -n 3 "$O/pytest_parity.log"
[ $rc -eq 0 ] || exit 1
bash "$R/tools/r06_cfg.sh" r06c6/deep "d3000 3000 3000 262144 nocpu" "d2100 2100 100 262144 nocpu" || exit 1
for V in alldeep; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  SNIPER_AMD_LIB=$L timeout -k 10 300 python3 -u "$R/tools/quick_parity.py" > "$O/qp_$V.log" 2>&1 || exit 1; tail -n 1 "$O/qp_$V.log"
  for cfg in "500 500 1048576" "1200 1000 262144"; do
    set -- $cfg
    SNIPER_AMD_LIB=$L timeout -k 10 200 python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --no-host-fed --steps 10 --warmup 2 \
        --lt $1 --ln $2 --sites $3 > "$O/ab_${V}_$1.json" 2>&1 || exit 1
    echo "$V $1x/$2x $(python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e sites/s' % r['value'], r['roofline']['avg_ms_by_kernel'])" "$O/ab_${V}_$1.json")"
  done
done
