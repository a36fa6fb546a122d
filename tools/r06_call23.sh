#!/bin/bash
# Round 6: the deep triage -- parity, then C5 / 1200x / C4 bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c23
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    --durations=8 -k "${K:-near_exit or synthetic_parity or deep_parity or group}" > "$O/pytest.log" 2>&1; rc=$?
tail -12 "$O/pytest.log"
[ $rc -eq 0 ] || exit $rc
for cfg in "c5 500 500 1048576" "d1200 1200 1000 262144" "c4 60 30 67108864" "c2 30 30 67108864" "c3 100 60 33554432"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --workload shard --no-cpu --no-host-fed --steps 10 --warmup 2 \
      --lt "$2" --ln "$3" --sites "$4" > "$O/bench_$1.json" 2> "$O/bench_$1.err" || { tail -5 "$O/bench_$1.err"; exit 1; }
  echo "$1 $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('%.3e sites/s' % d['value'], r['kernel'], r['avg_ms_by_kernel'], 'frac', r['frac'], 'traffic/alg', r.get('traffic_over_algorithmic'), r.get('traffic_bytes_per_site'), r.get('valu',{}).get('insts_per_site'))" "$O/bench_$1.json")"
done
