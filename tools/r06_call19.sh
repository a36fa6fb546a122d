#!/bin/bash
# Round 6: triage kernel with batched chunk loads -- parity subset (timed),
# C4 bench with counters, A/B against TRI_P = 2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c19
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    --durations=12 -k "${K:-near_exit}" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -16 "$O/pytest.log"
timeout -k 10 300 python3 bench.py --workload shard --no-cpu --no-host-fed --steps 10 --warmup 2 \
    --lt 60 --ln 30 --sites 67108864 > "$O/bench_c4.json" 2> "$O/bench_c4.err" || exit 1
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c4 %.3e sites/s' % d['value'], r['avg_ms_by_kernel'], 'frac', r['frac'], 'traffic/alg', r.get('traffic_over_algorithmic'), r.get('traffic_bytes_per_site'), r.get('valu'))" "$O/bench_c4.json"
timeout -k 10 900 bash tools/ab_libs.sh "$O/ab" cur p2
