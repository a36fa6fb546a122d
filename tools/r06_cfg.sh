#!/bin/bash
# Round-6 per-configuration evidence: one bench line (live PMC traffic, CPU
# baseline unless "nocpu") and one rocprofv3 --kernel-trace --stats run of the
# same workload per configuration; the kernel trace CSV is kept so that the
# per-dispatch durations can be set beside the bench's HIP-event times.
#   bash tools/r06_cfg.sh TAG "name lt ln sites cpu|nocpu" ...      (through gpurun)
set -euo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for cfg in "$@"; do
  set -- $cfg
  name=$1; lt=$2; ln=$3; n=$4
  cpu=""; [ "${5:-cpu}" = nocpu ] && cpu="--no-cpu"
  timeout -k 10 400 python3 "$R/bench.py" --workload shard $cpu --no-host-fed --steps 10 --warmup 2 \
      --lt "$lt" --ln "$ln" --sites "$n" > "$O/bench_$name.json" 2> "$O/bench_$name.err"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$name" -o run -- \
      python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --no-host-fed --steps 10 --warmup 2 \
      --lt "$lt" --ln "$ln" --sites "$n" > "$O/kt_$name.log" 2>&1)
  echo "$name $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('%.3e sites/s' % d['value'], r['kernel'], r['avg_ms_by_kernel'], 'frac', r['frac'], 'traffic/alg', r.get('traffic_over_algorithmic'))" "$O/bench_$name.json")"
done
