#!/bin/bash
# Kernel-level evidence for the non-headline depth configurations (SURVEY.md
# section 8d: C2 30x/30x, C3 100x/60x, C5 500x/500x, plus a 1200x/1000x deep panel):
# one bench line and one
# rocprofv3 --kernel-trace --stats summary per configuration.
#   bash tools/profile_configs.sh [TAG]      (through gpurun)
set -euo pipefail
TAG=${1:-r02cfg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
# sites per step: as many as the u32 read offsets allow at that depth
# the reference CPU baseline (1 core and all cgroup cores, sample sized for about the
# same CPU time at every depth) is taken at each BASELINE depth; d1200 is beyond them
for cfg in "c2 30 30 67108864 cpu" "c3 100 60 33554432 cpu" "c5 500 500 1048576 cpu" "d1200 1200 1000 262144 nocpu"; do
  set -- $cfg
  name=$1; lt=$2; ln=$3; n=$4
  cpu=""; [ "$5" = nocpu ] && cpu="--no-cpu"
  timeout -k 10 500 python3 "$R/bench.py" --workload shard $cpu --steps 10 --warmup 2 --lt "$lt" --ln "$ln" --sites "$n" \
      > "$O/bench_$name.json" 2> "$O/bench_$name.err"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$name" -o run -- \
      python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --no-host-fed --steps 5 --warmup 2 --lt "$lt" --ln "$ln" --sites "$n" > "$O/kt_$name.log" 2>&1)
  echo "$name $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.3e' % d['value'], d['roofline']['frac'])" "$O/bench_$name.json")"
done
