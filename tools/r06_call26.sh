#!/bin/bash
# Round 6: per-kernel times at C5 and 1200x/1000x after the deep triage.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c36
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
for cfg in "c5 500 500 1048576" "d1200 1200 1000 262144"; do
  set -- $cfg
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$1" -o run -- python3 bench.py --workload shard --no-cpu \
      --no-host-fed --no-pmc --steps 10 --warmup 2 --lt "$2" --ln "$3" --sites "$4" > "$O/bench_$1.json" 2> "$O/bench_$1.err" || { tail -5 "$O/bench_$1.err"; exit 1; }
  f=$(find "$O/prof_$1" -name '*kernel_stats.csv' | head -1)
  echo "== $1"; cut -d, -f1-5 "$f" | head -12
done
