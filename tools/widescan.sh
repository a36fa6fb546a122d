#!/bin/bash
# 500x/500x bench over wide-kernel grid sizes (SS_WIDE_GRID = workgroups per CU)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for g in 1 2 4 8 1 4; do
  v=$(SS_WIDE_GRID=$g timeout -k 10 200 python $R/bench.py --no-cpu --steps 10 --lt 500 --ln 500 --sites 1048576 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])")
  echo "wide grid/CU=$g $v"
done
for g in 128 256; do
  v=$(SS_MAIN_GRID=$g timeout -k 10 200 python $R/bench.py --no-cpu --steps 10 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])")
  echo "main grid/CU=$g $v"
done
