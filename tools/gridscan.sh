#!/bin/bash
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for g in 64 96 128 256 64 128 256; do
  echo "grid/CU=$g $(SS_MAIN_GRID=$g timeout -k 10 200 python $R/tools/ablate.py --masks 0 --reps 10 2>/dev/null | grep 'mask  0')"
done
