#!/bin/bash
# Round 6: routing counts of the device path at 500x/500x, 1200x/1000x, 60x/30x.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c30
mkdir -p "$O"
cd "$R"
for cfg in "500 500" "1200 1000" "60 30"; do
  set -- $cfg
  timeout -k 10 180 python3 -u tools/c5_fault_probe.py $1 $2 > "$O/probe_$1.log" 2>&1 || { tail -5 "$O/probe_$1.log"; exit 1; }
  echo "== $1/$2"; grep "^n " "$O/probe_$1.log"
done
