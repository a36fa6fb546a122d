#!/bin/bash
# round 6, call 15: the drop-in CLI end to end at 60x/30x (one shared GPU context per device)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c15
mkdir -p "$O"
timeout -k 10 300 python3 -u "$R/tools/r06_e2e.py" "$O/e2e_2Mb.json" --length 2000000 --contigs 4 > "$O/e2e_2Mb.log" 2>&1 || { tail -5 "$O/e2e_2Mb.log"; exit 1; }
tail -n 1 "$O/e2e_2Mb.log" | cut -c1-300
timeout -k 10 1100 python3 -u "$R/tools/r06_e2e.py" "$O/e2e_50Mb_60x30.json" > "$O/e2e_50Mb.log" 2>&1 || { tail -5 "$O/e2e_50Mb.log"; exit 1; }
tail -n 1 "$O/e2e_50Mb.log"
