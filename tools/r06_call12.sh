#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c12
mkdir -p "$O"
timeout -k 10 200 python3 -u "$R/tools/debug_route.py" > "$O/debug_base.log" 2>&1; cat "$O/debug_base.log" | tail -25
SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_route2048.so timeout -k 10 200 python3 -u "$R/tools/debug_route.py" > "$O/debug_2048.log" 2>&1; tail -5 "$O/debug_2048.log"
