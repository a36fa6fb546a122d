#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c13
mkdir -p "$O"
SNIPER_AMD_LIB=$R/somatic-sniper_amd/build/libsniper_amd_dbg.so timeout -k 10 200 python3 -u "$R/tools/debug_route.py" > "$O/debug_dbg.log" 2>&1; grep -v amdgpu.ids "$O/debug_dbg.log" | head -30
