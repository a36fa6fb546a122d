#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c20
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python3 -u tools/triage_timing2.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/tools/triage_timing2.py" > "$O/kt.log" 2>&1
python3 - "$O" <<'PY'
import csv, os, sys
for dp, _, fs in os.walk(sys.argv[1] + "/kt"):
    if "run_kernel_trace.csv" in fs:
        for x in csv.DictReader(open(os.path.join(dp, "run_kernel_trace.csv"))):
            if "ss_score" in x["Kernel_Name"]:
                print(x["Kernel_Name"][:22], x["Grid_Size"] if "Grid_Size" in x else "", (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6)
PY
