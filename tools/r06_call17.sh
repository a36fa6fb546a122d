#!/bin/bash
# Round 6: triage-kernel shape A/B at C4 (headline workload) + the kernel split.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c17
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --no-pmc --no-cpu --no-host-fed --strong-steps 0 > "$O/kt.log" 2>&1) || exit 1
python3 - "$O" <<'PY'
import csv, os, sys
for dp, _, fs in os.walk(sys.argv[1] + "/kt"):
    if "run_kernel_stats.csv" in fs:
        for x in csv.DictReader(open(os.path.join(dp, "run_kernel_stats.csv"))):
            print(x["Name"][:40], x["Calls"], x["AverageNs"], x["TotalDurationNs"])
PY
timeout -k 10 1200 bash tools/ab_libs.sh "$O/ab" cur b256w4 b512w5 b256w3
