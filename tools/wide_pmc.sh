#!/bin/bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/widepmc
mkdir -p "$O"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM \
  --output-format csv -d "$O/pmc" -o run -- python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --lt 500 --ln 500 --sites 262144 --steps 2 --warmup 1 > "$O/log" 2>&1
python3 "$R/tools/pmc_kernels.py" "$O/pmc" --sites 262144
