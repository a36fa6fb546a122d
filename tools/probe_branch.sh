set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/br; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --pmc-child --workload shard --sites 16777216 --lt 60 --ln 30 > $O/p1.log 2>&1
python3 $R/tools/pmc_kernels.py $O/p1 --sites 16777216
