#!/bin/bash
# round-5 closing measurements in one call: the full GPU suite, the default bench line with its
# rocprofv3 kernel-trace summary, then the C2 / C3 / C5 / 1200x1000 lines and summaries
set -o pipefail
O=gpurun_out/r05final5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
bash tools/profile_round.sh r05final5 > $O/round.log 2>&1 || { tail -20 $O/round.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['roofline']['frac'], d['roofline']['valu']['insts_per_site'])"
bash tools/profile_configs.sh r05cfg5
