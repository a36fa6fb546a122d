#!/bin/bash
# round 5, GPU call 4: group-kernel tests on the lazy record arena, then the default bench + rocprof stats
O=gpurun_out/r05c4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_multi_rank.py \
  tests/test_gpu_parity.py -k "group or wide or deep or routing or quirk or contexts or outlives or guard or two_streams" \
  > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-pmc --no-cpu --no-host-fed --strong-steps 0 \
  > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/kt.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/kt -name "*stats*"
