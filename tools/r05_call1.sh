#!/bin/bash
# round 5, GPU call 1: allocator diagnosis + the new context tests
set -o pipefail
O=gpurun_out/r05c1; mkdir -p $O
B=somatic-sniper_amd/build
echo "== pool_race" | tee $O/progress.log
timeout -k 10 150 $B/pool_race pool 4 40 > $O/pool_race_pool.txt 2>&1; echo "rc $?" >> $O/pool_race_pool.txt
tail -2 $O/pool_race_pool.txt | tee -a $O/progress.log
timeout -k 10 150 $B/pool_race malloc 4 40 > $O/pool_race_malloc.txt 2>&1; echo "rc $?" >> $O/pool_race_malloc.txt
tail -2 $O/pool_race_malloc.txt | tee -a $O/progress.log
echo "== repro diag_pool" | tee -a $O/progress.log
REPRO_OUT=r05c1/repro_pool REPRO_NATIVE=somatic-sniper_amd/build/diag_pool/bam-somaticsniper \
  timeout -k 10 400 python -u tools/repro_groups.py 25 > $O/repro_pool.txt 2>&1 || true
tail -3 $O/repro_pool.txt | tee -a $O/progress.log
echo "== repro product" | tee -a $O/progress.log
REPRO_OUT=r05c1/repro_cache timeout -k 10 400 python -u tools/repro_groups.py 25 > $O/repro_cache.txt 2>&1 || true
tail -3 $O/repro_cache.txt | tee -a $O/progress.log
echo "== pytest" | tee -a $O/progress.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_multi_rank.py \
  > $O/pytest_multi.log 2>&1
rc=$?
tail -5 $O/pytest_multi.log | tee -a $O/progress.log
exit $rc
