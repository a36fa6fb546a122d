#!/bin/bash
# round 5, GPU call 2: which part of the stream-ordered pool path loses the calls
O=gpurun_out/r05c2; mkdir -p $O
for v in pool pool_stage_malloc pool_sync pool_keepstream; do
  echo "== $v" | tee -a $O/progress.log
  REPRO_KEEP_ALL=1 REPRO_OUT=r05c2/$v REPRO_NATIVE=somatic-sniper_amd/build/diag_$v/bam-somaticsniper \
    timeout -k 10 300 python -u tools/repro_groups.py 40 > $O/$v.txt 2>&1
  rc=$?
  tail -1 $O/$v.txt | tee -a $O/progress.log
  [ $rc -eq 0 ] || { echo "rc $rc"; exit $rc; }
done
