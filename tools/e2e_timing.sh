#!/bin/bash
# Phase times (SS_TIMING=1) of the native CLI on one synthetic BAM pair:
#   bash tools/e2e_timing.sh [LENGTH_BP] [DEPTH_T] [DEPTH_N]
set -euo pipefail
LEN=${1:-5000000}; DT=${2:-60}; DN=${3:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=/tmp/ss_tim_$$
mkdir -p "$W"
trap 'rm -rf "$W"' EXIT
timeout -k 10 600 python3 "$R/tools/bamsim.py" "$W" --length "$LEN" --depth-t "$DT" --depth-n "$DN" >/dev/null
cd "$W"
for rep in 1 2; do
  for nb in 1048576 262144; do
    echo "--- run $rep SS_BATCH=$nb"
    s=$(date +%s%N)
    SS_BATCH=$nb SS_TIMING=1 timeout -k 10 300 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam out$nb.txt 2>&1 | grep -E "pileup done|ready|output written|exit"
    e=$(date +%s%N)
    echo "wall $(( (e - s) / 1000000 )) ms"
  done
  cmp out1048576.txt out262144.txt
done
