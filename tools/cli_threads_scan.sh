#!/bin/bash
# Pileup-only timing of the native CLI under different host thread splits
# (BGZF inflate threads per BAM x window builders per sample) on one synthetic
# pair, to size the defaults for the GPU box's CPU share.
#   bash tools/cli_threads_scan.sh [LENGTH_BP] [DEPTH_T] [DEPTH_N]
set -euo pipefail
LEN=${1:-10000000}; DT=${2:-30}; DN=${3:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=/tmp/ss_thr_$$
mkdir -p "$W"
trap 'rm -rf "$W"' EXIT
timeout -k 10 600 python3 "$R/tools/bamsim.py" "$W" --length "$LEN" --depth-t "$DT" --depth-n "$DN" --contigs 2 >/dev/null
cd "$W"
SS_PILEUP_ONLY=1 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam warm.out 2>/dev/null
for cfg in "4 3" "2 2" "3 3" "6 3" "4 5" "6 5" "8 6"; do
  set -- $cfg
  for rep in 1 2; do
    t0=$(date +%s.%N)
    SS_BGZF_THREADS=$1 SS_PILEUP_WORKERS=$2 SS_PILEUP_ONLY=1 timeout -k 10 300 \
      "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam po.out 2>/dev/null
    t1=$(date +%s.%N)
    python3 -c "import sys; print('bgzf %s workers %s: %.3f s' % (sys.argv[1], sys.argv[2], float(sys.argv[4]) - float(sys.argv[3])))" $1 $2 $t0 $t1
  done
done
