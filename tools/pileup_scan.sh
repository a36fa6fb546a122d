#!/bin/bash
# Pileup-only wall time of the native CLI over thread settings (one synthetic BAM pair):
#   bash tools/pileup_scan.sh [LENGTH_BP] [DEPTH_T] [DEPTH_N]
set -euo pipefail
LEN=${1:-5000000}; DT=${2:-60}; DN=${3:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=/tmp/ss_scan_$$
mkdir -p "$W"
trap 'rm -rf "$W"' EXIT
timeout -k 10 600 python3 "$R/tools/bamsim.py" "$W" --length "$LEN" --depth-t "$DT" --depth-n "$DN" >/dev/null
cd "$W"
run() {   # label, env...
  local label=$1; shift
  local s e
  s=$(date +%s%N)
  env "$@" SS_PILEUP_ONLY=1 timeout -k 10 300 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam po.out 2>/dev/null
  e=$(date +%s%N)
  echo "$label $(( (e - s) / 1000000 )) ms"
}
run warmup SS_PILEUP_THREADS=2
for rep in 1 2; do
  run walk-threaded SS_PILEUP_THREADS=1
  for w in 1 2 3 4 6; do run "column w=$w bgzf=4" SS_PILEUP_WORKERS=$w; done
  for b in 2 6 8; do run "column w=3 bgzf=$b" SS_PILEUP_WORKERS=3 SS_BGZF_THREADS=$b; done
done
