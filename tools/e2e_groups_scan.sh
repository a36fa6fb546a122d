#!/bin/bash
# Contig-group configurations on one generated pair (no reference run):
# pileup-only and scored, phase times from SS_TIMING, into gpurun_out/.
#   bash tools/e2e_groups_scan.sh [LENGTH_BP] [CONTIGS]
set -euo pipefail
LEN=${1:-50000000}; NC=${2:-8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=/tmp/ss_e2es_$$
O=$R/gpurun_out/e2e_scan
mkdir -p "$W" "$O"
trap 'rm -rf "$W"' EXIT
timeout -k 10 900 python3 "$R/tools/bamsim.py" "$W" --length "$LEN" --depth-t 30 --depth-n 30 --contigs "$NC" >/dev/null 2>> "$O/progress.log"
cd "$W"
"$R/somatic-sniper_amd/ss-index" tumor.bam && "$R/somatic-sniper_amd/ss-index" normal.bam
run() {   # name, env...
  local name=$1; shift
  local s=$(date +%s.%N)
  env SS_TIMING=1 "$@" timeout -k 10 300 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam "$name.out" 2> "$O/$name.err"
  local e=$(date +%s.%N)
  echo "$name $(python3 -c "print(round($e - $s, 2))")" | tee -a "$O/times.txt"
}
run s1 SS_CONTIG_GROUPS=1
run po_s1 SS_CONTIG_GROUPS=1 SS_PILEUP_ONLY=1
for g in 2 4 8; do
  run po_g$g SS_CONTIG_GROUPS=$g SS_PILEUP_ONLY=1 SS_BGZF_THREADS=2
  run g$g SS_CONTIG_GROUPS=$g SS_BGZF_THREADS=2
done
run g4_b4 SS_CONTIG_GROUPS=4 SS_BGZF_THREADS=4
run g6_b2 SS_CONTIG_GROUPS=6 SS_BGZF_THREADS=2
for f in g2 g4 g8 g4_b4 g6_b2; do cmp s1.out $f.out; done && echo "outputs identical" | tee -a "$O/times.txt"
