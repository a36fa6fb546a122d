#!/bin/bash
# End-to-end CLI timing with indexed BAMs:
# the reference CLI, the native CLI's single streaming walk, and its
# contig-parallel pileup (SS_CONTIG_GROUPS ranges, bam_index.h), outputs
# compared byte for byte.  Writes one JSON line.
#   bash tools/e2e_groups.sh [LENGTH_BP] [DEPTH_T] [DEPTH_N] [CONTIGS]
set -euo pipefail
LEN=${1:-50000000}; DT=${2:-30}; DN=${3:-30}; NC=${4:-8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=/tmp/ss_e2eg_$$
mkdir -p "$W" "$R/gpurun_out"
TICK=
trap '[ -n "$TICK" ] && kill $TICK 2>/dev/null; rm -rf "$W"; true' EXIT
ts() { date +%s.%N; }
P=$R/gpurun_out/e2e_progress.log
: > "$P"
# progress for long silent steps: the step's name and elapsed seconds every 30 s
tick() { local what=$1; local s=0; while sleep 30; do s=$((s + 30)); echo "$what ${s}s" >> "$P"; done; }
t0=$(ts)
timeout -k 10 900 python3 "$R/tools/bamsim.py" "$W" --length "$LEN" --depth-t "$DT" --depth-n "$DN" --contigs "$NC" >/dev/null 2>> "$P"
t1=$(ts)
cd "$W"
timeout -k 10 300 "$R/somatic-sniper_amd/ss-index" tumor.bam
timeout -k 10 300 "$R/somatic-sniper_amd/ss-index" normal.bam
t2=$(ts)
tick "reference CLI" & TICK=$!
timeout -k 10 900 "$R/oracle/_ref/bam-somaticsniper" -f ref.fa tumor.bam normal.bam ref.out 2> ref.err
kill $TICK; TICK=
echo "reference done" >> "$P"
t3=$(ts)
SS_CONTIG_GROUPS=1 timeout -k 10 600 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam s.out 2> s.err
t4=$(ts)
SS_CONTIG_GROUPS=4 SS_BGZF_THREADS=2 timeout -k 10 600 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam g4.out 2> g4.err
t5=$(ts)
SS_CONTIG_GROUPS=8 SS_BGZF_THREADS=2 SS_PILEUP_WORKERS=2 timeout -k 10 600 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam g8.out 2> g8.err
t6=$(ts)
same=true
for f in s.out g4.out g8.out; do cmp ref.out "$f" || same=false; done
python3 - "$t0" "$t1" "$t2" "$t3" "$t4" "$t5" "$t6" "$same" "$LEN" "$DT" "$DN" "$NC" "$(grep -c . ref.out || true)" <<'PY'
import json, os, sys
t = list(map(float, sys.argv[1:8]))
same, L, dt, dn, nc, lines = sys.argv[8] == "true", int(sys.argv[9]), sys.argv[10], sys.argv[11], int(sys.argv[12]), int(sys.argv[13])
ref, s, g4, g8 = t[3] - t[2], t[4] - t[3], t[5] - t[4], t[6] - t[5]
print(json.dumps({"genome_bp": L, "contigs": nc, "depth": f"{dt}/{dn}", "format": "classic", "emitted_lines": lines,
                  "gen_s": round(t[1] - t[0], 2), "index_both_s": round(t[2] - t[1], 2),
                  "reference_cli_s": round(ref, 2), "native_stream_s": round(s, 2),
                  "native_groups4_s": round(g4, 2), "native_groups8_s": round(g8, 2),
                  "groups8_vs_stream": round(s / g8, 2), "groups4_vs_stream": round(s / g4, 2),
                  "outputs_identical": same, "host_cpus_visible": os.cpu_count()}))
PY
cat ref.err s.err g8.err >&2
