#!/bin/bash
# End-to-end CLI timing on a synthetic BAM pair: reference CLI (1 thread) vs
# the native CLI (GPU scoring; also with several scorers, SS_DEVICES), outputs
# compared byte for byte (classic format, BASELINE config C2 at 50 Mb 30/30).
#   CONTIGS=4 bash tools/e2e_bench.sh [LENGTH_BP] [DEPTH_T] [DEPTH_N]
set -euo pipefail
LEN=${1:-5000000}; DT=${2:-60}; DN=${3:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=/tmp/ss_e2e_$$
mkdir -p "$W" "$R/gpurun_out"
trap 'rm -rf "$W"' EXIT
t0=$(date +%s.%N)
timeout -k 10 600 python3 "$R/tools/bamsim.py" "$W" --length "$LEN" --depth-t "$DT" --depth-n "$DN" --contigs "${CONTIGS:-2}" >/dev/null
t1=$(date +%s.%N)
cd "$W"
ls -la "$W" > "$R/gpurun_out/e2e_files.txt"
timeout -k 10 900 "$R/oracle/_ref/bam-somaticsniper" -f ref.fa tumor.bam normal.bam ref.out 2> ref.err
t2=$(date +%s.%N)
timeout -k 10 600 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam nat.out 2> nat.err
t3=$(date +%s.%N)
SS_PILEUP_ONLY=1 timeout -k 10 600 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam po.out 2>/dev/null
t4=$(date +%s.%N)
SS_DEVICES=${E2E_DEVICES:-0,0} timeout -k 10 600 "$R/somatic-sniper_amd/bam-somaticsniper" -f ref.fa tumor.bam normal.bam multi.out 2> multi.err
cmp ref.out nat.out && cmp ref.out multi.out && same=true || same=false
sites_scored=$(grep -c . ref.out || true)
sites=$(( LEN ))
python3 - "$t0" "$t1" "$t2" "$t3" "$t4" "$same" "$LEN" "$DT" "$DN" "${CONTIGS:-2}" "$sites_scored" <<'PY'
import json, sys
t0, t1, t2, t3, t4 = map(float, sys.argv[1:6])
same, L, dt, dn = sys.argv[6] == "true", int(sys.argv[7]), sys.argv[8], sys.argv[9]
print(json.dumps({"genome_bp": L, "contigs": int(sys.argv[10]), "emitted_lines": int(sys.argv[11]),
                  "format": "classic", "depth": f"{dt}/{dn}", "gen_s": round(t1 - t0, 2),
                  "reference_cli_s": round(t2 - t1, 2), "native_cli_s": round(t3 - t2, 2),
                  "native_pileup_only_s": round(t4 - t3, 2), "outputs_identical": same,
                  "reference_positions_per_s": round(L / (t2 - t1)), "native_positions_per_s": round(L / (t3 - t2))}))
PY
cat ref.err nat.err >&2; wc -l ref.out nat.out >&2
