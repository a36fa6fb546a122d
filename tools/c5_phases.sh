#!/bin/bash
# Group-kernel phase costs at C5 (500xT/500xN): for each variant library
# build/libsniper_amd_<V>.so (tools/ablate.py g* ablations), the bench's
# per-kernel HIP-event times on 2^20 sites; the first variant also gets the
# live PMC passes (VALU per site of ss_score_group).
#   bash tools/c5_phases.sh base gnosort gnomerge gnorec gnofold gnofin
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5
mkdir -p "$O"
first=1
for V in "$@"; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  PMC="--no-pmc"
  [ $first -eq 1 ] && PMC=""
  first=0
  SNIPER_AMD_LIB=$L timeout -k 10 300 python "$R/bench.py" --workload shard --no-cpu $PMC --steps 5 --warmup 2 \
      --lt ${C5_LT:-500} --ln ${C5_LN:-500} --sites ${C5_SITES:-1048576} > "$O/$V.json" 2> "$O/$V.err" \
      || { echo "$V failed"; tail -5 "$O/$V.err"; exit 1; }
  python3 - "$O/$V.json" "$V" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rf = r["roofline"]
print(sys.argv[2], "%.3e sites/s" % r["value"], "ms", rf["avg_ms_by_kernel"], "valu", rf.get("valu", {}).get("insts_per_site"))
PY
done
