#!/bin/bash
# HBM-side counters of ss_score_main for each variant library
# build/libsniper_amd_<V>.so (SNIPER_AMD_LIB), one rocprofv3 --pmc pass per
# counter group over a shard-workload bench (16M sites, 60xT/30xN unless
# TP_ARGS says otherwise): per-launch means of FETCH_SIZE (KiB, doubled per
# MI355X_MICROARCH.md for streaming reads), WRITE_SIZE, TCC hit / miss.
#   bash tools/traffic_probe.sh new r3 abl
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/traffic
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
for V in "$@"; do
  L=$R/somatic-sniper_amd/build/libsniper_amd_$V.so
  i=0
  for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    i=$((i + 1))
    SNIPER_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$O/$V.$i" -o run -- \
        python3 "$R/bench.py" --workload shard --no-cpu --no-pmc --steps 3 --warmup 1 --sites ${TP_SITES:-16777216} ${TP_ARGS:-} \
        > "$O/$V.$i.log" 2>&1 || { echo "$V pass $i ($ctrs) failed"; tail -5 "$O/$V.$i.log"; exit 1; }
  done
  python3 - "$O" "$V" "${TP_SITES:-16777216}" <<'PY'
import csv, glob, sys, collections, json
o, v, sites = sys.argv[1], sys.argv[2], float(sys.argv[3])
vals = collections.defaultdict(list)
for f in glob.glob(f"{o}/{v}.*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "ss_score_main" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), x in per.items():
        vals[c].append((int(d), x))
res = {}
for c, xs in vals.items():
    xs = [x for _, x in sorted(xs)][1:] or [x for _, x in xs]     # first launch: cold tables
    res[c] = sum(xs) / len(xs)
out = {"variant": v, "sites_per_launch": sites, **{k: round(x, 1) for k, x in res.items()}}
if "FETCH_SIZE" in res:
    out["read_B_per_site_x2"] = round(2 * 1024 * res["FETCH_SIZE"] / sites, 2)
if "WRITE_SIZE" in res:
    out["write_B_per_site"] = round(1024 * res["WRITE_SIZE"] / sites, 2)
if "TCC_EA0_RDREQ_sum" in res:
    out["rdreq_64B_per_site"] = round(64 * res["TCC_EA0_RDREQ_sum"] / sites, 2)
print(json.dumps(out))
PY
done
