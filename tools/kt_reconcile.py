#!/usr/bin/env python3
"""Reconcile the bench's HIP-event kernel times with rocprofv3's trace of the
SAME process (tools/r06_cfg.sh / r06_final_cfg.sh run the bench under
`rocprofv3 --kernel-trace --stats`): the mean over the timed dispatches (the
last `launches_timed` ones of the dominant kernel; the warmups' first,
cold, dispatches excluded) against the HIP-event mean the bench printed, and
the --stats average (all dispatches, warmups included) beside them.  A kernel
class 'a+b' (the triage and main kernels) is summed per launch.
    python3 tools/kt_reconcile.py <kt dir> <bench log of that run>"""
import csv
import json
import os
import sys


def main(ktdir, log):
    line = [x for x in open(log).read().splitlines() if x.startswith("{")][-1]
    r = json.loads(line)["roofline"]
    kern = r["kernel"]
    trace = stats = None
    for dp, _, fs in os.walk(ktdir):
        if "run_kernel_trace.csv" in fs:
            trace = os.path.join(dp, "run_kernel_trace.csv")
        if "run_kernel_stats.csv" in fs:
            stats = os.path.join(dp, "run_kernel_stats.csv")
    # a kernel class ('ss_score_triage+ss_score_main'): its dispatches summed
    # per launch, the last name closing a launch
    names = kern.split("+")
    disp = sorted((int(x["Dispatch_Id"]), x["Kernel_Name"].split("(")[0],
                   (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6)
                  for x in csv.DictReader(open(trace)) if x["Kernel_Name"].split("(")[0] in names)
    rows, acc = [], 0.0
    for did, name, d in disp:
        acc += d
        if name == names[-1]:
            rows.append((did, acc))
            acc = 0.0
    n = r["launches_timed"]
    timed = [d for _, d in rows[-n:]]
    avg_stats = None
    for x in csv.DictReader(open(stats)):
        if x["Name"].split("(")[0] in names:
            avg_stats = (avg_stats or 0.0) + float(x["AverageNs"]) / 1e6
    out = {"kernel": kern, "dispatches": len(rows), "timed": n,
           "hip_events_ms": r["avg_kernel_ms"],
           "rocprof_timed_dispatches_ms": round(sum(timed) / len(timed), 4),
           "rocprof_stats_all_dispatches_ms": round(avg_stats, 4) if avg_stats else None,
           "first_dispatches_ms": [round(d, 4) for _, d in rows[:3]]}
    out["timed_vs_hip_events"] = round(out["rocprof_timed_dispatches_ms"] / out["hip_events_ms"] - 1.0, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
