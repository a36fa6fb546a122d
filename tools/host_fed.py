#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-fed entry point ss_score_batch_host
(host batch -> pinned staging -> H2D -> kernels -> D2H -> calls sorted).
This is what the reference-side shim sees; it is NOT bench.py's `value`
(that one starts with inputs resident in HBM).  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=1 << 22)
    ap.add_argument("--lt", type=float, default=60)
    ap.add_argument("--ln", type=float, default=30)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pinned", action="store_true", help="inputs in ss_host_alloc memory (no staging copy)")
    args = ap.parse_args()
    from __graft_entry__ import load_package
    pkg = load_package()
    t0 = time.perf_counter()
    b = pkg.synth_batch_host(pkg.Synth.default(args.lt, args.ln), 0, args.sites)
    gen_s = time.perf_counter() - t0
    if args.pinned:
        b = b.pinned()
    ctx = pkg.Context()
    ctx.score_batch(b)                       # warm-up (allocations, first launch)
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        ctx.score_batch(b)
        times.append(time.perf_counter() - t0)
    best, mean = min(times), sum(times) / len(times)
    nbytes = b.ref.nbytes + b.off_tumor.nbytes + b.off_normal.nbytes + b.reads_tumor.nbytes + \
        b.reads_normal.nbytes
    print(json.dumps({"path": "ss_score_batch_host (PCIe-inclusive)", "pinned_inputs": args.pinned,
                      "sites": args.sites,
                      "lt": args.lt, "ln": args.ln, "input_bytes": nbytes,
                      "sites_per_s_best": round(args.sites / best, 1),
                      "sites_per_s_mean": round(args.sites / mean, 1),
                      "h2d_input_GBps_best": round(nbytes / best / 1e9, 2),
                      "host_synth_s": round(gen_s, 2)}))


if __name__ == "__main__":
    main()
