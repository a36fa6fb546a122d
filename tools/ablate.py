#!/usr/bin/env python3
"""Phase ablation timing of ss_score_main (diagnostic; outputs are wrong under
SS_DIAG!=0).  Bits: 1 skip bitonic sort, 2 skip ordered fold, 4 skip
likelihood/consensus, 8 skip site decision.  Prints main-kernel ms per variant."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=1 << 22)
    ap.add_argument("--lt", type=float, default=60)
    ap.add_argument("--ln", type=float, default=30)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--masks", default="0,1,2,4,8,3,6,7,15")
    args = ap.parse_args()
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    ctx = pkg.Context()
    d = ctx.synth_device(pkg.Synth.default(args.lt, args.ln), 0, args.sites)
    score = torch.empty(args.sites, dtype=torch.int32, device="cuda")
    out = {}
    for m in [int(x, 0) for x in args.masks.split(",")]:
        os.environ["SS_DIAG"] = str(m)
        for _ in range(2):
            ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"], score=score)
        ctx.set_kernel_timing(True)
        for _ in range(args.reps):
            ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"], score=score)
        t = ctx.kernel_time_log()
        ctx.set_kernel_timing(False)
        out[m] = round(float(t.mean()), 4)
        print(f"mask {m:2d}: {out[m]:.3f} ms  ({args.sites / (out[m] * 1e-3):.3e} sites/s)", flush=True)
    os.environ["SS_DIAG"] = "0"
    print(json.dumps({"sites": args.sites, "lt": args.lt, "ln": args.ln, "ms": out}))


if __name__ == "__main__":
    main()
