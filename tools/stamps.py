#!/usr/bin/env python3
"""Per-phase wave-cycle breakdown of ss_score_main from an SS_STAMP build
(diagnostic; `make -C somatic-sniper_amd variant V=stamp DEFS=-DSS_STAMP=1`).

    SNIPER_AMD_LIB=somatic-sniper_amd/build/libsniper_amd_stamp.so python tools/stamps.py

Prints the kernel time and, per phase, the cycles summed over all waves per
site (s_memtime ticks = shader cycles)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ["wait reads", "A loop", "next sub", "B fold", "C glf fin", "D decide", "prologue", "A keys",
         "A network", "A counts", "A records", "C dma", "C geno_p", "W sort", "W finish", "W other"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=1 << 22)
    ap.add_argument("--lt", type=float, default=60)
    ap.add_argument("--ln", type=float, default=30)
    args = ap.parse_args()
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    ctx = pkg.Context()
    lib = ctypes.CDLL(os.environ["SNIPER_AMD_LIB"])
    acc = (ctypes.c_ulonglong * 16)()
    d = ctx.synth_device(pkg.Synth.default(args.lt, args.ln), 0, args.sites)
    score = torch.empty(args.sites, dtype=torch.int32, device="cuda")
    ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"], score=score)
    torch.cuda.synchronize()
    lib.ss_debug_stamps(acc)
    ctx.set_kernel_timing(True)
    ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"], score=score)
    torch.cuda.synchronize()
    ms = float(ctx.kernel_time_log().mean())
    ctx.set_kernel_timing(False)
    assert lib.ss_debug_stamps(acc) == 0
    tot = sum(acc)
    print(f"{args.lt:g}x/{args.ln:g}x  {args.sites} sites  kernel {ms:.3f} ms  "
          f"({args.sites / ms * 1e3:.3e} sites/s)  wave-cycles/site {tot / args.sites:.0f}")
    for n, v in zip(NAMES, acc):
        if v:
            print(f"  {n:11s} {v / args.sites:8.1f} cyc/site  {100.0 * v / tot:5.1f} %")


if __name__ == "__main__":
    main()
