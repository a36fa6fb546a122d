#!/usr/bin/env python3
"""Main-class kernel time vs batch size, with and without glf records (no
triage with glf)."""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests")]
import numpy as np  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
with pkg.Context(pkg.Params.default(), device=0) as ctx:
    for n in (64, 640, 6000, 65536, 1 << 18):
        b = pkg.synth_batch_host(pkg.Synth.default(60, 30), 0, n)
        for glf in (False, True):
            ctx.score_batch(b, want_glf=glf)
            ctx.set_kernel_timing(True)
            ctx.score_batch(b, want_glf=glf)
            ctx.set_kernel_timing(False)
            print(f"n {n} glf {glf}: main {np.mean(ctx.kernel_time_log('main')):.3f} ms", flush=True)
