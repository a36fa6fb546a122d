#!/usr/bin/env python3
"""Per-kernel times (HIP events) of host-path batches of a few shapes: the
triage + main class, the group and deep kernels, and the whole launch.
    python3 tools/triage_timing.py"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests")]
import numpy as np  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
shapes = [("60x30 n6000", dict(lt=60, ln=30), 6000), ("60x30 n2^20", dict(lt=60, ln=30), 1 << 20),
          ("noisy 120x110 n6000", dict(lt=120, ln=110, p_error=0.1, p_somatic=0.02, p_germline=0.02), 6000),
          ("noisy 30x20 n6000", dict(lt=30, ln=20, p_error=0.1, p_somatic=0.02, p_germline=0.02), 6000)]
with pkg.Context(pkg.Params.default(), device=0) as ctx:
    for name, kw, n in shapes:
        lt, ln = kw.pop("lt"), kw.pop("ln")
        b = pkg.synth_batch_host(pkg.Synth.default(lt, ln, **kw), 0, n)
        ctx.score_batch(b)
        ctx.set_kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(3):
            ctx.score_batch(b)
        wall = (time.perf_counter() - t0) / 3
        ctx.set_kernel_timing(False)
        print(f"{name}: wall {wall * 1e3:.2f} ms/batch; " +
              " ".join(f"{k} {np.mean(ctx.kernel_time_log(k)):.3f}" for k in ("main", "wide", "deep", "all")),
              flush=True)
