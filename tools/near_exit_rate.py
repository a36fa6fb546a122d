#!/usr/bin/env python3
"""Fraction of synthetic sites the triage kernels' early exit decides (the CPU
model tests/near_exit_model.py, default options), per depth configuration,
with the single-chain and the per-strand (deep triage) esum bound.
    python3 tools/near_exit_rate.py [n_sites]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests")]
import numpy as np  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402
from near_exit_model import near_exit, near_tables  # noqa: E402
from oracle import binding as oracle  # noqa: E402

pkg = load_package()
oracle.load()

REF16 = {"A": 1, "C": 2, "G": 4, "T": 8}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
o = oracle.Oracle(oracle.opts_to_params([]))
t = o.tables()
tabs = near_tables(t["fk"], t["coef"], t["lhet"], t["q_r"])
for lt, ln in ((30, 30), (60, 30), (100, 60), (500, 500), (1200, 1000)):
    b = pkg.synth_batch_host(pkg.Synth.default(lt, ln), 0, n)
    ex = exs = 0
    small = 0
    for i in range(b.n_sites):
        rc, rt, rn = b.site(i)
        r16 = REF16.get(chr(rc).upper(), 15)
        if len(rt) <= 128 and len(rn) <= 128:
            small += 1
        ex += near_exit(r16, rt, rn, tabs, t)
        exs += near_exit(r16, rt, rn, tabs, t, per_strand=True)
    print(f"{lt}x/{ln}x: {ex}/{b.n_sites} sites exit ({ex / b.n_sites:.3f}), per-strand bound {exs} "
          f"({exs / b.n_sites:.3f}); <=128 reads per sample: {small}")
