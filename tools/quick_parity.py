#!/usr/bin/env python3
"""Fast GPU-vs-oracle parity probe for kernel A/B work (SNIPER_AMD_LIB selects
the library).  Prints mismatching sites per configuration / option set."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from __graft_entry__ import load_package
    from oracle import binding as ob
    from test_gpu_parity import EXOTIC, params_from_opts
    pkg = load_package()
    print("library:", pkg.library_path())
    cfgs = [(60, 30, {}), (30, 30, EXOTIC), (100, 60, EXOTIC), (3, 2, dict(p_wild_qual=0.3, p_del=0.3)),
            (200, 150, EXOTIC), (500, 500, EXOTIC), (700, 300, {}), (560, 470, dict(EXOTIC, p_wild_qual=0.0))]
    bad = 0
    for lt, ln, kw in cfgs:
        b = pkg.synth_batch_host(pkg.Synth.default(lt, ln, seed=7, **kw), 0, 4000 if lt + ln < 500 else 1500)
        for opts in ([], ["-J"], ["-p"]):
            with pkg.Context(params_from_opts(pkg, opts), device=0) as ctx:
                s, c, g = ctx.score_batch(b, want_glf=True)
            o = ob.Oracle(ob.opts_to_params(list(opts)))
            os_, oc, og = o.score_batch(b.ref, b.off_tumor, b.off_normal, b.reads_tumor, b.reads_normal)
            ns = int((s != os_).sum())
            ng = int((g.view(np.uint8).reshape(b.n_sites, -1) != og.view(np.uint8).reshape(b.n_sites, -1)).any(1).sum())
            bad += ns + ng
            print(f"{lt}/{ln} {' '.join(opts) or 'default'}: score mismatches {ns}, glf mismatches {ng}", flush=True)
    print("QUICK_PARITY", "OK" if bad == 0 else f"FAIL {bad}")


if __name__ == "__main__":
    main()
