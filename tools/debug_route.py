#!/usr/bin/env python3
"""Debug aid (round 6): the test_group_unit_boundaries[1023/1020] batch, GPU vs
oracle, with per-site depths and read statistics of the mismatching sites."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from __graft_entry__ import load_package
    from oracle import binding as ob
    from test_gpu_parity import EXOTIC
    pkg = load_package()
    print("library:", pkg.library_path())
    for lt, ln, n in ((1023, 1020, 30), (1200, 1000, 60)):
        b = pkg.synth_batch_host(pkg.Synth.default(lt, ln, **EXOTIC), 11, n)
        with pkg.Context(pkg.Params.default(), device=0) as ctx:
            s, c, g = ctx.score_batch(b, want_glf=True)
            s2, _, _ = ctx.score_batch(b, want_glf=False)
        o = ob.Oracle(ob.opts_to_params([]))
        os_, oc, og = o.score_batch(b.ref, b.off_tumor, b.off_normal, b.reads_tumor, b.reads_normal)
        bad = np.nonzero(s != os_)[0]
        print(f"{lt}/{ln}: {bad.size} mismatches (glf run), {int((s2 != os_).sum())} (no-glf run)")
        for i in bad[:10]:
            nt = int(b.off_tumor[i + 1] - b.off_tumor[i]); nn = int(b.off_normal[i + 1] - b.off_normal[i])
            rt = b.reads_tumor[b.off_tumor[i]:b.off_tumor[i + 1]]
            rn = b.reads_normal[b.off_normal[i]:b.off_normal[i + 1]]
            def wild(r):
                mq = r & 0xff; bq = (r >> 8) & 0xff; mn = np.minimum(mq, bq)
                return int(((mn >= 64) | ((mn < 4) & (bq >= 64))).sum())
            print(f"  site {i}: ref {chr(b.ref[i])} nt {nt} nn {nn} wild reads {wild(rt)}/{wild(rn)} gpu {s[i]} "
                  f"oracle {os_[i]} glf-gpu {g[i].tobytes().hex() if g is not None else None}")


if __name__ == "__main__":
    main()
