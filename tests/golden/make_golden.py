#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REAL reference.

Runs in the build container only (needs oracle/_ref/ref_harness, compiled from
/root/reference by `make -f oracle/ref.mk`).  For each case it stores, in one
compressed .npz (numpy, no pickle):
  inputs   ref, off_tumor, off_normal, reads_tumor, reads_normal (packed batch)
  outputs  per option set: glf_somatic return value per site; for the option sets
           that change the genotype model (default, -T/-N/-r) also both glf1_t
           records and consensus words; emitted lines (classic + VCF text) for the
           default options.
The reference is driven exactly as sniper_pileup.c:256-258 calls glf_somatic
(see oracle/ref_harness.c).  Inputs come from the deterministic generator in
somatic-sniper_amd/csrc/ss_synth.c plus hand-built quirk sites (SURVEY.md
Appendix A).

    python tests/golden/make_golden.py [case ...]
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from __graft_entry__ import load_package   # noqa: E402
from oracle import binding as ob           # noqa: E402

EXOTIC = dict(p_wild_qual=0.05, p_eq=0.02, p_iupac=0.02, p_nbase=0.02, p_ref_n=0.02,
              p_ref_lower=0.05, p_ref_iupac=0.02, p_germline=0.03, p_somatic=0.05, vaf=0.4,
              p_del=0.05)
OPTSETS = {"default": [], "J": ["-J"], "p": ["-p"], "s1e-6": ["-s", "1e-6"],
           "TNr": ["-T", "0.9", "-N", "3", "-r", "0.01"], "Q0LG": ["-Q", "0", "-L", "-G"],
           "JpQ0": ["-J", "-p", "-Q", "0"], "L": ["-L"], "G": ["-G"]}
GLF_SETS = ("default", "TNr")


def cases(pkg):
    from test_gpu_parity import quirk_sites  # same hand-built sites as the GPU test
    S = pkg.Synth.default
    yield "c30", pkg.synth_batch_host(S(30, 30, seed=11), 0, 2000), ("default", "J", "p")
    yield "c60x", pkg.synth_batch_host(S(60, 30, seed=12, **EXOTIC), 0, 2500), tuple(OPTSETS)
    yield "c100", pkg.synth_batch_host(S(100, 60, seed=13, **EXOTIC), 0, 1000), ("default", "J", "TNr")
    yield "low", pkg.synth_batch_host(S(3, 2, seed=14, p_wild_qual=0.3, p_del=0.3, p_somatic=0.1,
                                        p_germline=0.1), 0, 3000), tuple(OPTSETS)
    yield "deep", pkg.synth_batch_host(S(700, 700, seed=15, fixed_depth=1, **EXOTIC), 0, 40), ("default", "J")
    yield "deep300", pkg.synth_batch_host(S(300, 300, seed=16, **EXOTIC), 0, 100), ("default",)
    yield "quirks", pkg.Batch.from_sites(quirk_sites(pkg)), tuple(OPTSETS)


def main():
    pkg = load_package()
    if not os.path.exists(ob.REF_HARNESS):
        sys.exit("build the reference first: make -f oracle/ref.mk")
    only = set(sys.argv[1:])                  # case names to regenerate (default: all)
    for name, b, sets in cases(pkg):
        if only and name not in only:
            continue
        out = {"ref": b.ref, "off_tumor": b.off_tumor, "off_normal": b.off_normal,
               "reads_tumor": b.reads_tumor, "reads_normal": b.reads_normal}
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "b.ssb")
            ob.write_ssb(path, b.ref, b.off_tumor, b.off_normal, b.reads_tumor, b.reads_normal)
            for s in sets:
                rec, txt = ob.run_ref_dump(path, OPTSETS[s], d)
                out[f"ret_{s}"] = rec["ret"].copy()
                if s in GLF_SETS:
                    out[f"cns_{s}"] = np.stack([rec["cns_tumor"], rec["cns_normal"]], 1)
                    out[f"glf_{s}"] = rec["glf"].view(np.uint8).reshape(len(rec), -1).copy()
                if s == "default":
                    out["classic_default"] = np.frombuffer(txt.encode(), np.uint8)
                    _, vcf = ob.run_ref_dump(path, ["-F", "vcf"], d)
                    out["vcf_default"] = np.frombuffer(vcf.encode(), np.uint8)
        fn = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(fn, **out)
        print(f"{fn}: {b.n_sites} sites, {os.path.getsize(fn) / 1e3:.0f} kB, sets {','.join(sets)}")


if __name__ == "__main__":
    main()
