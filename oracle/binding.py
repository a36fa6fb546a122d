"""oracle/binding.py -- ctypes binding of the CPU restatement (oracle/ss_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the CHECKER.  The product package never
imports anything under oracle/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")
REF_CLI = os.path.join(HERE, "_ref", "bam-somaticsniper")

GLF_DTYPE = np.dtype([("ref_base", "u1"), ("max_mapQ", "u1"), ("lk", "u1", (10,)),
                      ("min_lk", "u1"), ("pad", "u1"), ("depth", "<u4")], align=True)
CALL_DTYPE = np.dtype([("site", "<u4"), ("somatic_score", "<i4"), ("cns_tumor", "<u4"),
                       ("cns_normal", "<u4"), ("joint_cq", "<i2"), ("snp_q_tumor", "u1"),
                       ("snp_q_normal", "u1"), ("joint_gt_tumor", "u1"), ("joint_gt_normal", "u1"),
                       ("status_tumor", "u1"), ("status_normal", "u1"), ("ref_base4", "u1"),
                       ("flags", "u1"), ("pad", "<u2")], align=True)
# per-site record written by `ref_harness dump`: ret, cnsT, cnsN, glfT, glfN
REF_SITE_DTYPE = np.dtype([("ret", "<i4"), ("cns_tumor", "<u4"), ("cns_normal", "<u4"),
                           ("glf", GLF_DTYPE, (2,))], align=True)


class OParams(C.Structure):
    _fields_ = [
        ("theta", C.c_float), ("n_hap", C.c_int), ("het_rate", C.c_float), ("eta", C.c_float),
        ("cap_mapQ", C.c_int), ("min_somatic_qual", C.c_int), ("use_priors", C.c_int),
        ("use_joint_priors", C.c_int), ("somatic_rate", C.c_double), ("include_loh", C.c_int),
        ("include_gor", C.c_int),
    ]


def oparams(theta=0.85, n_hap=2, het_rate=0.001, min_q=15, priors=True, joint=False,
            rate=0.01, loh=True, gor=True) -> OParams:
    return OParams(theta, n_hap, het_rate, 0.03, 60, min_q, int(priors), int(joint), rate,
                   int(loh), int(gor))


def opts_to_params(opts: list[str]) -> OParams:
    """CLI-style option list (-T -N -r -p -J -s -Q -L -G) -> OParams (main.c:80-99)."""
    kw = {}
    it = iter(opts)
    for o in it:
        if o == "-T": kw["theta"] = float(next(it))
        elif o == "-N": kw["n_hap"] = int(next(it))
        elif o == "-r": kw["het_rate"] = float(next(it))
        elif o == "-p": kw["priors"] = False
        elif o == "-J": kw["joint"] = True
        elif o == "-s": kw["rate"] = float(next(it)); kw["joint"] = True
        elif o == "-Q": kw["min_q"] = int(next(it))
        elif o == "-L": kw["loh"] = False
        elif o == "-G": kw["gor"] = False
        elif o == "-F": next(it)
        else: raise ValueError(o)
    return oparams(**kw)


_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        lib.orc_model_create.argtypes = [vp]
        lib.orc_model_create.restype = vp
        lib.orc_model_destroy.argtypes = [vp]
        for f in ("orc_model_fk", "orc_model_coef", "orc_model_lhet"):
            getattr(lib, f).argtypes = [vp]
            getattr(lib, f).restype = C.POINTER(C.c_double)
        for f in ("orc_model_qadd", "orc_model_prior", "orc_model_jprior"):
            getattr(lib, f).argtypes = [vp]
            getattr(lib, f).restype = C.POINTER(C.c_int)
        lib.orc_model_q_r.argtypes = [vp]
        lib.orc_model_q_r.restype = C.c_float
        lib.orc_nt16_of.argtypes = [C.c_int]
        lib.orc_score_batch.argtypes = [vp, C.c_uint64, vp, vp, vp, vp, vp, vp, vp, vp, C.c_long]
        lib.orc_score_batch.restype = C.c_long
        lib.orc_glfgen.argtypes = [vp, vp, C.c_int, C.c_int, vp]
        lib.orc_glf2cns.argtypes = [vp, C.c_int]
        lib.orc_glf2cns.restype = C.c_uint32
        # the reference's entry points under ss_ names (ss_oracle.c, end of file)
        lib.ss_maqcns_init.argtypes = [vp]
        lib.ss_maqcns_init.restype = vp
        lib.ss_maqcns_destroy.argtypes = [vp]
        lib.ss_maqcns_glfgen.argtypes = [vp, C.c_int, vp, C.c_int, vp]
        lib.ss_glf2cns.argtypes = [vp, C.c_int]
        lib.ss_glf2cns.restype = C.c_uint32
        lib.ss_glf_somatic.argtypes = [vp, C.c_int, C.c_int, vp, C.c_int, vp, vp, vp, vp]
        lib.ss_glf_somatic.restype = C.c_int
        _LIB = lib
    return _LIB


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


class Oracle:
    """CPU restatement of the scorer for one parameter set."""

    def __init__(self, params: OParams | None = None):
        self.lib = load()
        self.params = params if params is not None else oparams()
        self.m = self.lib.orc_model_create(C.byref(self.params))

    def __del__(self):
        if getattr(self, "m", None):
            self.lib.orc_model_destroy(self.m)
            self.m = None

    def tables(self):
        L, m = self.lib, self.m
        fk = np.ctypeslib.as_array(L.orc_model_fk(m), (256,)).copy()
        coef = np.ctypeslib.as_array(L.orc_model_coef(m), (64 << 16,)).copy()
        lhet = np.ctypeslib.as_array(L.orc_model_lhet(m), (65536,)).copy()
        qadd = np.ctypeslib.as_array(L.orc_model_qadd(m), (1024,)).copy()
        prior = np.ctypeslib.as_array(L.orc_model_prior(m), (160,)).copy()
        jprior = np.ctypeslib.as_array(L.orc_model_jprior(m), (1600,)).copy()
        return {"fk": fk, "coef": coef, "lhet": lhet, "q_r": L.orc_model_q_r(m), "qadd": qadd,
                "prior": prior, "jprior": jprior}

    def score_batch(self, ref, off_t, off_n, reads_t, reads_n, want_glf=True):
        n = int(ref.shape[0])
        ref = np.ascontiguousarray(ref, np.uint8)
        off_t = np.ascontiguousarray(off_t, np.uint32)
        off_n = np.ascontiguousarray(off_n, np.uint32)
        reads_t = np.ascontiguousarray(reads_t, np.uint32)
        reads_n = np.ascontiguousarray(reads_n, np.uint32)
        score = np.empty(n, np.int32)
        glf = np.zeros((n, 2), GLF_DTYPE) if want_glf else None
        cap = max(64, n // 16)
        calls = np.zeros(cap, CALL_DTYPE)
        ne = self.lib.orc_score_batch(self.m, n, _p(ref), _p(off_t), _p(off_n), _p(reads_t),
                                      _p(reads_n), _p(score), _p(glf), _p(calls), cap)
        if ne > cap:
            calls = np.zeros(ne, CALL_DTYPE)
            self.lib.orc_score_batch(self.m, n, _p(ref), _p(off_t), _p(off_n), _p(reads_t),
                                     _p(reads_n), _p(score), _p(glf), _p(calls), ne)
        return score, calls[:ne], glf


# ---------------------------------------------------------------------- files
def write_ssb(path, ref, off_t, off_n, reads_t, reads_n):
    """SSB1 batch file consumed by `ref_harness dump`."""
    n = int(ref.shape[0])
    nt, nn = int(off_t[-1]), int(off_n[-1])
    with open(path, "wb") as f:
        f.write(b"SSB1" + np.uint32(1).tobytes() + np.array([n, nt, nn], "<u8").tobytes())
        r = np.zeros((n + 3) & ~3, np.uint8)
        r[:n] = ref
        f.write(r.tobytes())
        for a in (off_t, off_n):
            f.write(np.ascontiguousarray(a, "<u4").tobytes())
        for a, k in ((reads_t, nt), (reads_n, nn)):
            f.write(np.ascontiguousarray(a[:k], "<u4").tobytes())


def run_ref_dump(batch_path, opts, workdir):
    """Run the compiled reference on a batch file; returns (sites record array, text)."""
    out = os.path.join(workdir, "ref.ssr")
    txt = os.path.join(workdir, "ref.txt")
    subprocess.run([REF_HARNESS, "dump", batch_path, out, txt] + list(opts), check=True)
    rec = np.fromfile(out, REF_SITE_DTYPE)
    with open(txt) as f:
        return rec, f.read()
