"""somatic-sniper_amd -- MI355X-native SomaticSniper site scorer (Python host mirror).

The product is the C ABI in ``include/sniper_amd.h`` implemented by
``libsniper_amd.so`` (HIP kernels for gfx950 + host C).  This module is a thin
ctypes binding that mirrors the reference's interface for the scoring path:

=============================================  ===========================================
reference (src/lib/sniper/...)                 here
=============================================  ===========================================
``sniper_maqcns_init/prepare`` +               ``Context(params)`` (tables built on the
``qAddTableInit/makeSoloPrior/                 host, uploaded to the GPU)
make_joint_prior`` (main.c:115-127)
``sniper_maqcns_glfgen(n, pl, ref_base, bm)``  ``Context.sniper_maqcns_glfgen(reads, ref_char)``
(sniper_maqcns.c:127)
``sniper_glf2cns(g, q_r)`` (:250)               ``Context.sniper_glf2cns(...)`` (from the GPU
                                               consensus word)
``glf_somatic(tid,pos,n1,n2,pl1,pl2,d,fh)``    ``Context.glf_somatic(ref_char, reads_t, reads_n)``
(somatic_sniper.c:109)                         single site, same return value
``bam_sspileup_file`` driving the callback     ``Context.score_batch`` (host arrays) and
(sniper_pileup.c:226-266)                      ``Context.score_device`` (HBM-resident)
=============================================  ===========================================

There is no CPU fallback: if the shared library or a GPU is missing every entry
point raises.  (The CPU restatement under ``oracle/`` is test infrastructure and
is never imported from here.)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

__all__ = [
    "Params", "Synth", "Batch", "Context", "SniperError", "library_path", "load_library",
    "synth_batch_host", "model_check", "pack_read", "SS_GLF_DTYPE", "SS_CALL_DTYPE", "EXPORTED_SYMBOLS",
]

_HERE = os.path.dirname(os.path.abspath(__file__))

SS_OK, SS_E_INVAL, SS_E_HIP, SS_E_NOMEM, SS_E_TABLES, SS_E_CAPACITY, SS_E_NODEV = 0, -1, -2, -3, -4, -5, -6
SS_E_CORRUPT = -7

# every symbol include/sniper_amd.h declares
EXPORTED_SYMBOLS = (
    "ss_abi_version", "ss_strerror", "ss_params_default", "ss_ctx_create", "ss_ctx_destroy",
    "ss_score_batch_device", "ss_score_batch_host", "ss_ctx_check", "ss_table_hashes",
    "ss_table_copy", "ss_synth_default", "ss_synth_batch_host", "ss_synth_batch_device",
    "ss_set_kernel_timing", "ss_last_kernel_ms", "ss_kernel_time_log", "ss_kernel_time_log_k", "ss_model_check", "ss_model_pinned",
    "ss_model_last_source",
    "ss_host_alloc", "ss_host_free",
)


class SniperError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        lib = _LIB
        msg = lib.ss_strerror(code).decode() if lib is not None else str(code)
        super().__init__(f"{what}: {msg} (code {code})" if what else f"{msg} (code {code})")
        self.code = code


# --------------------------------------------------------------------------- structs
class Params(C.Structure):
    """ss_params_t -- CLI options of bam-somaticsniper (main.c:70-99)."""
    _fields_ = [
        ("theta", C.c_float), ("n_hap", C.c_int), ("het_rate", C.c_float), ("eta", C.c_float),
        ("cap_mapQ", C.c_int), ("min_somatic_qual", C.c_int), ("use_priors", C.c_int),
        ("use_joint_priors", C.c_int), ("somatic_rate", C.c_double), ("include_loh", C.c_int),
        ("include_gor", C.c_int),
    ]

    @classmethod
    def default(cls, **kw) -> "Params":
        p = cls()
        load_library().ss_params_default(C.byref(p))
        for k, v in kw.items():
            if not hasattr(p, k):
                raise AttributeError(k)
            setattr(p, k, v)
        return p


class _Batch(C.Structure):
    _fields_ = [("n_sites", C.c_uint64), ("ref", C.c_void_p), ("off_tumor", C.c_void_p),
                ("off_normal", C.c_void_p), ("reads_tumor", C.c_void_p),
                ("reads_normal", C.c_void_p)]


class _Out(C.Structure):
    _fields_ = [("score", C.c_void_p), ("calls", C.c_void_p), ("calls_cap", C.c_uint32),
                ("n_calls", C.c_void_p), ("glf", C.c_void_p), ("n_qadd_clamped", C.c_void_p)]


class Synth(C.Structure):
    """ss_synth_t -- deterministic synthetic pileup model."""
    _fields_ = [
        ("seed", C.c_uint64), ("shard", C.c_uint32), ("lambda_tumor", C.c_double),
        ("lambda_normal", C.c_double), ("fixed_depth", C.c_int), ("p_error", C.c_double),
        ("p_nbase", C.c_double), ("p_eq", C.c_double), ("p_iupac", C.c_double),
        ("p_del", C.c_double), ("p_mapq60", C.c_double), ("baseq_lo", C.c_int),
        ("baseq_hi", C.c_int), ("mapq_hi", C.c_int), ("p_wild_qual", C.c_double),
        ("p_somatic", C.c_double), ("vaf", C.c_double), ("p_germline", C.c_double),
        ("p_ref_n", C.c_double), ("p_ref_lower", C.c_double), ("p_ref_iupac", C.c_double),
    ]

    @classmethod
    def default(cls, lambda_tumor: float, lambda_normal: float, **kw) -> "Synth":
        s = cls()
        load_library().ss_synth_default(C.byref(s), C.c_double(lambda_tumor), C.c_double(lambda_normal))
        for k, v in kw.items():
            if not hasattr(s, k):
                raise AttributeError(k)
            setattr(s, k, v)
        return s


SS_GLF_DTYPE = np.dtype([("ref_base", "u1"), ("max_mapQ", "u1"), ("lk", "u1", (10,)),
                         ("min_lk", "u1"), ("pad", "u1"), ("depth", "<u4")], align=True)
SS_CALL_DTYPE = np.dtype([("site", "<u4"), ("somatic_score", "<i4"), ("cns_tumor", "<u4"),
                          ("cns_normal", "<u4"), ("joint_cq", "<i2"), ("snp_q_tumor", "u1"),
                          ("snp_q_normal", "u1"), ("joint_gt_tumor", "u1"),
                          ("joint_gt_normal", "u1"), ("status_tumor", "u1"),
                          ("status_normal", "u1"), ("ref_base4", "u1"), ("flags", "u1"),
                          ("pad", "<u2")], align=True)
assert SS_GLF_DTYPE.itemsize == 20 and SS_CALL_DTYPE.itemsize == 28


def pack_read(mapq: int, baseq: int, nt16: int, strand: int) -> int:
    """SS_READ_PACK: mapQ[7:0] baseQ[15:8] nt16[19:16] strand[20]."""
    return (mapq & 0xFF) | (baseq & 0xFF) << 8 | (nt16 & 0xF) << 16 | (strand & 1) << 20


@dataclass
class Batch:
    """A CSR batch of pileup sites (host numpy arrays)."""
    ref: np.ndarray          # u8 [n]
    off_tumor: np.ndarray    # u32 [n+1]
    off_normal: np.ndarray   # u32 [n+1]
    reads_tumor: np.ndarray  # u32
    reads_normal: np.ndarray  # u32

    @property
    def n_sites(self) -> int:
        return int(self.ref.shape[0])

    def site(self, i: int):
        t = self.reads_tumor[self.off_tumor[i]:self.off_tumor[i + 1]]
        n = self.reads_normal[self.off_normal[i]:self.off_normal[i + 1]]
        return int(self.ref[i]), t, n

    @classmethod
    def from_sites(cls, sites) -> "Batch":
        """sites: iterable of (ref_char:int|str, tumor_reads, normal_reads)."""
        ref, ot, on, rt, rn = [], [0], [0], [], []
        for r, t, n in sites:
            ref.append(ord(r) if isinstance(r, str) else int(r))
            rt.extend(int(x) for x in t)
            rn.extend(int(x) for x in n)
            ot.append(len(rt))
            on.append(len(rn))
        return cls(np.asarray(ref, np.uint8), np.asarray(ot, np.uint32), np.asarray(on, np.uint32),
                   np.asarray(rt, np.uint32), np.asarray(rn, np.uint32))

    def contiguous(self) -> "Batch":
        return Batch(*(np.ascontiguousarray(a) for a in (self.ref, self.off_tumor, self.off_normal,
                                                            self.reads_tumor, self.reads_normal)))

    def pinned(self) -> "Batch":
        """A copy whose arrays live in page-locked memory from ss_host_alloc
        (ss_score_batch_host then copies them to the device without staging).
        The memory is freed when the returned arrays are garbage-collected."""
        import weakref
        lib = load_library()
        out = []
        for a in (self.ref, self.off_tumor, self.off_normal, self.reads_tumor, self.reads_normal):
            nbytes = max(1, a.nbytes)
            p = lib.ss_host_alloc(nbytes)
            if not p:
                raise MemoryError("ss_host_alloc failed")
            buf = (C.c_char * nbytes).from_address(p)
            v = np.frombuffer(buf, dtype=a.dtype, count=a.size)
            v[...] = a
            weakref.finalize(buf, lib.ss_host_free, p)
            out.append(v)
        return Batch(*out)

    def algorithmic_bytes(self) -> int:
        """4 B per packed read + 16 B per site."""
        return 4 * (int(self.off_tumor[-1]) + int(self.off_normal[-1])) + 16 * self.n_sites


# --------------------------------------------------------------------------- library
_LIB = None


def library_path() -> str:
    return os.environ.get("SNIPER_AMD_LIB") or os.path.join(_HERE, "libsniper_amd.so")


def load_library():
    """Load libsniper_amd.so; raise loudly if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = library_path()
    if not os.path.exists(path):
        raise RuntimeError(f"libsniper_amd.so not found at {path}: run __graft_entry__.build() "
                           f"(make -C somatic-sniper_amd); there is no CPU fallback")
    if os.environ.get("SNIPER_AMD_NO_TORCH") != "1":
        # One HIP runtime per process: PyTorch ships its own libamdhip64 with the
        # same soname (libamdhip64.so.7).  Loading torch first makes our NEEDED
        # entry bind to torch's copy, so device pointers and streams handed over
        # from torch tensors live in the same runtime as our kernels.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = C.CDLL(path)
    vp, u64, u32 = C.c_void_p, C.c_uint64, C.c_uint32
    lib.ss_abi_version.restype = C.c_int
    lib.ss_strerror.restype = C.c_char_p
    lib.ss_strerror.argtypes = [C.c_int]
    lib.ss_params_default.argtypes = [vp]
    lib.ss_ctx_create.argtypes = [vp, C.c_int, C.POINTER(vp)]
    lib.ss_ctx_destroy.argtypes = [vp]
    lib.ss_score_batch_device.argtypes = [vp, vp, vp, vp]
    lib.ss_score_batch_host.argtypes = [vp, vp, vp]
    lib.ss_host_alloc.restype = vp
    lib.ss_host_alloc.argtypes = [C.c_size_t]
    lib.ss_host_free.argtypes = [vp]
    lib.ss_ctx_check.argtypes = [vp]
    lib.ss_table_hashes.argtypes = [vp, vp, vp, vp, vp]
    lib.ss_table_copy.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    lib.ss_synth_default.argtypes = [vp, C.c_double, C.c_double]
    lib.ss_synth_batch_host.argtypes = [vp, u64, u64, vp, vp, vp, vp, vp, vp, vp]
    lib.ss_synth_batch_device.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, vp]
    lib.ss_set_kernel_timing.argtypes = [vp, C.c_int]
    lib.ss_last_kernel_ms.argtypes = [vp]
    lib.ss_last_kernel_ms.restype = C.c_double
    lib.ss_model_check.argtypes = [vp, vp, vp]
    lib.ss_model_pinned.argtypes = [vp]
    if hasattr(lib, "ss_model_last_source"):      # absent from round-1 builds (A/B runs against them)
        lib.ss_model_last_source.restype = C.c_int
    lib.ss_kernel_time_log.argtypes = [vp, vp, C.c_int]
    lib.ss_kernel_time_log_k.argtypes = [vp, C.c_int, vp, C.c_int]
    if hasattr(lib, "ss__test_poke_table"):         # test hook, not in the public header
        lib.ss__test_poke_table.argtypes = [vp, u64, C.c_int]
    if hasattr(lib, "ss__test_route_counts"):       # test hook, not in the public header
        lib.ss__test_route_counts.argtypes = [vp, C.POINTER(C.c_uint32)]
    if lib.ss_abi_version() != 1:
        raise RuntimeError("libsniper_amd.so ABI mismatch")
    _LIB = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _check(rc: int, what: str):
    if rc != SS_OK:
        raise SniperError(rc, what)


def model_check(params: Params | None = None):
    """Build the model tables on the host (no GPU needed) and return their hashes and
    whether they equal a recorded run of the compiled reference (sniper_maqcns.c:27-100
    evaluated with this host's libm / x87, as the reference itself does)."""
    lib = load_library()
    p = params if params is not None else Params.default()
    h = (C.c_uint64 * 3)()
    qr = C.c_float()
    _check(lib.ss_model_check(C.byref(p), h, C.byref(qr)), "ss_model_check")
    return {"fk": f"{h[0]:016x}", "coef": f"{h[1]:016x}", "lhet": f"{h[2]:016x}", "q_r": qr.value,
            "pinned": bool(lib.ss_model_pinned(h)),
            "source": {0: "built", 1: "process", 2: "disk"}.get(
                lib.ss_model_last_source() if hasattr(lib, "ss_model_last_source") else -1, "none")}


def synth_batch_host(synth: Synth, first_site: int, n_sites: int) -> Batch:
    """Host twin of the device generator (bit-identical bytes)."""
    lib = load_library()
    ref = np.empty(n_sites, np.uint8)
    ot = np.empty(n_sites + 1, np.uint32)
    on = np.empty(n_sites + 1, np.uint32)
    nt, nn = C.c_uint64(), C.c_uint64()
    _check(lib.ss_synth_batch_host(C.byref(synth), first_site, n_sites, _ptr(ref), _ptr(ot), _ptr(on),
                                   None, None, C.byref(nt), C.byref(nn)), "ss_synth_batch_host")
    rt = np.empty(nt.value, np.uint32)
    rn = np.empty(nn.value, np.uint32)
    _check(lib.ss_synth_batch_host(C.byref(synth), first_site, n_sites, _ptr(ref), _ptr(ot), _ptr(on),
                                   _ptr(rt) or None, _ptr(rn) or None, C.byref(nt), C.byref(nn)),
           "ss_synth_batch_host")
    if nt.value == 0 or nn.value == 0:  # degenerate all-deleted batches
        rt = np.zeros(nt.value, np.uint32)
        rn = np.zeros(nn.value, np.uint32)
    return Batch(ref, ot, on, rt, rn)


class Context:
    """One scorer context on one GPU (sniper_maqcns_t + pu_data2_t equivalent)."""

    def __init__(self, params: Params | None = None, device: int = 0):
        self.lib = load_library()
        self.params = params if params is not None else Params.default()
        h = C.c_void_p()
        _check(self.lib.ss_ctx_create(C.byref(self.params), device, C.byref(h)), "ss_ctx_create")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.lib.ss_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- tables ------------------------------------------------------------------
    def table_hashes(self):
        fk, coef, lhet, qr = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_float()
        _check(self.lib.ss_table_hashes(self.h, C.byref(fk), C.byref(coef), C.byref(lhet),
                                        C.byref(qr)), "ss_table_hashes")
        return {"fk": f"{fk.value:016x}", "coef": f"{coef.value:016x}",
                "lhet": f"{lhet.value:016x}", "q_r": qr.value}

    # -- batches -----------------------------------------------------------------
    def score_batch(self, b: Batch, calls_cap: int | None = None, want_glf: bool = False):
        """Score a host batch; returns (score[n] i32, calls structured array, glf or None)."""
        b = b.contiguous()
        n = b.n_sites
        score = np.empty(n, np.int32)
        cap = max(16, n // 64) if calls_cap is None else calls_cap
        calls = np.zeros(cap, SS_CALL_DTYPE)
        glf = np.zeros((n, 2), SS_GLF_DTYPE) if want_glf else None
        ncalls, nclamp = C.c_uint32(), C.c_uint32()
        bt = _Batch(n, _ptr(b.ref), _ptr(b.off_tumor), _ptr(b.off_normal), _ptr(b.reads_tumor),
                    _ptr(b.reads_normal))
        out = _Out(_ptr(score), _ptr(calls), cap, C.addressof(ncalls),
                   _ptr(glf) if want_glf else None, C.addressof(nclamp))
        rc = self.lib.ss_score_batch_host(self.h, C.byref(bt), C.byref(out))
        if rc == SS_E_CAPACITY and ncalls.value > cap and calls_cap is None:
            return self.score_batch(b, calls_cap=int(ncalls.value), want_glf=want_glf)
        _check(rc, "ss_score_batch_host")
        self.last_clamped = int(nclamp.value)
        return score, calls[: min(ncalls.value, cap)].copy(), glf

    def score_device(self, ref, off_t, off_n, reads_t, reads_n, score, calls=None, calls_cap=0,
                     n_calls=None, glf=None, stream=None, n_sites=None):
        """Score an HBM-resident batch; arguments are torch CUDA tensors (or raw ints).
        Asynchronous on `stream` (torch.cuda.Stream or raw handle)."""
        def p(x):
            if x is None:
                return None
            return x if isinstance(x, int) else x.data_ptr()
        n = int(n_sites if n_sites is not None else ref.numel())
        bt = _Batch(n, p(ref), p(off_t), p(off_n), p(reads_t), p(reads_n))
        out = _Out(p(score), p(calls), calls_cap, p(n_calls), p(glf), None)
        sh = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        _check(self.lib.ss_score_batch_device(self.h, C.byref(bt), C.byref(out), sh),
               "ss_score_batch_device")

    def synth_device(self, synth: Synth, first_site: int, n_sites: int, device=None):
        """Generate a synthetic batch directly in HBM; returns torch tensors."""
        import torch
        dev = device if device is not None else torch.device("cuda", self.device)
        ref = torch.empty(n_sites, dtype=torch.uint8, device=dev)
        ot = torch.empty(n_sites + 1, dtype=torch.int32, device=dev)
        on = torch.empty(n_sites + 1, dtype=torch.int32, device=dev)
        nt, nn = C.c_uint64(), C.c_uint64()
        torch.cuda.synchronize(dev)
        _check(self.lib.ss_synth_batch_device(self.h, C.byref(synth), first_site, n_sites,
                                              ref.data_ptr(), ot.data_ptr(), on.data_ptr(), None, None,
                                              C.byref(nt), C.byref(nn)), "ss_synth_batch_device")
        rt = torch.empty(max(1, nt.value), dtype=torch.int32, device=dev)
        rn = torch.empty(max(1, nn.value), dtype=torch.int32, device=dev)
        _check(self.lib.ss_synth_batch_device(self.h, C.byref(synth), first_site, n_sites,
                                              ref.data_ptr(), ot.data_ptr(), on.data_ptr(),
                                              rt.data_ptr(), rn.data_ptr(), C.byref(nt), C.byref(nn)),
               "ss_synth_batch_device")
        return {"ref": ref, "off_tumor": ot, "off_normal": on, "reads_tumor": rt,
                "reads_normal": rn, "n_reads": (int(nt.value), int(nn.value)), "n_sites": n_sites}

    def check(self):
        _check(self.lib.ss_ctx_check(self.h), "device work")

    def _poke_table(self, byte_offset: int, value: int):
        """Test hook: overwrite one byte of the device tables (ss_ctx_check must then fail)."""
        _check(self.lib.ss__test_poke_table(self.h, byte_offset, value), "ss__test_poke_table")

    def _route_counts(self):
        """Test hook: the latest launch's routing -- the deep triage's blocks,
        the sites left to the main kernel, those it queued for the group and
        the deep kernels."""
        out = (C.c_uint32 * 4)()
        _check(self.lib.ss__test_route_counts(self.h, out), "ss__test_route_counts")
        return {"deep_triage_blocks": out[0], "main_sites": out[1], "group_sites": out[2], "deep_sites": out[3]}

    def set_kernel_timing(self, enable: bool):
        _check(self.lib.ss_set_kernel_timing(self.h, 1 if enable else 0), "ss_set_kernel_timing")

    def last_kernel_ms(self) -> float:
        return float(self.lib.ss_last_kernel_ms(self.h))

    KERNELS = {"main": 0, "wide": 1, "deep": 2, "all": 3}   # SS_KT_*

    def kernel_time_log(self, kernel: str = "main") -> np.ndarray:
        """Durations (ms) of one kernel of every launch since set_kernel_timing(True):
        "main" (ss_score_main), "wide" (ss_score_group: the wide list), "deep" (ss_score_deep) or "all" (the launch)."""
        buf = np.zeros(4096, np.float64)
        n = self.lib.ss_kernel_time_log_k(self.h, self.KERNELS[kernel], buf.ctypes.data, buf.size)
        if n < 0:
            raise SniperError(n, "ss_kernel_time_log_k")
        return buf[:n].copy()

    # -- reference-named single-site helpers ---------------------------------------
    def glf_somatic(self, ref_char, reads_tumor, reads_normal) -> int:
        """Return value of glf_somatic (somatic_sniper.c:109) for one site, on the GPU."""
        s, _, _ = self.score_batch(Batch.from_sites([(ref_char, reads_tumor, reads_normal)]))
        return int(s[0])

    def sniper_maqcns_glfgen(self, reads, ref_char):
        """glf1_t of one sample (sniper_maqcns.c:127) computed by the GPU kernel."""
        _, _, g = self.score_batch(Batch.from_sites([(ref_char, reads, [pack_read(60, 30, 1, 0)])]),
                                   want_glf=True)
        return g[0, 0]

    @staticmethod
    def sniper_glf2cns_fields(cns: int):
        """Decode a consensus word: (cns, cns2, rms_mapQ, cnsQ, cnsQ2) (sniper_maqcns.h:28)."""
        return cns >> 28, (cns >> 24) & 0xF, (cns >> 16) & 0xFF, (cns >> 8) & 0xFF, cns & 0xFF
