"""The CPU oracle (oracle/ss_oracle.c) against golden vectors produced by the REAL
reference (tests/golden/make_golden.py drives oracle/_ref/ref_harness, i.e.
glf_somatic / sniper_maqcns_glfgen compiled from /root/reference).

Bit-exact: every site's glf_somatic return value for every option set, both
glf1_t records and both consensus words for the model-changing option sets, and
the set of emitted sites (== number and positions of the reference's output
lines).  The reference's coef table is CPU-dependent (x87 expl/logl, DESIGN.md
"Tables"); the fixtures were made on the build host, so on a host whose tables
differ the test is skipped rather than compared against another machine's run.
"""
import glob
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))
BUILD_HOST_COEF = "86dcc255eecf756d"

OPTSETS = {"default": [], "J": ["-J"], "p": ["-p"], "s1e-6": ["-s", "1e-6"],
           "TNr": ["-T", "0.9", "-N", "3", "-r", "0.01"], "Q0LG": ["-Q", "0", "-L", "-G"],
           "JpQ0": ["-J", "-p", "-Q", "0"], "L": ["-L"], "G": ["-G"]}


def _fnv(b):
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


@pytest.fixture(scope="module")
def same_tables_as_build_host(oracle):
    t = oracle.Oracle().tables()
    if _fnv(t["coef"].tobytes()) != BUILD_HOST_COEF:
        pytest.skip("this host's reference tables differ from the build host's (x87 expl/logl)")


def test_golden_files_present():
    names = {os.path.basename(p) for p in GOLDEN}
    assert {"c30.npz", "c60x.npz", "c100.npz", "low.npz", "deep.npz", "deep300.npz", "quirks.npz"} <= names


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_oracle_matches_reference_golden(oracle, same_tables_as_build_host, path):
    z = np.load(path, allow_pickle=False)
    args = (z["ref"], z["off_tumor"], z["off_normal"], z["reads_tumor"], z["reads_normal"])
    n = z["ref"].shape[0]
    sets = [k[4:] for k in z.files if k.startswith("ret_")]
    assert sets
    for s in sets:
        o = oracle.Oracle(oracle.opts_to_params(OPTSETS[s]))
        score, calls, glf = o.score_batch(*args)
        ref_ret = z[f"ret_{s}"]
        bad = np.nonzero(score != ref_ret)[0]
        assert bad.size == 0, f"{s}: sites {bad[:5]} oracle {score[bad[:5]]} reference {ref_ret[bad[:5]]}"
        if f"glf_{s}" in z.files:
            g = glf.view(np.uint8).reshape(n, -1)
            assert (g == z[f"glf_{s}"]).all(), s
            q_r = int(o.lib.orc_model_q_r(o.m) + 0.5)
            cns = np.array([[o.lib.orc_glf2cns(glf[i:i + 1, m].ctypes.data, q_r) for m in (0, 1)]
                            for i in range(n)], np.uint32)
            live = ref_ret >= 0          # glf2cns only runs past the depth gate
            assert (cns[live] == z[f"cns_{s}"][live]).all(), s
        if s == "default":
            # emitted sites: one classic line per call, position column = site + 1
            lines = bytes(z["classic_default"]).decode().splitlines()
            assert len(lines) == len(calls)
            pos = [int(l.split("\t")[1]) - 1 for l in lines]
            assert pos == calls["site"].tolist()
            # tumor/normal genotype + SSC columns follow from the call record
            rev = "=ACMGRSVTWYHKDBN"
            for l, c in zip(lines, calls):
                f = l.split("\t")
                assert f[3] == rev[c["cns_tumor"] >> 28] and f[4] == rev[c["cns_normal"] >> 28]
                assert int(f[5]) == c["somatic_score"]
                assert int(f[6]) == (c["cns_tumor"] >> 8) & 0xFF
                assert int(f[7]) == c["snp_q_tumor"] and int(f[10]) == c["snp_q_normal"]


def test_reference_named_entry_points(oracle, same_tables_as_build_host):
    """The model API under the reference's names (SURVEY.md section 8b:
    ss_maqcns_init / ss_maqcns_glfgen / ss_glf2cns / ss_glf_somatic /
    ss_maqcns_destroy), called site by site as sniper_pileup.c:256-258 calls
    glf_somatic, against the reference's golden returns, glf records and
    consensus words."""
    import ctypes as C
    z = np.load(os.path.join(HERE, "golden", "c60x.npz"), allow_pickle=False)
    lib = oracle.load()
    o = oracle.Oracle()                                  # default params, as z's "default" set
    m = lib.ss_maqcns_init(C.byref(o.params))
    assert m
    try:
        q_r = int(lib.orc_model_q_r(m) + 0.5)
        ot, on = z["off_tumor"], z["off_normal"]
        rt = np.ascontiguousarray(z["reads_tumor"], np.uint32)
        rn = np.ascontiguousarray(z["reads_normal"], np.uint32)
        call = (C.c_uint8 * 64)()
        n = min(400, z["ref"].shape[0])
        glf_ref = z["glf_default"]                       # (n, 2 x 20 B ss_glf_t)
        gsz = glf_ref.shape[1] // 2
        for i in range(n):
            g2 = (C.c_uint8 * 64)()
            nt, nn = int(ot[i + 1] - ot[i]), int(on[i + 1] - on[i])
            pt = rt[ot[i]:].ctypes.data if nt else None
            pn = rn[on[i]:].ctypes.data if nn else None
            r = lib.ss_glf_somatic(m, int(z["ref"][i]), nt, pt, nn, pn, g2, C.byref(g2, gsz), call)
            assert r == int(z["ret_default"][i]), i
            assert bytes(g2)[:2 * gsz] == glf_ref[i].tobytes(), i
            if r >= 0:
                cns = [lib.ss_glf2cns(C.byref(g2, k * gsz), q_r) for k in (0, 1)]
                assert cns == z["cns_default"][i].tolist(), i
            # glfgen alone (tumor) equals glf_somatic's tumor record
            g1 = (C.c_uint8 * 64)()
            lib.ss_maqcns_glfgen(m, nt, pt, int(lib.orc_nt16_of(int(z["ref"][i]))), g1)
            assert bytes(g1)[:gsz] == bytes(g2)[:gsz], i
    finally:
        lib.ss_maqcns_destroy(m)
