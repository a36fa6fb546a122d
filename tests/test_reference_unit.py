"""The reference's own unit tests, ported ("port as own tests").

* test/lib/sniper/TestAlleleUtil.cpp -- count_alleles, genotype_set_difference,
  the exhaustive 14x14 is_loh matrix and the should_filter_as_loh / _gor cases,
  asserted on `allele_util` below: a restatement of allele_util.c:13-28 /
  allele_util.h:23-35 that is also the expectation the GPU decision test
  (test_decision_matrix_gpu) checks the kernel's emit flags and statuses against.
* test/lib/sniper/TestDqStats.cpp -- print_mean_quality_values' strings, on the
  native CLI's printer (cli/sniper_output.c ss_put_masked).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
A, C, G, T = 1, 2, 4, 8


class allele_util:
    """allele_util.c / allele_util.h, restated (genotypes as nt16 bit sets)."""
    @staticmethod
    def count_alleles(a):
        return (a & 1) + ((a >> 1) & 1) + ((a >> 2) & 1) + ((a >> 3) & 1)

    @staticmethod
    def genotype_set_difference(a, b):
        return a & ~b

    @staticmethod
    def is_proper_subset(a, b):
        return b != a and (a & b) == a

    is_loh = is_proper_subset

    @classmethod
    def should_filter_as_loh(cls, ref, tumor, normal):
        return int(cls.is_proper_subset(tumor, normal))

    @classmethod
    def should_filter_as_gor(cls, ref, tumor, normal):
        return int(not cls.is_proper_subset(ref, normal) and cls.genotype_set_difference(tumor, normal) == ref)


U = allele_util


# ------------------------------------------------------------- TestAlleleUtil.cpp
def test_count_alleles():
    for v, n in [(0, 0), (A, 1), (C, 1), (A | C, 2), (G, 1), (A | G, 2), (C | G, 2), (A | C | G, 3), (T, 1),
                 (A | T, 2), (C | T, 2), (A | C | T, 3), (G | T, 2), (A | G | T, 3), (A | C | T | G, 4)]:
        assert U.count_alleles(v) == n


def test_genotype_set_difference():
    assert U.genotype_set_difference(A | C, C) == A
    assert U.genotype_set_difference(A | C | G, C) == A | G
    assert U.genotype_set_difference(A | C, A | C) == 0
    assert U.genotype_set_difference(A, A | C) == 0


LOH_PAIRS = [(A, A | C), (C, A | C), (A, A | G), (G, A | G), (A, A | T), (T, A | T), (C, C | G), (G, C | G),
             (C, C | T), (T, C | T), (G, G | T), (T, G | T),
             (A, A | C | G), (C, A | C | G), (G, A | C | G), (A | C, A | C | G), (A | G, A | C | G), (C | G, A | C | G),
             (A, A | C | T), (C, A | C | T), (T, A | C | T), (A | C, A | C | T), (A | T, A | C | T), (C | T, A | C | T),
             (A, A | G | T), (G, A | G | T), (T, A | G | T), (A | G, A | G | T), (A | T, A | G | T), (G | T, A | G | T),
             (C, C | G | T), (G, C | G | T), (T, C | G | T), (C | G, C | G | T), (C | T, C | G | T), (G | T, C | G | T)]


def test_is_loh_matrix():
    for i in range(4):                                    # single alleles: never LOH
        for j in range(1, 9):
            assert not U.is_loh(j, 1 << i)
    for orig in range(1, 15):                             # the exhaustive 14 x 14 matrix
        for mut in range(1, 15):
            assert U.is_loh(mut, orig) == ((mut, orig) in LOH_PAIRS), (mut, orig)
    for i in range(1, 15):                                # N
        assert U.is_loh(i, A | C | G | T)


def test_should_filter_as_loh():
    ref = A
    assert U.should_filter_as_loh(ref, A, A | G) and U.should_filter_as_loh(ref, G, A | G)
    assert U.should_filter_as_loh(ref, G, C | G) and U.should_filter_as_loh(ref, C, C | G)
    assert not U.is_loh(A | G, G) and U.is_loh(G, A | G)
    assert not U.should_filter_as_loh(ref, A | G, G)
    for i in range(1, 15):
        assert not U.should_filter_as_loh(A, i, A)
        assert not U.should_filter_as_loh(A, i, i)
    assert not U.should_filter_as_loh(A, A | C | G, A | C)
    assert not U.should_filter_as_loh(A, A | T, A | C)
    assert not U.should_filter_as_loh(A, T, A | C)
    assert not U.should_filter_as_loh(A, T | G, G)
    assert not U.should_filter_as_loh(A, C | G, G)
    assert not U.should_filter_as_loh(A, A | G, G)
    assert not U.should_filter_as_loh(A, A, G)


def test_should_filter_as_gor():
    ref = A
    assert U.should_filter_as_gor(ref, A, G) and U.should_filter_as_gor(ref, A | G, G)
    assert U.should_filter_as_gor(ref, A | G, C | G) and U.should_filter_as_gor(ref, T | A, T | G)
    assert U.should_filter_as_gor(A, A, G)
    for i in range(1, 15):
        assert not U.should_filter_as_gor(A, i, A)
        assert not U.should_filter_as_gor(A, i, i)
    assert not U.should_filter_as_gor(A, A | C | G, A | C)
    assert not U.should_filter_as_gor(A, A | T, A | C)
    assert not U.should_filter_as_gor(A, T, A | C)
    assert U.should_filter_as_gor(A, A | T | C, T | C)
    assert not U.should_filter_as_gor(A, T | G, G)
    assert not U.should_filter_as_gor(A, C | G, G)


# ---------------------------------------------------------------- TestDqStats.cpp
@pytest.fixture(scope="module")
def out_lib(tmp_path_factory):
    so = tmp_path_factory.mktemp("cliout") / "libsniper_output.so"
    cli = os.path.join(ROOT, "somatic-sniper_amd", "cli")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-I", cli, "-I", os.path.join(ROOT, "include"), "-o", str(so),
                    os.path.join(cli, "sniper_output.c")], check=True)
    lib = ctypes.CDLL(str(so))
    lib.ss_put_masked.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
    return lib


def _printed(out_lib, bases, vals):
    libc = ctypes.CDLL(None)
    libc.tmpfile.restype = ctypes.c_void_p
    libc.fseek.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int]
    libc.fread.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    fh = libc.tmpfile()
    out_lib.ss_put_masked(fh, bases, (ctypes.c_uint32 * 4)(*vals))
    libc.fseek(fh, 0, 0)
    buf = ctypes.create_string_buffer(4096)
    n = libc.fread(buf, 1, 4095, fh)
    libc.fclose(fh)
    return buf.raw[:n].decode()


def test_print_mean_quality_values(out_lib):
    qual = [1, 2, 3, 4]
    assert _printed(out_lib, 1, qual) == "1"
    assert _printed(out_lib, 6, qual) == "2,3"
    assert _printed(out_lib, 3, qual) == "1,2"
    assert _printed(out_lib, 0, qual) == "0"


# ------------------------------------------- the decision kernel on the same rules
GENOTYPES = [A, C, G, T, A | C, A | G, A | T, C | G, C | T, G | T]   # what glf2cns can call (diploid)
STATUS = {"WILDTYPE": 0, "GERMLINE": 1, "SOMATIC": 2, "LOH": 3, "UNKNOWN": 4}   # allele_util.h:14-20


def _reads(pkg, gt, n=24):
    """n high-quality reads supporting genotype gt (hom: all one base; het: half/half)."""
    bases = [b for b in (A, C, G, T) if gt & b]
    return [pkg.pack_read(60, 40, bases[i % len(bases)], i & 1) for i in range(n)]


def decision_sites(pkg):
    sites, want = [], []
    for ref in "ACGT":
        for tg in GENOTYPES:
            for ng in GENOTYPES:
                sites.append((ref, _reads(pkg, tg), _reads(pkg, ng)))
                want.append(({"A": A, "C": C, "G": G, "T": T}[ref], tg, ng))
    return sites, want


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [["-Q", "0"], ["-Q", "0", "-L"], ["-Q", "0", "-G"], ["-Q", "0", "-L", "-G"]])
def test_decision_matrix_gpu(pkg, oracle, opts):
    """Every (ref, tumor genotype, normal genotype) the consensus caller can
    produce (4 x 10 x 10 sites; the 3-allele and N genotypes of the 14 x 14
    matrix cannot come out of sniper_glf2cns), under -L / -G: the kernel's
    emit decisions and statuses equal allele_util's rules (somatic_sniper.c:
    216-262) and the oracle, bit for bit."""
    from test_gpu_parity import assert_parity, params_from_opts
    sites, want = decision_sites(pkg)
    batch = pkg.Batch.from_sites(sites)
    score, calls = assert_parity(pkg, oracle, batch, opts)
    p = params_from_opts(pkg, opts)
    by_site = {int(c["site"]): c for c in calls}
    n_emit = 0
    for i, (rb4, tg, ng) in enumerate(want):
        assert score[i] != -1
        candidate = tg != ng                                 # rb4, t1, n1 never 15 here
        if not candidate:
            assert score[i] == 255 and i not in by_site
            continue
        qps = int(score[i])
        emit = (p.min_somatic_qual <= qps and (p.include_loh or not U.should_filter_as_loh(rb4, tg, ng))
                and (p.include_gor or not U.should_filter_as_gor(rb4, tg, ng)))
        assert (i in by_site) == emit, (i, rb4, tg, ng, qps, opts)
        if emit:
            n_emit += 1
            c = by_site[i]
            assert (int(c["cns_tumor"]) >> 28, int(c["cns_normal"]) >> 28) == (tg, ng)
            st = ("GERMLINE" if tg == ng else "LOH" if U.is_loh(tg, ng) else "SOMATIC" if qps > 0 else "UNKNOWN")
            assert c["status_tumor"] == STATUS[st]
            assert c["status_normal"] == STATUS["WILDTYPE" if ng == rb4 else "GERMLINE"]
    assert n_emit > 50
