"""Sanitizer builds of the host code (ASan/UBSan/TSan on the host C).

`make -C somatic-sniper_amd sanitize` builds the native CLI (threaded BGZF
reader + inflate pool, column-pileup reader and window builders, the
pileup -> scorer batch ring) with ASan+UBSan and with TSan, and the threaded
table builder / disk cache / host generator (tests/native/tables_driver.c).
The CLIs run pileup-only (SS_PILEUP_ONLY=1: the GPU scorer is never created)
over every test dataset in all three pileup modes; their site streams must
equal the reference's and the sanitizers must stay silent (halt on the first
report, leak check on).  CPU only: no GPU code is instrumented."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "somatic-sniper_amd", "build", "san")
REF_DUMP = os.path.join(ROOT, "oracle", "_ref", "bam-somaticsniper-dump")
ENV = {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=1:abort_on_error=0",
       "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
       "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "somatic-sniper_amd"), "sanitize"], check=True,
                   capture_output=True, timeout=600)
    return SAN


def _run(cmd, cwd, env):
    return subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=900,
                          env=dict(os.environ, **ENV, **env))


@pytest.mark.skipif(not os.path.exists(REF_DUMP), reason="reference dump CLI not built")
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_cli_pileup_under_sanitizers(san_build, datasets, kind):
    cli = os.path.join(san_build, f"bam-somaticsniper-{kind}")
    for d, fa, t, n in datasets:
        ref_name = "ref_san.dump"
        p = _run([REF_DUMP, "-f", fa, t, n, "ref_san.out"], d, {"SS_DUMP_PILEUP": ref_name})
        assert p.returncode == 0, p.stderr
        ref = open(os.path.join(d, ref_name), "rb").read() if os.path.exists(os.path.join(d, ref_name)) else b""
        for mode in ("2", "1", "0"):
            name = f"{kind}_{mode}.dump"
            p = _run([cli, "-f", fa, t, n, f"{kind}.out"], d,
                     {"SS_PILEUP_ONLY": "1", "SS_PILEUP_THREADS": mode, "SS_DUMP_PILEUP": name})
            assert p.returncode == 0 and "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, \
                (d, mode, p.stderr[-3000:])
            path = os.path.join(d, name)
            got = open(path, "rb").read() if os.path.exists(path) else b""
            assert got == ref, (d, kind, mode)


@pytest.mark.skipif(not os.path.exists(REF_DUMP), reason="reference dump CLI not built")
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_contig_groups_under_sanitizers(san_build, datasets, tmp_path, kind):
    """The contig-parallel pileup (indexed copies of the datasets, 3 ranges:
    per range two seeked BGZF readers with inflate pools, two column streams
    and the merge, the ranges' memory streams concatenated at the end) under
    ASan/UBSan and TSan; site streams equal the reference's."""
    import shutil
    index = os.path.join(ROOT, "somatic-sniper_amd", "ss-index")
    if not os.path.exists(index):
        pytest.skip("ss-index not built")
    cli = os.path.join(san_build, f"bam-somaticsniper-{kind}")
    for i, (d, fa, t, n) in enumerate(datasets):
        dst = tmp_path / f"s{i}"
        dst.mkdir()
        for f in os.listdir(d):
            if f.endswith((".bam", ".fa", ".fai")):
                shutil.copy(os.path.join(d, f), dst / f)
        if any(subprocess.run([index, b], cwd=str(dst), capture_output=True).returncode for b in (t, n)):
            continue                          # the unsorted pair: no index, streaming walk
        p = _run([REF_DUMP, "-f", fa, t, n, "ref_g.out"], str(dst), {"SS_DUMP_PILEUP": "ref_g.dump"})
        assert p.returncode == 0, p.stderr
        ref = (dst / "ref_g.dump").read_bytes() if (dst / "ref_g.dump").exists() else b""
        p = _run([cli, "-f", fa, t, n, "g.out"], str(dst),
                 {"SS_PILEUP_ONLY": "1", "SS_CONTIG_GROUPS": "3", "SS_DUMP_PILEUP": "g.dump"})
        assert p.returncode == 0 and "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, \
            (d, p.stderr[-3000:])
        got = (dst / "g.dump").read_bytes() if (dst / "g.dump").exists() else b""
        assert got == ref, (d, kind)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_table_builder_under_sanitizers(san_build, tmp_path, kind):
    """Four threads building two parameter sets at once (8 coef threads each),
    through the process cache and a fresh disk cache, then the host generator."""
    exe = os.path.join(san_build, f"tables-{kind}")
    for _ in range(2):                       # second run loads the blobs the first wrote
        p = _run([exe], str(tmp_path), {"SS_TABLE_CACHE": str(tmp_path / "cache")})
        assert p.returncode == 0 and "ok=1" in p.stdout, p.stderr[-3000:]
        assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-3000:]
