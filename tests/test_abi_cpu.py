"""CPU-only checks of the product library: it loads, exports every symbol the
header declares, builds bit-exact host tables, and its host synthetic generator
is deterministic.  No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# FNV-1a-64 of the reference's own tables (oracle/_ref/ref_harness tables).
REF_HASHES = {"fk": "11bb85867221ee37", "coef": "86dcc255eecf756d", "lhet": "ff15c0af94a22f15"}


def header_symbols():
    src = open(os.path.join(ROOT, "include", "sniper_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ss_[a-z0-9_]+)\s*\(", src)) - {"ss_ctx"})


def test_library_exports_every_header_symbol(pkg):
    lib = pkg.load_library()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"missing export {s}"
    assert set(syms) == set(pkg.EXPORTED_SYMBOLS)
    assert lib.ss_abi_version() == 1


def test_strerror_and_nodev(pkg):
    lib = pkg.load_library()
    assert b"ok" == lib.ss_strerror(0)
    assert lib.ss_strerror(-5)


def test_params_default_matches_reference_cli(pkg):
    p = pkg.Params.default()
    # sniper_maqcns.c:107-111 and main.c:70-78
    assert abs(p.theta - 0.85) < 1e-7 and p.n_hap == 2 and abs(p.het_rate - 0.001) < 1e-9
    assert abs(p.eta - 0.03) < 1e-8 and p.cap_mapQ == 60 and p.min_somatic_qual == 15
    assert p.use_priors == 1 and p.use_joint_priors == 0 and p.somatic_rate == 0.01
    assert p.include_loh == 1 and p.include_gor == 1


def test_host_tables_match_reference_hashes(pkg):
    """Product host tables == the compiled reference's tables on THIS host."""
    import json
    import subprocess
    from oracle import binding as ob
    h = pkg.model_check()
    assert h["pinned"], h
    if os.path.exists(ob.REF_HARNESS):
        ref = json.loads(subprocess.run([ob.REF_HARNESS, "tables"], check=True, capture_output=True,
                                        text=True).stdout)
        for k in ("fk", "coef", "lhet"):
            assert h[k] == ref[k], k
        assert abs(h["q_r"] - ref["q_r"]) < 1e-6
    else:
        assert h["fk"] == REF_HASHES["fk"] and h["lhet"] == REF_HASHES["lhet"]
    assert abs(h["q_r"] - 26.9856968) < 1e-5


def _fnv1a64(b: bytes) -> str:
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def test_host_tables_match_oracle_for_nondefault(pkg, oracle):
    """Non-default -T/-N/-r: no reference hash exists, so the product's host tables
    are compared with the independently written oracle's (both pinned on the
    defaults above)."""
    p = pkg.Params.default(theta=0.9, n_hap=3, het_rate=0.01)
    h = pkg.model_check(p)
    t = oracle.Oracle(oracle.oparams(theta=0.9, n_hap=3, het_rate=0.01)).tables()
    assert h["fk"] == _fnv1a64(t["fk"].tobytes())
    assert h["lhet"] == _fnv1a64(t["lhet"].tobytes())
    assert h["q_r"] == t["q_r"]


def test_synth_host_deterministic_and_shaped(pkg):
    s = pkg.Synth.default(60, 30)
    a = pkg.synth_batch_host(s, 1000, 2000)
    b = pkg.synth_batch_host(s, 1000, 2000)
    for x, y in zip((a.ref, a.off_tumor, a.off_normal, a.reads_tumor, a.reads_normal),
                    (b.ref, b.off_tumor, b.off_normal, b.reads_tumor, b.reads_normal)):
        assert (x == y).all()
    # windows are independent of batch boundaries (counter-based)
    c = pkg.synth_batch_host(s, 1500, 500)
    assert (c.ref == a.ref[500:1000]).all()
    assert (c.reads_tumor == a.reads_tumor[a.off_tumor[500]:a.off_tumor[1000]]).all()
    dt = np.diff(a.off_tumor.astype(np.int64))
    dn = np.diff(a.off_normal.astype(np.int64))
    assert 55 < dt.mean() < 63 and 27 < dn.mean() < 32
    assert set(np.unique(a.ref).tolist()) <= set(b"ACGT")
    mq = a.reads_tumor & 0xFF
    assert 0.85 < (mq == 60).mean() < 0.95
    bq = (a.reads_tumor >> 8) & 0xFF
    assert bq.min() >= 2 and bq.max() <= 41


def test_ctx_create_without_gpu_fails_loudly(pkg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg.SniperError) as e:
        pkg.Context(pkg.Params.default())
    assert e.value.code == pkg.SS_E_NODEV


# ----------------------------------------------------------- table reuse (8(f) row 3)
_CHECK = ("import sys, time, json; sys.path.insert(0, {root!r});"
          "from __graft_entry__ import load_package; pkg = load_package();"
          "t0 = time.perf_counter(); a = pkg.model_check(pkg.Params.default({kw}));"
          "t1 = time.perf_counter(); b = pkg.model_check(pkg.Params.default({kw}));"
          "print(json.dumps(dict(first=a, second=b, secs=t1 - t0)))")


def _model_check_proc(cache, kw=""):
    import json
    import subprocess
    import sys
    env = dict(os.environ, SS_TABLE_CACHE=str(cache), SNIPER_AMD_NO_TORCH="1")
    p = subprocess.run([sys.executable, "-c", _CHECK.format(root=ROOT, kw=kw)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_table_cache_reuse_and_corruption(tmp_path):
    """The 32 MB x87 tables are built once per process and once per machine:
    a second context in the process shares them, a later process loads the
    verified disk blob instead of rebuilding (timed), a corrupted blob is
    detected by its hashes and rebuilt, other parameters get their own blob,
    and SS_TABLE_CACHE=off never touches the disk."""
    cache = tmp_path / "tabs"
    r1 = _model_check_proc(cache)
    assert r1["first"]["source"] == "built" and r1["second"]["source"] == "process"
    blobs = sorted(cache.iterdir())
    assert len(blobs) == 1 and blobs[0].stat().st_size > 32 << 20
    r2 = _model_check_proc(cache)
    assert r2["first"]["source"] == "disk"
    for k in ("fk", "coef", "lhet", "q_r", "pinned"):
        assert r2["first"][k] == r1["first"][k], k
    assert r2["secs"] < r1["secs"] / 2, (r2["secs"], r1["secs"])
    # corrupt one coef double: detected, rebuilt, the blob rewritten
    raw = bytearray(blobs[0].read_bytes())
    raw[4096 + 1234567] ^= 0x40
    blobs[0].write_bytes(bytes(raw))
    r3 = _model_check_proc(cache)
    assert r3["first"]["source"] == "built" and r3["first"]["coef"] == r1["first"]["coef"]
    assert _model_check_proc(cache)["first"]["source"] == "disk"
    # a truncated blob is not trusted either
    blobs[0].write_bytes(bytes(raw[: len(raw) // 2]))
    assert _model_check_proc(cache)["first"]["source"] == "built"
    # other table parameters: their own blob
    r5 = _model_check_proc(cache, kw="theta=0.9")
    assert r5["first"]["source"] == "built" and r5["first"]["coef"] != r1["first"]["coef"]
    assert len(list(cache.iterdir())) == 2
    off = _model_check_proc("off")
    assert off["first"]["source"] == "built" and off["first"]["coef"] == r1["first"]["coef"]


def _samtools_nt16():
    """bam_nt16_table (samtools-0.1.6 bam_import.c:23-40), rebuilt here."""
    t = [15] * 256
    for i, ch in enumerate("=ACMGRSVTWYHKDBN"):
        t[ord(ch)] = i
        if ch.isalpha():
            t[ord(ch.lower())] = i
    for i in range(4):
        t[ord("0") + i] = 1 << i
    return bytes(t)


def test_nt16_table_immutable_under_concurrent_builds(pkg):
    """Every context uploads the process's nt16 table (ss_capi.hip).  It must
    equal samtools' at every moment, also while 8 threads build contexts'
    host models at once: round 3's table was rewritten by every build, and a
    context that copied it mid-rewrite saw nt16 = 15 for real bases and
    dropped every candidate."""
    import threading
    lib = pkg.load_library()
    tab = (ctypes.c_ubyte * 256).in_dll(lib, "ss_nt16_table")
    want = _samtools_nt16()
    assert bytes(tab) == want
    stop = threading.Event()
    bad = []

    def build(theta):
        for _ in range(3):
            pkg.model_check(pkg.Params.default(theta=theta))

    def watch():
        while not stop.is_set():
            if bytes(tab) != want:
                bad.append(1)

    w = threading.Thread(target=watch)
    w.start()
    th = [threading.Thread(target=build, args=(0.85 if i % 2 else 0.9,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    stop.set()
    w.join()
    assert not bad and bytes(tab) == want
