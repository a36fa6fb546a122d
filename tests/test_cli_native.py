"""The native drop-in CLI (somatic-sniper_amd/bam-somaticsniper: own BGZF/BAM
reader, FASTA index, dual pileup and writers; GPU scoring through the C ABI)
against the reference CLI compiled from /root/reference (oracle/_ref).

CPU tests compare the site stream the two walkers hand to the scorer: the
native SS_DUMP_PILEUP/SS_PILEUP_ONLY hook against the reference CLI whose
glf_somatic is wrapped to dump the same fields (oracle/pileup_dump_shim.c).
GPU tests compare the output files byte for byte for every format and option
set, and the reference's own integration test (expected.vcf)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "somatic-sniper_amd", "bam-somaticsniper")
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "bam-somaticsniper")
REF_DUMP = os.path.join(ROOT, "oracle", "_ref", "bam-somaticsniper-dump")
ITEST = os.path.join(ROOT, "tests", "golden", "integration")

INDEX = os.path.join(ROOT, "somatic-sniper_amd", "ss-index")
need_native = pytest.mark.skipif(not os.path.exists(NATIVE), reason="native CLI not built")
need_index = pytest.mark.skipif(not os.path.exists(INDEX), reason="ss-index not built")
need_ref = pytest.mark.skipif(not os.path.exists(REF_CLI), reason="reference CLI not built")
need_dump = pytest.mark.skipif(not os.path.exists(REF_DUMP), reason="reference dump CLI not built")

OPTSETS = [[], ["-Q", "0"], ["-J"], ["-J", "-s", "1e-5", "-Q", "5"], ["-p", "-Q", "0"],
           ["-L", "-G", "-Q", "0"], ["-T", "0.9", "-N", "3", "-r", "0.01"], ["-q", "20", "-Q", "0"]]


def _run(cmd, cwd, env=None):
    return subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=600,
                          env=dict(os.environ, **(env or {})))


def _dump(cli, d, fa, t, n, opts, native, threads="1"):
    name = f"{'nat' if native else 'ref'}_{abs(hash(tuple(opts)))}.dump"
    env = {"SS_DUMP_PILEUP": name}
    if native:
        env["SS_PILEUP_ONLY"] = "1"
        env["SS_PILEUP_THREADS"] = threads
    p = _run([cli] + opts + ["-f", fa, t, n, "out_" + name], d, env)
    assert p.returncode == 0, p.stderr
    path = os.path.join(d, name)       # the reference shim only creates it at the first site
    return open(path, "rb").read() if os.path.exists(path) else b""


@need_native
@need_dump
@pytest.mark.parametrize("opts", [[], ["-q", "20"], ["-q", "61"]])
@pytest.mark.parametrize("threads", ["2", "1", "0"])
def test_pileup_site_stream_matches_reference(datasets, opts, threads):
    """threads: column pileup (2), the tumor and normal walks on their own threads (1), or
    both walks on one thread (0)."""
    for d, fa, t, n in datasets:
        ref = _dump(REF_DUMP, d, fa, t, n, opts, native=False)
        nat = _dump(NATIVE, d, fa, t, n, opts, native=True, threads=threads)
        assert nat == ref, (d, opts)


def _indexed_copy(d, fa, t, n, dst):
    """The dataset in its own directory with a .bai per BAM (ss-index); returns
    whether both indexes were written (an unsorted BAM gets none)."""
    dst.mkdir(exist_ok=True)
    for f in os.listdir(d):
        if f.endswith((".bam", ".fa", ".fai", ".fasta")):
            shutil.copy(os.path.join(d, f), dst / f)
    ok = [subprocess.run([INDEX, b], cwd=str(dst), capture_output=True).returncode == 0 for b in (t, n)]
    return all(ok)


@need_native
@need_dump
@need_index
@pytest.mark.parametrize("groups", ["2", "3", "7"])
@pytest.mark.parametrize("opts", [[], ["-q", "20"]])
def test_contig_groups_site_stream_matches_reference(datasets, tmp_path, groups, opts):
    """Indexed BAMs: the contig ranges pileup in parallel, each walk seeded from
    the last record its file loads before the range (column_pileup.h), and the
    concatenated site stream equals the reference walk's -- the first-read-drop
    at contig starts, unmapped / masked reads and an empty normal included.
    The unsorted pair gets no index (ss-index refuses it, as samtools index
    does) and takes the streaming walk."""
    indexed = grouped = 0
    for i, (d, fa, t, n) in enumerate(datasets):
        dst = tmp_path / f"ds{i}"
        both = _indexed_copy(d, fa, t, n, dst)
        indexed += both
        ref = _dump(REF_DUMP, d, fa, t, n, opts, native=False)
        name = "grp.dump"
        p = _run([NATIVE] + opts + ["-f", fa, t, n, "out_grp"], str(dst),
                 {"SS_DUMP_PILEUP": name, "SS_PILEUP_ONLY": "1", "SS_CONTIG_GROUPS": groups, "SS_TIMING": "1"})
        assert p.returncode == 0, p.stderr
        grouped += "contig groups done" in p.stderr
        assert both or "contig groups done" not in p.stderr
        path = dst / name
        nat = path.read_bytes() if path.exists() else b""
        assert nat == ref, (d, opts, groups)
    assert indexed >= 6 and grouped >= 3      # single-contig pairs keep one range


@need_native
@need_dump
@need_index
@pytest.mark.parametrize("opts", [[], ["-q", "40"]])
def test_contig_groups_multi_window_contigs(tmp_path, opts):
    """Contigs spanning several 16 kb linear-index windows, short contigs
    between long ones, unmapped and odd-CIGAR reads and -q 40 (most reads of a
    contig's tail filtered, so the seed search walks back through windows and
    contigs): the grouped site stream equals the reference walk's for 2..9
    ranges."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bamgen
    for seed, kw in [(11, dict(lengths=(70000, 400, 50000, 300, 30000), depth_t=6, depth_n=5, odd_cigars=True,
                               unmapped=True)),
                     (12, dict(lengths=(20000,) * 8, depth_t=4, depth_n=3))]:
        d = tmp_path / f"mw{seed}"
        d.mkdir()
        bamgen.make_pair(str(d), seed=seed, **kw)
        for b in ("tumor.bam", "normal.bam"):
            assert subprocess.run([INDEX, b], cwd=str(d)).returncode == 0
        ref = _dump(REF_DUMP, str(d), "ref.fa", "tumor.bam", "normal.bam", opts, native=False)
        assert ref
        for groups in ("2", "3", "5", "9"):
            name = f"g{groups}.dump"
            p = _run([NATIVE] + opts + ["-f", "ref.fa", "tumor.bam", "normal.bam", "out_" + name], str(d),
                     {"SS_DUMP_PILEUP": name, "SS_PILEUP_ONLY": "1", "SS_CONTIG_GROUPS": groups, "SS_TIMING": "1"})
            assert p.returncode == 0 and "contig groups done" in p.stderr, p.stderr
            assert (d / name).read_bytes() == ref, (seed, opts, groups)


@need_index
def test_index_refuses_unsorted_and_reads_back(datasets, tmp_path):
    """ss-index writes a loadable index for every coordinate-sorted BAM and
    refuses the pair with unsorted positions."""
    results = []
    for i, (d, fa, t, n) in enumerate(datasets):
        results.append(_indexed_copy(d, fa, t, n, tmp_path / f"x{i}"))
    assert results[-1] is False and all(results[:-1])


@need_native
@need_ref
def test_fasta_index_matches_reference(datasets, tmp_path):
    for d, fa, *_ in datasets:
        a, b = tmp_path / "a", tmp_path / "b"
        a.mkdir(exist_ok=True)
        b.mkdir(exist_ok=True)
        shutil.copy(os.path.join(d, fa), a / fa)
        shutil.copy(os.path.join(d, fa), b / fa)
        _run([REF_CLI, "-f", fa, "x.bam", "y.bam", "o"], str(a))          # builds a/fa.fai, then fails on the BAMs
        _run([NATIVE, "-f", fa, "x.bam", "y.bam", "o"], str(b), {"SS_PILEUP_ONLY": "1", "SS_DUMP_PILEUP": "d"})
        assert (a / (fa + ".fai")).read_bytes() == (b / (fa + ".fai")).read_bytes()


@need_native
def test_native_cli_fails_loudly_without_gpu(datasets):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    d, fa, t, n = datasets[0]
    p = _run([NATIVE, "-f", fa, t, n, "out.txt"], d)
    assert p.returncode != 0 and "GPU scorer" in p.stderr


@need_native
def test_native_cli_usage_and_errors(tmp_path):
    p = _run([NATIVE], str(tmp_path))
    assert p.returncode == 1 and "-f FILE   REQUIRED reference sequence" in p.stderr
    p = _run([NATIVE, "-I", "x"], str(tmp_path))
    assert p.returncode == 1 and "Unrecognizd option '-I'." in p.stderr
    p = _run([NATIVE, "-v"], str(tmp_path))
    assert p.returncode == 0 and p.stdout.startswith("Somatic Sniper version")


@need_native
@pytest.mark.parametrize("devs,msg", [("0,x", "bad entry"), ("0,,1", "bad entry"), ("-1", "bad entry"),
                                      ("1,1", "listed twice"), (",".join(map(str, range(17))), "more than 16")])
def test_ss_devices_rejects_bad_lists(datasets, devs, msg):
    """SS_DEVICES must be a list of distinct GPU indices: a typo fails loudly
    before any GPU work instead of quietly sharing or renumbering devices."""
    d, fa, t, n = datasets[0]
    p = _run([NATIVE, "-f", fa, t, n, "devs.out"], d, {"SS_DEVICES": devs})
    assert p.returncode == 1 and "SS_DEVICES" in p.stderr and msg in p.stderr, p.stderr


@pytest.mark.gpu
@need_native
def test_native_integration_expected_vcf(datasets):
    d, fa, t, n = datasets[0]
    p = _run([NATIVE, "-F", "vcf", "-f", fa, t, n, "native.vcf"], d)
    assert p.returncode == 0, p.stderr
    drop = ("##fileDate", "##reference")
    keep = lambda s: [l for l in s.splitlines() if not l.startswith(drop)]
    assert keep(open(os.path.join(d, "native.vcf")).read()) == keep(open(os.path.join(ITEST, "expected.vcf")).read())


@pytest.mark.gpu
@need_native
@need_ref
@pytest.mark.parametrize("fmt", ["classic", "vcf", "bed"])
def test_native_cli_matches_reference(datasets, fmt):
    strip = lambda s: "".join(l for l in s.splitlines(True) if not l.startswith("##fileDate"))
    for d, fa, t, n in datasets:
        for opts in OPTSETS:
            args = ["-F", fmt] + opts + ["-f", fa, t, n]
            pr = _run([REF_CLI] + args + ["ref.out"], d)
            pn = _run([NATIVE] + args + ["nat.out"], d, {"SS_BATCH": "1000"})
            assert pr.returncode == 0 and pn.returncode == 0, (pr.stderr, pn.stderr)
            ref = open(os.path.join(d, "ref.out")).read()
            nat = open(os.path.join(d, "nat.out")).read()
            assert strip(nat) == strip(ref), (d, fmt, opts)
            quiet = lambda e: e.replace("[fai_load] build FASTA index.\n", "")
            assert quiet(pn.stderr) == quiet(pr.stderr), (pn.stderr, pr.stderr)


@need_native
@need_ref
def test_bad_output_format_matches_reference(datasets, tmp_path):
    """-F with an unknown name (output_format.c:31-32): same message, exit code
    and (empty) output file as the reference CLI, before any GPU work."""
    d, fa, t, n = datasets[0]
    pr = _run([REF_CLI, "-F", "foo", "-f", fa, t, n, "ref.out"], d)
    pn = _run([NATIVE, "-F", "foo", "-f", fa, t, n, "nat.out"], d)
    quiet = lambda e: e.replace("[fai_load] build FASTA index.\n", "")
    assert pr.returncode == pn.returncode == 1
    assert quiet(pn.stderr) == quiet(pr.stderr) and "unknown output format: 'foo'. Abort!" in pn.stderr
    assert open(os.path.join(d, "nat.out")).read() == open(os.path.join(d, "ref.out")).read()


@pytest.mark.gpu
@need_native
@need_ref
@pytest.mark.parametrize("fmt", ["vcf", "classic"])
def test_sample_ids_and_stdin_match_reference(datasets, fmt):
    """-n / -t sample names in the VCF header (output_vcf.c:189-191) and the
    tumor BAM read from stdin as '-' (main.c:128), byte-identical to the
    reference CLI given the same arguments."""
    strip = lambda s: "".join(l for l in s.splitlines(True) if not l.startswith("##fileDate"))
    for d, fa, t, n in datasets[:3]:
        args = ["-F", fmt, "-n", "NORMAL_X", "-t", "TUMOR_Y", "-f", fa]
        pr = _run([REF_CLI] + args + [t, n, "ref_ids.out"], d)
        pn = _run([NATIVE] + args + [t, n, "nat_ids.out"], d)
        assert pr.returncode == 0 and pn.returncode == 0, (pr.stderr, pn.stderr)
        ref = open(os.path.join(d, "ref_ids.out")).read()
        assert strip(open(os.path.join(d, "nat_ids.out")).read()) == strip(ref)
        if fmt == "vcf":
            assert "NORMAL_X\tTUMOR_Y" in ref
        outs = []
        for cli, name in ((REF_CLI, "ref_stdin.out"), (NATIVE, "nat_stdin.out")):
            with open(os.path.join(d, t), "rb") as fin:
                p = subprocess.run([cli, "-F", fmt, "-f", fa, "-", n, name], cwd=d, stdin=fin,
                                   capture_output=True, text=True, timeout=600)
            assert p.returncode == 0, p.stderr
            outs.append((strip(open(os.path.join(d, name)).read()), p.stderr))
        assert outs[0][0] == outs[1][0]
        quiet = lambda e: e.replace("[fai_load] build FASTA index.\n", "")
        assert quiet(outs[0][1]) == quiet(outs[1][1])


@pytest.mark.gpu
@need_native
@need_ref
@need_index
def test_contig_groups_output_matches_reference(datasets, tmp_path):
    """Indexed BAMs, contig ranges scored in parallel (each range its own
    pileup, batches and GPU scorer), outputs concatenated in contig order:
    byte-identical to the reference CLI for every format and several option
    sets, with one and two scorers per range."""
    strip = lambda s: "".join(l for l in s.splitlines(True) if not l.startswith("##fileDate"))
    for i, (d, fa, t, n) in enumerate(datasets):
        dst = tmp_path / f"g{i}"
        if not _indexed_copy(d, fa, t, n, dst):
            continue
        for fmt, opts in (("classic", []), ("vcf", ["-Q", "0"]), ("bed", ["-J", "-Q", "5"]), ("classic", ["-q", "20", "-Q", "0"])):
            args = ["-F", fmt] + opts + ["-f", fa, t, n]
            pr = _run([REF_CLI] + args + ["ref.out"], d)
            assert pr.returncode == 0, pr.stderr
            ref = strip(open(os.path.join(d, "ref.out")).read())
            for env in ({"SS_CONTIG_GROUPS": "3", "SS_BATCH": "500"},
                        {"SS_CONTIG_GROUPS": "2", "SS_DEVICES": "0,0", "SS_DEVICES_SHARED": "1"}):
                pn = _run([NATIVE] + args + ["nat.out"], str(dst), env)
                assert pn.returncode == 0, pn.stderr
                assert strip((dst / "nat.out").read_text()) == ref, (d, fmt, opts, env)


@pytest.mark.gpu
@need_native
@need_ref
@need_index
def test_contig_groups_concurrent_contexts_repeated(datasets, tmp_path):
    """2 contig ranges x 2 scorers on one device: four contexts created at the
    same moment on four threads.  With stream-ordered device allocation about
    one run in five lost a batch's calls (tools/repro_groups.py);
    every one of 10 runs must equal the reference CLI."""
    strip = lambda s: "".join(l for l in s.splitlines(True) if not l.startswith("##fileDate"))
    d, fa, t, n = datasets[2]                   # bamgen seed 2, 60x/30x, 4 contigs
    dst = tmp_path / "rep"
    assert _indexed_copy(d, fa, t, n, dst)
    args = ["-F", "vcf", "-Q", "0", "-f", fa, t, n]
    pr = _run([REF_CLI] + args + ["ref_rep.out"], d)
    assert pr.returncode == 0, pr.stderr
    ref = strip(open(os.path.join(d, "ref_rep.out")).read())
    env = {"SS_CONTIG_GROUPS": "2", "SS_DEVICES": "0,0", "SS_DEVICES_SHARED": "1"}
    for r in range(10):
        pn = _run([NATIVE] + args + ["nat_rep.out"], str(dst), env)
        assert pn.returncode == 0, pn.stderr
        assert strip((dst / "nat_rep.out").read_text()) == ref, f"run {r}"


@pytest.mark.gpu
@need_native
@need_ref
def test_multi_scorer_output_identical(datasets):
    """SS_DEVICES with several scorers (all on the box's one GPU here; one
    per device on a multi-GPU node) and small batches, so consecutive batches
    are scored concurrently by different contexts: the output is written in
    batch order and equals the single-scorer run and the reference CLI."""
    for d, fa, t, n in datasets:
        for fmt in ("classic", "vcf"):
            args = ["-F", fmt, "-Q", "0", "-f", fa, t, n]
            pr = _run([REF_CLI] + args + ["ref_ms.out"], d)
            p1 = _run([NATIVE] + args + ["one_ms.out"], d, {"SS_BATCH": "97"})
            p3 = _run([NATIVE] + args + ["three_ms.out"], d, {"SS_BATCH": "97", "SS_DEVICES": "0,0,0",
                                                                   "SS_DEVICES_SHARED": "1"})
            assert pr.returncode == p1.returncode == p3.returncode == 0, (p1.stderr, p3.stderr)
            strip = lambda s: "".join(l for l in s.splitlines(True) if not l.startswith("##fileDate"))
            ref = strip(open(os.path.join(d, "ref_ms.out")).read())
            assert strip(open(os.path.join(d, "one_ms.out")).read()) == ref
            assert strip(open(os.path.join(d, "three_ms.out")).read()) == ref, (d, fmt)


def _grouped_dump(d, fa, t, n, groups="3", opts=()):
    name = "chk.dump"
    p = _run([NATIVE] + list(opts) + ["-f", fa, t, n, "out_chk"], str(d),
             {"SS_DUMP_PILEUP": name, "SS_PILEUP_ONLY": "1", "SS_CONTIG_GROUPS": groups, "SS_TIMING": "1"})
    assert p.returncode == 0, p.stderr
    path = d / name
    return (path.read_bytes() if path.exists() else b""), "contig groups done" in p.stderr


@need_native
@need_dump
@need_index
def test_stale_or_foreign_index_takes_streaming_walk(tmp_path):
    """The reference never reads an index, so one that does not describe its
    BAM must not change a byte: an index older than its BAM (htslib's
    staleness test) and another file's index (records at the wrong offsets)
    are both refused, the streaming walk runs, and the site stream equals the
    reference's.  A fresh, matching index runs the contig groups."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bamgen
    fa, t, n = "ref.fa", "tumor.bam", "normal.bam"
    d, d5 = tmp_path / "src", tmp_path / "src5"
    for x, seed, dep in ((d, 12, (4, 3)), (d5, 13, (5, 4))):
        x.mkdir()
        bamgen.make_pair(str(x), seed=seed, lengths=(20000,) * 8, depth_t=dep[0], depth_n=dep[1])
    d, d5 = str(d), str(d5)
    ref = _dump(REF_DUMP, d, fa, t, n, [], native=False)
    dst = tmp_path / "fresh"
    assert _indexed_copy(d, fa, t, n, dst)
    got, grouped = _grouped_dump(dst, fa, t, n)
    assert got == ref and grouped
    # stale: the BAM rewritten (same bytes) after its index was made
    st = os.stat(dst / t)
    os.utime(dst / (t + ".bai"), ns=(st.st_atime_ns, st.st_mtime_ns - 10 ** 9))
    got, grouped = _grouped_dump(dst, fa, t, n)
    assert got == ref and not grouped
    # an index stamped in whole seconds (a second-resolution copy) in the same
    # second as its BAM (htslib's whole-second test): used
    sec = st.st_mtime_ns // 10 ** 9 * 10 ** 9
    os.utime(dst / t, ns=(st.st_atime_ns, sec + 5 * 10 ** 8))
    os.utime(dst / (t + ".bai"), ns=(st.st_atime_ns, sec))
    got, grouped = _grouped_dump(dst, fa, t, n)
    assert got == ref and grouped
    # both stamped to the nanosecond: the BAM rewritten later in the same second
    # as its index is refused; an index written after its BAM in that second is used
    os.utime(dst / (t + ".bai"), ns=(st.st_atime_ns, sec + 2 * 10 ** 8))
    got, grouped = _grouped_dump(dst, fa, t, n)
    assert got == ref and not grouped
    os.utime(dst / (t + ".bai"), ns=(st.st_atime_ns, sec + 7 * 10 ** 8))
    got, grouped = _grouped_dump(dst, fa, t, n)
    assert got == ref and grouped
    # foreign: the tumor BAM carries another dataset's index (same contig count)
    dst2 = tmp_path / "foreign"
    assert _indexed_copy(d, fa, t, n, dst2)
    other = tmp_path / "other"
    assert _indexed_copy(d5, fa, t, n, other)
    shutil.copy(other / (t + ".bai"), dst2 / (t + ".bai"))
    got, grouped = _grouped_dump(dst2, fa, t, n)
    assert got == ref and not grouped


def _htslib_layout(src, dst):
    """Rewrite an ss-index BAI the way htslib's `samtools index` lays it out
    (hts.c hts_idx_finish / update_loff): a pseudo-bin 37450 per placed contig
    (its [first, last) offsets and mapped / unmapped counts), leading linear-index
    windows before the first read set to the contig's first offset instead of 0,
    and the trailing n_no_coor count."""
    import struct
    b = open(src, "rb").read()
    o = 8
    n_ref = struct.unpack_from("<i", b, 4)[0]
    out = bytearray(b[:8])
    for _ in range(n_ref):
        n_bin = struct.unpack_from("<i", b, o)[0]
        o += 4
        bins, lo, hi = [], None, None
        for _ in range(n_bin):
            bin_id, n_chunk = struct.unpack_from("<Ii", b, o)
            chunks = struct.unpack_from(f"<{2 * n_chunk}Q", b, o + 8)
            bins.append(b[o:o + 8 + 16 * n_chunk])
            o += 8 + 16 * n_chunk
            lo = min([lo] + list(chunks[0::2])) if lo is not None else min(chunks[0::2])
            hi = max([hi] + list(chunks[1::2])) if hi is not None else max(chunks[1::2])
        n_intv = struct.unpack_from("<i", b, o)[0]
        lin = list(struct.unpack_from(f"<{n_intv}Q", b, o + 4))
        o += 4 + 8 * n_intv
        if n_bin:
            bins.append(struct.pack("<Ii4Q", 37450, 2, lo, hi, 1000, 3))
            k = 0
            while k < len(lin) and lin[k] == 0:
                lin[k] = lo
                k += 1
        out += struct.pack("<i", len(bins)) + b"".join(bins)
        out += struct.pack("<i", n_intv) + struct.pack(f"<{n_intv}Q", *lin)
    assert o == len(b)
    out += struct.pack("<Q", 7)                 # n_no_coor
    open(dst, "wb").write(bytes(out))


@need_native
@need_dump
@need_index
@pytest.mark.parametrize("opts", [[], ["-q", "40"]])
def test_contig_groups_with_htslib_layout_index(tmp_path, opts):
    """Indexes as htslib writes them (pseudo-bin, filled leading linear-index
    windows, n_no_coor) drive the contig groups to the reference's site stream
    too, for 2..9 ranges over contigs spanning several linear windows."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bamgen
    d = tmp_path / "hts"
    d.mkdir()
    bamgen.make_pair(str(d), seed=11, lengths=(70000, 400, 50000, 300, 30000), depth_t=6, depth_n=5,
                     odd_cigars=True, unmapped=True)
    for b in ("tumor.bam", "normal.bam"):
        assert subprocess.run([INDEX, b, str(d / (b + ".ss.bai"))], cwd=str(d)).returncode == 0
        _htslib_layout(d / (b + ".ss.bai"), d / (b + ".bai"))
        assert (d / (b + ".bai")).read_bytes() != (d / (b + ".ss.bai")).read_bytes()
    ref = _dump(REF_DUMP, str(d), "ref.fa", "tumor.bam", "normal.bam", opts, native=False)
    assert ref
    for groups in ("2", "3", "5", "9"):
        got, grouped = _grouped_dump(d, "ref.fa", "tumor.bam", "normal.bam", groups, opts)
        assert grouped and got == ref, (opts, groups)
