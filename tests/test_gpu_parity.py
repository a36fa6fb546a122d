"""GPU parity: the HIP scorer (through the C ABI) against the CPU oracle.

Bit-exact on every integer output of the reference path: glf_somatic's return
value per site (somatic_sniper.c:109-273), both glf1_t records
(sniper_maqcns.c:127-248) and every emitted call (its cns words, snp_q, joint
genotypes, status).  The oracle itself is pinned to the compiled reference by
tests/test_oracle_golden.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EXOTIC = dict(p_wild_qual=0.05, p_eq=0.02, p_iupac=0.02, p_nbase=0.02, p_ref_n=0.02,
              p_ref_lower=0.05, p_ref_iupac=0.02, p_germline=0.03, p_somatic=0.05, vaf=0.4,
              p_del=0.05)

OPTSETS = [[], ["-J"], ["-p"], ["-s", "1e-6"], ["-T", "0.9", "-N", "3", "-r", "0.01"],
           ["-Q", "0", "-L", "-G"], ["-J", "-p", "-Q", "0"], ["-L"], ["-G"]]


def params_from_opts(pkg, opts):
    p = pkg.Params.default()
    it = iter(opts)
    for o in it:
        if o == "-T": p.theta = float(next(it))
        elif o == "-N": p.n_hap = int(next(it))
        elif o == "-r": p.het_rate = float(next(it))
        elif o == "-p": p.use_priors = 0
        elif o == "-J": p.use_joint_priors = 1
        elif o == "-s": p.somatic_rate = float(next(it)); p.use_joint_priors = 1
        elif o == "-Q": p.min_somatic_qual = int(next(it))
        elif o == "-L": p.include_loh = 0
        elif o == "-G": p.include_gor = 0
    return p


def assert_parity(pkg, oracle, batch, opts=(), ctx=None):
    """Every output against the oracle, twice: with glf records requested and
    without (the way the CLI and the bench score)."""
    own = ctx is None
    if own:
        ctx = pkg.Context(params_from_opts(pkg, opts), device=0)
    try:
        score, calls, glf = ctx.score_batch(batch, want_glf=True)
        score_x, calls_x, _ = ctx.score_batch(batch, want_glf=False)
    finally:
        if own:
            ctx.close()
    o = oracle.Oracle(oracle.opts_to_params(list(opts)))
    o_score, o_calls, o_glf = o.score_batch(batch.ref, batch.off_tumor, batch.off_normal,
                                            batch.reads_tumor, batch.reads_normal)
    bad = np.nonzero(score != o_score)[0]
    assert bad.size == 0, f"{bad.size} score mismatches, first {bad[:5]}: gpu {score[bad[:5]]} oracle {o_score[bad[:5]]}"
    gb = glf.view(np.uint8).reshape(batch.n_sites, -1) != o_glf.view(np.uint8).reshape(batch.n_sites, -1)
    bad = np.nonzero(gb.any(1))[0]
    assert bad.size == 0, f"{bad.size} glf mismatches, first site {bad[0]}: gpu {glf[bad[0]]} oracle {o_glf[bad[0]]}"
    assert len(calls) == len(o_calls)
    assert (calls.view(np.uint8) == o_calls.view(np.uint8)).all()
    bad = np.nonzero(score_x != o_score)[0]
    assert bad.size == 0, f"no glf: {bad.size} score mismatches, first {bad[:5]}: gpu {score_x[bad[:5]]} " \
                          f"oracle {o_score[bad[:5]]}"
    assert len(calls_x) == len(o_calls) and (calls_x.view(np.uint8) == o_calls.view(np.uint8)).all()
    return score, calls


@pytest.mark.parametrize("lt,ln,kw", [(30, 30, {}), (60, 30, {}), (60, 30, EXOTIC), (100, 60, EXOTIC),
                                      (3, 2, dict(p_wild_qual=0.3, p_del=0.3, p_somatic=0.1, p_germline=0.1))])
@pytest.mark.parametrize("opts", OPTSETS)
def test_synthetic_parity(pkg, oracle, lt, ln, kw, opts):
    batch = pkg.synth_batch_host(pkg.Synth.default(lt, ln, seed=1234 + lt, **kw), 0, 3000)
    assert_parity(pkg, oracle, batch, opts)


@pytest.mark.parametrize("lt,ln,fixed,n,wild", [(300, 300, 0, 300, 0.05), (700, 700, 1, 60, 0.05),
                                                (500, 500, 0, 200, 0.05), (250, 270, 0, 400, 0.05),
                                                (300, 300, 0, 300, 0.0), (500, 500, 0, 200, 0.0),
                                                (700, 700, 1, 60, 0.0), (600, 500, 0, 120, 0.0),
                                                (500, 500, 0, 300, 0.0005)])
@pytest.mark.parametrize("opts", OPTSETS)
def test_deep_parity(pkg, oracle, lt, ln, fixed, n, wild, opts):
    """Sites beyond the main kernel's 512 sort slots -> wide kernel (and the
    deep kernel past 2048); > 255 reads per class saturates w, > 255 total
    rescales c (Appendix A.4).  The wide kernel's 8-bit fold records hold
    q < 64, so a site with a read of minq >= 64 (wild qualities: baseQ / mapQ
    up to 255) is scored by the deep kernel instead: wild = 0.05 sends every
    wide site there, 0 none, 5e-4 about a quarter (mixed routing).  Every
    option set: -T/-N/-r change the fk / coef / lhet tables the wide and deep
    folds and likelihoods read, -J/-p/-L/-G/-Q the decision."""
    kw = dict(EXOTIC, p_wild_qual=wild)
    batch = pkg.synth_batch_host(pkg.Synth.default(lt, ln, fixed_depth=fixed, **kw), 0, n)
    assert_parity(pkg, oracle, batch, opts)


@pytest.mark.parametrize("lt,ln,fixed,n,wild", [(1200, 1000, 0, 60, 0.0), (1500, 600, 1, 30, 0.0),
                                                (2000, 2000, 1, 12, 0.0), (2100, 100, 1, 8, 0.0),
                                                (1200, 1000, 0, 40, 0.0005), (1030, 1030, 1, 20, 0.05),
                                                (700, 480, 1, 40, 0.0), (480, 1050, 1, 40, 0.0),
                                                (1000, 300, 1, 40, 0.0), (560, 470, 0, 200, 0.0),
                                                (560, 470, 0, 120, 0.0005)])
@pytest.mark.parametrize("opts", OPTSETS)
def test_wide_sample_units_parity(pkg, oracle, lt, ln, fixed, n, wild, opts):
    """Sites past 2048 sort slots whose samples have at most 2048 reads each:
    the wide kernel sorts each sample in a network of its own (sort units),
    K = 8 or 16 per sample; a sample beyond 2048 (2100/100) and sites with
    wild qualities go to the deep kernel.  Sites past 1024 slots with one
    sample of at most 512 reads (700/480, 480/1050, 1000/300, Poisson
    560/470) are units too: K = 4 for the small sample, 8 for the other."""
    kw = dict(EXOTIC, p_wild_qual=wild)
    batch = pkg.synth_batch_host(pkg.Synth.default(lt, ln, fixed_depth=fixed, **kw), 3, n)
    assert_parity(pkg, oracle, batch, opts)


@pytest.mark.parametrize("lt,ln,n", [(130, 126, 80), (255, 250, 60), (514, 508, 50), (1023, 1020, 30),
                                     (2040, 40, 20), (140, 3, 60), (2, 600, 40)])
@pytest.mark.parametrize("opts", [OPTSETS[0], OPTSETS[-1]])
def test_group_unit_boundaries(pkg, oracle, lt, ln, n, opts):
    """Lane-group sort units (ss_score_group) at lane-count and network-size
    boundaries: Poisson depths straddling 128 / 256 / 512 / 1024 / 2048 reads
    per sample, so units of 1 .. 16 lanes (networks of 1, 2, 4, 8 and 16 lanes,
    and the deep kernel past 2048) mix in one batch of lanes, plus sites with a
    tiny or empty second sample."""
    batch = pkg.synth_batch_host(pkg.Synth.default(lt, ln, **EXOTIC), 11, n)
    assert_parity(pkg, oracle, batch, opts)


@pytest.mark.parametrize("seed", [21, 22])
def test_group_dense_unit_packing(pkg, oracle, seed):
    """Units take ceil(n / 128) lanes (1 .. 16, not only powers of two) and are
    packed by descending size into 64-lane batches, so a chunk mixes units of
    3, 5, 6, 7, 9 .. 15 lanes whose virtual pad lanes belong to the next unit,
    and batches end in empty lanes.  Depths spread over 129 .. 2048 reads per
    sample, tumor and normal drawn independently, sites interleaved."""
    import random
    rnd = random.Random(seed)
    lams = [(200, 700), (330, 1450), (650, 260), (900, 1180), (1150, 390), (1400, 1900), (1700, 540),
            (1950, 1020)]
    parts = [pkg.synth_batch_host(pkg.Synth.default(lt, ln, **EXOTIC), 30 + k, 9)
             for k, (lt, ln) in enumerate(lams)]
    sites = [b.site(i) for b in parts for i in range(b.n_sites)]
    rnd.shuffle(sites)
    assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), OPTSETS[0])


@pytest.mark.parametrize("n_group", [1, 31, 32, 33, 95])
@pytest.mark.parametrize("wild", [0.0, 0.002])
def test_group_chunk_sizes(pkg, oracle, n_group, wild):
    """The group kernel takes its listed sites 32 at a time (one chunk: the
    records of all 32 fold together, one lane per (site, sample)): listed
    counts below, at and just past a chunk, interleaved with main-kernel
    sites so the listed order crosses main-wave segments; with wild reads a
    chunk's sites leave for the deep kernel and the rest are compacted."""
    deep = pkg.synth_batch_host(pkg.Synth.default(520, 480, **dict(EXOTIC, p_wild_qual=wild)), 5, n_group)
    shallow = pkg.synth_batch_host(pkg.Synth.default(40, 30, **dict(EXOTIC, p_wild_qual=0.0)), 6, 3 * n_group + 50)
    sites = []
    for i in range(shallow.n_sites):
        sites.append(shallow.site(i))
        if i % 3 == 1 and i // 3 < deep.n_sites:
            sites.append(deep.site(i // 3))
    assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), OPTSETS[0])


@pytest.mark.parametrize("opts", OPTSETS)
def test_kernel_routing_mix(pkg, oracle, opts):
    """One batch whose sites take every route: main kernel (<= 512 sort slots),
    wide kernel (<= 2048), and the deep kernel via the wide kernel's overflow
    list (histogram fold, any depth), interleaved so each kernel sees
    non-contiguous site indices; under every option set."""
    parts = [pkg.synth_batch_host(pkg.Synth.default(lt, ln, fixed_depth=1, **EXOTIC), 7 * k, n)
             for k, (lt, ln, n) in enumerate([(60, 30, 40), (600, 500, 12), (1500, 1200, 6), (4200, 300, 3),
                                              (30, 2, 40), (900, 900, 6)])]
    sites = []
    for i in range(40):
        for b in parts:
            if i < b.n_sites:
                sites.append(b.site(i))
    with pkg.Context(params_from_opts(pkg, opts), device=0) as c:
        assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), opts, ctx=c)
        c.check()


def test_pinned_host_batch(pkg, oracle, ctx):
    """Inputs in ss_host_alloc memory take the no-staging H2D path of
    ss_score_batch_host: same results as pageable inputs and the oracle."""
    b = pkg.synth_batch_host(pkg.Synth.default(60, 30, **EXOTIC), 5, 3000)
    p = b.pinned()
    assert (p.reads_tumor == b.reads_tumor).all() and (p.off_normal == b.off_normal).all()
    s1, c1, g1 = ctx.score_batch(b, want_glf=True)
    s2, c2, g2 = ctx.score_batch(p, want_glf=True)
    assert (s1 == s2).all() and (g1.view(np.uint8) == g2.view(np.uint8)).all()
    assert (c1.view(np.uint8) == c2.view(np.uint8)).all()
    assert_parity(pkg, oracle, p, ctx=ctx)


def _malformed_base(pkg):
    b = pkg.synth_batch_host(pkg.Synth.default(60, 30, **EXOTIC), 11, 300)
    wide = pkg.synth_batch_host(pkg.Synth.default(700, 600, fixed_depth=1, **EXOTIC), 3, 4)
    sites = [b.site(i) for i in range(b.n_sites)]
    sites[200:200] = [wide.site(i) for i in range(wide.n_sites)]
    return pkg.Batch.from_sites(sites)


def _score_device(pkg, ctx, b):
    """Score a host batch through ss_score_batch_device; returns (score, rc of ss_ctx_check)."""
    import torch
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(dev)
    score = torch.full((b.n_sites,), 12345, dtype=torch.int32, device=dev)
    ctx.score_device(t(b.ref, np.uint8), t(b.off_tumor, np.int32), t(b.off_normal, np.int32),
                     t(b.reads_tumor, np.int32), t(b.reads_normal, np.int32), score=score)
    try:
        ctx.check()
        rc = pkg.SS_OK
    except pkg.SniperError as e:
        rc = e.code
    return score.cpu().numpy(), rc


@pytest.mark.parametrize("case", ["tumor_minus_1", "normal_minus_7_wide", "past_end", "both_past_end"])
def test_malformed_offsets_reported(pkg, oracle, ctx, case):
    """Malformed offsets never steer a load outside the batch's reads, and the
    batch is reported: ss_ctx_check returns SS_E_INVAL.  A site whose own
    offsets decrease wraps its read count to ~2^32 and is routed through the
    deep lists to the deep kernel, which scores it -2 without touching reads.
    Cases, one malformation per batch: a tumor count of -1 (odd: count + pad
    wraps to a small slot total, the main kernel's trap), a normal count of -7
    next to a wide site, an offset past off[n] (so a later site decreases),
    and two offsets past the end with equal values (a zero-length site between
    them, then the decrease).  The context stays usable."""
    good = _malformed_base(pkg)
    ot, on = good.off_tumor.copy(), good.off_normal.copy()
    n = good.n_sites
    if case == "tumor_minus_1":
        assert ot[5] >= 1
        ot[6] = ot[5] - 1
        minus2 = [5]
    elif case == "normal_minus_7_wide":
        assert on[202] >= 7
        on[203] = on[202] - 7
        minus2 = [202]
    elif case == "past_end":
        ot[100] = ot[n] + 1000                        # site 99 runs past the end, site 100 decreases
        minus2 = [99, 100]
    else:
        ot[50] = ot[51] = ot[n] + 77
        minus2 = [49, 50, 51]                         # 49 and 50 run past the end, 51 decreases
    bad = pkg.Batch(good.ref, ot, on, good.reads_tumor, good.reads_normal)
    with pytest.raises(pkg.SniperError) as ei:
        ctx.score_batch(bad)
    assert ei.value.code == pkg.SS_E_INVAL
    ctx.check()                                   # the sticky bit was cleared
    score, rc = _score_device(pkg, ctx, bad)
    assert rc == pkg.SS_E_INVAL
    assert all(score[i] == -2 for i in minus2), [(i, score[i]) for i in minus2]
    ref_score, _, _ = ctx.score_batch(good)
    untouched = [i for i in range(n) if ot[i] == good.off_tumor[i] and ot[i + 1] == good.off_tumor[i + 1]
                 and on[i] == good.off_normal[i] and on[i + 1] == good.off_normal[i + 1]]
    assert (score[untouched] == ref_score[untouched]).all()
    assert_parity(pkg, oracle, good, ctx=ctx)


def test_deep_kernel_any_depth(pkg, oracle, ctx):
    """The deep kernel has no depth limit: one site with 1.1 M tumor reads and
    ~10^5 normal reads (the round-1 build gave up beyond 2^20 per sample) next
    to ordinary sites, bit-exact with the oracle."""
    big = pkg.synth_batch_host(pkg.Synth.default(1_100_000, 100_000, fixed_depth=1, **EXOTIC), 0, 1)
    small = pkg.synth_batch_host(pkg.Synth.default(60, 30, **EXOTIC), 9, 50)
    sites = [small.site(i) for i in range(25)] + [big.site(0)] + [small.site(i) for i in range(25, 50)]
    assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), ctx=ctx)
    ctx.check()


def test_many_deep_sites(pkg, oracle, ctx):
    """Thousands of sites beyond the wide kernel's 2048 slots in one batch:
    the deep list is sized from the batch (no fixed cap, no overflow)."""
    b = pkg.synth_batch_host(pkg.Synth.default(1200, 1000, **EXOTIC), 0, 3000)
    assert_parity(pkg, oracle, b, ctx=ctx)
    ctx.check()


@pytest.mark.parametrize("opts", OPTSETS)
def test_deep_windows_full_quality_range(pkg, oracle, opts):
    """Deep sites whose reads span mapQ and baseQ 0..255 (every bin of the
    deep kernel's 1136 per group is reachable), both strands, every nt16 code:
    the histogram is built and folded in several LDS windows from the top
    down, the chain carried across them.  Depths straddle the window count
    and the wide/deep boundary; one site has a single high-q read above a
    bulk of low-q ones."""
    rng = np.random.default_rng(77)
    sites = []
    for k, (nt_, nn_) in enumerate([(2100, 10), (2500, 1500), (40, 2600), (5000, 3000), (1030, 1030)]):
        mk = lambda n: [pkg.pack_read(int(rng.integers(0, 256)), int(rng.integers(0, 256)),
                                      int(rng.integers(0, 16)), int(rng.integers(0, 2))) for _ in range(n)]
        sites.append(("ACGT"[k % 4], mk(nt_), mk(nn_)))
    lowq = [pkg.pack_read(60, int(5 + i % 20), 1 + (i % 3), i & 1) for i in range(2400)]
    sites.append(("A", lowq + [pkg.pack_read(250, 240, 8, 1)], lowq[:900]))
    with pkg.Context(params_from_opts(pkg, opts), device=0) as c:
        assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), opts, ctx=c)
        c.check()


def test_giant_parity(pkg, oracle, ctx):
    """> 4096 reads in a sample (the round-1 giant route) -> deep kernel."""
    big = pkg.synth_batch_host(pkg.Synth.default(6000, 4500, fixed_depth=1, **EXOTIC), 0, 6)
    small = pkg.synth_batch_host(pkg.Synth.default(40, 40, **EXOTIC), 100, 20)
    sites = [big.site(i) for i in range(big.n_sites)] + [small.site(i) for i in range(small.n_sites)]
    assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), ctx=ctx)


def _r(pkg, mq, bq, nt, st):
    return pkg.pack_read(mq, bq, nt, st)


def quirk_sites(pkg):
    R = lambda mq, bq, nt, st=0: _r(pkg, mq, bq, nt, st)
    A, C_, G, T, N, EQ, M = 1, 2, 4, 8, 15, 0, 3
    s = []
    # Appendix A.1: N and IUPAC reads count as A; '=' resolves to the ref base
    s.append(("C", [R(60, 30, N)] * 10, [R(60, 30, C_)] * 10))
    s.append(("C", [R(60, 30, M)] * 10, [R(60, 30, C_)] * 10))
    s.append(("G", [R(60, 30, EQ)] * 8 + [R(60, 30, T)] * 6, [R(60, 30, G)] * 9))
    # A.2: q clamp; mapQ 0 reads still contribute with q=4; baseQ&0x3f==0 and min<4 drop
    s.append(("A", [R(0, 30, T)] * 12 + [R(60, 30, A)] * 3, [R(60, 30, A)] * 12))
    s.append(("A", [R(2, 64, T)] * 12 + [R(1, 128, T)] * 4 + [R(60, 30, A)] * 3, [R(60, 30, A)] * 12))
    s.append(("A", [R(0, 0, T)] * 12 + [R(60, 30, A)] * 3, [R(60, 30, A)] * 12))
    # A.3: mapQ >= 128 (rms uses mapQ & 0x7f), mapQ 255
    s.append(("T", [R(200, 35, A, 1)] * 9 + [R(255, 20, T)] * 9, [R(130, 30, T)] * 9))
    # depth 1 / all reads q==0 / all-deleted (empty packed list -> -1)
    s.append(("A", [R(60, 30, C_)], [R(60, 30, A)]))
    s.append(("A", [R(0, 0, C_)] * 3, [R(0, 0, A)] * 2))
    s.append(("A", [], [R(60, 30, A)] * 5))
    s.append(("A", [R(60, 30, A)] * 5, []))
    # ref 'N' (skipped), ref 'n' (scored, never a candidate), IUPAC ref, '=' ref
    s.append(("N", [R(60, 30, T)] * 10, [R(60, 30, A)] * 10))
    s.append(("n", [R(60, 30, T)] * 10, [R(60, 30, A)] * 10))
    s.append(("R", [R(60, 30, T)] * 10, [R(60, 30, A)] * 10))
    s.append(("=", [R(60, 30, EQ)] * 10, [R(60, 30, A)] * 10))
    s.append(("a", [R(60, 30, T)] * 10, [R(60, 30, A)] * 10))
    # strong somatic, LOH, gain of reference, germline het
    s.append(("A", [R(60, 35, T, i & 1) for i in range(20)], [R(60, 35, A, i & 1) for i in range(20)]))
    s.append(("A", [R(60, 35, T)] * 20, [R(60, 35, A)] * 10 + [R(60, 35, T)] * 10))
    s.append(("A", [R(60, 35, A)] * 10 + [R(60, 35, T)] * 10, [R(60, 35, T)] * 20))
    s.append(("A", [R(60, 35, A)] * 10 + [R(60, 35, G)] * 10, [R(60, 35, A)] * 10 + [R(60, 35, G)] * 10))
    # exactly 64 / 65 / 128 / 129 / 256 reads (register-sort boundaries), strands mixed
    for n in (63, 64, 65, 127, 128, 129, 255, 256, 257):
        s.append(("C", [R(60, 10 + (i * 7) % 31, C_ if i % 9 else G, i & 1) for i in range(n)],
                  [R(60, 10 + (i * 5) % 31, C_, (i >> 1) & 1) for i in range(n // 2 + 1)]))
    # every key field at its maximum in the NORMAL sample (mapQ = baseQ = 255,
    # T, reverse strand): a contributing read whose 16-bit sort key would equal
    # the pad key; at main-kernel, wide-kernel and deep-kernel depths
    for nt_, nn_ in ((10, 10), (300, 300), (1500, 1000)):
        s.append(("A", [R(60, 30, A)] * nt_,
                  [R(255, 255, T, 1)] * (nn_ // 2) + [R(255, 255, T, i & 1) for i in range(nn_ - nn_ // 2)]))
    # Rescaled counts summing to 256 (sniper_maqcns.c:178-182: four classes of
    # odd counts over 508 reads round 63.5 -> 64 each; 2540 = 4 x 635 likewise):
    # the coef index bar_e<<16 | c<<8 | tmp2 (:195, :206) then ORs bit 16 into
    # bar_e<<16 -- an odd bar_e keeps its row, an even one moves to bar_e + 1,
    # n = 0 in both, and bar_e = 63 stays in the table.  Quality q gives
    # bar_e = q: even (30), odd (31, 45), 63, and 70 clamped to 63 (minq >= 64:
    # the deep kernel); 508 reads per sample go to the group kernel, 2540 to
    # the deep kernel; the last site has unequal odd counts (201/101/103/103)
    # and is a candidate (SSC 4 at default options).
    def c256(q, per, bases=(A, C_, G, T), mq=None):
        out = []
        for b_, n_ in zip(bases, per):
            out += [R(q if mq is None else mq, q, b_, i & 1) for i in range(n_)]
        return out
    s.append(("A", c256(30, (127,) * 4, mq=60), c256(31, (127,) * 4, mq=60)))
    s.append(("C", c256(63, (127,) * 4), c256(31, (127,) * 4, mq=60)))
    s.append(("G", c256(30, (635,) * 4, mq=60), c256(63, (635,) * 4)))
    s.append(("T", c256(70, (127,) * 4), c256(45, (127,) * 4, mq=60)))
    s.append(("A", c256(40, (201, 101, 103, 103), bases=(T, A, C_, G), mq=60),
              c256(40, (201, 101, 103, 103), bases=(A, C_, G, T), mq=60)))
    return s


@pytest.mark.parametrize("opts", OPTSETS)
def test_quirk_parity(pkg, oracle, opts):
    batch = pkg.Batch.from_sites(quirk_sites(pkg))
    score, _ = assert_parity(pkg, oracle, batch, opts)
    assert score[9] == -1 and score[10] == -1     # empty packed sample
    assert score[11] == -1                        # ref N
    assert score[12] == 255                       # ref n: scored, not a candidate


@pytest.mark.parametrize("opts", [[], ["-J"]])
def test_single_strand_chains_parity(pkg, oracle, opts):
    """Fold chains as long as the lane path allows on one strand: w runs up to
    127, the last fk entry the main kernel's LDS copy keeps (entries 128 .. 255
    are zeros that lanes with fewer than four records left read, ln_chain).
    128 + 128 reads (separate mode), 100 + 28 (joint mode), 128 reads of a
    non-reference base, and a block of such sites next to shallow ones so that
    most lanes sit the long steps out."""
    R = lambda mq, bq, nt, st=0: _r(pkg, mq, bq, nt, st)
    A, C_, G, T = 1, 2, 4, 8
    s = []
    for k in range(3):
        s.append(("A", [R(60, 10 + (i * 7 + k) % 31, T, 0) for i in range(128)],
                  [R(60, 20 + (i * 3 + k) % 17, T, 1) for i in range(128)]))
        s.append(("G", [R(60, 5 + (i * 11 + k) % 40, G, 1) for i in range(100)],
                  [R(60, 30, G, 0)] * 27 + [R(60, 30, A, 0)]))
        s.append(("C", [R(60, 4 + (i * 5 + k) % 50, A, k & 1) for i in range(128)],
                  [R(60, 33, C_, 0)] * 40))
    for i in range(64 - len(s)):
        s.append(("T", [R(60, 30, T, i & 1)] * (1 + i % 5), [R(60, 30, T, 0)] * (1 + i % 3)))
    assert_parity(pkg, oracle, pkg.Batch.from_sites(s), opts)


def all_reference_sites(pkg):
    """Sites whose every read is on the reference base (round 5 measured an
    early exit for them): the count of reads of minq >= 24
    from 0 to all, at depths 1 .. 128 (the lane path's limit) and 129 (the
    group kernel); reads that count as the reference only through nt16
    semantics (N / IUPAC as A, '='); a single non-reference read that does not
    contribute (q = 0); soft-masked, 'n' and IUPAC references; somatic-looking
    sites among them; and single-strand low-quality (q 4) sites where another
    homozygote ties the reference's and sniper_glf2cns calls another base."""
    R = lambda mq, bq, nt, st=0: _r(pkg, mq, bq, nt, st)
    A, C_, G, T, N, EQ, M = 1, 2, 4, 8, 15, 0, 3
    code = {"A": A, "C": C_, "G": G, "T": T}
    rng = np.random.default_rng(7)
    s = []
    for i, n in enumerate([1, 2, 3, 7, 16, 30, 31, 60, 61, 64, 89, 100, 127, 128, 129]):
        for c24 in sorted({0, 1, max(0, n // 8 - 1), n // 8, n // 4, n}):
            c24 = min(c24, n)
            ref = "ACGT"[(i + c24) % 4]
            b = code[ref]
            t = [R(60, 24 + int(rng.integers(0, 18)), b, j & 1) for j in range(c24)] + \
                [R(int(rng.integers(0, 61)), 2 + int(rng.integers(0, 22)), b, j & 1) for j in range(n - c24)]
            nn = max(1, n // 2)
            nm = [R(60, 10 + int(rng.integers(0, 30)), b, j & 1) for j in range(nn)]
            s.append((ref, t, nm))
    for ref in "ACGT":
        b = code[ref]
        s.append((ref, [R(60, 30, N)] * 5 + [R(60, 30, b)] * 40, [R(60, 30, b)] * 30))       # N counts as A
        s.append((ref, [R(60, 30, M)] * 3 + [R(60, 30, b)] * 40, [R(60, 30, b)] * 30))       # IUPAC counts as A
        s.append((ref, [R(60, 30, EQ)] * 10 + [R(60, 30, b)] * 40, [R(60, 30, EQ)] * 30))    # '=' is the reference
        s.append((ref, [R(0, 0, T if b != T else A)] + [R(60, 30, b)] * 40, [R(60, 30, b)] * 30))  # q = 0 non-ref
        s.append((ref.lower(), [R(60, 30, b)] * 40, [R(60, 30, b)] * 30))                   # soft-masked reference
        s.append((ref, [R(60, 35, T if b != T else A, j & 1) for j in range(20)], [R(60, 35, b)] * 20))
    for ch in "nRYMK":
        s.append((ch, [R(60, 30, A)] * 40, [R(60, 30, A)] * 30))
    # every read on the reference, one strand, of low quality (q 4): the other
    # homozygotes' p (esum + coef[bar_e][n][n], coef < 0) rounds to lk 0 and
    # ties the reference's, and sniper_glf2cns calls another base (18 of these
    # sites score 0 or 9 in the reference)
    for ref in "CGT":
        b = code[ref]
        for n in (20, 60, 100, 128):
            s.append((ref, [R(60, 2 + (j % 2), b, 0) for j in range(n)], [R(60, 30, b)] * 30))
            s.append((ref, [R(60, 30, b)] * 30, [R(60, 2 + (j % 2), b, 1) for j in range(n)]))
    return s


@pytest.mark.parametrize("opts", [[], ["-J"], ["-T", "0.9", "-N", "3", "-r", "0.01"], ["-p", "-Q", "0"],
                                  ["-T", "1.2"]])
def test_all_reference_sites_parity(pkg, oracle, opts):
    """all_reference_sites against the oracle, with and without glf records,
    plus 60x/30x and 30x/25x batches with few errors (most sites
    all-reference; the shallow one takes the main kernel's early exit when
    scored without glf)."""
    batch = pkg.Batch.from_sites(all_reference_sites(pkg))
    assert_parity(pkg, oracle, batch, opts)
    for lt, ln in ((60, 30), (30, 25)):
        clean = pkg.synth_batch_host(pkg.Synth.default(lt, ln, seed=77, p_error=0.002, p_nbase=0.0005,
                                                       p_somatic=0.01, p_germline=0.01), 0, 20000)
        assert_parity(pkg, oracle, clean, opts)


@pytest.mark.parametrize("opts", [[], ["-J"], ["-p", "-Q", "0"]])
def test_early_exit_mixed_blocks(pkg, oracle, opts):
    """The main kernel's early exit is decided per 64-site block (mean depth
    <= 256 reads per site, in a batch of mean <= 264): shallow blocks
    (25x/20x) and deep ones (150x/120x, many of their sites past the lane
    path's 128 reads per sample) alternate, so the undecided sites of shallow
    blocks wait in the wave's queue while deep blocks are scored directly,
    and the queue's last, partial batch is scored at the end."""
    sh = pkg.synth_batch_host(pkg.Synth.default(25, 20, seed=91, **EXOTIC), 0, 64 * 40)
    dp = pkg.synth_batch_host(pkg.Synth.default(150, 120, seed=92, **EXOTIC), 0, 64 * 40 + 17)
    sites = []
    for b in range(40):
        sites += [sh.site(64 * b + i) for i in range(64)]
        sites += [dp.site(64 * b + i) for i in range(64)]
    sites += [dp.site(64 * 40 + i) for i in range(17)]
    assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), opts)


@pytest.mark.parametrize("opts", [[], ["-J"], ["-T", "0.9", "-N", "3", "-r", "0.01"], ["-p", "-Q", "0"],
                                  ["-T", "1.2"]])
def test_near_exit_parity(pkg, oracle, opts):
    """The early exit's near-reference test (round 6: up to three
    off-reference reads per sample) on the sites that press its
    bounds hardest (tests/test_early_exit_bound.py: few q-24 reference reads,
    off-reference reads of every quality, base, strand and baseQ class, some
    samples with one read more than the exit takes) and on synthetic pileups
    at 10x the default error rate with germline and somatic sites, at depths
    on both sides of the lane path's limits: every score, call and glf record
    against the oracle, with glf records (no exit) and without (exit)."""
    from test_early_exit_bound import _pressing_sites
    rng = np.random.default_rng(4242 + len(opts))
    assert_parity(pkg, oracle, pkg.Batch.from_sites(_pressing_sites(pkg, rng, 6000)), opts)
    for lt, ln in ((30, 20), (60, 30), (100, 60), (120, 110)):
        b = pkg.synth_batch_host(pkg.Synth.default(lt, ln, seed=55 + lt, p_error=0.1, p_somatic=0.02,
                                                   p_germline=0.02), 0, 6000)
        assert_parity(pkg, oracle, b, opts)


@pytest.mark.parametrize("opts", [[], ["-J"], ["-T", "0.9", "-N", "3", "-r", "0.01"], ["-T", "1.2"]])
def test_near_exit_deep_parity(pkg, oracle, opts):
    """The deep triage (samples of 129 .. 2048 reads, counts rescaled past 255,
    up to 16 off-reference reads per sample) on deep sites
    built to press its bounds (tests/test_early_exit_bound.py) and on
    synthetic panels at default and 10x error rates, mixed with shallow
    blocks: every output against the oracle, with and without glf."""
    from test_early_exit_bound import _pressing_sites
    rng = np.random.default_rng(9100 + len(opts))
    sites = _pressing_sites(pkg, rng, 600, nmax=700, mmax=17, c24max=80)
    sites += _pressing_sites(pkg, rng, 60, nmax=2048, mmax=17, c24max=80)
    sites += _pressing_sites(pkg, rng, 640, nmax=128)
    assert_parity(pkg, oracle, pkg.Batch.from_sites(sites), opts)
    for lt, ln, kw in ((500, 500, {}), (300, 280, dict(p_error=0.03, p_somatic=0.02, p_germline=0.02)),
                       (1200, 1000, {}), (150, 100, {})):
        b = pkg.synth_batch_host(pkg.Synth.default(lt, ln, seed=31 + lt, **kw), 0, 1200)
        assert_parity(pkg, oracle, b, opts)


@pytest.mark.parametrize("lt,ln,deep,left", [(60, 30, False, 0.01), (100, 60, False, 0.04), (500, 500, True, 0.001),
                                              (1200, 1000, True, 0.04)])
def test_triage_routing(pkg, lt, ln, deep, left):
    """Where the device path sends a synthetic batch's sites (the performance
    contract of DESIGN.md 4.0-4.0.1, not a parity check): the triage kernels
    decide all but a few per thousand, the deep triage takes exactly the
    blocks past 128 mean reads per sample, and what is left reaches the main
    kernel's list and, past 128 reads, the group or deep kernel."""
    import torch
    n = 1 << 16
    dev = torch.device("cuda", 0)
    with pkg.Context(pkg.Params.default(), device=0) as ctx:
        d = ctx.synth_device(pkg.Synth.default(lt, ln, seed=5), 0, n, device=dev)
        score = torch.empty(n, dtype=torch.int32, device=dev)
        ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"], score=score)
        torch.cuda.synchronize(dev)
        ctx.check()
        r = ctx._route_counts()
    assert r["deep_triage_blocks"] == (n // 64 if deep else 0), r
    assert r["main_sites"] <= left * n, r
    assert r["group_sites"] + r["deep_sites"] <= r["main_sites"], r
    assert (score.cpu().numpy() == 255).mean() > 0.9


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_misaligned_read_arrays(pkg, oracle, shift):
    """Device-resident read arrays that start 4, 8 or 12 bytes past a 16-byte
    boundary (views into larger buffers): the kernels' 16-byte chunk loads
    are then misaligned everywhere and the last site's last chunk ends within
    three elements of the array's end.  Deep, shallow and mixed blocks, every
    score against the oracle, with the routing through both triage kernels
    checked."""
    import torch
    from test_early_exit_bound import _pressing_sites
    rng = np.random.default_rng(4400 + shift)
    sites = _pressing_sites(pkg, rng, 200, nmax=700, mmax=17, c24max=80)
    sites += _pressing_sites(pkg, rng, 200, nmax=128)
    b1 = pkg.synth_batch_host(pkg.Synth.default(500, 500, seed=77 + shift), 0, 256)
    b2 = pkg.synth_batch_host(pkg.Synth.default(60, 30, seed=78 + shift), 0, 256)
    sites += [b1.site(i) for i in range(b1.n_sites)] + [b2.site(i) for i in range(b2.n_sites)]
    batch = pkg.Batch.from_sites(sites)
    o = oracle.Oracle(oracle.opts_to_params([]))
    o_score, _, _ = o.score_batch(batch.ref, batch.off_tumor, batch.off_normal, batch.reads_tumor,
                                  batch.reads_normal, want_glf=False)
    dev = torch.device("cuda", 0)

    def shifted(x):
        buf = torch.full((x.size + shift + 4,), 0xFFFFFFFF, dtype=torch.int64).to(torch.int32)
        buf[shift:shift + x.size] = torch.from_numpy(x.view(np.int32))
        return buf.to(dev)[shift:shift + x.size]

    rt, rn = shifted(batch.reads_tumor), shifted(batch.reads_normal)
    assert rt.data_ptr() % 16 == 4 * shift and rn.data_ptr() % 16 == 4 * shift
    t = {k: torch.from_numpy(getattr(batch, k).view(np.int32) if getattr(batch, k).dtype == np.uint32
                             else getattr(batch, k)).to(dev) for k in ("ref", "off_tumor", "off_normal")}
    score = torch.empty(batch.n_sites, dtype=torch.int32, device=dev)
    with pkg.Context(pkg.Params.default(), device=0) as ctx:
        ctx.score_device(t["ref"], t["off_tumor"], t["off_normal"], rt, rn, score=score)
        torch.cuda.synchronize(dev)
        ctx.check()
        route = ctx._route_counts()
    got = score.cpu().numpy()
    bad = np.nonzero(got != o_score)[0]
    assert bad.size == 0, f"{bad.size} score mismatches, first {bad[:5]}: gpu {got[bad[:5]]} oracle {o_score[bad[:5]]}"
    assert route["deep_triage_blocks"] > 0


@pytest.mark.parametrize("opts", [[], ["-J"], ["-p", "-Q", "0"], ["-T", "1.2"]])
def test_all_reference_sites_match_real_reference(pkg, tmp_path, opts):
    """all_reference_sites through the compiled reference on THIS machine vs
    the GPU (no glf records requested)."""
    import os
    from oracle import binding as ob
    if not os.path.exists(ob.REF_HARNESS):
        pytest.skip("reference harness not built")
    b = pkg.Batch.from_sites(all_reference_sites(pkg))
    path = str(tmp_path / "e.ssb")
    ob.write_ssb(path, b.ref, b.off_tumor, b.off_normal, b.reads_tumor, b.reads_normal)
    rec, txt = ob.run_ref_dump(path, opts, str(tmp_path))
    with pkg.Context(params_from_opts(pkg, opts)) as c:
        score, calls, _ = c.score_batch(b, want_glf=False)
    assert (score == rec["ret"]).all(), np.nonzero(score != rec["ret"])
    assert len(calls) == txt.count("\n")


@pytest.mark.parametrize("opts", [[], ["-J"], ["-p", "-Q", "0"]])
def test_quirks_match_real_reference_on_this_host(pkg, tmp_path, opts):
    """The hand-built quirk sites (Appendix A, the sum-of-counts-256 coef index
    included) through the compiled reference on THIS machine vs the GPU."""
    import os
    from oracle import binding as ob
    if not os.path.exists(ob.REF_HARNESS):
        pytest.skip("reference harness not built")
    b = pkg.Batch.from_sites(quirk_sites(pkg))
    path = str(tmp_path / "q.ssb")
    ob.write_ssb(path, b.ref, b.off_tumor, b.off_normal, b.reads_tumor, b.reads_normal)
    rec, txt = ob.run_ref_dump(path, opts, str(tmp_path))
    with pkg.Context(params_from_opts(pkg, opts)) as c:
        score, calls, glf = c.score_batch(b, want_glf=True)
    assert (score == rec["ret"]).all(), np.nonzero(score != rec["ret"])
    assert (glf.view(np.uint8) == rec["glf"].view(np.uint8)).all()
    assert len(calls) == txt.count("\n")


def test_device_synth_matches_host(pkg, ctx):
    torch = pytest.importorskip("torch")
    synth = pkg.Synth.default(60, 30, **EXOTIC)
    d = ctx.synth_device(synth, 777, 5000)
    h = pkg.synth_batch_host(synth, 777, 5000)
    nt, nn = d["n_reads"]
    assert nt == h.off_tumor[-1] and nn == h.off_normal[-1]
    assert (d["ref"].cpu().numpy() == h.ref).all()
    assert (d["off_tumor"].cpu().numpy().view(np.uint32) == h.off_tumor).all()
    assert (d["off_normal"].cpu().numpy().view(np.uint32) == h.off_normal).all()
    assert (d["reads_tumor"][:nt].cpu().numpy().view(np.uint32) == h.reads_tumor).all()
    assert (d["reads_normal"][:nn].cpu().numpy().view(np.uint32) == h.reads_normal).all()


def test_device_batch_full_size_properties(pkg, oracle, ctx):
    """BASELINE workload shape (60x/30x) at 2M sites, HBM-resident: deterministic,
    sampled windows bit-exact against the oracle, calls compacted correctly."""
    torch = pytest.importorskip("torch")
    n = 2_000_000
    synth = pkg.Synth.default(60, 30)
    d = ctx.synth_device(synth, 0, n)
    dev = d["ref"].device
    score = torch.empty(n, dtype=torch.int32, device=dev)
    cap = 1 << 16
    calls = torch.zeros(cap * 28, dtype=torch.uint8, device=dev)
    ncalls = torch.zeros(1, dtype=torch.int32, device=dev)
    args = (d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"])
    ctx.score_device(*args, score=score, calls=calls, calls_cap=cap, n_calls=ncalls)
    ctx.check()
    s1 = score.cpu().numpy()
    ctx.score_device(*args, score=score, calls=calls, calls_cap=cap, n_calls=ncalls)
    ctx.check()
    assert (score.cpu().numpy() == s1).all(), "non-deterministic"
    k = int(ncalls.item())
    c = calls.cpu().numpy()[: k * 28].view(pkg.SS_CALL_DTYPE)
    assert len(np.unique(c["site"])) == k
    assert set(np.unique(s1)) >= {255}
    emitted = np.sort(c["site"])
    for first in (0, 777_777, n - 4000):
        h = pkg.synth_batch_host(synth, first, 4000)
        o_score, o_calls, _ = oracle.Oracle().score_batch(h.ref, h.off_tumor, h.off_normal,
                                                          h.reads_tumor, h.reads_normal, want_glf=False)
        assert (s1[first:first + 4000] == o_score).all()
        win = emitted[(emitted >= first) & (emitted < first + 4000)] - first
        assert (win == o_calls["site"]).all()


def test_gpu_matches_real_reference_on_this_host(pkg, tmp_path):
    """The compiled reference (oracle/_ref/ref_harness, built from /root/reference
    and shipped as a binary) run on THIS machine vs the GPU, same inputs."""
    import os
    from oracle import binding as ob
    if not os.path.exists(ob.REF_HARNESS):
        pytest.skip("reference harness not built")
    for lt, ln, kw, opts in [(60, 30, EXOTIC, []), (60, 30, EXOTIC, ["-J"]), (100, 60, {}, []),
                             (3, 2, dict(p_wild_qual=0.3, p_del=0.3, p_somatic=0.1), ["-Q", "0"]),
                             (400, 400, EXOTIC, [])]:
        b = pkg.synth_batch_host(pkg.Synth.default(lt, ln, seed=99, **kw), 0, 2000 if lt < 300 else 60)
        path = str(tmp_path / "b.ssb")
        ob.write_ssb(path, b.ref, b.off_tumor, b.off_normal, b.reads_tumor, b.reads_normal)
        rec, txt = ob.run_ref_dump(path, opts, str(tmp_path))
        with pkg.Context(params_from_opts(pkg, opts)) as c:
            score, calls, glf = c.score_batch(b, want_glf=True)
        assert (score == rec["ret"]).all()
        assert (glf.view(np.uint8) == rec["glf"].view(np.uint8)).all()
        assert len(calls) == txt.count("\n")


@pytest.mark.parametrize("lt,ln,n,opts", [(60, 30, 1 << 22, []), (30, 30, 1 << 22, []), (100, 60, 1 << 21, []),
                                          (500, 500, 1 << 16, []), (500, 500, 1 << 16, ["-J"]),
                                          (500, 500, 1 << 16, ["-T", "0.9", "-N", "3", "-r", "0.01"])])
def test_full_size_batch_vs_real_reference(pkg, tmp_path, lt, ln, n, opts):
    """Large batches of the BASELINE depth configurations (C4 60x/30x -- the
    headline --, C2, C3, C5; default seed, shard 0), generated and scored in
    HBM, against the compiled reference's glf_somatic on the same sites run on
    this host by 16 processes (oracle/_ref/ref_harness synth --first): every
    site's return value bit-exact.  C5 (the wide kernel's depth) also under
    -J and under -T/-N/-r (other fk / coef / lhet tables)."""
    import os
    import subprocess
    torch = pytest.importorskip("torch")
    from oracle import binding as ob
    if not os.path.exists(ob.REF_HARNESS):
        pytest.skip("reference harness not built")
    procs = 16
    with pkg.Context(params_from_opts(pkg, opts), device=0) as ctx:
        d = ctx.synth_device(pkg.Synth.default(lt, ln), 0, n)
        score = torch.empty(n, dtype=torch.int32, device=d["ref"].device)
        ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"],
                         score=score)
        ctx.check()
        gpu = score.cpu().numpy()
        del d
    step = n // procs
    runs = []
    for k in range(procs):
        out = str(tmp_path / f"s{k}.bin")
        runs.append((out, subprocess.Popen([ob.REF_HARNESS, "synth", str(lt), str(ln), str(step), "--first",
                                            str(k * step), "--scores", out] + list(opts),
                                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)))
    for out, p in runs:
        assert p.wait(timeout=100) == 0, p.stderr.read()[-500:]
    ref = np.concatenate([np.fromfile(out, np.int32) for out, _ in runs])
    assert ref.shape == (n,)
    bad = np.nonzero(gpu != ref)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: gpu {gpu[bad[:5]]} reference {ref[bad[:5]]}"
    assert (ref == 255).sum() > n // 2


def test_tables_equal_reference_on_this_host(pkg):
    import json
    import os
    import subprocess
    from oracle import binding as ob
    if not os.path.exists(ob.REF_HARNESS):
        pytest.skip("reference harness not built")
    ref = json.loads(subprocess.run([ob.REF_HARNESS, "tables"], check=True, capture_output=True,
                                    text=True).stdout)
    with pkg.Context() as c:
        h = c.table_hashes()
    for k in ("fk", "coef", "lhet"):
        assert h[k] == ref[k], k
