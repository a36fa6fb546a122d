"""The main kernel's early exit (ss_kernels.hip ln_classify /
ln_near_sample) scores a site 255 without its full likelihoods when, in both
samples, at most three contributing reads lie off the reference base and the
bounds of ss_capi.hip near_tables prove that sniper_glf2cns calls the
reference homozygote (tests/near_exit_model.py restates both).

These CPU tests check that rule's soundness against the oracle (pinned to the
compiled reference by test_oracle_golden.py): every site the model exits must
score 255 in the oracle.  The sites press the bound hardest -- few reads of
q >= 24 on the reference (exactly the smallest weight the bound assumes), the
rest at q 4 or not contributing, one strand or alternating strands, and up to
three off-reference reads of every quality, base, strand and baseQ tie-break
class -- under option sets that change the model tables, including theta > 1
(fk increasing; the reference's -T has no range check, main.c:83).  No GPU."""
import numpy as np
import pytest

from near_exit_model import MAXN, NEAR_K, near_exit, near_tables

NEAR_K_SHALLOW = 3          # off-reference reads per sample the shallow triage takes

OPTS = [[], ["-J"], ["-T", "0.9", "-N", "3", "-r", "0.01"], ["-p", "-Q", "0"], ["-T", "1.2"]]
REF16 = {"A": 1, "C": 2, "G": 4, "T": 8}


def _pressing_sites(pkg, rng, n_sites, nmax=128, mmax=NEAR_K_SHALLOW + 1, c24max=14):
    sites = []
    for _ in range(n_sites):
        refc = "ACGT"[rng.integers(4)]
        r = "ACGT".index(refc)
        smp = []
        for _s in range(2):
            n = int(rng.integers(1, nmax + 1))
            c24 = int(min(n, rng.integers(0, c24max)))
            alt = bool(rng.integers(2))
            rest_bq = int(rng.choice([4, 4, 0, 7, 23, 130]))
            reads = [pkg.pack_read(60, 24, 1 << r, (i & 1) if alt else 0) for i in range(c24)]
            reads += [pkg.pack_read(60 if rest_bq else int(rng.integers(0, 60)), rest_bq, 1 << r,
                                    (i & 1) if alt else int(rng.integers(2))) for i in range(n - c24)]
            m = int(rng.integers(0, mmax + 1))           # sometimes one more than the exit takes
            for _j in range(m):
                b = int(rng.integers(4))
                nt16 = int(rng.choice([1 << b, 15, 5, 0])) if b != r else 15
                bq = int(rng.choice([int(rng.integers(1, 64)), int(rng.integers(64, 256)), 2, 3, 64, 128]))
                mq = int(rng.choice([60, int(rng.integers(0, 256)), 2]))
                reads.insert(int(rng.integers(len(reads) + 1)),
                             pkg.pack_read(mq, bq, nt16, int(rng.integers(2))))
            smp.append(reads[:nmax])
        sites.append((refc, smp[0], smp[1]))
    return sites


def _ref16(rc):
    return REF16.get((rc if isinstance(rc, str) else chr(rc)).upper(), 15)


def _check(pkg, oracle, o, sites, t, tabs, min_exits, per_strand=False):
    exits = np.array([near_exit(_ref16(rc), rt, rn, tabs, t, per_strand) for rc, rt, rn in sites])
    batch = pkg.Batch.from_sites(sites)
    score, _, _ = o.score_batch(batch.ref, batch.off_tumor, batch.off_normal, batch.reads_tumor,
                                batch.reads_normal, want_glf=False)
    bad = np.nonzero(exits & (score != 255))[0]
    assert bad.size == 0, f"{bad.size} sites the exit scores 255 score otherwise, first {bad[:5]} {score[bad[:5]]}"
    assert exits.sum() >= min_exits, f"the exit took only {exits.sum()} of {len(sites)} sites"
    assert (~exits).sum() > 0
    return exits


@pytest.mark.parametrize("opts", OPTS)
def test_near_exit_sound_pressing(pkg, oracle, opts):
    o = oracle.Oracle(oracle.opts_to_params(list(opts)))
    t = o.tables()
    tabs = near_tables(t["fk"], t["coef"], t["lhet"], t["q_r"])
    if tabs is None:
        pytest.skip("q_r < 1: the exit is disabled")
    rng = np.random.default_rng(20260 + len(opts))
    sites = _pressing_sites(pkg, rng, 2500)
    _check(pkg, oracle, o, sites, t, tabs, min_exits=150)
    # the deep triage's per-strand bound on the same sites (it takes every
    # site of a block past 128 mean reads, shallow ones included)
    _check(pkg, oracle, o, sites, t, tabs, min_exits=150, per_strand=True)


@pytest.mark.parametrize("opts", [[], ["-T", "1.2"], ["-T", "0.9", "-N", "3", "-r", "0.01"]])
def test_near_exit_sound_deep(pkg, oracle, opts):
    """the deep triage's samples (129 .. 2048 reads: counts rescaled past
    255, up to 16 off-reference reads per sample), pressed the same way"""
    o = oracle.Oracle(oracle.opts_to_params(list(opts)))
    t = o.tables()
    tabs = near_tables(t["fk"], t["coef"], t["lhet"], t["q_r"])
    rng = np.random.default_rng(777 + len(opts))
    sites = _pressing_sites(pkg, rng, 400, nmax=700, mmax=NEAR_K + 1, c24max=80)
    sites += _pressing_sites(pkg, rng, 40, nmax=MAXN, mmax=NEAR_K + 1, c24max=80)
    _check(pkg, oracle, o, sites, t, tabs, min_exits=5, per_strand=True)


@pytest.mark.parametrize("opts", [[], ["-T", "1.2"]])
def test_near_exit_sound_noisy_synth(pkg, oracle, opts):
    """synthetic pileups at 10x the default error rate, with germline and
    somatic sites, at 30x/20x: most sites carry off-reference reads"""
    o = oracle.Oracle(oracle.opts_to_params(list(opts)))
    t = o.tables()
    tabs = near_tables(t["fk"], t["coef"], t["lhet"], t["q_r"])
    b = pkg.synth_batch_host(pkg.Synth.default(30, 20, p_error=0.1, p_somatic=0.02, p_germline=0.02), 0, 2500)
    sites = [b.site(i) for i in range(b.n_sites)]
    _check(pkg, oracle, o, sites, t, tabs, min_exits=200)


def test_near_tables_bound_esum(oracle):
    """esr[c] never exceeds the smallest esum of c q-24 reads: the reads
    alternate strands (weights fk[0], fk[0], fk[1], ..) or keep one (fk[0],
    fk[1], ..), whichever is smaller, with the float accumulation of the fold"""
    for opts in OPTS:
        o = oracle.Oracle(oracle.opts_to_params(list(opts)))
        t = o.tables()
        tabs = near_tables(t["fk"], t["coef"], t["lhet"], t["q_r"])
        if tabs is None:
            continue
        fk = t["fk"]
        for c in range(1, 129):
            lo = None
            for alt in (False, True):
                e = np.float32(0)
                for i in range(c):
                    e = np.float32(float(e) + float(fk[i // 2 if alt else i]) * 24.0)
                lo = e if lo is None else min(lo, e)
            assert tabs[0][c] <= lo, (opts, c, tabs[0][c], lo)
