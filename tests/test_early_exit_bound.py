"""The main kernel's early exit (ss_kernels.hip ln_classify)
scores an all-reference site 255 without computing likelihoods when each
sample has at least thr[n] reads of minq >= 24, thr from the host table
(ss_capi.hip fast_table: the smallest c24 with
24 * (m[0] + .. + m[c24 - 1]) * (1 - 1e-4) + min coef[q][n'][n'] >= 1 over
q in [4, 63], n' <= n, m[k] = min(fk[0 .. k]), enabled only with q_r >= 1).
The running minimum keeps the bound sound when fk increases (theta > 1, which
the reference's -T accepts: main.c:83 has no range check).

This CPU test restates that table from the oracle's own model tables and
checks the rule's soundness against the oracle (pinned to the compiled
reference by test_oracle_golden.py) on the sites that press it hardest, at
every depth 1 .. 128: exactly thr[n] reads of q 24 (the smallest weight the
bound assumes), every other read at the lowest contributing quality (q 4) or
not contributing at all, one strand or alternating strands, every reference
base, under option sets that change the model tables.  No GPU."""
import numpy as np
import pytest


def fast_thresholds(fk, coef, q_r):
    """ss_capi.hip fast_table, restated: 255 = the exit never applies."""
    thr = np.full(256, 255, np.int64)
    if q_r < 1:
        return thr
    F = np.zeros(130)
    run_min = fk[0]
    for k in range(129):
        run_min = min(run_min, fk[min(k, 255)])
        F[k + 1] = F[k] + run_min
    cm = 1e300
    for n in range(1, 129):
        cm = min(cm, min(coef[q << 16 | n << 8 | n] for q in range(4, 64)))
        for c in range(1, n + 1):
            if 24.0 * F[c] * (1.0 - 1e-4) + cm >= 1.0:
                thr[n] = c
                break
    return thr


def _sample(pkg, base, n, c24, rest_bq, alternate):
    # alternating strands give the q-24 reads the weights fk[0], fk[0], fk[1],
    # fk[1], ...: the smallest ones when fk increases (theta > 1)
    reads = [pkg.pack_read(60, 24, base, (i & 1) if alternate else 0) for i in range(c24)]
    reads += [pkg.pack_read(60, rest_bq, base, (i & 1) if alternate else 0) for i in range(n - c24)]
    return reads


@pytest.mark.parametrize("opts", [[], ["-J"], ["-T", "0.9", "-N", "3", "-r", "0.01"], ["-p", "-Q", "0"],
                                  ["-T", "1.2"]])
def test_early_exit_thresholds_sound(pkg, oracle, opts):
    o = oracle.Oracle(oracle.opts_to_params(list(opts)))
    t = o.tables()
    thr = fast_thresholds(t["fk"], t["coef"], t["q_r"])
    if t["q_r"] < 1:
        pytest.skip("q_r < 1: the exit is disabled")
    assert (thr[1:129] < 255).any(), "the exit would never apply"
    sites = []
    for n in range(1, 129):
        if thr[n] == 255:
            continue
        for base, refc in ((1, "A"), (2, "C"), (4, "G"), (8, "T")):
            for rest_bq, alternate in ((4, False), (4, True), (0, True)):
                t_reads = _sample(pkg, base, n, int(thr[n]), rest_bq, alternate)
                m = max(1, n // 2)          # the normal at another depth, at its own threshold
                if thr[m] == 255:
                    continue
                n_reads = _sample(pkg, base, m, int(thr[m]), rest_bq, not alternate)
                sites.append((refc, t_reads, n_reads))
    assert len(sites) > 1000
    batch = pkg.Batch.from_sites(sites)
    score, _, _ = o.score_batch(batch.ref, batch.off_tumor, batch.off_normal, batch.reads_tumor,
                                batch.reads_normal, want_glf=False)
    bad = np.nonzero(score != 255)[0]
    assert bad.size == 0, f"{bad.size} all-reference sites at the threshold not scored 255, first {bad[:5]}"
