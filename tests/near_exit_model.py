"""CPU restatement of the main kernel's early exit (ss_kernels.hip ln_classify /
ln_near_sample) -- test infrastructure, not a product path.

For a site of reference A/C/G/T with <= 2048 reads per sample, the exit writes
255 (not a candidate, somatic_sniper.c:156) when in both samples
  * at most NEAR_K contributing reads lie off the reference base's group (the
    kernels take 3 in blocks of <= 128 reads per sample, 16 past them: their
    exits are a subset of this model's);
  * those reads' group chains (sniper_maqcns.c:162-172) give the four
    genotypes with the reference base exactly (:184-214), and a lower bound
    esr[c24] + cmin[tot] covers the six without it (ss_capi.hip near_tables;
    the deep triage bounds the reference group's two strand chains apart,
    esr[c24 on strand 0] + esr[c24 on strand 1]: per_strand);
  * the bounds put the reference homozygote first in sniper_glf2cns
    (:250-273), with the homozygote fix (:216-233) not firing.
`near_tables` restates the host tables, `near_exit` the device test with the
same float / double operations, so the soundness test can score the sites the
model exits with the oracle (tests/test_early_exit_bound.py)."""
import numpy as np

NEAR_K = 16          # off-reference reads per sample (the deep test's; the shallow one takes 3)
MAXN = 2048          # reads per sample
NT4 = {1: 0, 2: 1, 4: 2, 8: 3}
F32 = np.float32


def _round_down_f(x):
    f = np.float32(x)
    if float(f) > x:
        f = np.nextafter(f, np.float32(-np.inf))
    return f


def near_tables(fk, coef, lhet, q_r):
    """ss_capi.hip near_tables: (esr[2052], cmin[260]) float32, None when disabled."""
    q_r_int = int(q_r + 0.5)
    if q_r_int < 1:
        return None
    esr = np.zeros(2052, np.float32)
    cmin = np.full(260, -1e30, np.float32)
    F, run_min = 0.0, fk[0]
    for k in range(MAXN):
        run_min = min(run_min, fk[min(k, 255)])
        F += run_min
        esr[k + 1] = _round_down_f(24.0 * F * (1.0 - 2e-4))
    lh = min(0.0, float(np.min(-4.343 * lhet)))
    for n in range(1, 257):
        # the reference's index, OR and all (n = 256 aliases into the next q row)
        idx = [(q << 16) | (n << 8) | k for q in range(4, 64) for k in range(1, n + 1)]
        cm = float(np.min(coef[idx]))
        cmin[n] = _round_down_f(cm + lh - 0.01)
    return esr, cmin


def _bar_e(e, f):
    be = int(float(F32(e) / F32(f)) + 0.5)
    return 4 if be < 4 else (63 if be > 63 else be)


def _sample(reads, r, ref16, tabs, t, per_strand=False):
    """one sample's test; None = the exit does not apply"""
    esr, cmin = tabs
    fk, coef, lhet, q_r_int = t["fk"], t["coef"], t["lhet"], int(t["q_r"] + 0.5)
    c = [0, 0, 0, 0]
    c24 = c24s1 = 0
    keys = []
    for x in reads:
        x = int(x)
        mapq, bq, nt16, st = x & 0xFF, (x >> 8) & 0xFF, (x >> 16) & 0xF, (x >> 20) & 1
        minq = min(mapq, bq)
        if minq == 0 and (bq & 0x3F) == 0:
            continue                                   # q = 0 after the clamp: not contributing
        code = nt16 if nt16 else ref16
        nt4 = NT4.get(code, 4)
        base, hb = (nt4, 1) if nt4 < 4 else (0, 0)
        c[base] += 1
        if minq >= 24:
            c24 += 1
            c24s1 += st
        if base != r:
            keys.append(base << 13 | minq << 5 | hb << 4 | st << 3 | (bq >> 6) << 1 | (1 if bq & 0x3F else 0))
    if len(keys) > NEAR_K:
        return None
    keys.sort(reverse=True)
    es, fs = [F32(0)] * 4, [F32(0)] * 4
    seen = {}
    c24nr = c24nr1 = 0
    for key in keys:
        x = (key >> 13) & 3
        minq = (key >> 5) & 0xFF
        q = max(minq, (key & 1) << 2)
        g = key & 0x6008
        w = seen.get(g, 0)
        seen[g] = w + 1
        fv = float(fk[w])
        es[x] = F32(float(es[x]) + fv * float(q))
        fs[x] = F32(float(fs[x]) + fv)
        if minq >= 24:
            c24nr += 1
            c24nr1 += (key >> 3) & 1
    if sum(c) > 255:                                    # the rescale of sniper_maqcns.c:178-182
        t0 = sum(c)
        c = [int(254.0 * cj / t0 + 0.5) for cj in c]
    tot = sum(c)
    pv = []
    for tt in range(4):
        x = tt + (1 if tt >= r else 0) if tt < 3 else r
        e, f, c2 = F32(0), F32(0), 0
        for i in range(4):
            if i != r and i != x:
                e = F32(e + es[i])
                f = F32(f + fs[i])
                c2 += c[i]
        cf = float(coef[_bar_e(e, f) << 16 | tot << 8 | c2]) if c2 else 0.0
        if tt == 3:
            v = F32(float(e) + cf) if c2 else F32(0)
        else:
            j0, k0 = min(r, x), max(r, x)
            lh = -4.343 * float(lhet[c[j0] << 8 | c[k0]])
            v = F32((lh + float(e)) + cf) if c2 else F32(lh)
        pv.append(F32(0) if v < 0 else v)
    if per_strand:
        r1 = c24s1 - c24nr1
        e_r = F32(esr[c24 - c24nr - r1] + esr[r1])
    else:
        e_r = esr[c24 - c24nr]
    lb = F32(e_r + cmin[tot])
    phr = pv[3]
    min_p = min(phr, pv[0], pv[1], pv[2])
    ok = e_r > max(es) and F32(lb - phr) >= 3 and F32(phr - min_p) <= 250 and c[r] > 0
    lhr = int(float(F32(phr - min_p)) + 0.5)
    for tt in range(3):
        d = F32(pv[tt] - min_p)
        sc = (255 if float(d) > 255.0 else int(float(d) + 0.5)) + q_r_int
        ok = ok and (sc > lhr if tt < r else sc >= lhr)
    return ok


def near_exit(ref16, reads_t, reads_n, tabs, t, per_strand=False):
    """True when the exit scores the site 255 through the near-reference test
    (ref16: the reference's nt16 code; 'N', empty samples and IUPAC
    references are decided before this test).  per_strand: the deep
    triage's bound of the reference group's esum."""
    if tabs is None or ref16 not in NT4 or not (1 <= len(reads_t) <= MAXN and 1 <= len(reads_n) <= MAXN):
        return False
    r = NT4[ref16]
    return (bool(_sample(reads_t, r, ref16, tabs, t, per_strand)) and
            bool(_sample(reads_n, r, ref16, tabs, t, per_strand)))
