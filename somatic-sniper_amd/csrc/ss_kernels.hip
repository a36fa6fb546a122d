/*
 * ss_kernels.hip -- CDNA4 (gfx950) kernels of the somatic site scorer.
 *
 * One pileup site = one call of the reference's glf_somatic
 * (src/lib/sniper/somatic_sniper.c:109-273): two MAQ genotype-likelihood
 * evaluations (sniper_maqcns_glfgen, sniper_maqcns.c:127-248), two consensus
 * calls (sniper_glf2cns, :250-273) and the Phred-space somatic posterior.
 *
 * Work decomposition (DESIGN.md "Kernels"):
 *   ss_score_main   one 64-lane wave scores a GROUP of up to 8 sites:
 *     A  per site and sample, the wave loads the packed reads (coalesced),
 *        builds order keys and bitonic-sorts them in registers (1/2/4 keys per
 *        lane); sorted keys land in a per-wave LDS arena, grouped by base.
 *     B  ordered fold: lane (site, sample, base) walks its base group in
 *        descending key order accumulating esum/fsum -- the reference's float
 *        accumulators fed double increments (sniper_maqcns.c:162-172); this is
 *        the inherently serial part, 64 independent chains per wave.
 *     C  every lane evaluates the 10 genotype likelihoods + quantisation +
 *        consensus for its (site, sample) from quad-shuffled sums.
 *     D  lane s decides site s: gate, SNV candidate test, posteriors, joint
 *        prior, emit filter; emitted sites are compacted with one atomic.
 *   ss_score_deep   one 256-thread block per site with a sample deeper than
 *        SS_MAIN_MAXN: block bitonic sort in LDS (<= SS_DEEP_MAXN keys per
 *        sample) or, for giant pileups, in a global scratch slice; then the
 *        same B/C/D device code.
 *
 * Bit-exactness: built with -ffp-contract=off (no FMA contraction); float
 * division and double sqrt are correctly rounded (sqrt re-checked with fma);
 * accumulation order equals the reference's descending-key order.
 */
#include "ss_kernels.h"

#define SENT 0xffffffffu
#define GMAX 8              /* sites per wave group               */

namespace {

/* --------------------------------------------------------------------------
 * small helpers
 * ------------------------------------------------------------------------ */
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

/* bam_nt16_nt4_table (sniper_maqcns.c:19): single-base codes -> 0..3, else 4 */
__device__ __forceinline__ uint32_t nt16_to_nt4(uint32_t b)
{
    return (b != 0u && (b & (b - 1u)) == 0u) ? (uint32_t)__builtin_ctz(b) : 4u;
}

/* Sum over the 64 lanes with DPP row shifts + row broadcasts (no LDS
 * round trip); the total ends in lane 63 and is returned wave-uniform. */
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false); /* row_shr:1 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false); /* row_shr:2 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false); /* row_shr:4 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false); /* row_shr:8 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); /* row_bcast:15 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); /* row_bcast:31 */
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

/* --------------------------------------------------------------------------
 * Order key of one packed read (sniper_maqcns.c:144-156 restated).
 *
 * The reference sorts  minq<<24 | hasbase<<21 | strand<<18 | nt4<<16 |
 * baseQ<<8 | mapQ  and folds in descending order, one accumulator per base.
 * Only the order WITHIN a base matters, and within a base nt4 is constant, so
 * we sort on  base<<26 | minq<<18 | hasbase<<17 | strand<<16 | baseQ<<8 | mapQ,
 * which yields each base's reads as one contiguous ascending run whose
 * descending walk is exactly the reference's sequence.  Reads whose clamped
 * quality q is 0 never touch esum/fsum/w/c (:165-172): they become SENT and
 * sort to the end.  rms (:173) is accumulated for every read.
 * ------------------------------------------------------------------------ */
__device__ __forceinline__ uint32_t read_key(uint32_t rd, uint32_t ref16, uint32_t cap,
                                             uint32_t &rms_term)
{
    const uint32_t mq = rd & 0xffu, bq = (rd >> 8) & 0xffu;
    const uint32_t nt = (rd >> 16) & 0xfu, st = (rd >> 20) & 1u;
    uint32_t t = mq & 0x7fu;
    t = t < cap ? t : cap;
    rms_term = t * t;
    const uint32_t minq = mq < bq ? mq : bq;
    const bool valid = minq != 0u || (bq & 0x3fu) != 0u;
    const uint32_t nt4 = nt16_to_nt4(nt ? nt : ref16);
    const uint32_t hb = nt4 < 4u ? 1u : 0u;
    const uint32_t base = hb ? nt4 : 0u;  /* N / IUPAC count as A (Appendix A.1) */
    return valid ? (base << 26 | minq << 18 | hb << 17 | st << 16 | bq << 8 | mq) : SENT;
}

/* --------------------------------------------------------------------------
 * Wave bitonic sort, ascending, of 64*K keys held lane-major (element
 * e = lane*K + r in v[r]).  Distances < K are register compare-exchanges,
 * larger ones cross lanes.  Input placement is arbitrary.
 * ------------------------------------------------------------------------ */
template <int K>
__device__ __forceinline__ void wave_bitonic(uint32_t (&v)[K])
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t k = 2; k <= 64u * K; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (j >= (uint32_t)K) {
                const int lj = (int)(j / K);
#pragma unroll
                for (int r = 0; r < K; ++r) {
                    const uint32_t e = lane * K + r;
                    const uint32_t o = (uint32_t)__shfl_xor((int)v[r], lj);
                    const bool up = (e & k) == 0u, lower = (e & j) == 0u;
                    v[r] = (lower == up) ? (v[r] < o ? v[r] : o) : (v[r] > o ? v[r] : o);
                }
            } else {
#pragma unroll
                for (int r = 0; r < K; ++r) {
                    const int r2 = r ^ (int)j;
                    if (r2 > r) {
                        const uint32_t e = lane * K + r;
                        const bool up = (e & k) == 0u;
                        const uint32_t a = v[r], b = v[r2];
                        const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
                        v[r] = up ? lo : hi;
                        v[r2] = up ? hi : lo;
                    }
                }
            }
        }
    }
}

/* per (site, sample) bookkeeping kept in LDS */
struct SlotMeta {
    uint32_t base;      /* arena offset of the sorted keys */
    uint32_t start[4];  /* base group start (relative)      */
    uint32_t cnt[4];    /* base group size == reference c[] before rescale */
    uint32_t n;         /* non-deleted depth                */
    uint32_t rms_lo, rms_hi;
};

struct SlotRes {
    uint8_t  lk[12];
    uint32_t cns;
    uint32_t depth;
    uint8_t  min_lk, rms_q, pad0, pad1;
};

struct SiteInfo {
    uint32_t site;
    uint32_t refc;
};

/* Phase A for one sample of one site, K keys per lane (n <= 64*K). */
template <int K>
__device__ __forceinline__ void sort_sample(const uint32_t *__restrict__ reads, uint32_t n,
                                            uint32_t ref16, uint32_t cap, uint32_t *arena,
                                            SlotMeta &meta, uint32_t &nvalid, uint32_t diag)
{
    const uint32_t lane = lane_id();
    uint32_t v[K];
    uint32_t rs = 0;
#pragma unroll
    for (int r = 0; r < K; ++r) {
        const uint32_t idx = (uint32_t)r * 64u + lane;   /* coalesced load */
        uint32_t t = 0;
        v[r] = SENT;
        if (idx < n) {
            v[r] = read_key(reads[idx], ref16, cap, t);
            rs += t;
        }
    }
    if (!(diag & 1u)) wave_bitonic<K>(v);
    uint32_t nv = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int r = 0; r < K; ++r) {
        nv += (uint32_t)__popcll(__ballot(v[r] != SENT));
        c1 += (uint32_t)__popcll(__ballot(v[r] < (1u << 26)));
        c2 += (uint32_t)__popcll(__ballot(v[r] < (2u << 26)));
        c3 += (uint32_t)__popcll(__ballot(v[r] < (3u << 26)));
    }
#pragma unroll
    for (int r = 0; r < K; ++r)
        if (v[r] != SENT) arena[lane * K + r] = v[r];
    const uint32_t rms = wave_sum(rs);
    if (lane == 0) {
        meta.start[0] = 0; meta.start[1] = c1; meta.start[2] = c2; meta.start[3] = c3;
        meta.cnt[0] = c1; meta.cnt[1] = c2 - c1; meta.cnt[2] = c3 - c2; meta.cnt[3] = nv - c3;
        meta.n = n;
        meta.rms_lo = rms;
        meta.rms_hi = 0;
    }
    nvalid = nv;
}

/* --------------------------------------------------------------------------
 * Phase B: ordered fold of one base group (sniper_maqcns.c:162-172).
 * keys: ascending run of the group; walked from the top.  fk from LDS.
 * ------------------------------------------------------------------------ */
__device__ __forceinline__ void fold_group(const uint32_t *keys, uint32_t cnt, const double *fk,
                                           float &es_out, float &fs_out)
{
    float es = 0.0f, fs = 0.0f;
    uint32_t w0 = 0, w1 = 0;
    uint32_t t = cnt;
    uint32_t key = t ? keys[t - 1] : 0u;
    while (t) {
        --t;
        const uint32_t cur = key;
        if (t) key = keys[t - 1];            /* prefetch the next key */
        const uint32_t minq = (cur >> 18) & 0xffu, bq = (cur >> 8) & 0xffu;
        const uint32_t st = (cur >> 16) & 1u;
        const uint32_t q = (minq < 4u && (bq & 0x3fu) != 0u) ? 4u : minq;
        const uint32_t w = st ? w1 : w0;
        const double f = fk[w];
        es = (float)((double)es + f * (double)q);
        fs = (float)((double)fs + f);
        const uint32_t wn = w < 255u ? w + 1u : 255u;
        if (st) w1 = wn; else w0 = wn;
    }
    es_out = es;
    fs_out = fs;
}

/* correctly rounded sqrt of a non-negative double (re-checked with exact fma
 * residuals so the result does not depend on the library's rounding). */
__device__ __forceinline__ double cr_sqrt(double d)
{
    double s = __builtin_sqrt(d);
    if (!(d > 0.0) || __builtin_isinf(d)) return s;
    /* neighbours of a positive finite double: +-1 in the bit pattern */
    const double up = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, s) + 1ull);
    const double dn = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, s) - 1ull);
    const double r = __builtin_fabs(__builtin_fma(-s, s, d));
    const double ru = __builtin_fabs(__builtin_fma(-up, up, d));
    const double rd = __builtin_fabs(__builtin_fma(-dn, dn, d));
    if (ru < r) s = up;
    else if (rd < r) s = dn;
    return s;
}

__device__ __forceinline__ int clamp_bar_e(float e, float f)
{
    int be = (int)((double)(e / f) + 0.5);
    be = be < 4 ? 4 : be;
    return be > 63 ? 63 : be;
}

/* --------------------------------------------------------------------------
 * Phase C: likelihoods + quantisation + consensus for one (site, sample)
 * (sniper_maqcns.c:176-248 and sniper_glf2cns :250-273), computed by the
 * 4 lanes of a quad: lane q evaluates genotypes {q, q+4, q+8} (upper-triangle
 * order AA AC AG AT CC CG CT GG GT TT), then the 10 p values are exchanged
 * with DPP quad broadcasts and every lane finishes redundantly.
 * ------------------------------------------------------------------------ */
__device__ __forceinline__ float quad_bcast(float v, int src)
{
    const int x = __builtin_bit_cast(int, v);
    int r;
    switch (src) {  /* quad_perm(src,src,src,src) */
    case 0: r = __builtin_amdgcn_mov_dpp(x, 0x00, 0xf, 0xf, false); break;
    case 1: r = __builtin_amdgcn_mov_dpp(x, 0x55, 0xf, 0xf, false); break;
    case 2: r = __builtin_amdgcn_mov_dpp(x, 0xaa, 0xf, 0xf, false); break;
    default: r = __builtin_amdgcn_mov_dpp(x, 0xff, 0xf, 0xf, false); break;
    }
    return __builtin_bit_cast(float, r);
}

/* genotype g -> alleles (j <= k) */
__device__ __forceinline__ void geno_jk(int g, int &j, int &k)
{
    j = g < 4 ? 0 : (g < 7 ? 1 : (g < 9 ? 2 : 3));
    k = g < 4 ? g : (g < 7 ? g - 3 : (g < 9 ? g - 5 : 3));
}

/* p for genotype (j,k) (sniper_maqcns.c:184-214); the sums skip {j,k} in
 * ascending base order exactly like the reference's loops. */
__device__ __forceinline__ float geno_p(int j, int k, const float es[4], const float fs[4],
                                        const uint32_t c[4], uint32_t tot, const ss_dev_model &m)
{
    float e = 0.0f, f = 0.0f;
    uint32_t c2 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool use = i != j && i != k;
        e = use ? e + es[i] : e;
        f = use ? f + fs[i] : f;
        c2 += use ? c[i] : 0u;
    }
    const bool hom = j == k;
    const double lh = hom ? 0.0 : -4.343 * m.lhet[c[j] << 8 | c[k]];
    float v;
    if (c2) {
        const double cf = m.coef[(uint32_t)clamp_bar_e(e, f) << 16 | tot << 8 | c2];
        v = hom ? (float)((double)e + cf) : (float)((lh + (double)e) + cf);
    } else {
        v = hom ? 0.0f : (float)lh;
    }
    return v < 0.0f ? 0.0f : v;
}

__device__ __forceinline__ void glf_and_cns(int q, const float es[4], const float fs[4],
                                            const uint32_t craw[4], uint32_t n, uint64_t rms,
                                            const ss_dev_model &m, uint32_t lk[10],
                                            uint32_t &min_lk, uint32_t &rms_q, uint32_t &cns)
{
    uint32_t c[4] = {craw[0], craw[1], craw[2], craw[3]};
    uint32_t tot = c[0] + c[1] + c[2] + c[3];
    if (tot > 255u) {
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = (uint32_t)(int)(254.0 * (double)c[j] / (double)(int)tot + 0.5);
        tot = c[0] + c[1] + c[2] + c[3];
    }
    /* this lane's genotypes q, q+4, q+8 */
    float mine[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        const int g = q + 4 * t;
        int j, k;
        geno_jk(g < 10 ? g : 9, j, k);
        mine[t] = (g < 10) ? geno_p(j, k, es, fs, c, tot, m) : 0.0f;
    }
    float p[10];
#pragma unroll
    for (int g = 0; g < 10; ++g) p[g] = quad_bcast(mine[g >> 2], g & 3);
    {   /* reduce the best-supported base's homozygote (:216-233) */
        float hi1 = -1.0f, hi2 = -1.0f, lo1 = 1e30f, lo2 = 1e30f;
        int hik = -1, lok = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (es[k] > hi1) { hi2 = hi1; hi1 = es[k]; hik = k; }
            else if (es[k] > hi2) hi2 = es[k];
        }
        const int diag[4] = {0, 4, 7, 9};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float d = p[diag[k]];
            if (d < lo1) { lo2 = lo1; lo1 = d; lok = k; }
            else if (d < lo2) lo2 = d;
        }
        if (hi1 > hi2 && (lok != hik || (double)lo1 + 1.0 > (double)lo2)) {
            const float nv = lo1 > 1.0f ? (float)((double)lo1 - 1.0) : 0.0f;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k == hik) p[diag[k]] = nv;
        }
    }
    float min_p = 1e30f;
#pragma unroll
    for (int g = 0; g < 10; ++g)
        if (p[g] < min_p) min_p = p[g];
    min_lk = (double)min_p > 255.0 ? 255u : (uint32_t)(int)((double)min_p + 0.5);
#pragma unroll
    for (int g = 0; g < 10; ++g) {
        const float d = p[g] - min_p;
        lk[g] = (double)d > 255.0 ? 255u : (uint32_t)(int)((double)d + 0.5);
    }
    rms_q = n ? (uint32_t)(uint8_t)(cr_sqrt((double)rms / (double)(int)n) + .499) : 0u;
    /* sniper_glf2cns: best / second / third over genotypes in index order */
    const int gi[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
    const int gj[10] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};
    int b1 = 10000, b2 = 10000, b3 = 10000, g1 = -1, g2 = -1;
#pragma unroll
    for (int g = 0; g < 10; ++g) {
        const int s = (int)lk[g] + (gi[g] == gj[g] ? 0 : m.q_r_int);
        if (s < b1) { b3 = b2; b2 = b1; b1 = s; g2 = g1; g1 = g; }
        else if (s < b2) { b3 = b2; b2 = s; g2 = g; }
        else if (s < b3) b3 = s;
    }
    uint32_t x = 0;
#pragma unroll
    for (int g = 0; g < 10; ++g) {
        if (g == g1) x |= (1u << gi[g] | 1u << gj[g]) << 28;
        if (g == g2) x |= (1u << gi[g] | 1u << gj[g]) << 24;
    }
    if (g1 < 0) x |= 0xfu << 28;
    if (g2 < 0) x |= 0xfu << 24;
    x |= (rms_q & 0xffu) << 16;
    x |= b2 < 10000 ? (uint32_t)(b2 - b1 < 256 ? b2 - b1 : 255) << 8 : 0xffu << 8;
    x |= (b2 < 10000 && b3 < 10000) ? (uint32_t)(b3 - b2 < 256 ? b3 - b2 : 255) : 0xffu;
    cns = x;
}

/* qAdd (somatic_sniper.c:18) with the out-of-range index clamped + counted */
__device__ __forceinline__ int qadd(const int32_t *T, int x, int y, int &clamped)
{
    int idx = 512 + y - x;
    if (idx < 0) { idx = 0; ++clamped; }
    else if (idx > 1023) { idx = 1023; ++clamped; }
    return x + T[idx];
}

__device__ __forceinline__ bool proper_subset(int a, int b) { return b != a && (a & b) == a; }

/* --------------------------------------------------------------------------
 * Phase D: the site decision of glf_somatic (somatic_sniper.c:117-273).
 * ------------------------------------------------------------------------ */
__device__ void decide_site(const ss_score_args &a, uint32_t site, uint32_t refc,
                            const SlotRes &rt, const SlotRes &rn)
{
    const ss_dev_model &m = a.m;
    const int rb = (int)refc;
    const int rb4 = m.nt16[refc & 0xffu];
    if (!(rb != 'N' && rt.depth > 0u && rn.depth > 0u)) { a.score[site] = -1; return; }
    const uint32_t ct = rt.cns, cn = rn.cns;
    const int t1 = (int)(ct >> 28), t2 = (int)(ct >> 24 & 0xf), ts1 = (int)(ct >> 8 & 0xff), ts2 = (int)(ct & 0xff);
    const int n1 = (int)(cn >> 28), n2 = (int)(cn >> 24 & 0xf), ns1 = (int)(cn >> 8 & 0xff), ns2 = (int)(cn & 0xff);
    if (!(rb4 != 15 && t1 != 15 && n1 != 15 && t1 != n1)) { a.score[site] = 255; return; }

    /* ---- SNV candidate (rare): somatic_sniper.c:157-262 ---- */
    int clamped = 0;
    int tq = t2 == rb4 ? ts1 : ts1 + ts2;
    if (tq > 255) tq = 255;
    int nq = 0;
    if (n1 != 15 && n1 != rb4) {
        nq = n2 == rb4 ? ns1 : ns1 + ns2;
        if (nq > 255) nq = 255;
    }
    int qps = 255, jt = 0, jn = 0, jcq = 255;
    if (m.use_joint) {
        /* joint prior over (normal i, tumor j) with RAW glf lk (:180) */
        int marg = 255, best = 1000, bi = -1, bj = -1;
#pragma unroll 1
        for (int i = 0; i < 10; ++i)
#pragma unroll 1
            for (int j = 0; j < 10; ++j) {
                int v = (int)rn.lk[i] + (int)rt.lk[j] + m.jprior[(rb4 * 10 + i) * 10 + j];
                if (v > 255) v = 255;
                if (v < best) { best = v; bi = i; bj = j; }
                marg = qadd(m.qadd, marg, v, clamped);
            }
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            int v = (int)rn.lk[j] + (int)rt.lk[j] + m.jprior[(rb4 * 10 + j) * 10 + j];
            if (v > 255) v = 255;
            const int l = v - marg;
            qps = qadd(m.qadd, qps, l, clamped);
            if (j != bj) jcq = qadd(m.qadd, jcq, l, clamped);  /* stale-index quirk, :196 */
        }
        if (jcq > 255) jcq = 255;
        const int gb[10] = {1, 3, 5, 9, 2, 6, 10, 4, 12, 8};
        jn = gb[bi];
        jt = gb[bj];
    } else {
        /* calculatePosteriors (:79-99) for both samples, then the sum (:209-214);
         * x_j is recomputed in the second pass instead of kept in an array */
        int st = 255, sn = 255;
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            const int xt = (int)rt.lk[j] + m.prior[rb4 * 10 + j];
            const int xn = (int)rn.lk[j] + m.prior[rb4 * 10 + j];
            st = qadd(m.qadd, xt, st, clamped);
            sn = qadd(m.qadd, xn, sn, clamped);
        }
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            int vt = (int)rt.lk[j] + m.prior[rb4 * 10 + j] - st;
            int vn = (int)rn.lk[j] + m.prior[rb4 * 10 + j] - sn;
            if (vt > 255) vt = 255;
            if (vn > 255) vn = 255;
            qps = qadd(m.qadd, qps, vt + vn, clamped);
        }
    }
    a.score[site] = qps;
    if (clamped && a.n_clamped) atomicAdd(a.n_clamped, (uint32_t)clamped);
    const int tg = jt ? jt : t1, ng = jn ? jn : n1;
    const bool emit = m.min_somatic_qual <= qps &&
                      (m.include_loh || !proper_subset(tg, ng)) &&
                      (m.include_gor || !(!proper_subset(rb4, ng) && (tg & ~ng) == rb4));
    if (!emit || !a.calls) return;
    const uint32_t slot = atomicAdd(a.n_calls, 1u);
    if (slot >= a.calls_cap) return;
    ss_call_t c;
    c.site = site;
    c.somatic_score = qps;
    c.cns_tumor = ct;
    c.cns_normal = cn;
    c.joint_cq = (int16_t)jcq;
    c.snp_q_tumor = (uint8_t)tq;
    c.snp_q_normal = (uint8_t)nq;
    c.joint_gt_tumor = (uint8_t)jt;
    c.joint_gt_normal = (uint8_t)jn;
    c.status_tumor = (uint8_t)(tg == ng ? SS_GERMLINE
                              : proper_subset(tg, ng) ? SS_LOH : (qps > 0 ? SS_SOMATIC : SS_UNKNOWN));
    c.status_normal = (uint8_t)(n1 == rb4 ? SS_WILDTYPE : SS_GERMLINE);
    c.ref_base4 = (uint8_t)rb4;
    c.flags = clamped ? SS_CALL_QADD_CLAMPED : 0;
    c.pad = 0;
    a.calls[slot] = c;
}

__device__ __forceinline__ void store_glf(ss_glf_t *dst, uint32_t ref16, const uint32_t lk[10],
                                          uint32_t min_lk, uint32_t rms_q, uint32_t depth)
{
    uint32_t w[5];
    w[0] = (ref16 & 0xffu) | (rms_q & 0xffu) << 8 | (lk[0] & 0xffu) << 16 | (lk[1] & 0xffu) << 24;
    w[1] = lk[2] | lk[3] << 8 | lk[4] << 16 | lk[5] << 24;
    w[2] = lk[6] | lk[7] << 8 | lk[8] << 16 | lk[9] << 24;
    w[3] = min_lk & 0xffu;
    w[4] = depth;
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
#pragma unroll
    for (int i = 0; i < 5; ++i) d[i] = w[i];
}

/* --------------------------------------------------------------------------
 * Phases B + C + D for G sites whose slots are in LDS.  Called by every lane
 * of one wave.  keys_of(slot) gives the arena of that slot.
 * ------------------------------------------------------------------------ */
template <typename KeysOf>
__device__ __forceinline__ void finish_group(const ss_score_args &a, int G, const SlotMeta *meta,
                                             SlotRes *res, const SiteInfo *sinfo,
                                             const double *fk, KeysOf keys_of)
{
    const uint32_t lane = lane_id();
    const int s = (int)(lane >> 3), slot = (int)(lane >> 2), b = (int)(lane & 3u);
    float es = 0.0f, fs = 0.0f;
    if (s < G) {
        const SlotMeta &mt = meta[slot];
        if (!(a.diag & 2u)) fold_group(keys_of(slot) + mt.start[b], mt.cnt[b], fk, es, fs);
        else { es = (float)mt.cnt[b]; fs = es; }
    }
    /* gather the quad's four bases (all lanes active for the DPP moves) */
    float E[4], F[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        E[i] = quad_bcast(es, i);
        F[i] = quad_bcast(fs, i);
    }
    if (s < G) {
        const SlotMeta &mt = meta[slot];
        const uint32_t cnt[4] = {mt.cnt[0], mt.cnt[1], mt.cnt[2], mt.cnt[3]};
        const uint64_t rms = (uint64_t)mt.rms_lo | (uint64_t)mt.rms_hi << 32;
        uint32_t lk[10], min_lk, rms_q, cns;
        if (!(a.diag & 4u)) glf_and_cns(b, E, F, cnt, mt.n, rms, a.m, lk, min_lk, rms_q, cns);
        else {
#pragma unroll
            for (int g = 0; g < 10; ++g) lk[g] = (uint32_t)E[g & 3] & 0xffu;
            min_lk = 0; rms_q = 0; cns = (uint32_t)F[0];
        }
        if (b == 0) {
            SlotRes &r = res[slot];
#pragma unroll
            for (int g = 0; g < 10; ++g) r.lk[g] = (uint8_t)lk[g];
            r.cns = cns;
            r.depth = mt.n > 16777215u ? 16777215u : mt.n;
            r.min_lk = (uint8_t)min_lk;
            r.rms_q = (uint8_t)rms_q;
            if (a.glf) {
                const uint32_t site = sinfo[s].site;
                const uint32_t ref16 = a.m.nt16[sinfo[s].refc & 0xffu];
                store_glf(&a.glf[2ull * site + (slot & 1)], ref16, lk, min_lk, rms_q, r.depth);
            }
        }
    }
    wave_sync();
    if ((int)lane < G) {
        if (!(a.diag & 8u)) decide_site(a, sinfo[lane].site, sinfo[lane].refc, res[2 * lane], res[2 * lane + 1]);
        else a.score[sinfo[lane].site] = (int32_t)res[2 * lane].cns;
    }
    wave_sync();
}

/* --------------------------------------------------------------------------
 * Main kernel.
 *
 * Each wave walks 8-site BLOCKS (block b = sites [8b, 8b+8), grid-strided over
 * waves).  A block's reads are contiguous in both CSR arrays, so a sub-group of
 * its sites is staged into LDS with LDS-DMA (global_load_lds, no VGPRs) as two
 * contiguous runs: [tumor reads | normal reads].  Two staging buffers per wave
 * form a software pipeline: the DMA of the NEXT sub-group is issued right after
 * phase A of the current one and lands while the current one folds (phase B
 * has no VMEM, so nothing forces an early drain).  The staged reads are sorted
 * in place, so the staging buffer is also the sorted-key arena of phase B.
 * The block descriptor (offsets + ref chars of the 8 sites) lives in one VGPR
 * and is prefetched one block ahead.
 * ------------------------------------------------------------------------ */
#define STG 1024            /* staged u32 per buffer (per wave) */

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void glb_void_t;

struct MainLds {
    uint32_t stage[4][2][STG];
    SlotMeta meta[4][2 * GMAX];
    SlotRes  res[4][2 * GMAX];
    SiteInfo sinfo[4][GMAX];
};

__device__ __forceinline__ void phase_a_sample(const uint32_t *reads, uint32_t n, uint32_t ref16,
                                               uint32_t cap, uint32_t *arena, SlotMeta &meta,
                                               uint32_t &nv, uint32_t diag)
{
    if (n <= 64u) sort_sample<1>(reads, n, ref16, cap, arena, meta, nv, diag);
    else if (n <= 128u) sort_sample<2>(reads, n, ref16, cap, arena, meta, nv, diag);
    else sort_sample<4>(reads, n, ref16, cap, arena, meta, nv, diag);
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

/* lanes 0..8: off_t[s..s+8], lanes 16..24: off_n[s..s+8], lanes 32..39: ref[s..s+7] */
__device__ __forceinline__ uint32_t load_desc(const ss_score_args &a, uint64_t s)
{
    const uint32_t lane = lane_id();
    uint32_t v = 0;
    if (lane < 9u) {
        if (s + lane <= a.n_sites) v = a.off_t[s + lane];
    } else if (lane >= 16u && lane < 25u) {
        if (s + (lane - 16u) <= a.n_sites) v = a.off_n[s + (lane - 16u)];
    } else if (lane >= 32u && lane < 40u) {
        if (s + (lane - 32u) < a.n_sites) v = a.ref[s + (lane - 32u)];
    }
    return v;
}

__device__ __forceinline__ void push_deep(const ss_score_args &a, uint32_t site)
{
    if (lane_id() == 0) {
        const uint32_t d = atomicAdd(a.deep_count, 1u);
        if (d < a.deep_cap) a.deep_list[d] = site;
        else atomicOr(a.err, SS_KERR_DEEP_OVERFLOW);
    }
}

struct Sub {
    uint32_t a, b;        /* site range [a, b) within the block */
    uint32_t t0, lt;      /* tumor read run  */
    uint32_t n0, ln;      /* normal read run */
};

/* Largest run of sites from `pos` whose reads fit one staging buffer.  A site
 * that alone exceeds it is deep by construction and goes to the deep list. */
__device__ __forceinline__ Sub form_sub(const ss_score_args &a, uint32_t desc, uint32_t nsite,
                                        uint32_t pos, uint64_t sblk)
{
    uint32_t i = pos, tot = 0;
    while (i < nsite) {
        const uint32_t sz = (rl(desc, i + 1u) - rl(desc, i)) + (rl(desc, i + 17u) - rl(desc, i + 16u));
        if (sz > STG) {
            if (i == pos) { push_deep(a, (uint32_t)(sblk + i)); pos = ++i; continue; }
            break;
        }
        if (tot + sz > STG) break;
        tot += sz;
        ++i;
    }
    Sub r;
    r.a = pos;
    r.b = i;
    r.t0 = rl(desc, pos);
    r.lt = rl(desc, i) - r.t0;
    r.n0 = rl(desc, pos + 16u);
    r.ln = rl(desc, i + 16u) - r.n0;
    return r;
}

__device__ __forceinline__ void issue_dma(const ss_score_args &a, const Sub &r, uint32_t *buf)
{
    const uint32_t lane = lane_id();
    for (uint32_t i = 0; i < r.lt; i += 64u)
        if (i + lane < r.lt)
            __builtin_amdgcn_global_load_lds((glb_void_t *)(a.reads_t + r.t0 + i + lane),
                                             (lds_void_t *)(buf + i), 4, 0, 0);
    for (uint32_t i = 0; i < r.ln; i += 64u)
        if (i + lane < r.ln)
            __builtin_amdgcn_global_load_lds((glb_void_t *)(a.reads_n + r.n0 + i + lane),
                                             (lds_void_t *)(buf + r.lt + i), 4, 0, 0);
}

}  // namespace

__global__ __launch_bounds__(SS_MAIN_BLOCK) void ss_score_main(ss_score_args a)
{
    __shared__ double fk[256];
    __shared__ MainLds L;
    const uint32_t lane = lane_id();
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) fk[i] = a.m.fk[i];
    __syncthreads();

    SlotMeta *meta = L.meta[wv];
    SlotRes *res = L.res[wv];
    SiteInfo *sinfo = L.sinfo[wv];
    const uint64_t nwaves = (uint64_t)gridDim.x * (SS_MAIN_BLOCK / 64);
    const uint64_t nblocks = (a.n_sites + GMAX - 1) / GMAX;
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;

    /* ---- prologue: first non-empty sub-group, its DMA, next descriptor ---- */
    uint64_t blk = (uint64_t)blockIdx.x * (SS_MAIN_BLOCK / 64) + wv;
    if (blk >= nblocks) return;
    uint32_t desc = load_desc(a, blk * GMAX);
    uint32_t nsite = (uint32_t)(a.n_sites - blk * GMAX < GMAX ? a.n_sites - blk * GMAX : GMAX);
    Sub cur = form_sub(a, desc, nsite, 0, blk * GMAX);
    uint64_t nblk = blk + nwaves;
    uint32_t ndesc = nblk < nblocks ? load_desc(a, nblk * GMAX) : 0u;
    while (cur.a == cur.b) {               /* whole block deep */
        blk = nblk;
        if (blk >= nblocks) return;
        desc = ndesc;
        nsite = (uint32_t)(a.n_sites - blk * GMAX < GMAX ? a.n_sites - blk * GMAX : GMAX);
        nblk = blk + nwaves;
        ndesc = nblk < nblocks ? load_desc(a, nblk * GMAX) : 0u;
        cur = form_sub(a, desc, nsite, 0, blk * GMAX);
    }
    uint32_t c = 0;
    issue_dma(a, cur, L.stage[wv][0]);

    for (;;) {
        uint32_t *stage = L.stage[wv][c];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   /* this sub-group's DMA has landed */
        /* ---- phase A: sort the sub-group's samples in place ---- */
        int G = 0;
        for (uint32_t i = cur.a; i < cur.b; ++i) {
            const uint32_t site = (uint32_t)(blk * GMAX + i);
            const uint32_t t_i = rl(desc, i), nt = rl(desc, i + 1u) - t_i;
            const uint32_t n_i = rl(desc, i + 16u), nn = rl(desc, i + 17u) - n_i;
            if (nt > SS_MAIN_MAXN || nn > SS_MAIN_MAXN) { push_deep(a, site); continue; }
            const uint32_t refc = rl(desc, i + 32u) & 0xffu;
            const uint32_t ref16 = a.m.nt16[refc];
            const uint32_t bt = t_i - cur.t0, bn = cur.lt + (n_i - cur.n0);
            uint32_t nv;
            if (lane == 0) {
                sinfo[G].site = site;
                sinfo[G].refc = refc;
                meta[2 * G].base = bt;
                meta[2 * G + 1].base = bn;
            }
            phase_a_sample(stage + bt, nt, ref16, cap, stage + bt, meta[2 * G], nv, a.diag);
            phase_a_sample(stage + bn, nn, ref16, cap, stage + bn, meta[2 * G + 1], nv, a.diag);
            ++G;
        }
        /* ---- next sub-group: same block, else the next non-empty block ---- */
        Sub nxt;
        bool have = false;
        if (cur.b < nsite) {
            nxt = form_sub(a, desc, nsite, cur.b, blk * GMAX);
            have = nxt.a < nxt.b;
        }
        while (!have) {
            blk = nblk;
            if (blk >= nblocks) break;
            desc = ndesc;
            nsite = (uint32_t)(a.n_sites - blk * GMAX < GMAX ? a.n_sites - blk * GMAX : GMAX);
            nblk = blk + nwaves;
            ndesc = nblk < nblocks ? load_desc(a, nblk * GMAX) : 0u;
            nxt = form_sub(a, desc, nsite, 0, blk * GMAX);
            have = nxt.a < nxt.b;
        }
        if (have) issue_dma(a, nxt, L.stage[wv][c ^ 1u]);
        /* ---- phases B, C, D (the DMA above lands meanwhile) ---- */
        wave_sync();
        if (G > 0)
            finish_group(a, G, meta, res, sinfo, fk,
                         [&](int slot) -> const uint32_t * { return stage + meta[slot].base; });
        if (!have) break;
        cur = nxt;
        c ^= 1u;
    }
}

/* --------------------------------------------------------------------------
 * Deep kernel: one block per site whose deeper sample exceeds SS_MAIN_MAXN.
 * GIANT = false: LDS sort (<= SS_DEEP_MAXN per sample), deeper sites are
 * forwarded to the giant list.  GIANT = true: a global scratch slice per block.
 * ------------------------------------------------------------------------ */
namespace {

__device__ void block_bitonic(uint32_t *buf, uint32_t P)
{
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < (P >> 1); t += blockDim.x) {
                const uint32_t i = ((t & ~(j - 1u)) << 1) | (t & (j - 1u));
                const uint32_t p = i | j;
                const bool up = (i & k) == 0u;
                const uint32_t x = buf[i], y = buf[p];
                if ((x > y) == up) { buf[i] = y; buf[p] = x; }
            }
            __syncthreads();
        }
}

struct DeepLds {
    SlotMeta meta[2];
    SlotRes res[2];
    SiteInfo sinfo[1];
    uint32_t cnt[2][4];
    unsigned long long rms[2];
};

/* block-wide sort of one sample into buf; fills meta (thread 0) */
__device__ void deep_sample(const uint32_t *reads, uint32_t n, uint32_t ref16, uint32_t cap,
                            uint32_t *buf, DeepLds &D, int m)
{
    uint32_t P = 64;
    while (P < n) P <<= 1;
    if (threadIdx.x < 4) D.cnt[m][threadIdx.x] = 0;
    if (threadIdx.x == 0) D.rms[m] = 0ull;
    __syncthreads();
    unsigned long long rs = 0;
    for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
        uint32_t t = 0, v = SENT;
        if (i < n) { v = read_key(reads[i], ref16, cap, t); rs += t; }
        buf[i] = v;
    }
    atomicAdd(&D.rms[m], rs);
    __syncthreads();
    block_bitonic(buf, P);
    uint32_t c[4] = {0, 0, 0, 0};
    for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
        const uint32_t v = buf[i];
        if (v != SENT) ++c[v >> 26];
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) if (c[b]) atomicAdd(&D.cnt[m][b], c[b]);
    __syncthreads();
    if (threadIdx.x == 0) {
        SlotMeta &mt = D.meta[m];
        uint32_t acc = 0;
        for (int b = 0; b < 4; ++b) { mt.start[b] = acc; mt.cnt[b] = D.cnt[m][b]; acc += D.cnt[m][b]; }
        mt.base = 0;
        mt.n = n;
        mt.rms_lo = (uint32_t)D.rms[m];
        mt.rms_hi = (uint32_t)(D.rms[m] >> 32);
    }
}

}  // namespace

template <bool GIANT>
__global__ __launch_bounds__(SS_DEEP_BLOCK) void ss_score_deep(ss_score_args a)
{
    __shared__ double fk[256];
    __shared__ DeepLds D;
    __shared__ uint32_t lbuf[GIANT ? 1 : 2][GIANT ? 1 : SS_DEEP_MAXN];
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) fk[i] = a.m.fk[i];
    __syncthreads();
    const uint32_t count = GIANT ? *a.giant_count : *a.deep_count;
    const uint32_t lim = GIANT ? (count < a.giant_cap ? count : a.giant_cap)
                               : (count < a.deep_cap ? count : a.deep_cap);
    const uint32_t *list = GIANT ? a.giant_list : a.deep_list;
    uint32_t *bt, *bn;
    if (GIANT) {
        bt = a.giant_scratch + (size_t)blockIdx.x * 2u * a.giant_keys;
        bn = bt + a.giant_keys;
    } else {
        bt = lbuf[0];
        bn = lbuf[GIANT ? 0 : 1];
    }
    const uint32_t maxn = GIANT ? a.giant_keys : (uint32_t)SS_DEEP_MAXN;
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;
    for (uint32_t w = blockIdx.x; w < lim; w += gridDim.x) {
        const uint32_t s = list[w];
        const uint32_t ot = a.off_t[s], nt = a.off_t[s + 1] - ot;
        const uint32_t on = a.off_n[s], nn = a.off_n[s + 1] - on;
        if (nt > maxn || nn > maxn) {
            if (threadIdx.x == 0) {
                if (!GIANT) {
                    const uint32_t d = atomicAdd(a.giant_count, 1u);
                    if (d < a.giant_cap) a.giant_list[d] = s;
                    else atomicOr(a.err, SS_KERR_GIANT_OVERFLOW);
                } else {
                    atomicOr(a.err, SS_KERR_TOO_DEEP);
                    a.score[s] = -2;
                }
            }
            continue;
        }
        const uint32_t refc = a.ref[s];
        const uint32_t ref16 = a.m.nt16[refc];
        if (threadIdx.x == 0) { D.sinfo[0].site = s; D.sinfo[0].refc = refc; }
        deep_sample(a.reads_t + ot, nt, ref16, cap, bt, D, 0);
        deep_sample(a.reads_n + on, nn, ref16, cap, bn, D, 1);
        __syncthreads();
        if (threadIdx.x < 64)
            finish_group(a, 1, D.meta, D.res, D.sinfo, fk,
                         [&](int slot) -> const uint32_t * { return slot ? bn : bt; });
        __syncthreads();
    }
}

/* --------------------------------------------------------------------------
 * Synthetic generator (device twin of ss_synth.c; same ss_synth_core.h code).
 * ------------------------------------------------------------------------ */
__global__ void ss_synth_depth_kernel(ss_synth_k_t k, uint64_t first, uint64_t n, uint8_t *ref,
                                      uint32_t *dt, uint32_t *dn)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        ss_site_draw_t d;
        uint32_t j, r, c;
        ss_synth_site(&k, first + i, &d);
        ref[i] = d.ref_char;
        for (j = c = 0; j < d.raw_tumor; ++j) c += (uint32_t)ss_synth_read(&k, first + i, &d, 0, j, &r);
        dt[i] = c;
        for (j = c = 0; j < d.raw_normal; ++j) c += (uint32_t)ss_synth_read(&k, first + i, &d, 1, j, &r);
        dn[i] = c;
    }
}

__global__ void ss_synth_reads_kernel(ss_synth_k_t k, uint64_t first, uint64_t n,
                                      const uint32_t *off_t, const uint32_t *off_n, uint32_t *rt,
                                      uint32_t *rn)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        ss_site_draw_t d;
        uint32_t j, r;
        uint32_t *pt = rt + off_t[i], *pn = rn + off_n[i];
        ss_synth_site(&k, first + i, &d);
        for (j = 0; j < d.raw_tumor; ++j)
            if (ss_synth_read(&k, first + i, &d, 0, j, &r)) *pt++ = r;
        for (j = 0; j < d.raw_normal; ++j)
            if (ss_synth_read(&k, first + i, &d, 1, j, &r)) *pn++ = r;
    }
}

/* --------------------------------------------------------------------------
 * launchers
 * ------------------------------------------------------------------------ */
int ss_launch_score(const ss_score_args &a, int main_grid, int deep_grid, hipStream_t s,
                    hipEvent_t ev0, hipEvent_t ev1)
{
    hipError_t e;
    if (ev0) (void)hipEventRecord(ev0, s);
    hipLaunchKernelGGL(ss_score_main, dim3(main_grid), dim3(SS_MAIN_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    if (ev1) (void)hipEventRecord(ev1, s);
    hipLaunchKernelGGL(ss_score_deep<false>, dim3(deep_grid), dim3(SS_DEEP_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(ss_score_deep<true>, dim3(SS_GIANT_BLOCKS), dim3(SS_DEEP_BLOCK), 0, s, a);
    return (int)hipGetLastError();
}

int ss_launch_synth_depth(const ss_synth_k_t &k, uint64_t first, uint64_t n, uint8_t *ref,
                          uint32_t *dt, uint32_t *dn, hipStream_t s)
{
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(ss_synth_depth_kernel, dim3((unsigned)blocks), dim3(256), 0, s, k, first, n,
                       ref, dt, dn);
    return (int)hipGetLastError();
}

int ss_launch_synth_reads(const ss_synth_k_t &k, uint64_t first, uint64_t n,
                          const uint32_t *off_t, const uint32_t *off_n, uint32_t *rt,
                          uint32_t *rn, hipStream_t s)
{
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(ss_synth_reads_kernel, dim3((unsigned)blocks), dim3(256), 0, s, k, first, n,
                       off_t, off_n, rt, rn);
    return (int)hipGetLastError();
}
