/*
 * ss_kernels.hip -- CDNA4 (gfx950) kernels of the somatic site scorer.
 *
 * One pileup site = one call of the reference's glf_somatic
 * (src/lib/sniper/somatic_sniper.c:109-273): two MAQ genotype-likelihood
 * evaluations (sniper_maqcns_glfgen, sniper_maqcns.c:127-248), two consensus
 * calls (sniper_glf2cns, :250-273) and the Phred-space somatic posterior.
 *
 * Work decomposition (DESIGN.md "Kernels"):
 *   ss_score_main   persistent waves walk 16-site blocks.  A block's reads are
 *     staged into LDS by LDS-DMA; per site ONE wave-wide bitonic sort of 16-bit
 *     keys (two per VGPR, both samples) orders the reads, which become 16-bit
 *     fold records written back over the staged reads.  Then two lanes per
 *     (site, sample) run the ordered esum / fsum fold (the reference's float
 *     accumulators fed double increments, sniper_maqcns.c:162-172), split the
 *     10 genotype likelihoods between them, and lane s decides site s (gate,
 *     SNV candidate test, posteriors / joint prior, emit filter).  The DMA of
 *     the next sub-group overlaps the likelihood and decision phases.
 *   ss_score_wide   sites with 513..2048 sort slots (the main kernel lists
 *     them): the same packed network at 1024 / 2048 keys, 16 sites folded and
 *     finished together.
 *   ss_score_deep   one wave per site beyond that (any depth) or with
 *     malformed offsets: counting sort of the order-relevant key fields in
 *     LDS windows, then the same ordered fold, likelihood and decision code.
 *
 * Bit-exactness: built with -ffp-contract=off (no FMA contraction); float
 * division and double sqrt are correctly rounded (sqrt re-checked with fma);
 * accumulation order equals the reference's descending-key order.
 */
#include "ss_kernels.h"

#define SENT 0xffffffffu

/* Fixed tuning of the shipped kernels (each measured on MI355X):
 * one code path per choice, no run-time or build-time alternatives. */
#define SS_FOLD_UNROLL 8  /* fold loop unroll (2 -> 8: +0.5% main, +4% at 500x/500x) */
#define SS_PRIO_SORT 3    /* wave priority raised over the sort network (+1.8%) */
#define SS_PRIO_WIDE 1    /* the same over the wide kernel's network (+3.7% at 500x/500x) */
/* `#pragma unroll N` with N from a macro: the count reaches the pragma expanded */
#define SS_PRAGMA(x) _Pragma(#x)
#define SS_UNROLL(n) SS_PRAGMA(unroll n)
#ifndef SS_STAMP
#define SS_STAMP 0        /* profiling builds only (make variant): per-phase s_memtime cycle totals */
#endif

/* Phase stamps (SS_STAMP builds only): wave-uniform cycle accumulators,
 * summed over waves into ss_stamp_acc at exit; read by ss_debug_stamps(). */
#define SS_NSTAMP 16
#if SS_STAMP
__device__ unsigned long long ss_stamp_acc[SS_NSTAMP];
struct Stamps {
    uint64_t prev, acc[SS_NSTAMP];
    __device__ void start() { prev = __builtin_amdgcn_s_memtime(); for (int i = 0; i < SS_NSTAMP; ++i) acc[i] = 0; }
    __device__ void mark(int i) { const uint64_t t = __builtin_amdgcn_s_memtime(); acc[i] += t - prev; prev = t; }
    __device__ void flush() {
        if (__lane_id() == 0)
            for (int i = 0; i < SS_NSTAMP; ++i) atomicAdd(&ss_stamp_acc[i], (unsigned long long)acc[i]);
    }
};
#else
struct Stamps {
    __device__ void start() {}
    __device__ void mark(int) {}
    __device__ void flush() {}
};
#endif

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

/* sums over lanes 0..31 and 32..63 (returned in lanes 31 and 63) */
__device__ __forceinline__ uint32_t wave_halfsums(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false); /* row_shr:1 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false); /* row_shr:2 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false); /* row_shr:4 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false); /* row_shr:8 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); /* row_bcast:15 */
    return v;
}

struct SlotRes {
    uint8_t  lk[12];
    uint32_t cns;
    uint32_t depth;
    uint8_t  min_lk, rms_q, pad0, pad1;
};

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
    const double lh = hom ? 0.0 : -4.343 * ss_tab_lhet(m)[c[j] << 8 | c[k]];
    float v;
    if (c2) {
        /* the reference's layout, kept on the device: rescaled counts can sum
         * to 256, and tot = 256 then reads row q + 1, n = 0 exactly as the
         * reference does (a transposed, q-minor copy measured no faster and
         * broke that aliasing) */
        const double cf = ss_tab_coef(m)[(uint32_t)clamp_bar_e(e, f) << 16 | tot << 8 | c2];
        v = hom ? (float)((double)e + cf) : (float)((lh + (double)e) + cf);
    } else {
        v = hom ? 0.0f : (float)lh;
    }
    return v < 0.0f ? 0.0f : v;
}

/* geno_p for the five genotypes role * 5 + t of one lane, with every table
 * gather issued before any is consumed: indices are computed unconditionally
 * (an unused one points at entry 0), so the ten loads go out back to back and
 * the lane waits for memory once instead of once per genotype and table.  The
 * arithmetic on the loaded values is geno_p's, operation for operation. */
template <int T0, int T1>
__device__ __forceinline__ void geno_p_range(uint32_t role, const float es[4], const float fs[4],
                                             const uint32_t c[4], uint32_t tot, const ss_dev_model &m,
                                             float out[5])
{
    float ev[5];
    uint32_t c2v[5];
    bool homv[5];
    double lhv[5], cfv[5];
#pragma unroll
    for (int t = T0; t < T1; ++t) {
        int j, k;
        geno_jk((int)role * 5 + t, j, k);
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
        const uint32_t il = hom ? 0u : (c[j] << 8 | c[k]);
        const uint32_t ic = c2 ? ((uint32_t)clamp_bar_e(e, f) << 16 | tot << 8 | c2) : 0u;
        lhv[t] = ss_tab_lhet(m)[il];
        cfv[t] = ss_tab_coef(m)[ic];
        ev[t] = e;
        c2v[t] = c2;
        homv[t] = hom;
    }
#pragma unroll
    for (int t = T0; t < T1; ++t) {
        const double lh = homv[t] ? 0.0 : -4.343 * lhv[t];
        float v;
        if (c2v[t]) v = homv[t] ? (float)((double)ev[t] + cfv[t]) : (float)((lh + (double)ev[t]) + cfv[t]);
        else v = homv[t] ? 0.0f : (float)lh;
        out[t] = v < 0.0f ? 0.0f : v;
    }
}

/* the five genotypes in batches of three and two (all five at once spills;
 * one at a time waits once per genotype: -2.4%) */
__device__ __forceinline__ void geno_p5(uint32_t role, const float es[4], const float fs[4],
                                        const uint32_t c[4], uint32_t tot, const ss_dev_model &m,
                                        float out[5])
{
    geno_p_range<0, 3>(role, es, fs, c, tot, m, out);
    geno_p_range<3, 5>(role, es, fs, c, tot, m, out);
}

/* counts rescale of sniper_maqcns.c:178-182 */
__device__ __forceinline__ uint32_t rescale_counts(const uint32_t craw[4], uint32_t c[4])
{
    uint32_t tot = craw[0] + craw[1] + craw[2] + craw[3];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = craw[j];
    if (tot > 255u) {
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = (uint32_t)(int)(254.0 * (double)c[j] / (double)(int)tot + 0.5);
        tot = c[0] + c[1] + c[2] + c[3];
    }
    return tot;
}

/* hom fix, quantisation and glf2cns from the 10 genotype p values
 * (sniper_maqcns.c:216-244, sniper_glf2cns :250-273). */
__device__ __forceinline__ void glf_finish(float p[10], const float es[4], uint32_t n, uint64_t rms,
                                           const ss_dev_model &m, uint32_t lk[10],
                                           uint32_t &min_lk, uint32_t &rms_q, uint32_t &cns)
{
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

/* quad-cooperative version (deep kernel): lane q of the quad evaluates
 * genotypes {q, q+4, q+8}, DPP quad broadcasts exchange them. */
__device__ __forceinline__ void glf_and_cns(int q, const float es[4], const float fs[4],
                                            const uint32_t craw[4], uint32_t n, uint64_t rms,
                                            const ss_dev_model &m, uint32_t lk[10],
                                            uint32_t &min_lk, uint32_t &rms_q, uint32_t &cns)
{
    uint32_t c[4];
    const uint32_t tot = rescale_counts(craw, c);
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
    glf_finish(p, es, n, rms, m, lk, min_lk, rms_q, cns);
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
    const int rb = (int)(refc & 0xffu);      /* refc: ref char | nt16 code << 8 */
    const int rb4 = (int)(refc >> 8);
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
    if ((m.flags & SS_MF_JOINT)) {
        /* joint prior over (normal i, tumor j) with RAW glf lk (:180) */
        int marg = 255, best = 1000, bi = -1, bj = -1;
#pragma unroll 1
        for (int i = 0; i < 10; ++i)
#pragma unroll 1
            for (int j = 0; j < 10; ++j) {
                int v = (int)rn.lk[i] + (int)rt.lk[j] + ss_tab_jprior(m)[(rb4 * 10 + i) * 10 + j];
                if (v > 255) v = 255;
                if (v < best) { best = v; bi = i; bj = j; }
                marg = qadd(ss_tab_qadd(m), marg, v, clamped);
            }
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            int v = (int)rn.lk[j] + (int)rt.lk[j] + ss_tab_jprior(m)[(rb4 * 10 + j) * 10 + j];
            if (v > 255) v = 255;
            const int l = v - marg;
            qps = qadd(ss_tab_qadd(m), qps, l, clamped);
            if (j != bj) jcq = qadd(ss_tab_qadd(m), jcq, l, clamped);  /* stale-index quirk, :196 */
        }
        if (jcq > 255) jcq = 255;
        /* glfBase (somatic_sniper.c:26): genotype index -> nt16 bit set */
        int gj, gk;
        geno_jk(bi, gj, gk);
        jn = 1 << gj | 1 << gk;
        geno_jk(bj, gj, gk);
        jt = 1 << gj | 1 << gk;
    } else {
        /* calculatePosteriors (:79-99) for both samples, then the sum (:209-214);
         * x_j is recomputed in the second pass instead of kept in an array */
        int st = 255, sn = 255;
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            const int xt = (int)rt.lk[j] + ss_tab_prior(m)[rb4 * 10 + j];
            const int xn = (int)rn.lk[j] + ss_tab_prior(m)[rb4 * 10 + j];
            st = qadd(ss_tab_qadd(m), xt, st, clamped);
            sn = qadd(ss_tab_qadd(m), xn, sn, clamped);
        }
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            int vt = (int)rt.lk[j] + ss_tab_prior(m)[rb4 * 10 + j] - st;
            int vn = (int)rn.lk[j] + ss_tab_prior(m)[rb4 * 10 + j] - sn;
            if (vt > 255) vt = 255;
            if (vn > 255) vn = 255;
            qps = qadd(ss_tab_qadd(m), qps, vt + vn, clamped);
        }
    }
    a.score[site] = qps;
    if (clamped && a.n_clamped) atomicAdd(a.n_clamped, (uint32_t)clamped);
    const int tg = jt ? jt : t1, ng = jn ? jn : n1;
    const bool emit = m.min_somatic_qual <= qps &&
                      ((m.flags & SS_MF_LOH) || !proper_subset(tg, ng)) &&
                      ((m.flags & SS_MF_GOR) || !(!proper_subset(rb4, ng) && (tg & ~ng) == rb4));
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
 * Main kernel.
 *
 * A wave walks 16-site BLOCKS (grid-strided).  A block's reads are contiguous
 * in both CSR arrays, so a run of its sites ("sub-group") is staged into LDS
 * with LDS-DMA (global_load_lds, no VGPRs) as [tumor reads | normal reads];
 * the DMA of the next sub-group is issued after this one's fold and lands
 * while the likelihood/decision phases run.
 *
 * Phase A, per site: ONE wave-wide bitonic sort of 16-bit keys packed two per
 * VGPR covers both samples (sample bit on top):
 *   sample<<15 | base<<13 | minq<<5 | hasbase<<4 | strand<<3 | t
 * where t in 0..6 encodes baseQ relative to 64/128/192 when minq < 4 (the only
 * case where the reference's baseQ tie-break changes the clamped q, see
 * read_key16) and 0 otherwise.  Inside one (sample, base) group the reference's
 * descending key walk visits elements in exactly this order up to swaps of
 * elements with identical (q, strand), which leave every float sum unchanged.
 * Sorted keys are turned into 16-bit fold records (q | strand<<8) and written
 * back over the site's own staged reads (tumor records into its tumor run,
 * normal records into its normal run).
 *
 * Phases B+C: lane (site, sample) walks its sample's four base groups (longest
 * first, so the wave-wide trip count is set by one long chain per lane) and
 * then evaluates the 10 genotypes.  Phase D: lane s decides site s.
 * ------------------------------------------------------------------------ */
#define GB 16               /* sites per block                 */
#define STG 2048            /* staged u32 per wave             */
#define PK_MAX 512          /* nT + nN handled by the packed sort (K <= 4) */

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void glb_void_t;

struct Slot3 {
    uint32_t rec_n;      /* u32 index of the fold records | non-deleted depth << 16 */
    uint32_t cnt01;      /* cnt[0] | cnt[1] << 16 */
    uint32_t cnt23;      /* cnt[2] | cnt[3] << 16 */
    uint32_t rms;        /* sum of min(mapQ & 0x7f, cap)^2 */
};


struct MainLds {
    uint32_t stage[SS_MAIN_BLOCK / 64][STG];
    Slot3    slot[SS_MAIN_BLOCK / 64][2 * GB];
    SlotRes  res[SS_MAIN_BLOCK / 64][2 * GB];
    uint32_t site[SS_MAIN_BLOCK / 64][GB];
    uint32_t refc[SS_MAIN_BLOCK / 64][GB];
};

/* 16-bit order key (see the section comment); 0xffff = no contribution or pad.
 *   sample<<15 | base<<13 | minq<<5 | hasbase<<4 | strand<<3 | E<<1 | nz
 * E = baseQ >> 6 and nz = (baseQ & 0x3f) != 0 order the reads of one
 * (minq < 4, hasbase, strand) class exactly as the reference's baseQ tie-break
 * does as far as the clamp of sniper_maqcns.c:165 is concerned (classes
 * 1..63 | 64 | 65..127 | 128 | ...); for minq >= 4 they only reorder reads with
 * identical (q, strand), which leaves every sum unchanged.
 * base / hasbase come from two per-site tables with 2-bit fields indexed by
 * 2*nt16 (entry 0, '=', already resolved to the reference base):
 * tb = base, th = hasbase; see nt_tables(). */
__device__ __forceinline__ uint32_t read_key16(uint32_t rd, uint32_t tb, uint32_t th,
                                               uint32_t samplebit)
{
    const uint32_t minq = min(rd & 0xffu, (rd >> 8) & 0xffu);
    const uint32_t lo6 = rd & 0x3f00u;
    const uint32_t nz = lo6 != 0u ? 1u : 0u;
    const uint32_t nt2 = (rd >> 15) & 0x1eu;
    const uint32_t base = __builtin_amdgcn_ubfe(tb, nt2, 2u);
    const uint32_t hb = __builtin_amdgcn_ubfe(th, nt2, 1u);
    const uint32_t E = __builtin_amdgcn_ubfe(rd, 14u, 2u);
    const uint32_t st = __builtin_amdgcn_ubfe(rd, 20u, 1u);
    const uint32_t key = samplebit | base << 13 | minq << 5 | hb << 4 | st << 3 | E << 1 | nz;
    /* a contributing normal read can have every field at its maximum (mapQ =
     * baseQ = 255, T, reverse): 0xfffe keeps it below the pad key, and for
     * minq >= 4 the E / nz bits only order reads of equal (q, strand) */
    return (minq | lo6) != 0u ? min(key, 0xfffeu) : 0xffffu;
}

/* per-site base tables of read_key16 (bam_nt16_nt4_table semantics,
 * sniper_maqcns.c:19,153-154: single-base codes -> 0..3 with hasbase, every
 * other code counts as A without hasbase; code 0 '=' -> the reference base). */
__device__ __forceinline__ void nt_tables(uint32_t ref16, uint32_t &tb, uint32_t &th)
{
    constexpr uint32_t TB = 1u << 4 | 2u << 8 | 3u << 16;     /* C=2 -> 1, G=4 -> 2, T=8 -> 3 */
    constexpr uint32_t TH = 1u << 2 | 1u << 4 | 1u << 8 | 1u << 16;
    tb = TB | ((TB >> (2u * ref16)) & 3u);
    th = TH | ((TH >> (2u * ref16)) & 1u);
}

/* fold record of a sorted key (u32):
 *   bits 0..7   clamped q (sniper_maqcns.c:165)   -- esum multiplier
 *   bit  16     1                                  -- fsum multiplier
 *   bits 24..31 strand << 4 (the field offset of its w counter, see fold_sample) */
__device__ __forceinline__ uint32_t key_to_rec(uint32_t k)
{
    /* q = (minq < 4 && nz) ? 4 : minq  ==  max(minq, nz * 4) */
    const uint32_t q = max((k >> 5) & 0xffu, (k & 1u) << 2);
    return q | 1u << 16 | (k & 8u) << 25;
}

/* 8-bit fold record (wide kernel: twice the sites of a 16-bit record in the
 * same LDS arena, so a sub-group fills the 16 sites of the fold), for sites
 * whose contributing reads all have minq < 64 (wide_q_fits):
 *   bits 0..5 q | bit 6 strand | bit 7 1 (fsum multiplier);
 * (r >> 2) & 16 is strand << 4 like the u32 record's top byte. */
__device__ __forceinline__ uint32_t key_to_rec8(uint32_t k)
{
    const uint32_t q = max((k >> 5) & 0xffu, (k & 1u) << 2);
    return q | (k & 8u) << 3 | 1u << 7;
}

/* every contributing key of the lane's registers has minq < 64 (key bits 11, 12 clear) */
template <int K>
__device__ __forceinline__ bool wide_q_fits(const uint32_t (&v)[1][K])
{
    bool ok = true;
#pragma unroll
    for (int r = 0; r < K; ++r) {
        const uint32_t lo = v[0][r] & 0xffffu, hi = v[0][r] >> 16;
        ok = ok && (lo == 0xffffu || (lo & 0x1800u) == 0u) && (hi == 0xffffu || (hi & 0x1800u) == 0u);
    }
    return ok;
}

template <typename RecT> struct RecForm;
template <> struct RecForm<uint32_t> {
    static __device__ __forceinline__ uint32_t shift(uint32_t r) { return r >> 24; }
    static constexpr uint32_t ONE_BIT = 16u, QBITS = 8u;
};
template <> struct RecForm<uint8_t> {
    static __device__ __forceinline__ uint32_t shift(uint32_t r) { return (r >> 2) & 16u; }
    static constexpr uint32_t ONE_BIT = 7u, QBITS = 6u;
};

__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const us2 x = __builtin_bit_cast(us2, a), y = __builtin_bit_cast(us2, b);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, y));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const us2 x = __builtin_bit_cast(us2, a), y = __builtin_bit_cast(us2, b);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}

/* min / max of x with halfswap(o): the swap is an operand select (op_sel),
 * not an instruction */
__device__ __forceinline__ uint32_t pk_min_swo(uint32_t x, uint32_t o)
{
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(x), "v"(o));
    return r;
}
__device__ __forceinline__ uint32_t pk_max_swo(uint32_t x, uint32_t o)
{
    uint32_t r;
    asm("v_pk_max_u16 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(x), "v"(o));
    return r;
}
/* halfswap(max(x, halfswap(o))) = max(halfswap(x), o) */
__device__ __forceinline__ uint32_t pk_max_swx(uint32_t x, uint32_t o)
{
    uint32_t r;
    asm("v_pk_max_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(x), "v"(o));
    return r;
}

/* x from lane ^ LJ: DPP quad permutes for 1 and 2, bank-masked DPP row
 * shifts for 4 and 8, ds_swizzle for 16 and 31, v_permlane32_swap for 32,
 * DPP mirrors for 3, 7 and 15. */

template <int LJ>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x)
{
    const int xi = (int)x;
    if constexpr (LJ == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(xi, 0xb1, 0xf, 0xf, false);  /* quad_perm 1,0,3,2 */
    } else if constexpr (LJ == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(xi, 0x4e, 0xf, 0xf, false);  /* quad_perm 2,3,0,1 */
    } else if constexpr (LJ == 4) {
        /* banks 0,2 read lane + 4, banks 1,3 lane - 4: two bank-masked moves
         * (the first one's other banks are don't-care: no zeroed old value) */
        const int up = __builtin_amdgcn_mov_dpp(xi, 0x104, 0xf, 0x5, false);          /* row_shl:4 */
        return (uint32_t)__builtin_amdgcn_update_dpp(up, xi, 0x114, 0xf, 0xa, false); /* row_shr:4 */
    } else if constexpr (LJ == 8) {
        const int up = __builtin_amdgcn_mov_dpp(xi, 0x108, 0xf, 0x3, false);          /* row_shl:8 */
        return (uint32_t)__builtin_amdgcn_update_dpp(up, xi, 0x118, 0xf, 0xc, false); /* row_shr:8 */
    } else if constexpr (LJ == 16) {
        /* ds_swizzle bit-mask mode (and 0x1f, xor 0x10): LDS crossbar, no VALU */
        return (uint32_t)__builtin_amdgcn_ds_swizzle(xi, 0x401f);
    } else if constexpr (LJ == 31) {
        return (uint32_t)__builtin_amdgcn_ds_swizzle(xi, 0x7c1f);                  /* xor 0x1f */
    } else if constexpr (LJ == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane_id() & 32u) ? r[0] : r[1];
    } else if constexpr (LJ == 3) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(xi, 0x1b, 0xf, 0xf, false);   /* quad_perm 3,2,1,0 */
    } else if constexpr (LJ == 7) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(xi, 0x141, 0xf, 0xf, false);  /* row_half_mirror */
    } else if constexpr (LJ == 15) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(xi, 0x140, 0xf, 0xf, false);  /* row_mirror */
    } else {
        static_assert(LJ == 63, "unsupported lane xor");
        return xor_lane<32>(xor_lane<31>(x));
    }
}

/* Cross-lane compare-exchange of packed u16 pairs: lanes with bit LJ clear
 * keep min(x, o), lanes with it set keep max(x, o).  (An exec-masked max,
 * 2 VALU instead of 3, measured slower: SALU exec writes.) */
template <int LJ>
__device__ __forceinline__ uint32_t cx_lanes(uint32_t x, uint32_t o)
{
    return (lane_id() & (uint32_t)LJ) ? pk_max(x, o) : pk_min(x, o);
}

/* In-register compare-exchange of the two halves: lo = min, hi = max, by two
 * SDWA word ops instead of swap + min + max + merge.  The second op reads the
 * first one's result through dst_unused:UNUSED_PRESERVE; back to back that
 * read is stale on gfx950 (measured), so either one independent instruction
 * (cx_halves2: two registers interleaved) or one wait state separates them. */
__device__ __forceinline__ uint32_t cx_halves(uint32_t x)
{
    uint32_t r;
    asm volatile("v_max_u16_sdwa %0, %1, %1 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                 "s_nop 0\n\t"
                 "v_min_u16_sdwa %0, %1, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1"
                 : "=&v"(r)
                 : "v"(x));
    return r;
}

__device__ __forceinline__ void cx_halves2(uint32_t &x0, uint32_t &x1)
{
    uint32_t r0, r1;
    asm volatile("v_max_u16_sdwa %0, %2, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                 "v_max_u16_sdwa %1, %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                 "v_min_u16_sdwa %0, %2, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                 "v_min_u16_sdwa %1, %3, %3 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1"
                 : "=&v"(r0), "=&v"(r1)
                 : "v"(x0), "v"(x1));
    x0 = r0;
    x1 = r1;
}

/* cx_halves over every register of the M x K set, two at a time */
template <int M, int K>
__device__ __forceinline__ void halves_all(uint32_t (&v)[M][K])
{
    constexpr int N = M * K;
#pragma unroll
    for (int i = 0; i + 1 < N; i += 2) cx_halves2(v[i / K][i % K], v[(i + 1) / K][(i + 1) % K]);
    if constexpr (N & 1) v[M - 1][K - 1] = cx_halves(v[M - 1][K - 1]);
}

/* half cleaners e <-> e ^ j for j = J, J/2, ..., 1 (compile-time recursion);
 * M independent networks are advanced together so their dependency chains
 * (and DPP wait states) interleave. */
template <int M, int K, uint32_t J>
__device__ __forceinline__ void half_clean(uint32_t (&v)[M][K])
{
    constexpr uint32_t E = 2u * K;
    if constexpr (J == 0) {
        return;
    } else {
        if constexpr (J >= E) {
            constexpr uint32_t lj = J / E;
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int r = 0; r < K; ++r) {
                    const uint32_t o = xor_lane<(int)lj>(v[m][r]);
                    v[m][r] = cx_lanes<(int)lj>(v[m][r], o);
                }
        } else if constexpr (J >= 2u) {
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int r = 0; r < K; ++r) {
                    const int r2 = r ^ (int)(J >> 1);
                    if (r2 > r) {
                        const uint32_t mn = pk_min(v[m][r], v[m][r2]), mx = pk_max(v[m][r], v[m][r2]);
                        v[m][r] = mn;
                        v[m][r2] = mx;
                    }
                }
        } else {
            halves_all<M, K>(v);
        }
        half_clean<M, K, (J >> 1)>(v);
    }
}

/* Bitonic sort (the "flip" formulation: every comparator puts the minimum at
 * the lower index, so all directions are single lane bits), ascending, of
 * 128*K u16 keys: element e = lane*2K + 2r + h lives in half h of v[m][r]. */
template <int M, int K, uint32_t k>
__device__ __forceinline__ void flip_stage(uint32_t (&v)[M][K])
{
    constexpr uint32_t E = 2u * K;
    /* mirror: e <-> e ^ (k-1) */
    if constexpr (k == 2) {
        halves_all<M, K>(v);                              /* e <-> e ^ 1: the two halves */
    } else if constexpr (k <= E) {
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int r = 0; r < K; ++r) {
                const int r2 = ((2 * r) ^ (int)(k - 1)) >> 1;
                if (r2 > r) {
                    const uint32_t mn = pk_min_swo(v[m][r], v[m][r2]);
                    const uint32_t mx = pk_max_swx(v[m][r], v[m][r2]);
                    v[m][r] = mn;
                    v[m][r2] = mx;
                }
            }
    } else {
        constexpr uint32_t mx_lane = k / E - 1u;          /* lane xor of the mirror */
        constexpr int lbit = (int)((mx_lane + 1u) >> 1);    /* lanes with it set keep the max */
#pragma unroll
        for (int m = 0; m < M; ++m) {
            uint32_t nv[K];
#pragma unroll
            for (int r = 0; r < K; ++r) {
                const uint32_t o = xor_lane<(int)mx_lane>(v[m][K - 1 - r]);    /* halves swapped in the op */
                const uint32_t hi = pk_max_swo(v[m][r], o), lo = pk_min_swo(v[m][r], o);
                nv[r] = (lane_id() & (uint32_t)lbit) ? hi : lo;
            }
#pragma unroll
            for (int r = 0; r < K; ++r) v[m][r] = nv[r];
        }
    }
    half_clean<M, K, (k >> 2)>(v);
}

/* level k of the network; the top level (k = 128K, the merge of the two
 * halves) only when `top` (wave-uniform) */
template <int M, int K, uint32_t k>
__device__ __forceinline__ void flip_level(uint32_t (&v)[M][K], bool top)
{
    if constexpr (k < 128u * K) flip_stage<M, K, k>(v);
    else if constexpr (k == 128u * K) { if (top) flip_stage<M, K, k>(v); }
}

template <int M, int K>
__device__ __forceinline__ void packed_bitonic_flip(uint32_t (&v)[M][K], bool top = true)
{
    static_assert(K == 1 || K == 2 || K == 4 || K == 8 || K == 16, "sort size");
    flip_level<M, K, 2>(v, top);
    flip_level<M, K, 4>(v, top);
    flip_level<M, K, 8>(v, top);
    flip_level<M, K, 16>(v, top);
    flip_level<M, K, 32>(v, top);
    flip_level<M, K, 64>(v, top);
    flip_level<M, K, 128>(v, top);
    flip_level<M, K, 256>(v, top);
    flip_level<M, K, 512>(v, top);
    flip_level<M, K, 1024>(v, top);
    flip_level<M, K, 2048>(v, top);
}

/* Split placement.  Every normal key carries the sample bit, so when each
 * sample fits in half of the network (nt, nn <= 64K) and the normal reads go
 * to network elements 64K.. (lanes 32..63), the levels below the top leave the
 * array [tumor sorted, pads | normal sorted, pads]: each sample sorted in its
 * half, and the top merge level (7 of the 28 comparator stages at K = 1) is
 * skipped.  The normal run then starts at element 64K instead of c4. */
template <int K>
__device__ __forceinline__ bool split_fits(uint32_t nt, uint32_t nn)
{
    return nt <= 64u * K && nn <= 64u * K;
}

/* number of u16 keys (both halves of all K registers) below x, wave-wide.
 * The empty asm pins the count where it is computed: otherwise the scheduler
 * clusters all the compares and keeps every 64-bit ballot live (SGPR spills). */
template <int K>
__device__ __forceinline__ uint32_t count_below(const uint32_t (&v)[K], uint32_t x)
{
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < K; ++r) {
        c += (uint32_t)__popcll(__ballot((v[r] & 0xffffu) < x));
        c += (uint32_t)__popcll(__ballot((v[r] >> 16) < x));
    }
    asm volatile("" : "+s"(c));
    return c;
}

/* Phase A for M sites at once (independent networks interleaved): each
 * site's staged reads are keyed, sorted, and its fold records are written
 * back over them (u16 view); slot[2m], slot[2m+1] receive its bookkeeping. */
struct SiteA {
    uint32_t bt, nt, bn, nn, ref16;
};

/* Group sizes (sample, base) do not depend on the order, so they are counted
 * from the keys before the sort, next to the rms sums: each contributing key
 * adds one to its base's field of a per-lane counter (8-bit fields when a
 * sample has at most 128 sort slots, K = 1; else 16-bit fields, two words),
 * and one wave reduction per word replaces the eight ballot-and-popcount
 * boundary counts over the sorted network. */
template <int K>
struct GroupCount {
    static constexpr bool NARROW = K == 1;
    static constexpr int NW = NARROW ? 1 : 2;
    uint32_t t[NW], n[NW];        /* per-lane partial counts: tumor, normal */
    __device__ __forceinline__ void zero()
    {
#pragma unroll
        for (int i = 0; i < NW; ++i) t[i] = n[i] = 0u;
    }
    /* the lane's key pair (k0, k1) of one sample; 0xffff (pad or q = 0) adds nothing */
    __device__ __forceinline__ void add(uint32_t k0, uint32_t k1, bool tum)
    {
        uint32_t inc[NW];
        if constexpr (NARROW) {
            inc[0] = (k0 != 0xffffu ? 1u << ((k0 >> 10) & 0x18u) : 0u) +      /* 8 * base */
                     (k1 != 0xffffu ? 1u << ((k1 >> 10) & 0x18u) : 0u);
        } else {
            const uint32_t o0 = k0 != 0xffffu ? 1u << ((k0 >> 9) & 16u) : 0u; /* 16 * (base & 1) */
            const uint32_t o1 = k1 != 0xffffu ? 1u << ((k1 >> 9) & 16u) : 0u;
            const bool h0 = (k0 >> 14) & 1u, h1 = (k1 >> 14) & 1u;
            inc[0] = (h0 ? 0u : o0) + (h1 ? 0u : o1);
            inc[1] = (h0 ? o0 : 0u) + (h1 ? o1 : 0u);
        }
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            t[i] += tum ? inc[i] : 0u;
            n[i] += tum ? 0u : inc[i];
        }
    }
    /* base b's count from reduced words */
    static __device__ __forceinline__ uint32_t field(const uint32_t *w, int b)
    {
        if constexpr (NARROW) return (w[0] >> (8 * b)) & 0xffu;
        else return (w[b >> 1] >> (16 * (b & 1))) & 0xffffu;
    }
};

template <int K, int M>
__device__ __forceinline__ void sort_sites(uint32_t *stage, const SiteA (&S)[M], uint32_t cap,
                                           Slot3 *slot, Stamps &st)
{
    const uint32_t lane = lane_id();
    uint32_t v[M][K];
    uint32_t rs_t[M], rs_n[M];
    GroupCount<K> gc[M];
    /* input placement (the two elements of a lane are adjacent reads of ONE
     * sample and come from LDS with one ds_read2; a pad element is invalid) */
    bool split = true;
#pragma unroll
    for (int m = 0; m < M; ++m) split = split && split_fits<K>(S[m].nt, S[m].nn);
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const uint32_t nt = S[m].nt, nn = S[m].nn, ntr = nt + (nt & 1u);
        uint32_t tb, th;
        nt_tables(S[m].ref16, tb, th);
        uint32_t a_t = 0, a_n = 0;
        if constexpr (K == 1) gc[m].zero();
#pragma unroll
        for (int r = 0; r < K; ++r) {
            /* i0: index of the lane's first read within its sample.  Split:
             * lanes 0..31 (network elements < 64K) take the tumor, 32..63 the
             * normal.  Otherwise reads are spread over all lanes (the network
             * is indifferent to its input order). */
            const uint32_t e0 = ((uint32_t)r * 64u + lane) * 2u;
            const uint32_t es = ((uint32_t)r * 32u + (lane & 31u)) * 2u;
            const bool tum = split ? lane < 32u : e0 < ntr;
            const uint32_t i0 = split ? es : (tum ? e0 : e0 - ntr);
            const uint32_t idx = i0 + (tum ? S[m].bt : S[m].bn);
            const uint32_t lim = tum ? nt : nn;
            const uint32_t rd0 = stage[idx], rd1 = stage[idx + 1u];
            const uint32_t sb = tum ? 0u : 0x8000u;
            uint32_t k0 = read_key16(rd0, tb, th, sb);
            uint32_t k1 = read_key16(rd1, tb, th, sb);
            const bool in0 = i0 < lim, in1 = i0 + 1u < lim;
            k0 = in0 ? k0 : 0xffffu;
            k1 = in1 ? k1 : 0xffffu;
            const uint32_t t0 = min(rd0 & 0x7fu, cap), t1 = min(rd1 & 0x7fu, cap);
            const uint32_t x = (in0 ? t0 * t0 : 0u) + (in1 ? t1 * t1 : 0u);
            a_t += tum ? x : 0u;                      /* tumor part (non-split) */
            a_n += x;                                 /* both samples */
            if constexpr (K == 1) gc[m].add(k0, k1, tum);
            v[m][r] = k0 | k1 << 16;
        }
        rs_t[m] = a_t;
        rs_n[m] = a_n;
    }
    st.mark(7);
    if (SS_PRIO_SORT) __builtin_amdgcn_s_setprio(SS_PRIO_SORT);
    packed_bitonic_flip<M, K>(v, !split);
    if (SS_PRIO_SORT) __builtin_amdgcn_s_setprio(0);
    st.mark(8);
    uint32_t *rec = stage;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const uint32_t nt = S[m].nt, nn = S[m].nn, bt = S[m].bt, bn = S[m].bn;
        /* boundaries c1..c8 of the (sample, base) groups in the sorted
         * network: at K = 1 from the group sizes counted before the sort (8-bit
         * fields, one word per sample); at K = 2, 4 by ballot over the sorted
         * keys (a sample's 256 reads can overflow an 8-bit field, and two-word
         * counts measured 1.8% slower at 100x/60x) */
        uint32_t c1, c2, c3, c4, c5, c6, c7, c8;
        if constexpr (K == 1) {
            uint32_t wt[1], wn[1];
            if (split) {                  /* one sample per half-wave */
                const uint32_t h = wave_halfsums(gc[m].t[0] + gc[m].n[0]);
                wt[0] = (uint32_t)__builtin_amdgcn_readlane((int)h, 31);
                wn[0] = (uint32_t)__builtin_amdgcn_readlane((int)h, 63);
            } else {
                wt[0] = wave_sum(gc[m].t[0]);
                wn[0] = wave_sum(gc[m].n[0]);
            }
            c1 = GroupCount<K>::field(wt, 0); c2 = c1 + GroupCount<K>::field(wt, 1);
            c3 = c2 + GroupCount<K>::field(wt, 2); c4 = c3 + GroupCount<K>::field(wt, 3);
            c5 = c4 + GroupCount<K>::field(wn, 0); c6 = c5 + GroupCount<K>::field(wn, 1);
            c7 = c6 + GroupCount<K>::field(wn, 2); c8 = c7 + GroupCount<K>::field(wn, 3);
        } else {
            c1 = count_below<K>(v[m], 1u << 13); c2 = count_below<K>(v[m], 2u << 13);
            c3 = count_below<K>(v[m], 3u << 13); c4 = count_below<K>(v[m], 4u << 13);
            c5 = count_below<K>(v[m], 5u << 13); c6 = count_below<K>(v[m], 6u << 13);
            c7 = count_below<K>(v[m], 7u << 13); c8 = count_below<K>(v[m], 0xffffu);
        }
        st.mark(9);
        /* fold records back over the staged reads: tumor run, normal run */
        if (split) {
            /* one sample per half-wave: a per-lane base, constant offsets */
            const bool tl = lane < 32u;
            const uint32_t e0 = lane * (2u * K);
            const uint32_t lim = tl ? c4 : 64u * K + (c8 - c4);
            uint32_t *rl0 = rec + ((tl ? bt : bn - 64u * K) + e0);
#pragma unroll
            for (int r = 0; r < K; ++r)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (e0 + 2u * r + (uint32_t)h < lim)
                        rl0[2 * r + h] = key_to_rec((v[m][r] >> (16 * h)) & 0xffffu);
        } else {
#pragma unroll
            for (int r = 0; r < K; ++r) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t e = lane * (2u * K) + 2u * r + (uint32_t)h;
                    const uint32_t key = (v[m][r] >> (16 * h)) & 0xffffu;
                    const bool tum = e < c4;
                    if (e < c8) {
                        const uint32_t idx = tum ? bt + e : bn + (e - c4);
                        rec[idx] = key_to_rec(key);
                    }
                }
            }
        }
        /* rms sums: split placement has one sample per half-wave */
        uint32_t rms_t, rms_n;
        if (split) {
            const uint32_t h = wave_halfsums(rs_n[m]);
            rms_t = (uint32_t)__builtin_amdgcn_readlane((int)h, 31);
            rms_n = (uint32_t)__builtin_amdgcn_readlane((int)h, 63);
        } else {
            rms_t = wave_sum(rs_t[m]);
            rms_n = wave_sum(rs_n[m]) - rms_t;
        }
        if (lane == 0) {
            Slot3 &st_t = slot[2 * m], &st_n = slot[2 * m + 1];
            st_t.rec_n = bt | nt << 16;
            st_t.cnt01 = c1 | (c2 - c1) << 16;
            st_t.cnt23 = (c3 - c2) | (c4 - c3) << 16;
            st_t.rms = rms_t;
            st_n.rec_n = bn | nn << 16;
            st_n.cnt01 = (c5 - c4) | (c6 - c5) << 16;
            st_n.cnt23 = (c7 - c6) | (c8 - c7) << 16;
            st_n.rms = rms_n;
        }
        st.mark(10);
    }
}

/* Fold of one (site, sample) by TWO lanes: role 0 accumulates esum, role 1
 * fsum (sniper_maqcns.c:165-172).  Both run the same instruction stream:
 *   acc = (float)((double)acc + fk[w] * m),  m = q (esum) or 1.0 (fsum),
 * and fk[w]*1.0 == fk[w] exactly, so each chain is bit-identical to the
 * reference's.  m is pulled out of the record with a lane-dependent bit-field
 * extract.  The two per-strand w counters live in one register (16-bit
 * fields, counting in units of 8 = the byte stride of fk), selected by the
 * record's strand<<4 field and saturated at w = 255 (:170).  Base groups are
 * walked longest first, so the wave-wide trip count is set by one long chain
 * per lane. */
template <typename RecT>
__device__ __forceinline__ void fold_sample(const RecT *rec, const uint32_t cnt[4],
                                            const double *fk, uint32_t role, float acc[4])
{
    const uint32_t start1 = cnt[0], start2 = cnt[0] + cnt[1], start3 = start2 + cnt[2];
    const uint32_t moff = role ? RecForm<RecT>::ONE_BIT : 0u, mwid = role ? 1u : RecForm<RecT>::QBITS;
    const char *fkb = reinterpret_cast<const char *>(fk);
    uint32_t L = 0;
#pragma unroll
    for (uint32_t b = 1; b < 4; ++b) L = cnt[b] > (L == 0 ? cnt[0] : (L == 1 ? cnt[1] : cnt[2])) ? b : L;
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = 0.0f;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t b = i == 0 ? L : (i - 1u) + ((i - 1u) >= L ? 1u : 0u);
        const uint32_t s0 = b == 0 ? 0u : (b == 1 ? start1 : (b == 2 ? start2 : start3));
        const uint32_t t = b == 0 ? cnt[0] : (b == 1 ? cnt[1] : (b == 2 ? cnt[2] : cnt[3]));
        const RecT *p0 = rec + s0;
        float e = 0.0f;
        uint32_t W = 0;
        uint32_t k = t;                               /* records left, walked from the top */
        /* batches of SS_FOLD_UNROLL: the records and their fk[w] * m terms are
         * all loaded / formed before the dependent chain, which is then only
         * (double)e + term -> (float), as in the reference */
        while (k >= (uint32_t)SS_FOLD_UNROLL) {
            double term[SS_FOLD_UNROLL];
            uint32_t w8[SS_FOLD_UNROLL], m[SS_FOLD_UNROLL];
#pragma unroll
            for (int j = 0; j < SS_FOLD_UNROLL; ++j) {
                const uint32_t r = p0[k - 1u - (uint32_t)j];
                const uint32_t sh = RecForm<RecT>::shift(r);   /* 0 or 16 */
                const uint32_t w = __builtin_amdgcn_ubfe(W, sh, 16u);
                w8[j] = w < 2040u ? w : 2040u;
                W += 8u << sh;
                m[j] = __builtin_amdgcn_ubfe(r, moff, mwid);
            }
#pragma unroll
            for (int j = 0; j < SS_FOLD_UNROLL; ++j) term[j] = *reinterpret_cast<const double *>(fkb + w8[j]);
            /* keep the scheduler from pairing each load with its use (it would
             * wait for every fk load on its own) */
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < SS_FOLD_UNROLL; ++j) e = (float)((double)e + term[j] * (double)m[j]);
            k -= (uint32_t)SS_FOLD_UNROLL;
        }
        while (k) {
            --k;
            const uint32_t r = p0[k];
            const uint32_t sh = RecForm<RecT>::shift(r);
            uint32_t w8 = __builtin_amdgcn_ubfe(W, sh, 16u);
            w8 = w8 < 2040u ? w8 : 2040u;
            W += 8u << sh;
            const double f = *reinterpret_cast<const double *>(fkb + w8);
            const uint32_t m = __builtin_amdgcn_ubfe(r, moff, mwid);
            e = (float)((double)e + f * (double)m);
        }
#pragma unroll
        for (uint32_t bb = 0; bb < 4; ++bb)
            if (bb == b) acc[bb] = e;
    }
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

/* lanes 0..16: off_t[s..s+16], 17..32: ref[s..s+15], 33..49: off_n[s..s+16],
 * 50, 51: off_t[n_sites], off_n[n_sites] (the batch's read counts), 52: set by
 * begin_block when the block has an offset past the end (every site of the
 * block then goes to the deep lists, whose kernels test each site's own
 * offsets and score a malformed one -2) */
__device__ __forceinline__ uint32_t load_desc(const ss_score_args &a, uint32_t s)
{
    /* The block's bases are wave-uniform (scalar registers); the lane offset is
     * made opaque here so the compiler cannot hoist per-lane 64-bit pointers
     * out of the block loop (they would stay live for the whole kernel and
     * spill to scratch). */
    uint32_t lane = lane_id();
    asm volatile("" : "+v"(lane));
    const uint32_t *ot = a.off_t + s, *on = a.off_n + s;
    const uint8_t *rf = a.ref + s;
    const uint32_t rem = (uint32_t)a.n_sites - s;     /* > 0 */
    uint32_t v = 0;
    if (lane < 17u) {
        if (lane <= rem) v = ot[lane];
    } else if (lane < 33u) {
        if (lane - 17u < rem) {
            const uint32_t rc = rf[lane - 17u];
            v = rc | (uint32_t)ss_tab_nt16(a.m)[rc] << 8;
        }
    } else if (lane < 50u) {
        if (lane - 33u <= rem) v = on[lane - 33u];
    } else if (lane < 52u) {
        v = (lane == 50u ? a.off_t : a.off_n)[a.n_sites];
    }
    return v;
}
#define D_T(i) rl(desc, (i))
#define D_REF(i) rl(desc, 17u + (i))
#define D_N(i) rl(desc, 33u + (i))

/* Site sizes of a block (descriptor `desc`), lane i = site i: the inclusive
 * prefix sum of the sites' read counts (DPP row scan over lanes 0..15) and
 * the mask of sites that need more sort slots than the packed main-kernel
 * sort (PK_MAX, incl. the pad element).  Recomputed where needed rather than
 * kept live across the block (register pressure). */
/* a site the packed main-kernel sort cannot take: too many sort slots.  A
 * decreasing offset (malformed batch) wraps one count to ~2^32, so each
 * sample is also tested on its own: such sites go down the deep lists, whose
 * kernel scores them -2 without a read load. */
__device__ __forceinline__ bool off_packed(uint32_t t0, uint32_t t1, uint32_t n0, uint32_t n1)
{
    const uint32_t nt = t1 - t0, nn = n1 - n0;
    return nt + (nt & 1u) + nn > PK_MAX || max(nt, nn) > PK_MAX;
}

struct BlockScan {
    uint32_t incl;        /* per lane: reads of sites 0..lane */
    uint64_t deep;        /* wave-uniform */
};

__device__ __forceinline__ BlockScan scan_block(uint32_t desc, uint32_t nsite)
{
    const uint32_t lane = lane_id();
    /* lane i (< 16): off_t[i] is desc itself, off_t[i + 1] the next lane's
     * (DPP wave_shl:1); off_n[i] comes from lane 33 + i: lane 32 + i by a
     * permlane32 swap, then one more wave_shl:1 (no LDS address register) */
    const auto sw = __builtin_amdgcn_permlane32_swap(desc, desc, false, false);
    const uint32_t n0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sw[1], 0x130, 0xf, 0xf, false);
    const uint32_t t1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)desc, 0x130, 0xf, 0xf, false);
    const uint32_t n1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)n0, 0x130, 0xf, 0xf, false);
    const uint32_t sz = lane < nsite ? (t1 - desc) + (n1 - n0) : 0u;
    BlockScan r;
    const bool alldeep = rl(desc, 52u) != 0u;
    r.deep = __ballot(lane < nsite && (alldeep || off_packed(desc, t1, n0, n1)));
    int x = (int)sz;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);    /* row_shr:1 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);    /* row_shr:2 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);    /* row_shr:4 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);    /* row_shr:8 */
    r.incl = (uint32_t)x;
    return r;
}

/* A block becomes current.  An offset past the batch's read count
 * (descriptor lanes 50 / 51 hold off_t[n], off_n[n]) flags the batch
 * malformed and sends the WHOLE block to the deep lists (descriptor lane 52):
 * the wide and deep kernels test each site's own offsets, so a site that
 * runs past the end scores -2 like any other malformed site, and no site of
 * the block is scored on clamped, foreign reads.  The offsets are clamped as
 * well, so no load of this kernel ever leaves the reads.  Then every site too
 * deep for the packed sort is handed to the wide kernel: one list push per
 * block. */
__device__ __forceinline__ void begin_block(const ss_score_args &a, uint32_t &desc, uint32_t nsite,
                                            uint32_t sblk, uint32_t *seg, uint32_t &ndeep)
{
    const uint32_t lane = lane_id();
    bool alldeep = false;
    {
        const uint32_t end = lane < 17u ? rl(desc, 50u) : rl(desc, 51u);
        const bool off_lane = lane < 17u || (lane >= 33u && lane < 50u);
        const bool past = off_lane && desc > end;
        if (__ballot(past)) {
            if (lane == 0) atomicOr(a.err, SS_KERR_MALFORMED);
            desc = past ? end : (lane == 52u ? 1u : desc);
            alldeep = true;
        }
    }
    const int i = (int)(lane & 15u);
    const uint32_t t0 = (uint32_t)__shfl((int)desc, i), t1 = (uint32_t)__shfl((int)desc, i + 1);
    const uint32_t n0 = (uint32_t)__shfl((int)desc, 33 + i), n1 = (uint32_t)__shfl((int)desc, 34 + i);
    const bool deep = lane < nsite && (alldeep || off_packed(t0, t1, n0, n1));
    const uint64_t mask = __ballot(deep);
    if (mask == 0) return;
    if (deep) {
        const uint32_t d = ndeep + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
        if (d < a.deep_seg_cap) seg[d] = sblk + lane;
        else atomicOr(a.err, SS_KERR_DEEP_OVERFLOW);
    }
    ndeep += (uint32_t)__popcll(mask);
}

struct Sub {
    uint32_t a, b;        /* site range [a, b) within the block */
    uint32_t t0, lt;      /* tumor read run  */
    uint32_t n0, ln;      /* normal read run */
};

/* staged u32 available to one sub-group: the tumor run is rounded up to a
 * multiple of 4 (16-byte LDS-DMA pieces) before the normal run */
#define STG_RUNS (STG - 3)

/* Largest run of sites from `pos` whose reads fit one staging buffer; sites
 * too deep for the packed sort (listed by scan_block) are skipped at the
 * start of a run and end it elsewhere.  Wave-parallel over the block. */
__device__ __forceinline__ Sub form_sub(uint32_t desc, uint32_t nsite, uint32_t pos)
{
    const uint32_t lane = lane_id();
    const BlockScan bs = scan_block(desc, nsite);
    const uint64_t valid = (1ull << nsite) - 1ull;                 /* nsite <= GB < 64 */
    const uint64_t nd = ~bs.deep & valid & ~((1ull << pos) - 1ull);
    Sub r;
    if (nd == 0) {
        pos = nsite;
        r.b = nsite;
    } else {
        pos = (uint32_t)__builtin_ctzll(nd);
        const uint32_t base = pos ? rl(bs.incl, pos - 1u) : 0u;
        const bool stop = lane > pos && lane < nsite && (((bs.deep >> lane) & 1ull) || bs.incl - base > STG_RUNS);
        const uint64_t m = __ballot(stop);
        r.b = m ? (uint32_t)__builtin_ctzll(m) : nsite;
    }
    r.a = pos;
    r.t0 = D_T(pos);
    r.lt = D_T(r.b) - r.t0;
    r.n0 = D_N(pos);
    r.ln = D_N(r.b) - r.n0;
    return r;
}

/* offset of the normal run in the stage */
__device__ __forceinline__ uint32_t normal_base(const Sub &r) { return (r.lt + 3u) & ~3u; }

/* n u32 from src into LDS dst by LDS-DMA: 16-byte pieces, then up to 3 single words */
__device__ __forceinline__ void dma_run(const uint32_t *src, uint32_t n, uint32_t *dst)
{
    const uint32_t lane = lane_id();
    const uint32_t n4 = n & ~3u;
    for (uint32_t i = 0; i < n4; i += 256u)
        if (i + 4u * lane < n4)
            __builtin_amdgcn_global_load_lds((glb_void_t *)(src + i + 4u * lane), (lds_void_t *)(dst + i), 16, 0, 0);
    if (lane < n - n4)
        __builtin_amdgcn_global_load_lds((glb_void_t *)(src + n4 + lane), (lds_void_t *)(dst + n4), 4, 0, 0);
}

__device__ __forceinline__ void issue_dma(const ss_score_args &a, const Sub &r, uint32_t *buf)
{
    dma_run(a.reads_t + r.t0, r.lt, buf);
    dma_run(a.reads_n + r.n0, r.ln, buf + normal_base(r));
}

/* Phases B, C, D for the G sites of a sub-group.  Fold records are RecT
 * entries of `recs` (slot rec_n index); `stage` only receives the next DMA. */
template <typename RecT>
__device__ __forceinline__ void finish_sub(const ss_score_args &a, int G, const RecT *recs, uint32_t *stage,
                                           const Slot3 *slot, SlotRes *res, const uint32_t *sites,
                                           const uint32_t *refcs, const double *fk,
                                           bool have_next, const Sub &nxt, Stamps &st)
{
    const uint32_t lane = lane_id();
    const int sl = (int)(lane >> 1);               /* slot = site * 2 + sample */
    const uint32_t role = lane & 1u;               /* 0: esum lane, 1: fsum lane */
    const bool act = sl < 2 * G;
    float acc[4];
    uint32_t cnt[4], depth = 0, rms = 0;
    if (act) {
        const Slot3 &m3 = slot[sl];
        cnt[0] = m3.cnt01 & 0xffffu; cnt[1] = m3.cnt01 >> 16;
        cnt[2] = m3.cnt23 & 0xffffu; cnt[3] = m3.cnt23 >> 16;
        depth = m3.rec_n >> 16;
        rms = m3.rms;
        const RecT *rec = recs + (m3.rec_n & 0xffffu);
        fold_sample<RecT>(rec, cnt, fk, role, acc);
    } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) { acc[b] = 0.0f; cnt[b] = 0; }
    }
    wave_sync();
    st.mark(3);
    /* exchange esum / fsum within the lane pair (DPP, all lanes active) */
    float es[4], fs[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const float o = __builtin_bit_cast(float, xor_lane<1>(__builtin_bit_cast(uint32_t, acc[b])));
        es[b] = role ? o : acc[b];
        fs[b] = role ? acc[b] : o;
    }
    /* likelihoods: role 0 evaluates genotypes 0..4, role 1 genotypes 5..9 */
    uint32_t c[4];
    const uint32_t tot = rescale_counts(cnt, c);
    float mine[5];
    geno_p5(role, es, fs, c, tot, a.m, mine);
#pragma unroll
    for (int t = 0; t < 5; ++t) mine[t] = act ? mine[t] : 0.0f;
    float p[10];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const float o = __builtin_bit_cast(float, xor_lane<1>(__builtin_bit_cast(uint32_t, mine[t])));
        p[t] = role ? o : mine[t];
        p[5 + t] = role ? mine[t] : o;
    }
    /* Every fold record has been read and every likelihood gather has
     * landed: the next sub-group's reads may now stream into the stage while
     * the glf records and decisions are formed.  (Issued before the gathers,
     * the DMA was waited for at the first gather: vmcnt drains in issue
     * order.) */
    if (have_next) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_dma(a, nxt, stage);
    }
    st.mark(11);
    st.mark(12);
    if (act && role == 0u) {
        uint32_t lk[10], min_lk, rms_q, cns;
        glf_finish(p, es, depth, rms, a.m, lk, min_lk, rms_q, cns);
        SlotRes &r = res[sl];
        uint32_t *rw = reinterpret_cast<uint32_t *>(r.lk);
        rw[0] = lk[0] | lk[1] << 8 | lk[2] << 16 | lk[3] << 24;
        rw[1] = lk[4] | lk[5] << 8 | lk[6] << 16 | lk[7] << 24;
        rw[2] = lk[8] | lk[9] << 8;
        r.cns = cns;
        r.depth = depth;
        if (a.glf) {
            const uint32_t s = (uint32_t)sl >> 1;
            store_glf(&a.glf[2ull * sites[s] + (sl & 1)], refcs[s] >> 8, lk, min_lk,
                      rms_q, depth);
        }
    }
    wave_sync();
    st.mark(4);
    /* the decision reads both samples' records straight from LDS */
    if ((int)lane < G) decide_site(a, sites[lane], refcs[lane], res[2 * lane], res[2 * lane + 1]);
    wave_sync();
    st.mark(5);
}

}  // namespace

/* compiled for 4 waves per SIMD (the VGPR and the LDS budget both allow 4) */
__global__ __launch_bounds__(SS_MAIN_BLOCK) __attribute__((amdgpu_waves_per_eu(4)))
void ss_score_main(ss_score_args a)
{
    __shared__ double fk[256];
    __shared__ MainLds L;
    const uint32_t lane = lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   /* wave-uniform */
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) fk[i] = ss_tab_fk(a.m)[i];
    __syncthreads();
    Stamps st;
    st.start();

    uint32_t *stage = L.stage[wv];
    Slot3 *slot = L.slot[wv];
    SlotRes *res = L.res[wv];
    uint32_t *sites = L.site[wv], *refcs = L.refc[wv];
    /* block bookkeeping in 32-bit scalars (n_sites < 2^32, checked on the host) */
    const uint32_t nwaves = gridDim.x * (SS_MAIN_BLOCK / 64);
    const uint32_t n_sites = (uint32_t)a.n_sites;
    const uint32_t nblocks = (n_sites + GB - 1) / GB;
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;

    uint32_t blk = blockIdx.x * (SS_MAIN_BLOCK / 64) + wv;
    /* this wave's segment of the deep list; its length is stored on every exit */
    const uint32_t gw = blk;
    uint32_t *seg = a.deep_list + (size_t)gw * a.deep_seg_cap;
    uint32_t ndeep = 0;
    if (blk >= nblocks) {
        if (lane == 0) a.deep_seg_n[gw] = 0u;
        st.flush();
        return;
    }
    uint32_t desc = load_desc(a, blk * GB);
    uint32_t nsite = min(n_sites - blk * GB, (uint32_t)GB);
    uint32_t nblk = blk + nwaves;
    uint32_t ndesc = nblk < nblocks ? load_desc(a, nblk * GB) : 0u;
    begin_block(a, desc, nsite, blk * GB, seg, ndeep);
    Sub cur = form_sub(desc, nsite, 0);
    while (cur.a == cur.b) {               /* whole block deep */
        blk = nblk;
        if (blk >= nblocks) {
            if (lane == 0) a.deep_seg_n[gw] = ndeep;
            st.flush();
            return;
        }
        desc = ndesc;
        nsite = min(n_sites - blk * GB, (uint32_t)GB);
        nblk = blk + nwaves;
        ndesc = nblk < nblocks ? load_desc(a, nblk * GB) : 0u;
        begin_block(a, desc, nsite, blk * GB, seg, ndeep);
        cur = form_sub(desc, nsite, 0);
    }
    issue_dma(a, cur, stage);
    st.mark(6);

    for (;;) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   /* the sub-group's reads are in LDS */
        st.mark(0);
        /* ---- phase A ---- */
        int G = 0;
        for (uint32_t i = cur.a; i < cur.b;) {
            SiteA S2[2];
            uint32_t tot[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const uint32_t j = i + (uint32_t)m < cur.b ? i + (uint32_t)m : i;
                const uint32_t t_i = D_T(j), n_i = D_N(j);
                const uint32_t rdesc = D_REF(j);
                S2[m].nt = D_T(j + 1u) - t_i;
                S2[m].nn = D_N(j + 1u) - n_i;
                S2[m].bt = t_i - cur.t0;
                S2[m].bn = normal_base(cur) + (n_i - cur.n0);
                S2[m].ref16 = rdesc >> 8;
                tot[m] = S2[m].nt + (S2[m].nt & 1u) + S2[m].nn;   /* sort slots incl. pad */
                if (lane == 0 && i + (uint32_t)m < cur.b) {
                    sites[G + m] = blk * GB + j;
                    refcs[G + m] = rdesc & 0xffffu;      /* ref char | nt16 << 8 */
                }
            }
            if (i + 1u < cur.b && tot[0] <= 256u && tot[1] <= 256u) {   /* two sites, interleaved */
                if (tot[0] <= 128u && tot[1] <= 128u) sort_sites<1, 2>(stage, S2, cap, slot + 2 * G, st);
                else sort_sites<2, 2>(stage, S2, cap, slot + 2 * G, st);
                G += 2;
                i += 2;
                continue;
            }
            SiteA S1[1] = {S2[0]};
            if (tot[0] <= 128u) sort_sites<1, 1>(stage, S1, cap, slot + 2 * G, st);
            else if (tot[0] <= 256u) sort_sites<2, 1>(stage, S1, cap, slot + 2 * G, st);
            else sort_sites<4, 1>(stage, S1, cap, slot + 2 * G, st);
            ++G;
            ++i;
        }
        wave_sync();
        st.mark(1);
        /* ---- next sub-group: same block, else the next non-empty block ---- */
        Sub nxt;
        bool have = false;
        if (cur.b < nsite) {
            nxt = form_sub(desc, nsite, cur.b);
            have = nxt.a < nxt.b;
        }
        while (!have) {
            blk = nblk;
            if (blk >= nblocks) break;
            desc = ndesc;
            nsite = min(n_sites - blk * GB, (uint32_t)GB);
            nblk = blk + nwaves;
            ndesc = nblk < nblocks ? load_desc(a, nblk * GB) : 0u;
            begin_block(a, desc, nsite, blk * GB, seg, ndeep);
            nxt = form_sub(desc, nsite, 0);
            have = nxt.a < nxt.b;
        }
        st.mark(2);
        /* ---- phases B + C + D (the next DMA is issued after the fold) ---- */
        finish_sub<uint32_t>(a, G, stage, stage, slot, res, sites, refcs, fk, have, nxt, st);
        if (!have) break;
        cur = nxt;
    }
    if (lane == 0) a.deep_seg_n[gw] = ndeep;
    st.flush();
}

/* --------------------------------------------------------------------------
 * Wide kernel: the sites the main kernel left on the deep list (more than
 * PK_MAX sort slots, e.g. 500x/500x panels) whose samples have at most
 * SS_WIDE_MAXSLOTS reads each.
 *
 * One workgroup per CU, SS_WIDE_BLOCK / 64 independent waves sharing 144 KB
 * of LDS as per-wave arenas of 8-bit fold records.  A wave takes 16 list
 * entries at a time and, sort unit by sort unit, loads the packed reads
 * straight from HBM into registers, sorts them with the same packed bitonic
 * network as the main kernel (1024 or 2048 keys: K = 8 or 16 registers), and
 * writes the fold records into the arena.  A unit is a whole site of at most
 * SS_WIDE_MAXSLOTS sort slots (both samples in one network), else one of its
 * samples (1200x/1000x panels; also past 1024 slots when one sample has at
 * most 512 reads: K = 4 + K = 8 instead of one 2048-key network).  Then the sites are folded together -- lane =
 * (site, sample, role), so the wave runs up to 64 serial chains at once
 * instead of one -- and finished by the main kernel's code.  Larger or
 * malformed sites, and sites with a read of minq >= 64, go to the second
 * deep list (ss_score_deep).
 * ------------------------------------------------------------------------ */
namespace {

#define WIDE_WAVES (SS_WIDE_BLOCK / 64)
#define WIDE_LDS_REC 147456                /* u8 fold records per workgroup: 144 KB of LDS */
#define WIDE_ARENA (WIDE_LDS_REC / WIDE_WAVES)      /* per wave (< 2^16: Slot3 rec_n) */

struct alignas(16) WideLds {
    uint8_t arena[WIDE_WAVES][WIDE_ARENA];
    Slot3    slot[WIDE_WAVES][2 * GB];
    SlotRes  res[WIDE_WAVES][2 * GB];
    uint32_t site[WIDE_WAVES][GB];
    uint32_t refc[WIDE_WAVES][GB];
};

/* A wide site's packed reads in the sort placement (tumor [0, nt), normal
 * [ntr, ntr + nn)): element pair (e0, e0 + 1), e0 = 2 * (r * 64 + lane), in
 * rd[2r], rd[2r + 1]; 0 (no contribution) outside the site.  Issued one site
 * ahead of its sort so the HBM latency overlaps the previous site's work. */
struct WideSite {
    uint32_t ot, nt, on, nn;
    uint32_t ref;      /* ref char | nt16 code << 8, loaded with the offsets (one site ahead) */
    uint32_t unit;     /* 0 the whole site, 1 its tumor, 2 its normal (see wide_place) */
    uint32_t sp;       /* non-split placement: elements below sp are tumor reads, the rest normal */
    bool split;        /* unit 0, split placement (see split_fits): top level skipped */
    bool over;         /* a sample beyond SS_WIDE_MAXSLOTS reads or malformed offsets: deep kernel */
};

__device__ __forceinline__ void wide_place(WideSite &w, uint32_t end_t, uint32_t end_n)
{
    w.over = max(w.nt, w.nn) > SS_WIDE_MAXSLOTS ||
             w.ot + w.nt < w.ot || w.ot + w.nt > end_t || w.on + w.nn < w.on || w.on + w.nn > end_n;
    const uint32_t slots = w.nt + (w.nt & 1u) + w.nn;
    /* past 1024 slots with one sample of at most 512 reads: a 512-key and a
     * 1024-key network (45 x 4 + 55 x 8 register stages) instead of one split
     * 2048-key network (55 x 16) */
    const bool small_unit = slots > 1024u && max(w.nt, w.nn) <= 1024u && min(w.nt, w.nn) <= 512u;
    w.unit = !w.over && (slots > SS_WIDE_MAXSLOTS || small_unit) ? 1u : 0u;
    w.sp = w.unit ? 0xffffu : w.nt + (w.nt & 1u);
    const bool k8 = slots <= 1024u;                          /* the network sort_site_wide picks */
    w.split = !w.unit && (k8 ? split_fits<8>(w.nt, w.nn) : split_fits<16>(w.nt, w.nn));
}

/* the normal unit of a site whose tumor unit w was */
__device__ __forceinline__ WideSite wide_normal_unit(WideSite w)
{
    w.unit = 2u;
    w.sp = 0u;
    return w;
}

/* network size of a unit: reads it sorts (incl. the pad between samples) */
__device__ __forceinline__ uint32_t wide_unit_slots(const WideSite &w)
{
    return w.unit == 0u ? w.nt + (w.nt & 1u) + w.nn : (w.unit == 1u ? w.nt : w.nn);
}

/* All 16 register pairs, whatever the site's network: choosing 8 or 16 by a
 * branch put rd in scratch (measured 30% slower).  One base pointer and
 * limit per lane (split) or two (otherwise): 5% faster at 500x/500x than a
 * per-pair select of sample, index and pointer. */
__device__ __forceinline__ void wide_load(const ss_score_args &a, const WideSite &w, uint32_t (&rd)[32])
{
    const uint32_t lane = lane_id();
    if (w.split) {
        /* lanes 0..31 the tumor, 32..63 the normal: one base pointer per lane */
        const bool tl = lane < 32u;
        const uint32_t *bp = tl ? a.reads_t + w.ot : a.reads_n + w.on;
        const uint32_t lim = w.over ? 0u : (tl ? w.nt : w.nn);
        const uint32_t i00 = (lane & 31u) * 2u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t i0 = i00 + (uint32_t)r * 64u;
            rd[2 * r] = i0 < lim ? __builtin_nontemporal_load(bp + i0) : 0u;
            rd[2 * r + 1] = i0 + 1u < lim ? __builtin_nontemporal_load(bp + i0 + 1) : 0u;
        }
    } else {
        /* element e: tumor read e below sp, normal read e - sp above (a
         * unit takes one sample: sp past every element, or 0).  The normal
         * base is offset by -sp so that element e indexes it directly; for a
         * tumor unit it is never dereferenced. */
        const uint32_t sp = w.sp;
        const uint32_t *tp = a.reads_t + w.ot, *np = a.reads_n + w.on - sp;
        const uint32_t lt = w.over ? 0u : w.nt, ln = w.over ? 0u : sp + w.nn;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t e0 = ((uint32_t)r * 64u + lane) * 2u;            /* as in sort_sites */
            const bool tum = e0 < sp;
            const uint32_t *src = (tum ? tp : np) + e0;
            const uint32_t lim = tum ? lt : ln;
            rd[2 * r] = e0 < lim ? __builtin_nontemporal_load(src) : 0u;
            rd[2 * r + 1] = e0 + 1u < lim ? __builtin_nontemporal_load(src + 1) : 0u;
        }
    }
}

/* Returns the arena bytes the site's records take (a multiple of 2K, the
 * lane's share), or -1 (nothing written) when a contributing read has
 * minq >= 64: the 8-bit record cannot hold its q, and the site goes to the
 * deep kernel. */
template <int K>
__device__ __forceinline__ int sort_site_wide(const uint32_t (&rd)[32], const WideSite &w, uint32_t ref16,
                                               uint32_t cap, uint8_t *arena, uint32_t base, Slot3 *st2)
{
    const uint32_t lane = lane_id();
    const uint32_t nt = w.nt, nn = w.nn;
    uint32_t tb, th;
    nt_tables(ref16, tb, th);
    uint32_t v[1][K];
    uint32_t a_t = 0, a_n = 0;
    GroupCount<K> gc;
    gc.zero();
    /* registers whose elements are all pads (rd = 0: key 0xffff, no rms or
     * count) skip the key build: a wave-uniform bound on the live elements */
    const uint32_t live = w.split ? 2u * max(nt, nn) : wide_unit_slots(w);
#pragma unroll
    for (int r = 0; r < K; ++r) {
        if ((uint32_t)r * 128u >= live) {
            v[0][r] = 0xffffffffu;
            continue;
        }
        const uint32_t e0 = ((uint32_t)r * 64u + lane) * 2u;
        const bool tum = w.split ? lane < 32u : e0 < w.sp;
        const uint32_t rd0 = rd[2 * r], rd1 = rd[2 * r + 1];
        const uint32_t sb = tum ? 0u : 0x8000u;
        const uint32_t k0 = read_key16(rd0, tb, th, sb), k1 = read_key16(rd1, tb, th, sb);
        const uint32_t t0 = min(rd0 & 0x7fu, cap), t1 = min(rd1 & 0x7fu, cap);
        const uint32_t x = t0 * t0 + t1 * t1;
        a_t += tum ? x : 0u;
        a_n += tum ? 0u : x;
        gc.add(k0, k1, tum);
        v[0][r] = k0 | k1 << 16;
    }
    if (__ballot(!wide_q_fits<K>(v))) return -1;
    /* group sizes before the sort (see GroupCount) */
    uint32_t wt[2], wn[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        wt[i] = wave_sum(gc.t[i]);
        wn[i] = wave_sum(gc.n[i]);
    }
    if (SS_PRIO_WIDE) __builtin_amdgcn_s_setprio(SS_PRIO_WIDE);
    packed_bitonic_flip<1, K>(v, !w.split);
    if (SS_PRIO_WIDE) __builtin_amdgcn_s_setprio(0);
    const uint32_t c1 = GroupCount<K>::field(wt, 0), c2 = c1 + GroupCount<K>::field(wt, 1);
    const uint32_t c3 = c2 + GroupCount<K>::field(wt, 2), c4 = c3 + GroupCount<K>::field(wt, 3);
    const uint32_t c5 = c4 + GroupCount<K>::field(wn, 0), c6 = c5 + GroupCount<K>::field(wn, 1);
    const uint32_t c7 = c6 + GroupCount<K>::field(wn, 2), c8 = c7 + GroupCount<K>::field(wn, 3);
    /* The record of network element e goes to base + e: the lane's 2K
     * elements are contiguous, so they leave as 16-byte stores.  The tumor
     * groups start at base, the normal ones at base + nb; pad and q = 0
     * elements land past each sample's groups and are never read.  Lanes
     * wholly past the extent store nothing (the next site starts there). */
    const uint32_t nb = w.split ? 64u * K : c4;
    /* extents stay multiples of 16 bytes: every unit's stores are 16-byte aligned */
    constexpr uint32_t XR = K < 8 ? 16u : 2u * K;
    const uint32_t extent = ((w.split ? nb + (c8 - c4) : c8) + XR - 1u) & ~(XR - 1u);
    if constexpr (K == 4) {
        if (lane * 8u < extent) {
            uint32_t d[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t x = v[0][2 * j], y = v[0][2 * j + 1];
                d[j] = key_to_rec8(x & 0xffffu) | key_to_rec8(x >> 16) << 8 |
                       key_to_rec8(y & 0xffffu) << 16 | key_to_rec8(y >> 16) << 24;
            }
            *reinterpret_cast<uint2 *>(arena + base + lane * 8u) = make_uint2(d[0], d[1]);
        }
    } else if (lane * (2u * K) < extent) {
#pragma unroll
        for (int q = 0; q < K / 8; ++q) {
            uint32_t d[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t x = v[0][8 * q + 2 * j], y = v[0][8 * q + 2 * j + 1];
                d[j] = key_to_rec8(x & 0xffffu) | key_to_rec8(x >> 16) << 8 |
                       key_to_rec8(y & 0xffffu) << 16 | key_to_rec8(y >> 16) << 24;
            }
            *reinterpret_cast<uint4 *>(arena + base + lane * (2u * K) + 16u * (uint32_t)q) =
                make_uint4(d[0], d[1], d[2], d[3]);
        }
    }
    const uint32_t rms_t = wave_sum(a_t), rms_n = wave_sum(a_n);
    /* a sample unit fills only its sample's slot */
    if (lane == 0 && w.unit != 2u) {
        st2[0].rec_n = base | nt << 16;
        st2[0].cnt01 = c1 | (c2 - c1) << 16;
        st2[0].cnt23 = (c3 - c2) | (c4 - c3) << 16;
        st2[0].rms = rms_t;
    }
    if (lane == 0 && w.unit != 1u) {
        st2[1].rec_n = (base + nb) | nn << 16;
        st2[1].cnt01 = (c5 - c4) | (c6 - c5) << 16;
        st2[1].cnt23 = (c7 - c6) | (c8 - c7) << 16;
        st2[1].rms = rms_n;
    }
    return (int)extent;
}

}  // namespace

__global__ __launch_bounds__(SS_WIDE_BLOCK) void ss_score_wide(ss_score_args a)
{
    __shared__ double fk[256];
    __shared__ WideLds L;
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) fk[i] = ss_tab_fk(a.m)[i];
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   /* wave-uniform */
    uint8_t *arena = L.arena[wv];
    Slot3 *slot = L.slot[wv];
    SlotRes *res = L.res[wv];
    uint32_t *sites = L.site[wv], *refcs = L.refc[wv];
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;
    const Sub none = {0, 0, 0, 0, 0, 0};
    const uint32_t end_t = a.off_t[a.n_sites], end_n = a.off_n[a.n_sites];
    /* the main kernel's per-wave segments, GB entries at a time */
    for (uint32_t sg = blockIdx.x * WIDE_WAVES + wv; sg < a.deep_nseg; sg += gridDim.x * WIDE_WAVES)
    for (uint32_t first = 0, scount = min(a.deep_seg_n[sg], a.deep_seg_cap); first < scount; first += GB) {
        const uint32_t *list = a.deep_list + (size_t)sg * a.deep_seg_cap;
        const uint32_t nlist = scount - first < GB ? scount - first : GB;
        /* site i's reads are in flight while site i-1 is sorted */
        uint32_t i = 0, s_cur = 0;
        WideSite w_cur = {0, 0, 0, 0, 0, 0, 0, false, false};
        uint32_t rd[32];
        /* the chunk's descriptors, lane k = entry k, loaded at once (one
         * exposed chain of dependent loads per chunk, not per site) */
        uint32_t c_s = 0, c_ot = 0, c_ot1 = 0, c_on = 0, c_on1 = 0, c_ref = 0;
        if (lane < nlist) {
            c_s = list[first + lane];
            c_ot = a.off_t[c_s];
            c_ot1 = a.off_t[c_s + 1];
            c_on = a.off_n[c_s];
            c_on1 = a.off_n[c_s + 1];
            const uint32_t rc = a.ref[c_s];
            c_ref = rc | (uint32_t)ss_tab_nt16(a.m)[rc] << 8;
        }
        auto describe = [&](uint32_t k, uint32_t &s, WideSite &w) {
            s = rl(c_s, k);
            w.ot = rl(c_ot, k);
            w.nt = rl(c_ot1, k) - w.ot;
            w.on = rl(c_on, k);
            w.nn = rl(c_on1, k) - w.on;
            w.ref = rl(c_ref, k);
            wide_place(w, end_t, end_n);
        };
        if (nlist) {
            describe(0, s_cur, w_cur);
            wide_load(a, w_cur, rd);
        }
        uint32_t ext_t = 0;             /* arena bytes of the current site's tumor unit */
        bool dead = false;              /* that tumor unit sent the site to the deep list */
        while (i < nlist) {
            int G = 0;
            uint32_t used = 0;
            while (i < nlist) {
                const uint32_t s = s_cur;
                const WideSite w = w_cur;
                const uint32_t slots = wide_unit_slots(w);
                /* the most arena the site can take (sort_site_wide's extents), checked where a site starts */
                const uint32_t kb = slots <= 1024u ? 16u : 32u;
                const uint32_t bound = w.unit ? ((w.nt + 31u) & ~31u) + ((w.nn + 31u) & ~31u)
                                              : ((w.split ? 32u * kb + w.nn : slots) + kb - 1u) & ~(kb - 1u);
                if (w.unit != 2u && used + bound > WIDE_ARENA && !w.over) break;   /* next sub-group */
                uint32_t cur[32];
#pragma unroll
                for (int k = 0; k < 32; ++k) cur[k] = rd[k];
                if (w.unit == 1u) {                       /* next: the same site's normal */
                    w_cur = wide_normal_unit(w);
                    wide_load(a, w_cur, rd);
                } else {
                    if (i + 1 < nlist) {
                        describe(i + 1, s_cur, w_cur);
                        wide_load(a, w_cur, rd);
                    }
                    ++i;
                }
                if (w.unit == 2u && dead) {               /* already on the deep list */
                    dead = false;
                    continue;
                }
                const uint32_t ref16 = w.ref >> 8;
                const uint32_t base = used + (w.unit == 2u ? ext_t : 0u);
                const int ext = w.over ? -1
                              : w.unit && slots <= 512u ? sort_site_wide<4>(cur, w, ref16, cap, arena, base, slot + 2 * G)
                              : slots <= 1024u ? sort_site_wide<8>(cur, w, ref16, cap, arena, base, slot + 2 * G)
                                               : sort_site_wide<16>(cur, w, ref16, cap, arena, base, slot + 2 * G);
                if (ext < 0) {
                    if (lane == 0) {
                        const uint32_t d = atomicAdd(a.deep2_count, 1u);
                        if (d < a.deep_cap) a.deep2_list[d] = s;
                        else atomicOr(a.err, SS_KERR_DEEP_OVERFLOW);
                    }
                    dead = w.unit == 1u;
                    continue;
                }
                if (w.unit == 1u) {                       /* the site completes with its normal unit */
                    ext_t = (uint32_t)ext;
                    continue;
                }
                if (lane == 0) {
                    sites[G] = s;
                    refcs[G] = w.ref;
                }
                used += (w.unit == 2u ? ext_t : 0u) + (uint32_t)ext;
                ++G;
            }
            wave_sync();
            Stamps nost;
            if (G) finish_sub<uint8_t>(a, G, arena, nullptr, slot, res, sites, refcs, fk, false, none, nost);
        }
    }
}

/* --------------------------------------------------------------------------
 * Deep kernel: the sites the wide kernel cannot sort (more than
 * SS_WIDE_MAXSLOTS sort slots, any depth) and sites with malformed offsets.
 *
 * No sort: the fold only needs each (sample, base) group's reads in the
 * reference's descending key order (sniper_maqcns.c:157-172), and reads with
 * equal (q, strand) contribute identical terms (see read_key16), so a
 * counting sort over the order-relevant key fields is exact.  Bins of one
 * base group, ascending in key order (DBIN per group):
 *   minq <  4:  minq<<5 | hasbase<<4 | strand<<3 | E<<1 | nz        0..127
 *   minq >= 4:  128 + (minq - 4) * 4 + hasbase * 2 + strand         128..1135
 * (for minq >= 4, E and nz only order reads of equal q and strand).
 *
 * One wave per site, so a CU holds 12 sites at once.  A first pass over the
 * site's reads finds its highest occupied bin and the rms sums.  The bins
 * are then histogrammed in LDS one window of DW_BINS per group at a time,
 * from the top down (one window when every read has minq <= 60); after each
 * window 16 lanes -- (sample, base, role) -- walk their group's occupied
 * bins downwards through a bitmap and fold count-many steps per bin,
 * carrying the chain across windows: the reference's serial chain, O(depth),
 * with no depth limit and no scratch memory.  The quads then evaluate the
 * genotype likelihoods and lane 0 decides the site.
 * ------------------------------------------------------------------------ */
namespace {

#define DBIN 1136                       /* bins per group, all minq */
#define DW_BINS 368                     /* bins per group in one LDS window */
#define DW_HIST (8 * DW_BINS)
#define DW_OCC (DW_HIST / 32)
#define DEEP_WAVES (SS_DEEP_BLOCK / 64)
static_assert(DW_HIST % 32 == 0 && DW_BINS % 4 == 0, "bitmap words");

struct alignas(16) DeepWave {
    uint32_t hist[DW_HIST];
    uint32_t occ[DW_OCC];
    unsigned long long rms[2];
    SlotRes res[2];
};

/* group bin of one packed read, base << 16 | bin, or SENT when its clamped q
 * is 0 (no contribution, sniper_maqcns.c:165-166) */
__device__ __forceinline__ uint32_t deep_bin(uint32_t rd, uint32_t tb, uint32_t th)
{
    const uint32_t bq = (rd >> 8) & 0xffu;
    const uint32_t minq = min(rd & 0xffu, bq);
    const uint32_t nz = (bq & 0x3fu) != 0u ? 1u : 0u;
    const uint32_t nt2 = (rd >> 15) & 0x1eu;
    const uint32_t base = __builtin_amdgcn_ubfe(tb, nt2, 2u);
    const uint32_t hb = __builtin_amdgcn_ubfe(th, nt2, 1u);
    const uint32_t st = (rd >> 20) & 1u;
    const uint32_t idx = minq < 4u ? (minq << 5 | hb << 4 | st << 3 | (bq >> 6) << 1 | nz)
                                   : 128u + (minq - 4u) * 4u + hb * 2u + st;
    return (minq | nz) != 0u ? base << 16 | idx : SENT;
}

/* offsets of a site are usable iff they neither decrease nor pass the end of
 * the batch's reads (a malformed batch must not steer a load anywhere else) */
__device__ __forceinline__ bool site_wellformed(uint32_t o0, uint32_t o1, uint32_t end)
{
    return o0 <= o1 && o1 <= end;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

/* one pass over one sample's reads, eight in flight per lane: counts the
 * reads whose bin falls in [lo, hi) into the window histogram; mode 0 (the
 * first pass, lo = 0, hi = DW_BINS) also returns the highest bin + 1 over the
 * reads and adds the rms terms to rs */
template <int MODE>
__device__ __forceinline__ uint32_t deep_pass(const uint32_t *reads, uint32_t n, uint32_t tb, uint32_t th,
                                              uint32_t cap, uint32_t lo, uint32_t hi, uint32_t *hist,
                                              uint64_t &rs)
{
    const uint32_t lane = lane_id();
    uint32_t top = 0;
    for (uint64_t i = lane; i < n; i += 8u * 64u) {
        uint32_t rd[8];
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) {
            const uint64_t ix = i + j * 64u;
            rd[j] = ix < n ? __builtin_nontemporal_load(reads + ix) : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) {
            const uint32_t b = deep_bin(rd[j], tb, th);
            const uint32_t idx = b & 0xffffu;
            if (MODE == 0) {
                if (b != SENT) top = max(top, idx + 1u);
                const uint32_t t = min(rd[j] & 0x7fu, cap);
                rs += t * t;
            }
            if (b != SENT && idx >= lo && idx < hi) atomicAdd(&hist[(b >> 16) * DW_BINS + idx - lo], 1u);
        }
    }
    return top;
}

__device__ __forceinline__ void deep_zero(uint32_t *hist)
{
    uint4 *h4 = reinterpret_cast<uint4 *>(hist);
    for (uint32_t i = lane_id(); i < DW_HIST / 4u; i += 64u) h4[i] = make_uint4(0u, 0u, 0u, 0u);
}

/* ordered fold of one (sample, base) group over the window's bins [lo, hi),
 * walked downwards; e, the two strand w counters and the count carry over
 * from the window above (sniper_maqcns.c:160-172) */
__device__ __forceinline__ void deep_fold(const uint32_t *hist, const uint32_t *occ, uint32_t gbin,
                                          uint32_t lo, uint32_t hi, const double *fk, uint32_t role,
                                          float &e, uint32_t &w0, uint32_t &w1, uint32_t &c)
{
    const uint32_t b_lo = gbin, b_hi = gbin + (hi - lo);   /* window slots of this group */
    for (int wi = (int)((b_hi - 1u) >> 5); wi >= (int)(b_lo >> 5); --wi) {
        uint32_t bits = occ[wi];
        const uint32_t b0 = (uint32_t)wi * 32u;
        if (b0 < b_lo) bits &= ~0u << (b_lo - b0);
        if (b0 + 32u > b_hi) bits &= ~0u >> (b0 + 32u - b_hi);
        while (bits) {
            const uint32_t j = 31u - (uint32_t)__builtin_clz(bits);
            bits &= ~(1u << j);
            const uint32_t idx = b0 + j - b_lo + lo;        /* group bin */
            const uint32_t k = hist[b0 + j];
            const uint32_t q = idx < 128u ? max(idx >> 5, (idx & 1u) << 2) : (idx - 128u) / 4u + 4u;
            const uint32_t st = idx < 128u ? (idx >> 3) & 1u : idx & 1u;
            const double mul = role ? 1.0 : (double)q;
            const uint32_t w = st ? w1 : w0;
            /* batches of 8 steps: the eight fk[w] loads are issued before the
             * dependent chain (w advances by one per read, saturating at 255);
             * full batches first, then one masked batch for the rest of the
             * bin.  Measured slower: adding +0.0 for masked steps instead of
             * the select, batches of 16, and loading the next batch during
             * the current chain. */
            uint32_t r = 0;
            for (; r + 8u <= k; r += 8u) {
                double f[8];
#pragma unroll
                for (uint32_t t = 0; t < 8u; ++t) f[t] = fk[min(w + min(r, 256u) + t, 255u)];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (uint32_t t = 0; t < 8u; ++t) e = (float)((double)e + f[t] * mul);
            }
            if (r < k) {
                double f[8];
#pragma unroll
                for (uint32_t t = 0; t < 8u; ++t) f[t] = fk[min(w + min(r, 256u) + t, 255u)];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (uint32_t t = 0; t < 8u; ++t) {
                    const float en = (float)((double)e + f[t] * mul);
                    e = r + t < k ? en : e;
                }
            }
            const uint32_t wn = min(w + min(k, 256u), 255u);
            if (st) w1 = wn; else w0 = wn;
            c += k;
        }
    }
}

}  // namespace

__global__ __launch_bounds__(SS_DEEP_BLOCK) void ss_score_deep(ss_score_args a)
{
    __shared__ double fk[256];
    __shared__ DeepWave DW[DEEP_WAVES];
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) fk[i] = ss_tab_fk(a.m)[i];
    __syncthreads();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    DeepWave &D = DW[wv];
    const uint32_t count = *a.deep2_count;
    const uint32_t lim = count < a.deep_cap ? count : a.deep_cap;
    const uint32_t end_t = a.off_t[a.n_sites], end_n = a.off_n[a.n_sites];
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;
    const uint32_t lane = lane_id();
    const uint32_t grp = ((lane >> 3) & 1u) * 4u + ((lane >> 1) & 3u);  /* fold lanes 0..15: sample, base */
    for (uint32_t w = blockIdx.x * DEEP_WAVES + wv; w < lim; w += gridDim.x * DEEP_WAVES) {
        const uint32_t s = a.deep2_list[w];
        const uint32_t ot = a.off_t[s], ot1 = a.off_t[s + 1], on = a.off_n[s], on1 = a.off_n[s + 1];
        if (!site_wellformed(ot, ot1, end_t) || !site_wellformed(on, on1, end_n)) {
            if (lane == 0) {
                atomicOr(a.err, SS_KERR_MALFORMED);
                a.score[s] = -2;
            }
            continue;                                  /* wave-uniform */
        }
        const uint32_t nt = ot1 - ot, nn = on1 - on;
        const uint32_t refc = a.ref[s];
        const uint32_t ref16 = ss_tab_nt16(a.m)[refc];
        uint32_t tb, th;
        nt_tables(ref16, tb, th);
        if (lane < 2u) D.rms[lane] = 0ull;
        deep_zero(D.hist);
        wave_sync();
        /* the first pass also counts the bottom window: when every bin is in
         * it (minq <= 60 everywhere) it is the only pass */
        uint64_t rt = 0, rn = 0;
        uint32_t top = max(deep_pass<0>(a.reads_t + ot, nt, tb, th, cap, 0, DW_BINS, D.hist, rt),
                           deep_pass<0>(a.reads_n + on, nn, tb, th, cap, 0, DW_BINS, D.hist + 4 * DW_BINS, rn));
        top = wave_max(top);
        atomicAdd(&D.rms[0], (unsigned long long)rt);
        atomicAdd(&D.rms[1], (unsigned long long)rn);
        float acc = 0.0f;
        uint32_t w0 = 0, w1 = 0, cnt = 0;
        bool counted = top <= DW_BINS;
        for (uint32_t hi = top; hi > 0u;) {            /* windows, top down (wave-uniform) */
            const uint32_t lo = hi > DW_BINS ? hi - DW_BINS : 0u;
            if (!counted) {
                wave_sync();
                deep_zero(D.hist);
                wave_sync();
                uint64_t unused = 0;
                deep_pass<1>(a.reads_t + ot, nt, tb, th, cap, lo, hi, D.hist, unused);
                deep_pass<1>(a.reads_n + on, nn, tb, th, cap, lo, hi, D.hist + 4 * DW_BINS, unused);
            }
            counted = false;
            wave_sync();
            for (uint32_t wd = lane; wd < DW_OCC; wd += 64u) {
                const uint4 *h4 = reinterpret_cast<const uint4 *>(D.hist + wd * 32u);
                uint32_t bits = 0;
#pragma unroll
                for (uint32_t j = 0; j < 8u; ++j) {
                    const uint4 h = h4[j];
                    bits |= (h.x != 0u ? 1u : 0u) << (4u * j) | (h.y != 0u ? 2u : 0u) << (4u * j) |
                            (h.z != 0u ? 4u : 0u) << (4u * j) | (h.w != 0u ? 8u : 0u) << (4u * j);
                }
                D.occ[wd] = bits;
            }
            wave_sync();
            if (lane < 16u) deep_fold(D.hist, D.occ, grp * DW_BINS, lo, hi, fk, lane & 1u, acc, w0, w1, cnt);
            wave_sync();
            hi = lo;
        }
        /* lanes 0..3 finish the tumor, 4..7 the normal (quad-cooperative) */
        const uint32_t smp = (lane >> 2) & 1u;
        float es[4], fs[4];
        uint32_t c[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int src = (int)(smp * 8u + 2u * (uint32_t)b);
            es[b] = __shfl(acc, src);
            fs[b] = __shfl(acc, src + 1);
            c[b] = (uint32_t)__shfl((int)cnt, src);
        }
        const uint32_t n = smp ? nn : nt;
        const uint64_t rms = D.rms[smp];
        uint32_t lk[10], min_lk, rms_q, cns;
        glf_and_cns((int)(lane & 3u), es, fs, c, n, rms, a.m, lk, min_lk, rms_q, cns);
        if (lane == 0u || lane == 4u) {
            SlotRes &r = D.res[smp];
#pragma unroll
            for (int g = 0; g < 10; ++g) r.lk[g] = (uint8_t)lk[g];
            r.cns = cns;
            r.depth = n > 16777215u ? 16777215u : n;
            r.min_lk = (uint8_t)min_lk;
            r.rms_q = (uint8_t)rms_q;
            if (a.glf) store_glf(&a.glf[2ull * s + smp], ref16, lk, min_lk, rms_q, r.depth);
        }
        wave_sync();
        if (lane == 0u) decide_site(a, s, refc | ref16 << 8, D.res[0], D.res[1]);
        wave_sync();
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
int ss_launch_score(const ss_score_args &a, int main_grid, int wide_grid, int deep_grid, hipStream_t s,
                    const hipEvent_t *ev)
{
    hipError_t e;
    if (ev) (void)hipEventRecord(ev[0], s);
    hipLaunchKernelGGL(ss_score_main, dim3(main_grid), dim3(SS_MAIN_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    if (ev) (void)hipEventRecord(ev[1], s);
    hipLaunchKernelGGL(ss_score_wide, dim3(wide_grid), dim3(SS_WIDE_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    if (ev) (void)hipEventRecord(ev[2], s);
    hipLaunchKernelGGL(ss_score_deep, dim3(deep_grid), dim3(SS_DEEP_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    if (ev) (void)hipEventRecord(ev[3], s);
    return (int)hipSuccess;
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

#if SS_STAMP
/* diagnostic builds: per-phase cycle totals of ss_score_main (summed over
 * waves), then reset.  Phases: 0 wait for the staged reads, 1 phase A loop
 * remainder, 2 next sub-group, 3 fold, 4 glf finish + stores, 5 decision,
 * 6 prologue, 7 key build, 8 sort network, 9 group counts, 10 record
 * write-back + rms, 11 DMA issue, 12 genotype likelihoods. */
extern "C" __attribute__((visibility("default"))) int ss_debug_stamps(unsigned long long *out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ss_stamp_acc), sizeof(unsigned long long) * SS_NSTAMP) != hipSuccess)
        return -1;
    static const unsigned long long zero[SS_NSTAMP] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(ss_stamp_acc), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
#endif
