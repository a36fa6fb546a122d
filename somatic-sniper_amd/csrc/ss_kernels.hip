/*
 * ss_kernels.hip -- CDNA4 (gfx950) kernels of the somatic site scorer.
 *
 * One pileup site = one call of the reference's glf_somatic
 * (src/lib/sniper/somatic_sniper.c:109-273): two MAQ genotype-likelihood
 * evaluations (sniper_maqcns_glfgen, sniper_maqcns.c:127-248), two consensus
 * calls (sniper_glf2cns, :250-273) and the Phred-space somatic posterior.
 *
 * Work decomposition, one launch = three kernels in order:
 *   ss_score_main   one LANE per site: a wave walks blocks of 64 consecutive
 *     sites (grid-strided).  Per lane: the site's packed reads (x4 loads into
 *     registers) become 16-bit order keys in a 128-element bitonic network in
 *     registers (two keys per VGPR, packed min / max), the sorted keys become
 *     8-bit fold records in LDS, then the ordered esum / fsum fold (the
 *     reference's float accumulators fed double increments,
 *     sniper_maqcns.c:162-172), the 10 genotype likelihoods, glf2cns and the
 *     site decision (gate, SNV candidate test, posteriors / joint prior, emit
 *     filter), all inside the lane.  Sites past the network (> 128 reads in a
 *     sample), with a read of minq >= 64 or malformed offsets are listed.
 *   ss_score_group  the listed sites with at most 2048 reads per sample: per
 *     (site, sample) a unit of 1..16 lanes sorts 128 keys per lane as above
 *     and merges across lanes (DPP); the records go to a per-wave buffer
 *     in HBM / L2, and a chunk of 32 sites is folded one lane per (site,
 *     sample) and finished together; 12 waves per CU.
 *   ss_score_deep   one wave per site beyond that (any depth), with a wild
 *     read or malformed offsets: counting sort of the order-relevant key
 *     fields in LDS windows, then the same ordered fold, likelihood and
 *     decision code.
 *
 * Bit-exactness: built with -ffp-contract=off (no FMA contraction); float
 * division and double sqrt are correctly rounded (sqrt re-checked with fma);
 * accumulation order equals the reference's descending-key order.
 */
#include <cstdio>

#include "ss_kernels.h"

#define SENT 0xffffffffu

/* Fixed tuning of the shipped kernels (each measured on MI355X):
 * one code path per choice, no run-time or build-time alternatives. */
namespace {

/* --------------------------------------------------------------------------
 * small helpers
 * ------------------------------------------------------------------------ */
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

/* the lane index recomputed where it is used (volatile, so not hoisted out
 * of a loop and kept live across it: in the group kernel such copies spilled) */
__device__ __forceinline__ uint32_t lane_id_here()
{
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

/* List appends staged per wave in a register (lanes [0, n) of `held` hold
 * the staged entries, n wave-uniform) and published 64 entries per atomic,
 * the rest once per workgroup at its end (stage_wg_flush): returning atomics
 * on one address serialise at about 11 ns each on MI355X
 * (tools/atomic_probe.hip), so one per wave per 64-site block cost the
 * triage kernel 0.19 ms per launch at 500x. */
__device__ __forceinline__ void stage_push(uint32_t &held, uint32_t &n, bool need, uint32_t val, uint32_t *cnt,
                                           uint32_t *lst, uint32_t lane)
{
    const uint64_t m = __ballot(need);
    if (!m) return;
    const uint32_t c = (uint32_t)__popcll(m);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    /* a permutation of the lanes: the entries to lanes n, n + 1, .. (mod 64)
     * in lane order, every other lane after them */
    const uint32_t rank = need ? below : c + (lane - below);
    const uint32_t p = (uint32_t)__builtin_amdgcn_ds_permute((int)(((n + rank) & 63u) << 2), (int)val);
    if (n + c < 64u) {
        held = lane >= n && lane < n + c ? p : held;
        n += c;
    } else {
        const uint32_t full = lane >= n ? p : held;
        uint32_t base = 0;
        if (lane == 0u) base = atomicAdd(cnt, 64u);
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
        lst[base + lane] = full;
        n = n + c - 64u;                                 /* lanes [0, n) received the rest */
        held = p;
    }
}

/* every wave's staged entries, one atomic for the workgroup; scratch: LDS of
 * 2 + 64 * waves words no wave uses any more */
__device__ __forceinline__ void stage_wg_flush(uint32_t held, uint32_t n, uint32_t *cnt, uint32_t *lst,
                                               uint32_t *scratch, uint32_t lane)
{
    __syncthreads();
    if (threadIdx.x == 0u) scratch[0] = 0u;
    __syncthreads();
    uint32_t off = 0;
    if (lane == 0u && n != 0u) off = atomicAdd(&scratch[0], n);
    off = (uint32_t)__builtin_amdgcn_readfirstlane((int)off);
    if (lane < n) scratch[2u + off + lane] = held;
    __syncthreads();
    const uint32_t total = scratch[0];
    if (total == 0u) return;                             /* workgroup-uniform */
    if (threadIdx.x == 0u) scratch[1] = atomicAdd(cnt, total);
    __syncthreads();
    const uint32_t base = scratch[1];
    for (uint32_t i = threadIdx.x; i < total; i += blockDim.x) lst[base + i] = scratch[2u + i];
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

/* clamp_bar_e without the IEEE division in the common case: e / f <= 63 (e
 * sums fk * q, f the same fk, q <= 63) and e * rcp(f) lies within a few ulp
 * (< 2^-16) of the correctly rounded quotient, so floor(q + 0.5) is exact
 * unless q + 0.5 falls within 2^-12 of an integer; those lanes (rare) take
 * the exact division in a wave-uniform branch.  Callers pass f > 0 (a
 * genotype without other reads passes 1: its index is unused). */
__device__ __forceinline__ int bar_e_fast(float e, float f)
{
    const float r = e * __builtin_amdgcn_rcpf(f) + 0.5f;
    const float fr = __builtin_amdgcn_fractf(r);
    /* near an integer (fr < 2^-12 or > 1 - 2^-12) as one compare whose lane
     * mask is the ballot itself (a ballot of an OR of two compares went
     * through a VGPR and back); at the band's edges either path is exact */
    const float d = __builtin_fabsf(fr - 0.5f);
    int be = (int)__builtin_floorf(r);
    if (__ballot(d > 0.5f - 0x1p-12f)) {
        if (d > 0.5f - 0x1p-12f) be = (int)((double)(e / f) + 0.5);
    }
    be = be < 4 ? 4 : be;
    return be > 63 ? 63 : be;
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
        /* the reference's layout and index, kept on the device: rescaled
         * counts can sum to 256, and tot << 8 is then bit 16, which the OR
         * merges into bar_e << 16 (sniper_maqcns.c:195,206): an odd bar_e
         * keeps its row, an even one reads row bar_e + 1, both at n = 0 (a
         * row sniper_cal_coef leaves zero); bar_e = 63 stays in the table.
         * (A transposed, q-minor copy measured no faster and broke that
         * aliasing.) */
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
                                             float *out)
{
    float ev[T1];
    uint32_t c2v[T1];
    bool homv[T1];
    double lhv[T1], cfv[T1];
#pragma unroll
    for (int t = T0; t < T1; ++t) {
        int j, k;
        geno_jk((int)role * 5 + t, j, k);
        /* the reference's sums start at 0.0f: 0.0f + x == x for these x >= +0 */
        float e = 0.0f, f = 0.0f;
        uint32_t c2 = 0;
        bool first = true;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i == j || i == k) continue;              /* compile-time */
            e = first ? es[i] : e + es[i];
            f = first ? fs[i] : f + fs[i];
            c2 += c[i];
            first = false;
        }
        const bool hom = j == k;
        const uint32_t il = hom ? 0u : (c[j] << 8 | c[k]);
        /* bar_e for every lane, no branch on c2; a lane with c2 = 0 (f = 0,
         * its index unused) divides by 1 instead, so no inf / NaN reaches the
         * float-to-int conversion (undefined in C++, poison in LLVM) */
        const uint32_t be = (uint32_t)bar_e_fast(e, c2 ? f : 1.0f);
        const uint32_t ic = c2 ? (be << 16 | tot << 8 | c2) : 0u;
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
template <typename TT>
__device__ __forceinline__ int qadd(const TT *T, int x, int y, int &clamped)
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
template <typename TT>
__device__ void decide_site(const ss_score_args &a, const TT *QT, uint32_t site, uint32_t refc,
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
                marg = qadd(QT, marg, v, clamped);
            }
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            int v = (int)rn.lk[j] + (int)rt.lk[j] + ss_tab_jprior(m)[(rb4 * 10 + j) * 10 + j];
            if (v > 255) v = 255;
            const int l = v - marg;
            qps = qadd(QT, qps, l, clamped);
            if (j != bj) jcq = qadd(QT, jcq, l, clamped);  /* stale-index quirk, :196 */
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
            st = qadd(QT, xt, st, clamped);
            sn = qadd(QT, xn, sn, clamped);
        }
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            int vt = (int)rt.lk[j] + ss_tab_prior(m)[rb4 * 10 + j] - st;
            int vn = (int)rn.lk[j] + ss_tab_prior(m)[rb4 * 10 + j] - sn;
            if (vt > 255) vt = 255;
            if (vn > 255) vn = 255;
            qps = qadd(QT, qps, vt + vn, clamped);
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
 * Shared machinery of the lane-group kernel (sites past the main kernel's
 * per-lane network): 8-bit fold records, packed u16 min / max,
 * cross-lane exchanges, the one-lane ordered fold and the chunk finish
 * (likelihoods, quantisation, decision).
 *
 * 16-bit order key of a read (ln_chunk builds it):
 *   sample<<15 | base<<13 | minq<<5 | hasbase<<4 | strand<<3 | E<<1 | nz
 * E = baseQ >> 6 and nz = (baseQ & 0x3f) != 0 order the reads of one
 * (minq < 4, hasbase, strand) class exactly as the reference's baseQ
 * tie-break does as far as the clamp of sniper_maqcns.c:165 is concerned.
 * Inside one (sample, base) group the reference's descending key walk
 * (sniper_maqcns.c:157-172) visits elements in exactly this order up to swaps
 * of elements with identical (q, strand), which leave every float sum
 * unchanged.
 * ------------------------------------------------------------------------ */
#define GB 32               /* sites per group-kernel chunk (one fold lane per (site, sample)) */

struct Slot3 {
    uint32_t rec_n;      /* first record byte (17 bits) | non-deleted depth << 17 */
    uint32_t cnt01;      /* cnt[0] | cnt[1] << 16 */
    uint32_t cnt23;      /* cnt[2] | cnt[3] << 16 */
    uint32_t rms;        /* sum of min(mapQ & 0x7f, cap)^2 */
};


/* per-site base tables of the deep kernel's bins (bam_nt16_nt4_table semantics,
 * sniper_maqcns.c:19,153-154: single-base codes -> 0..3 with hasbase, every
 * other code counts as A without hasbase; code 0 '=' -> the reference base). */
__device__ __forceinline__ void nt_tables(uint32_t ref16, uint32_t &tb, uint32_t &th)
{
    constexpr uint32_t TB = 1u << 4 | 2u << 8 | 3u << 16;     /* C=2 -> 1, G=4 -> 2, T=8 -> 3 */
    constexpr uint32_t TH = 1u << 2 | 1u << 4 | 1u << 8 | 1u << 16;
    tb = TB | ((TB >> (2u * ref16)) & 3u);
    th = TH | ((TH >> (2u * ref16)) & 1u);
}

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

/* Fold of one (site, sample) by one lane: esum and fsum (sniper_maqcns.c:
 * 165-172) as two float accumulators fed double increments,
 *   e = (float)((double)e + fk[w] * q),  f = (float)((double)f + fk[w]),
 * in the reference's order, so each is bit-identical to the reference's.  The
 * two per-strand w counters live in one register (16-bit fields, counting in
 * units of 8 = the byte stride of fk), selected by the record's strand<<4
 * field and saturated at w = 255 (:170).  Base groups are walked longest
 * first, so the wave-wide trip count is set by one long chain per lane.
 *
 * The records lie in the wave's global buffer (L2): a chain is walked from
 * its top in blocks of 16 records, each block five dwords (one unaligned
 * 16-byte window) loaded two blocks ahead, four records per step through
 * v_alignbyte as in the main kernel's fold.  A step past the chain's end
 * reads fk's zero entry (x + 0.0 == x). */
#define GP_FK_ZERO 256

/* the five dwords that hold records top - 16 .. top - 1 (buffer positions;
 * top - 16 may lie before the buffer's start, inside its pad) */
__device__ __forceinline__ void gp_block(const uint8_t *buf, int top, uint32_t (&w)[5])
{
    const uint32_t *p = reinterpret_cast<const uint32_t *>(buf + ((top - 16) & ~3));
#pragma unroll
    for (int q = 0; q < 5; ++q) w[q] = p[q];
}

/* four steps of a chain from the window R of records k0 - 3 .. k0 (k0 in the
 * top byte); steps j >= m read fk's zero entry */
template <bool TAIL>
__device__ __forceinline__ void gp_steps(const char *fkb, uint32_t R, int m, uint32_t &W, float &e, float &f)
{
    double t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t r = R >> (24 - 8 * j);                      /* record k0 - j in the low byte */
        const uint32_t sh = (r >> 2) & 16u;                        /* strand << 4 */
        uint32_t w8 = __builtin_amdgcn_ubfe(W, sh, 16u);
        w8 = w8 < 2040u ? w8 : 2040u;
        if (TAIL) w8 = j < m ? w8 : 8u * GP_FK_ZERO;
        W += 8u << sh;
        t[j] = *reinterpret_cast<const double *>(fkb + w8);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t q = (R >> (24 - 8 * j)) & 63u;
        e = (float)((double)e + t[j] * (double)q);
        f = (float)((double)f + t[j]);
    }
}

/* the 16 records below top in four steps (m: how many of them belong to the
 * chain); steps that no lane of the wave needs are skipped */
template <bool TAIL>
__device__ __forceinline__ void gp_block_steps(const char *fkb, const uint32_t (&w)[5], int top, int m,
                                               uint32_t &W, float &e, float &f)
{
    const uint32_t q = (uint32_t)(top - 16) & 3u;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if (TAIL && !__ballot(m > 4 * s)) break;
        gp_steps<TAIL>(fkb, __builtin_amdgcn_alignbyte(w[4 - s], w[3 - s], q), m - 4 * s, W, e, f);
    }
}

/* chain of records [s0, s0 + n) of the buffer, from the top; w holds the
 * block below s0 + n (loaded by the caller) */
__device__ __forceinline__ void gp_chain(const uint8_t *buf, uint32_t s0, uint32_t n, uint32_t (&w)[5],
                                         const char *fkb, float &e, float &f)
{
    e = 0.0f;
    f = 0.0f;
    uint32_t W = 0;
    if (__ballot(n >= 16u)) {
        /* whole blocks while any lane has 16 records left, the next two
         * blocks in flight; a lane with fewer keeps its state and its window
         * (which then holds its last, partial block) by selects */
        uint32_t wn[5];
        gp_block(buf, max((int)(s0 + n) - 16, 0), wn);
        for (uint32_t i = 0; __ballot(i + 16u <= n); i += 16u) {
            const bool act = i + 16u <= n;
            const int top = (int)(s0 + n) - (int)i;
            uint32_t wnn[5];
            gp_block(buf, max(top - 32, 0), wnn);
            float e2 = e, f2 = f;
            uint32_t W2 = W;
            gp_block_steps<false>(fkb, w, top, 16, W2, e2, f2);
            e = act ? e2 : e;
            f = act ? f2 : f;
            W = act ? W2 : W;
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                w[q] = act ? wn[q] : w[q];
                wn[q] = act ? wnn[q] : wn[q];
            }
        }
    }
    /* the lane's last 0 .. 15 records (below its whole blocks): window w */
    const uint32_t m = n & 15u;
    if (__ballot(m > 0u)) {
        if (m > 0u) gp_block_steps<true>(fkb, w, (int)(s0 + m), (int)m, W, e, f);
    }
}

__device__ __forceinline__ void fold_sample(const uint8_t *buf, uint32_t s0, const uint32_t cnt[4],
                                            const double *fk, float es[4], float fs[4])
{
    const uint32_t start1 = s0 + cnt[0], start2 = start1 + cnt[1], start3 = start2 + cnt[2];
    const char *fkb = reinterpret_cast<const char *>(fk);
    uint32_t L = 0;
#pragma unroll
    for (uint32_t b = 1; b < 4; ++b) L = cnt[b] > (L == 0 ? cnt[0] : (L == 1 ? cnt[1] : cnt[2])) ? b : L;
    /* the four chains in walking order (the largest first), and the top
     * block of each, all loaded up front */
    uint32_t sb[4], tb[4], bb[4];
    uint32_t w[4][5];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t b = i == 0 ? L : (i - 1u) + ((i - 1u) >= L ? 1u : 0u);
        bb[i] = b;
        sb[i] = b == 0 ? s0 : (b == 1 ? start1 : (b == 2 ? start2 : start3));
        tb[i] = b == 0 ? cnt[0] : (b == 1 ? cnt[1] : (b == 2 ? cnt[2] : cnt[3]));
        gp_block(buf, (int)(sb[i] + tb[i]), w[i]);
    }
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        float e, f;
        gp_chain(buf, sb[i], tb[i], w[i], fkb, e, f);
#pragma unroll
        for (uint32_t b2 = 0; b2 < 4; ++b2)
            if (b2 == bb[i]) { es[b2] = e; fs[b2] = f; }
    }
}

/* Maximum over the 64 lanes with DPP row shifts + row broadcasts, returned
 * wave-uniform (an SGPR): no LDS permute and no per-lane permute addresses
 * held in VGPRs across the main kernel's block loop.  Lanes whose DPP source
 * lies outside the row keep `old` = 0, the identity of an unsigned max. */
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false)); /* row_shr:1 */
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false)); /* row_shr:2 */
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false)); /* row_shr:4 */
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false)); /* row_shr:8 */
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false)); /* row_bcast:15 */
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false)); /* row_bcast:31 */
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

/* inclusive prefix sum over the 64 lanes (DPP row shifts, then row
 * broadcasts; lanes without a source add the `old` 0) */
__device__ __forceinline__ uint32_t wave_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false); /* row_shr:1 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false); /* row_shr:2 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false); /* row_shr:4 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false); /* row_shr:8 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); /* row_bcast:15 */
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); /* row_bcast:31 */
    return v;
}

/* Phases B, C, D for the G sites of a chunk: lane = slot (site * 2 + sample)
 * folds, evaluates the ten genotypes and quantises its sample; lane = site
 * decides.  Fold records are bytes of the wave's global buffer `recs` (slot
 * rec_n index). */
__device__ __forceinline__ void finish_sub(const ss_score_args &a, int G, const uint8_t *recs,
                                           const Slot3 *slot, SlotRes *res, const uint32_t *sites,
                                           const uint32_t *refcs, const double *fk, const int16_t *qtab)
{
    const uint32_t lane = lane_id_here();           /* slot addresses formed here */
    const uint32_t sl = lane;
    const bool act = sl < 2u * (uint32_t)G;
    float es[4], fs[4];
    uint32_t cnt[4], depth = 0, rms = 0;
    if (act) {
        const Slot3 &m3 = slot[sl];
        cnt[0] = m3.cnt01 & 0xffffu; cnt[1] = m3.cnt01 >> 16;
        cnt[2] = m3.cnt23 & 0xffffu; cnt[3] = m3.cnt23 >> 16;
        depth = m3.rec_n >> 17;
        rms = m3.rms;
        fold_sample(recs, m3.rec_n & 0x1ffffu, cnt, fk, es, fs);
    } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) { es[b] = fs[b] = 0.0f; cnt[b] = 0; }
    }
    uint32_t c[4];
    const uint32_t tot = rescale_counts(cnt, c);
    float p[10];
    geno_p5(0u, es, fs, c, tot, a.m, p);
    geno_p5(1u, es, fs, c, tot, a.m, p + 5);
    if (act) {
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
            const uint32_t s = sl >> 1;
            store_glf(&a.glf[2ull * sites[s] + (sl & 1u)], refcs[s] >> 8, lk, min_lk, rms_q, depth);
        }
    }
    wave_sync();
    /* the decision reads both samples' records straight from LDS */
    if ((int)lane < G) decide_site(a, qtab, sites[lane], refcs[lane], res[2 * lane], res[2 * lane + 1]);
    wave_sync();
}

}  // namespace

/* --------------------------------------------------------------------------
 * Main kernel: one LANE per site.
 *
 * A wave scores 64 consecutive sites -- lane l takes site l of its block --
 * and the blocks are grid-strided.  Everything per site runs inside its lane,
 * serially, so one VALU instruction advances 64 sites:
 *   1. key build: the site's packed reads (x4 loads straight into registers)
 *      become 16-bit order keys (see above) in a per-lane bitonic network of
 *      LN_N elements; the rms sums and the group sizes (contributing reads per
 *      (sample, base)) are accumulated on the way.
 *   2. sort: the network, in registers, two keys per register: every
 *      instruction is the compare-exchange of two element pairs
 *      (v_pk_min_u16 / v_pk_max_u16), no cross-lane traffic.
 *   3. records: sorted keys become 8-bit fold records (q | strand << 6) in
 *      LDS, dword-interleaved by lane, so every per-lane index is conflict-free.
 *   4. fold (sniper_maqcns.c:160-175): per sample, the chain of its largest
 *      base group, then the other three (usually empty or tiny), each in the
 *      reference's descending key order: float accumulators fed double
 *      increments, w counters per strand.
 *   5. likelihoods, homozygote fix, quantisation, glf2cns per sample
 *      (:176-273), then the site decision of glf_somatic (somatic_sniper.c).
 * When every site of the wave has at most LN_N sort slots (tumor rounded up to
 * 4, then normal) both samples share one network ("joint"); otherwise the
 * tumor, then the normal is sorted and folded on its own ("separate").  Sites
 * with more than LN_N reads in a sample, malformed offsets, or a contributing
 * read of minq >= 64 (the 8-bit record holds q < 64) are listed for the group
 * kernel (which hands the last two kinds on to the deep kernel).
 * ------------------------------------------------------------------------ */
namespace {

#define LN_N 128                     /* elements of the per-lane network          */
#define LN_R (LN_N / 2)              /* its packed registers                      */
#define LN_C (LN_N / 4)              /* 4-element chunks (one x4 load each)       */
#define LN_P 4                       /* chunk loads in flight ahead of the key build */
#define LN_WAVES (SS_MAIN_BLOCK / 64)
#ifndef SS_EARLY_MAX_READS
#define SS_EARLY_MAX_READS 256u      /* blocks of at most this mean (tumor + normal) reads per site take the early exit */
#endif

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));

struct LaneLds {
    union {
        /* fold record of element e, lane l: byte (e + 4) & 3 of rec[(e + 4) >> 2][l]; row 0 is a
         * pad and row LN_C + 1 is never used, so a chain reads any 4-record window with two rows */
        uint32_t rec[LN_C + 2][64];
        SlotRes res[64][2];          /* the two samples' results, for the decision */
    };
    uint32_t tres[5][64];            /* the tumor's results while the normal is sorted (registers) */
};

/* Network layout: register r holds element r in its low half and element
 * N - 1 - r, bit-complemented, in its high half.  A compare-exchange of
 * elements e < e' puts the minimum at e; for a pair of registers (r, r ^ m)
 * with r < r ^ m that is a min into r and a max into r ^ m in BOTH halves
 * (the complement turns the high halves' reversed order into the same
 * direction), so one v_pk_min_u16 + v_pk_max_u16 pair serves two element
 * pairs.  The only other stage, element r against N - 1 - r, stays inside
 * register r: min(lo, ~hi) to lo and its complement ~max to hi. */
__device__ __forceinline__ void ln_ce(uint32_t &lo, uint32_t &hi)
{
    const uint32_t mn = pk_min(lo, hi), mx = pk_max(lo, hi);
    lo = mn;
    hi = mx;
}

__device__ __forceinline__ uint32_t ln_ce_self(uint32_t x)
{
    return pk_min_swo(x, ~x);        /* (min(a, b), min(~b, ~a)) for x = (a, ~b) */
}

template <int R, int M>
__device__ __forceinline__ void ln_stage(uint32_t (&v)[R])
{
#pragma unroll
    for (int r = 0; r < R; ++r)
        if ((r ^ M) > r) ln_ce(v[r], v[r ^ M]);
}

template <int R, int J>
__device__ __forceinline__ void ln_clean(uint32_t (&v)[R])
{
    if constexpr (J >= 1) {
        ln_stage<R, J>(v);
        ln_clean<R, J / 2>(v);
    }
}

/* level K of the flip-form bitonic sort: mirror e <-> e ^ (K - 1), then the
 * half cleaners e <-> e ^ j, j = K/4 .. 1 (every comparator min-to-lower) */
template <int R, int K>
__device__ __forceinline__ void ln_levels(uint32_t (&v)[R])
{
    if constexpr (K <= 2 * R) {
        if constexpr (K == 2 * R) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = ln_ce_self(v[r]);
        } else {
            ln_stage<R, K - 1>(v);
        }
        ln_clean<R, K / 4>(v);
        ln_levels<R, 2 * K>(v);
    }
}

/* sorted element e (ascending) */
template <int R>
__device__ __forceinline__ uint32_t ln_elem(const uint32_t (&v)[R], int e)
{
    return e < R ? (v[e] & 0xffffu) : (~v[2 * R - 1 - e] >> 16);
}


/* Key-build lookup table (LDS, per workgroup), 8-byte entries: for a read's
 * nt16 code and strand, the site's reference code and the sample, .x the
 * ref-dependent part of its 16-bit order key (sample << 15 | base << 13 |
 * hasbase << 4 | strand << 3; bam_nt16_nt4_table semantics,
 * sniper_maqcns.c:19,153-154: single-base codes give their base with hasbase,
 * '=' the reference's, any other code counts as A without hasbase; bit 31 set
 * when that base is not the reference's, for the early exit) and .y the read's
 * group count increment (1 << 8 * base).  Entry 0 belongs to a
 * non-contributing read (clamped q = 0, or a pad): key 0xffff, no count.  Row
 * (sample, ref16) starts at byte 256 * (1 + sample * 16 + ref16) and a read
 * indexes it by (nt16 | strand << 4) * 8 = (read >> 13) & 0xf8, XOR-swizzled
 * by the row (ln_lut_row). */
#define LN_LUT_BYTES (256 * (1 + 2 * 16))

/* Rows are 256 B, i.e. exactly the 64 LDS banks, so the same entry of two rows
 * would sit in the same banks and lanes of different references / samples
 * reading it would conflict: entry k of row r is stored at k ^ (r & 31), and a
 * read's offset is (read >> 13 & 0xf8) ^ ln_lut_row(r) (one v_bitop3). */
__device__ __forceinline__ uint32_t ln_lut_row(uint32_t r)
{
    return 256u * r | (r & 31u) << 3;
}

__device__ __forceinline__ void ln_lut_build(uint2 *lut)
{
    for (uint32_t i = threadIdx.x; i < LN_LUT_BYTES / 8u; i += blockDim.x) {
        const uint32_t rw = i >> 5, smp = rw >= 17u ? 1u : 0u, ref16 = (rw - 1u) & 15u;
        const uint32_t nt16 = i & 15u, st = (i >> 4) & 1u;
        const uint32_t code = nt16 ? nt16 : ref16;
        const uint32_t nt4 = code == 1u ? 0u : code == 2u ? 1u : code == 4u ? 2u : code == 8u ? 3u : 4u;
        const uint32_t hb = nt4 < 4u ? 1u : 0u, base = hb ? nt4 : 0u;
        /* bit 31: the read's group is not the reference base's (the early
         * exit's count pass; the key build keeps the low 16 bits) */
        const uint32_t rcode = ref16 == 1u ? 0u : ref16 == 2u ? 1u : ref16 == 4u ? 2u : ref16 == 8u ? 3u : 0u;
        lut[(rw << 5) | ((i ^ rw) & 31u)] = rw == 0u ? make_uint2(0xffffu, 0u)
                          : make_uint2(smp << 15 | base << 13 | hb << 4 | st << 3 | (base != rcode ? 1u << 31 : 0u),
                                       1u << (8u * base));
    }
}

/* one pass of the key build: the lane's elements [0, na) are reads
 * ba[oa..oa+na), [na4, na4 + nb) reads bb[ob..ob+nb) (na4 = na rounded up to
 * 4, so a chunk of 4 elements comes from one sample), every other element is
 * a pad (0xffff).  la / lb: the samples' rows of the lookup table.  Returns
 * the per-sample rms sums and group sizes (four 8-bit fields, base b at 8b)
 * and the largest minq of any read (>= 64: the site needs 16-bit records).
 * Every x4 load stays inside the batch's reads (the caller routes a block that
 * would pass their end to the group kernel); elements past a sample's reads are
 * zeroed, which makes them non-contributing (key 0xffff, rms 0). */
struct LaneIn {
    const uint32_t *pa, *pb;         /* element e's read: pa + e (e < na4), pb + e (e >= na4) */
    uint32_t na, nb, na4;
    uint32_t nca, nab;               /* A's chunks (na4 / 4); na4 + nb */
    uint32_t la, lb;                 /* A's and B's lookup rows (ln_lut_row) */
    uint32_t clast;                  /* CLAMP loads: chunks past this one load it again */
    uint32_t cstep;                  /* STRIDE: words from one chunk of the lane to its next */
    uint32_t tail;                   /* wave-uniform (an SGPR, 0 / 1): an x4 load could pass the end of the reads */
};

/* a wave-uniform flag as an SGPR integer: branches on it stay scalar (a bool
 * kept across the chunk loads was re-materialised in a VGPR at every load) */
__device__ __forceinline__ uint32_t ln_uniform(bool b)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane(b ? 1 : 0);
}

struct LaneAcc {
    uint32_t rms_a, rms_b, cnt_a, cnt_b;
    uint32_t maxq;
};

/* the x4 load of chunk c (elements 4c .. 4c+3): A's reads below na4, then
 * B's.  Unconditional: a chunk past the lane's reads loads whatever follows
 * them in B's array (the caller makes sure that stays inside the batch's
 * reads; ln_chunk zeroes the words), so the load needs no branch, its offset
 * is the instruction's immediate and the loads in flight stay in fixed
 * registers.  In a tail block (the batch's last sites, or a batch of fewer
 * than 4 reads) the lane loads word by word, only its own reads. */
/* TM: 0 = test in.tail at every load, 1 = the caller knows it is 0, 2 = 1 */
template <bool CLAMP, bool STRIDE, int TM = 0>
__device__ __forceinline__ void ln_load(const LaneIn &in, uint32_t c, uint32_t (&x)[4])
{
    const bool fa = c < in.nca;
    const uint32_t cc = CLAMP ? min(c, in.clast) : c;
    const uint32_t *src = (fa ? in.pa : in.pb) + (STRIDE ? cc * in.cstep : 4u * cc);
    if (TM == 2 || (TM == 0 && in.tail)) {   /* wave-uniform: word loads, none past the lane's reads */
        const int lim = (int)(fa ? in.na : in.nab) - (int)(STRIDE ? c * in.cstep : 4u * c);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            x[t] = 0u;
            if (t < lim) x[t] = src[t];
        }
        return;
    }
    const u32x4_a4 q4 = *reinterpret_cast<const u32x4_a4 *>(src);
    x[0] = q4.x; x[1] = q4.y; x[2] = q4.z; x[3] = q4.w;
}

/* (x != 0) as 0 / 1 in one VALU op (the compiler's form is a compare and a select) */
__device__ __forceinline__ uint32_t ln_nz(uint32_t x)
{
    uint32_t r;
    asm("v_min_u32 %0, 1, %1" : "=v"(r) : "v"(x));
    return r;
}

/* keys of chunk c from its loaded words x; rms / group sizes into acc.
 * Elements past the sample's reads are masked to 0 (a non-contributing read);
 * a non-contributing read's lookup offset is multiplied by 0 (entry 0). */
template <bool STRIDE>
__device__ __forceinline__ void ln_chunk(const LaneIn &in, const uint2 *lut, uint32_t c, uint32_t cap,
                                         const uint32_t (&x)[4], uint32_t (&v)[LN_R], LaneAcc &acc)
{
    const uint32_t c4 = 4u * c;
    const bool fa = c < in.nca;
    const int lim = (int)(fa ? in.na : in.nab) - (int)(STRIDE ? c * in.cstep : c4);
    uint32_t valid, vl;                             /* bit t: element c4 + t is a read */
    asm("v_med3_i32 %0, %1, 0, 4" : "=v"(vl) : "v"(lim));
    asm("v_bfm_b32 %0, %1, 0" : "=v"(valid) : "v"(vl));
    const uint32_t row = fa ? in.la : in.lb;
    uint32_t rd[4], minq[4], lo6[4], y[4];
    uint2 ent[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {                 /* the four table reads go out together */
        uint32_t vm;                                /* 0 or ~0 (the compiler's form: compare + select) */
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(vm) : "v"(valid), "i"(t));
        rd[t] = x[t] & vm;
        asm("v_min_u32_sdwa %0, %1, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1"
            : "=v"(minq[t]) : "v"(rd[t]));                       /* min(mapQ, baseQ) in one op */
        lo6[t] = rd[t] & 0x3f00u;
        y[t] = rd[t] >> 13;
        /* contributing unless the clamped q is 0 (sniper_maqcns.c:165-167) */
        const uint32_t off = __umul24((y[t] & 0xf8u) ^ row, ln_nz(minq[t] | lo6[t]));
        ent[t] = *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(lut) + off);
    }
    uint32_t crms = 0, ccnt = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        acc.maxq = max(acc.maxq, minq[t]);
        /* E = baseQ >> 6 at bit 1, nz = (baseQ & 0x3f) != 0 at bit 0 */
        const uint32_t key = ent[t].x | minq[t] << 5 | (y[t] & 6u) | ln_nz(lo6[t]);   /* < 2^16 */
        ccnt += ent[t].y;
        const uint32_t e = c4 + (uint32_t)t;
        if (e < LN_R) v[e] = key & 0xffffu;                         /* high half 0: a pad, see below */
        else v[LN_N - 1 - e] |= (key ^ 0xffffu) << 16;
    }
    /* rms terms min(mapQ & 0x7f, cap)^2 two at a time: the mapQ bytes of two
     * reads in the halves of one register, clamped with v_pk_min_u16 and
     * squared + summed by v_dot2_u32_u16 */
#pragma unroll
    for (int t = 0; t < 4; t += 2) {
        uint32_t p = __builtin_amdgcn_perm(rd[t + 1], rd[t], 0x0c040c00u) & 0x007f007fu;
        p = pk_min(p, cap * 0x10001u);
        crms = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p), __builtin_bit_cast(u16x2_t, p), crms, false);
    }
    /* totals and A's share (B's = total - A's); crms < 2^24 */
    acc.rms_b += crms;
    asm("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc.rms_a) : "v"(fa ? 1u : 0u), "v"(crms));
    acc.cnt_b += ccnt;
    acc.cnt_a += fa ? ccnt : 0u;
}

template <bool CLAMP = false, bool STRIDE = false, int TM = 0>
__device__ __forceinline__ LaneAcc ln_keys(const LaneIn &in, const uint2 *lut, uint32_t nch, uint32_t cap,
                                           uint32_t (&v)[LN_R])
{
    LaneAcc acc = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < LN_R; ++r) v[r] = 0x0000ffffu;     /* pads: lo 0xffff, hi ~0xffff */
    /* groups of LN_P chunks, two buffers: group g + 1 is loaded while group g
     * is keyed (the loop unrolls fully: static buffer and v indices; skipped
     * groups are wave-uniform) */
    constexpr int NG = LN_C / LN_P;
    uint32_t buf[2][LN_P][4];
    if (nch > 0u) {
#pragma unroll
        for (int j = 0; j < LN_P; ++j) ln_load<CLAMP, STRIDE, TM>(in, (uint32_t)j, buf[0][j]);
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if ((uint32_t)(g * LN_P) >= nch) continue;
        if (g + 1 < NG && (uint32_t)((g + 1) * LN_P) < nch) {
#pragma unroll
            for (int j = 0; j < LN_P; ++j) ln_load<CLAMP, STRIDE, TM>(in, (uint32_t)((g + 1) * LN_P + j), buf[(g + 1) & 1][j]);
        }
#pragma unroll
        for (int j = 0; j < LN_P; ++j) ln_chunk<STRIDE>(in, lut, (uint32_t)(g * LN_P + j), cap, buf[g & 1][j], v, acc);
    }
    /* a high half never keyed stays 0: the complement of the pad key */
    acc.rms_b -= acc.rms_a;          /* totals -> B's share */
    acc.cnt_b -= acc.cnt_a;
    return acc;
}

/* The sorted registers become fold records in place, two per register:
 * register r's elements r (low half) and 127 - r (high half, complemented)
 * give records q | strand << 6 (| 1 << 7 with WIDE: the group fold's fsum
 * multiplier, key_to_rec8) in bytes 0 and 2, computed on both halves at once
 * (q = max(minq, nz << 2), sniper_maqcns.c:165, for minq < 64 -- sites with a
 * larger one are not scored from these records).  Registers whose elements
 * are all past nel are left alone (wave-uniform bound). */
template <bool WIDE>
__device__ __forceinline__ void ln_to_records(uint32_t (&v)[LN_R], uint32_t nel)
{
#pragma unroll
    for (int r = 0; r < LN_R; ++r) {
        if ((uint32_t)r >= nel && (uint32_t)(LN_N - 1 - r) >= nel) continue;
        const uint32_t x = v[r] ^ 0xffff0000u;                   /* both keys plain */
        const uint32_t q = pk_max((x >> 5) & 0x003f003fu, (x << 2) & 0x00040004u);
        v[r] = ((x << 3) & 0x00400040u) | q | (WIDE ? 0x00800080u : 0u);
    }
}

/* records of elements 4i .. 4i + 3 from the converted registers, one dword */
__device__ __forceinline__ uint32_t ln_rec_dword(const uint32_t (&v)[LN_R], int i)
{
    if (4 * i < LN_R) {              /* low halves of registers 4i .. 4i + 3 (byte 0 of each) */
        const uint32_t a = __builtin_amdgcn_perm(v[4 * i + 1], v[4 * i], 0x0c0c0400u);
        const uint32_t b = __builtin_amdgcn_perm(v[4 * i + 3], v[4 * i + 2], 0x04000c0cu);
        return a | b;
    }
    const int r0 = LN_N - 1 - 4 * i;  /* high halves of registers r0, r0 - 1, r0 - 2, r0 - 3 (byte 2) */
    const uint32_t a = __builtin_amdgcn_perm(v[r0 - 1], v[r0], 0x0c0c0602u);
    const uint32_t b = __builtin_amdgcn_perm(v[r0 - 3], v[r0 - 2], 0x06020c0cu);
    return a | b;
}

/* sorted elements [0, nel) as records into the lane's LDS column */
__device__ __forceinline__ void ln_records(uint32_t (&v)[LN_R], uint32_t nel, LaneLds &L, uint32_t lane)
{
    ln_to_records<false>(v, nel);
#pragma unroll
    for (int i = 0; i < LN_C; ++i) {
        if ((uint32_t)(4 * i) >= nel) continue;              /* wave-uniform */
        L.rec[i + 1][lane] = ln_rec_dword(v, i);
    }
}

/* the ordered chain of one (sample, base) group: records [s0, s0 + n),
 * walked from the top (sniper_maqcns.c:162-172), four records per step: their
 * window comes from two LDS rows (v_alignbyte), the four fk reads go out
 * together and only the float accumulations stay serial.  Past the chain's
 * end a read takes fk's zero entry (LN_FK_ZERO), which leaves e and f as they
 * are (x + 0.0 == x), so lanes of shorter chains need no mask. */
#define LN_FK_ZERO 256
/* fk entries the lane path can use: a chain holds at most LN_N = 128 records,
 * so w <= 127; the main kernel's LDS copy keeps entries 128 .. 256 zero, and a
 * lane that sits a step out reads from there (ln_chain) */
#define LN_FK_LIVE 128
static_assert(LN_FK_LIVE >= LN_N && 2 * LN_FK_LIVE <= LN_FK_ZERO,
              "a lane's counters (w < LN_N) must stay below the zeroed half, and w + LN_FK_LIVE inside the table");

/* four steps of a chain from the window R of records k0 - 3 .. k0; steps
 * j >= m (past the chain's end) read fk's zero entry */
template <bool TAIL>
__device__ __forceinline__ void ln_steps(const char *fkb, uint32_t R, uint32_t m, uint32_t inc, uint32_t &W, float &e,
                                         float &f)
{
    double t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t r = R >> (24 - 8 * j);                     /* record k0 - j in the low byte */
        const uint32_t sh = (r >> 2) & 16u;                       /* strand << 4 */
        uint32_t w8 = __builtin_amdgcn_ubfe(W, sh, 16u);
        if (TAIL) w8 = (uint32_t)j < m ? w8 : 8u * LN_FK_ZERO;
        W += inc << sh;
        t[j] = *reinterpret_cast<const double *>(fkb + w8);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t q = (R >> (24 - 8 * j)) & 63u;
        e = (float)((double)e + t[j] * (double)q);
        f = (float)((double)f + t[j]);
    }
}

/* window of records k0 - 3 .. k0 (k0 = s0 + n - 1 - i) at column byte k0 + 1 */
__device__ __forceinline__ uint32_t ln_window(const uint32_t *colw, uint32_t b)
{
    const uint32_t row = (b >> 2) * 64u;
    return __builtin_amdgcn_alignbyte(colw[row + 64u], colw[row], b & 3u);
}

__device__ __forceinline__ void ln_chain(const LaneLds &L, uint32_t lane, uint32_t s0, uint32_t n,
                                         const double *fk, float &e, float &f)
{
    const uint32_t *colw = &L.rec[0][lane];
    const char *fkb = reinterpret_cast<const char *>(fk);
    e = 0.0f;
    f = 0.0f;
    uint32_t W = 0;                  /* strand 0 count in bits 0..15, strand 1 in 16..31 (units of 8 B) */
    /* whole groups of four steps; a lane whose chain has fewer left computes
     * them on a harmless window without counting, its counters moved into
     * fk's zeroed upper half (w <= 127: entries 128 .. 255), so e and f stay
     * as they are (no exec mask: the masked form cost phi copies and exec
     * bookkeeping every step, 4.5% of the kernel) */
    const uint32_t zw = 8u * LN_FK_LIVE * 0x10001u;
    if (__ballot(n >= 4u)) {
        uint32_t i = 0;
        do {
            const bool act = i + 4u <= n;
            W = act ? W : W | zw;
            ln_steps<false>(fkb, ln_window(colw, act ? s0 + n - i : 3u), 4u, act ? 8u : 0u, W, e, f);
            i += 4u;
        } while (__ballot(i + 4u <= n));
        W &= ~zw;
    }
    /* the lane's last 1..3 steps */
    const uint32_t i = n & ~3u;
    if (__ballot(i < n))
        if (i < n) ln_steps<true>(fkb, ln_window(colw, s0 + n - i), n - i, 8u, W, e, f);
}

/* the three groups other than the lane's largest, walked together: one record
 * of each per step (their chains are usually 0 - 2 records, so this is one or
 * two steps where three chain loops cost a 4-record step each).  Record i of
 * a chain is byte (i + 4) & 3 of row (i + 4) >> 2 of the lane's column; past
 * its end a chain reads fk's zero entry. */
__device__ __forceinline__ void ln_chain3(const LaneLds &L, uint32_t lane, const uint32_t (&s0)[3],
                                          const uint32_t (&n)[3], const double *fk, float (&e)[3], float (&f)[3])
{
    const uint8_t *col = reinterpret_cast<const uint8_t *>(&L.rec[0][lane]);
    const char *fkb = reinterpret_cast<const char *>(fk);
    uint32_t W[3] = {0u, 0u, 0u};
    const uint32_t mx = max(max(n[0], n[1]), n[2]);
#pragma unroll
    for (int k = 0; k < 3; ++k) { e[k] = 0.0f; f[k] = 0.0f; }
    if (!__ballot(mx > 0u)) return;
    uint32_t i = 0;
    do {
        uint32_t r[3];
        double t[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const bool act = i < n[k];
            const uint32_t b = (act ? s0[k] + n[k] - 1u - i : 0u) + 4u;
            r[k] = col[(b >> 2) * 256u + (b & 3u)];
            const uint32_t sh = (r[k] >> 2) & 16u;
            const uint32_t w8 = __builtin_amdgcn_ubfe(W[k], sh, 16u);
            W[k] += 8u << sh;
            t[k] = *reinterpret_cast<const double *>(fkb + (act ? w8 : 8u * LN_FK_ZERO));
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            e[k] = (float)((double)e[k] + t[k] * (double)(r[k] & 63u));
            f[k] = (float)((double)f[k] + t[k]);
        }
        ++i;
    } while (__ballot(i < mx));
}

/* fold of one sample: group sizes cnt (8-bit fields), records from s0 */
__device__ __forceinline__ void ln_fold(const LaneLds &L, uint32_t lane, uint32_t s0, uint32_t cnt,
                                        const double *fk, float es[4], float fs[4], uint32_t c[4])
{
    uint32_t st[4];
    uint32_t big = 0, cb = 0, run = s0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        c[b] = (cnt >> (8 * b)) & 0xffu;
        st[b] = run;
        run += c[b];
        if (c[b] > cb) { cb = c[b]; big = (uint32_t)b; }
    }
    /* the largest group first (one long chain per lane), then the rest */
    float e, f;
    const uint32_t sbig = big == 0 ? st[0] : (big == 1 ? st[1] : (big == 2 ? st[2] : st[3]));
    ln_chain(L, lane, sbig, cb, fk, e, f);
    /* the other three together, unless one of them is long (a heterozygous
     * site: then chain by chain, four records per step) */
    const uint32_t o0 = big == 0u ? 1u : 0u, o1 = big <= 1u ? 2u : 1u, o2 = big <= 2u ? 3u : 2u;
    const uint32_t so[3] = {o0 == 0u ? st[0] : st[1], o1 == 1u ? st[1] : st[2], o2 == 2u ? st[2] : st[3]};
    const uint32_t no[3] = {o0 == 0u ? c[0] : c[1], o1 == 1u ? c[1] : c[2], o2 == 2u ? c[2] : c[3]};
    if (!__ballot(max(max(no[0], no[1]), no[2]) > 6u)) {
        float eo[3], fo[3];
        ln_chain3(L, lane, so, no, fk, eo, fo);
        es[0] = big == 0u ? e : eo[0];
        fs[0] = big == 0u ? f : fo[0];
        es[1] = big == 1u ? e : (big == 0u ? eo[0] : eo[1]);
        fs[1] = big == 1u ? f : (big == 0u ? fo[0] : fo[1]);
        es[2] = big == 2u ? e : (big <= 1u ? eo[1] : eo[2]);
        fs[2] = big == 2u ? f : (big <= 1u ? fo[1] : fo[2]);
        es[3] = big == 3u ? e : eo[2];
        fs[3] = big == 3u ? f : fo[2];
        return;
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        float eb, fb;
        const bool isbig = (uint32_t)b == big;
        ln_chain(L, lane, st[b], isbig ? 0u : c[b], fk, eb, fb);
        es[b] = isbig ? e : eb;
        fs[b] = isbig ? f : fb;
    }
}

/* likelihoods .. glf2cns of one sample into r (sniper_maqcns.c:176-273) */
__device__ __forceinline__ void ln_finish(const float es[4], const float fs[4], const uint32_t craw[4],
                                          uint32_t n, uint32_t rms, const ss_dev_model &m, uint32_t &lk03,
                                          uint32_t &lk47, uint32_t &lk89, uint32_t &cns, uint32_t &mq)
{
    uint32_t c[4];
    const uint32_t tot = rescale_counts(craw, c);
    float p[10];
    geno_p_range<0, 10>(0u, es, fs, c, tot, m, p);
    uint32_t lk[10], min_lk, rms_q;
    glf_finish(p, es, n, rms, m, lk, min_lk, rms_q, cns);
    lk03 = lk[0] | lk[1] << 8 | lk[2] << 16 | lk[3] << 24;
    lk47 = lk[4] | lk[5] << 8 | lk[6] << 16 | lk[7] << 24;
    lk89 = lk[8] | lk[9] << 8;
    mq = min_lk | rms_q << 8;
}

__device__ __forceinline__ void ln_store_res(SlotRes &r, uint32_t lk03, uint32_t lk47, uint32_t lk89, uint32_t cns,
                                             uint32_t n, uint32_t mq)
{
    uint32_t *w = reinterpret_cast<uint32_t *>(r.lk);
    w[0] = lk03;
    w[1] = lk47;
    w[2] = lk89;
    r.cns = cns;
    r.depth = n;
    r.min_lk = (uint8_t)(mq & 0xffu);
    r.rms_q = (uint8_t)(mq >> 8);
}

__device__ __forceinline__ void ln_store_glf(ss_glf_t *dst, uint32_t ref16, uint32_t lk03, uint32_t lk47, uint32_t lk89,
                                             uint32_t mq, uint32_t depth)
{
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    d[0] = (ref16 & 0xffu) | (mq >> 8 & 0xffu) << 8 | (lk03 & 0xffffu) << 16;
    d[1] = lk03 >> 16 | (lk47 & 0xffffu) << 16;
    d[2] = lk47 >> 16 | lk89 << 16;
    d[3] = mq & 0xffu;
    d[4] = depth;
}

}  // namespace

/* The kernel's arguments re-read from the kernarg segment where they are
 * used (the pointer is opaque to the compiler): the fields of the per-block
 * tail (decision, glf stores, list appends) then do not stay live in SGPRs
 * across the block loop, which spilled them to VGPR lanes. */
__device__ __forceinline__ const ss_score_args &kernarg_args()
{
    typedef const __attribute__((address_space(4))) ss_score_args *kptr;
    kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const ss_score_args *)p;
}

/* The lane path for one block of 64 sites, lane = site s (insite: a real
 * site): key build, sort, records, fold, likelihoods, decision; sites it does
 * not score are appended to the wave's segment of the group kernel's list
 * (ndeep: entries so far). */
__device__ __forceinline__ void ln_block(const ss_score_args &a, uint32_t s, bool insite, const uint2 *lut,
                                         const double *fk, const int16_t *qtab, LaneLds &L, uint32_t lane,
                                         uint32_t gw, uint32_t cap, uint32_t end_t, uint32_t end_n,
                                         uint32_t &ndeep)
{
    uint32_t ot = 0, ot1 = 0, on = 0, on1 = 0, refc = 'N';
    if (insite) {
        ot = a.off_t[s];
        ot1 = a.off_t[s + 1];
        on = a.off_n[s];
        on1 = a.off_n[s + 1];
        refc = a.ref[s];
    }
    const uint32_t ref16 = ss_tab_nt16(a.m)[refc];
    const uint32_t nt = ot1 - ot, nn = on1 - on;
    const bool formed = ot <= ot1 && ot1 <= end_t && on <= on1 && on1 <= end_n;
    bool ok = insite && formed && nt <= LN_N && nn <= LN_N;
    const uint32_t nt4 = (nt + 3u) & ~3u, nn4 = (nn + 3u) & ~3u;
    /* wave-uniform shape: joint when every ok site fits one network */
    /* a block whose x4 loads could pass the end of the batch's reads (its
     * last sites) loads word by word; so does a batch of fewer than 4
     * tumor reads (the x4 loads of read-less chunks go to reads_t[0..3]) */
    const bool tail = __ballot(ok && (ot + nt4 > end_t || on + nn4 > end_n)) || end_t < 4u;
    const bool joint = !__ballot(ok && nt4 + nn > LN_N);
    bool wild = false;
    uint32_t lkN03 = 0, lkN47 = 0, lkN89 = 0, cnsN = 0, mqN = 0;
    /* joint: one pass, both samples; separate: the tumor, then the normal */
    for (uint32_t pass = 0; pass < (joint ? 1u : 2u); ++pass) {
        LaneIn in;
        const bool nrm = pass == 1u;
        in.na = ok ? (nrm ? nn : nt) : 0u;
        in.na4 = ok ? (nrm ? nn4 : nt4) : 0u;
        in.nb = joint && ok ? nn : 0u;
        in.nca = in.na4 >> 2;
        /* opaque: otherwise the chunk tests c < nca become 4c < na4, whose
         * constants 68 .. 124 are not inline and took 16 SGPRs */
        asm("" : "+v"(in.nca));
        in.nab = in.na4 + in.nb;
        const uint32_t ob = ok ? on : 0u, oa = ok ? (nrm ? on : ot) : 0u;
        in.pa = (nrm ? a.reads_n : a.reads_t) + oa;
        /* chunks past A's reads: joint mode, the normal's reads; a pass of one
         * sample (no B part), the reads after A's in the same array -- the
         * next sites', which their lanes load anyway (the tumor pass used to
         * read the normal's reads here, loaded again by the normal pass) */
        const bool solo = !joint;
        in.pb = solo ? in.pa : a.reads_n + ob - in.na4;
        in.la = ln_lut_row(1u + (nrm ? 16u : 0u) + ref16);
        in.lb = ln_lut_row(17u + ref16);
        const uint32_t nch = wave_max((in.nab + 3u) >> 2);
        /* x4 loads reach pb + 4 nch: word loads if that could pass the end of the reads */
        in.tail = ln_uniform(tail || __ballot(solo ? (uint64_t)oa + 4u * nch > (uint64_t)(nrm ? end_n : end_t)
                                                   : (uint64_t)ob + 4u * nch > (uint64_t)end_n + in.na4));
        uint32_t v[LN_R];
        /* the tail test once per pass, not at every chunk load (the common
         * case has no word-load path at all) */
        LaneAcc acc;
        if (in.tail) acc = ln_keys<false, false, 2>(in, lut, nch, cap, v);
        else acc = ln_keys<false, false, 1>(in, lut, nch, cap, v);
        /* a read of minq >= 64 needs 16-bit records: the site goes to the group kernel */
        wild = wild || acc.maxq >= 64u;
        ln_levels<LN_R, 2>(v);
        ln_records(v, 4u * nch, L, lane);
        /* fold and finish the pass's samples: A (its records from 0), then
         * in joint mode B (after A's contributing reads) */
        const uint32_t ca = acc.cnt_a;
        const uint32_t tot_a = (ca & 0xffu) + (ca >> 8 & 0xffu) + (ca >> 16 & 0xffu) + (ca >> 24);
        for (uint32_t k = 0; k < (joint ? 2u : 1u); ++k) {
            const bool smpN = nrm || k == 1u;
            float es[4], fs[4];
            uint32_t c[4];
            ln_fold(L, lane, k ? tot_a : 0u, k ? acc.cnt_b : acc.cnt_a, fk, es, fs, c);
            uint32_t l03, l47, l89, cn, mq;
            ln_finish(es, fs, c, smpN ? nn : nt, k ? acc.rms_b : acc.rms_a, a.m, l03, l47, l89, cn, mq);
            if (smpN) {
                lkN03 = l03; lkN47 = l47; lkN89 = l89; cnsN = cn; mqN = mq;
            } else {
                L.tres[0][lane] = l03; L.tres[1][lane] = l47; L.tres[2][lane] = l89;
                L.tres[3][lane] = cn;  L.tres[4][lane] = mq;
            }
        }
        wave_sync();                                     /* the pass's records are read */
    }
    ok = ok && !wild;
    /* sites with a sample past SS_ROUTE_DEEP reads go straight to the deep
     * kernel's list (one atomic per wave), where its counting sort beats the
     * group kernel's network */
    const bool todeep = insite && !ok && formed && (nt > SS_ROUTE_DEEP || nn > SS_ROUTE_DEEP);
    const uint64_t dm = __ballot(todeep);
    if (dm) {
        const ss_score_args &k = kernarg_args();
        uint32_t d0 = 0;
        if (lane == (uint32_t)__builtin_ctzll(dm)) d0 = atomicAdd(k.deep2_count, (uint32_t)__popcll(dm));
        d0 = (uint32_t)__builtin_amdgcn_readlane((int)d0, (int)__builtin_ctzll(dm));
        if (todeep) {
            const uint32_t d = d0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
            if (d < k.deep_cap) k.deep2_list[d] = s;
            else atomicOr(k.err, SS_KERR_DEEP_OVERFLOW);
        }
    }
    /* the other sites the lane path does not score: the group kernel's list
     * (one segment per wave, no atomics) */
    const bool listed = insite && !ok && !todeep;
    const uint64_t out = __ballot(listed);
    if (out) {
        if (listed) {
            const uint32_t d = ndeep + __builtin_amdgcn_mbcnt_hi((uint32_t)(out >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)out, 0u));
            const ss_score_args &k = kernarg_args();
            if (d < k.deep_seg_cap) k.deep_list[(size_t)gw * k.deep_seg_cap + d] = s;
            else atomicOr(k.err, SS_KERR_DEEP_OVERFLOW);
        }
        ndeep += (uint32_t)__popcll(out);
    }
    if (!formed && insite) atomicOr(kernarg_args().err, SS_KERR_MALFORMED);
    const uint32_t dt = nt > 16777215u ? 16777215u : nt, dn = nn > 16777215u ? 16777215u : nn;
    const uint32_t lkT03 = L.tres[0][lane], lkT47 = L.tres[1][lane], lkT89 = L.tres[2][lane];
    const uint32_t cnsT = L.tres[3][lane], mqT = L.tres[4][lane];
    wave_sync();                                         /* res overlays the records */
    if (ok) {
        ln_store_res(L.res[lane][0], lkT03, lkT47, lkT89, cnsT, dt, mqT);
        ln_store_res(L.res[lane][1], lkN03, lkN47, lkN89, cnsN, dn, mqN);
        ss_glf_t *glf = kernarg_args().glf;
        if (glf) {
            ln_store_glf(&glf[2ull * s], ref16, lkT03, lkT47, lkT89, mqT, dt);
            ln_store_glf(&glf[2ull * s + 1], ref16, lkN03, lkN47, lkN89, mqN, dn);
        }
    }
    wave_sync();
    if (ok) decide_site(kernarg_args(), qtab, s, refc | ref16 << 8, L.res[lane][0], L.res[lane][1]);
    wave_sync();
}

/* The early exit's count pass (the triage kernel, round 6) reads a site's
 * reads with TG lanes: the site's joint element list -- the tumor's reads,
 * padded to 4, then the normal's -- in 4-read chunks, lane j of the site's
 * group taking chunks j, j + TG, ..., so one load instruction reads TG x 16
 * contiguous bytes of each of 64 / TG sites.  (Lane per site, every load
 * instruction touched 64 lines: the texture address and data units were busy
 * 83% / 94% of the kernel's cycles at C4) */
#ifndef TRI_P
#define TRI_P 4u                     /* chunk load instructions in flight per round */
#endif
#define SS_NEAR_SLOTS 4u             /* captured chunks per site: more means more than four off-reference reads */

/* per wave: a round's per-site totals and the sites' captured chunks */
struct TriLds {
    uint4    cap[64][SS_NEAR_SLOTS];         /* chunks with an off-reference read, element order */
    uint32_t capf[64];                       /* per slot (byte): its element flags | 16 for the normal's */
    uint32_t cnt_t[64], cnt_n[64];           /* contributing reads per group (8-bit fields) */
    uint32_t c24[64];                        /* contributing reads of minq >= 24: tumor | normal << 16 */
    uint32_t nfl[64];                        /* chunks captured (past SS_NEAR_SLOTS: some lost) */
};

/* one chunk of the count pass: per sample the contributing reads' group
 * counts and its reads of minq >= 24 (lim: elements of the chunk that are
 * reads); returns the element flags of the contributing reads whose group is
 * not the reference base's (the lookup table's bit 31) */
template <bool S1 = false>
__device__ __forceinline__ uint32_t tri_chunk(const uint2 *lut, const uint32_t (&x)[4], int lim, uint32_t row, bool fa,
                                              uint32_t &cnt_a, uint32_t &cnt_t, uint32_t &c24, uint32_t *c24s1 = nullptr)
{
    uint32_t valid, vl;
    asm("v_med3_i32 %0, %1, 0, 4" : "=v"(vl) : "v"(lim));
    asm("v_bfm_b32 %0, %1, 0" : "=v"(valid) : "v"(vl));
    uint32_t minq[4];
    uint2 ent[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        uint32_t vm;
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(vm) : "v"(valid), "i"(t));
        const uint32_t rd = x[t] & vm;
        asm("v_min_u32_sdwa %0, %1, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1"
            : "=v"(minq[t]) : "v"(rd));
        /* a non-contributing read (clamped q = 0) or a masked element reads entry 0: no count, no flag */
        const uint32_t off = __umul24(((rd >> 13) & 0xf8u) ^ row, ln_nz(minq[t] | (rd & 0x3f00u)));
        ent[t] = *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(lut) + off);
    }
    uint32_t cc = 0, q = 0, q1 = 0, fl = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        cc += ent[t].y;
        q += minq[t] >= 24u ? 1u : 0u;             /* minq >= 24: contributing */
        if (S1) q1 += minq[t] >= 24u ? (x[t] >> 20) & 1u : 0u;   /* of them on strand 1 (masked: minq 0) */
        fl |= (ent[t].x >> 31) << t;
    }
    cnt_t += cc;
    cnt_a += fa ? cc : 0u;
    c24 += fa ? q : q << 16;
    if (S1) *c24s1 += fa ? q1 : q1 << 16;
    return fl;
}

/* sum over the TG = 4 or 8 lanes of a site's group (DPP: quad_perm xor 1,
 * xor 2, then for 8 row_half_mirror, which pairs lane i with 7 - i of the
 * other quad) */
__device__ __forceinline__ uint32_t tri_gsum(uint32_t lg, uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false);    /* quad_perm [1,0,3,2] */
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);    /* quad_perm [2,3,0,1] */
    if (lg == 3u) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);   /* row_half_mirror */
    return v;
}

#define SS_NEAR_K 3u                 /* non-reference contributing reads per sample the early exit evaluates */

__device__ __forceinline__ uint32_t ln_ffbl(uint32_t x)
{
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ uint32_t ln_sel4(const uint32_t (&v)[4], uint32_t i)
{
    return i == 0u ? v[0] : i == 1u ? v[1] : i == 2u ? v[2] : v[3];
}
__device__ __forceinline__ float ln_sel4f(const float (&v)[4], uint32_t i)
{
    return i == 0u ? v[0] : i == 1u ? v[1] : i == 2u ? v[2] : v[3];
}

__device__ __forceinline__ bool ln_near_eval(const float (&es)[4], const float (&fs)[4], const uint32_t (&craw)[4],
                                             float esr, uint32_t r, const ss_dev_model &m);

/* One sample of the early exit's near-reference test (see tri_block):
 * keys (descending after the sort) of its <= SS_NEAR_K non-reference
 * contributing reads, 0 = none; c its contributing reads per group (the
 * reference group's count included), c24 its contributing reads of
 * minq >= 24.  True when sniper_glf2cns (sniper_maqcns.c:250-273) is proven to
 * call the reference homozygote. */
__device__ __forceinline__ bool ln_near_sample(uint32_t (&k)[SS_NEAR_K], const uint32_t (&c)[4], uint32_t c24,
                                               uint32_t r, const ss_dev_model &m, const double *fk)
{
    static_assert(SS_NEAR_K == 3u, "the sort below is for three keys");
    {   /* descending */
        uint32_t a0 = max(k[0], k[1]), a1 = min(k[0], k[1]);
        const uint32_t b1 = max(a1, k[2]), b2 = min(a1, k[2]);
        k[0] = max(a0, b1);
        k[1] = min(a0, b1);
        k[2] = b2;
    }
    /* the non-reference groups' chains (sniper_maqcns.c:162-172): within a
     * group the keys are walked in descending order, w counts per strand */
    float es[4] = {0.0f, 0.0f, 0.0f, 0.0f}, fs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const char *fkb = reinterpret_cast<const char *>(fk);
    uint32_t c24nr = 0;
#pragma unroll
    for (uint32_t i = 0; i < SS_NEAR_K; ++i) {
        const uint32_t key = k[i];
        if (!__ballot(key != 0u)) break;
        const uint32_t x = (key >> 13) & 3u;
        const uint32_t minq = (key >> 5) & 0xffu;
        const uint32_t q = max(minq, (key & 1u) << 2);        /* sniper_maqcns.c:165 */
        uint32_t w = 0;
#pragma unroll
        for (uint32_t j = 0; j < i; ++j) w += ((k[j] ^ key) & 0x6008u) == 0u ? 1u : 0u;   /* same group, strand */
        const double fv = *reinterpret_cast<const double *>(fkb + 8u * (key ? w : (uint32_t)LN_FK_ZERO));
        const float e0 = ln_sel4f(es, x), f0 = ln_sel4f(fs, x);
        const float e1 = (float)((double)e0 + fv * (double)q);
        const float f1 = (float)((double)f0 + fv);
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b) {
            es[b] = b == x ? e1 : es[b];
            fs[b] = b == x ? f1 : fs[b];
        }
        c24nr += key && minq >= 24u ? 1u : 0u;
    }
    return ln_near_eval(es, fs, c, ss_tab_esr(m)[min(c24 - c24nr, SS_NEAR_MAXN)], r, m);
}

/* The genotype part of the near-reference test for one sample: es / fs the
 * non-reference groups' chains (the reference group's entries 0, unused),
 * craw its contributing reads per group, c24r the reference group's reads of
 * minq >= 24.  True when sniper_glf2cns (sniper_maqcns.c:250-273) is proven
 * to call the reference homozygote. */
__device__ __forceinline__ bool ln_near_eval(const float (&es)[4], const float (&fs)[4], const uint32_t (&craw)[4],
                                             float esr, uint32_t r, const ss_dev_model &m)
{
    /* the counts' rescale (:178-182), as rescale_counts: tot <= 256 after it */
    uint32_t c[4];
    uint32_t tot = craw[0] + craw[1] + craw[2] + craw[3];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = craw[j];
    if (__ballot(tot > 255u)) {
        if (tot > 255u) {
#pragma unroll
            for (int j = 0; j < 4; ++j) c[j] = (uint32_t)(int)(254.0 * (double)craw[j] / (double)(int)tot + 0.5);
            tot = c[0] + c[1] + c[2] + c[3];
        }
    }
    /* the genotypes with the reference base, as geno_p (:184-214): t = 3 the
     * homozygote, t < 3 the heterozygote with base x_t */
    float pv[4];
    uint32_t icv[4], ilv[4], c2v[4];
    float ev[4];
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t) {
        const uint32_t x = t < 3u ? t + (t >= r ? 1u : 0u) : r;
        float e = 0.0f, f = 0.0f;
        uint32_t c2 = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
            const bool use = i != r && i != x;
            e = use ? e + es[i] : e;
            f = use ? f + fs[i] : f;
            c2 += use ? c[i] : 0u;
        }
        const uint32_t be = (uint32_t)bar_e_fast(e, c2 ? f : 1.0f);
        icv[t] = c2 ? (be << 16 | tot << 8 | c2) : 0u;
        const uint32_t j0 = min(r, x), k0 = max(r, x);
        ilv[t] = t < 3u ? (ln_sel4(c, j0) << 8 | ln_sel4(c, k0)) : 0u;
        c2v[t] = c2;
        ev[t] = e;
    }
    double cf[4], lv[4];
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t) {
        cf[t] = ss_tab_coef(m)[icv[t]];
        lv[t] = ss_tab_lhet(m)[ilv[t]];
    }
    const float cmn = ss_tab_cmin(m)[tot];
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t) {
        float v;
        if (t == 3u) {
            v = c2v[t] ? (float)((double)ev[t] + cf[t]) : 0.0f;
        } else {
            const double lh = -4.343 * lv[t];
            v = c2v[t] ? (float)((lh + (double)ev[t]) + cf[t]) : (float)lh;
        }
        pv[t] = v < 0.0f ? 0.0f : v;
    }
    /* every genotype without the reference base has p >= esum[ref] + lh + coef
     * >= lb (ss_capi.hip near_tables), and esum[ref] > every other esum, so
     * the homozygote fix (:216-233) picks the reference homozygote's row and
     * leaves it (its p is the smallest diagonal by more than 1); those
     * genotypes then quantise above the reference homozygote */
    const float lb = esr + cmn;
    const float phr = pv[3];
    const float min_p = min(min(phr, pv[0]), min(pv[1], pv[2]));
    /* (bitwise: no short-circuit branches); the reference group keeps a
     * count after the rescale, so every genotype without it has tmp2 > 0 */
    bool ok = (esr > max(max(es[0], es[1]), max(es[2], es[3]))) & (lb - phr >= 3.0f) & (phr - min_p <= 250.0f) &
              (ln_sel4(c, r) > 0u);
    const int lhr = (int)((double)(phr - min_p) + 0.5);
#pragma unroll
    for (uint32_t t = 0; t < 3u; ++t) {
        const float d = pv[t] - min_p;
        const int sc = ((double)d > 255.0 ? 255 : (int)((double)d + 0.5)) + m.q_r_int;
        /* sniper_glf2cns takes the first minimum in genotype order: a
         * heterozygote (x, r) with x < r comes before the homozygote */
        ok = ok & (t < r ? sc > lhr : sc >= lhr);
    }
    return ok;
}

/* Early exit of the lane path (rounds 5-6), the triage
 * kernel's work for one block of 64 sites (lane = site): a count pass over
 * the sites' reads decides the sites whose result needs no full likelihood
 * computation and writes their score; the others are returned (false) and
 * listed for the main kernel.  Exact -- the reference's own outcome -- and
 * never taken when glf records are requested:
 *   - ref char 'N' or an empty sample: -1 (somatic_sniper.c:127);
 *   - a reference code of 15 other than 'N' ('n', ...): 255, never an SNV
 *     candidate (:156);
 *   - reference A/C/G/T, at most 128 reads per sample and at most SS_NEAR_K
 *     contributing reads per sample off the reference base (round 6; round 5
 *     took none): those reads are kept from the count pass and folded exactly,
 *     which gives each sample's four genotypes with the reference base exactly
 *     (their e sums skip the reference group, :188-208), and a lower bound for
 *     the six without it (ss_capi.hip near_tables).  When the bounds put the
 *     reference homozygote first in sniper_glf2cns in both samples, t1 == n1
 *     and the site scores 255 (:156).
 * Returns true when it wrote the site's score. */
__device__ __forceinline__ bool tri_block(const ss_score_args &a, const uint2 *lut, const double *fk, TriLds &T,
                                          uint32_t lane, uint32_t s, bool insite, uint32_t end_t, uint32_t end_n,
                                          uint32_t lg)
{
    uint32_t ot = 0, ot1 = 0, on = 0, on1 = 0, refc = 'N';
    if (insite) {
        ot = a.off_t[s];
        ot1 = a.off_t[s + 1];
        on = a.off_n[s];
        on1 = a.off_n[s + 1];
        refc = a.ref[s];
    }
    const uint32_t ref16 = ss_tab_nt16(a.m)[refc];
    const uint32_t nt = ot1 - ot, nn = on1 - on;
    const bool small = insite && ot <= ot1 && ot1 <= end_t && on <= on1 && on1 <= end_n && nt <= LN_N && nn <= LN_N;
    bool done = false;
    int32_t sc = 255;
    if (small && (refc == 'N' || nt == 0u || nn == 0u)) {
        done = true;
        sc = -1;
    } else if (small && ref16 == 15u) {
        done = true;
    }
    const bool acgt = ref16 == 1u || ref16 == 2u || ref16 == 4u || ref16 == 8u;
    const bool cand = small && !done && acgt;
    if (__ballot(cand)) {
        const uint32_t nt4 = (nt + 3u) & ~3u;
        /* word loads when a site's x4 loads could pass the end of the batch's reads */
        const uint32_t tm = ln_uniform(__ballot(cand && ((uint64_t)ot + nt4 > end_t ||
                                                         (uint64_t)on + ((nn + 3u) & ~3u) > end_n)) ||
                                       end_t < 4u || end_n < 4u);
        /* each round: TG lanes per site (group g = lane / TG takes site
         * round * 64 / TG + g), the site's description by ds_bpermute */
        const uint32_t TG = 1u << lg;                     /* lanes per site: 4 or 8 (wave-uniform) */
        const uint32_t j = lane & (TG - 1u);
        const uint32_t pk = cand ? (nt | nn << 8 | ref16 << 16) : 0u;    /* nt, nn <= 128 */
        /* TG rounds of 64 / TG sites each */
#pragma unroll 1
        for (uint32_t r = 0; r < TG; ++r) {
            const uint32_t site = r << (6u - lg) | lane >> lg;
            const int sa = (int)(site << 2);
            const uint32_t g_pk = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)pk);
            const uint32_t g_ot = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)ot);
            const uint32_t g_on = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)on);
            const uint32_t g_nt = g_pk & 0xffu, g_nn = (g_pk >> 8) & 0xffu, g_ref16 = (g_pk >> 16) & 0xfu;
            const uint32_t g_nt4 = (g_nt + 3u) & ~3u;
            const uint32_t g_nchk = g_pk ? (g_nt4 + g_nn + 3u) >> 2 : 0u;    /* the site's chunks (0: not a candidate) */
            const uint32_t K = wave_max((g_nchk + TG - 1u) >> lg);
            if (K == 0u) continue;
            const uint32_t la = ln_lut_row(1u + g_ref16), lb = ln_lut_row(17u + g_ref16);
            const uint32_t *pt = a.reads_t + g_ot, *pn = a.reads_n + g_on - g_nt4;
            uint32_t cnt_a = 0, cnt_t = 0, c24 = 0, gn = 0;
            /* TRI_P chunk instructions of the round in flight together (one
             * memory latency per TRI_P, not per chunk) */
#pragma unroll 1
            for (uint32_t kb = 0; kb < K; kb += TRI_P) {
            uint32_t xb[TRI_P][4];
#pragma unroll
            for (uint32_t u = 0; u < TRI_P; ++u) {
                const uint32_t c = (kb + u) * TG + j;
                const bool live = c < g_nchk;
                const bool fa = 4u * c < g_nt4;
                const uint32_t *src = (fa ? pt : pn) + 4u * c;
                const int lim = live ? (int)(fa ? g_nt : g_nt4 + g_nn) - (int)(4u * c) : 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) xb[u][t] = 0u;
                if (tm) {
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        if (t < lim) xb[u][t] = src[t];
                } else if (live) {
                    const u32x4_a4 q4 = *reinterpret_cast<const u32x4_a4 *>(src);
                    xb[u][0] = q4.x; xb[u][1] = q4.y; xb[u][2] = q4.z; xb[u][3] = q4.w;
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < TRI_P; ++u) {
                if (kb + u >= K) break;                          /* wave-uniform */
                const uint32_t c = (kb + u) * TG + j;
                const bool live = c < g_nchk;
                const bool fa = 4u * c < g_nt4;
                const int lim = live ? (int)(fa ? g_nt : g_nt4 + g_nn) - (int)(4u * c) : 0;
                const uint32_t (&x)[4] = xb[u];
                const uint32_t fl = tri_chunk(lut, x, lim, fa ? la : lb, fa, cnt_a, cnt_t, c24);
                /* a chunk with an off-reference read: kept for its site, in
                 * element order (slot = the group's earlier chunks) */
                const uint64_t bal = __ballot(fl != 0u);
                if (bal) {
                    const uint32_t gb = (uint32_t)(bal >> (lane & ~(TG - 1u))) & ((1u << TG) - 1u);
                    const uint32_t slot = gn + (uint32_t)__popc(gb & ((1u << j) - 1u));
                    if (fl != 0u && slot < SS_NEAR_SLOTS) {
                        T.cap[site][slot] = make_uint4(x[0], x[1], x[2], x[3]);
                        reinterpret_cast<uint8_t *>(&T.capf[site])[slot] = (uint8_t)(fl | (fa ? 0u : 16u));
                    }
                    gn += (uint32_t)__popc(gb);
                }
            }
            }
            cnt_a = tri_gsum(lg, cnt_a);
            cnt_t = tri_gsum(lg, cnt_t);
            c24 = tri_gsum(lg, c24);
            if (j == 0u) {
                T.cnt_t[site] = cnt_a;
                T.cnt_n[site] = cnt_t - cnt_a;
                T.c24[site] = c24;
                T.nfl[site] = gn;
            }
        }
        wave_sync();
        /* lane = site again */
        uint32_t cnt_T = 0, cnt_N = 0, c24s = 0, nflc = 0, cf = 0;
        if (cand) {
            cnt_T = T.cnt_t[lane];
            cnt_N = T.cnt_n[lane];
            c24s = T.c24[lane];
            nflc = T.nfl[lane];
            cf = T.capf[lane];
        }
        const uint32_t r = (uint32_t)__builtin_ctz(ref16 | 16u);     /* the reference base (0..3 for cand) */
        uint32_t ca[4], cb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ca[i] = (cnt_T >> (8 * i)) & 0xffu;
            cb[i] = (cnt_N >> (8 * i)) & 0xffu;
        }
        const uint32_t ma = ca[0] + ca[1] + ca[2] + ca[3] - ln_sel4(ca, r);
        const uint32_t mb = cb[0] + cb[1] + cb[2] + cb[3] - ln_sel4(cb, r);
        /* the captured slots' flags (4 bits per slot) and samples */
        const uint32_t nv = min(nflc, SS_NEAR_SLOTS);
        uint32_t fl_all = (cf & 0xfu) | ((cf >> 8) & 0xfu) << 4 | ((cf >> 16) & 0xfu) << 8 | ((cf >> 24) & 0xfu) << 12;
        const uint32_t smp_all = ((cf >> 4) & 1u) | ((cf >> 12) & 1u) << 1 | ((cf >> 20) & 1u) << 2 | ((cf >> 28) & 1u) << 3;
        fl_all &= (1u << (4u * nv)) - 1u;
        /* every off-reference read captured: a site past SS_NEAR_SLOTS flagged
         * chunks lost some (and may not take the exit) */
        const bool ok = cand && ma <= SS_NEAR_K && mb <= SS_NEAR_K && (uint32_t)__popc(fl_all) == ma + mb;
        if (__ballot(ok)) {
            /* the off-reference reads from the captured chunks, in element
             * order (the tumor's first); at most 2 SS_NEAR_K of them matter */
            if (!ok) fl_all = 0u;
            uint32_t key[2 * SS_NEAR_K];
            const uint32_t *cw = reinterpret_cast<const uint32_t *>(&T.cap[lane][0]);
            const uint32_t la = ln_lut_row(1u + ref16), lb = ln_lut_row(17u + ref16);
#pragma unroll
            for (uint32_t i = 0; i < 2u * SS_NEAR_K; ++i) {
                const bool has = fl_all != 0u;
                const uint32_t bpos = ln_ffbl(fl_all) & 15u;
                fl_all &= fl_all - 1u;
                const uint32_t slot = bpos >> 2;
                const uint32_t rd = has ? cw[4u * slot + (bpos & 3u)] : 0u;
                const uint32_t row = (smp_all >> slot) & 1u ? lb : la;
                uint32_t minq;
                asm("v_min_u32_sdwa %0, %1, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1"
                    : "=v"(minq) : "v"(rd));
                const uint32_t ex = reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(lut) +
                                                                   (((rd >> 13) & 0xf8u) ^ row))->x;
                /* the key build's 16-bit key (ln_chunk), minq in 8 bits (5..12) */
                const uint32_t kk = (ex & 0xffffu) | minq << 5 | ((rd >> 13) & 6u) | ln_nz(rd & 0x3f00u);
                key[i] = has ? kk : 0u;
            }
            uint32_t kt[SS_NEAR_K], kn[SS_NEAR_K];
#pragma unroll
            for (uint32_t i = 0; i < SS_NEAR_K; ++i) {
                kt[i] = i < ma ? key[i] : 0u;
                const uint32_t jj = ma + i;                  /* <= 2K - 1 */
                const uint32_t kj = jj == 0u ? key[0] : jj == 1u ? key[1] : jj == 2u ? key[2] : jj == 3u ? key[3]
                                  : jj == 4u ? key[4] : key[5];
                kn[i] = i < mb ? kj : 0u;
            }
            /* both samples on every lane (no divergent region; a lane that
             * is not ok has no keys and its answer is dropped) */
            const bool okt = ln_near_sample(kt, ca, c24s & 0xffffu, r, a.m, fk);
            const bool okn = ln_near_sample(kn, cb, c24s >> 16, r, a.m, fk);
            done = done || (ok & okt & okn);
        }
        wave_sync();                                     /* T is reused by the next block */
    }
    if (done) kernarg_args().score[s] = sc;
    return done;
}

/* Triage kernel (round 6): the early exit (tri_block) for every 64-site
 * block of mean depth <= SS_EARLY_MAX_READS, lane = site; the sites it does
 * not decide are appended to the main kernel's list, the deeper blocks
 * themselves to the deep triage's (both staged per wave, stage_push).
 * Launched only when no glf records are requested and the host's bound
 * tables are valid (SS_MF_FAST); otherwise the main kernel scores every site
 * itself.  Its own kernel because the exit path needs far fewer registers
 * than the main kernel's 128-key network. */
__global__ __launch_bounds__(SS_TRIAGE_BLOCK) __attribute__((amdgpu_waves_per_eu(SS_TRIAGE_WAVES_PER_EU)))
void ss_score_triage(ss_score_args a)
{
    __shared__ double fk[LN_FK_ZERO + 1];
    __shared__ uint2 lut[LN_LUT_BYTES / 8];
    __shared__ TriLds TL[SS_TRIAGE_BLOCK / 64];
    for (uint32_t i = threadIdx.x; i <= LN_FK_ZERO; i += blockDim.x) fk[i] = i < LN_FK_LIVE ? ss_tab_fk(a.m)[i] : 0.0;
    ln_lut_build(lut);
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (SS_TRIAGE_BLOCK / 64);
    const uint32_t n_sites = (uint32_t)a.n_sites;
    const uint32_t nblocks = (n_sites + 63u) / 64u;
    const uint32_t end_t = a.off_t[n_sites], end_n = a.off_n[n_sites];
    uint32_t nb = 0, hb = 0;
    for (uint32_t blk = blockIdx.x * (SS_TRIAGE_BLOCK / 64) + wv; blk < nblocks; blk += nwaves) {
        const uint32_t s = blk * 64u + lane;
        const bool insite = s < n_sites;
        /* the block's reads from its offsets (scalar loads) */
        bool shallow, narrow;
        {
            const ss_score_args &k = kernarg_args();
            const uint32_t s0 = blk * 64u, s1 = min(s0 + 64u, n_sites);
            const uint32_t breads = (k.off_t[s1] - k.off_t[s0]) + (k.off_n[s1] - k.off_n[s0]);
            shallow = breads <= SS_EARLY_MAX_READS * (s1 - s0);
            narrow = breads <= (SS_EARLY_MAX_READS / 2u) * (s1 - s0);
        }
        const ss_score_args &k = kernarg_args();
        if (shallow) {
            /* every lane of the wave (tri_block's DPP / ballot / bpermute
             * exchanges read all 64 lanes; it handles lanes past the batch).
             * Up to 128 mean reads per site 4 lanes per site (16 sites per
             * round: C4 +6%, C2 +12%), past that 8 (C3: 4 lanes -1.5%) */
            const bool d = tri_block(kernarg_args(), lut, fk, TL[wv], lane, s, insite, end_t, end_n, narrow ? 2u : 3u);
            /* an undecided site (more than 3 off-reference reads, a sample past
             * 128 reads, or a real candidate) gets the deep triage's wider test */
            const bool need = insite && !d;
            const uint64_t m = __ballot(need);
            if (m) {                                     /* few at 30x .. 100x: one atomic per wave */
                const uint32_t first = (uint32_t)__builtin_ctzll(m);
                uint32_t base = 0;
                if (lane == first) base = atomicAdd(k.dsite_count, (uint32_t)__popcll(m));
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)first);
                if (need) k.dsite_list[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = s;
            }
        } else {
            stage_push(hb, nb, lane == 0u, blk, k.dtri_count, k.dtri_list, lane);
        }
    }
    const ss_score_args &k = kernarg_args();
    uint32_t *scratch = reinterpret_cast<uint32_t *>(&TL[0]);
    static_assert(sizeof(TL) >= 4u * (2u + SS_TRIAGE_BLOCK), "flush scratch");
    stage_wg_flush(hb, nb, k.dtri_count, k.dtri_list, scratch, lane);
}

/* --------------------------------------------------------------------------
 * Deep triage (round 6): the early exit for sites with a sample of 129 ..
 * SS_NEAR_MAXN reads (the triage kernel lists its deeper blocks for it).
 * The same test as tri_block with counts past 255 rescaled
 * (sniper_maqcns.c:178-182) and up to SS_NEAR_KD off-reference reads per
 * sample: 16 lanes per site, TRD_P chunk loads in flight per lane, 16-bit
 * group counts, the off-reference reads' 16-bit keys kept in LDS (in element
 * order, the tumor's first), and a 16-key network per sample for their
 * chains.
 * ------------------------------------------------------------------------ */
#define TGD 16u                      /* lanes per site */
#define SS_NEAR_KD 16u               /* off-reference contributing reads per sample the deep test evaluates */
#define SS_NEAR_WORDS 32u            /* off-reference reads kept per site */
#define TRD_P 8u                     /* chunk loads in flight per lane (16, or two batches of 8
                                        in flight: 10% slower at 3 waves per SIMD) */

struct TriLdsD {
    uint16_t capk[64][SS_NEAR_WORDS + 2];    /* the keys (trd_key) of the site's off-reference reads, element
                                                order (+2: an odd word stride) */
    uint32_t t02[64], t13[64], n02[64], n13[64]; /* contributing reads of bases 0 | 2 << 16, 1 | 3 << 16 */
    uint32_t c24[64];                        /* contributing reads of minq >= 24: tumor | normal << 16 */
    uint32_t c24s1[64];                      /* of them on strand 1 */
    uint32_t nw[64];                         /* off-reference reads seen (past SS_NEAR_WORDS: some lost) */
};

/* sum over the 16 lanes of a DPP row */
__device__ __forceinline__ uint32_t trd_gsum(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false);    /* quad_perm [1,0,3,2] */
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);    /* quad_perm [2,3,0,1] */
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);   /* row_half_mirror */
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false);   /* row_mirror */
    return v;
}

/* exclusive prefix sum over the 16 lanes of a DPP row */
__device__ __forceinline__ uint32_t trd_xscan(uint32_t v)
{
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   /* row_shr:1 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   /* row_shr:2 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   /* row_shr:4 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   /* row_shr:8 */
    return x - v;
}

/* the deep test's key of an off-reference read: the key build's 16-bit key
 * without the sample bit (so 0xffff is a pad), minq in 8 bits (5..12) */
__device__ __forceinline__ uint32_t trd_key(const uint2 *lut, uint32_t rd, uint32_t row)
{
    const uint32_t minq = min(rd & 0xffu, (rd >> 8) & 0xffu);
    const uint32_t ex = reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(lut) + (((rd >> 13) & 0xf8u) ^ row))->x;
    return (ex & 0x7fffu) | minq << 5 | ((rd >> 13) & 6u) | min(rd & 0x3f00u, 1u);
}

/* One sample of the deep test: v its off-reference reads' keys in the lane
 * network's layout (16 elements, pads 0xffff), nk their number (<=
 * SS_NEAR_KD), c / c24 as ln_near_sample */
__device__ __forceinline__ bool ln_near_sample16(uint32_t (&v)[8], uint32_t nk, const uint32_t (&c)[4], uint32_t c24,
                                                 uint32_t c24s1, uint32_t r, const ss_dev_model &m, const double *fk)
{
    ln_levels<8, 2>(v);                                  /* ascending; the pads on top */
    float es[4] = {0.0f, 0.0f, 0.0f, 0.0f}, fs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const char *fkb = reinterpret_cast<const char *>(fk);
    uint64_t W = 0;                                      /* w per (group, strand): 8-bit fields */
    uint32_t c24nr = 0, c24nr1 = 0;
    const uint32_t nmax = wave_max(nk);
    /* the chains in the reference's descending walk: key nk - 1 down to 0 */
#pragma unroll
    for (int e = 15; e >= 0; --e) {
        if ((uint32_t)e >= nmax) continue;               /* wave-uniform */
        const uint32_t key = ln_elem<8>(v, e);
        const bool live = (uint32_t)e < nk;
        const uint32_t x = (key >> 13) & 3u;
        const uint32_t minq = (key >> 5) & 0xffu;
        const uint32_t q = max(minq, (key & 1u) << 2);    /* sniper_maqcns.c:165 */
        const uint32_t sh = 8u * (2u * x + ((key >> 3) & 1u));
        const uint32_t w = (uint32_t)(W >> sh) & 0xffu;
        W += live ? 1ull << sh : 0ull;
        const double fv = *reinterpret_cast<const double *>(fkb + 8u * (live ? w : (uint32_t)LN_FK_ZERO));
        const float e0 = ln_sel4f(es, x), f0 = ln_sel4f(fs, x);
        const float e1 = (float)((double)e0 + fv * (double)q);
        const float f1 = (float)((double)f0 + fv);
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b) {
            es[b] = b == x ? e1 : es[b];
            fs[b] = b == x ? f1 : fs[b];
        }
        c24nr += live && minq >= 24u ? 1u : 0u;
        c24nr1 += live && minq >= 24u ? (key >> 3) & 1u : 0u;
    }
    /* the reference group's reads of minq >= 24 lead its two strand chains
     * (their keys sort first within a group), so its esum is at least the
     * sum of the two chains' bounds (ss_capi.hip near_tables: esr is rounded
     * down with a 2e-4 margin that covers this float add) */
    const uint32_t r1 = c24s1 - c24nr1, r0 = (c24 - c24nr) - r1;
    const float *esr = ss_tab_esr(m);
    return ln_near_eval(es, fs, c, esr[min(r0, SS_NEAR_MAXN)] + esr[min(r1, SS_NEAR_MAXN)], r, m);
}

/* the deep triage's work for one block of up to 64 listed sites (lane =
 * list entry); true when it wrote the site's score */
__device__ __forceinline__ bool trd_block(const ss_score_args &a, const uint2 *lut, const double *fk, TriLdsD &T,
                                          uint32_t lane, uint32_t s, bool insite, uint32_t end_t, uint32_t end_n)
{
    uint32_t ot = 0, ot1 = 0, on = 0, on1 = 0, refc = 'N';
    if (insite) {
        ot = a.off_t[s];
        ot1 = a.off_t[s + 1];
        on = a.off_n[s];
        on1 = a.off_n[s + 1];
        refc = a.ref[s];
    }
    const uint32_t ref16 = ss_tab_nt16(a.m)[refc];
    const uint32_t nt = ot1 - ot, nn = on1 - on;
    const bool small = insite && ot <= ot1 && ot1 <= end_t && on <= on1 && on1 <= end_n && nt <= SS_NEAR_MAXN &&
                       nn <= SS_NEAR_MAXN;
    bool done = false;
    int32_t sc = 255;
    if (small && (refc == 'N' || nt == 0u || nn == 0u)) {
        done = true;
        sc = -1;
    } else if (small && ref16 == 15u) {
        done = true;
    }
    const bool acgt = ref16 == 1u || ref16 == 2u || ref16 == 4u || ref16 == 8u;
    const bool cand = small && !done && acgt;
    if (__ballot(cand)) {
        const uint32_t nt4 = (nt + 3u) & ~3u;
        const uint32_t tm = ln_uniform(__ballot(cand && ((uint64_t)ot + nt4 > end_t ||
                                                         (uint64_t)on + ((nn + 3u) & ~3u) > end_n)) ||
                                       end_t < 4u || end_n < 4u);
        const uint32_t j = lane & (TGD - 1u);
        const uint32_t pk = cand ? (nt | nn << 12 | ref16 << 24) : 0u;   /* nt, nn <= 2048 */
        /* TGD rounds of 64 / TGD sites each */
#pragma unroll 1
        for (uint32_t rr = 0; rr < TGD; ++rr) {
            const uint32_t site = rr * (64u / TGD) + lane / TGD;
            const int sa = (int)(site << 2);
            const uint32_t g_pk = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)pk);
            const uint32_t g_ot = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)ot);
            const uint32_t g_on = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)on);
            const uint32_t g_nt = g_pk & 0xfffu, g_nn = (g_pk >> 12) & 0xfffu, g_ref16 = (g_pk >> 24) & 0xfu;
            const uint32_t g_nt4 = (g_nt + 3u) & ~3u;
            const uint32_t g_nchk = g_pk ? (g_nt4 + g_nn + 3u) >> 2 : 0u;
            const uint32_t K = wave_max((g_nchk + TGD - 1u) / TGD);
            if (K == 0u) continue;
            const uint32_t la = ln_lut_row(1u + g_ref16), lb = ln_lut_row(17u + g_ref16);
            const uint32_t *pt = a.reads_t + g_ot, *pn = a.reads_n + g_on - g_nt4;
            uint32_t t02 = 0, t13 = 0, n02 = 0, n13 = 0, c24 = 0, c24s1 = 0, gw = 0;
            /* a batch of TRD_P chunk loads per lane (a macro: as a lambda taking
             * the array by reference it cost 50 VGPRs), and its processing
             * (the kernel is VALU-bound: its time follows the instructions of
             * tri_chunk and the capture) */
#define TRD_LOAD1(XB)                                                                           \
        const bool fa = 4u * c < g_nt4;                                                         \
        const uint32_t *src = (fa ? pt : pn) + 4u * c;                                          \
        const int lim = live ? (int)(fa ? g_nt : g_nt4 + g_nn) - (int)(4u * c) : 0;             \
        _Pragma("unroll") for (int t = 0; t < 4; ++t) XB[u][t] = 0u;                            \
        if (tm) {                                                                               \
            _Pragma("unroll") for (int t = 0; t < 4; ++t) if (t < lim) XB[u][t] = src[t];       \
        } else if (live) {                                                                      \
            const u32x4_a4 q4 = *reinterpret_cast<const u32x4_a4 *>(src);                       \
            XB[u][0] = q4.x; XB[u][1] = q4.y; XB[u][2] = q4.z; XB[u][3] = q4.w;                 \
        }
#define TRD_LOAD(XB, KB)                                                                        \
    _Pragma("unroll") for (uint32_t u = 0; u < TRD_P; ++u) {                                    \
        const uint32_t c = ((KB) + u) * TGD + j;                                                \
        const bool live = c < g_nchk;                                                           \
        TRD_LOAD1(XB)                                                                           \
    }
            auto pr = [&](const uint32_t (&xb)[TRD_P][4], uint32_t kb) {
#pragma unroll
                for (uint32_t u = 0; u < TRD_P; ++u) {
                    if (kb + u >= K) break;                      /* wave-uniform */
                    const uint32_t c = (kb + u) * TGD + j;
                    const bool live = c < g_nchk;
                    const bool fa = 4u * c < g_nt4;
                    const int lim = live ? (int)(fa ? g_nt : g_nt4 + g_nn) - (int)(4u * c) : 0;
                    uint32_t ca8 = 0, ct8 = 0;
                    const uint32_t fl = tri_chunk<true>(lut, xb[u], lim, fa ? la : lb, fa, ca8, ct8, c24, &c24s1);
                    /* the chunk's 8-bit counts (<= 4 each) into 16-bit fields */
                    const uint32_t e02 = ct8 & 0x00ff00ffu, e13 = (ct8 >> 8) & 0x00ff00ffu;
                    t02 += fa ? e02 : 0u;
                    t13 += fa ? e13 : 0u;
                    n02 += fa ? 0u : e02;
                    n13 += fa ? 0u : e13;
                    /* the off-reference reads' keys, in element order */
                    if (__ballot(fl != 0u)) {
                        const uint32_t nf = (uint32_t)__popc(fl);
                        const uint32_t pre = gw + trd_xscan(nf);
#pragma unroll
                        for (uint32_t t = 0; t < 4u; ++t) {
                            const uint32_t idx = pre + (uint32_t)__popc(fl & ((1u << t) - 1u));
                            if (((fl >> t) & 1u) && idx < SS_NEAR_WORDS)
                                T.capk[site][idx] = (uint16_t)trd_key(lut, xb[u][t], fa ? la : lb);
                        }
                        gw += trd_gsum(nf);
                    }
                }
            };
#pragma unroll 1
            for (uint32_t kb = 0; kb < K; kb += TRD_P) {
                uint32_t xb[TRD_P][4];
                TRD_LOAD(xb, kb)
                pr(xb, kb);
            }
#undef TRD_LOAD
#undef TRD_LOAD1
            t02 = trd_gsum(t02);
            t13 = trd_gsum(t13);
            n02 = trd_gsum(n02);
            n13 = trd_gsum(n13);
            c24 = trd_gsum(c24);
            c24s1 = trd_gsum(c24s1);
            if (j == 0u) {
                T.t02[site] = t02;
                T.t13[site] = t13;
                T.n02[site] = n02;
                T.n13[site] = n13;
                T.c24[site] = c24;
                T.c24s1[site] = c24s1;
                T.nw[site] = gw;
            }
        }
        wave_sync();
        /* lane = site again */
        uint32_t ca[4] = {0u, 0u, 0u, 0u}, cb[4] = {0u, 0u, 0u, 0u}, c24s = 0, c24s1 = 0, nwc = 0;
        if (cand) {
            const uint32_t a02 = T.t02[lane], a13 = T.t13[lane], b02 = T.n02[lane], b13 = T.n13[lane];
            ca[0] = a02 & 0xffffu; ca[1] = a13 & 0xffffu; ca[2] = a02 >> 16; ca[3] = a13 >> 16;
            cb[0] = b02 & 0xffffu; cb[1] = b13 & 0xffffu; cb[2] = b02 >> 16; cb[3] = b13 >> 16;
            c24s = T.c24[lane];
            c24s1 = T.c24s1[lane];
            nwc = T.nw[lane];
        }
        const uint32_t r = (uint32_t)__builtin_ctz(ref16 | 16u);
        const uint32_t ma = ca[0] + ca[1] + ca[2] + ca[3] - ln_sel4(ca, r);
        const uint32_t mb = cb[0] + cb[1] + cb[2] + cb[3] - ln_sel4(cb, r);
        const bool ok = cand && ma <= SS_NEAR_KD && mb <= SS_NEAR_KD && nwc == ma + mb;
        if (__ballot(ok)) {
            const uint32_t nka = ok ? ma : 0u, nkb = ok ? mb : 0u;
            const uint32_t kmax = wave_max(max(nka, nkb));
            uint32_t vt[8], vn[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) vt[i] = vn[i] = 0x0000ffffu;    /* pads: lo 0xffff, hi ~0xffff */
#pragma unroll
            for (uint32_t i = 0; i < SS_NEAR_KD; ++i) {
                if (i >= kmax) break;                            /* wave-uniform */
                const uint32_t kt = i < nka ? (uint32_t)T.capk[lane][i] : 0xffffu;
                const uint32_t kn = i < nkb ? (uint32_t)T.capk[lane][nka + i] : 0xffffu;
                if (i < 8u) {
                    vt[i] = (vt[i] & 0xffff0000u) | kt;
                    vn[i] = (vn[i] & 0xffff0000u) | kn;
                } else {
                    vt[15 - i] = (vt[15 - i] & 0x0000ffffu) | (kt ^ 0xffffu) << 16;
                    vn[15 - i] = (vn[15 - i] & 0x0000ffffu) | (kn ^ 0xffffu) << 16;
                }
            }
            /* both samples on every lane (a lane that is not ok has no keys
             * and its answer is dropped) */
            const bool okt = ln_near_sample16(vt, nka, ca, c24s & 0xffffu, c24s1 & 0xffffu, r, a.m, fk);
            const bool okn = ln_near_sample16(vn, nkb, cb, c24s >> 16, c24s1 >> 16, r, a.m, fk);
            done = done || (ok & okt & okn);
        }
        wave_sync();                                     /* T is reused by the next block */
    }
    if (done) kernarg_args().score[s] = sc;
    return done;
}

/* Deep triage kernel: the blocks the triage kernel found past
 * SS_EARLY_MAX_READS mean reads (a wave per listed block, lane = site), then
 * the sites the triage kernel's narrower test left (64 per wave: up to 16
 * off-reference reads per sample here, 3 there); undecided sites go on to the
 * main kernel's list. */
__global__ __launch_bounds__(SS_TRIAGE_DEEP_BLOCK) void ss_score_triage_deep(ss_score_args a)
{
    __shared__ double fk[LN_FK_ZERO + 1];
    __shared__ uint2 lut[LN_LUT_BYTES / 8];
    __shared__ TriLdsD TL[SS_TRIAGE_DEEP_BLOCK / 64];
    const uint32_t n_sites = (uint32_t)a.n_sites;
    const uint32_t nlisted = min(*a.dtri_count, (n_sites + 63u) / 64u);
    const uint32_t nsl = min(*a.dsite_count, n_sites);
    const uint32_t nitems = nlisted + (nsl + 63u) / 64u;        /* listed blocks, then groups of 64 listed sites */
    if (blockIdx.x * (SS_TRIAGE_DEEP_BLOCK / 64) >= nitems) return;
    for (uint32_t i = threadIdx.x; i <= LN_FK_ZERO; i += blockDim.x) fk[i] = i < LN_FK_LIVE ? ss_tab_fk(a.m)[i] : 0.0;
    ln_lut_build(lut);
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (SS_TRIAGE_DEEP_BLOCK / 64);
    const uint32_t end_t = a.off_t[n_sites], end_n = a.off_n[n_sites];
    uint32_t ns = 0, hs = 0;
    for (uint32_t i = blockIdx.x * (SS_TRIAGE_DEEP_BLOCK / 64) + wv; i < nitems; i += nwaves) {
        uint32_t s;
        bool insite;
        if (i < nlisted) {                               /* wave-uniform */
            s = kernarg_args().dtri_list[i] * 64u + lane;
            insite = s < n_sites;
        } else {
            const uint32_t e = (i - nlisted) * 64u + lane;
            insite = e < nsl;
            s = insite ? kernarg_args().dsite_list[e] : 0u;
        }
        const bool d = trd_block(kernarg_args(), lut, fk, TL[wv], lane, insite ? s : 0u, insite, end_t, end_n);
        const ss_score_args &k = kernarg_args();
        stage_push(hs, ns, insite && !d, s, k.tri_count, k.tri_list, lane);
    }
    const ss_score_args &k = kernarg_args();
    static_assert(sizeof(TL) >= 4u * (2u + SS_TRIAGE_DEEP_BLOCK), "flush scratch");
    stage_wg_flush(hs, ns, k.tri_count, k.tri_list, reinterpret_cast<uint32_t *>(&TL[0]), lane);
}

/* compiled for 3 waves per SIMD: the per-lane network's 64 registers, the
 * chunk loads in flight and the key arithmetic need about 160 VGPRs (at 128
 * the compiler spills); the records take 8 KB of LDS per wave.  Scores the
 * triage kernel's list (a.tri_list) or, without one, every site. */
__global__ __launch_bounds__(SS_MAIN_BLOCK) __attribute__((amdgpu_waves_per_eu(3)))
void ss_score_main(ss_score_args a)
{
    __shared__ double fk[LN_FK_ZERO + 1];
    __shared__ uint2 lut[LN_LUT_BYTES / 8];
    __shared__ LaneLds LL[LN_WAVES];
    /* qAddTable (somatic_sniper.c:13,101-107) in LDS as int16 (its entries lie
     * in [-512, 0]; 2 KB keeps 3 workgroups per CU within 160 KB) */
    __shared__ int16_t qtab[1024];
    const uint32_t n_sites = (uint32_t)a.n_sites;
    const bool listed = a.tri_list != nullptr;
    const uint32_t n = listed ? min(*a.tri_count, n_sites) : n_sites;
    const uint32_t nblocks = (n + 63u) / 64u;
    const uint32_t nwaves = gridDim.x * LN_WAVES;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t gw = blockIdx.x * LN_WAVES + wv;
    if (blockIdx.x * LN_WAVES >= nblocks) return;      /* no block for this workgroup (a short list) */
    for (uint32_t i = threadIdx.x; i <= LN_FK_ZERO; i += blockDim.x) fk[i] = i < LN_FK_LIVE ? ss_tab_fk(a.m)[i] : 0.0;
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) qtab[i] = (int16_t)ss_tab_qadd(a.m)[i];
    ln_lut_build(lut);
    __syncthreads();
    const uint32_t lane = lane_id();
    LaneLds &L = LL[wv];
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;
    const uint32_t end_t = a.off_t[n_sites], end_n = a.off_n[n_sites];
    uint32_t ndeep = 0;
    for (uint32_t blk = gw; blk < nblocks; blk += nwaves) {
        const uint32_t i = blk * 64u + lane;
        const bool insite = i < n;
        uint32_t s = i;
        if (listed) s = insite ? kernarg_args().tri_list[i] : 0u;
        ln_block(kernarg_args(), s, insite, lut, fk, qtab, L, lane, gw, cap, end_t, end_n, ndeep);
    }
    if (lane == 0 && ndeep) {
        /* one atomic numbers the segment and places its entries, so the
         * offsets ascend with the segment index (the group kernel searches them) */
        const ss_score_args &k = kernarg_args();
        const unsigned long long r = atomicAdd(k.deep_acc, 1ull << 32 | ndeep);
        k.deep_segs[r >> 32] = gw;
        k.deep_off[r >> 32] = (uint32_t)r;
    }
}


/* --------------------------------------------------------------------------
 * Group kernel: the wide list's sites with at most SS_WIDE_MAXSLOTS reads per
 * sample, sorted by lane groups (round 3; replaces the wave-per-site network
 * of round 2's ss_score_wide).
 *
 * A sort unit is one (site, sample) of n reads; it takes U = ceil(n / 128)
 * lanes (1 .. 16, 128 reads each; round 5) and sorts as a network of P = the
 * power of two >= U lanes whose lanes U .. P - 1 are virtual (pads only).  A
 * unit's reads are dealt to its lanes in 4-read chunks, round-robin, so one
 * load instruction reads each unit's next 16 U contiguous bytes.  Every lane
 * builds and sorts its keys exactly as the main kernel does (ln_keys,
 * ln_levels: complemented high halves, packed min / max), then the unit's
 * lanes merge across lanes, level 256 .. 128 P of the same flip-form bitonic
 * network: a mirror stage with the unit's lane j ^ (M - 1), cleaners with
 * j ^ M/4 .. j ^ 1 (ds_bpermute from the unit's first lane: no alignment
 * needed), the in-lane stage at distance 64 and the in-lane cleaners.  In a
 * cross-lane stage the lower lane keeps the minimum elements: in this layout
 * that is min in the low half and max in the (complemented) high half, one
 * v_bfi_b32 per register with a per-lane mask; a lane whose partner is
 * virtual keeps its registers (gp_xstage).  Units are packed by descending U,
 * next-fit, so every unit sits in one wave-sized batch of lanes; a batch
 * merges up to its largest P (lanes of smaller units sit the larger levels
 * out).  The sorted contributing keys leave as 8-bit fold records in the
 * wave's record buffer (HBM / L2), per unit in ascending order, and
 * finish_sub does the 32-site fold, likelihoods and decision.
 * ------------------------------------------------------------------------ */
namespace {

#define GP_WAVES (SS_WIDE_BLOCK / 64)         /* 12 waves, one workgroup per CU (168 VGPRs: 3 per SIMD) */
#define GP_UNITS (2 * GB)
/* lane positions of a chunk's units: at most 64 units of <= 16 lanes, packed
 * by descending size into 64-lane batches that waste < 16 lanes each, so at
 * most 21 batches (1024 / 49 + 1) */
#define GP_LANEPOS (21 * 64)

/* Per wave: the chunk's sites and units are kept here, not in registers, so
 * that the sort and merge (64 registers of keys) leave room for 3 waves per
 * SIMD; lanes read the entries they need. */
struct alignas(16) GroupLds {
    Slot3    slot[GP_WAVES][2 * GB];
    SlotRes  res[GP_WAVES][2 * GB];
    uint32_t site[GP_WAVES][GB];                   /* the chunk's sites, then (compacted) the scored ones */
    uint32_t refc[GP_WAVES][GB];                   /* ref char | nt16 << 8 (then compacted like site) */
    uint32_t c_site[GP_WAVES][GB];                 /* chunk entry k: site */
    uint32_t c_ot[GP_WAVES][GB], c_on[GP_WAVES][GB];   /* its first tumor / normal read */
    uint32_t c_ref[GP_WAVES][GB];                  /* ref char | nt16 << 8 | ok << 31 */
    uint32_t u_n[GP_WAVES][GP_UNITS];              /* unit u = (entry u / 2, sample u & 1): reads */
    uint32_t u_off[GP_WAVES][GP_UNITS];            /* its first lane position */
    uint32_t u_base[GP_WAVES][GP_UNITS];           /* its first record byte */
    uint32_t ucnt[GP_WAVES][GP_UNITS][4];          /* per unit: counts of bases 0, 2 | 1, 3 (16-bit), rms, wild */
    uint8_t  unit_of[GP_WAVES][GP_LANEPOS];        /* lane position -> unit (0xff: a lane no unit uses) */
};

/* cross-lane compare-exchange of lane j of a unit with its lane j ^ LJ, read
 * by ds_bpermute from the unit's first lane pb (units need no alignment; the
 * exchange runs on the LDS crossbar, not the VALU).  The lower lane keeps
 * (min lo, max hi).  A unit of U lanes sorts as one of P = pow2 >= U lanes
 * whose lanes U .. P - 1 hold only pads; this lane is then always the lower
 * one of the pair and must stay as it is (a virtual lane only ever receives
 * maxima, i.e. pads): it reads itself, which a plain stage leaves unchanged,
 * and a mirror stage reads the neutral 0x0000ffff instead (pad key low, its
 * complement high). */
template <int LJ, bool MIRROR>
__device__ __forceinline__ void gp_xstage(uint32_t (&v)[LN_R], uint32_t j, uint32_t pb, uint32_t U)
{
    const uint32_t pj = j ^ (uint32_t)LJ;
    const bool pad = pj >= U;
    const int addr = (int)((pb + (pad ? j : pj)) << 2);
    const uint32_t msk = (j & (MIRROR ? (uint32_t)((LJ + 1) >> 1) : (uint32_t)LJ)) ? 0xffff0000u : 0x0000ffffu;
#pragma unroll
    for (int r = 0; r < LN_R; ++r) {
        uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v[r]);
        if (MIRROR) o = pad ? 0x0000ffffu : o;
        uint32_t mn, mx;
        if (MIRROR) {                        /* partner element 127 - r: swap and complement */
            const uint32_t c = ~o;
            mn = pk_min_swo(v[r], c);
            mx = pk_max_swo(v[r], c);
        } else {
            mn = pk_min(v[r], o);
            mx = pk_max(v[r], o);
        }
        v[r] = (mn & msk) | (mx & ~msk);
    }
}

/* in-lane stage at distance 64: element r (low half of r) against r + 64 (high half of 63 - r) */
__device__ __forceinline__ void gp_stage64(uint32_t (&v)[LN_R])
{
#pragma unroll
    for (int r = 0; r < LN_R / 2; ++r) {
        const uint32_t x = v[r], y = v[LN_R - 1 - r];
        v[r] = pk_min_swo(x, ~y);
        v[LN_R - 1 - r] = pk_min_swo(y, ~x);
    }
}

/* level 128 M of a unit (M lanes merged), lane index j inside the unit */
template <int M>
__device__ __forceinline__ void gp_level(uint32_t (&v)[LN_R], uint32_t j, uint32_t pb, uint32_t U)
{
    gp_xstage<M - 1, true>(v, j, pb, U);
    if constexpr (M >= 16) gp_xstage<4, false>(v, j, pb, U);
    if constexpr (M >= 8) gp_xstage<2, false>(v, j, pb, U);
    if constexpr (M >= 4) gp_xstage<1, false>(v, j, pb, U);
    gp_stage64(v);
    ln_clean<LN_R, 32>(v);
}

/* lanes of a unit of n reads (128 each), and the network size it sorts as */
__device__ __forceinline__ uint32_t gp_lanes(uint32_t n)
{
    return n <= 128u ? 1u : (n + 127u) >> 7;
}
__device__ __forceinline__ uint32_t gp_pow2(uint32_t U)
{
    return U <= 1u ? 1u : U <= 2u ? 2u : U <= 4u ? 4u : U <= 8u ? 8u : 16u;
}

}  // namespace

__global__ __launch_bounds__(SS_WIDE_BLOCK) void ss_score_group(ss_score_args a)
{
    __shared__ double fk[GP_FK_ZERO + 1];
    __shared__ uint2 lut[LN_LUT_BYTES / 8];
    __shared__ GroupLds L;
    __shared__ int16_t qtab[1024];                  /* qAddTable, as in ss_score_main */
    const unsigned long long acc0 = *a.deep_acc;
    const uint32_t nsegs = min((uint32_t)(acc0 >> 32), a.deep_nseg), total = (uint32_t)acc0;
    if (nsegs == 0u) return;
    for (uint32_t i = threadIdx.x; i <= GP_FK_ZERO; i += blockDim.x) fk[i] = i < 256u ? ss_tab_fk(a.m)[i] : 0.0;
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) qtab[i] = (int16_t)ss_tab_qadd(a.m)[i];
    ln_lut_build(lut);
    __syncthreads();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    /* the wave's fold records: a global (L2-resident) buffer that holds any
     * chunk (32 sites x 2 x 2048 records), so a chunk's sites always fold
     * together; its address is re-derived where used (not held in SGPRs) */
    const size_t arena_off = (size_t)(blockIdx.x * GP_WAVES + wv) * SS_GRP_REC_BYTES + SS_GRP_REC_PAD;
    Slot3 *slot = L.slot[wv];
    SlotRes *res = L.res[wv];
    uint32_t *sites = L.site[wv], *refcs = L.refc[wv];
    uint32_t (*ucnt)[4] = L.ucnt[wv];
    uint8_t *unit_of = L.unit_of[wv];
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;
    const uint32_t end_t = a.off_t[a.n_sites], end_n = a.off_n[a.n_sites];
    /* chunks of GB sites, fewer when the list is short: a few deep sites left
     * by the triage (500x: about 1 in 10^4) then spread over that many waves
     * instead of queueing in one (a 32-site chunk of 1000-read samples took
     * one wave 0.2 ms) */
    const uint32_t gsz = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)min((uint32_t)GB, max(1u, (total + gridDim.x * GP_WAVES - 1u) / (gridDim.x * GP_WAVES))));
    for (;;) {
        /* per chunk: the lane's LDS addresses are formed inside the loop */
        const uint32_t lane = lane_id_here();
        uint32_t ch = 0;
        if (lane == 0u) ch = atomicAdd(kernarg_args().wide_next, 1u);
        const uint32_t first = (uint32_t)__builtin_amdgcn_readfirstlane((int)ch) * gsz;
        if (first >= total) break;
        const uint32_t G = total - first < gsz ? total - first : gsz;
        /* the chunk's entries, lane k = entry k, into LDS */
        {
            const ss_score_args &k = kernarg_args();
            uint32_t lo = 0, hi = nsegs;
            while (hi - lo > 1u) {
                const uint32_t mid = (lo + hi) >> 1;
                if (k.deep_off[mid] <= first) lo = mid;
                else hi = mid;
            }
            if (lane < G) {
                const uint32_t p = first + lane;
                uint32_t sg = lo;
                while (sg + 1u < nsegs && k.deep_off[sg + 1u] <= p) ++sg;
                const uint32_t cs = k.deep_list[(size_t)k.deep_segs[sg] * k.deep_seg_cap + (p - k.deep_off[sg])];
                const uint32_t ot = k.off_t[cs], ot1 = k.off_t[cs + 1];
                const uint32_t on = k.off_n[cs], on1 = k.off_n[cs + 1];
                const uint32_t rc = k.ref[cs];
                const bool ok = ot <= ot1 && ot1 <= end_t && on <= on1 && on1 <= end_n &&
                                ot1 - ot <= SS_WIDE_MAXSLOTS && on1 - on <= SS_WIDE_MAXSLOTS;
                L.c_site[wv][lane] = cs;
                L.c_ot[wv][lane] = ot;
                L.c_on[wv][lane] = on;
                L.c_ref[wv][lane] = rc | (uint32_t)ss_tab_nt16(k.m)[rc] << 8 | (ok ? 1u << 31 : 0u);
                L.u_n[wv][2u * lane] = ok ? ot1 - ot : 0u;
                L.u_n[wv][2u * lane + 1u] = ok ? on1 - on : 0u;
                if (!ok) {                                /* malformed or too deep: the deep kernel */
                    const uint32_t d = atomicAdd(k.deep2_count, 1u);
                    if (d < k.deep_cap) k.deep2_list[d] = cs;
                    else atomicOr(k.err, SS_KERR_DEEP_OVERFLOW);
                }
            }
        }
        wave_sync();
        uint32_t T = 0;
        {
            /* units: lane u < 2G is unit u = (entry u / 2, sample u & 1) of
             * U = ceil(n / 128) lanes, packed by descending U into 64-lane
             * batches (a unit never straddles one; the rest of a batch that
             * cannot take the next unit stays empty); record bases in unit
             * order rounded up to 16 bytes (x4 stores) */
            const bool is_u = lane < 2u * G;
            const uint32_t n_u = is_u ? L.u_n[wv][lane] : 0u;
            const uint32_t U_u = gp_lanes(n_u);
            uint32_t off_u = 0;
            for (uint32_t c = 16u; c >= 1u; --c) {
                const uint64_t mk = __ballot(is_u && U_u == c);
                if (!mk) continue;
                const uint32_t k = (uint32_t)__popcll(mk);
                const uint32_t q = 64u / c;                       /* units of c per batch */
                const uint32_t room = 64u - (T & 63u), f0 = room / c;   /* in the current batch */
                const uint32_t nb = T + room;                     /* the next batch */
                if (is_u && U_u == c) {
                    const uint32_t i = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                    off_u = i < f0 ? T + c * i : nb + 64u * ((i - f0) / q) + c * ((i - f0) % q);
                }
                T = k <= f0 ? T + c * k : nb + 64u * ((k - f0 - 1u) / q) + c * ((k - f0 - 1u) % q + 1u);
            }
            const uint32_t sz = is_u ? ((n_u + 15u) & ~15u) : 0u;
            const uint32_t base = wave_scan(sz);
            for (uint32_t p = lane; p < T; p += 64u) unit_of[p] = 0xffu;
            wave_sync();
            if (is_u) {
                L.u_off[wv][lane] = off_u;
                L.u_base[wv][lane] = base - sz;           /* exclusive */
                for (uint32_t t = 0; t < U_u; ++t) unit_of[off_u + t] = (uint8_t)lane;
                uint32_t z = 0u;                              /* (not a zero vector kept live) */
                asm volatile("" : "+v"(z));
                ucnt[lane][0] = ucnt[lane][1] = ucnt[lane][2] = ucnt[lane][3] = z;
            }
        }
        wave_sync();
        for (uint32_t b0 = 0; b0 < T; b0 += 64u) {
            const uint32_t p = b0 + lane;
            const uint32_t uo = p < T ? (uint32_t)unit_of[p] : 0xffu;
            const bool act = uo != 0xffu;
            const uint32_t u = act ? uo : 0u;
            const uint32_t un = L.u_n[wv][u], uU = gp_lanes(un), uP = gp_pow2(uU);
            const uint32_t site_l = u >> 1, smp = u & 1u;
            const uint32_t j = p - L.u_off[wv][u];
            const uint32_t pb = L.u_off[wv][u] - b0;            /* the unit's first lane in this batch */
            LaneIn in;
            const uint32_t *base_s = smp ? kernarg_args().reads_n : kernarg_args().reads_t;
            const uint32_t ustart = act ? (smp ? L.c_on[wv][site_l] : L.c_ot[wv][site_l]) : 0u;
            /* the unit's reads in 4-read chunks dealt round-robin over its U
             * lanes (lane j: chunks j, j + U, ..): one load instruction reads
             * each unit's next 16 U bytes, contiguous across its lanes (any
             * partition of a unit's reads sorts the same: the lanes merge).
             * A lane loads only its unit's reads: chunks past its last load
             * that one again (CLAMP), and a lane without reads loads the
             * unit's first chunk, never another unit's reads */
            const uint32_t cst = 4u * uU;
            in.na = act && un > 4u * j ? un - 4u * j : 0u;
            in.cstep = cst;
            in.nca = LN_C;                  /* every chunk is A's (nb = 0) */
            asm("" : "+v"(in.nca));
            in.na4 = in.na;
            in.nb = 0u;
            in.nab = in.na;
            const uint32_t start = ustart + (in.na ? 4u * j : 0u);
            in.clast = in.na ? (in.na - 1u) / cst : 0u;
            const uint32_t nch = wave_max(in.na ? in.clast + 1u : 0u);
            const uint32_t last_w = in.clast * cst + 4u;     /* words past start the lane may load */
            in.pa = base_s + start;
            in.pb = in.pa;
            in.la = in.lb = ln_lut_row(1u + smp * 16u + ((L.c_ref[wv][site_l] >> 8) & 0xffu));
            const uint32_t endv = smp ? end_n : end_t;
            in.tail = ln_uniform(__ballot((uint64_t)start + last_w > (uint64_t)endv) || end_t < 4u || end_n < 4u);
            uint32_t v[LN_R];
            const LaneAcc acc = ln_keys<true, true>(in, lut, nch, cap, v);
            /* the unit's counts before the sort: acc is not live across it */
            if (act) {
                const uint32_t c = acc.cnt_a;
                atomicAdd(&ucnt[u][0], c & 0x00ff00ffu);
                atomicAdd(&ucnt[u][1], (c >> 8) & 0x00ff00ffu);
                atomicAdd(&ucnt[u][2], acc.rms_a);
                if (acc.maxq >= 64u) ucnt[u][3] = 1u;     /* 8-bit records cannot hold its q */
            }
            ln_levels<LN_R, 2>(v);
            if (__ballot(act && uP >= 2u)) { if (act && uP >= 2u) gp_level<2>(v, j, pb, uU); }
            if (__ballot(act && uP >= 4u)) { if (act && uP >= 4u) gp_level<4>(v, j, pb, uU); }
            if (__ballot(act && uP >= 8u)) { if (act && uP >= 8u) gp_level<8>(v, j, pb, uU); }
            if (__ballot(act && uP >= 16u)) { if (act && uP >= 16u) gp_level<16>(v, j, pb, uU); }
            wave_sync();
            /* the unit's contributing keys as records, ascending, 16 per store:
             * past lim they stay inside the lane's 128 slots and the unit's
             * 16-byte rounding */
            const uint32_t ca = act ? ucnt[u][0] : 0u, cb = act ? ucnt[u][1] : 0u;
            const uint32_t tot = (ca & 0xffffu) + (ca >> 16) + (cb & 0xffffu) + (cb >> 16);
            const int lim = act ? min(max((int)tot - (int)(128u * j), 0), 128) : 0;
            const uint32_t ubase = L.u_base[wv][u] + 128u * j;
            ln_to_records<true>(v, wave_max((uint32_t)lim));
            uint8_t *gbuf = kernarg_args().grp_rec + arena_off;
#pragma unroll
            for (int i = 0; i < LN_C; i += 4) {
                if (!__ballot(4 * i < lim)) continue;
                if (4 * i < lim)
                    *reinterpret_cast<uint4 *>(gbuf + ubase + 4u * (uint32_t)i) =
                        make_uint4(ln_rec_dword(v, i), ln_rec_dword(v, i + 1), ln_rec_dword(v, i + 2),
                                   ln_rec_dword(v, i + 3));
            }
            wave_sync();
        }
        /* slots of the sites that stay (no wild read, well formed), compacted */
        const bool is_u = lane < 2u * G;
        const uint32_t wild_u = is_u ? ucnt[lane][3] : 0u;
        const uint64_t wildm = __ballot(wild_u != 0u);
        const bool site_lane = lane < G;
        const uint32_t cref = site_lane ? L.c_ref[wv][lane] : 0u;
        const bool c_ok = (cref >> 31) != 0u;
        const bool stay = site_lane && c_ok && !((wildm >> (2u * lane)) & 3u);
        const uint64_t staym = __ballot(stay);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(staym >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)staym, 0u));
        if (site_lane && c_ok && !stay) {                    /* a wild read: the deep kernel */
            const ss_score_args &k = kernarg_args();
            const uint32_t d = atomicAdd(k.deep2_count, 1u);
            if (d < k.deep_cap) k.deep2_list[d] = L.c_site[wv][lane];
            else atomicOr(k.err, SS_KERR_DEEP_OVERFLOW);
        }
        /* unit lanes publish their slot under the site's rank */
        const uint32_t us = lane >> 1;
        const uint32_t rank_u = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(us << 2), (int)rank);
        const bool stay_u = is_u && ((staym >> us) & 1ull);
        if (stay_u) {
            Slot3 &st = slot[2u * rank_u + (lane & 1u)];
            const uint32_t ca = ucnt[lane][0], cb = ucnt[lane][1];
            st.rec_n = L.u_base[wv][lane] | L.u_n[wv][lane] << 17;
            st.cnt01 = (ca & 0xffffu) | (cb & 0xffffu) << 16;
            st.cnt23 = (ca >> 16) | (cb >> 16) << 16;
            st.rms = ucnt[lane][2];
        }
        const uint32_t cs = site_lane ? L.c_site[wv][lane] : 0u;
        if (stay) {
            sites[rank] = cs;
            refcs[rank] = cref & 0xffffu;
        }
        const uint32_t G2 = (uint32_t)__popcll(staym);
        /* the records' global stores complete before any lane reads them */
        __builtin_amdgcn_s_waitcnt(0x0f70);                  /* vmcnt(0) */
        wave_sync();
        if (G2) finish_sub(kernarg_args(), (int)G2, kernarg_args().grp_rec + arena_off, slot, res, sites, refcs, fk, qtab);
    }
}

/* --------------------------------------------------------------------------
 * Wild kernel (ss_score_wild, the deep kernel of rounds 1-5): the sites the
 * deep kernel (below) hands on -- a read of minq >= 64 (bins past the bottom
 * window), a sample of more than SS_BINS_MAXN reads, malformed offsets.  Any
 * depth, any quality.
 *
 * No sort: the fold only needs each (sample, base) group's reads in the
 * reference's descending key order (sniper_maqcns.c:157-172), and reads with
 * equal (q, strand) contribute identical terms (see the order key), so a
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
#define DEEP_WAVES (SS_WILD_BLOCK / 64)
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

__global__ __launch_bounds__(SS_WILD_BLOCK) void ss_score_wild(ss_score_args a)
{
    __shared__ double fk[256];
    __shared__ DeepWave DW[DEEP_WAVES];
    __shared__ int16_t qtab[1024];                  /* qAddTable, as in ss_score_main */
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) fk[i] = ss_tab_fk(a.m)[i];
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) qtab[i] = (int16_t)ss_tab_qadd(a.m)[i];
    __syncthreads();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    DeepWave &D = DW[wv];
    const uint32_t count = *a.deep3_count;
    const uint32_t lim = count < a.deep_cap ? count : a.deep_cap;
    const uint32_t end_t = a.off_t[a.n_sites], end_n = a.off_n[a.n_sites];
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;
    const uint32_t lane = lane_id();
    const uint32_t grp = ((lane >> 3) & 1u) * 4u + ((lane >> 1) & 3u);  /* fold lanes 0..15: sample, base */
    for (uint32_t w = blockIdx.x * DEEP_WAVES + wv; w < lim; w += gridDim.x * DEEP_WAVES) {
        /* arguments re-read from the kernarg segment where used: they do not
         * stay live in SGPRs across the site loop (44 SGPR spills before) */
        const ss_score_args &k = kernarg_args();
        const uint32_t s = k.deep3_list[w];
        const uint32_t ot = k.off_t[s], ot1 = k.off_t[s + 1], on = k.off_n[s], on1 = k.off_n[s + 1];
        if (!site_wellformed(ot, ot1, end_t) || !site_wellformed(on, on1, end_n)) {
            if (lane == 0) {
                atomicOr(k.err, SS_KERR_MALFORMED);
                k.score[s] = -2;
            }
            continue;                                  /* wave-uniform */
        }
        const uint32_t nt = ot1 - ot, nn = on1 - on;
        const uint32_t refc = k.ref[s];
        const uint32_t ref16 = ss_tab_nt16(k.m)[refc];
        uint32_t tb, th;
        nt_tables(ref16, tb, th);
        if (lane < 2u) D.rms[lane] = 0ull;
        deep_zero(D.hist);
        wave_sync();
        /* the first pass also counts the bottom window: when every bin is in
         * it (minq <= 60 everywhere) it is the only pass */
        uint64_t rt = 0, rn = 0;
        uint32_t top = max(deep_pass<0>(k.reads_t + ot, nt, tb, th, cap, 0, DW_BINS, D.hist, rt),
                           deep_pass<0>(k.reads_n + on, nn, tb, th, cap, 0, DW_BINS, D.hist + 4 * DW_BINS, rn));
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
                deep_pass<1>(k.reads_t + ot, nt, tb, th, cap, lo, hi, D.hist, unused);
                deep_pass<1>(k.reads_n + on, nn, tb, th, cap, lo, hi, D.hist + 4 * DW_BINS, unused);
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
        glf_and_cns((int)(lane & 3u), es, fs, c, n, rms, k.m, lk, min_lk, rms_q, cns);
        if (lane == 0u || lane == 4u) {
            SlotRes &r = D.res[smp];
#pragma unroll
            for (int g = 0; g < 10; ++g) r.lk[g] = (uint8_t)lk[g];
            r.cns = cns;
            r.depth = n > 16777215u ? 16777215u : n;
            r.min_lk = (uint8_t)min_lk;
            r.rms_q = (uint8_t)rms_q;
            if (k.glf) store_glf(&k.glf[2ull * s + smp], ref16, lk, min_lk, rms_q, r.depth);
        }
        wave_sync();
        if (lane == 0u) decide_site(k, qtab, s, refc | ref16 << 8, D.res[0], D.res[1]);
        wave_sync();
    }
}

/* --------------------------------------------------------------------------
 * Deep kernel (round 6): the group kernel's overflow list -- sites with a
 * sample past SS_WIDE_MAXSLOTS reads, and the ones it routes on (a read of
 * minq >= 64, malformed offsets: this kernel passes those to ss_score_wild,
 * with samples past SS_BINS_MAXN reads).
 *
 * Counting sort, as ss_score_wild, but with the work laid out for 64 lanes:
 *   1. per site (the whole wave): each sample's reads are counted into a
 *      16-bit histogram of order bins in LDS (ds_add, eight loads in flight
 *      per lane); slots per sample: group A the deep bins 0..367 (hasbase
 *      orders A before N / IUPAC reads there), C / G / T the same bins without
 *      the hasbase bit (always 1), 184 each -- 960 slots in all.  The
 *      histogram then becomes runs (q | strand << 6 | count << 7, count <=
 *      511) in the reference's walk order -- per group, descending key -- by
 *      ballot compaction, 64 slots per row, appended to the wave's run list;
 *   2. per round of up to 32 sites (when the run list or the round is full):
 *      lane = (site, sample) folds its unit's four group chains from its runs
 *      (the largest group first), one read per step with fk[w] from LDS --
 *      the reference's serial float chains, every lane busy -- then evaluates
 *      the ten genotypes, and lane = site decides.
 * Rounds 1-5 folded one site per wave with 16 of 64 lanes (ss_score_wild):
 * 33,000 VALU instructions per site at 3000x/3000x, 0.045 of the HBM roofline.
 * ------------------------------------------------------------------------ */
namespace {

#define BN_WAVES (SS_DEEP_BLOCK / 64)
#define BN_SLOTS 640                    /* bin slots per sample: group A 256, C / G / T 128 each */
#define BN_ROWS (BN_SLOTS / 64)         /* compaction rows: A 0..3, C 4..5, G 6..7, T 8..9 */
#define BN_SITES 32                     /* sites per fold round: lane = (site, sample) */
#define BN_CHUNK 16                     /* list entries a wave draws at a time */
#define BN_ENT_CAP 6072                 /* runs per wave: a whole site always fits an empty list */
#define BN_FK_ZERO 256
static_assert(BN_ENT_CAP >= 2 * (BN_SLOTS + SS_BINS_MAXN / 511 + 1), "a site's runs fit an empty list");

struct alignas(16) BinsLds {
    uint32_t hist[2][BN_SLOTS];          /* tumor, normal: one 32-bit count per slot (both strands of a
                                            minq in different words: fewer lanes on one LDS address) */
    uint32_t slut[32];                   /* read nt16 | strand << 4: histogram byte offset of its minq-0 slot
                                            << 8 | log2(bytes per minq) */
    union {
        uint16_t ent[BN_ENT_CAP];        /* runs: q | strand << 6 | count << 7 */
        SlotRes  res[2 * BN_SITES];      /* after a round's fold: its results, for the decision */
    };
    uint16_t u_gs[2 * BN_SITES][6];      /* unit: first run of groups 0..3, then the unit's end */
    uint32_t u_cnt[2 * BN_SITES][4];     /* unit: contributing reads per group */
    uint32_t u_rms[2 * BN_SITES];        /* unit: rms sum (< 2^16 reads x 3600) */
    uint32_t u_n[2 * BN_SITES];          /* unit: non-deleted depth */
    uint32_t s_site[BN_SITES];
    uint32_t s_refc[BN_SITES];           /* ref char | nt16 << 8 */
};

/* Histogram slots of one sample.  A read of minq < 64 whose clamped q is > 0
 * (sniper_maqcns.c:165-166) counts in
 *   group A (base 0):   4 minq + 2 hasbase + strand       (256 slots)
 *   group C, G, T:      gb + 2 minq + strand, gb = 128 (base + 1), hasbase = 1
 * and the fold walks a group from its top slot down: the reference's
 * descending key order (:144-157) up to swaps of reads with equal (q, strand).
 * For minq < 4 the key's baseQ bits order reads further (E = baseQ >> 6 and
 * baseQ & 0x3f != 0 set q, deep_bin); with baseQ < 64 they are all q = 4 and
 * need no more slots.  A read of minq >= 64, or of minq < 4 and baseQ >= 64,
 * sends its site to ss_score_wild (never produced by short-read aligners). */
__device__ __forceinline__ uint32_t bn_gbase(uint32_t g) { return g ? 128u * (g + 1u) : 0u; }

/* the lookup rows for a site of reference code ref16: lane = strand << 4 |
 * read nt16 (bam_nt16_nt4_table semantics, :153-154: '=' is the reference,
 * N / IUPAC count as A without hasbase) */
__device__ __forceinline__ void bn_slut_build(BinsLds &B, uint32_t ref16)
{
    const uint32_t lane = lane_id();
    const uint32_t st = (lane >> 4) & 1u, nt16 = lane & 15u;
    const uint32_t code = nt16 ? nt16 : ref16;
    const uint32_t nt4 = code == 1u ? 0u : code == 2u ? 1u : code == 4u ? 2u : code == 8u ? 3u : 4u;
    const uint32_t hb = nt4 < 4u ? 1u : 0u, base = hb ? nt4 : 0u;
    /* byte offset of the read's minq-0 slot: A 4 (2 hasbase + strand), else
     * 4 (gb + strand); bytes per minq: A 16, else 8 */
    const uint32_t wb = base ? 4u * (bn_gbase(base) + st) : 4u * (2u * hb + st);
    if (lane < 32u) B.slut[lane] = wb << 8 | (base ? 3u : 4u);
}

/* run code (q | strand << 6) of a slot of group g: q = max(minq, 4) */
__device__ __forceinline__ uint32_t bn_code(uint32_t slot, uint32_t g)
{
    const uint32_t minq = g ? (slot - bn_gbase(g)) >> 1 : slot >> 2;
    return max(minq, 4u) | (slot & 1u) << 6;
}

/* eight reads per lane from reads[i0 ..] (lane + 64 j), indices clamped to
 * the last read so no load is predicated; none for an empty sample */
__device__ __forceinline__ void bn_issue(const uint32_t *reads, uint32_t n, uint32_t i0, uint32_t (&rd)[8])
{
    const uint32_t lane = lane_id();
    if (n) {                                          /* wave-uniform */
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) rd[j] = __builtin_nontemporal_load(reads + min(i0 + lane + j * 64u, n - 1u));
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) rd[j] = 0u;
    }
}

/* eight reads of one sample (rd[j] = read i0 + lane + 64 j) into its histogram */
__device__ __forceinline__ void bn_count8(const uint32_t (&rd)[8], uint32_t i0, uint32_t n, const uint32_t *slut,
                                          uint32_t cap, char *hb, uint32_t &rs, bool &wild)
{
    const uint32_t lane = lane_id();
    /* the eight lookups first, then the addresses (pinned in registers: the
     * compiler would otherwise sink each lookup into its atomic's branch and
     * wait for it there), then the atomics */
    uint32_t x[8], addr[8];
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) {
        x[j] = i0 + lane + j * 64u < n ? rd[j] : 0u;          /* 0: no contribution, no rms */
        addr[j] = slut[(x[j] >> 16) & 31u];
    }
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) {
        const uint32_t minq = min(x[j] & 0xffu, (x[j] >> 8) & 0xffu);
        addr[j] = (addr[j] >> 8) + (minq << (addr[j] & 31u));
        asm volatile("" : "+v"(addr[j]));
    }
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) {
        const uint32_t bq = (x[j] >> 8) & 0xffu;
        const uint32_t minq = min(x[j] & 0xffu, bq);
        const uint32_t t = min(x[j] & 0x7fu, cap);
        rs += t * t;
        const bool w = minq >= 64u || (minq < 4u && bq >= 64u);
        wild |= w;
        if (bq != 0u && !w) atomicAdd(reinterpret_cast<uint32_t *>(hb + addr[j]), 1u);
    }
}

/* one sample's reads into its (zeroed) histogram: the first 512 arrive in
 * `pre` (issued one site ahead and used in place: a register copy of loads
 * in flight would wait for every younger load, the next site's among them),
 * the rest 512 at a time, double-buffered; adds the rms terms (:173-174) to rs; true when a
 * read needs ss_score_wild */
__device__ __forceinline__ bool bn_pass(const uint32_t *reads, uint32_t n, const uint32_t (&pre)[8],
                                        const uint32_t *slut, uint32_t cap, uint32_t *hist, uint32_t &rs)
{
    bool wild = false;
    char *hb = reinterpret_cast<char *>(hist);
    if (n) bn_count8(pre, 0u, n, slut, cap, hb, rs, wild);
    if (n > 8u * 64u) {                               /* deep samples: each batch issued before the one before it is counted */
        uint32_t rd[8];
        bn_issue(reads, n, 8u * 64u, rd);
        for (uint32_t i0 = 8u * 64u; i0 < n; i0 += 8u * 64u) {
            uint32_t nx[8];
            const bool more = i0 + 8u * 64u < n;
            if (more) bn_issue(reads, n, i0 + 8u * 64u, nx);
            bn_count8(rd, i0, n, slut, cap, hb, rs, wild);
            if (more) {
#pragma unroll
                for (uint32_t j = 0; j < 8u; ++j) rd[j] = nx[j];
            }
        }
    }
    return wild;
}

/* a unit's histogram as runs in the fold's walk order -- groups A, C, G, T,
 * each from its top slot down (the reference's descending key walk) --
 * appended at ent[pos ..] (writes stop at BN_ENT_CAP; the caller checks the
 * returned end); the groups' first runs go to gs[0..3], the end to gs[4],
 * their contributing reads to cnt[0..3] (wave-uniform); returns the new end.
 * Row r holds walk positions 64 r + lane. */
__device__ __forceinline__ uint32_t bn_runs(const uint32_t *hist, uint16_t *ent, uint32_t pos, uint32_t (&gs)[5],
                                            uint32_t (&cnt)[4])
{
    const uint32_t lane = lane_id();
    uint32_t part = 0;
#pragma unroll
    for (uint32_t r = 0; r < BN_ROWS; ++r) {
        const uint32_t g = r < 4u ? 0u : (r - 2u) >> 1;
        const uint32_t r0 = g ? 2u * g + 2u : 0u;            /* the group's first row */
        const uint32_t gb = bn_gbase(g), gsz = g ? 128u : 256u;
        if (r == r0) gs[g] = pos;
        const uint32_t slot = gb + gsz - 1u - (64u * (r - r0) + lane);
        const uint32_t c = hist[slot];
        const uint32_t code = bn_code(slot, g);
        if (!__ballot(c > 511u)) {
            const uint64_t m = __ballot(c != 0u);
            const uint32_t off = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (c && pos + off < BN_ENT_CAP) ent[pos + off] = (uint16_t)(code | c << 7);
            pos += (uint32_t)__popcll(m);
        } else {                                   /* a bin of more than 511 reads: several runs */
            const uint32_t ne = (c + 510u) / 511u;
            const uint32_t incl = wave_scan(ne);
            uint32_t o = pos + incl - ne;
            for (uint32_t left = c; left;) {
                const uint32_t x = min(left, 511u);
                if (o < BN_ENT_CAP) ent[o] = (uint16_t)(code | x << 7);
                ++o;
                left -= x;
            }
            pos += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        part += c;
        if (r == 3u || r == 5u || r == 7u || r == 9u) {
            cnt[g] = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan(part), 63);
            part = 0;
        }
    }
    gs[4] = pos;
    return pos;
}

/* one group chain of a unit from its runs ent[e0 ..] (T reads), one read per
 * step: e = (float)((double)e + fk[w] * q), f = (float)((double)f + fk[w])
 * (sniper_maqcns.c:167-170) with per-strand w counters (16-bit fields of W,
 * saturated at 255 where used).  The wave steps to its longest chain; a lane
 * past its own reads adds fk's zero entry (x + 0.0 == x).  Software
 * pipelined: step t + 1 is decoded and its fk[w] read from LDS before step
 * t's float arithmetic, so the LDS latency hides under it. */
struct BnCur {
    uint32_t rem, q, sh, ptr, nxt;
};

/* decode step t of a chain (advancing to the next run when the current one
 * is used up) and return its fk index */
__device__ __forceinline__ uint32_t bn_step_idx(const uint16_t *ent, BnCur &c, uint32_t W, uint32_t t, uint32_t T)
{
    const bool live = t < T;
    const bool take = c.rem == 0u && live;
    c.q = take ? (c.nxt & 63u) : c.q;
    c.sh = take ? ((c.nxt >> 2) & 16u) : c.sh;          /* strand << 4 */
    c.rem = take ? (c.nxt >> 7) : c.rem;
    c.ptr += take ? 1u : 0u;
    c.nxt = ent[c.ptr];
    c.rem -= live ? 1u : 0u;
    const uint32_t w = __builtin_amdgcn_ubfe(W, c.sh, 16u);
    return live ? min(w, 255u) : (uint32_t)BN_FK_ZERO;
}

__device__ __forceinline__ void bn_chain(const uint16_t *ent, uint32_t e0, uint32_t T, const double *fk, float &e,
                                         float &f)
{
    e = 0.0f;
    f = 0.0f;
    const uint32_t Tm = wave_max(T);
    if (Tm == 0u) return;
    BnCur c = {0u, 0u, 0u, e0, ent[e0]};
    uint32_t W = 0;
    double fv = fk[bn_step_idx(ent, c, W, 0u, T)];
    uint32_t qc = c.q, shc = c.sh;
    for (uint32_t t = 0; t < Tm; ++t) {
        W += 1u << shc;                                     /* step t's strand counter */
        const double fvn = fk[bn_step_idx(ent, c, W, t + 1u, T)];
        e = (float)((double)e + fv * (double)qc);
        f = (float)((double)f + fv);
        fv = fvn;
        qc = c.q;
        shc = c.sh;
    }
}

/* fold, likelihoods, quantisation and the decision for the round's sites.
 * Inlined at its one call site: kernarg_args() reads the kernel's argument
 * segment, whose pointer a called (not inlined) function does not have. */
__device__ __forceinline__ void bn_round(BinsLds &B, uint32_t nsite, const double *fk, const int16_t *qtab)
{
    const ss_score_args &a = kernarg_args();
    const uint32_t lane = lane_id();
    const bool act = lane < 2u * nsite;
    const uint32_t u = act ? lane : 0u;
    uint32_t cnt[4], gs[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        cnt[g] = act ? B.u_cnt[u][g] : 0u;
        gs[g] = B.u_gs[u][g];
    }
    uint32_t L = 0;
#pragma unroll
    for (uint32_t b = 1; b < 4; ++b) L = cnt[b] > (L == 0 ? cnt[0] : (L == 1 ? cnt[1] : cnt[2])) ? b : L;
    float es[4], fs[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        /* the largest group first, then the other three */
        const uint32_t g = i == 0 ? L : (i - 1u) + ((i - 1u) >= L ? 1u : 0u);
        const uint32_t e0 = g == 0 ? gs[0] : (g == 1 ? gs[1] : (g == 2 ? gs[2] : gs[3]));
        const uint32_t T = g == 0 ? cnt[0] : (g == 1 ? cnt[1] : (g == 2 ? cnt[2] : cnt[3]));
        float e, f;
        bn_chain(B.ent, e0, T, fk, e, f);
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b)
            if (b == g) { es[b] = e; fs[b] = f; }
    }
    uint32_t c[4];
    const uint32_t tot = rescale_counts(cnt, c);
    float p[10];
    geno_p5(0u, es, fs, c, tot, a.m, p);
    geno_p5(1u, es, fs, c, tot, a.m, p + 5);
    if (act) {
        const uint32_t n = B.u_n[u];
        uint32_t lk[10], min_lk, rms_q, cns;
        glf_finish(p, es, n, B.u_rms[u], a.m, lk, min_lk, rms_q, cns);
        SlotRes &r = B.res[u];
        uint32_t *rw = reinterpret_cast<uint32_t *>(r.lk);
        rw[0] = lk[0] | lk[1] << 8 | lk[2] << 16 | lk[3] << 24;
        rw[1] = lk[4] | lk[5] << 8 | lk[6] << 16 | lk[7] << 24;
        rw[2] = lk[8] | lk[9] << 8;
        r.cns = cns;
        r.depth = n;
        if (a.glf) {
            const uint32_t sl = u >> 1;
            store_glf(&a.glf[2ull * B.s_site[sl] + (u & 1u)], B.s_refc[sl] >> 8, lk, min_lk, rms_q, n);
        }
    }
    wave_sync();
    if (lane < nsite) decide_site(a, qtab, B.s_site[lane], B.s_refc[lane], B.res[2u * lane], B.res[2u * lane + 1u]);
    wave_sync();
}

/* a counted site's units (its runs are written) as round slot i */
__device__ __forceinline__ void bn_unit_info(BinsLds &B, uint32_t i, uint32_t s, uint32_t refc, uint32_t ref16,
                                             uint32_t nt, uint32_t nn, uint32_t rts, uint32_t rns,
                                             const uint32_t (&gsT)[5],
                                             const uint32_t (&gsN)[5], const uint32_t (&cT)[4],
                                             const uint32_t (&cN)[4])
{
    if (lane_id() == 0u) {
        const uint32_t uT = 2u * i, uN = uT + 1u;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            B.u_gs[uT][g] = (uint16_t)gsT[g];
            B.u_gs[uN][g] = (uint16_t)gsN[g];
            B.u_cnt[uT][g] = cT[g];
            B.u_cnt[uN][g] = cN[g];
        }
        B.u_gs[uT][4] = (uint16_t)gsT[4];
        B.u_gs[uN][4] = (uint16_t)gsN[4];
        B.u_rms[uT] = rts;
        B.u_rms[uN] = rns;
        B.u_n[uT] = nt;
        B.u_n[uN] = nn;
        B.s_site[i] = s;
        B.s_refc[i] = refc | ref16 << 8;
    }
    wave_sync();
}

/* descriptors of a chunk of the wave's list, lane i < BN_CHUNK = entry i */
struct BnDesc {
    uint32_t s, ot, on, nt, nn;
    uint32_t fl;                             /* usable (well formed, <= SS_BINS_MAXN per sample) | ref << 8 | nt16 << 16 */
};

/* lane i's copy of a descriptor, wave-uniform */
__device__ __forceinline__ uint32_t bn_rl(uint32_t v, uint32_t i)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i);
}

/* draw the next chunk of the list from the kernel's counter and load its
 * descriptors into lanes 0 .. BN_CHUNK - 1 (not waited for); returns its
 * entries, 0 at the end of the list */
__device__ __forceinline__ uint32_t bn_grab_desc(uint32_t count, BnDesc &d)
{
    const uint32_t lane = lane_id();
    const ss_score_args &k = kernarg_args();
    uint32_t ch = 0;
    if (lane == 0u) ch = atomicAdd(k.deep_next, 1u);
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ch) * BN_CHUNK;
    if (c0 >= count) return 0u;
    const uint32_t len = min(count - c0, (uint32_t)BN_CHUNK);
    const uint32_t end_t = k.off_t[k.n_sites], end_n = k.off_n[k.n_sites];
    const uint32_t e = c0 + min(lane, len - 1u);
    const uint32_t st = k.deep2_list[e];
    const uint32_t ot = k.off_t[st], ot1 = k.off_t[st + 1], on = k.off_n[st], on1 = k.off_n[st + 1];
    const uint32_t rc = k.ref[st];
    const bool ok = site_wellformed(ot, ot1, end_t) && site_wellformed(on, on1, end_n) && ot1 - ot <= SS_BINS_MAXN &&
                    on1 - on <= SS_BINS_MAXN;
    d.s = st;
    d.ot = ot;
    d.on = on;
    d.nt = ok ? ot1 - ot : 0u;
    d.nn = ok ? on1 - on : 0u;
    d.fl = (ok ? 1u : 0u) | rc << 8 | (uint32_t)ss_tab_nt16(k.m)[rc] << 16;
    return len;
}

/* hand a site on to ss_score_wild */
__device__ __forceinline__ void bn_to_wild(uint32_t s)
{
    const ss_score_args &k = kernarg_args();
    if (lane_id() == 0u) {
        const uint32_t d = atomicAdd(k.deep3_count, 1u);
        if (d < k.deep_cap) k.deep3_list[d] = s;
        else atomicOr(k.err, SS_KERR_DEEP_OVERFLOW);
    }
}

}  // namespace

__global__ __launch_bounds__(SS_DEEP_BLOCK) void ss_score_deep(ss_score_args a)
{
    __shared__ double fk[BN_FK_ZERO + 1];
    __shared__ int16_t qtab[1024];                  /* qAddTable, as in ss_score_main */
    __shared__ BinsLds BL[BN_WAVES];
    const uint32_t count0 = *a.deep2_count;
    const uint32_t count = count0 < a.deep_cap ? count0 : a.deep_cap;
    if (count == 0u) return;
    for (uint32_t i = threadIdx.x; i <= BN_FK_ZERO; i += blockDim.x) fk[i] = i < 256u ? ss_tab_fk(a.m)[i] : 0.0;
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) qtab[i] = (int16_t)ss_tab_qadd(a.m)[i];
    __syncthreads();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    BinsLds &B = BL[wv];
    const uint32_t lane = lane_id();
    const uint32_t cap = (uint32_t)a.m.cap_mapQ;
    /* Descriptors of a chunk of BN_CHUNK list entries sit in lanes 0..15 (one
     * entry per lane, read out with readlane), the next chunk's are loaded
     * while this one is scored, and the next site's first reads while the
     * site before it is counted: no dependent load chain per site. */
    BnDesc D, ND;
    uint32_t clen = bn_grab_desc(count, D);         /* entries of the current chunk (uniform) */
    uint32_t nlen = clen ? bn_grab_desc(count, ND) : 0u;
    uint32_t idx = 0;                               /* the next entry of the current chunk */
    uint32_t nsite = 0, nent = 0;                   /* the current round */
    /* the site whose histograms are built (s, depths, reference, rms sums) */
    uint32_t s = 0, nt = 0, nn = 0, refc = 0, ref16 = 0;
    uint32_t rts = 0, rns = 0;
    /* the first 512 reads per sample of the next site */
    uint32_t pft[8], pfn[8];
    if (clen) {
        const ss_score_args &k = kernarg_args();
        bn_issue(k.reads_t + bn_rl(D.ot, 0u), bn_rl(D.nt, 0u), 0u, pft);
        bn_issue(k.reads_n + bn_rl(D.on, 0u), bn_rl(D.nn, 0u), 0u, pfn);
    }
    /* one bn_round call site: each iteration counts a site, writes its runs
     * when they fit the round, and folds the round when it is full, when the
     * site's runs did not fit (they are written again behind the folded
     * round: the histograms stay), or at the end of the list */
    for (;;) {
        bool ready = false;
        if (clen && idx == clen) {                  /* the next chunk becomes the current one */
            D = ND;
            clen = nlen;
            idx = 0;
            nlen = clen ? bn_grab_desc(count, ND) : 0u;
        }
        const bool end = clen == 0u;
        if (!end) {
            const ss_score_args &k = kernarg_args();
            s = bn_rl(D.s, idx);
            const uint32_t ot = bn_rl(D.ot, idx), on = bn_rl(D.on, idx);
            nt = bn_rl(D.nt, idx);
            nn = bn_rl(D.nn, idx);
            const uint32_t fl = bn_rl(D.fl, idx);
            ++idx;
            uint32_t pt[8], pn[8];
#pragma unroll
            for (uint32_t j = 0; j < 8u; ++j) { pt[j] = pft[j]; pn[j] = pfn[j]; }
            /* the next site's first reads go out now: the chunk's next entry,
             * or the next chunk's first */
            if (idx < clen) {
                bn_issue(k.reads_t + bn_rl(D.ot, idx), bn_rl(D.nt, idx), 0u, pft);
                bn_issue(k.reads_n + bn_rl(D.on, idx), bn_rl(D.nn, idx), 0u, pfn);
            } else if (nlen) {
                bn_issue(k.reads_t + bn_rl(ND.ot, 0u), bn_rl(ND.nt, 0u), 0u, pft);
                bn_issue(k.reads_n + bn_rl(ND.on, 0u), bn_rl(ND.nn, 0u), 0u, pfn);
            }
            if (!(fl & 1u)) {
                bn_to_wild(s);                         /* it reports malformed offsets (-2) */
            } else {
                refc = (fl >> 8) & 0xffu;
                ref16 = fl >> 16;
                bn_slut_build(B, ref16);
                {
                    uint4 *h4 = reinterpret_cast<uint4 *>(&B.hist[0][0]);
                    for (uint32_t i = lane; i < BN_SLOTS / 2u; i += 64u) h4[i] = make_uint4(0u, 0u, 0u, 0u);
                }
                wave_sync();
                uint32_t rt = 0, rn = 0;
                bool wild = bn_pass(k.reads_t + ot, nt, pt, B.slut, cap, B.hist[0], rt);
                wild |= bn_pass(k.reads_n + on, nn, pn, B.slut, cap, B.hist[1], rn);
                if (__ballot(wild)) {                  /* ss_score_wild's windows and baseQ bins */
                    bn_to_wild(s);
                } else {
                    rts = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan(rt), 63);   /* rms sums */
                    rns = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan(rn), 63);
                    wave_sync();
                    ready = true;
                }
            }
        }
        uint32_t gsT[5], gsN[5], cT[4], cN[4];
        if (ready && nsite < BN_SITES) {
            const uint32_t e2 = bn_runs(B.hist[1], B.ent, bn_runs(B.hist[0], B.ent, nent, gsT, cT), gsN, cN);
            if (e2 <= BN_ENT_CAP) {
                bn_unit_info(B, nsite, s, refc, ref16, nt, nn, rts, rns, gsT, gsN, cT, cN);
                ++nsite;
                nent = e2;
                ready = false;
            }
        }
        if (ready || nsite == BN_SITES || (end && nsite)) {
            bn_round(B, nsite, fk, qtab);
            nsite = 0;
            nent = 0;
            if (ready) {
                nent = bn_runs(B.hist[1], B.ent, bn_runs(B.hist[0], B.ent, 0u, gsT, cT), gsN, cN);
                bn_unit_info(B, 0u, s, refc, ref16, nt, nn, rts, rns, gsT, gsN, cT, cN);
                nsite = 1;
            }
        }
        if (end && nsite == 0u) break;
    }
}

/* --------------------------------------------------------------------------
 * Synthetic generator (device twin of ss_synth.c; same ss_synth_core.h code).
 * ------------------------------------------------------------------------ */
/* depths per site, and their 64-bit totals into sums[0..1] (the host checks
 * that the 32-bit read offsets cannot wrap) */
__global__ void ss_synth_depth_kernel(ss_synth_k_t k, uint64_t first, uint64_t n, uint8_t *ref,
                                      uint32_t *dt, uint32_t *dn, unsigned long long *sums)
{
    unsigned long long st = 0, sn = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        ss_site_draw_t d;
        uint32_t j, r, c;
        ss_synth_site(&k, first + i, &d);
        ref[i] = d.ref_char;
        for (j = c = 0; j < d.raw_tumor; ++j) c += (uint32_t)ss_synth_read(&k, first + i, &d, 0, j, &r);
        dt[i] = c;
        st += c;
        for (j = c = 0; j < d.raw_normal; ++j) c += (uint32_t)ss_synth_read(&k, first + i, &d, 1, j, &r);
        dn[i] = c;
        sn += c;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        st += __shfl_xor(st, o);
        sn += __shfl_xor(sn, o);
    }
    if (__lane_id() == 0) {
        atomicAdd(&sums[0], st);
        atomicAdd(&sums[1], sn);
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
 * Table fingerprint: the context's device table image as three position-keyed
 * word sums (coef, lhet, everything after lhet), the same function as the
 * host's ss_tab_fp_words (ss_tables.c).  ss_ctx_create and ss_ctx_check compare
 * them with the host's sums, so a device table that no longer holds what was
 * uploaded is reported (SS_E_TABLES) instead of scoring silently wrong.
 * ------------------------------------------------------------------------ */
__device__ __forceinline__ unsigned long long fp_mix(unsigned long long x)
{
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void ss_tab_fingerprint(const unsigned long long *w, unsigned long long *out)
{
    constexpr size_t NW = SS_TAB_BYTES / 8, W_LHET = SS_TAB_LHET / 8, W_REST = SS_TAB_FK / 8;
    unsigned long long s0 = 0, s1 = 0, s2 = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NW; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned long long v = fp_mix(w[i] + (unsigned long long)i * 0x9e3779b97f4a7c15ull);
        if (i < W_LHET) s0 += v;
        else if (i < W_REST) s1 += v;
        else s2 += v;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_xor(s0, o);
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
    }
    if ((threadIdx.x & 63u) == 0u) {
        atomicAdd(&out[0], s0);
        atomicAdd(&out[1], s1);
        atomicAdd(&out[2], s2);
    }
}
static_assert(SS_TAB_BYTES % 8 == 0 && SS_TAB_LHET % 8 == 0 && SS_TAB_FK % 8 == 0, "table words");

/* --------------------------------------------------------------------------
 * launchers
 * ------------------------------------------------------------------------ */
int ss_launch_tab_fingerprint(const uint8_t *tab, unsigned long long *out3, hipStream_t s)
{
    hipLaunchKernelGGL(ss_tab_fingerprint, dim3(1024), dim3(256), 0, s, (const unsigned long long *)tab, out3);
    return (int)hipGetLastError();
}

#ifdef SS_DEBUG_SYNC
/* A/B builds only: wait for each kernel and name the one that failed */
#define SS_DBG_SYNC(name)                                                                          \
    do {                                                                                           \
        hipError_t de = hipStreamSynchronize(s);                                                   \
        if (de != hipSuccess) {                                                                    \
            fprintf(stderr, "[sniper_amd debug] %s: %s\n", name, hipGetErrorString(de));           \
            return (int)de;                                                                        \
        }                                                                                          \
    } while (0)
#else
#define SS_DBG_SYNC(name) do { } while (0)
#endif

int ss_launch_score(const ss_score_args &a, int triage_grid, int triage_deep_grid, int main_grid, int wide_grid,
                    int deep_grid, int wild_grid, hipStream_t s, const hipEvent_t *ev)
{
    hipError_t e;
    if (ev) (void)hipEventRecord(ev[0], s);
    if (a.tri_list) {
        hipLaunchKernelGGL(ss_score_triage, dim3(triage_grid), dim3(SS_TRIAGE_BLOCK), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
        SS_DBG_SYNC("ss_score_triage");
        hipLaunchKernelGGL(ss_score_triage_deep, dim3(triage_deep_grid), dim3(SS_TRIAGE_DEEP_BLOCK), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
        SS_DBG_SYNC("ss_score_triage_deep");
    }
    hipLaunchKernelGGL(ss_score_main, dim3(main_grid), dim3(SS_MAIN_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    SS_DBG_SYNC("ss_score_main");
    if (ev) (void)hipEventRecord(ev[1], s);
    hipLaunchKernelGGL(ss_score_group, dim3(wide_grid), dim3(SS_WIDE_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    SS_DBG_SYNC("ss_score_group");
    if (ev) (void)hipEventRecord(ev[2], s);
    hipLaunchKernelGGL(ss_score_deep, dim3(deep_grid), dim3(SS_DEEP_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    SS_DBG_SYNC("ss_score_deep");
    hipLaunchKernelGGL(ss_score_wild, dim3(wild_grid), dim3(SS_WILD_BLOCK), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    if (ev) (void)hipEventRecord(ev[3], s);
    return (int)hipSuccess;
}

int ss_launch_synth_depth(const ss_synth_k_t &k, uint64_t first, uint64_t n, uint8_t *ref,
                          uint32_t *dt, uint32_t *dn, unsigned long long *sums, hipStream_t s)
{
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(ss_synth_depth_kernel, dim3((unsigned)blocks), dim3(256), 0, s, k, first, n,
                       ref, dt, dn, sums);
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


