/*
 * ss_synth_core.h -- counter-based synthetic pileup generator, shared verbatim by
 * the host generator (ss_synth.c, gcc) and the device generator (ss_device.hip),
 * so both produce identical bytes.  Only integer arithmetic happens here; every
 * probability is turned into a u32 threshold once on the host (ss_synth_prepare).
 *
 * Model ("Synthetic inputs"): per site a uniform ACGT ref
 * base; Poisson(lambda) raw depth per sample (clamped >= 1); per read a deletion
 * draw (dropped), base = true allele with a uniform error substitution, N / '=' /
 * IUPAC read bases at small rates, baseQ ~ U[lo,hi], mapQ = 60 w.p. p_mapq60 else
 * U[0,hi]; somatic sites carry an alt allele in the tumor at the given VAF.
 */
#ifndef SS_SYNTH_CORE_H
#define SS_SYNTH_CORE_H

#include <stdint.h>

#ifdef __HIPCC__
#define SS_HD __host__ __device__
#else
#define SS_HD
#endif

#define SS_SYNTH_MAXCDF 8192

typedef struct ss_synth_k {
    uint64_t seed;
    uint32_t shard;
    uint32_t thr_error, thr_nbase, thr_eq, thr_iupac, thr_del, thr_mapq60, thr_wild;
    uint32_t thr_somatic, thr_vaf, thr_germ, thr_ref_n, thr_ref_lower, thr_ref_iupac;
    uint32_t baseq_lo, baseq_span, mapq_span;
    uint32_t fixed_depth, depth_tumor, depth_normal;
    uint32_t ncdf_tumor, ncdf_normal;
    const uint32_t *cdf_tumor;    /* cdf[k] = P(depth <= k) * 2^32, last = 0xffffffff */
    const uint32_t *cdf_normal;
} ss_synth_k_t;

SS_HD static inline uint64_t ss_mix64(uint64_t z)
{
    z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 27; z *= 0x94d049bb133111ebull;
    z ^= z >> 31;
    return z;
}

/* One 64-bit draw keyed by (seed, shard, site, stream, idx). */
SS_HD static inline uint64_t ss_draw(const ss_synth_k_t *k, uint64_t site,
                                     uint32_t stream, uint32_t idx)
{
    uint64_t h = ss_mix64(k->seed + 0x9e3779b97f4a7c15ull * ((uint64_t)k->shard + 1u));
    h = ss_mix64(h ^ (site * 0xd1b54a32d192ed03ull));
    h = ss_mix64(h ^ (((uint64_t)stream << 32) | idx));
    return h;
}

SS_HD static inline uint32_t ss_cdf_pick(const uint32_t *cdf, uint32_t n, uint32_t u)
{
    /* smallest k with u < cdf[k]; cdf is non-decreasing and cdf[n-1] = 0xffffffff */
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}

/* IUPAC two/three-base codes (nt16) used for ambiguous read / ref bases. */
SS_HD static inline uint32_t ss_iupac_nt16(uint32_t u)
{
    /* M R W S Y K V H D B */
    switch (u % 10u) {
    case 0: return 3;  case 1: return 5;  case 2: return 9;  case 3: return 6;
    case 4: return 10; case 5: return 12; case 6: return 7;  case 7: return 11;
    case 8: return 13; default: return 14;
    }
}

typedef struct ss_site_draw {
    uint8_t  ref_char;
    uint32_t ref_nt4;      /* 0..3 true ref allele */
    uint32_t alt_nt4;      /* alt allele for somatic/germline sites */
    uint32_t kind;         /* 0 plain, 1 somatic, 2 germline het */
    uint32_t raw_tumor, raw_normal;
} ss_site_draw_t;

SS_HD static inline void ss_synth_site(const ss_synth_k_t *k, uint64_t site, ss_site_draw_t *d)
{
    const uint64_t h0 = ss_draw(k, site, 0, 0);
    const uint64_t h1 = ss_draw(k, site, 0, 1);
    const uint32_t a = (uint32_t)h0, b = (uint32_t)(h0 >> 32);
    const uint32_t c = (uint32_t)h1, e = (uint32_t)(h1 >> 32);
    const char acgt[4] = {'A', 'C', 'G', 'T'};
    const char iupac[10] = {'M', 'R', 'W', 'S', 'Y', 'K', 'V', 'H', 'D', 'B'};
    uint8_t rc;
    d->ref_nt4 = a & 3u;
    rc = (uint8_t)acgt[d->ref_nt4];
    if (b < k->thr_ref_n) rc = 'N';
    else if (b - k->thr_ref_n < k->thr_ref_iupac) rc = (uint8_t)iupac[(a >> 8) % 10u];
    if (((a >> 16) & 0xffffu) < (k->thr_ref_lower >> 16) && rc >= 'A' && rc <= 'Z')
        rc = (uint8_t)(rc + ('a' - 'A'));
    d->ref_char = rc;
    d->alt_nt4 = (d->ref_nt4 + 1u + (e % 3u)) & 3u;
    d->kind = (c < k->thr_somatic) ? 1u : ((c - k->thr_somatic) < k->thr_germ ? 2u : 0u);
    if (k->fixed_depth) {
        d->raw_tumor = k->depth_tumor;
        d->raw_normal = k->depth_normal;
    } else {
        const uint64_t h2 = ss_draw(k, site, 0, 2);
        d->raw_tumor = ss_cdf_pick(k->cdf_tumor, k->ncdf_tumor, (uint32_t)h2);
        d->raw_normal = ss_cdf_pick(k->cdf_normal, k->ncdf_normal, (uint32_t)(h2 >> 32));
    }
    if (d->raw_tumor < 1u) d->raw_tumor = 1u;
    if (d->raw_normal < 1u) d->raw_normal = 1u;
}

/* Read j of `sample` (0 tumor, 1 normal).  Returns 0 if the read is a deletion
 * (dropped from the packed batch), else 1 with the packed read in *out.
 * Three independent 64-bit draws per read: (deletion, strand/wild),
 * (allele, error class), (error base / baseQ / mapQ). */
SS_HD static inline int ss_synth_read(const ss_synth_k_t *k, uint64_t site,
                                      const ss_site_draw_t *d, uint32_t sample,
                                      uint32_t j, uint32_t *out)
{
    const uint64_t r0 = ss_draw(k, site, 1u + sample, 3u * j);
    const uint32_t u0 = (uint32_t)r0, u1 = (uint32_t)(r0 >> 32);
    uint64_t r1, r2;
    uint32_t u2, u3, u4, u5, allele, nt16, baseq, mapq, strand;
    if (u0 < k->thr_del) return 0;
    r1 = ss_draw(k, site, 1u + sample, 3u * j + 1u);
    r2 = ss_draw(k, site, 1u + sample, 3u * j + 2u);
    u2 = (uint32_t)r1; u3 = (uint32_t)(r1 >> 32);
    u4 = (uint32_t)r2; u5 = (uint32_t)(r2 >> 32);
    allele = d->ref_nt4;
    if ((d->kind == 1u && sample == 0u) || d->kind == 2u)
        if (u2 < k->thr_vaf) allele = d->alt_nt4;
    nt16 = 1u << allele;
    if (u3 < k->thr_error) {
        nt16 = 1u << (u4 & 3u);
    } else {
        uint32_t v = u3 - k->thr_error;
        if (v < k->thr_nbase) nt16 = 15u;
        else if ((v -= k->thr_nbase) < k->thr_eq) nt16 = 0u;
        else if ((v -= k->thr_eq) < k->thr_iupac) nt16 = ss_iupac_nt16(u4 >> 2);
    }
    strand = u1 & 1u;
    if ((u1 >> 1) < (k->thr_wild >> 1)) {
        baseq = (u4 >> 8) & 0xffu;
        mapq = (u4 >> 16) & 0xffu;
    } else {
        baseq = k->baseq_lo + ((u4 >> 8) & 0xffffu) % k->baseq_span;
        mapq = (u5 < k->thr_mapq60) ? 60u : ((u4 >> 24) % k->mapq_span);
    }
    *out = (mapq & 0xffu) | ((baseq & 0xffu) << 8) | (nt16 << 16) | (strand << 20);
    return 1;
}

#endif /* SS_SYNTH_CORE_H */
