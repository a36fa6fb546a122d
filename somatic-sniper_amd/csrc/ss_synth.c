/*
 * ss_synth.c -- host side of the deterministic synthetic pileup generator.
 *
 * ss_synth_prepare() turns the public ss_synth_t (probabilities, Poisson means)
 * into the integer-only ss_synth_k_t that ss_synth_core.h consumes on both the
 * host and the device; ss_synth_batch_host() fills a CSR site batch.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "sniper_amd.h"
#include "ss_synth.h"

static uint32_t prob_threshold(double p)
{
    if (!(p > 0.0)) return 0u;
    if (p >= 1.0) return 0xffffffffu;
    return (uint32_t)(p * 4294967296.0);
}

void ss_synth_default(ss_synth_t *s, double lambda_tumor, double lambda_normal)
{
    memset(s, 0, sizeof(*s));
    s->seed = 0x5EED5A1DC0FFEE01ull;
    s->lambda_tumor = lambda_tumor;
    s->lambda_normal = lambda_normal;
    s->p_error = 0.01;
    s->p_nbase = 0.001;
    s->p_del = 0.01;
    s->p_mapq60 = 0.9;
    s->baseq_lo = 2;
    s->baseq_hi = 41;
    s->mapq_hi = 60;
    s->p_somatic = 1e-4;
    s->vaf = 0.3;
}

/* cdf[k] = P(X <= k) * 2^32 for X ~ Poisson(lambda); returns the table length. */
static uint32_t poisson_cdf(double lambda, uint32_t *cdf)
{
    double cum = 0.0;
    uint32_t n, k;
    double kmax = ceil(lambda + 12.0 * sqrt(lambda > 0 ? lambda : 0) + 30.0);
    n = kmax >= SS_SYNTH_MAXCDF ? SS_SYNTH_MAXCDF : (uint32_t)kmax + 1u;
    for (k = 0; k < n; ++k) {
        double lp = lambda > 0 ? -lambda + k * log(lambda) - lgamma((double)k + 1.0)
                               : (k == 0 ? 0.0 : -INFINITY);
        cum += exp(lp);
        cdf[k] = cum >= 1.0 ? 0xffffffffu : (uint32_t)(cum * 4294967296.0);
    }
    cdf[n - 1] = 0xffffffffu;
    return n;
}

int ss_synth_prepare(const ss_synth_t *s, ss_synth_k_t *k, uint32_t *cdf_tumor,
                     uint32_t *cdf_normal)
{
    if (!s || !k) return SS_E_INVAL;
    if (s->baseq_hi < s->baseq_lo || s->baseq_lo < 0 || s->baseq_hi > 255 ||
        s->mapq_hi < 0 || s->mapq_hi > 255)
        return SS_E_INVAL;
    if (s->lambda_tumor < 0 || s->lambda_normal < 0) return SS_E_INVAL;
    memset(k, 0, sizeof(*k));
    k->seed = s->seed;
    k->shard = s->shard;
    k->thr_error = prob_threshold(s->p_error);
    k->thr_nbase = prob_threshold(s->p_nbase);
    k->thr_eq = prob_threshold(s->p_eq);
    k->thr_iupac = prob_threshold(s->p_iupac);
    k->thr_del = prob_threshold(s->p_del);
    k->thr_mapq60 = prob_threshold(s->p_mapq60);
    k->thr_wild = prob_threshold(s->p_wild_qual);
    k->thr_somatic = prob_threshold(s->p_somatic);
    k->thr_vaf = prob_threshold(s->vaf);
    k->thr_germ = prob_threshold(s->p_germline);
    k->thr_ref_n = prob_threshold(s->p_ref_n);
    k->thr_ref_lower = prob_threshold(s->p_ref_lower);
    k->thr_ref_iupac = prob_threshold(s->p_ref_iupac);
    k->baseq_lo = (uint32_t)s->baseq_lo;
    k->baseq_span = (uint32_t)(s->baseq_hi - s->baseq_lo + 1);
    k->mapq_span = (uint32_t)(s->mapq_hi + 1);
    k->fixed_depth = s->fixed_depth ? 1u : 0u;
    if (k->fixed_depth) {
        k->depth_tumor = (uint32_t)(s->lambda_tumor + 0.5);
        k->depth_normal = (uint32_t)(s->lambda_normal + 0.5);
        k->ncdf_tumor = k->ncdf_normal = 1;
        cdf_tumor[0] = cdf_normal[0] = 0xffffffffu;
    } else {
        k->ncdf_tumor = poisson_cdf(s->lambda_tumor, cdf_tumor);
        k->ncdf_normal = poisson_cdf(s->lambda_normal, cdf_normal);
    }
    k->cdf_tumor = cdf_tumor;
    k->cdf_normal = cdf_normal;
    return SS_OK;
}

/* Packed (non-deleted) depth of one site, both samples. */
void ss_synth_site_depth(const ss_synth_k_t *k, uint64_t site, uint8_t *ref,
                         uint32_t *dt, uint32_t *dn)
{
    ss_site_draw_t d;
    uint32_t j, r, n;
    ss_synth_site(k, site, &d);
    *ref = d.ref_char;
    for (j = n = 0; j < d.raw_tumor; ++j) n += (uint32_t)ss_synth_read(k, site, &d, 0, j, &r);
    *dt = n;
    for (j = n = 0; j < d.raw_normal; ++j) n += (uint32_t)ss_synth_read(k, site, &d, 1, j, &r);
    *dn = n;
}

void ss_synth_site_reads(const ss_synth_k_t *k, uint64_t site, uint32_t *rt, uint32_t *rn)
{
    ss_site_draw_t d;
    uint32_t j, r;
    ss_synth_site(k, site, &d);
    for (j = 0; j < d.raw_tumor; ++j)
        if (ss_synth_read(k, site, &d, 0, j, &r)) *rt++ = r;
    for (j = 0; j < d.raw_normal; ++j)
        if (ss_synth_read(k, site, &d, 1, j, &r)) *rn++ = r;
}

int ss_synth_batch_host(const ss_synth_t *s, uint64_t first_site, uint64_t n_sites,
                        uint8_t *ref, uint32_t *off_tumor, uint32_t *off_normal,
                        uint32_t *reads_tumor, uint32_t *reads_normal,
                        uint64_t *n_reads_tumor, uint64_t *n_reads_normal)
{
    ss_synth_k_t k;
    uint32_t *cdf = (uint32_t *)malloc(2u * SS_SYNTH_MAXCDF * sizeof(uint32_t));
    uint64_t i, at = 0, an = 0;
    int rc;
    if (!cdf) return SS_E_NOMEM;
    if (!ref || !off_tumor || !off_normal) { free(cdf); return SS_E_INVAL; }
    rc = ss_synth_prepare(s, &k, cdf, cdf + SS_SYNTH_MAXCDF);
    if (rc) { free(cdf); return rc; }
    for (i = 0; i < n_sites; ++i) {
        uint32_t dt, dn;
        ss_synth_site_depth(&k, first_site + i, &ref[i], &dt, &dn);
        if (at + dt > 0xffffffffull || an + dn > 0xffffffffull) { free(cdf); return SS_E_INVAL; }
        off_tumor[i] = (uint32_t)at;
        off_normal[i] = (uint32_t)an;
        at += dt;
        an += dn;
    }
    off_tumor[n_sites] = (uint32_t)at;
    off_normal[n_sites] = (uint32_t)an;
    if (n_reads_tumor) *n_reads_tumor = at;
    if (n_reads_normal) *n_reads_normal = an;
    if (reads_tumor && reads_normal)
        for (i = 0; i < n_sites; ++i)
            ss_synth_site_reads(&k, first_site + i, reads_tumor + off_tumor[i],
                                reads_normal + off_normal[i]);
    free(cdf);
    return SS_OK;
}
