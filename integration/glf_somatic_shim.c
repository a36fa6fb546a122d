/*
 * glf_somatic_shim.c -- the reference-side binding of the C ABI.
 *
 * Linked into the reference's OWN bam-somaticsniper (main.c, sniper_pileup.c,
 * output_*.c, samtools 0.1.6 -- unchanged sources) with
 *     -Wl,--wrap=glf_somatic -Wl,--wrap=bam_sspileup_file -Wl,--wrap=makeSoloPrior
 * so that the per-site callback main.c:146 hands to bam_sspileup_file
 * (glf_somatic, somatic_sniper.c:109, type bam_sspileup_f somatic_sniper.h:42)
 * becomes a batching shim over ss_score_batch_host (include/sniper_amd.h):
 *
 *   __wrap_glf_somatic        copies the site (ref char, packed non-deleted
 *                             reads of both samples) into a host batch; the
 *                             pileup arrays are only valid during the call
 *                             (sniper_pileup.c:194-199), so nothing is kept
 *                             by pointer.  Flushes when the batch is full.
 *   __wrap_bam_sspileup_file  runs the reference's dual pileup, then flushes.
 *   __wrap_makeSoloPrior      records that -p was NOT given (main.c keeps
 *                             use_priors in a local, main.c:117-120).
 *
 * A flush scores the batch on the GPU and writes every emitted site, in
 * (tid, pos) order, through the reference's own output formatter
 * (output_formatter_write, output_format.c) with the per-sample depth and
 * quality statistics computed from the packed reads (ss_dqstats below, the
 * get_dqstats rules of dqstats.c:6-53).  The callback's return value is
 * ignored by its caller (sniper_pileup.c:258); the shim returns 0.
 *
 * Environment: SS_DEVICE (default 0), SS_SHIM_BATCH (sites per flush).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "somatic_sniper.h"
#include "output_format.h"
#include "dqstats.h"
#include "sniper_amd.h"

int  __real_bam_sspileup_file(bamFile fp1, bamFile fp2, int mask, int thresh, bam_sspileup_f func,
                              void *func_data, FILE *snp_fh);
void __real_makeSoloPrior(void);

typedef struct {
    size_t    n, cap;          /* sites */
    size_t    nt, capt, nn, capn;
    uint8_t  *ref;
    uint32_t *off_t, *off_n;
    uint32_t *reads_t, *reads_n;
    uint32_t *tid, *pos;
    int32_t  *score;
    ss_call_t *calls;
    size_t    calls_cap;
} shim_batch_t;

static ss_ctx_t    *g_ctx;
static shim_batch_t g_b;
static int          g_use_priors;
static pu_data2_t  *g_d;
static FILE        *g_fh;

static void die(const char *what, int rc)
{
    fprintf(stderr, "[sniper_amd shim] %s failed: %s\n", what, ss_strerror(rc));
    exit(1);
}

static void *grow(void *p, size_t *cap, size_t need, size_t elem)
{
    if (need <= *cap) return p;
    size_t c = *cap ? *cap : 1024;
    while (c < need) c *= 2;
    p = realloc(p, c * elem);
    if (!p) { fprintf(stderr, "[sniper_amd shim] out of memory\n"); exit(1); }
    *cap = c;
    return p;
}

void __wrap_makeSoloPrior(void)
{
    g_use_priors = 1;
    __real_makeSoloPrior();
}

static void shim_init(pu_data2_t *d)
{
    ss_params_t p;
    ss_params_default(&p);
    p.theta = d->c->theta;
    p.n_hap = d->c->n_hap;
    p.het_rate = d->c->het_rate;
    p.eta = d->c->eta;
    p.cap_mapQ = d->c->cap_mapQ;
    p.min_somatic_qual = d->min_somatic_qual;
    p.use_priors = g_use_priors;
    p.use_joint_priors = d->use_joint_priors;
    p.somatic_rate = d->somatic_mutation_rate;
    p.include_loh = d->include_loh;
    p.include_gor = d->include_gor;
    const char *dev = getenv("SS_DEVICE");
    int rc = ss_ctx_create(&p, dev ? atoi(dev) : 0, &g_ctx);
    if (rc) die("ss_ctx_create", rc);
    const char *bs = getenv("SS_SHIM_BATCH");
    g_b.cap = 0;
    size_t want = bs ? (size_t)atol(bs) : ((size_t)1 << 20);
    g_b.ref = grow(NULL, &g_b.cap, want, 1);
    size_t c = 0; g_b.tid = grow(NULL, &c, g_b.cap, 4);
    c = 0; g_b.pos = grow(NULL, &c, g_b.cap, 4);
    c = 0; g_b.score = grow(NULL, &c, g_b.cap, 4);
    c = 0; g_b.off_t = grow(NULL, &c, g_b.cap + 1, 4);
    c = 0; g_b.off_n = grow(NULL, &c, g_b.cap + 1, 4);
    g_b.off_t[0] = g_b.off_n[0] = 0;
    g_b.calls_cap = 0;   /* emitted calls are only collected into a non-empty buffer */
    g_b.calls = grow(NULL, &g_b.calls_cap, 4096, sizeof(ss_call_t));
    g_d = d;
}

/* one packed u32 per read glfgen would use (sniper_maqcns.c:146-154) */
static size_t pack(const bam_pileup1_t *pl, int n, uint32_t **dst, size_t *len, size_t *cap)
{
    *dst = grow(*dst, cap, *len + (size_t)n, 4);
    size_t k = 0;
    for (int i = 0; i < n; ++i) {
        const bam_pileup1_t *p = pl + i;
        if (p->is_del || (p->b->core.flag & BAM_FUNMAP)) continue;
        (*dst)[*len + k++] = SS_READ_PACK(p->b->core.qual, bam1_qual(p->b)[p->qpos],
                                          bam1_seqi(bam1_seq(p->b), p->qpos), bam1_strand(p->b));
    }
    *len += k;
    return k;
}

/* get_dqstats (dqstats.c:6-53) over packed reads: deleted / unmapped reads
 * were never packed, which is exactly the set get_dqstats skips. */
static void ss_dqstats(const uint32_t *r, uint32_t n, int ref_base, uint32_t wanted, dqstats_t *q)
{
    memset(q, 0, sizeof *q);
    for (uint32_t i = 0; i < n; ++i) {
        const int base = (int)SS_READ_NT16(r[i]);
        const uint32_t mq = SS_READ_MAPQ(r[i]), bq = SS_READ_BASEQ(r[i]);
        q->total_depth++;
        q->total_mean_mapQ += mq;
        q->dp4[(base == ref_base ? 0 : 2) + SS_READ_STRAND(r[i])]++;
        for (int j = 0; j < 4; ++j) {
            const int bit = 1 << j;
            if ((base & bit) != base) continue;
            q->base_occ[j]++;
            if (bit & wanted) { q->mean_baseQ[j] += bq; q->mean_mapQ[j] += mq; }
        }
    }
    for (int j = 0; j < 4; ++j)
        if (q->base_occ[j]) {
            q->mean_baseQ[j] = (uint32_t)(q->mean_baseQ[j] / (double)q->base_occ[j] + .499);
            q->mean_mapQ[j] = (uint32_t)(q->mean_mapQ[j] / (double)q->base_occ[j] + .499);
        }
    if (q->total_depth) q->total_mean_mapQ = (uint32_t)(q->total_mean_mapQ / (double)q->total_depth + .499);
}

static void shim_flush(void)
{
    if (!g_ctx || g_b.n == 0) return;
    ss_batch_t b = {g_b.n, g_b.ref, g_b.off_t, g_b.off_n, g_b.reads_t, g_b.reads_n};
    uint32_t ncalls = 0, nclamp = 0;
    for (;;) {
        ss_out_t o = {g_b.score, g_b.calls, (uint32_t)g_b.calls_cap, &ncalls, NULL, &nclamp};
        int rc = ss_score_batch_host(g_ctx, &b, &o);
        /* grow and re-score only when the emitted calls did not fit; any
         * other error (including a capacity error of the device work lists)
         * is final */
        if (rc == SS_E_CAPACITY && ncalls > g_b.calls_cap) {
            size_t c = g_b.calls_cap;
            g_b.calls = grow(g_b.calls, &c, ncalls, sizeof(ss_call_t));
            g_b.calls_cap = c;
            continue;
        }
        if (rc) die("ss_score_batch_host", rc);
        break;
    }
    for (uint32_t i = 0; i < ncalls; ++i) {          /* sorted by site == (tid, pos) order */
        const ss_call_t *c = &g_b.calls[i];
        const uint32_t s = c->site;
        const int rb4 = c->ref_base4;
        sniper_output_t out;
        memset(&out, 0, sizeof out);
        out.seq_name = g_d->h1->target_name[g_b.tid[s]];
        out.pos = g_b.pos[s];
        out.ref_base = g_b.ref[s];
        out.ref_base4 = rb4;
        const int tb = (int)(c->cns_tumor >> 28), nb = (int)(c->cns_normal >> 28);
        const int tg = c->joint_gt_tumor ? c->joint_gt_tumor : tb;
        const int ng = c->joint_gt_normal ? c->joint_gt_normal : nb;
        out.tumor.genotype = tb;
        out.tumor.consensus_quality = (int)(c->cns_tumor >> 8 & 0xff);
        out.tumor.variant_allele_quality = c->snp_q_tumor;
        out.tumor.somatic_score = c->somatic_score;
        out.tumor.joint_genotype = c->joint_gt_tumor;
        out.tumor.joint_consensus_quality = c->joint_cq;
        out.tumor.variant_status = (variant_status_t)c->status_tumor;
        ss_dqstats(g_b.reads_t + g_b.off_t[s], g_b.off_t[s + 1] - g_b.off_t[s], rb4,
                   (uint32_t)(rb4 | tg | ng), &out.tumor.dqstats);
        out.normal.genotype = nb;
        out.normal.consensus_quality = (int)(c->cns_normal >> 8 & 0xff);
        out.normal.variant_allele_quality = c->snp_q_normal;
        out.normal.somatic_score = -1;
        out.normal.joint_genotype = c->joint_gt_normal;
        out.normal.joint_consensus_quality = c->joint_cq;
        out.normal.variant_status = (variant_status_t)c->status_normal;
        ss_dqstats(g_b.reads_n + g_b.off_n[s], g_b.off_n[s + 1] - g_b.off_n[s], rb4,
                   (uint32_t)(rb4 | ng | tg), &out.normal.dqstats);
        output_formatter_write(g_d->output_formatter, &out);
        fflush(g_fh);
    }
    g_b.n = g_b.nt = g_b.nn = 0;
}

int __wrap_glf_somatic(uint32_t tid, uint32_t pos, int n1, int n2, const bam_pileup1_t *pl1,
                       const bam_pileup1_t *pl2, void *data, FILE *snp_fh)
{
    pu_data2_t *d = (pu_data2_t *)data;
    if (!g_ctx) shim_init(d);
    g_fh = snp_fh;
    /* contig sequence cache, as glf_somatic keeps it (somatic_sniper.c:112-117) */
    if (d->fai && (int)tid != d->tid) {
        free(d->ref);
        d->ref = fai_fetch(d->fai, d->h1->target_name[tid], &d->len);
        d->tid = tid;
    }
    const size_t s = g_b.n;
    g_b.ref[s] = (uint8_t)((d->ref && (int)pos < d->len) ? d->ref[pos] : 'N');
    g_b.tid[s] = tid;
    g_b.pos[s] = pos;
    pack(pl1, n1, &g_b.reads_t, &g_b.nt, &g_b.capt);
    pack(pl2, n2, &g_b.reads_n, &g_b.nn, &g_b.capn);
    g_b.off_t[s + 1] = (uint32_t)g_b.nt;
    g_b.off_n[s + 1] = (uint32_t)g_b.nn;
    g_b.n = s + 1;
    if (g_b.n == g_b.cap || g_b.nt > 0xC0000000u || g_b.nn > 0xC0000000u) shim_flush();
    return 0;
}

int __wrap_bam_sspileup_file(bamFile fp1, bamFile fp2, int mask, int thresh, bam_sspileup_f func,
                             void *func_data, FILE *snp_fh)
{
    const int rc = __real_bam_sspileup_file(fp1, fp2, mask, thresh, func, func_data, snp_fh);
    shim_flush();
    if (g_ctx) { ss_ctx_destroy(g_ctx); g_ctx = NULL; }
    free(g_b.ref); free(g_b.off_t); free(g_b.off_n); free(g_b.reads_t); free(g_b.reads_n);
    free(g_b.tid); free(g_b.pos); free(g_b.score); free(g_b.calls);
    memset(&g_b, 0, sizeof g_b);
    return rc;
}
