/*
 * sniper_cli.c -- bam-somaticsniper, MI355X build.
 *
 * Command line, messages and outputs follow the reference CLI
 * (src/exe/bam-somaticsniper/main.c:27-162); the site walk is dual_pileup.c
 * (sniper_pileup.c restated), the per-site scoring is the C ABI
 * (include/sniper_amd.h) on the GPU, fed in batches by this file:
 *
 *   pileup thread                      scorer threads (one per GPU)
 *   ----------------------------       -------------------------------------
 *   pack sites into batch k      ->    ss_score_batch_host(batch k) on the
 *   (while earlier batches are         slot's context / device, then,
 *   being scored)                      in batch order, dqstats + writer for
 *                                      every emitted site ((tid, pos) order)
 *
 * Several GPUs (SS_DEVICES=0,1,...): one streaming dual pileup per run (the
 * reference's, with its first-read-drop and lockstep rules untouched) hands
 * consecutive batches to whichever device's scorer is free; outputs are
 * written strictly in batch order, so the file is identical for any number
 * of devices ("one streaming pileup per BAM feeding all
 * GPUs").
 *
 * Contig groups: when both BAMs have an index (.bai; the reference does not
 * need one, so this is optional), the contigs are cut into SS_CONTIG_GROUPS
 * (default 4) ranges of about equal compressed size, and each range runs its
 * own pileup (both files read from the range's first records, bam_index.h),
 * batches and scorer threads; scorer k of every range shares the process's
 * context k (one per device, created once: shared_ctx), and the ranges'
 * outputs are concatenated in contig order.
 * Each walk's state at a range start is seeded from the last record its file
 * loads before the range (column_pileup.h), so the sites, entries and output
 * bytes are those of the single streaming walk.
 *
 * A site is what glf_somatic (somatic_sniper.c:109) sees: the ref char of
 * the cached contig (fai fetch, :112-117) and the non-deleted, mapped reads of
 * both samples (sniper_maqcns.c:147).  There is no CPU scoring path: without a
 * usable GPU the program stops with an error.
 *
 * Environment: SS_DEVICE (GPU index, default 0), SS_DEVICES (comma list of GPU
 * indices, overrides SS_DEVICE; SS_DEVICES_SHARED=1 allows repeats), SS_BATCH (sites per batch,
 * default 2^20), SS_BGZF_THREADS (inflate threads per BAM, default 4),
 * SS_PILEUP_THREADS (2, default: column pileup, per sample a reader thread and
 * SS_PILEUP_WORKERS (default 3) window builders;
 * 1: tumor and normal walks on their own threads; 0: one thread),
 * SS_DUMP_PILEUP=FILE (test hook: also write every reported site, see
 * dump_site()), SS_PILEUP_ONLY=1 (test / timing hook: walk (and dump) without
 * scoring, so the pileup restatement is testable on a host without a GPU; no
 * output records are written), SS_TIMING=1 (phase times on stderr),
 * SS_CONTIG_GROUPS (contig ranges pileup in parallel when both BAMs are
 * indexed, default 4; 1 keeps the single streaming walk).
 */
#include <getopt.h>
#include <time.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "bam_index.h"
#include "bam_reader.h"
#include "bgzf_reader.h"
#include "dual_pileup.h"
#include "fasta_index.h"
#include "sniper_amd.h"
#include "sniper_output.h"

#ifndef SS_CLI_VERSION
#define SS_CLI_VERSION "mi355x-1.0"
#endif
#ifndef SS_CLI_COMMIT
#define SS_CLI_COMMIT "unknown"
#endif

/* ---- batches --------------------------------------------------------- */
typedef struct {
    size_t n, cap;
    size_t nt, capt, nn, capn;
    uint8_t *ref;
    uint32_t *off_t, *off_n, *reads_t, *reads_n, *tid, *pos;
    int32_t *score;
    ss_call_t *calls;
    size_t calls_cap;
} batch_t;

static void *xrealloc(void *p, size_t n)
{
    void *q = realloc(p, n ? n : 1);
    if (!q) { fprintf(stderr, "out of memory\n"); exit(1); }
    return q;
}

static void batch_init(batch_t *b, size_t cap)
{
    memset(b, 0, sizeof *b);
    b->cap = cap;
    b->ref = (uint8_t *)xrealloc(NULL, cap);
    b->off_t = (uint32_t *)xrealloc(NULL, (cap + 1) * 4);
    b->off_n = (uint32_t *)xrealloc(NULL, (cap + 1) * 4);
    b->tid = (uint32_t *)xrealloc(NULL, cap * 4);
    b->pos = (uint32_t *)xrealloc(NULL, cap * 4);
    b->score = (int32_t *)xrealloc(NULL, cap * 4);
    b->calls_cap = 4096;
    b->calls = (ss_call_t *)xrealloc(NULL, b->calls_cap * sizeof(ss_call_t));
    b->off_t[0] = b->off_n[0] = 0;
}

static void batch_free(batch_t *b)
{
    free(b->ref); free(b->off_t); free(b->off_n); free(b->reads_t); free(b->reads_n);
    free(b->tid); free(b->pos); free(b->score); free(b->calls);
}

/* ---- run state --------------------------------------------------------- */
/* batch ring: the pileup fills one while the others wait for, are in, or
 * wait to be written by the scorers, so the pileup runs ahead while the GPU
 * scorers are still being created and never waits for one batch's scoring.
 * Batch s (a sequence number) lives in slot s % n_bat. */
#define MAX_DEV 16
#define MAX_BATCH (MAX_DEV + 3)

typedef struct {
    /* reference */
    fasta_index_t *fai;
    bam_header_t *h1;
    int cur_tid, cur_len;
    char *cur_ref;
    /* scoring */
    FILE *out;
    int fmt;
    batch_t bat[MAX_BATCH];
    int n_bat;
    uint64_t seq_fill;        /* batch the pileup is filling (= batches submitted) */
    uint64_t seq_claim;       /* next submitted batch a scorer takes */
    uint64_t seq_write;       /* next batch to be written (output order) */
    int quit;
    int failed;               /* set by any scorer, read by all threads: __atomic only (failed_get/set) */
    pthread_t th[MAX_DEV];
    pthread_mutex_t mu;
    pthread_cond_t cv;
    FILE *dump;
    int pileup_only;
    /* GPU scorers: scorer slot k uses the process's context k (shared_ctx) */
    ss_params_t prm;
    int n_dev, device[MAX_DEV];
} run_t;

typedef struct {
    run_t *R;
    int k;                    /* scorer index */
} scorer_arg_t;

/* One GPU context per scorer slot for the whole process: the streaming walk's
 * scorer k and scorer k of every contig range share it, one batch at a time
 * (a context takes one launch at a time, include/sniper_amd.h), so a range
 * costs no context creation (table upload and fingerprint, about 0.25 s each
 * in round 5).  Created by the first scorer thread that needs it, while the
 * pileup runs. */
static ss_ctx_t *g_ctx[MAX_DEV];
static int g_ctx_rc[MAX_DEV];
static pthread_mutex_t g_ctx_make_mu[MAX_DEV], g_ctx_use_mu[MAX_DEV];

static ss_ctx_t *shared_ctx(const ss_params_t *prm, int k, int device)
{
    pthread_mutex_lock(&g_ctx_make_mu[k]);
    if (!g_ctx[k] && !g_ctx_rc[k]) g_ctx_rc[k] = ss_ctx_create(prm, device, &g_ctx[k]);
    const int rc = g_ctx_rc[k];
    pthread_mutex_unlock(&g_ctx_make_mu[k]);
    if (rc) {
        fprintf(stderr, "[bam-somaticsniper] cannot create the GPU scorer: %s\n", ss_strerror(rc));
        exit(1);
    }
    return g_ctx[k];
}

static int failed_get(run_t *R) { return __atomic_load_n(&R->failed, __ATOMIC_ACQUIRE); }
static void failed_set(run_t *R) { __atomic_store_n(&R->failed, 1, __ATOMIC_RELEASE); }

/* score batch b on context ctx; returns the number of emitted calls or -1 */
static long score_batch(run_t *R, ss_ctx_t *ctx, batch_t *b)
{
    ss_batch_t in = {b->n, b->ref, b->off_t, b->off_n, b->reads_t, b->reads_n};
    uint32_t ncalls = 0, nclamp = 0;
    for (;;) {
        ss_out_t o = {b->score, b->calls, (uint32_t)b->calls_cap, &ncalls, NULL, &nclamp};
        const int rc = ss_score_batch_host(ctx, &in, &o);
        if (rc == SS_E_CAPACITY && ncalls > b->calls_cap) {
            b->calls_cap = ncalls;
            b->calls = (ss_call_t *)xrealloc(b->calls, b->calls_cap * sizeof(ss_call_t));
            continue;
        }
        if (rc) {
            fprintf(stderr, "[bam-somaticsniper] GPU scoring failed: %s\n", ss_strerror(rc));
            failed_set(R);
            return -1;
        }
        return (long)ncalls;
    }
}

/* dqstats + writer for the emitted calls of a scored batch (in site order) */
static void write_batch(run_t *R, const batch_t *b, uint32_t ncalls)
{
    for (uint32_t i = 0; i < ncalls; ++i) {
        const ss_call_t *c = &b->calls[i];
        const uint32_t s = c->site;
        ss_site_out_t o;
        memset(&o, 0, sizeof o);
        o.seq_name = R->h1->name[b->tid[s]];
        o.pos = b->pos[s];
        o.ref_base = b->ref[s];
        o.ref_base4 = c->ref_base4;
        const int tb = (int)(c->cns_tumor >> 28), nb = (int)(c->cns_normal >> 28);
        const int tg = c->joint_gt_tumor ? c->joint_gt_tumor : tb;
        const int ng = c->joint_gt_normal ? c->joint_gt_normal : nb;
        o.tumor.genotype = tb;
        o.tumor.consensus_quality = (int)(c->cns_tumor >> 8 & 0xff);
        o.tumor.variant_allele_quality = c->snp_q_tumor;
        o.tumor.somatic_score = c->somatic_score;
        o.tumor.joint_genotype = c->joint_gt_tumor;
        o.tumor.joint_consensus_quality = c->joint_cq;
        o.tumor.variant_status = c->status_tumor;
        ss_dqstats_packed(b->reads_t + b->off_t[s], b->off_t[s + 1] - b->off_t[s], o.ref_base4,
                          (uint32_t)(o.ref_base4 | tg | ng), &o.tumor.dq);
        o.normal.genotype = nb;
        o.normal.consensus_quality = (int)(c->cns_normal >> 8 & 0xff);
        o.normal.variant_allele_quality = c->snp_q_normal;
        o.normal.somatic_score = -1;
        o.normal.joint_genotype = c->joint_gt_normal;
        o.normal.joint_consensus_quality = c->joint_cq;
        o.normal.variant_status = c->status_normal;
        ss_dqstats_packed(b->reads_n + b->off_n[s], b->off_n[s + 1] - b->off_n[s], o.ref_base4,
                          (uint32_t)(o.ref_base4 | ng | tg), &o.normal.dq);
        ss_write_site(R->out, R->fmt, &o);
    }
}

/* SS_TIMING=1: phase times on stderr (seconds since start) */
static double t_start;
static int timing, debug_batches;
static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}
static void stamp(const char *what)
{
    if (timing) fprintf(stderr, "[timing] %-24s %.3f s\n", what, now_s() - t_start);
}

static void *scorer_main(void *arg)
{
    run_t *R = ((scorer_arg_t *)arg)->R;
    const int k = ((scorer_arg_t *)arg)->k;
    ss_ctx_t *ctx = NULL;
    if (!R->pileup_only) {
        /* host tables (shared by the process) + device upload overlap the BAM decode and pileup */
        ctx = shared_ctx(&R->prm, k, R->device[k]);
        stamp("scorer ready");
    }
    pthread_mutex_lock(&R->mu);
    for (;;) {
        while (R->seq_claim == R->seq_fill && !R->quit) pthread_cond_wait(&R->cv, &R->mu);
        if (R->seq_claim == R->seq_fill) break;            /* quit and nothing left */
        const uint64_t s = R->seq_claim++;
        batch_t *b = &R->bat[s % (uint64_t)R->n_bat];
        pthread_mutex_unlock(&R->mu);
        long ncalls = -1;
        if (!failed_get(R)) {
            pthread_mutex_lock(&g_ctx_use_mu[k]);      /* the context is shared with other ranges' scorer k */
            ncalls = score_batch(R, ctx, b);
            pthread_mutex_unlock(&g_ctx_use_mu[k]);
        }
        stamp("batch scored");
        if (debug_batches)                                  /* SS_DEBUG_BATCHES=1: one line per scored batch */
            fprintf(stderr, "[batch] run %p scorer %d seq %llu sites %zu first %u:%u calls %ld\n", (void *)R, k,
                    (unsigned long long)s, b->n, b->n ? b->tid[0] : 0u, b->n ? b->pos[0] : 0u, ncalls);
        pthread_mutex_lock(&R->mu);
        while (R->seq_write != s) pthread_cond_wait(&R->cv, &R->mu);   /* output in batch order */
        pthread_mutex_unlock(&R->mu);
        if (ncalls > 0) write_batch(R, b, (uint32_t)ncalls);
        b->n = b->nt = b->nn = 0;
        pthread_mutex_lock(&R->mu);
        ++R->seq_write;
        pthread_cond_broadcast(&R->cv);
    }
    pthread_mutex_unlock(&R->mu);
    return NULL;
}

/* queue the filled batch for the scorers (in order); continue in the next
 * slot once its previous batch has been written */
static void submit(run_t *R)
{
    pthread_mutex_lock(&R->mu);
    ++R->seq_fill;
    pthread_cond_broadcast(&R->cv);
    while (R->seq_fill - R->seq_write >= (uint64_t)R->n_bat) pthread_cond_wait(&R->cv, &R->mu);
    pthread_mutex_unlock(&R->mu);
}

static batch_t *filling(run_t *R) { return &R->bat[R->seq_fill % (uint64_t)R->n_bat]; }

static void pack(batch_t *b, const uint32_t *pk, int np, int tumor)
{
    uint32_t **dst = tumor ? &b->reads_t : &b->reads_n;
    size_t *len = tumor ? &b->nt : &b->nn, *cap = tumor ? &b->capt : &b->capn;
    if (*len + (size_t)np > *cap) {
        size_t c = *cap ? *cap : 1 << 20;
        while (c < *len + (size_t)np) c *= 2;
        *dst = (uint32_t *)xrealloc(*dst, c * 4);
        *cap = c;
    }
    memcpy(*dst + *len, pk, 4 * (size_t)np);
    *len += (size_t)np;
}

/* test hook: tid pos n1 n2 refchar | tumor packed reads | normal packed reads */
static void dump_site(run_t *R, const batch_t *b, size_t s, int n1, int n2)
{
    fprintf(R->dump, "%u\t%u\t%d\t%d\t%d\t", b->tid[s], b->pos[s], n1, n2, b->ref[s]);
    for (uint32_t i = b->off_t[s]; i < b->off_t[s + 1]; ++i) fprintf(R->dump, "%x,", b->reads_t[i]);
    fputc('\t', R->dump);
    for (uint32_t i = b->off_n[s]; i < b->off_n[s + 1]; ++i) fprintf(R->dump, "%x,", b->reads_n[i]);
    fputc('\n', R->dump);
}

static int on_site(int32_t tid, int32_t pos, int n1, int n2, const uint32_t *pk1, int np1,
                   const uint32_t *pk2, int np2, void *data)
{
    run_t *R = (run_t *)data;
    if (tid < 0 || tid >= R->h1->n_ref) {       /* a record naming no header contig */
        fprintf(stderr, "[bam-somaticsniper] BAM record on contig %d: the header has %d\n", (int)tid,
                (int)R->h1->n_ref);
        failed_set(R);
        return 1;
    }
    if (R->fai && tid != R->cur_tid) {          /* contig cache (somatic_sniper.c:112-117) */
        free(R->cur_ref);
        R->cur_ref = fasta_fetch(R->fai, R->h1->name[tid], &R->cur_len);
        R->cur_tid = tid;
    }
    batch_t *b = filling(R);
    const size_t s = b->n;
    b->ref[s] = (uint8_t)((R->cur_ref && pos < R->cur_len) ? R->cur_ref[pos] : 'N');
    b->tid[s] = (uint32_t)tid;
    b->pos[s] = (uint32_t)pos;
    pack(b, pk1, np1, 1);
    pack(b, pk2, np2, 0);
    b->off_t[s + 1] = (uint32_t)b->nt;
    b->off_n[s + 1] = (uint32_t)b->nn;
    b->n = s + 1;
    if (R->dump) dump_site(R, b, s, n1, n2);
    if (R->pileup_only) {                       /* test hook: nothing is scored */
        b->n = b->nt = b->nn = 0;
        return 0;
    }
    if (b->n == b->cap || b->nt > 0xC0000000u || b->nn > 0xC0000000u) submit(R);
    return failed_get(R);
}

/* ---- command line --------------------------------------------------------- */
static void version_info(void)
{
    printf("Somatic Sniper version (%s) (commit %s)\n", SS_CLI_VERSION, SS_CLI_COMMIT);
}

static void usage(const char *progname, const ss_params_t *p, int mapq)
{
    const char *pn = strrchr(progname, '/');
    pn = pn ? pn + 1 : progname;
    fprintf(stderr, "\n\n%s [options] -f <ref.fasta> <tumor.bam> <normal.bam> <snp_output_file>\n\n", pn);
    fprintf(stderr, "Required Option: \n");
    fprintf(stderr, "        -f FILE   REQUIRED reference sequence in the FASTA format\n\n");
    fprintf(stderr, "Options: \n");
    fprintf(stderr, "        -v        Display version information\n\n");
    fprintf(stderr, "        -q INT    filtering reads with mapping quality less than INT [%d]\n", mapq);
    fprintf(stderr, "        -Q INT    filtering somatic snv output with somatic quality less than  INT [%d]\n",
            p->min_somatic_qual);
    fprintf(stderr, "        -L FLAG   do not report LOH variants as determined by genotypes\n");
    fprintf(stderr, "        -G FLAG   do not report Gain of Reference variants as determined by genotypes\n");
    fprintf(stderr, "        -p FLAG   disable priors in the somatic calculation. Increases sensitivity for solid tumors\n");
    fprintf(stderr, "        -J FLAG   Use prior probabilities accounting for the somatic mutation rate\n");
    fprintf(stderr, "        -s FLOAT  prior probability of a somatic mutation (implies -J) [%f]\n", p->somatic_rate);
    fprintf(stderr, "        -T FLOAT  theta in maq consensus calling model (for -c/-g) [%f]\n", p->theta);
    fprintf(stderr, "        -N INT    number of haplotypes in the sample (for -c/-g) [%d]\n", p->n_hap);
    fprintf(stderr, "        -r FLOAT  prior of a difference between two haplotypes (for -c/-g) [%f]\n", p->het_rate);
    fprintf(stderr, "        -n STRING normal sample id (for VCF header) [%s]\n", "NORMAL");
    fprintf(stderr, "        -t STRING tumor sample id (for VCF header) [%s]\n", "TUMOR");
    fprintf(stderr, "        -F STRING select output format [%s]\n", "classic");
    fprintf(stderr, "           Available formats:\n");
    for (int i = 0; i < ss_format_count(); ++i) fprintf(stderr, "             %s\n", ss_format_name(i));
    fprintf(stderr, "\n");
}

static int env_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

/* SS_DEVICES: a comma list of distinct GPU indices (at most MAX_DEV).  An
 * empty, non-numeric, negative or repeated entry, or too many entries, is an
 * error: a typo must not silently put two scorers on one GPU.  Several
 * scorers on one GPU on purpose (tests on a one-GPU host) need
 * SS_DEVICES_SHARED=1 as well. */
static int parse_devices(const char *s, int *dev, int *n)
{
    const char *sh = getenv("SS_DEVICES_SHARED");
    const int shared = sh && sh[0] == '1';
    const char *q = s;
    *n = 0;
    for (;;) {
        char *end;
        const long v = strtol(q, &end, 10);
        if (end == q || v < 0 || v > 1023 || (*end != ',' && *end != 0)) {
            fprintf(stderr, "[bam-somaticsniper] SS_DEVICES='%s': bad entry at '%s' (expected a comma list of "
                            "GPU indices)\n", s, q);
            return 1;
        }
        if (*n == MAX_DEV) {
            fprintf(stderr, "[bam-somaticsniper] SS_DEVICES='%s': more than %d devices\n", s, MAX_DEV);
            return 1;
        }
        for (int i = 0; i < *n && !shared; ++i)
            if (dev[i] == (int)v) {
                fprintf(stderr, "[bam-somaticsniper] SS_DEVICES='%s': device %ld listed twice\n", s, v);
                return 1;
            }
        dev[(*n)++] = (int)v;
        if (*end == 0) return 0;
        q = end + 1;
    }
}

/* ---- contig groups (indexed BAMs) ------------------------------------------ */
typedef struct {
    run_t R;
    const char *bam1, *bam2;
    int32_t t0, t1;           /* contigs [t0, t1) */
    uint64_t v1, v2;          /* the files' first records at or after t0 (UINT64_MAX: none) */
    col_seed_t s1, s2;
    int mapq, bthreads;
    char *obuf, *dbuf;        /* the group's output / dump, concatenated in group order */
    size_t olen, dlen;
    scorer_arg_t sarg[MAX_DEV];
    int err;
} group_t;

static void run_scorers_start(run_t *R, scorer_arg_t *sarg)
{
    for (int k = 0; k < R->n_dev; ++k) {
        sarg[k].R = R;
        sarg[k].k = k;
        pthread_create(&R->th[k], NULL, scorer_main, &sarg[k]);
    }
}

static void run_scorers_finish(run_t *R)
{
    if (filling(R)->n) submit(R);
    pthread_mutex_lock(&R->mu);
    R->quit = 1;
    pthread_cond_broadcast(&R->cv);
    pthread_mutex_unlock(&R->mu);
    for (int k = 0; k < R->n_dev; ++k) pthread_join(R->th[k], NULL);
}

static void *group_main(void *arg)
{
    group_t *g = (group_t *)arg;
    run_t *R = &g->R;
    run_scorers_start(R, g->sarg);
    if (g->v1 != UINT64_MAX && g->v2 != UINT64_MAX) {   /* a file without records here: no shared site */
        bgzf_reader_t *f1 = bgzf_open_at(g->bam1, g->bthreads, g->v1);
        bgzf_reader_t *f2 = bgzf_open_at(g->bam2, g->bthreads, g->v2);
        if (!f1 || !f2) {
            fprintf(stderr, "[bam-somaticsniper] cannot seek in the indexed BAMs\n");
            g->err = 1;
        } else if (dual_pileup_range(f1, f2, (int)SS_BAM_DEF_MASK, g->mapq, &g->s1, &g->s2, on_site, R)) {
            g->err = 1;
        }
        if (f1) bgzf_close(f1);
        if (f2) bgzf_close(f2);
    }
    run_scorers_finish(R);
    /* release the range's batches here, while other ranges still run (the
     * GPU contexts are the process's, destroyed at exit) */
    for (int k = 0; k < R->n_bat; ++k) batch_free(&R->bat[k]);
    R->n_bat = 0;
    return NULL;
}

/* Cuts [0, n_ref) into at most G ranges of about equal index size; returns
 * the number of ranges, their starts in t0[] (t0[n] = n_ref). */
static int cut_groups(const bai_t *a, const bai_t *b, int32_t n_ref, int G, int32_t *t0)
{
    double tot = 0;
    for (int32_t t = 0; t < n_ref; ++t) tot += (double)a->ref[t].bytes + (double)b->ref[t].bytes;
    int n = 0;
    t0[n++] = 0;
    double acc = 0;
    for (int32_t t = 0; t < n_ref && n < G; ++t) {
        acc += (double)a->ref[t].bytes + (double)b->ref[t].bytes;
        if (acc >= tot * n / G && t + 1 < n_ref && acc > 0) t0[n++] = t + 1;
    }
    t0[n] = n_ref;
    return n;
}

/* The contig-parallel run; returns 0 when it ran, 1 when the inputs do not
 * allow it (no index, stdin, a single range), -1 on failure. */
static int run_groups(run_t *base, const char *bam1, const char *bam2, int mapq, int bthreads, int cap,
                      const char *fn_fa)
{
    int G = env_int("SS_CONTIG_GROUPS", 4);
    if (G > 64) G = 64;
    if (G < 2 || env_int("SS_PILEUP_THREADS", 2) != 2 || !strcmp(bam1, "-") || !strcmp(bam2, "-")) return 1;
    bai_t *x1 = bai_load_for(bam1), *x2 = x1 ? bai_load_for(bam2) : NULL;
    const int32_t n_ref = base->h1->n_ref;
    if (!x1 || !x2 || x1->n_ref != n_ref || x2->n_ref < n_ref) { bai_free(x1); bai_free(x2); return 1; }
    int32_t t0[65];
    const int n = cut_groups(x1, x2, n_ref, G, t0);
    if (n < 2) { bai_free(x1); bai_free(x2); return 1; }
    group_t *g = (group_t *)calloc((size_t)n, sizeof(group_t));
    int bad = 0, stale = 0;
    for (int i = 0; i < n && !bad; ++i) {
        group_t *q = &g[i];
        q->bam1 = bam1;
        q->bam2 = bam2;
        q->t0 = t0[i];
        q->t1 = t0[i + 1];
        q->mapq = mapq;
        q->bthreads = bthreads;
        q->v1 = bai_first_at_or_after(x1, q->t0);
        q->v2 = bai_first_at_or_after(x2, q->t0);
        /* an index that does not agree with its file (stale, or another file's)
         * would seek mid-record or to the wrong contig: the streaming walk runs */
        if ((q->v1 != UINT64_MAX && bai_check_start(bam1, x1, q->t0)) ||
            (q->v2 != UINT64_MAX && bai_check_start(bam2, x2, q->t0))) {
            stale = 1;
            break;
        }
        const col_seed_t none = {0, 0, 0, i + 1 < n ? q->t1 : INT32_MAX};
        q->s1 = q->s2 = none;
        int32_t tid;
        int64_t pos;
        const uint32_t mask = SS_BAM_DEF_MASK;
        int r = bai_last_loaded_before(bam1, x1, q->t0, mask, mapq, &tid, &pos);
        if (r == -2) { stale = 1; break; }             /* the index is another file's */
        if (r < 0) bad = 1;
        else if (r) { q->s1.has_prev = 1; q->s1.prev_tid = tid; q->s1.prev_pos = pos; }
        r = bai_last_loaded_before(bam2, x2, q->t0, mask, mapq, &tid, &pos);
        if (r == -2) { stale = 1; break; }
        if (r < 0) bad = 1;
        else if (r) { q->s2.has_prev = 1; q->s2.prev_tid = tid; q->s2.prev_pos = pos; }
        if (timing)
            fprintf(stderr, "[timing] group %d contigs [%d, %d) start %llx / %llx seed %d:%d:%lld / %d:%d:%lld\n", i,
                    q->t0, q->t1, (unsigned long long)q->v1, (unsigned long long)q->v2, q->s1.has_prev, q->s1.prev_tid,
                    (long long)q->s1.prev_pos, q->s2.has_prev, q->s2.prev_tid, (long long)q->s2.prev_pos);
        run_t *R = &q->R;                                  /* the group's own run: fai handle, batches, scorers */
        R->h1 = base->h1;
        R->cur_tid = -1;
        R->fai = fasta_index_load(fn_fa);
        R->fmt = base->fmt;
        R->out = open_memstream(&q->obuf, &q->olen);
        if (base->dump) R->dump = open_memstream(&q->dbuf, &q->dlen);
        R->pileup_only = base->pileup_only;
        R->prm = base->prm;
        R->n_dev = base->n_dev;
        memcpy(R->device, base->device, sizeof R->device);
        R->n_bat = R->n_dev + 3;
        for (int k = 0; k < R->n_bat; ++k) batch_init(&R->bat[k], (size_t)cap);
        pthread_mutex_init(&R->mu, NULL);
        pthread_cond_init(&R->cv, NULL);
    }
    bai_free(x1);
    bai_free(x2);
    if (stale) {                                          /* nothing started yet: plain walk */
        if (timing) fprintf(stderr, "[timing] index does not match the BAM: streaming walk\n");
        for (int i = 0; i < n; ++i) {
            run_t *R = &g[i].R;
            if (!R->out) continue;
            fclose(R->out);
            if (R->dump) fclose(R->dump);
            free(g[i].obuf);
            free(g[i].dbuf);
            fasta_index_free(R->fai);
            for (int k = 0; k < R->n_bat; ++k) batch_free(&R->bat[k]);
            pthread_mutex_destroy(&R->mu);
            pthread_cond_destroy(&R->cv);
        }
        free(g);
        return 1;
    }
    if (bad) {
        fprintf(stderr, "[bam-somaticsniper] cannot read the indexed BAMs\n");
        return -1;
    }
    stamp("contig groups planned");
    pthread_t *th = (pthread_t *)calloc((size_t)n, sizeof(pthread_t));
    for (int i = 0; i < n; ++i) pthread_create(&th[i], NULL, group_main, &g[i]);
    int rc = 0;
    for (int i = 0; i < n; ++i) {
        pthread_join(th[i], NULL);
        run_t *R = &g[i].R;
        fclose(R->out);
        if (R->dump) fclose(R->dump);
        if (g[i].err || failed_get(R)) rc = -1;
        fwrite(g[i].obuf, 1, g[i].olen, base->out);      /* contig order */
        if (base->dump && g[i].dlen) fwrite(g[i].dbuf, 1, g[i].dlen, base->dump);
        free(g[i].obuf);
        free(g[i].dbuf);
        fasta_index_free(R->fai);
        free(R->cur_ref);
        pthread_mutex_destroy(&R->mu);
        pthread_cond_destroy(&R->cv);
    }
    free(th);
    free(g);
    stamp("contig groups done");
    return rc;
}

int main(int argc, char *argv[])
{
    t_start = now_s();
    for (int k = 0; k < MAX_DEV; ++k) {
        pthread_mutex_init(&g_ctx_make_mu[k], NULL);
        pthread_mutex_init(&g_ctx_use_mu[k], NULL);
    }
    timing = getenv("SS_TIMING") != NULL;
    debug_batches = getenv("SS_DEBUG_BATCHES") != NULL;
    ss_params_t prm;
    ss_params_default(&prm);
    const char *normal_id = "NORMAL", *tumor_id = "TUMOR", *fn_fa = NULL, *fmt_name = "classic";
    int mapq = 0, c;
    while ((c = getopt(argc, argv, "n:t:vf:T:N:r:I:q:Q:pLGJs:F:")) >= 0) {
        switch (c) {
        case 'f': fn_fa = optarg; break;
        case 'T': prm.theta = (float)atof(optarg); break;
        case 'N': prm.n_hap = atoi(optarg); break;
        case 'r': prm.het_rate = (float)atof(optarg); break;
        case 'q': mapq = atoi(optarg); break;
        case 'Q': prm.min_somatic_qual = atoi(optarg); break;
        case 'F': fmt_name = optarg; break;
        case 'p': prm.use_priors = 0; break;
        case 'J': prm.use_joint_priors = 1; break;
        case 's': prm.somatic_rate = atof(optarg); prm.use_joint_priors = 1; break;
        case 'v': version_info(); return 0;
        case 't': tumor_id = optarg; break;
        case 'n': normal_id = optarg; break;
        case 'L': prm.include_loh = 0; break;
        case 'G': prm.include_gor = 0; break;
        default: fprintf(stderr, "Unrecognizd option '-%c'.\n", c); return 1;
        }
    }
    if (optind == argc) { usage(argv[0], &prm, mapq); return 1; }
    if (argc - optind < 3) {          /* the reference dereferences missing arguments */
        usage(argv[0], &prm, mapq);
        return 1;
    }
    run_t R;
    memset(&R, 0, sizeof R);
    R.cur_tid = -1;
    if (fn_fa) R.fai = fasta_index_load(fn_fa);
    else {
        fprintf(stderr, "You MUST specify a reference sequence. It isn't optional.\n");
        exit(1);
    }
    if (prm.use_joint_priors)
        fprintf(stderr, "Using priors accounting for somatic mutation rate. Prior probability of a somatic "
                        "mutation is %f\n", prm.somatic_rate);
    fprintf(stderr, "Preparing to snipe some somatics\n");
    if (prm.use_priors) fprintf(stderr, "Using prior probabilities\n");
    const int bthreads = env_int("SS_BGZF_THREADS", 4);
    bgzf_reader_t *fp1 = bgzf_open(argv[optind], bthreads);
    fprintf(stderr, "Normal bam is %s\n", argv[optind + 1]);
    fprintf(stderr, "Tumor bam is %s\n", argv[optind]);
    bam_header_t h1, h2;
    if (!fp1 || bam_header_read(fp1, &h1)) {
        fprintf(stderr, "[bam-somaticsniper] cannot read BAM %s\n", argv[optind]);
        return 1;
    }
    bgzf_reader_t *fp2 = bgzf_open(argv[optind + 1], bthreads);
    if (!fp2 || bam_header_read(fp2, &h2)) {
        fprintf(stderr, "[bam-somaticsniper] cannot read BAM %s\n", argv[optind + 1]);
        return 1;
    }
    R.h1 = &h1;
    R.out = fopen(argv[optind + 2], "w");
    const int fmt = ss_format_lookup(fmt_name);
    if (fmt < 0) {
        fprintf(stderr, "unknown output format: '%s'. Abort!\n", fmt_name);
        exit(1);
    }
    R.fmt = fmt;
    if (!R.out) {
        fprintf(stderr, "Unable to open snp file!!!!!!!!!\n");
        exit(1);
    }
    const char *dump = getenv("SS_DUMP_PILEUP");
    if (dump && *dump) R.dump = fopen(dump, "w");
    const int pileup_only = env_int("SS_PILEUP_ONLY", 0);
    const int cap = env_int("SS_BATCH", 1 << 20);
    {   /* scorer devices: SS_DEVICES=0,1,.. or SS_DEVICE */
        const char *devs = getenv("SS_DEVICES");
        if (devs && *devs && parse_devices(devs, R.device, &R.n_dev)) return 1;
        if (R.n_dev == 0) R.device[R.n_dev++] = env_int("SS_DEVICE", 0);
    }
    R.pileup_only = pileup_only;
    R.prm = prm;
    ss_write_header(R.out, fmt, fn_fa, normal_id, tumor_id);
    const int bcap = cap > 0 ? cap : 1 << 20;
    /* indexed inputs: contig groups in parallel (returns 1 when not applicable) */
    const int grc = run_groups(&R, argv[optind], argv[optind + 1], mapq, bthreads, bcap, fn_fa);
    if (grc < 0) failed_set(&R);
    R.n_bat = grc == 1 ? R.n_dev + 3 : 0;
    for (int k = 0; k < R.n_bat; ++k) batch_init(&R.bat[k], (size_t)bcap);
    pthread_mutex_init(&R.mu, NULL);
    pthread_cond_init(&R.cv, NULL);
    if (grc == 1) {                                     /* the single streaming walk */
        scorer_arg_t sarg[MAX_DEV];
        run_scorers_start(&R, sarg);                    /* each creates its GPU scorer first */
        dual_pileup_run(fp1, fp2, (int)SS_BAM_DEF_MASK, mapq, env_int("SS_PILEUP_THREADS", 2), on_site, &R);
        stamp("pileup done");
        run_scorers_finish(&R);
    }
    bgzf_close(fp1);
    bgzf_close(fp2);
    bam_header_free(&h1);
    bam_header_free(&h2);
    fasta_index_free(R.fai);
    free(R.cur_ref);
    for (int k = 0; k < R.n_bat; ++k) batch_free(&R.bat[k]);
    stamp("output written");
    for (int k = 0; k < R.n_dev; ++k)
        if (g_ctx[k]) ss_ctx_destroy(g_ctx[k]);
    if (R.dump) fclose(R.dump);
    fclose(R.out);
    stamp("exit");
    return failed_get(&R) ? 1 : 0;
}
