/*
 * oracle/ref_harness.c -- drives the REAL reference scorer (compiled from
 * /root/reference by oracle/ref.mk) on our packed site batches.
 *
 * TEST INFRASTRUCTURE ONLY.  Used to (1) generate golden vectors from the actual
 * reference code, (2) pin the CPU restatement (oracle/ss_oracle.c), and (3) time
 * the reference hot path as bench.py's cpu_baseline ("kind": "reference").
 *
 * It fabricates, per packed read, a one-base bam1_t (seq + qual at qpos 0,
 * core.qual = mapQ, BAM_FREVERSE = strand) and a bam_pileup1_t pointing at it,
 * then calls the reference entry points exactly as sniper_pileup.c:256-258 does:
 *   glf_somatic(tid, pos, n1, n2, pl1, pl2, data, fh)     somatic_sniper.c:109
 * plus sniper_maqcns_glfgen / sniper_maqcns_call (sniper_maqcns.c:127,275) to
 * export the per-sample glf1_t and consensus words.
 * A sample whose packed depth is 0 is given one is_del=1 entry, which is what the
 * dual pileup hands glf_somatic when every read at the site is a deletion.
 *
 * usage:
 *   ref_harness tables
 *   ref_harness dump  BATCH.ssb OUT.ssr TEXT_OUT [opts]
 *   ref_harness synth LAMBDA_T LAMBDA_N N_SITES [--seed S] [--shard K] [--scores F] [opts]
 * opts: -T theta -N nhap -r het -p -J -s rate -Q minq -L -G -F fmt
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "bam.h"
#include "glf.h"
#include "sniper_maqcns.h"
#include "somatic_sniper.h"
#include "output_format.h"

#include "sniper_amd.h"

static uint64_t fnv1a(const void *p, size_t n, uint64_t h)
{
    const uint8_t *b = (const uint8_t *)p;
    size_t i;
    for (i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
    return h;
}
#define FNV0 0xcbf29ce484222325ull

typedef struct {
    bam1_t *b;
    uint8_t *data;
    bam_pileup1_t *pl;
    int cap;
} pile_t;

static void pile_reserve(pile_t *p, int n)
{
    int i;
    if (n <= p->cap) return;
    p->b = (bam1_t *)realloc(p->b, sizeof(bam1_t) * n);
    p->data = (uint8_t *)realloc(p->data, 4 * n);
    p->pl = (bam_pileup1_t *)realloc(p->pl, sizeof(bam_pileup1_t) * n);
    p->cap = n;
    for (i = 0; i < n; ++i) {
        memset(&p->b[i], 0, sizeof(bam1_t));
        p->b[i].data = p->data + 4 * i;
        p->b[i].data_len = p->b[i].m_data = 2;
        p->b[i].core.l_qseq = 1;
        memset(&p->pl[i], 0, sizeof(bam_pileup1_t));
        p->pl[i].b = &p->b[i];
    }
}

/* Build the pileup of one sample; returns the entry count handed to the callback. */
static int pile_fill(pile_t *p, const uint32_t *reads, int n)
{
    int i;
    pile_reserve(p, n > 0 ? n : 1);
    if (n == 0) { /* all reads deleted: one is_del entry */
        p->b[0].data[0] = 0; p->b[0].data[1] = 0; p->b[0].core.qual = 0; p->b[0].core.flag = 0;
        p->pl[0].is_del = 1; p->pl[0].qpos = 0;
        return 1;
    }
    for (i = 0; i < n; ++i) {
        uint32_t r = reads[i];
        bam1_t *b = &p->b[i];
        b->data[0] = (uint8_t)(SS_READ_NT16(r) << 4);
        b->data[1] = (uint8_t)SS_READ_BASEQ(r);
        b->core.qual = SS_READ_MAPQ(r);
        b->core.flag = SS_READ_STRAND(r) ? BAM_FREVERSE : 0;
        p->pl[i].is_del = 0;
        p->pl[i].qpos = 0;
    }
    return n;
}

typedef struct {
    float theta, het; int nhap, priors, joint, minq, loh, gor;
    double rate; const char *fmt;
} opts_t;

static int parse_opt(opts_t *o, int argc, char **argv, int *i)
{
    const char *a = argv[*i];
    if (!strcmp(a, "-T")) o->theta = (float)atof(argv[++*i]);
    else if (!strcmp(a, "-N")) o->nhap = atoi(argv[++*i]);
    else if (!strcmp(a, "-r")) o->het = (float)atof(argv[++*i]);
    else if (!strcmp(a, "-p")) o->priors = 0;
    else if (!strcmp(a, "-J")) o->joint = 1;
    else if (!strcmp(a, "-s")) { o->rate = atof(argv[++*i]); o->joint = 1; }
    else if (!strcmp(a, "-Q")) o->minq = atoi(argv[++*i]);
    else if (!strcmp(a, "-L")) o->loh = 0;
    else if (!strcmp(a, "-G")) o->gor = 0;
    else if (!strcmp(a, "-F")) o->fmt = argv[++*i];
    else return 0;
    (void)argc;
    return 1;
}

static pu_data2_t *setup(const opts_t *o, const char *ref, int len, FILE *fh,
                         output_formatter_t *fmt)
{
    pu_data2_t *d = (pu_data2_t *)calloc(1, sizeof(pu_data2_t));
    bam_header_t *h = bam_header_init();
    h->n_targets = 1;
    h->target_name = (char **)calloc(1, sizeof(char *));
    h->target_name[0] = strdup("synth");
    h->target_len = (uint32_t *)calloc(1, sizeof(uint32_t));
    h->target_len[0] = (uint32_t)len;
    d->h1 = d->h2 = h;
    d->c = sniper_maqcns_init();
    d->c->theta = o->theta; d->c->n_hap = o->nhap; d->c->het_rate = o->het;
    d->min_somatic_qual = o->minq;
    d->include_loh = o->loh; d->include_gor = o->gor;
    d->use_joint_priors = o->joint; d->somatic_mutation_rate = o->rate;
    d->mask = BAM_DEF_MASK;
    /* same order as main.c:115-127 */
    if (d->use_joint_priors) make_joint_prior(d->somatic_mutation_rate);
    sniper_maqcns_prepare(d->c);
    if (o->priors) makeSoloPrior();
    qAddTableInit();
    d->fai = NULL;
    d->tid = 0;
    d->ref = (char *)ref;
    d->len = len;
    *fmt = output_formatter_create(o->fmt, fh);
    d->output_formatter = fmt;
    return d;
}

static void glf_export(const glf1_t *g, ss_glf_t *o)
{
    int i;
    memset(o, 0, sizeof(*o));
    o->ref_base = g->ref_base; o->max_mapQ = g->max_mapQ;
    for (i = 0; i < 10; ++i) o->lk[i] = g->lk[i];
    o->min_lk = g->min_lk; o->depth = g->depth;
}

static void *read_all(const char *fn, size_t *n)
{
    FILE *f = fopen(fn, "rb");
    void *buf;
    if (!f) { perror(fn); exit(2); }
    fseek(f, 0, SEEK_END); *n = (size_t)ftell(f); fseek(f, 0, SEEK_SET);
    buf = malloc(*n ? *n : 1);
    if (fread(buf, 1, *n, f) != *n) { perror("fread"); exit(2); }
    fclose(f);
    return buf;
}

static int cmd_tables(void)
{
    sniper_maqcns_t *c = sniper_maqcns_init();
    sniper_maqcns_prepare(c);
    printf("{\"fk\": \"%016llx\", \"coef\": \"%016llx\", \"lhet\": \"%016llx\", \"q_r\": %.9g}\n",
           (unsigned long long)fnv1a(c->fk, 256 * 8, FNV0),
           (unsigned long long)fnv1a(c->coef, 64 * 65536 * 8, FNV0),
           (unsigned long long)fnv1a(c->lhet, 65536 * 8, FNV0), (double)c->q_r);
    sniper_maqcns_destroy(c);
    return 0;
}

static int cmd_dump(int argc, char **argv, opts_t *o)
{
    size_t sz, off;
    uint8_t *buf;
    uint64_t ns, nt, nn, i;
    const uint8_t *ref;
    const uint32_t *ot, *on, *rt, *rn;
    FILE *out, *txt;
    output_formatter_t fmt;
    pu_data2_t *d;
    pile_t pt = {0}, pn = {0};
    int a;
    if (argc < 5) return 2;
    for (a = 5; a < argc; ++a) if (!parse_opt(o, argc, argv, &a)) { fprintf(stderr, "bad opt %s\n", argv[a]); return 2; }
    buf = (uint8_t *)read_all(argv[2], &sz);
    if (sz < 32 || memcmp(buf, "SSB1", 4)) { fprintf(stderr, "bad batch file\n"); return 2; }
    memcpy(&ns, buf + 8, 8); memcpy(&nt, buf + 16, 8); memcpy(&nn, buf + 24, 8);
    off = 32;
    ref = buf + off; off += (ns + 3) & ~3ull;
    ot = (const uint32_t *)(buf + off); off += 4 * (ns + 1);
    on = (const uint32_t *)(buf + off); off += 4 * (ns + 1);
    rt = (const uint32_t *)(buf + off); off += 4 * nt;
    rn = (const uint32_t *)(buf + off); off += 4 * nn;
    if (off != sz) { fprintf(stderr, "batch size mismatch %zu vs %zu\n", off, sz); return 2; }
    out = fopen(argv[3], "wb");
    txt = fopen(argv[4], "w");
    if (!out || !txt) { perror("open"); return 2; }
    d = setup(o, (const char *)ref, (int)ns, txt, &fmt);
    for (i = 0; i < ns; ++i) {
        int n1 = pile_fill(&pt, rt + ot[i], (int)(ot[i + 1] - ot[i]));
        int n2 = pile_fill(&pn, rn + on[i], (int)(on[i + 1] - on[i]));
        int rb = ref[i];
        glf1_t *gt, *gn;
        ss_glf_t e[2];
        uint32_t ct, cn;
        int32_t ret;
        gt = sniper_maqcns_glfgen(n1, pt.pl, bam_nt16_table[rb], d->c);
        gn = sniper_maqcns_glfgen(n2, pn.pl, bam_nt16_table[rb], d->c);
        ct = sniper_maqcns_call(n1, gt, d->c);
        cn = sniper_maqcns_call(n2, gn, d->c);
        glf_export(gt, &e[0]); glf_export(gn, &e[1]);
        free(gt); free(gn);
        ret = glf_somatic(0, (uint32_t)i, n1, n2, pt.pl, pn.pl, d, txt);
        fwrite(&ret, 4, 1, out); fwrite(&ct, 4, 1, out); fwrite(&cn, 4, 1, out);
        fwrite(e, sizeof(e), 1, out);
    }
    fclose(out); fclose(txt);
    return 0;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int cmd_synth(int argc, char **argv, opts_t *o)
{
    ss_synth_t s;
    uint64_t ns, done = 0, first = 0, seed = 0x5EED5A1DC0FFEE01ull, h = FNV0, reads = 0;
    uint32_t shard = 0;
    const char *scores_fn = NULL;
    FILE *sf = NULL, *txt;
    double secs = 0.0;
    int a, chunk = 4096;
    long emitted = 0;
    uint8_t *ref;
    uint32_t *ot, *on, *rt = NULL, *rn = NULL;
    size_t rtc = 0, rnc = 0;
    int32_t *score;
    output_formatter_t fmt;
    pu_data2_t *d;
    pile_t pt = {0}, pn = {0};
    if (argc < 5) return 2;
    for (a = 5; a < argc; ++a) {
        if (!strcmp(argv[a], "--seed")) seed = strtoull(argv[++a], NULL, 0);
        else if (!strcmp(argv[a], "--shard")) shard = (uint32_t)atoi(argv[++a]);
        else if (!strcmp(argv[a], "--first")) first = strtoull(argv[++a], NULL, 0);   /* sites [first, first + n) */
        else if (!strcmp(argv[a], "--scores")) scores_fn = argv[++a];
        else if (!parse_opt(o, argc, argv, &a)) { fprintf(stderr, "bad opt %s\n", argv[a]); return 2; }
    }
    ss_synth_default(&s, atof(argv[2]), atof(argv[3]));
    s.seed = seed; s.shard = shard;
    ns = strtoull(argv[4], NULL, 0);
    txt = fopen("/dev/null", "w");
    if (scores_fn) sf = fopen(scores_fn, "wb");
    ref = (uint8_t *)malloc(chunk);
    ot = (uint32_t *)malloc(4 * (chunk + 1));
    on = (uint32_t *)malloc(4 * (chunk + 1));
    score = (int32_t *)malloc(4 * chunk);
    d = NULL;
    while (done < ns) {
        uint64_t m = ns - done < (uint64_t)chunk ? ns - done : (uint64_t)chunk, i, nt, nn;
        double t0;
        ss_synth_batch_host(&s, first + done, m, ref, ot, on, NULL, NULL, &nt, &nn);
        if (nt > rtc) { rtc = nt; rt = (uint32_t *)realloc(rt, 4 * rtc); }
        if (nn > rnc) { rnc = nn; rn = (uint32_t *)realloc(rn, 4 * rnc); }
        ss_synth_batch_host(&s, first + done, m, ref, ot, on, rt, rn, &nt, &nn);
        reads += nt + nn;
        if (!d) d = setup(o, (const char *)ref, chunk, txt, &fmt);
        d->ref = (char *)ref; d->len = (int)m;
        t0 = now_s();
        for (i = 0; i < m; ++i) {
            int n1 = pile_fill(&pt, rt + ot[i], (int)(ot[i + 1] - ot[i]));
            int n2 = pile_fill(&pn, rn + on[i], (int)(on[i + 1] - on[i]));
            score[i] = glf_somatic(0, (uint32_t)i, n1, n2, pt.pl, pn.pl, d, txt);
        }
        secs += now_s() - t0;
        for (i = 0; i < m; ++i) {
            if (score[i] >= 0 && score[i] != 255 && score[i] >= o->minq) ++emitted;
        }
        h = fnv1a(score, 4 * m, h);
        if (sf) fwrite(score, 4, m, sf);
        done += m;
    }
    if (sf) fclose(sf);
    printf("{\"sites\": %llu, \"reads\": %llu, \"seconds\": %.6f, \"sites_per_s\": %.1f, "
           "\"scores_fnv\": \"%016llx\", \"candidates_ge_minq\": %ld}\n",
           (unsigned long long)ns, (unsigned long long)reads, secs, secs > 0 ? ns / secs : 0.0,
           (unsigned long long)h, emitted);
    return 0;
}

int main(int argc, char **argv)
{
    opts_t o = {0.85f, 0.001f, 2, 1, 0, 15, 1, 1, 0.01, "classic"};
    if (argc < 2) goto usage;
    if (!strcmp(argv[1], "tables")) return cmd_tables();
    if (!strcmp(argv[1], "nt16")) { /* samtools-0.1.6/bam_import.c:23 */
        int i;
        for (i = 0; i < 256; ++i) printf("%d%c", bam_nt16_table[i], i == 255 ? '\n' : ',');
        return 0;
    }
    if (!strcmp(argv[1], "dump")) { int r = cmd_dump(argc, argv, &o); if (r == 2) goto usage; return r; }
    if (!strcmp(argv[1], "synth")) { int r = cmd_synth(argc, argv, &o); if (r == 2) goto usage; return r; }
usage:
    fprintf(stderr, "usage: ref_harness tables | dump BATCH OUT TXT [opts] | synth LT LN N [--seed S] [--shard K] [--first I] [--scores F] [opts]\n");
    return 2;
}
