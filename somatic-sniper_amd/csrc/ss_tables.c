/*
 * ss_tables.c -- host construction of the scorer's model tables.
 *
 * The tables are built on the HOST because they need x87 long double with
 * glibc's expl/logl (sniper_maqcns.c:59-100) -- the GPU has no 80-bit type.
 * They are then uploaded once per device (ss_capi.hip).  Everything here is
 * evaluated with the reference's C types and operand order so the doubles are
 * bit-identical; the result is checked against FNV-1a-64 hashes of the real
 * reference's tables (oracle/_ref/ref_harness tables) for default parameters.
 *
 *   fk[n], coef[q<<16|n<<8|k]   sniper_cal_coef   sniper_maqcns.c:59-100
 *   lhet[n1<<8|n2], q_r         sniper_cal_het    sniper_maqcns.c:27-56
 *   qadd[1024]                  qAddTableInit     somatic_sniper.c:101-107
 *   prior[16][10]               makeSoloPrior     somatic_sniper.c:29-45
 *   jprior[16][10][10]          make_joint_prior  somatic_sniper.c:47-77
 *
 * Build flags: -ffp-contract=off, no -ffast-math, no -march (x86-64 SSE2 double
 * + x87 long double, like the reference Release build).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "ss_host.h"

/* Reference hashes (FNV-1a-64 over little-endian doubles) of the default-parameter
 * tables, produced by the compiled reference itself (`oracle/_ref/ref_harness
 * tables`) on each host CPU family we run on.  The reference's coef table is
 * CPU-dependent: glibc's expl/logl use the x87 transcendental instructions,
 * whose last-bit results differ between Intel and AMD cores (98 of 4.2M coef
 * doubles differ).  The product therefore builds its tables on the host it runs
 * on -- exactly what the reference does there -- and records whether the result
 * matches a pinned reference run.  SS_STRICT_TABLES=1 turns an unpinned result
 * into SS_E_TABLES. */
static const uint64_t ss_ref_hashes[][3] = {
    /* Intel Xeon (build container), glibc 2.35 */
    {0x11bb85867221ee37ull, 0x86dcc255eecf756dull, 0xff15c0af94a22f15ull},
    /* AMD EPYC 9575F (MI355X host), glibc 2.35 */
    {0x11bb85867221ee37ull, 0x14fed40173e002b1ull, 0xff15c0af94a22f15ull},
};

int ss_model_pinned(const uint64_t h[3])
{
    size_t i;
    for (i = 0; i < sizeof(ss_ref_hashes) / sizeof(ss_ref_hashes[0]); ++i)
        if (h[0] == ss_ref_hashes[i][0] && h[1] == ss_ref_hashes[i][1] && h[2] == ss_ref_hashes[i][2])
            return 1;
    return 0;
}

unsigned char ss_nt16_table[256];

static void nt16_table_init(void)
{
    /* samtools-0.1.6 bam_nt16_table (bam_import.c:23-40): IUPAC letters in both
     * cases map to their 4-bit code, '=' to 0, colour digits 0-3 to A,C,G,T,
     * everything else to 15 (N). */
    static const char iupac[] = "=ACMGRSVTWYHKDBN";
    int c;
    for (c = 0; c < 256; ++c) ss_nt16_table[c] = 15;
    for (c = 0; c < 16; ++c) {
        unsigned char ch = (unsigned char)iupac[c];
        ss_nt16_table[ch] = (unsigned char)c;
        if (ch >= 'A' && ch <= 'Z') ss_nt16_table[ch | 0x20] = (unsigned char)c;
    }
    for (c = 0; c < 4; ++c) ss_nt16_table['0' + c] = (unsigned char)(1 << c);
}

uint64_t ss_fnv1a64(const void *p, size_t n)
{
    const unsigned char *b = (const unsigned char *)p;
    uint64_t h = 0xcbf29ce484222325ull;
    size_t i;
    for (i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

/* ---------------------------------------------------------------- coef ---- */
typedef struct {
    ss_host_model_t *m;
    const double *lbin;      /* log C(n,k) */
    const long double *fkh;  /* fk[k>>1] as long double (strand-halved decay) */
    int q_lo, q_hi;
} coef_job_t;

/* One error-quality row block: for every depth n the MAQ coefficients c_{n,k}
 * (sniper_maqcns.c:77-96). */
static void *coef_rows(void *arg)
{
    coef_job_t *j = (coef_job_t *)arg;
    long double suffix[257], beta[256], cum[256];
    int q, n, k;
    for (q = j->q_lo; q < j->q_hi; ++q) {
        const double eps = pow(10.0, -q / 10.0);
        const double l_eps = log(eps), l_1m = log(1.0 - eps);
        for (n = 1; n < 256; ++n) {
            double *out = j->m->coef + ((size_t)q << 16 | (size_t)n << 8);
            /* suffix[k] = sum_{i>=k} C(n,i) eps^i (1-eps)^(n-i); beta = ratio */
            suffix[n + 1] = 0.0;
            for (k = n; k >= 0; --k) {
                suffix[k] = suffix[k + 1] + expl(j->lbin[n << 8 | k] + k * l_eps + (n - k) * l_1m);
                beta[k] = suffix[k + 1] / suffix[k];
                if (beta[k] > 0.99) beta[k] = 0.99;
            }
            for (k = 0; k != n; ++k) cum[k] = -4.343 * j->fkh[k] * logl(beta[k] / eps);
            for (k = 1; k != n; ++k) cum[k] += cum[k - 1];
            for (k = 0; k <= n; ++k) {
                long double last = -4.343 * logl(1.0 - expl(j->fkh[k] * logl(beta[k])));
                out[k] = (k ? cum[k - 1] : 0) + last;
            }
        }
    }
    return NULL;
}

static int build_coef(ss_host_model_t *m)
{
    enum { NT = 8 };
    double *lbin = (double *)calloc(256 * 256, sizeof(double));
    long double fkh[256];
    pthread_t th[NT];
    coef_job_t job[NT];
    int n, k, t, started = 0;
    if (!lbin) return SS_E_NOMEM;
    m->coef = (double *)calloc((size_t)64 << 16, sizeof(double));
    if (!m->coef) { free(lbin); return SS_E_NOMEM; }
    m->fk[0] = 1.0;
    fkh[0] = 1.0;
    for (n = 1; n != 256; ++n) {
        /* theta / eta are float fields promoted to double (sniper_maqcns.h:14-17) */
        m->fk[n] = pow(m->prm.theta, n) * (1.0 - m->prm.eta) + m->prm.eta;
        fkh[n] = m->fk[n >> 1];
    }
    for (n = 1; n != 256; ++n)
        for (k = 1; k <= n; ++k)
            lbin[n << 8 | k] = lgamma(n + 1) - lgamma(k + 1) - lgamma(n - k + 1);
    /* q = 1..63 split over threads; each element is computed independently, so
     * the bytes do not depend on the split. */
    for (t = 0; t < NT; ++t) {
        job[t].m = m; job[t].lbin = lbin; job[t].fkh = fkh;
        job[t].q_lo = 1 + (63 * t) / NT;
        job[t].q_hi = 1 + (63 * (t + 1)) / NT;
    }
    for (t = 1; t < NT; ++t)
        if (pthread_create(&th[t], NULL, coef_rows, &job[t]) == 0) started |= 1 << t;
        else coef_rows(&job[t]);
    coef_rows(&job[0]);
    for (t = 1; t < NT; ++t)
        if (started & (1 << t)) pthread_join(th[t], NULL);
    free(lbin);
    return SS_OK;
}

/* ---------------------------------------------------------------- lhet ---- */
static int build_lhet(ss_host_model_t *m)
{
    const int H = m->prm.n_hap;
    double harmonic = 0.0, poly;
    int i, a, b;
    m->lhet = (double *)calloc(256 * 256, sizeof(double));
    if (!m->lhet) return SS_E_NOMEM;
    for (i = 1; i <= H - 1; ++i) harmonic += 1.0 / i;
    for (a = 0; a < 256; ++a) {
        for (b = 0; b < 256; ++b) {
            /* log P(D | het) for n1=a reads of one allele, n2=b of the other */
            const double lbinom = lgamma(a + b + 1) - lgamma(a + 1) - lgamma(b + 1);
            long double mix = 0.0;
            for (i = 1; i <= H - 1; ++i) {
                const double pk = 1.0 / i / harmonic;
                const double la = log((double)i / H);
                const double lb = log(1.0 - (double)i / H);
                mix += pk * 0.5 * (expl(la * b) * expl(lb * a) + expl(la * a) * expl(lb * b));
            }
            m->lhet[a << 8 | b] = lbinom + logl(mix);
        }
    }
    poly = m->prm.het_rate * harmonic;
    m->q_r = -4.343 * log(2.0 * poly / (1.0 - poly));
    m->q_r_int = (int)(m->q_r + .5);
    return SS_OK;
}

/* ------------------------------------------------- Phred-space tables ---- */
static int log_phred(double x)   /* logPhred, somatic_sniper.h:14 */
{
    return (int)(x < 1 ? (0.5 - 4.343 * log(x)) : (-0.5 - 4.343 * log(x)));
}

static int popcount4(int x) { return (x & 1) + (x >> 1 & 1) + (x >> 2 & 1) + (x >> 3 & 1); }

/* genotype index -> nt16 allele set (glfBase, somatic_sniper.c:26) */
const int ss_genotype_nt16[10] = {1, 3, 5, 9, 2, 6, 10, 4, 12, 8};

static void build_phred(ss_host_model_t *m)
{
    const double THETA = 0.001;  /* somatic_sniper.c:14 */
    int i, r, g, h;
    memset(m->qadd, 0, sizeof(m->qadd));  /* entries 1000..1023 stay 0 */
    for (i = 0; i < 1000; ++i) m->qadd[i] = log_phred(1 + (double)exp((double)(-(i - 512)) / 4.343));
    memset(m->prior, 0, sizeof(m->prior));
    memset(m->jprior, 0, sizeof(m->jprior));
    for (r = 0; r < 16; ++r) {
        for (g = 0; g < 10; ++g) {
            const int alle = ss_genotype_nt16[g];
            int germ;
            if ((alle & ~r) == 0) germ = 0;                       /* compatible with ref */
            else if (alle & r) germ = log_phred(THETA);           /* one novel allele    */
            else if (popcount4(alle) == 1) germ = log_phred(0.5 * THETA); /* hom mutant */
            else germ = log_phred(THETA * THETA);                 /* two mutations       */
            if (m->prm.use_priors) m->prior[r * 10 + g] = germ;
            if (!m->prm.use_joint_priors) continue;
            for (h = 0; h < 10; ++h) {
                const int tum = ss_genotype_nt16[h];
                int add;
                /* the reference tests isHet[h]/isHom[h] with the genotype INDEX h
                 * (somatic_sniper.c:66-70), i.e. popcount of h in {1,2}: true for
                 * every h except 0 and 7. */
                const int one_step = (alle & tum) && (popcount4(h) == 1 || (popcount4(h) == 2 && h <= 12));
                if (alle == tum) add = 0;
                else if (one_step) add = log_phred(m->prm.somatic_rate);
                else add = log_phred(m->prm.somatic_rate * m->prm.somatic_rate);
                m->jprior[(r * 10 + g) * 10 + h] = germ + add;
            }
        }
    }
}

/* ----------------------------------------------------------------- API ---- */
void ss_params_default(ss_params_t *p)
{
    memset(p, 0, sizeof(*p));
    p->theta = 0.85f;        /* sniper_maqcns.c:107-111 */
    p->n_hap = 2;
    p->het_rate = 0.001f;
    p->eta = 0.03f;
    p->cap_mapQ = 60;
    p->min_somatic_qual = 15; /* main.c:70-78 */
    p->use_priors = 1;
    p->use_joint_priors = 0;
    p->somatic_rate = 0.01;
    p->include_loh = 1;
    p->include_gor = 1;
}

static int params_are_default(const ss_params_t *p)
{
    ss_params_t d;
    ss_params_default(&d);
    return p->theta == d.theta && p->n_hap == d.n_hap && p->het_rate == d.het_rate &&
           p->eta == d.eta;
}

int ss_host_model_build(const ss_params_t *p, ss_host_model_t *m)
{
    int rc;
    memset(m, 0, sizeof(*m));
    if (!p || p->n_hap < 2 || p->n_hap > 255 || !(p->theta > 0.0f) || p->cap_mapQ < 0)
        return SS_E_INVAL;
    nt16_table_init();
    m->prm = *p;
    if ((rc = build_coef(m)) != SS_OK) goto fail;
    if ((rc = build_lhet(m)) != SS_OK) goto fail;
    build_phred(m);
    m->h_fk = ss_fnv1a64(m->fk, sizeof(m->fk));
    m->h_coef = ss_fnv1a64(m->coef, ((size_t)64 << 16) * sizeof(double));
    m->h_lhet = ss_fnv1a64(m->lhet, 65536 * sizeof(double));
    if (params_are_default(p)) {
        const uint64_t h[3] = {m->h_fk, m->h_coef, m->h_lhet};
        const char *strict = getenv("SS_STRICT_TABLES");
        m->pinned = ss_model_pinned(h);
        if (!m->pinned && strict && strict[0] == '1') {
            rc = SS_E_TABLES;   /* no pinned reference run produced these tables */
            goto fail;
        }
    }
    return SS_OK;
fail:
    ss_host_model_free(m);
    return rc;
}

void ss_host_model_free(ss_host_model_t *m)
{
    free(m->coef);
    free(m->lhet);
    m->coef = m->lhet = NULL;
}

int ss_model_check(const ss_params_t *p, uint64_t hashes[3], float *q_r)
{
    ss_host_model_t m;
    int rc = ss_host_model_build(p, &m);
    if (rc != SS_OK) {
        /* still report what this host computes, for diagnosis */
        if (rc == SS_E_TABLES && hashes) hashes[0] = hashes[1] = hashes[2] = 0;
        return rc;
    }
    if (hashes) { hashes[0] = m.h_fk; hashes[1] = m.h_coef; hashes[2] = m.h_lhet; }
    if (q_r) *q_r = m.q_r;
    ss_host_model_free(&m);
    return SS_OK;
}
