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
 *
 * Reuse: the reference rebuilds 32.5 MB of tables in
 * every process (0.63 s).  Here a built set is kept for the process (every
 * later context with the same table parameters shares it) and written to a
 * disk cache keyed by the table parameters AND the machine (CPU vendor /
 * family / model / stepping, glibc version): the tables are CPU-dependent, so
 * a blob is only ever reused on the kind of host that built it.  The key also
 * holds the builder's identity (SS_TABLE_BUILDER), so a blob from another
 * builder version is never picked up.  A blob is verified before use: the
 * FNV-1a hashes of its payload are recomputed and must equal the header's; a
 * corrupt or mismatching blob is ignored and replaced.  SS_TABLE_CACHE=<dir> chooses the
 * directory (default $XDG_CACHE_HOME/sniper_amd or ~/.cache/sniper_amd),
 * SS_TABLE_CACHE=off disables the disk cache.
 */
#include <errno.h>
#include <gnu/libc-version.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

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

/* samtools-0.1.6 bam_nt16_table (bam_import.c:23-40): the IUPAC letters of
 * "=ACMGRSVTWYHKDBN" in both cases map to their 4-bit code, '=' to 0, colour
 * digits 0-3 to A,C,G,T, everything else to 15 (N).  Immutable and initialised
 * at load time: contexts created concurrently from several threads upload it
 * while others are being built, so it must never be written at run time
 * (tests/test_abi_cpu.py::test_nt16_table_immutable_under_concurrent_builds). */
const unsigned char ss_nt16_table[256] = {
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
     1,  2,  4,  8, 15, 15, 15, 15, 15, 15, 15, 15, 15,  0, 15, 15,   /* '0'-'3', '=' */
    15,  1, 14,  2, 13, 15, 15,  4, 11, 15, 15, 12, 15,  3, 15, 15,   /* '@' 'A'..'O' */
    15, 15,  5,  6,  8, 15,  7,  9, 15, 10, 15, 15, 15, 15, 15, 15,   /* 'P'..'_'     */
    15,  1, 14,  2, 13, 15, 15,  4, 11, 15, 15, 12, 15,  3, 15, 15,   /* '`' 'a'..'o' */
    15, 15,  5,  6,  8, 15,  7,  9, 15, 10, 15, 15, 15, 15, 15, 15,   /* 'p'..DEL     */
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
    15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,
};

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

/* Position-keyed word sum (ss_kernels.hip ss_tab_fingerprint computes the same
 * on the device, in any order): word i of the device table image contributes
 * mix(w + i * golden).  Used to verify that a context's device tables still
 * hold what was uploaded (ss_ctx_create, ss_ctx_check). */
static uint64_t fp_mix(uint64_t x)
{
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

uint64_t ss_tab_fp_words(const void *p, size_t nwords, uint64_t first_word)
{
    const unsigned char *b = (const unsigned char *)p;
    uint64_t s = 0, w;
    size_t i;
    for (i = 0; i < nwords; ++i) {
        memcpy(&w, b + 8 * i, 8);
        s += fp_mix(w + (first_word + i) * 0x9e3779b97f4a7c15ull);
    }
    return s;
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

/* ------------------------------------------------------- table reuse ---- */
/* the parameters the big tables depend on (fk/coef: theta, eta; lhet/q_r:
 * n_hap, het_rate); the Phred tables are rebuilt per context (microseconds) */
typedef struct {
    float theta, eta, het_rate;
    int n_hap;
} tab_key_t;

typedef struct tab_entry {
    tab_key_t key;
    double fk[256];
    double *coef, *lhet;
    float q_r;
    int q_r_int;
    uint64_t h_fk, h_coef, h_lhet;
    uint64_t fp_coef, fp_lhet;           /* ss_tab_fp_words at their device offsets */
    struct tab_entry *next;
} tab_entry_t;

static pthread_mutex_t g_tab_lock = PTHREAD_MUTEX_INITIALIZER;
static tab_entry_t *g_tabs;               /* kept for the life of the process */
static __thread int g_last_source = -1;
static int g_warned_unpinned;

#define SS_COEF_N ((size_t)64 << 16)
#define SS_LHET_N ((size_t)65536)
#define SS_BLOB_MAGIC 0x3230424154535353ull   /* "SSSTAB02" */
/* Identity of the table builder: a blob written by another version of
 * build_coef / build_lhet / build flags must never be reused.  Bump the
 * version whenever either builder or the host compile flags change; the
 * string is part of the cache key (key_hash). */
#define SS_TABLE_BUILDER "ss_tables v3: build_coef/build_lhet x87, gcc -O2 -ffp-contract=off -fno-fast-math"

typedef struct {
    uint64_t magic, key_hash;
    uint64_t h_fk, h_coef, h_lhet;       /* FNV-1a-64 (the pinning hashes), recomputed on load */
    float q_r;
    int32_t q_r_int;
    uint64_t payload;                      /* bytes after the header */
} blob_hdr_t;

static tab_key_t tab_key(const ss_params_t *p)
{
    tab_key_t k;
    memset(&k, 0, sizeof k);
    k.theta = p->theta;
    k.eta = p->eta;
    k.het_rate = p->het_rate;
    k.n_hap = p->n_hap;
    return k;
}

/* machine signature: what the tables' last bits depend on */
static void machine_sig(char *out, size_t cap)
{
    char vendor[64] = "?", family[16] = "?", model[16] = "?", stepping[16] = "?", line[512];
    FILE *f = fopen("/proc/cpuinfo", "r");
    if (f) {
        while (fgets(line, sizeof line, f)) {
            char *v = strchr(line, ':');
            if (!v) continue;
            v += 1 + (v[1] == ' ');
            v[strcspn(v, "\n")] = 0;
            if (!strncmp(line, "vendor_id", 9)) snprintf(vendor, sizeof vendor, "%s", v);
            else if (!strncmp(line, "cpu family", 10)) snprintf(family, sizeof family, "%s", v);
            else if (!strncmp(line, "model\t", 6)) snprintf(model, sizeof model, "%s", v);
            else if (!strncmp(line, "stepping", 8)) { snprintf(stepping, sizeof stepping, "%s", v); break; }
        }
        fclose(f);
    }
    snprintf(out, cap, "%s/%s/%s/%s/glibc-%s/ld%zu", vendor, family, model, stepping, gnu_get_libc_version(),
             sizeof(long double));
}

static uint64_t key_hash(const tab_key_t *k)
{
    char sig[256];
    uint64_t h;
    machine_sig(sig, sizeof sig);
    h = ss_fnv1a64(k, sizeof *k) ^ 0x9e3779b97f4a7c15ull;
    h ^= ss_fnv1a64(SS_TABLE_BUILDER, sizeof SS_TABLE_BUILDER - 1) * 0xff51afd7ed558ccdull;
    return h ^ (ss_fnv1a64(sig, strlen(sig)) * 0x100000001b3ull);
}

/* cache directory; 0 when the disk cache is off */
static int cache_dir(char *out, size_t cap)
{
    const char *e = getenv("SS_TABLE_CACHE"), *x, *home;
    if (e && (!strcmp(e, "off") || !strcmp(e, "0") || !*e)) return 0;
    if (e) snprintf(out, cap, "%s", e);
    else if ((x = getenv("XDG_CACHE_HOME")) && *x) snprintf(out, cap, "%s/sniper_amd", x);
    else if ((home = getenv("HOME")) && *home) snprintf(out, cap, "%s/.cache/sniper_amd", home);
    else return 0;
    return 1;
}

static int blob_path(const tab_key_t *k, char *out, size_t cap)
{
    char dir[3072];
    if (!cache_dir(dir, sizeof dir)) return 0;
    snprintf(out, cap, "%s/tables-%016llx.bin", dir, (unsigned long long)key_hash(k));
    return 1;
}

static int blob_load(const tab_key_t *k, tab_entry_t *t)
{
    char path[4096];
    blob_hdr_t h;
    FILE *f;
    int ok = 0;
    if (!blob_path(k, path, sizeof path) || !(f = fopen(path, "rb"))) return 0;
    if (fread(&h, sizeof h, 1, f) == 1 && h.magic == SS_BLOB_MAGIC && h.key_hash == key_hash(k) &&
        h.payload == sizeof t->fk + (SS_COEF_N + SS_LHET_N) * sizeof(double) &&
        fread(t->fk, sizeof t->fk, 1, f) == 1 && fread(t->coef, sizeof(double), SS_COEF_N, f) == SS_COEF_N &&
        fread(t->lhet, sizeof(double), SS_LHET_N, f) == SS_LHET_N) {
        /* the pinning hashes are recomputed from the payload (about 30 ms), never
         * taken from the header: a corrupt, truncated or foreign blob whose bytes
         * differ from what its header claims is rebuilt */
        t->h_fk = ss_fnv1a64(t->fk, sizeof t->fk);
        t->h_coef = ss_fnv1a64(t->coef, SS_COEF_N * sizeof(double));
        t->h_lhet = ss_fnv1a64(t->lhet, SS_LHET_N * sizeof(double));
        ok = t->h_fk == h.h_fk && t->h_coef == h.h_coef && t->h_lhet == h.h_lhet;
        t->q_r = h.q_r;
        t->q_r_int = h.q_r_int;
    }
    fclose(f);
    return ok;
}

/* write-to-temp + rename, so a concurrent reader sees a whole blob or none */
static void blob_store(const tab_key_t *k, const tab_entry_t *t)
{
    char path[4096], tmp[4200], dir[3072];
    blob_hdr_t h;
    FILE *f;
    if (!cache_dir(dir, sizeof dir) || !blob_path(k, path, sizeof path)) return;
    {   /* mkdir -p of the directory */
        char d[3072];
        size_t i, n = strlen(dir);
        memcpy(d, dir, n + 1);
        for (i = 1; i <= n; ++i)
            if (d[i] == '/' || d[i] == 0) {
                const char c = d[i];
                d[i] = 0;
                if (mkdir(d, 0755) != 0 && errno != EEXIST) return;
                d[i] = c;
            }
    }
    snprintf(tmp, sizeof tmp, "%s.%d.tmp", path, (int)getpid());
    if (!(f = fopen(tmp, "wb"))) return;
    memset(&h, 0, sizeof h);
    h.magic = SS_BLOB_MAGIC;
    h.key_hash = key_hash(k);
    h.h_fk = t->h_fk;
    h.h_coef = t->h_coef;
    h.h_lhet = t->h_lhet;
    h.q_r = t->q_r;
    h.q_r_int = t->q_r_int;
    h.payload = sizeof t->fk + (SS_COEF_N + SS_LHET_N) * sizeof(double);
    if (fwrite(&h, sizeof h, 1, f) == 1 && fwrite(t->fk, sizeof t->fk, 1, f) == 1 &&
        fwrite(t->coef, sizeof(double), SS_COEF_N, f) == SS_COEF_N &&
        fwrite(t->lhet, sizeof(double), SS_LHET_N, f) == SS_LHET_N && fclose(f) == 0) {
        if (rename(tmp, path) != 0) unlink(tmp);
        return;
    }
    fclose(f);
    unlink(tmp);
}

/* the entry for p's table parameters: this process's, the disk cache's, or
 * freshly built (then stored).  Called with g_tab_lock held. */
static int tab_get(const ss_params_t *p, tab_entry_t **out, int *source)
{
    const tab_key_t k = tab_key(p);
    tab_entry_t *t;
    ss_host_model_t b;
    int rc;
    for (t = g_tabs; t; t = t->next)
        if (!memcmp(&t->key, &k, sizeof k)) { *out = t; *source = SS_TABLES_PROCESS; return SS_OK; }
    t = (tab_entry_t *)calloc(1, sizeof *t);
    if (!t) return SS_E_NOMEM;
    t->key = k;
    t->coef = (double *)malloc(SS_COEF_N * sizeof(double));
    t->lhet = (double *)malloc(SS_LHET_N * sizeof(double));
    if (!t->coef || !t->lhet) { free(t->coef); free(t->lhet); free(t); return SS_E_NOMEM; }
    if (blob_load(&k, t)) {
        *source = SS_TABLES_DISK;
    } else {
        memset(&b, 0, sizeof b);
        b.prm = *p;
        free(t->coef);
        free(t->lhet);
        t->coef = t->lhet = NULL;
        if ((rc = build_coef(&b)) != SS_OK || (rc = build_lhet(&b)) != SS_OK) {
            free(b.coef); free(b.lhet); free(t);
            return rc;
        }
        memcpy(t->fk, b.fk, sizeof t->fk);
        t->coef = b.coef;
        t->lhet = b.lhet;
        t->q_r = b.q_r;
        t->q_r_int = b.q_r_int;
        t->h_fk = ss_fnv1a64(t->fk, sizeof t->fk);
        t->h_coef = ss_fnv1a64(t->coef, SS_COEF_N * sizeof(double));
        t->h_lhet = ss_fnv1a64(t->lhet, SS_LHET_N * sizeof(double));
        blob_store(&k, t);
        *source = SS_TABLES_BUILT;
    }
    t->fp_coef = ss_tab_fp_words(t->coef, SS_COEF_N, SS_FP_COEF_WORD);
    t->fp_lhet = ss_tab_fp_words(t->lhet, SS_LHET_N, SS_FP_LHET_WORD);
    t->next = g_tabs;
    g_tabs = t;
    *out = t;
    return SS_OK;
}

int ss_host_model_build(const ss_params_t *p, ss_host_model_t *m)
{
    int rc, source = SS_TABLES_BUILT;
    tab_entry_t *t = NULL;
    memset(m, 0, sizeof(*m));
    if (!p || p->n_hap < 2 || p->n_hap > 255 || !(p->theta > 0.0f) || p->cap_mapQ < 0)
        return SS_E_INVAL;
    pthread_mutex_lock(&g_tab_lock);
    rc = tab_get(p, &t, &source);
    pthread_mutex_unlock(&g_tab_lock);
    if (rc != SS_OK) return rc;
    m->prm = *p;
    memcpy(m->fk, t->fk, sizeof m->fk);
    m->coef = t->coef;                     /* shared, owned by the process-wide entry */
    m->lhet = t->lhet;
    m->q_r = t->q_r;
    m->q_r_int = t->q_r_int;
    m->h_fk = t->h_fk;
    m->h_coef = t->h_coef;
    m->h_lhet = t->h_lhet;
    m->fp_coef = t->fp_coef;
    m->fp_lhet = t->fp_lhet;
    m->shared = t;
    m->source = source;
    g_last_source = source;
    build_phred(m);
    if (params_are_default(p)) {
        const uint64_t h[3] = {m->h_fk, m->h_coef, m->h_lhet};
        const char *strict = getenv("SS_STRICT_TABLES");
        m->pinned = ss_model_pinned(h);
        if (!m->pinned) {
            if (strict && strict[0] == '1') {
                memset(m, 0, sizeof(*m));
                return SS_E_TABLES;   /* no pinned reference run produced these tables */
            }
            pthread_mutex_lock(&g_tab_lock);
            if (!g_warned_unpinned) {
                g_warned_unpinned = 1;
                fprintf(stderr, "[sniper_amd] warning: the model tables built on this host (fk %016llx coef %016llx "
                        "lhet %016llx) match no pinned run of the reference; scores equal the reference's only if "
                        "it builds the same tables here (SS_STRICT_TABLES=1 refuses such tables)\n",
                        (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2]);
            }
            pthread_mutex_unlock(&g_tab_lock);
        }
    }
    return SS_OK;
}

void ss_host_model_free(ss_host_model_t *m)
{
    /* coef / lhet belong to the process-wide entry (reused by later contexts) */
    m->coef = m->lhet = NULL;
    m->shared = NULL;
}

int ss_model_last_source(void) { return g_last_source; }

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
