/* column_pileup.c -- see column_pileup.h for the rules being reproduced.
 *
 * A producer thread reads records, keeps the loaded ones in load order, and
 * whenever the finalisation frontier W has moved far enough it builds the
 * columns of the window [lo, hi) in two passes over the loaded reads:
 * difference arrays give every column's raw and packed entry counts, a prefix
 * sum gives each column's slice of the output, and a second pass scatters the
 * packed entries (load order within a column is kept because reads are
 * visited in load order).  The columns go to the consumer in chunks through
 * a small ring, as the positions of a compressed sparse row batch. */
#include "column_pileup.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bam_reader.h"

#define SEG_MIN    1024
#define SEG_MAX    2048
#define CHUNK_MIN  16384      /* columns per published chunk */
#define N_CHUNKS   8

typedef struct {
    int64_t beg, end;         /* reference span (bam_calend) */
    int64_t from;             /* first position not yet built for this read */
    uint32_t pk;              /* mapQ | strand << 20 */
    int single;               /* one M operation covering [beg, end) */
    bam_record_t b;
} cread_t;

typedef struct {
    int32_t *hdr;             /* tid, pos, r, np per column */
    uint32_t *pk;
    size_t n, cap, n_pk, cap_pk;
    int last;                 /* the stream ends after this chunk */
} chunk_t;

struct col_stream {
    bgzf_reader_t *fp;
    uint32_t flag_mask;
    int mapq_thresh;
    /* producer state */
    cread_t **act;            /* loaded reads, load order */
    int n_act, m_act;
    cread_t **pool;           /* recycled reads (their buffers are reused) */
    int n_pool, m_pool;
    int32_t *raw, *npk;       /* window difference arrays / counts, SEG_MAX + 1 */
    uint32_t *off;
    uint32_t *wbuf;           /* the window's entries */
    size_t cap_w;
    int error;
    /* ring */
    chunk_t chunks[N_CHUNKS];
    chunk_t *fill;
    uint64_t produced, consumed;
    int stop;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    pthread_t th;
    /* consumer cursor */
    chunk_t *cur;
    size_t step, pk_off;
    int ended;
};

static void *xalloc(void *p, size_t n)
{
    void *q = realloc(p, n ? n : 1);
    if (!q) { fprintf(stderr, "out of memory\n"); exit(1); }
    return q;
}

/* ---- ring -------------------------------------------------------------- */
static chunk_t *chunk_acquire(col_stream_t *S)
{
    pthread_mutex_lock(&S->mu);
    while (!S->stop && S->produced - S->consumed >= N_CHUNKS) pthread_cond_wait(&S->cv, &S->mu);
    chunk_t *c = S->stop ? NULL : &S->chunks[S->produced % N_CHUNKS];
    pthread_mutex_unlock(&S->mu);
    if (c) { c->n = c->n_pk = 0; c->last = 0; }
    return c;
}

static void chunk_publish(col_stream_t *S)
{
    pthread_mutex_lock(&S->mu);
    ++S->produced;
    pthread_cond_broadcast(&S->cv);
    pthread_mutex_unlock(&S->mu);
    S->fill = NULL;
}

/* ---- window build ---------------------------------------------------------- */
static void add_run(int32_t *d, int64_t a, int64_t b, int64_t lo, int64_t hi)
{
    if (a < lo) a = lo;
    if (b > hi) b = hi;
    if (a < b) { ++d[a - lo]; --d[b - lo]; }
}

/* Packed entries of query offsets q0 .. q0+n-1 appended to n consecutive
 * columns (off: each column's next output slot). */
static void scatter_run(uint32_t *restrict out, uint32_t *restrict off, uint32_t pk,
                        const uint8_t *restrict seq, const uint8_t *restrict qual, uint32_t q0, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t q = q0 + i;
        out[off[i]] = pk | (uint32_t)qual[q] << 8 | (uint32_t)((seq[q >> 1] >> ((~q & 1u) << 2)) & 0xfu) << 16;
    }
    for (uint32_t i = 0; i < n; ++i) ++off[i];
}

/* Builds and publishes the columns of contig tid in [lo, hi), hi - lo <= SEG_MAX.
 * Returns 0, or -1 when the consumer has gone. */
static int build_window(col_stream_t *S, int32_t tid, int64_t lo, int64_t hi)
{
    const int64_t len = hi - lo;
    int32_t *raw = S->raw, *npk = S->npk;
    memset(raw, 0, sizeof(int32_t) * (size_t)(len + 1));
    memset(npk, 0, sizeof(int32_t) * (size_t)(len + 1));
    /* pass 1: entry counts per column */
    for (int i = 0; i < S->n_act; ++i) {
        const cread_t *r = S->act[i];
        const int64_t from = r->from > lo ? r->from : lo;
        if (r->single) {
            add_run(raw, from, r->end, lo, hi);
            add_run(npk, from, r->end, lo, hi);
            continue;
        }
        const uint32_t *cig = bam_rec_cigar(&r->b);
        int64_t x = r->beg;
        for (int k = 0; k < r->b.n_cigar && x < hi; ++k) {
            const uint32_t op = cig[k] & 0xf, l = cig[k] >> 4;
            if (op == SS_CIG_M) {
                add_run(raw, x > from ? x : from, x + l, lo, hi);
                add_run(npk, x > from ? x : from, x + l, lo, hi);
                x += l;
            } else if (op == SS_CIG_D) {
                add_run(raw, x > from ? x : from, x + l, lo, hi);
                x += l;
            } else if (op == SS_CIG_N) {
                x += l;
            }
        }
    }
    /* prefix sums: counts, then each column's first output slot */
    uint32_t *off = S->off;
    int32_t cr = 0, cp = 0;
    uint32_t tot = 0;
    size_t ncol = 0;
    for (int64_t i = 0; i < len; ++i) {
        cr += raw[i];
        cp += npk[i];
        raw[i] = cr;
        off[i] = tot;
        tot += (uint32_t)cp;
        ncol += cr > 0;
    }
    if (ncol == 0) return 0;
    /* the chunk receives the window */
    if (!S->fill && !(S->fill = chunk_acquire(S))) return -1;
    chunk_t *c = S->fill;
    if (c->n + ncol > c->cap) {
        c->cap = 2 * (c->n + ncol) + 4096;
        c->hdr = (int32_t *)xalloc(c->hdr, sizeof(int32_t) * 4 * c->cap);
    }
    if (c->n_pk + tot > c->cap_pk) {
        c->cap_pk = 2 * (c->n_pk + tot) + 65536;
        c->pk = (uint32_t *)xalloc(c->pk, sizeof(uint32_t) * c->cap_pk);
    }
    /* the entries are scattered into a window buffer that stays in cache,
     * then appended to the chunk sequentially */
    if (tot > S->cap_w) {
        S->cap_w = 2 * tot;
        S->wbuf = (uint32_t *)xalloc(S->wbuf, sizeof(uint32_t) * S->cap_w);
    }
    uint32_t *out = S->wbuf;
    /* pass 2: scatter the packed entries, reads in load order */
    for (int i = 0; i < S->n_act; ++i) {
        const cread_t *r = S->act[i];
        const int64_t from = r->from > lo ? r->from : lo;
        const uint8_t *seq = bam_rec_seq(&r->b), *qual = bam_rec_qual(&r->b);
        if (r->single) {
            const int64_t a = from, b = r->end < hi ? r->end : hi;
            if (a < b) scatter_run(out, off + (a - lo), r->pk, seq, qual, (uint32_t)(a - r->beg), (uint32_t)(b - a));
            continue;
        }
        const uint32_t *cig = bam_rec_cigar(&r->b);
        int64_t x = r->beg, y = 0;
        for (int k = 0; k < r->b.n_cigar && x < hi; ++k) {
            const uint32_t op = cig[k] & 0xf, l = cig[k] >> 4;
            if (op == SS_CIG_M) {
                int64_t a = x > from ? x : from, b = x + l < hi ? x + l : hi;
                if (a < b) scatter_run(out, off + (a - lo), r->pk, seq, qual, (uint32_t)(y + (a - x)), (uint32_t)(b - a));
                x += l;
                y += l;
            } else if (op == SS_CIG_D || op == SS_CIG_N) {
                x += l;
            } else if (op == SS_CIG_I || op == SS_CIG_S) {
                y += l;
            }
        }
    }
    memcpy(c->pk + c->n_pk, out, sizeof(uint32_t) * tot);
    /* headers: off[] now holds each column's end slot */
    int32_t *h = c->hdr + 4 * c->n;
    uint32_t beg = 0;
    for (int64_t i = 0; i < len; ++i) {
        const uint32_t e = off[i];
        if (raw[i] > 0) {
            h[0] = tid;
            h[1] = (int32_t)(lo + i);
            h[2] = raw[i];
            h[3] = (int32_t)(e - beg);
            h += 4;
        }
        beg = e;
    }
    c->n += ncol;
    c->n_pk += tot;
    if (c->n >= CHUNK_MIN) chunk_publish(S);
    return 0;
}

/* Recycles the loaded reads with nothing left at or after position lo. */
static void purge(col_stream_t *S, int64_t lo)
{
    int k = 0;
    for (int i = 0; i < S->n_act; ++i) {
        cread_t *r = S->act[i];
        if (r->end <= lo || r->from >= r->end) {
            if (S->n_pool == S->m_pool) {
                S->m_pool = S->m_pool ? 2 * S->m_pool : 256;
                S->pool = (cread_t **)xalloc(S->pool, sizeof(cread_t *) * (size_t)S->m_pool);
            }
            S->pool[S->n_pool++] = r;
            continue;
        }
        if (r->from < lo) r->from = lo;
        S->act[k++] = r;
    }
    S->n_act = k;
}

/* Builds every column of contig tid before `upto` (INT64_MAX: the whole
 * contig; *lo is then left alone, the caller starts the next contig). */
static int build_until(col_stream_t *S, int32_t tid, int64_t *lo, int64_t upto)
{
    for (;;) {
        /* the first position any loaded read still covers, and the last */
        int64_t first = INT64_MAX, last = *lo;
        for (int i = 0; i < S->n_act; ++i) {
            const cread_t *r = S->act[i];
            const int64_t f = r->from > *lo ? r->from : *lo;
            if (f < r->end && f < first) first = f;
            if (r->end > last) last = r->end;
        }
        const int64_t stop = upto < last ? upto : last;
        if (first == INT64_MAX || first >= stop) {       /* nothing left before the frontier */
            if (upto != INT64_MAX && upto > *lo) *lo = upto;
            break;
        }
        const int64_t hi = stop - first > SEG_MAX ? first + SEG_MAX : stop;
        if (build_window(S, tid, first, hi)) return -1;
        *lo = hi;
        purge(S, hi);
        if (hi >= upto) break;
    }
    purge(S, *lo);
    return 0;
}

static cread_t *read_new(col_stream_t *S)
{
    if (S->n_pool) return S->pool[--S->n_pool];
    cread_t *r = (cread_t *)calloc(1, sizeof(cread_t));
    if (!r) { fprintf(stderr, "out of memory\n"); exit(1); }
    return r;
}

static void *producer_main(void *arg)
{
    col_stream_t *S = (col_stream_t *)arg;
    bam_record_t rec;
    memset(&rec, 0, sizeof rec);
    int32_t T = 0, max_tid = -1;     /* the walk's contig */
    int64_t W = 0;                   /* the walk's position at the next load */
    int64_t lo = 0;                  /* columns of T before lo are built */
    int rc;
    while ((rc = bam_record_read(S->fp, &rec)) > 0) {
        if ((rec.flag & S->flag_mask) || rec.mapq < S->mapq_thresh) continue;
        if (rec.tid < max_tid) {
            fprintf(stderr, "[bam_pileup_core] the input is not sorted. Abort!\n");
            abort();
        }
        max_tid = rec.tid;
        const int64_t beg = rec.pos, end = (int64_t)(int32_t)bam_rec_end(&rec);
        const int keep = end > W;
        int64_t from = beg > W ? beg : W;
        if (rec.tid != T) {              /* a later contig: the current one is complete */
            if (build_until(S, T, &lo, INT64_MAX)) goto out;
            T = rec.tid;
            from = beg;
            W = beg > 0 ? beg : 0;
            lo = 0;
        } else if (beg > W) {
            W = beg;
        }
        if (keep) {
            cread_t *r = read_new(S);
            bam_record_copy(&r->b, &rec);
            r->beg = beg;
            r->end = end;
            r->from = from;
            r->pk = (uint32_t)rec.mapq | ((rec.flag & SS_BAM_FREVERSE) ? 1u << 20 : 0u);
            r->single = rec.n_cigar == 1 && (bam_rec_cigar(&rec)[0] & 0xf) == SS_CIG_M;
            if (S->n_act == S->m_act) {
                S->m_act = S->m_act ? 2 * S->m_act : 1024;
                S->act = (cread_t **)xalloc(S->act, sizeof(cread_t *) * (size_t)S->m_act);
            }
            S->act[S->n_act++] = r;
        }
        if (W - lo >= SEG_MIN && build_until(S, T, &lo, W)) goto out;
    }
    if (rc < 0) S->error = 1;
    if (build_until(S, T, &lo, INT64_MAX)) goto out;
    if (!S->fill && !(S->fill = chunk_acquire(S))) goto out;
    S->fill->last = 1;
    chunk_publish(S);
out:
    bam_record_free(&rec);
    return NULL;
}

col_stream_t *col_stream_start(bgzf_reader_t *fp, int mask, int thresh)
{
    col_stream_t *S = (col_stream_t *)calloc(1, sizeof *S);
    if (!S) return NULL;
    S->fp = fp;
    S->flag_mask = mask < 0 ? SS_BAM_DEF_MASK : (SS_BAM_FUNMAP | (uint32_t)mask);
    S->mapq_thresh = thresh < 0 ? 0 : thresh;
    S->raw = (int32_t *)xalloc(NULL, sizeof(int32_t) * (SEG_MAX + 1));
    S->npk = (int32_t *)xalloc(NULL, sizeof(int32_t) * (SEG_MAX + 1));
    S->off = (uint32_t *)xalloc(NULL, sizeof(uint32_t) * (SEG_MAX + 1));
    pthread_mutex_init(&S->mu, NULL);
    pthread_cond_init(&S->cv, NULL);
    pthread_create(&S->th, NULL, producer_main, S);
    return S;
}

int col_stream_next(col_stream_t *S, int32_t *tid, int32_t *pos, int *r, const uint32_t **pk, int *np)
{
    for (;;) {
        if (S->ended) return 0;
        if (S->cur && S->step < S->cur->n) break;
        if (S->cur && S->cur->last) { S->ended = 1; return 0; }
        pthread_mutex_lock(&S->mu);
        if (S->cur) { ++S->consumed; pthread_cond_broadcast(&S->cv); }
        while (S->produced == S->consumed) pthread_cond_wait(&S->cv, &S->mu);
        S->cur = &S->chunks[S->consumed % N_CHUNKS];
        pthread_mutex_unlock(&S->mu);
        S->step = 0;
        S->pk_off = 0;
    }
    const int32_t *h = S->cur->hdr + 4 * S->step++;
    *tid = h[0];
    *pos = h[1];
    *r = h[2];
    *np = h[3];
    *pk = S->cur->pk + S->pk_off;
    S->pk_off += (size_t)h[3];
    return 1;
}

int col_stream_stop(col_stream_t *S)
{
    pthread_mutex_lock(&S->mu);
    S->stop = 1;
    S->consumed = S->produced;          /* release every chunk: the producer may be waiting */
    pthread_cond_broadcast(&S->cv);
    pthread_mutex_unlock(&S->mu);
    pthread_join(S->th, NULL);
    const int err = S->error;
    for (int c = 0; c < N_CHUNKS; ++c) { free(S->chunks[c].hdr); free(S->chunks[c].pk); }
    for (int i = 0; i < S->n_act; ++i) { bam_record_free(&S->act[i]->b); free(S->act[i]); }
    for (int i = 0; i < S->n_pool; ++i) { bam_record_free(&S->pool[i]->b); free(S->pool[i]); }
    free(S->act);
    free(S->pool);
    free(S->raw);
    free(S->npk);
    free(S->off);
    free(S->wbuf);
    pthread_mutex_destroy(&S->mu);
    pthread_cond_destroy(&S->cv);
    free(S);
    return err ? -1 : 0;
}
