/* column_pileup.c -- see column_pileup.h for the rules being reproduced.
 *
 * Per sample:
 *   - a reader thread reads records, applies the keep / coverage rules and
 *     keeps the loaded reads in load order.  Whenever the finalisation
 *     frontier W has moved far enough it cuts the positions behind it into
 *     windows of at most SEG_MAX positions and queues one job per window: the
 *     window and the loaded reads that reach into it;
 *   - worker threads build the jobs' columns, any job on any worker: pass 1
 *     adds each read's runs to difference arrays (raw and packed entry
 *     counts per column), a prefix sum gives every column its output slots,
 *     pass 2 scatters the packed entries, reads in load order, so the entries
 *     of a column keep the reference's pileup order;
 *   - the consumer (col_stream_next) drains the jobs in window order.
 * A read is recycled once the last job that references it has been drained.
 * Jobs live in a ring of N_JOBS slots; the reader waits for a free slot. */
#include "column_pileup.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bam_reader.h"

#define SEG_MIN    1024       /* frontier advance that cuts windows */
#define SEG_MAX    2048       /* positions per window */
#define N_JOBS     64
#define MAX_WORKERS 16

typedef struct {
    int64_t beg, end;         /* reference span (bam_calend) */
    int64_t from;             /* first position this read contributes to */
    uint64_t last_job;        /* the last job that references it (set when retired) */
    uint32_t pk;              /* mapQ | strand << 20 */
    int single;               /* one M operation covering [beg, end) */
    bam_record_t b;
} cread_t;

enum { JOB_FREE, JOB_READY, JOB_BUSY, JOB_DONE };

typedef struct {
    int state;
    int last;                 /* end-of-stream marker: no columns */
    uint64_t seq;
    int32_t tid;
    int64_t lo, hi;
    cread_t **reads;          /* loaded reads that reach into [lo, hi), load order */
    int n_reads, m_reads;
    int32_t *hdr;             /* tid, pos, r, np per column */
    uint32_t *pk;
    size_t n, cap, cap_pk;
} job_t;

typedef struct {
    int32_t *raw, *npk;       /* difference arrays / counts, SEG_MAX + 1 */
    uint32_t *off;
} scratch_t;

struct col_stream {
    bgzf_reader_t *fp;
    col_seed_t seed;
    uint32_t flag_mask;
    int mapq_thresh;
    int error;
    /* reader state */
    cread_t **act;            /* loaded reads, load order */
    int n_act, m_act;
    cread_t **retired;        /* FIFO of reads whose last job is queued, by last_job */
    size_t ret_head, ret_tail, m_ret;
    cread_t **pool;           /* recycled reads (their buffers are reused) */
    int n_pool, m_pool;
    /* job ring */
    job_t jobs[N_JOBS];
    uint64_t queued, next_build, drained;
    int stop, n_workers;
    pthread_mutex_t mu;
    pthread_cond_t cv_reader, cv_work, cv_done;
    pthread_t reader, workers[MAX_WORKERS];
    scratch_t scr[MAX_WORKERS];
    /* consumer cursor */
    job_t *cur;
    size_t step, pk_off;
    int ended;
};

static void *xalloc(void *p, size_t n)
{
    void *q = realloc(p, n ? n : 1);
    if (!q) { fprintf(stderr, "out of memory\n"); exit(1); }
    return q;
}

/* ---- window build (workers) ------------------------------------------------ */
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

static void build_job(job_t *J, scratch_t *sc)
{
    const int64_t lo = J->lo, hi = J->hi, len = hi - lo;
    int32_t *raw = sc->raw, *npk = sc->npk;
    uint32_t *off = sc->off;
    memset(raw, 0, sizeof(int32_t) * (size_t)(len + 1));
    memset(npk, 0, sizeof(int32_t) * (size_t)(len + 1));
    /* pass 1: entry counts per column */
    for (int i = 0; i < J->n_reads; ++i) {
        const cread_t *r = J->reads[i];
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
    J->n = ncol;
    if (ncol == 0) return;
    if (ncol > J->cap) {
        J->cap = ncol + 256;
        J->hdr = (int32_t *)xalloc(J->hdr, sizeof(int32_t) * 4 * J->cap);
    }
    if (tot > J->cap_pk) {
        J->cap_pk = tot + tot / 4 + 4096;
        J->pk = (uint32_t *)xalloc(J->pk, sizeof(uint32_t) * J->cap_pk);
    }
    uint32_t *out = J->pk;
    /* pass 2: scatter the packed entries, reads in load order */
    for (int i = 0; i < J->n_reads; ++i) {
        const cread_t *r = J->reads[i];
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
    /* headers: off[] now holds each column's end slot */
    int32_t *h = J->hdr;
    uint32_t beg = 0;
    for (int64_t i = 0; i < len; ++i) {
        const uint32_t e = off[i];
        if (raw[i] > 0) {
            h[0] = J->tid;
            h[1] = (int32_t)(lo + i);
            h[2] = raw[i];
            h[3] = (int32_t)(e - beg);
            h += 4;
        }
        beg = e;
    }
}

typedef struct {
    col_stream_t *S;
    int id;
} worker_arg_t;

static void *worker_main(void *arg)
{
    worker_arg_t *w = (worker_arg_t *)arg;
    col_stream_t *S = w->S;
    scratch_t *sc = &S->scr[w->id];
    free(w);
    pthread_mutex_lock(&S->mu);
    for (;;) {
        while (!S->stop && !(S->next_build < S->queued && S->jobs[S->next_build % N_JOBS].state == JOB_READY))
            pthread_cond_wait(&S->cv_work, &S->mu);
        if (S->stop) break;
        job_t *J = &S->jobs[S->next_build % N_JOBS];
        ++S->next_build;
        J->state = JOB_BUSY;
        pthread_mutex_unlock(&S->mu);
        if (!J->last) build_job(J, sc);
        pthread_mutex_lock(&S->mu);
        J->state = JOB_DONE;
        pthread_cond_broadcast(&S->cv_done);
    }
    pthread_mutex_unlock(&S->mu);
    return NULL;
}

/* ---- reader -------------------------------------------------------------------- */
static cread_t *read_new(col_stream_t *S)
{
    if (S->n_pool) return S->pool[--S->n_pool];
    cread_t *r = (cread_t *)calloc(1, sizeof(cread_t));
    if (!r) { fprintf(stderr, "out of memory\n"); exit(1); }
    return r;
}

/* Recycles the retired reads whose last job has been drained (reader thread,
 * mu held for `drained`). */
static void recycle(col_stream_t *S)
{
    while (S->ret_head < S->ret_tail) {
        cread_t *r = S->retired[S->ret_head % S->m_ret];
        if (r->last_job >= S->drained) break;
        ++S->ret_head;
        if (S->n_pool == S->m_pool) {
            S->m_pool = S->m_pool ? 2 * S->m_pool : 1024;
            S->pool = (cread_t **)xalloc(S->pool, sizeof(cread_t *) * (size_t)S->m_pool);
        }
        S->pool[S->n_pool++] = r;
    }
}

/* Appends r to the retired FIFO.  The FIFO and the pool belong to the reader
 * thread (recycle() runs there too), so no lock; last_job never decreases. */
static void retire(col_stream_t *S, cread_t *r, uint64_t last_job)
{
    r->last_job = last_job;
    if (S->ret_tail - S->ret_head == S->m_ret) {           /* grow the ring, keeping FIFO order */
        const size_t m = S->m_ret ? 2 * S->m_ret : 4096;
        cread_t **q = (cread_t **)xalloc(NULL, sizeof(cread_t *) * m);
        for (size_t i = S->ret_head; i < S->ret_tail; ++i) q[i - S->ret_head] = S->retired[i % S->m_ret];
        S->ret_tail -= S->ret_head;
        S->ret_head = 0;
        free(S->retired);
        S->retired = q;
        S->m_ret = m;
    }
    S->retired[S->ret_tail++ % S->m_ret] = r;
}

/* Takes the next job slot (waits for the consumer to drain one), or NULL once
 * the stream is stopped. */
static job_t *job_acquire(col_stream_t *S)
{
    pthread_mutex_lock(&S->mu);
    while (!S->stop && S->queued - S->drained >= N_JOBS) pthread_cond_wait(&S->cv_reader, &S->mu);
    recycle(S);
    job_t *J = S->stop ? NULL : &S->jobs[S->queued % N_JOBS];
    const uint64_t seq = S->queued;
    pthread_mutex_unlock(&S->mu);
    if (J) { J->n = 0; J->n_reads = 0; J->last = 0; J->seq = seq; }
    return J;
}

static void job_queue(col_stream_t *S, job_t *J)
{
    pthread_mutex_lock(&S->mu);
    J->state = JOB_READY;
    ++S->queued;
    pthread_cond_broadcast(&S->cv_work);
    pthread_mutex_unlock(&S->mu);
}

/* Queues the windows of contig tid before `upto` (INT64_MAX: the whole
 * contig); reads with nothing after a window are retired with it.  Returns
 * -1 once the stream is stopped. */
static int queue_until(col_stream_t *S, int32_t tid, int64_t *lo, int64_t upto)
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
        job_t *J = job_acquire(S);
        if (!J) return -1;
        J->tid = tid;
        J->lo = first;
        J->hi = hi;
        if (S->n_act > J->m_reads) {
            J->m_reads = S->n_act + 1024;
            J->reads = (cread_t **)xalloc(J->reads, sizeof(cread_t *) * (size_t)J->m_reads);
        }
        int k = 0;
        for (int i = 0; i < S->n_act; ++i) {
            cread_t *r = S->act[i];
            const int64_t f = r->from > first ? r->from : first;
            if (f < r->end && f < hi) J->reads[J->n_reads++] = r;
            if (r->end <= hi || r->from >= r->end) retire(S, r, J->seq);
            else S->act[k++] = r;
        }
        S->n_act = k;
        *lo = hi;
        job_queue(S, J);
        if (hi >= upto) break;
    }
    /* reads with nothing left at or after lo (no reference span, or passed) */
    int k = 0;
    for (int i = 0; i < S->n_act; ++i) {
        cread_t *r = S->act[i];
        if (r->end <= *lo || r->from >= r->end) retire(S, r, S->queued);
        else S->act[k++] = r;
    }
    S->n_act = k;
    return 0;
}

static void *reader_main(void *arg)
{
    col_stream_t *S = (col_stream_t *)arg;
    bam_record_t rec;
    memset(&rec, 0, sizeof rec);
    int32_t T = 0, max_tid = -1;     /* the walk's contig */
    int64_t W = 0;                   /* the walk's position at the next load */
    int64_t lo = 0;                  /* windows of T before lo are queued */
    if (S->seed.has_prev) {          /* the state right after the last record loaded before the range */
        T = max_tid = S->seed.prev_tid;
        W = S->seed.prev_pos > 0 ? S->seed.prev_pos : 0;
    }
    int rc;
    while ((rc = bam_record_read(S->fp, &rec)) > 0) {
        if (rec.tid >= S->seed.stop_tid) break;            /* the next range's first record */
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
            if (queue_until(S, T, &lo, INT64_MAX)) goto out;
            T = rec.tid;
            from = beg;
            W = beg > 0 ? beg : 0;
            lo = 0;
        } else if (beg > W) {
            W = beg;
        }
        if (keep) {
            if (!S->n_pool) {                           /* take back drained reads first */
                pthread_mutex_lock(&S->mu);
                recycle(S);
                pthread_mutex_unlock(&S->mu);
            }
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
        if (W - lo >= SEG_MIN && queue_until(S, T, &lo, W)) goto out;
    }
    if (rc < 0) S->error = 1;
    if (queue_until(S, T, &lo, INT64_MAX)) goto out;
    job_t *J = job_acquire(S);
    if (J) {
        J->last = 1;
        job_queue(S, J);
    }
out:
    bam_record_free(&rec);
    return NULL;
}

col_stream_t *col_stream_start(bgzf_reader_t *fp, int mask, int thresh, int n_workers)
{
    const col_seed_t whole = {0, 0, 0, INT32_MAX};
    return col_stream_start_at(fp, mask, thresh, n_workers, &whole);
}

col_stream_t *col_stream_start_at(bgzf_reader_t *fp, int mask, int thresh, int n_workers, const col_seed_t *seed)
{
    col_stream_t *S = (col_stream_t *)calloc(1, sizeof *S);
    if (!S) return NULL;
    S->fp = fp;
    S->seed = *seed;
    S->flag_mask = mask < 0 ? SS_BAM_DEF_MASK : (SS_BAM_FUNMAP | (uint32_t)mask);
    S->mapq_thresh = thresh < 0 ? 0 : thresh;
    S->n_workers = n_workers < 1 ? 1 : (n_workers > MAX_WORKERS ? MAX_WORKERS : n_workers);
    pthread_mutex_init(&S->mu, NULL);
    pthread_cond_init(&S->cv_reader, NULL);
    pthread_cond_init(&S->cv_work, NULL);
    pthread_cond_init(&S->cv_done, NULL);
    for (int w = 0; w < S->n_workers; ++w) {
        S->scr[w].raw = (int32_t *)xalloc(NULL, sizeof(int32_t) * (SEG_MAX + 1));
        S->scr[w].npk = (int32_t *)xalloc(NULL, sizeof(int32_t) * (SEG_MAX + 1));
        S->scr[w].off = (uint32_t *)xalloc(NULL, sizeof(uint32_t) * (SEG_MAX + 1));
        worker_arg_t *a = (worker_arg_t *)xalloc(NULL, sizeof *a);
        a->S = S;
        a->id = w;
        pthread_create(&S->workers[w], NULL, worker_main, a);
    }
    pthread_create(&S->reader, NULL, reader_main, S);
    return S;
}

int col_stream_next(col_stream_t *S, int32_t *tid, int32_t *pos, int *r, const uint32_t **pk, int *np)
{
    for (;;) {
        if (S->ended) return 0;
        if (S->cur && S->step < S->cur->n) break;
        pthread_mutex_lock(&S->mu);
        if (S->cur) {                                   /* drained: the slot goes back to the reader */
            S->cur->state = JOB_FREE;
            ++S->drained;
            pthread_cond_broadcast(&S->cv_reader);
        }
        job_t *J = &S->jobs[S->drained % N_JOBS];
        while (!(S->drained < S->queued && J->state == JOB_DONE)) pthread_cond_wait(&S->cv_done, &S->mu);
        pthread_mutex_unlock(&S->mu);
        S->cur = J;
        S->step = 0;
        S->pk_off = 0;
        if (J->last) { S->ended = 1; return 0; }
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
    pthread_cond_broadcast(&S->cv_reader);
    pthread_cond_broadcast(&S->cv_work);
    pthread_mutex_unlock(&S->mu);
    pthread_join(S->reader, NULL);
    for (int w = 0; w < S->n_workers; ++w) pthread_join(S->workers[w], NULL);
    const int err = S->error;
    for (int j = 0; j < N_JOBS; ++j) { free(S->jobs[j].reads); free(S->jobs[j].hdr); free(S->jobs[j].pk); }
    for (int w = 0; w < S->n_workers; ++w) { free(S->scr[w].raw); free(S->scr[w].npk); free(S->scr[w].off); }
    for (int i = 0; i < S->n_act; ++i) { bam_record_free(&S->act[i]->b); free(S->act[i]); }
    for (size_t i = S->ret_head; i < S->ret_tail; ++i) {
        cread_t *r = S->retired[i % S->m_ret];
        bam_record_free(&r->b);
        free(r);
    }
    for (int i = 0; i < S->n_pool; ++i) { bam_record_free(&S->pool[i]->b); free(S->pool[i]); }
    free(S->act);
    free(S->retired);
    free(S->pool);
    pthread_mutex_destroy(&S->mu);
    pthread_cond_destroy(&S->cv_reader);
    pthread_cond_destroy(&S->cv_work);
    pthread_cond_destroy(&S->cv_done);
    free(S);
    return err ? -1 : 0;
}
