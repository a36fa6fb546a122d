/* dual_pileup.c -- see dual_pileup.h for the behaviour being reproduced. */
#include "dual_pileup.h"

#include "column_pileup.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct pl_node {
    /* hot fields first: read on every visited position */
    int32_t tid;
    uint32_t beg, end;
    uint32_t pk;                  /* mapQ | strand << 20 of the record */
    const uint8_t *seq, *qual;
    uint32_t span;                /* length of the single M operation, or 0 */
    struct pl_node *next;         /* free-list link */
    bam_record_t b;
} pl_node_t;

#define SLAB 512

typedef struct {
    /* Loaded reads in load order (the reference's linked list, kept here as
     * an array that is compacted in order).  `tail` is the spare node that
     * receives the next record: with no loaded reads the reference's list
     * head IS that spare node, whose record is then the last one copied into
     * it -- or, for a node recycled from the pool, whatever it held before
     * (the pool is LIFO like samtools' mempool, so this is reproduced). */
    pl_node_t **act;
    int n_act, m_act;
    pl_node_t *tail;
    pl_node_t *free_list;
    int32_t tid, pos, max_tid, max_pos;
    int is_eof;
    uint32_t flag_mask;
    int mapq_thresh;
    pl_entry_t *pu;
    int max_pu;
    bgzf_reader_t *fp;
    bam_record_t rec;          /* read buffer */
    int error;
    pl_node_t **slabs;
    int n_slabs, slab_used;
} walker_t;

static pl_node_t *node_new(walker_t *w)
{
    pl_node_t *p = w->free_list;
    if (p) {
        w->free_list = p->next;
        p->next = NULL;
        return p;
    }
    if (w->slab_used == SLAB || !w->slabs) {     /* fresh nodes come from contiguous slabs */
        pl_node_t **sl = (pl_node_t **)realloc(w->slabs, sizeof(pl_node_t *) * (size_t)(w->n_slabs + 1));
        pl_node_t *blk = (pl_node_t *)calloc(SLAB, sizeof(pl_node_t));
        if (!sl || !blk) { fprintf(stderr, "out of memory\n"); exit(1); }
        w->slabs = sl;
        w->slabs[w->n_slabs++] = blk;
        w->slab_used = 0;
    }
    return &w->slabs[w->n_slabs - 1][w->slab_used++];
}

static void node_free(walker_t *w, pl_node_t *p)
{
    p->next = w->free_list;
    w->free_list = p;
}

/* Position `pos` within read b: query offset and deletion flag, or 0 when
 * the read does not contribute there (reference skip; resolve_cigar :59-111). */
static int locate(const bam_record_t *b, uint32_t pos, int32_t *qpos, uint8_t *is_del)
{
    const uint32_t *cig = bam_rec_cigar(b);
    if (b->n_cigar == 1 && (cig[0] & 0xf) == SS_CIG_M && pos - (uint32_t)b->pos < (cig[0] >> 4)) {
        *qpos = (int32_t)(pos - (uint32_t)b->pos);        /* a plain match: the common case */
        *is_del = 0;
        return 1;
    }
    uint32_t x = (uint32_t)b->pos, y = 0;
    int keep = 1;
    *qpos = -1;
    *is_del = 0;
    for (int k = 0; k < b->n_cigar; ++k) {
        const uint32_t op = cig[k] & 0xf, l = cig[k] >> 4;
        if (op == SS_CIG_M) {
            if (x + l > pos) { *is_del = 0; *qpos = (int32_t)(y + (pos - x)); }
            x += l;
            y += l;
        } else if (op == SS_CIG_D) {
            if (x + l > pos) { *is_del = 1; *qpos = (int32_t)(y + (pos - x)); }
            x += l;
        } else if (op == SS_CIG_N) {
            x += l;
        } else if (op == SS_CIG_I || op == SS_CIG_S) {
            y += l;
        }
        if (x > pos) {
            if (op == SS_CIG_N) keep = 0;
            break;
        }
    }
    if (x <= pos) {
        fprintf(stderr, "[bam_pileup] read %.*s does not cover position %u (CIGAR operations the "
                        "pileup does not model). Abort!\n", (int)b->l_qname, (const char *)b->data, pos);
        abort();
    }
    return keep;
}

static void walker_init(walker_t *w, bgzf_reader_t *fp, int mask, int thresh)
{
    memset(w, 0, sizeof *w);
    w->fp = fp;
    w->tail = node_new(w);
    (void)node_new(w);        /* the reference's dummy node: keeps pool allocation in step */
    w->max_tid = w->max_pos = -1;
    w->flag_mask = mask < 0 ? SS_BAM_DEF_MASK : (SS_BAM_FUNMAP | (uint32_t)mask);
    w->mapq_thresh = thresh < 0 ? 0 : thresh;
}

static void walker_free(walker_t *w)
{
    for (int i = 0; i < w->n_slabs; ++i) {
        const int n = i == w->n_slabs - 1 ? w->slab_used : SLAB;
        for (int k = 0; k < n; ++k) bam_record_free(&w->slabs[i][k].b);
        free(w->slabs[i]);
    }
    free(w->slabs);
    free(w->act);
    bam_record_free(&w->rec);
    free(w->pu);
}

/* One step of the walk (get_next_pos): advance to the next position and
 * return its number of pileup entries (>= 0), or -1 when the file is done. */
static int next_pos(walker_t *w)
{
    if (w->max_pos != -1) {
        const pl_node_t *head = w->n_act ? w->act[0] : w->tail;
        if (w->tid < head->tid) { w->tid = head->tid; w->pos = 0; }
        else ++w->pos;
    }
    if (w->is_eof && w->n_act == 0) return -1;
    for (;;) {
        if (w->is_eof || w->max_tid > w->tid || (w->max_tid == w->tid && w->max_pos > w->pos)) {
            if (w->n_act > w->max_pu) {
                w->max_pu = w->n_act + 256;
                w->pu = (pl_entry_t *)realloc(w->pu, sizeof(pl_entry_t) * (size_t)w->max_pu);
                if (!w->pu) { fprintf(stderr, "out of memory\n"); exit(1); }
            }
            const int32_t tid = w->tid;
            const uint32_t pos = (uint32_t)w->pos;
            int n = 0, k = 0;
            for (int i = 0; i < w->n_act; ++i) {
                pl_node_t *p = w->act[i];
                if (p->tid < tid || (p->tid == tid && p->end <= pos)) {   /* passed: back to the pool */
                    node_free(w, p);
                    continue;
                }
                w->act[k++] = p;
                if (p->tid != tid || p->beg > pos) continue;
                pl_entry_t *e = &w->pu[n];
                e->b = &p->b;
                const uint32_t off = pos - p->beg;
                if (off < p->span) {                    /* a plain match: the common case */
                    e->qpos = (int32_t)off;
                    e->is_del = 0;
                } else if (!locate(&p->b, pos, &e->qpos, &e->is_del)) {
                    continue;                           /* inside a reference skip */
                }
                if (!e->is_del) {
                    const int q = e->qpos;
                    e->packed = p->pk | (uint32_t)p->qual[q] << 8 |
                                (uint32_t)((p->seq[q >> 1] >> ((~q & 1) << 2)) & 0xf) << 16;
                }
                ++n;
            }
            w->n_act = k;
            return n;
        }
        const int rc = bam_record_read(w->fp, &w->rec);
        if (rc > 0) {
            if (!(w->rec.flag & w->flag_mask) && !(w->rec.mapq < w->mapq_thresh)) {
                pl_node_t *t = w->tail;
                bam_record_copy(&t->b, &w->rec);
                t->tid = w->rec.tid;
                t->beg = (uint32_t)w->rec.pos;
                t->end = bam_rec_end(&w->rec);
                t->pk = (uint32_t)w->rec.mapq | ((w->rec.flag & SS_BAM_FREVERSE) ? 1u << 20 : 0u);
                t->seq = bam_rec_seq(&t->b);
                t->qual = bam_rec_qual(&t->b);
                t->span = (t->b.n_cigar == 1 && (bam_rec_cigar(&t->b)[0] & 0xf) == SS_CIG_M)
                              ? bam_rec_cigar(&t->b)[0] >> 4 : 0u;
                if (w->rec.tid < w->max_tid) {
                    fprintf(stderr, "[bam_pileup_core] the input is not sorted. Abort!\n");
                    abort();
                }
                w->max_tid = w->rec.tid;
                w->max_pos = (int32_t)t->beg;
                if (t->end > (uint32_t)w->pos) {            /* kept: it joins the loaded reads */
                    if (w->n_act == w->m_act) {
                        w->m_act = w->m_act ? 2 * w->m_act : 256;
                        w->act = (pl_node_t **)realloc(w->act, sizeof(pl_node_t *) * (size_t)w->m_act);
                        if (!w->act) { fprintf(stderr, "out of memory\n"); exit(1); }
                    }
                    w->act[w->n_act++] = t;
                    w->tail = node_new(w);
                }
            }
        } else {
            if (rc < 0) w->error = 1;
            w->is_eof = 1;
        }
    }
}

/* packed non-deleted reads of the current position's entries */
static int packed_of(const walker_t *w, int n, uint32_t *dst)
{
    int k = 0;
    for (int i = 0; i < n; ++i)
        if (!w->pu[i].is_del) dst[k++] = w->pu[i].packed;
    return k;
}

/* ---- threaded mode: each walk produces a stream of steps -------------------
 * One step per next_pos call: {tid, pos, r, np} + np packed reads.  Steps go
 * to the consumer in chunks through a small ring (single producer, single
 * consumer).  A walk runs ahead of the lockstep loop by at most the ring. */
#define CHUNK_STEPS 4096
#define N_CHUNKS 8

typedef struct {
    int32_t *hdr;            /* 4 ints per step */
    uint32_t *pk;
    size_t n_steps, n_pk, cap_pk;
} chunk_t;

typedef struct {
    walker_t *w;
    chunk_t chunks[N_CHUNKS];
    uint64_t produced, consumed;     /* chunk counters */
    int stop;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    pthread_t th;
    /* consumer cursor */
    chunk_t *cur;
    size_t step, pk_off;
    int ended;                       /* the walk returned -1: it keeps returning -1 */
} stream_t;

static void *walk_main(void *arg)
{
    stream_t *S = (stream_t *)arg;
    walker_t *w = S->w;
    uint32_t *tmp = NULL;
    int m_tmp = 0;
    for (int done = 0; !done;) {
        pthread_mutex_lock(&S->mu);
        while (!S->stop && S->produced - S->consumed >= N_CHUNKS) pthread_cond_wait(&S->cv, &S->mu);
        const int stop = S->stop;
        pthread_mutex_unlock(&S->mu);
        if (stop) break;
        chunk_t *c = &S->chunks[S->produced % N_CHUNKS];
        c->n_steps = c->n_pk = 0;
        while (c->n_steps < CHUNK_STEPS) {
            const int r = next_pos(w);
            int np = 0;
            if (r > 0) {
                if (r > m_tmp) { m_tmp = r + 256; tmp = (uint32_t *)realloc(tmp, 4 * (size_t)m_tmp); }
                np = packed_of(w, r, tmp);
                if (c->n_pk + (size_t)np > c->cap_pk) {
                    c->cap_pk = 2 * (c->n_pk + (size_t)np) + 4096;
                    c->pk = (uint32_t *)realloc(c->pk, 4 * c->cap_pk);
                    if (!c->pk) { fprintf(stderr, "out of memory\n"); exit(1); }
                }
                memcpy(c->pk + c->n_pk, tmp, 4 * (size_t)np);
                c->n_pk += (size_t)np;
            }
            int32_t *h = c->hdr + 4 * c->n_steps++;
            h[0] = w->tid; h[1] = w->pos; h[2] = r; h[3] = np;
            if (r < 0) { done = 1; break; }
        }
        pthread_mutex_lock(&S->mu);
        ++S->produced;
        pthread_cond_broadcast(&S->cv);
        pthread_mutex_unlock(&S->mu);
    }
    free(tmp);
    return NULL;
}

/* next step of a stream: returns r and sets tid/pos/packed view */
static int stream_next(stream_t *S, int32_t *tid, int32_t *pos, const uint32_t **pk, int *np)
{
    if (S->ended) { *np = 0; return -1; }    /* next_pos after the end returns -1 again */
    if (!S->cur || S->step == S->cur->n_steps) {
        pthread_mutex_lock(&S->mu);
        if (S->cur) { ++S->consumed; pthread_cond_broadcast(&S->cv); }
        while (S->produced == S->consumed) pthread_cond_wait(&S->cv, &S->mu);
        S->cur = &S->chunks[S->consumed % N_CHUNKS];
        pthread_mutex_unlock(&S->mu);
        S->step = 0;
        S->pk_off = 0;
    }
    const int32_t *h = S->cur->hdr + 4 * S->step++;
    *tid = h[0]; *pos = h[1]; *np = h[3];
    *pk = S->cur->pk + S->pk_off;
    S->pk_off += (size_t)h[3];
    if (h[2] < 0) S->ended = 1;
    return h[2];
}

/* Column mode: both samples' reported columns (column_pileup.h), merged in
 * (tid, pos) order.  The lockstep loop of the walk reports exactly the
 * positions both walks report with entries: a walk that moves to a later
 * contig has no entries left on the earlier one, so the positions it skips
 * the other walk through are never shared. */
static int column_run(bgzf_reader_t *fp1, bgzf_reader_t *fp2, int mask, int thresh, const col_seed_t *s1,
                      const col_seed_t *s2, dual_site_fn fn, void *data)
{
    const char *ew = getenv("SS_PILEUP_WORKERS");
    const int nw = ew && *ew ? atoi(ew) : 3;                 /* window builders per sample */
    col_stream_t *a = col_stream_start_at(fp1, mask, thresh, nw, s1);
    col_stream_t *b = col_stream_start_at(fp2, mask, thresh, nw, s2);
    if (!a || !b) { fprintf(stderr, "out of memory\n"); exit(1); }
    int32_t t1, p1, t2, p2;
    int r1, r2, np1, np2;
    const uint32_t *pk1, *pk2;
    int v1 = col_stream_next(a, &t1, &p1, &r1, &pk1, &np1);
    int v2 = col_stream_next(b, &t2, &p2, &r2, &pk2, &np2);
    while (v1 && v2) {
        if (t1 < t2 || (t1 == t2 && p1 < p2)) {
            v1 = col_stream_next(a, &t1, &p1, &r1, &pk1, &np1);
        } else if (t2 < t1 || p2 < p1) {
            v2 = col_stream_next(b, &t2, &p2, &r2, &pk2, &np2);
        } else {
            if (fn(t1, p1, r1, r2, pk1, np1, pk2, np2, data)) break;
            v1 = col_stream_next(a, &t1, &p1, &r1, &pk1, &np1);
            v2 = col_stream_next(b, &t2, &p2, &r2, &pk2, &np2);
        }
    }
    const int e1 = col_stream_stop(a), e2 = col_stream_stop(b);
    if (e1 || e2) {
        fprintf(stderr, "[dual_pileup] truncated or malformed BAM record\n");
        return -1;
    }
    return 0;
}

int dual_pileup_run(bgzf_reader_t *fp1, bgzf_reader_t *fp2, int mask, int thresh, int threaded,
                    dual_site_fn fn, void *data)
{
    if (threaded == 2) {
        const col_seed_t whole = {0, 0, 0, INT32_MAX};
        return column_run(fp1, fp2, mask, thresh, &whole, &whole, fn, data);
    }
    walker_t *w1 = (walker_t *)malloc(sizeof(walker_t)), *w2 = (walker_t *)malloc(sizeof(walker_t));
    if (!w1 || !w2) { free(w1); free(w2); return -1; }
    walker_init(w1, fp1, mask, thresh);
    walker_init(w2, fp2, mask, thresh);
    int r1 = -1, r2 = -1, stop = 0;
    if (!threaded) {
        uint32_t *pk1 = NULL, *pk2 = NULL;
        int m1 = 0, m2 = 0;
        while (!stop && (r1 = next_pos(w1)) >= 0 && (r2 = next_pos(w2)) >= 0) {
            do {
                if (w2->tid > w1->tid)
                    while (w2->tid > w1->tid && (r1 = next_pos(w1)) >= 0) {}
                if (w1->tid > w2->tid)
                    while (w2->tid < w1->tid && (r2 = next_pos(w2)) >= 0) {}
            } while (w2->tid != w1->tid && r1 >= 0 && r2 >= 0);
            if (r1 > 0 && r2 > 0) {
                if (w1->tid != w2->tid || w1->pos != w2->pos) {
                    fprintf(stderr, "[dual_pileup] tumor and normal walks out of step. Abort!\n");
                    abort();
                }
                if (r1 > m1) { m1 = r1 + 256; pk1 = (uint32_t *)realloc(pk1, 4 * (size_t)m1); }
                if (r2 > m2) { m2 = r2 + 256; pk2 = (uint32_t *)realloc(pk2, 4 * (size_t)m2); }
                const int np1 = packed_of(w1, r1, pk1), np2 = packed_of(w2, r2, pk2);
                stop = fn(w1->tid, w1->pos, r1, r2, pk1, np1, pk2, np2, data);
            }
        }
        free(pk1);
        free(pk2);
    } else {
        stream_t *S = (stream_t *)calloc(2, sizeof(stream_t));
        if (!S) return -1;
        for (int k = 0; k < 2; ++k) {
            S[k].w = k ? w2 : w1;
            for (int c = 0; c < N_CHUNKS; ++c) {
                S[k].chunks[c].hdr = (int32_t *)malloc(sizeof(int32_t) * 4 * CHUNK_STEPS);
                if (!S[k].chunks[c].hdr) { fprintf(stderr, "out of memory\n"); exit(1); }
            }
            pthread_mutex_init(&S[k].mu, NULL);
            pthread_cond_init(&S[k].cv, NULL);
            pthread_create(&S[k].th, NULL, walk_main, &S[k]);
        }
        int32_t t1 = 0, p1 = 0, t2 = 0, p2 = 0;
        const uint32_t *pk1 = NULL, *pk2 = NULL;
        int np1 = 0, np2 = 0;
        while (!stop && (r1 = stream_next(&S[0], &t1, &p1, &pk1, &np1)) >= 0 &&
               (r2 = stream_next(&S[1], &t2, &p2, &pk2, &np2)) >= 0) {
            do {
                if (t2 > t1)
                    while (t2 > t1 && (r1 = stream_next(&S[0], &t1, &p1, &pk1, &np1)) >= 0) {}
                if (t1 > t2)
                    while (t2 < t1 && (r2 = stream_next(&S[1], &t2, &p2, &pk2, &np2)) >= 0) {}
            } while (t2 != t1 && r1 >= 0 && r2 >= 0);
            if (r1 > 0 && r2 > 0) {
                if (t1 != t2 || p1 != p2) {
                    fprintf(stderr, "[dual_pileup] tumor and normal walks out of step. Abort!\n");
                    abort();
                }
                stop = fn(t1, p1, r1, r2, pk1, np1, pk2, np2, data);
            }
        }
        for (int k = 0; k < 2; ++k) {
            pthread_mutex_lock(&S[k].mu);
            S[k].stop = 1;
            if (S[k].cur) ++S[k].consumed;
            S[k].consumed = S[k].produced;      /* release every chunk: the walk may be waiting */
            pthread_cond_broadcast(&S[k].cv);
            pthread_mutex_unlock(&S[k].mu);
            pthread_join(S[k].th, NULL);
            for (int c = 0; c < N_CHUNKS; ++c) { free(S[k].chunks[c].hdr); free(S[k].chunks[c].pk); }
            pthread_mutex_destroy(&S[k].mu);
            pthread_cond_destroy(&S[k].cv);
        }
        free(S);
    }
    const int err = w1->error || w2->error;
    if (err) fprintf(stderr, "[dual_pileup] truncated or malformed BAM record\n");
    walker_free(w1);
    walker_free(w2);
    free(w1);
    free(w2);
    return err ? -1 : 0;
}

int dual_pileup_range(bgzf_reader_t *fp1, bgzf_reader_t *fp2, int mask, int thresh, const col_seed_t *s1,
                      const col_seed_t *s2, dual_site_fn fn, void *data)
{
    return column_run(fp1, fp2, mask, thresh, s1, s2, fn, data);
}
