/* dual_pileup.c -- see dual_pileup.h for the behaviour being reproduced. */
#include "dual_pileup.h"

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

int dual_pileup_run(bgzf_reader_t *fp1, bgzf_reader_t *fp2, int mask, int thresh, dual_site_fn fn,
                    void *data)
{
    walker_t *w1 = (walker_t *)malloc(sizeof(walker_t)), *w2 = (walker_t *)malloc(sizeof(walker_t));
    if (!w1 || !w2) { free(w1); free(w2); return -1; }
    walker_init(w1, fp1, mask, thresh);
    walker_init(w2, fp2, mask, thresh);
    int r1 = -1, r2 = -1, stop = 0;
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
            stop = fn(w1->tid, w1->pos, r1, r2, w1->pu, w2->pu, data);
        }
    }
    const int err = w1->error || w2->error;
    if (err) fprintf(stderr, "[dual_pileup] truncated or malformed BAM record\n");
    walker_free(w1);
    walker_free(w2);
    free(w1);
    free(w2);
    return err ? -1 : 0;
}
