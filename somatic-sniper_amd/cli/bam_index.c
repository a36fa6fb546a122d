/* bam_index.c -- see bam_index.h.
 *
 * Index layout (SAM spec 5.2): "BAI\1", n_ref, then per reference n_bin
 * bins (bin id, n_chunk, chunks of [begin, end) virtual offsets) and n_intv
 * linear-index offsets; newer writers add a pseudo-bin 37450 of metadata
 * (skipped) and a trailing unplaced-read count (ignored). */
#include "bam_index.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "bam_reader.h"
#include "bgzf_reader.h"

#define PSEUDO_BIN 37450u
#define N_BINS     37450u

static int rd(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

static bai_t *bai_load(const char *path)
{
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    char magic[4];
    int32_t n_ref;
    bai_t *x = NULL;
    if (rd(f, magic, 4) || memcmp(magic, "BAI\1", 4) || rd(f, &n_ref, 4) || n_ref < 0) goto bad;
    x = (bai_t *)calloc(1, sizeof *x);
    x->n_ref = n_ref;
    x->ref = (bai_ref_t *)calloc((size_t)n_ref + 1, sizeof(bai_ref_t));
    for (int32_t t = 0; t < n_ref; ++t) {
        bai_ref_t *r = &x->ref[t];
        r->first = UINT64_MAX;
        int32_t n_bin;
        if (rd(f, &n_bin, 4) || n_bin < 0) goto bad;
        for (int32_t b = 0; b < n_bin; ++b) {
            uint32_t bin;
            int32_t n_chunk;
            if (rd(f, &bin, 4) || rd(f, &n_chunk, 4) || n_chunk < 0) goto bad;
            for (int32_t c = 0; c < n_chunk; ++c) {
                uint64_t cb[2];
                if (rd(f, cb, 16)) goto bad;
                if (bin == PSEUDO_BIN) continue;
                if (cb[0] < r->first) r->first = cb[0];
                if (cb[1] > cb[0]) r->bytes += (cb[1] >> 16) - (cb[0] >> 16) + 1;
            }
        }
        if (rd(f, &r->n_intv, 4) || r->n_intv < 0) goto bad;
        r->ioff = (uint64_t *)malloc(8 * (size_t)r->n_intv + 8);
        if (r->n_intv && rd(f, r->ioff, 8 * (size_t)r->n_intv)) goto bad;
    }
    fclose(f);
    return x;
bad:
    fclose(f);
    bai_free(x);
    return NULL;
}

/* an index older than its BAM is stale: it may describe a file since
 * rewritten; it is not used and the CLI takes the streaming walk instead (same
 * output, no contig-parallel pileup).  When both mtimes carry nanoseconds
 * (tv_nsec != 0 on both) they are compared to the nanosecond, so an index
 * written earlier in the same second as a rewrite of its BAM is refused.  On
 * a second-resolution filesystem, or for copies that kept only seconds, the
 * test is htslib's whole-second one (hts.c idx_test_and_fetch, which only
 * warns): an index of the same second is used, and bai_check_start still
 * verifies it against the file. */
static bai_t *bai_load_fresh(const char *idx_path, const struct stat *bam_st)
{
    struct stat st;
    if (stat(idx_path, &st) != 0) return NULL;
    if (st.st_mtime < bam_st->st_mtime) return NULL;
    if (st.st_mtime == bam_st->st_mtime && st.st_mtim.tv_nsec != 0 && bam_st->st_mtim.tv_nsec != 0 &&
        st.st_mtim.tv_nsec < bam_st->st_mtim.tv_nsec)
        return NULL;
    return bai_load(idx_path);
}

bai_t *bai_load_for(const char *bam_path)
{
    struct stat bst;
    if (stat(bam_path, &bst) != 0) return NULL;
    const size_t n = strlen(bam_path);
    char *p = (char *)malloc(n + 5);
    snprintf(p, n + 5, "%s.bai", bam_path);
    bai_t *x = bai_load_fresh(p, &bst);
    if (!x && n > 4 && strcmp(bam_path + n - 4, ".bam") == 0) {
        memcpy(p, bam_path, n - 4);
        memcpy(p + n - 4, ".bai", 5);
        x = bai_load_fresh(p, &bst);
    }
    free(p);
    return x;
}

int bai_check_start(const char *bam_path, const bai_t *x, int32_t t0)
{
    int32_t t = t0 < 0 ? 0 : t0;
    while (t < x->n_ref && x->ref[t].first == UINT64_MAX) ++t;
    if (t >= x->n_ref) return 0;                       /* nothing indexed from t0 on */
    bgzf_reader_t *fp = bgzf_open_at(bam_path, 0, x->ref[t].first);
    if (!fp) return -1;
    bam_record_t rec;
    memset(&rec, 0, sizeof rec);
    const int rc = bam_record_read(fp, &rec);
    /* the record there must be on the contig the index says it starts */
    const int ok = rc > 0 && rec.tid == t && rec.pos >= -1;
    bam_record_free(&rec);
    bgzf_close(fp);
    return ok ? 0 : -1;
}

void bai_free(bai_t *x)
{
    if (!x) return;
    for (int32_t t = 0; t < x->n_ref; ++t) free(x->ref[t].ioff);
    free(x->ref);
    free(x);
}

uint64_t bai_first_at_or_after(const bai_t *x, int32_t t0)
{
    for (int32_t t = t0 < 0 ? 0 : t0; t < x->n_ref; ++t)
        if (x->ref[t].first != UINT64_MAX) return x->ref[t].first;
    return UINT64_MAX;
}

/* records from voffset `start` (an index offset of contig t) up to the first
 * one on contig t0 or later: the last that the pileup loads.  1 found, 0 none,
 * -1 read error, -2 the first record is not on contig t (the index does not
 * describe this file). */
static int scan_tail(const char *bam_path, uint64_t start, int32_t t, int32_t t0, uint32_t mask, int thresh,
                     int32_t *tid, int64_t *pos)
{
    bgzf_reader_t *fp = bgzf_open_at(bam_path, 0, start);
    if (!fp) return -1;
    bam_record_t rec;
    memset(&rec, 0, sizeof rec);
    int found = 0, rc, first = 1;
    while ((rc = bam_record_read(fp, &rec)) > 0) {
        if (first && rec.tid != t) { rc = -2; break; }
        first = 0;
        if (rec.tid >= t0 || rec.tid < 0) break;
        if ((rec.flag & mask) || rec.mapq < thresh) continue;
        *tid = rec.tid;
        *pos = rec.pos;
        found = 1;
    }
    bam_record_free(&rec);
    bgzf_close(fp);
    return rc == -2 ? -2 : rc < 0 ? -1 : found;
}

int bai_last_loaded_before(const char *bam_path, const bai_t *x, int32_t t0, uint32_t mask, int thresh,
                           int32_t *tid, int64_t *pos)
{
    for (int32_t t = (t0 > x->n_ref ? x->n_ref : t0) - 1; t >= 0; --t) {
        const bai_ref_t *r = &x->ref[t];
        if (r->first == UINT64_MAX) continue;
        /* the contig's last window first, then exponentially further back */
        int32_t i = r->n_intv - 1, step = 1;
        for (;;) {
            while (i >= 0 && (r->ioff[i] == 0 || r->ioff[i] < r->first)) --i;
            const uint64_t start = i >= 0 ? r->ioff[i] : r->first;
            const int rc = scan_tail(bam_path, start, t, t0, mask, thresh, tid, pos);
            if (rc != 0) return rc;
            if (start == r->first) break;                  /* the whole contig: nothing loaded */
            i -= step;
            step *= 2;
        }
    }
    return 0;
}

/* ---- builder ------------------------------------------------------------- */
static uint32_t reg2bin(int64_t beg, int64_t end)
{
    --end;
    if (beg >> 14 == end >> 14) return (uint32_t)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (uint32_t)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (uint32_t)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (uint32_t)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (uint32_t)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

typedef struct {
    uint64_t *c;       /* begin, end pairs */
    int32_t n, m;
} chunks_t;

typedef struct {
    chunks_t bins[N_BINS];
    uint64_t *lin;
    int32_t n_lin, m_lin;
} ref_acc_t;

static void put_ref(FILE *o, ref_acc_t *A)
{
    int32_t n_bin = 0;
    for (uint32_t b = 0; b < N_BINS; ++b) n_bin += A->bins[b].n > 0;
    fwrite(&n_bin, 4, 1, o);
    for (uint32_t b = 0; b < N_BINS; ++b) {
        chunks_t *C = &A->bins[b];
        if (!C->n) continue;
        const int32_t nc = C->n / 2;
        fwrite(&b, 4, 1, o);
        fwrite(&nc, 4, 1, o);
        fwrite(C->c, 8, (size_t)C->n, o);
        C->n = 0;
    }
    for (int32_t i = 1; i < A->n_lin; ++i)                /* empty windows take the previous offset */
        if (!A->lin[i]) A->lin[i] = A->lin[i - 1];
    fwrite(&A->n_lin, 4, 1, o);
    fwrite(A->lin, 8, (size_t)A->n_lin, o);
    if (A->n_lin) memset(A->lin, 0, 8 * (size_t)A->n_lin);   /* the next contig starts empty */
    A->n_lin = 0;
}

static void put_empty(FILE *o)
{
    const int32_t z[2] = {0, 0};
    fwrite(z, 4, 2, o);
}

int bai_build(const char *bam_path, const char *out_path)
{
    bgzf_reader_t *fp = bgzf_open(bam_path, 0);
    if (!fp) return -1;
    bam_header_t h;
    if (bam_header_read(fp, &h)) { bgzf_close(fp); return -1; }
    FILE *o = fopen(out_path, "wb");
    if (!o) { bam_header_free(&h); bgzf_close(fp); return -1; }
    fwrite("BAI\1", 1, 4, o);
    fwrite(&h.n_ref, 4, 1, o);
    ref_acc_t *A = (ref_acc_t *)calloc(1, sizeof *A);
    bam_record_t rec;
    memset(&rec, 0, sizeof rec);
    int32_t cur = -1;          /* contig being accumulated; contigs before it are written */
    int64_t last_pos = -1;
    int rc, err = 0;
    uint64_t v0 = (uint64_t)bgzf_tell(fp);
    while ((rc = bam_record_read(fp, &rec)) > 0) {
        const uint64_t v1 = (uint64_t)bgzf_tell(fp);
        if (rec.tid < 0) { v0 = v1; continue; }           /* unplaced reads: not indexed */
        /* an index implies a coordinate-sorted file (samtools index refuses others) */
        if (rec.tid < cur || rec.tid >= h.n_ref || (rec.tid == cur && rec.pos < last_pos)) { err = 1; break; }
        last_pos = rec.pos;
        if (cur < rec.tid) {                               /* finish `cur`, empty contigs up to tid */
            if (cur >= 0) put_ref(o, A);
            for (++cur; cur < rec.tid; ++cur) put_empty(o);
        }
        const int64_t beg = rec.pos < 0 ? 0 : rec.pos;
        int64_t end = (int64_t)bam_rec_end(&rec);
        if (end <= beg) end = beg + 1;
        /* BAI bins and linear windows cover [0, 2^29) only (SAM spec 5.2; samtools
         * index asks for CSI beyond): a longer contig cannot be indexed here */
        if (end > ((int64_t)1 << 29)) { err = 1; break; }
        chunks_t *C = &A->bins[reg2bin(beg, end)];
        if (C->n && C->c[C->n - 1] == v0) C->c[C->n - 1] = v1;      /* contiguous: extend */
        else {
            if (C->n + 2 > C->m) {
                C->m = C->m ? 2 * C->m : 8;
                C->c = (uint64_t *)realloc(C->c, 8 * (size_t)C->m);
            }
            C->c[C->n++] = v0;
            C->c[C->n++] = v1;
        }
        const int32_t w0 = (int32_t)(beg >> 14), w1 = (int32_t)((end - 1) >> 14);
        if (w1 >= A->m_lin) {
            const int32_t m = (w1 + 1) * 2;
            A->lin = (uint64_t *)realloc(A->lin, 8 * (size_t)m);
            memset(A->lin + A->m_lin, 0, 8 * (size_t)(m - A->m_lin));
            A->m_lin = m;
        }
        if (w1 >= A->n_lin) A->n_lin = w1 + 1;
        for (int32_t w = w0; w <= w1; ++w)
            if (!A->lin[w]) A->lin[w] = v0;
        v0 = v1;
    }
    if (rc < 0) err = 1;
    if (!err) {
        if (cur >= 0) put_ref(o, A);
        for (int32_t t = cur + 1; t < h.n_ref; ++t) put_empty(o);
    }
    for (uint32_t b = 0; b < N_BINS; ++b) free(A->bins[b].c);
    free(A->lin);
    free(A);
    bam_record_free(&rec);
    bam_header_free(&h);
    bgzf_close(fp);
    if (fclose(o) != 0) err = 1;
    if (err) remove(out_path);
    return err ? -1 : 0;
}

#ifdef SS_INDEX_MAIN
/* ss-index <in.bam> [out.bai]: writes in.bam.bai (test and bench data) */
int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s <in.bam> [out.bai]\n", argv[0]);
        return 1;
    }
    char def[4096];
    snprintf(def, sizeof def, "%s.bai", argv[1]);
    if (bai_build(argv[1], argc > 2 ? argv[2] : def)) {
        fprintf(stderr, "[ss-index] cannot index %s\n", argv[1]);
        return 1;
    }
    return 0;
}
#endif
