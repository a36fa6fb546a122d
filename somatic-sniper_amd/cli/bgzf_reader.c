/* bgzf_reader.c -- see bgzf_reader.h.
 *
 * A BGZF file is a series of gzip members of at most 64 KiB each, whose gzip
 * header carries the member size in the "BC" extra subfield.  Members are
 * independent, so they are inflated in parallel: one I/O thread cuts the file
 * into members and queues them in a ring of slots, workers inflate slots, and
 * the consumer drains slots strictly in file order. */
#include "bgzf_reader.h"

#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define BLK_MAX  65536
#define N_SLOTS  64

enum { SLOT_FREE, SLOT_LOADED, SLOT_BUSY, SLOT_DONE, SLOT_EOF, SLOT_ERR };

typedef struct {
    int state;
    uint32_t clen, ulen, pos;
    uint8_t cbuf[BLK_MAX];
    uint8_t ubuf[BLK_MAX];
} slot_t;

struct bgzf_reader {
    FILE *fp;
    int own_fp;
    int n_threads;
    /* synchronous mode */
    slot_t *one;
    void *dec;
    int eof;
    int64_t coff_cur, coff_next;   /* file offsets of the current member and the next one */
    /* threaded mode */
    slot_t *slots;
    slot_t *cur;          /* the slot the consumer is draining (it owns it: no lock) */
    uint64_t next_load, next_read, next_work;
    int stop, io_done;
    pthread_mutex_t mu;
    pthread_cond_t cv_load, cv_work, cv_read;
    pthread_t io;
    pthread_t *workers;
    char err[160];
};

/* Reads one member into s (compressed payload + trailer sizes).  Returns 1,
 * 0 at clean end of file, -1 on error. */
static int read_member(FILE *fp, slot_t *s, char *err)
{
    uint8_t h[18];
    size_t got = fread(h, 1, 12, fp);
    if (got == 0) return 0;
    if (got != 12 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) {
        snprintf(err, 160, "not a BGZF file (bad gzip member header)");
        return -1;
    }
    const uint32_t xlen = (uint32_t)h[10] | (uint32_t)h[11] << 8;
    uint8_t extra[256];
    if (xlen > sizeof extra || fread(extra, 1, xlen, fp) != xlen) {
        snprintf(err, 160, "truncated BGZF header");
        return -1;
    }
    int bsize = -1;
    for (uint32_t p = 0; p + 4 <= xlen;) {
        const uint32_t sl = (uint32_t)extra[p + 2] | (uint32_t)extra[p + 3] << 8;
        if (extra[p] == 'B' && extra[p + 1] == 'C' && sl == 2 && p + 6 <= xlen)
            bsize = (int)((uint32_t)extra[p + 4] | (uint32_t)extra[p + 5] << 8);
        p += 4 + sl;
    }
    if (bsize < 0) {
        snprintf(err, 160, "gzip member without a BGZF block size");
        return -1;
    }
    const long clen = (long)bsize + 1 - 12 - (long)xlen;      /* deflate data + 8-byte trailer */
    if (clen < 8 || clen > BLK_MAX || fread(s->cbuf, 1, (size_t)clen, fp) != (size_t)clen) {
        snprintf(err, 160, "truncated BGZF block");
        return -1;
    }
    s->clen = (uint32_t)clen;
    return 1;
}

/* libdeflate (whole-buffer DEFLATE, 2-3x zlib's inflate rate) is used when
 * the system has it; zlib otherwise.  Only its stable C ABI (libdeflate.h,
 * v1.x) is bound, at run time, so the build does not need its header. */
typedef struct {
    void *(*alloc)(void);
    void (*release)(void *);
    int (*decompress)(void *, const void *, size_t, void *, size_t, size_t *);
    uint32_t (*crc)(uint32_t, const void *, size_t);
} deflate_lib_t;

static deflate_lib_t LD;
static pthread_once_t ld_once = PTHREAD_ONCE_INIT;

static void ld_load(void)
{
    const char *off = getenv("SS_NO_LIBDEFLATE");
    if (off && *off && *off != '0') return;
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    deflate_lib_t l;
    *(void **)&l.alloc = dlsym(h, "libdeflate_alloc_decompressor");
    *(void **)&l.release = dlsym(h, "libdeflate_free_decompressor");
    *(void **)&l.decompress = dlsym(h, "libdeflate_deflate_decompress");
    *(void **)&l.crc = dlsym(h, "libdeflate_crc32");
    if (l.alloc && l.release && l.decompress && l.crc) LD = l;
}

/* per-thread decompressor: NULL selects zlib */
static void *dec_new(void)
{
    pthread_once(&ld_once, ld_load);
    return LD.alloc ? LD.alloc() : NULL;
}

static void dec_free(void *d)
{
    if (d) LD.release(d);
}

static int inflate_member(slot_t *s, void *dec)
{
    const uint8_t *t = s->cbuf + s->clen - 8;
    const uint32_t isize = (uint32_t)t[4] | (uint32_t)t[5] << 8 | (uint32_t)t[6] << 16 | (uint32_t)t[7] << 24;
    if (isize > BLK_MAX) return -1;
    const uint32_t crc = (uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
    if (dec) {
        size_t got = 0;
        if (LD.decompress(dec, s->cbuf, s->clen - 8, s->ubuf, BLK_MAX, &got) != 0 || got != isize) return -1;
        if (LD.crc(0, s->ubuf, isize) != crc) return -1;
        s->ulen = isize;
        s->pos = 0;
        return 0;
    }
    z_stream z;
    memset(&z, 0, sizeof z);
    if (inflateInit2(&z, -15) != Z_OK) return -1;
    z.next_in = s->cbuf;
    z.avail_in = s->clen - 8;
    z.next_out = s->ubuf;
    z.avail_out = BLK_MAX;
    const int rc = inflate(&z, Z_FINISH);
    inflateEnd(&z);
    if (rc != Z_STREAM_END || z.total_out != isize) return -1;
    if ((uint32_t)crc32(0L, s->ubuf, isize) != crc) return -1;
    s->ulen = isize;
    s->pos = 0;
    return 0;
}

static void *io_main(void *arg)
{
    bgzf_reader_t *r = (bgzf_reader_t *)arg;
    for (;;) {
        pthread_mutex_lock(&r->mu);
        slot_t *s = &r->slots[r->next_load % N_SLOTS];
        while (!r->stop && s->state != SLOT_FREE) pthread_cond_wait(&r->cv_load, &r->mu);
        if (r->stop) { pthread_mutex_unlock(&r->mu); return NULL; }
        pthread_mutex_unlock(&r->mu);
        char err[160] = {0};
        const int rc = read_member(r->fp, s, err);
        pthread_mutex_lock(&r->mu);
        if (rc == 1) s->state = SLOT_LOADED;
        else {
            s->state = rc == 0 ? SLOT_EOF : SLOT_ERR;
            if (rc < 0) memcpy(r->err, err, sizeof err);
            r->io_done = 1;
        }
        ++r->next_load;
        pthread_cond_broadcast(&r->cv_work);
        pthread_cond_broadcast(&r->cv_read);
        const int done = rc != 1;
        pthread_mutex_unlock(&r->mu);
        if (done) return NULL;
    }
}

static void *worker_main(void *arg)
{
    bgzf_reader_t *r = (bgzf_reader_t *)arg;
    void *dec = dec_new();
    pthread_mutex_lock(&r->mu);
    for (;;) {
        while (!r->stop && r->next_work >= r->next_load && !r->io_done)
            pthread_cond_wait(&r->cv_work, &r->mu);
        if (r->stop || r->next_work >= r->next_load) break;
        slot_t *s = &r->slots[r->next_work % N_SLOTS];
        if (s->state != SLOT_LOADED) break;            /* end-of-file or error marker */
        ++r->next_work;
        s->state = SLOT_BUSY;
        pthread_mutex_unlock(&r->mu);
        const int rc = inflate_member(s, dec);
        pthread_mutex_lock(&r->mu);
        s->state = rc == 0 ? SLOT_DONE : SLOT_ERR;
        if (rc) snprintf(r->err, sizeof r->err, "corrupt BGZF block (inflate / CRC)");
        pthread_cond_broadcast(&r->cv_read);
    }
    pthread_cond_broadcast(&r->cv_work);
    pthread_mutex_unlock(&r->mu);
    dec_free(dec);
    return NULL;
}

static bgzf_reader_t *open_common(const char *path, int n_threads, int64_t coff)
{
    bgzf_reader_t *r = (bgzf_reader_t *)calloc(1, sizeof *r);
    if (!r) return NULL;
    if (strcmp(path, "-") == 0) r->fp = stdin;
    else { r->fp = fopen(path, "rb"); r->own_fp = 1; }
    if (!r->fp) { free(r); return NULL; }
    if (coff > 0 && fseeko(r->fp, (off_t)coff, SEEK_SET) != 0) { fclose(r->fp); free(r); return NULL; }
    r->coff_cur = r->coff_next = coff;
    r->n_threads = n_threads;
    if (n_threads <= 0) {
        r->one = (slot_t *)calloc(1, sizeof(slot_t));
        if (!r->one) { bgzf_close(r); return NULL; }
        r->one->state = SLOT_FREE;
        r->dec = dec_new();
        return r;
    }
    r->slots = (slot_t *)calloc(N_SLOTS, sizeof(slot_t));
    r->workers = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    if (!r->slots || !r->workers) { bgzf_close(r); return NULL; }
    pthread_mutex_init(&r->mu, NULL);
    pthread_cond_init(&r->cv_load, NULL);
    pthread_cond_init(&r->cv_work, NULL);
    pthread_cond_init(&r->cv_read, NULL);
    pthread_create(&r->io, NULL, io_main, r);
    for (int i = 0; i < n_threads; ++i) pthread_create(&r->workers[i], NULL, worker_main, r);
    return r;
}

bgzf_reader_t *bgzf_open(const char *path, int n_threads) { return open_common(path, n_threads, 0); }

bgzf_reader_t *bgzf_open_at(const char *path, int n_threads, uint64_t voff)
{
    if (strcmp(path, "-") == 0) return NULL;
    bgzf_reader_t *r = open_common(path, n_threads, (int64_t)(voff >> 16));
    if (!r) return NULL;
    uint8_t skip[65536];
    const size_t k = (size_t)(voff & 0xffffu);
    if (k && bgzf_read(r, skip, k) != (long)k) { bgzf_close(r); return NULL; }
    return r;
}

int64_t bgzf_tell(const bgzf_reader_t *r)
{
    if (r->slots) return -1;
    const slot_t *s = r->one;
    if (s->state != SLOT_DONE || s->pos == s->ulen) return r->coff_next << 16;
    return r->coff_cur << 16 | (int64_t)s->pos;
}

long bgzf_read(bgzf_reader_t *r, void *dst, size_t n)
{
    uint8_t *out = (uint8_t *)dst;
    size_t done = 0;
    if (!r->slots) {                                   /* synchronous */
        slot_t *s = r->one;
        while (done < n) {
            if (s->state != SLOT_DONE || s->pos == s->ulen) {
                if (r->eof) break;
                const int64_t at = r->coff_next;
                const int rc = read_member(r->fp, s, r->err);
                if (rc == 0) { r->eof = 1; break; }
                if (rc < 0 || inflate_member(s, r->dec)) {
                    if (!r->err[0]) snprintf(r->err, sizeof r->err, "corrupt BGZF block (inflate / CRC)");
                    return -1;
                }
                s->state = SLOT_DONE;
                r->coff_cur = at;
                r->coff_next = (int64_t)ftello(r->fp);
                continue;
            }
            size_t k = s->ulen - s->pos;
            if (k > n - done) k = n - done;
            memcpy(out + done, s->ubuf + s->pos, k);
            s->pos += (uint32_t)k;
            done += k;
        }
        return (long)done;
    }
    while (done < n) {
        slot_t *s = r->cur;
        if (!s) {                                      /* wait for the next member in file order */
            pthread_mutex_lock(&r->mu);
            s = &r->slots[r->next_read % N_SLOTS];
            while (r->next_read >= r->next_load || (s->state != SLOT_DONE && s->state != SLOT_EOF &&
                                                     s->state != SLOT_ERR))
                pthread_cond_wait(&r->cv_read, &r->mu);
            const int st = s->state;
            pthread_mutex_unlock(&r->mu);
            if (st == SLOT_EOF) break;
            if (st == SLOT_ERR) return -1;
            r->cur = s;
        }
        size_t k = s->ulen - s->pos;
        if (k > n - done) k = n - done;
        memcpy(out + done, s->ubuf + s->pos, k);
        s->pos += (uint32_t)k;
        done += k;
        if (s->pos == s->ulen) {                       /* drained: hand the slot back to the loader */
            r->cur = NULL;
            pthread_mutex_lock(&r->mu);
            s->state = SLOT_FREE;
            ++r->next_read;
            pthread_cond_broadcast(&r->cv_load);
            pthread_mutex_unlock(&r->mu);
        }
    }
    return (long)done;
}

const char *bgzf_error(const bgzf_reader_t *r) { return r->err[0] ? r->err : "ok"; }

void bgzf_close(bgzf_reader_t *r)
{
    if (!r) return;
    if (r->slots) {
        pthread_mutex_lock(&r->mu);
        r->stop = 1;
        pthread_cond_broadcast(&r->cv_load);
        pthread_cond_broadcast(&r->cv_work);
        pthread_mutex_unlock(&r->mu);
        pthread_join(r->io, NULL);
        for (int i = 0; i < r->n_threads; ++i) pthread_join(r->workers[i], NULL);
        pthread_mutex_destroy(&r->mu);
        pthread_cond_destroy(&r->cv_load);
        pthread_cond_destroy(&r->cv_work);
        pthread_cond_destroy(&r->cv_read);
    }
    free(r->slots);
    free(r->workers);
    free(r->one);
    dec_free(r->dec);
    if (r->own_fp && r->fp) fclose(r->fp);
    free(r);
}
