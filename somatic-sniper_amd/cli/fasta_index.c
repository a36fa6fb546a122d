/* fasta_index.c -- see fasta_index.h.  Plain (uncompressed) FASTA only. */
#include "fasta_index.h"

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    char *name;
    int64_t len, offset;
    int32_t line_blen, line_len;
} fai_entry_t;

struct fasta_index {
    FILE *fp;
    fai_entry_t *e;
    int n, m;
    /* open-addressing name -> entry index (the last entry of a name wins) */
    int *slot;
    int n_slot;
};

static uint64_t hash_str(const char *s)
{
    uint64_t h = 1469598103934665603ull;
    for (; *s; ++s) h = (h ^ (uint8_t)*s) * 1099511628211ull;
    return h;
}

static int add_entry(fasta_index_t *fi, const char *name, int64_t len, int64_t off, int32_t blen, int32_t llen)
{
    if (fi->n == fi->m) {
        fi->m = fi->m ? fi->m * 2 : 16;
        fai_entry_t *e = (fai_entry_t *)realloc(fi->e, (size_t)fi->m * sizeof *e);
        if (!e) return -1;
        fi->e = e;
    }
    fai_entry_t *t = &fi->e[fi->n++];
    t->name = strdup(name);
    t->len = len;
    t->offset = off;
    t->line_blen = blen;
    t->line_len = llen;
    return t->name ? 0 : -1;
}

static int build_hash(fasta_index_t *fi)
{
    fi->n_slot = 16;
    while (fi->n_slot < 2 * fi->n) fi->n_slot <<= 1;
    fi->slot = (int *)malloc((size_t)fi->n_slot * sizeof(int));
    if (!fi->slot) return -1;
    for (int i = 0; i < fi->n_slot; ++i) fi->slot[i] = -1;
    for (int i = 0; i < fi->n; ++i) {
        uint64_t h = hash_str(fi->e[i].name) & (uint64_t)(fi->n_slot - 1);
        while (fi->slot[h] >= 0 && strcmp(fi->e[fi->slot[h]].name, fi->e[i].name) != 0)
            h = (h + 1) & (uint64_t)(fi->n_slot - 1);
        fi->slot[h] = i;
    }
    return 0;
}

static const fai_entry_t *find(const fasta_index_t *fi, const char *name)
{
    uint64_t h = hash_str(name) & (uint64_t)(fi->n_slot - 1);
    while (fi->slot[h] >= 0) {
        if (strcmp(fi->e[fi->slot[h]].name, name) == 0) return &fi->e[fi->slot[h]];
        h = (h + 1) & (uint64_t)(fi->n_slot - 1);
    }
    return NULL;
}

/* Scan the FASTA once, recording per sequence its base count, the offset of
 * its first base and its line geometry.
 *
 * This is a close restatement of samtools 0.1.6 fai_build_core
 * (samtools-0.1.6/faidx.c:59-129, vendored in the reference as
 * vendor/samtools-0.1.6.tar.gz): the same line-state machine (state 0/1/2/3,
 * the l1/l2-style line_blen/line_len bookkeeping), the same branch order and
 * the same error messages.  It is kept that close on purpose: the .fai bytes
 * the reference writes next to the FASTA and its stderr on malformed input
 * are part of the CLI's parity contract (tests/test_cli_native.py compares
 * both).  The I/O (stdio instead of RAZF) and the name table are this file's
 * own. */
static int build_index(fasta_index_t *fi, FILE *fp, const char *fn)
{
    char *name = NULL;
    size_t m_name = 0;
    int64_t len = -1, offset = 0, pos = 0;
    int32_t line_len = -1, line_blen = -1;
    int state = 0;   /* 1: just after a header, 0: regular lines, 2: a short line seen, 3: then a blank */
    int c;
    while ((c = fgetc(fp)) != EOF) {
        ++pos;
        if (c == '\n') {
            if (state == 1) { offset = pos; continue; }
            if ((state == 0 && len < 0) || state == 2) continue;
        }
        if (c == '>') {
            if (len >= 0 && add_entry(fi, name, len, offset, line_blen, line_len)) return -1;
            size_t l = 0;
            while ((c = fgetc(fp)) != EOF) {
                ++pos;
                if (isspace(c)) break;
                if (l + 2 > m_name) {
                    m_name = m_name ? 2 * m_name : 64;
                    name = (char *)realloc(name, m_name);
                    if (!name) return -1;
                }
                name[l++] = (char)c;
            }
            if (!name) { name = (char *)malloc(1); if (!name) return -1; }
            name[l] = 0;
            if (c == EOF) {
                fprintf(stderr, "[fai_build_core] the last entry has no sequence\n");
                free(name);
                return -1;
            }
            if (c != '\n')
                while ((c = fgetc(fp)) != EOF) { ++pos; if (c == '\n') break; }
            state = 1;
            len = 0;
            offset = pos;
            continue;
        }
        if (state == 3) {
            fprintf(stderr, "[fai_build_core] inlined empty line is not allowed in sequence '%s'.\n", name);
            free(name);
            return -1;
        }
        if (state == 2) state = 3;
        int32_t l1 = 0, l2 = 0;
        for (;;) {
            ++l1;
            if (isgraph(c)) ++l2;
            c = fgetc(fp);
            if (c == EOF) break;
            ++pos;
            if (c == '\n') break;
        }
        if (state == 3 && l2) {
            fprintf(stderr, "[fai_build_core] different line length in sequence '%s'.\n", name);
            free(name);
            return -1;
        }
        ++l1;
        len += l2;
        if (l2 >= 0x10000) {
            fprintf(stderr, "[fai_build_core] line length exceeds 65535 in sequence '%s'.\n", name);
            free(name);
            return -1;
        }
        if (state == 1) { line_len = l1; line_blen = l2; state = 0; }
        else if (state == 0 && (l1 != line_len || l2 != line_blen)) state = 2;
        if (c == EOF) break;
    }
    if (name && add_entry(fi, name, len, offset, line_blen, line_len)) return -1;
    free(name);
    (void)fn;
    return 0;
}

fasta_index_t *fasta_index_load(const char *fn)
{
    fasta_index_t *fi = (fasta_index_t *)calloc(1, sizeof *fi);
    if (!fi) return NULL;
    size_t ln = strlen(fn);
    char *ifn = (char *)malloc(ln + 5);
    if (!ifn) { free(fi); return NULL; }
    memcpy(ifn, fn, ln);
    memcpy(ifn + ln, ".fai", 5);
    FILE *ip = fopen(ifn, "rb");
    if (!ip) {
        fprintf(stderr, "[fai_load] build FASTA index.\n");
        FILE *fp = fopen(fn, "rb");
        if (!fp) {
            fprintf(stderr, "[fai_build] fail to open the FASTA file.\n");
            fprintf(stderr, "[fai_load] fail to open FASTA index.\n");
            goto fail;
        }
        const int rc = build_index(fi, fp, fn);
        fclose(fp);
        if (rc) goto fail;
        FILE *op = fopen(ifn, "wb");
        if (!op) {
            fprintf(stderr, "[fai_build] fail to write FASTA index.\n");
            fprintf(stderr, "[fai_load] fail to open FASTA index.\n");
            goto fail;
        }
        for (int i = 0; i < fi->n; ++i)
            fprintf(op, "%s\t%d\t%lld\t%d\t%d\n", fi->e[i].name, (int)fi->e[i].len,
                    (long long)fi->e[i].offset, fi->e[i].line_blen, fi->e[i].line_len);
        fclose(op);
    } else {
        char buf[0x10000];
        while (fgets(buf, sizeof buf, ip)) {
            char *p = buf;
            while (*p && isgraph((unsigned char)*p)) ++p;
            *p = 0;
            ++p;
            int len = 0, blen = 0, llen = 0;
            long long off = 0;
            sscanf(p, "%d%lld%d%d", &len, &off, &blen, &llen);
            if (add_entry(fi, buf, len, off, blen, llen)) { fclose(ip); goto fail; }
        }
        fclose(ip);
    }
    if (build_hash(fi)) goto fail;
    fi->fp = fopen(fn, "rb");
    if (!fi->fp) {
        fprintf(stderr, "[fai_load] fail to open FASTA file.\n");
        goto fail;
    }
    free(ifn);
    return fi;
fail:
    free(ifn);
    fasta_index_free(fi);
    return NULL;
}

void fasta_index_free(fasta_index_t *fi)
{
    if (!fi) return;
    for (int i = 0; i < fi->n; ++i) free(fi->e[i].name);
    free(fi->e);
    free(fi->slot);
    if (fi->fp) fclose(fi->fp);
    free(fi);
}

char *fasta_fetch(const fasta_index_t *fi, const char *region, int *len)
{
    const size_t l = strlen(region);
    char *s = (char *)malloc(l + 1);
    if (!s) { *len = 0; return NULL; }
    size_t k = 0;
    for (size_t i = 0; i < l; ++i)                   /* commas and blanks are squeezed out */
        if (region[i] != ',' && !isspace((unsigned char)region[i])) s[k++] = region[i];
    s[k] = 0;
    size_t i = 0;
    while (i < k && s[i] != ':') ++i;
    s[i] = 0;
    const fai_entry_t *e = fi->slot ? find(fi, s) : NULL;
    if (!e) { *len = 0; free(s); return NULL; }
    int64_t beg, end;
    if (i == k) {
        beg = 0;
        end = e->len;
    } else {
        const char *p = s + i + 1;
        while (i < k && s[i] != '-') ++i;
        beg = atoi(p);
        end = i < k ? atoi(s + i + 1) : e->len;
    }
    if (beg > 0) --beg;
    if (beg >= e->len) beg = e->len;
    if (end >= e->len) end = e->len;
    if (beg > end) beg = end;
    free(s);
    char *out = (char *)malloc((size_t)(end - beg) + 2);
    if (!out) { *len = 0; return NULL; }
    int n = 0;
    if (e->line_blen > 0) {
        const int64_t at = e->offset + beg / e->line_blen * e->line_len + beg % e->line_blen;
        if (fseeko(fi->fp, (off_t)at, SEEK_SET) == 0) {
            int c;
            while (n < end - beg && (c = fgetc(fi->fp)) != EOF)
                if (isgraph(c)) out[n++] = (char)c;
        }
    }
    out[n] = 0;
    *len = n;
    return out;
}
