/* bam_reader.c -- see bam_reader.h.  Little-endian hosts only (x86-64). */
#include "bam_reader.h"

#include <stdlib.h>
#include <string.h>

static int rd(bgzf_reader_t *fp, void *p, size_t n) { return bgzf_read(fp, p, n) == (long)n ? 0 : -1; }

int bam_header_read(bgzf_reader_t *fp, bam_header_t *h)
{
    memset(h, 0, sizeof *h);
    char magic[4];
    int32_t l_text;
    if (rd(fp, magic, 4) || memcmp(magic, "BAM\1", 4) || rd(fp, &l_text, 4) || l_text < 0) return -1;
    char *text = (char *)malloc((size_t)l_text + 1);
    if (!text || rd(fp, text, (size_t)l_text)) { free(text); return -1; }
    free(text);                        /* @RG etc. are not used by the scorer */
    if (rd(fp, &h->n_ref, 4) || h->n_ref < 0) return -1;
    h->name = (char **)calloc((size_t)h->n_ref + 1, sizeof(char *));
    h->len = (int32_t *)calloc((size_t)h->n_ref + 1, sizeof(int32_t));
    if (!h->name || !h->len) return -1;
    for (int32_t i = 0; i < h->n_ref; ++i) {
        int32_t l;
        if (rd(fp, &l, 4) || l <= 0) return -1;
        h->name[i] = (char *)malloc((size_t)l + 1);
        if (!h->name[i] || rd(fp, h->name[i], (size_t)l) || rd(fp, &h->len[i], 4)) return -1;
        h->name[i][l] = 0;
    }
    return 0;
}

void bam_header_free(bam_header_t *h)
{
    if (h->name)
        for (int32_t i = 0; i < h->n_ref; ++i) free(h->name[i]);
    free(h->name);
    free(h->len);
    memset(h, 0, sizeof *h);
}

int bam_record_read(bgzf_reader_t *fp, bam_record_t *b)
{
    int32_t bs;
    const long got = bgzf_read(fp, &bs, 4);
    if (got == 0) return 0;
    if (got != 4 || bs < 32) return -1;
    uint32_t core[8];
    if (rd(fp, core, 32)) return -1;
    b->tid = (int32_t)core[0];
    b->pos = (int32_t)core[1];
    b->l_qname = (uint8_t)(core[2] & 0xff);
    b->mapq = (uint8_t)(core[2] >> 8 & 0xff);
    b->n_cigar = (uint16_t)(core[3] & 0xffff);
    b->flag = (uint16_t)(core[3] >> 16);
    b->l_seq = (int32_t)core[4];
    /* the read name is padded with NULs to a multiple of 4 bytes so that the
     * CIGAR words after it are aligned (the file's layout does not align them) */
    const int32_t pad = (4 - (b->l_qname & 3)) & 3;
    b->l_data = bs - 32 + pad;
    if (b->l_data > b->m_data) {
        int32_t m = b->l_data + 64;
        uint8_t *d = (uint8_t *)realloc(b->data, (size_t)m);
        if (!d) return -1;
        b->data = d;
        b->m_data = m;
    }
    if (b->l_qname > bs - 32) return -1;
    if (rd(fp, b->data, (size_t)b->l_qname)) return -1;
    memset(b->data + b->l_qname, 0, (size_t)pad);
    if (rd(fp, b->data + b->l_qname + pad, (size_t)(bs - 32 - b->l_qname))) return -1;
    b->l_qname += pad;
    if (b->l_seq < 0 || (int64_t)b->l_qname + 4 * (int64_t)b->n_cigar + ((b->l_seq + 1) >> 1) + b->l_seq >
                            b->l_data)
        return -1;
    return 1;
}

void bam_record_copy(bam_record_t *dst, const bam_record_t *src)
{
    uint8_t *d = dst->data;
    int32_t m = dst->m_data;
    if (src->l_data > m) {
        m = src->l_data + 64;
        d = (uint8_t *)realloc(d, (size_t)m);
        if (!d) abort();
    }
    *dst = *src;
    dst->data = d;
    dst->m_data = m;
    memcpy(d, src->data, (size_t)src->l_data);
}

void bam_record_free(bam_record_t *b)
{
    free(b->data);
    memset(b, 0, sizeof *b);
}

uint32_t bam_rec_end(const bam_record_t *b)
{
    const uint32_t *c = bam_rec_cigar(b);
    uint32_t end = (uint32_t)b->pos;
    for (int k = 0; k < b->n_cigar; ++k) {
        const uint32_t op = c[k] & 0xf;
        if (op == SS_CIG_M || op == SS_CIG_D || op == SS_CIG_N) end += c[k] >> 4;
    }
    return end;
}
