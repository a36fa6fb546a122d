/* bam_reader.h -- BAM header and alignment records (SAM spec section 4.2)
 * over a bgzf_reader_t.  Only what the pileup needs is decoded. */
#ifndef SS_BAM_READER_H
#define SS_BAM_READER_H

#include <stdint.h>

#include "bgzf_reader.h"

#define SS_BAM_FUNMAP    4u
#define SS_BAM_FREVERSE  16u
#define SS_BAM_FSECONDARY 256u
#define SS_BAM_FQCFAIL   512u
#define SS_BAM_FDUP      1024u
/* samtools-0.1.6/bam.h:121 */
#define SS_BAM_DEF_MASK (SS_BAM_FUNMAP | SS_BAM_FSECONDARY | SS_BAM_FQCFAIL | SS_BAM_FDUP)

enum { SS_CIG_M = 0, SS_CIG_I, SS_CIG_D, SS_CIG_N, SS_CIG_S, SS_CIG_H, SS_CIG_P };

typedef struct {
    int32_t n_ref;
    char **name;
    int32_t *len;
} bam_header_t;

typedef struct {
    int32_t tid, pos;
    uint8_t mapq;
    uint16_t flag, n_cigar;
    int32_t l_seq;
    uint16_t l_qname;    /* incl. the NUL padding that aligns the CIGAR */
    uint8_t *data;        /* qname | cigar (u32) | seq (4-bit) | qual | aux */
    int32_t l_data, m_data;
} bam_record_t;

int  bam_header_read(bgzf_reader_t *fp, bam_header_t *h);   /* 0 ok */
void bam_header_free(bam_header_t *h);
/* 1 = record read, 0 = end of file, -1 = truncated / malformed */
int  bam_record_read(bgzf_reader_t *fp, bam_record_t *b);
void bam_record_free(bam_record_t *b);
void bam_record_copy(bam_record_t *dst, const bam_record_t *src);

static inline const uint32_t *bam_rec_cigar(const bam_record_t *b)
{
    return (const uint32_t *)(b->data + b->l_qname);
}
static inline const uint8_t *bam_rec_seq(const bam_record_t *b)
{
    return b->data + b->l_qname + 4 * (int)b->n_cigar;
}
static inline const uint8_t *bam_rec_qual(const bam_record_t *b)
{
    return bam_rec_seq(b) + ((b->l_seq + 1) >> 1);
}
static inline uint32_t bam_rec_base(const bam_record_t *b, int qpos)
{
    return (bam_rec_seq(b)[qpos >> 1] >> ((~qpos & 1) << 2)) & 0xfu;
}
/* reference end (samtools bam_calend: M, D and N consume the reference) */
uint32_t bam_rec_end(const bam_record_t *b);

#endif
