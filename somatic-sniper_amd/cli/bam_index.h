/* bam_index.h -- the BAM index (.bai, SAM spec section 5.2; samtools-0.1.6
 * bam_index.c:397 bam_index_load, :479 bam_fetch) as the contig-parallel
 * pileup uses it: where each contig's records start, the 16 kb linear index
 * to read a contig's tail, and a compressed-size estimate per contig.  Also a
 * builder (the `ss-index` tool and the tests make indexes with it). */
#ifndef SS_BAM_INDEX_H
#define SS_BAM_INDEX_H

#include <stdint.h>

typedef struct {
    uint64_t first;        /* virtual offset of the contig's first record (UINT64_MAX: none) */
    uint64_t bytes;        /* compressed bytes its chunks span (load-balancing estimate) */
    int32_t n_intv;
    uint64_t *ioff;        /* linear index: smallest virtual offset of a record overlapping 16 kb window i */
} bai_ref_t;

typedef struct {
    int32_t n_ref;
    bai_ref_t *ref;
} bai_t;

/* path.bai, or path with ".bam" replaced by ".bai"; NULL if neither loads or
 * the index is older than the BAM (stale) */
bai_t *bai_load_for(const char *bam_path);
void bai_free(bai_t *x);
/* Writes the index of bam_path to out_path; 0 on success. */
int bai_build(const char *bam_path, const char *out_path);

/* The last record before contig t0 that the pileup loads (flag & mask == 0,
 * mapQ >= thresh): its contig and position, found by reading the tail of the
 * last contig before t0 that has records (its last linear-index windows,
 * further back only when none of them passes the filter).  Returns 1 with
 * *tid / *pos, 0 when no such record exists, -1 on a read error, -2 when a
 * record at one of the index's offsets is not on the contig the index gives
 * (an index of another file). */
int bai_last_loaded_before(const char *bam_path, const bai_t *x, int32_t t0, uint32_t mask, int thresh,
                           int32_t *tid, int64_t *pos);
/* Virtual offset of the first record of contig t0 or later (UINT64_MAX: none). */
uint64_t bai_first_at_or_after(const bai_t *x, int32_t t0);
/* 0 when the record at the index's first offset of contig t0 or later reads
 * back and lies on that very contig (or nothing is indexed from t0 on): the
 * index agrees with the file there; -1 otherwise. */
int bai_check_start(const char *bam_path, const bai_t *x, int32_t t0);

#endif
