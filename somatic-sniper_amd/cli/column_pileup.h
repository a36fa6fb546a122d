/* column_pileup.h -- one sample's pileup columns built by scattering reads
 * into a window of positions instead of walking every position over the
 * loaded reads (src/lib/sniper/sniper_pileup.c:172-224 does the latter).
 *
 * The stream holds exactly the positions the reference walk reports with at
 * least one pileup entry, with the same raw entry counts and the same entries
 * in the same (load) order.  The walk's observable rules, derived from
 * get_next_pos (:172-224) and resolve_cigar (:57-111) for input sorted by
 * contig (the only order the reference accepts, :211):
 *   - the walk position W when record k is loaded is 0 for the first record;
 *     afterwards W = max(W, beg(k-1)) if record k-1 was on the walk's contig,
 *     and beg(k-1) if it started a later contig (the walk enters that contig
 *     at 0 and advances to beg(k-1) before it loads again);
 *   - a record is kept iff its reference end (bam_calend: M, D and N ops)
 *     is > W -- for the first record of a later contig, W is a position on
 *     the PREVIOUS contig;
 *   - a kept record on the walk's contig contributes from max(beg, W) on
 *     (positions before W were already reported); one on a later contig
 *     contributes from beg;
 *   - M positions are entries with a base, D positions deleted entries
 *     (raw count only), N positions nothing; I and S advance the query
 *     offset; other ops (H, P, =, X) move neither coordinate, as in
 *     resolve_cigar;
 *   - all columns before W are final once record k is loaded, and a later
 *     contig finalises every column of the current one. */
#ifndef SS_COLUMN_PILEUP_H
#define SS_COLUMN_PILEUP_H

#include <stdint.h>

#include "bgzf_reader.h"

typedef struct col_stream col_stream_t;

/* Starts the reader thread over fp (header already read) and n_workers
 * window-building threads.  mask / thresh as in dual_pileup_run. */
col_stream_t *col_stream_start(bgzf_reader_t *fp, int mask, int thresh, int n_workers);

/* A stream over one range of contigs (the contig-parallel pileup): fp is
 * positioned at the range's first record; the walk state is what the whole
 * file's walk has there -- by the rules above it depends only on the last
 * record loaded before it (its contig becomes the walk's contig and its
 * position W) -- and the stream ends at the first record of contig
 * stop_tid. */
typedef struct {
    int has_prev;            /* 0: the range starts the file (walk at contig 0, W = 0) */
    int32_t prev_tid;
    int64_t prev_pos;
    int32_t stop_tid;        /* INT32_MAX: to the end of the file */
} col_seed_t;
col_stream_t *col_stream_start_at(bgzf_reader_t *fp, int mask, int thresh, int n_workers, const col_seed_t *seed);
/* Next reported column: 1 with its contig, position, raw entry count r and
 * the np packed non-deleted entries (valid until the next call); 0 at the
 * end of the stream. */
int col_stream_next(col_stream_t *S, int32_t *tid, int32_t *pos, int *r, const uint32_t **pk, int *np);
/* Stops the producer and frees the stream; returns -1 if it met a read error. */
int col_stream_stop(col_stream_t *S);

#endif
