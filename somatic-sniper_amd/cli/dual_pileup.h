/* dual_pileup.h -- the tumor/normal lockstep pileup walk of the reference CLI
 * (src/lib/sniper/sniper_pileup.c:57-266), restated with the same observable
 * behaviour, quirks included:
 *   - every position of a contig is visited from 0 (get_next_pos :172-224);
 *   - a newly read record is kept only if it ends after the CURRENT position,
 *     even when it lies on a later contig (the first read of a new contig can
 *     be dropped, :216);
 *   - masked-flag reads and reads below the mapping-quality threshold are
 *     never loaded (:208); sortedness is checked on the contig index only;
 *   - a position is reported when both samples have at least one pileup entry
 *     (deletions count, reference skips do not); the walk stops as soon as
 *     either file is exhausted (:245-259). */
#ifndef SS_DUAL_PILEUP_H
#define SS_DUAL_PILEUP_H

#include <stdint.h>

#include "bam_reader.h"
#include "column_pileup.h"

typedef struct {
    const bam_record_t *b;
    int32_t qpos;
    uint8_t is_del;
    uint32_t packed;      /* SS_READ_PACK of this entry (valid when !is_del) */
} pl_entry_t;

/* Called for every reported position with the raw entry counts n1 / n2
 * (deletions included) and the packed non-deleted reads (SS_READ_PACK) of
 * each sample in pileup order; return non-zero to stop the walk. */
typedef int (*dual_site_fn)(int32_t tid, int32_t pos, int n1, int n2, const uint32_t *pk1, int np1,
                            const uint32_t *pk2, int np2, void *data);

/* mask < 0 selects SS_BAM_DEF_MASK, otherwise SS_BAM_FUNMAP | mask
 * (bam_plbuf_set_mask :148-152); thresh < 0 is 0.  threaded: 0 walks both
 * samples position by position on the calling thread; 1 runs each sample's
 * walk on its own thread (the two walks only meet in the lockstep loop, so
 * the reported sites are the same); 2 builds each sample's columns by
 * scattering reads over windows of positions on its own thread
 * (column_pileup.h) and merges the two column streams -- same sites, same
 * entries in the same order, a fraction of the work per entry.  Returns 0,
 * or -1 on a read error (message on stderr). */
int dual_pileup_run(bgzf_reader_t *fp1, bgzf_reader_t *fp2, int mask, int thresh, int threaded,
                    dual_site_fn fn, void *data);

/* Column mode over one contig range of both files (the contig-parallel
 * pileup, sniper_cli.c): fp1 / fp2 positioned at the range's first records,
 * s1 / s2 the walks' states there (column_pileup.h).  The sites reported are
 * those of the whole-file walk on the range's contigs: both walks' states
 * depend only on their own files, and the lockstep loop reports exactly the
 * positions both walks report with entries (column_run). */
int dual_pileup_range(bgzf_reader_t *fp1, bgzf_reader_t *fp2, int mask, int thresh, const col_seed_t *s1,
                      const col_seed_t *s2, dual_site_fn fn, void *data);

#endif
