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

typedef struct {
    const bam_record_t *b;
    int32_t qpos;
    uint8_t is_del;
    uint32_t packed;      /* SS_READ_PACK of this entry (valid when !is_del) */
} pl_entry_t;

/* Called for every reported position; return non-zero to stop the walk. */
typedef int (*dual_site_fn)(int32_t tid, int32_t pos, int n1, int n2, const pl_entry_t *pu1,
                            const pl_entry_t *pu2, void *data);

/* mask < 0 selects SS_BAM_DEF_MASK, otherwise SS_BAM_FUNMAP | mask
 * (bam_plbuf_set_mask :148-152); thresh < 0 is 0.  Returns 0, or -1 on a read
 * error (message on stderr). */
int dual_pileup_run(bgzf_reader_t *fp1, bgzf_reader_t *fp2, int mask, int thresh, dual_site_fn fn,
                    void *data);

#endif
