/* fasta_index.h -- FASTA + .fai index (the faidx format: name, length, byte
 * offset, bases per line, bytes per line), with the reference CLI's fetch
 * semantics (samtools-0.1.6 faidx.c fai_fetch, used at somatic_sniper.c:114). */
#ifndef SS_FASTA_INDEX_H
#define SS_FASTA_INDEX_H

#include <stdint.h>

typedef struct fasta_index fasta_index_t;

/* Opens fn and fn.fai; builds and writes fn.fai when it is missing
 * (printing "[fai_load] build FASTA index." like samtools). NULL on error. */
fasta_index_t *fasta_index_load(const char *fn);
void fasta_index_free(fasta_index_t *fi);
/* Sequence of a region string "name" or "name:beg-end" (1-based, commas and
 * blanks removed), exactly as fai_fetch parses it.  malloc'ed, *len set; NULL
 * and *len = 0 when the name is unknown. */
char *fasta_fetch(const fasta_index_t *fi, const char *region, int *len);

#endif
