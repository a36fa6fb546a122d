/* bgzf_reader.h -- sequential reader of BGZF files (the BAM container,
 * SAM spec section 4.1) with block-parallel inflation on a thread pool. */
#ifndef SS_BGZF_READER_H
#define SS_BGZF_READER_H

#include <stddef.h>
#include <stdint.h>

typedef struct bgzf_reader bgzf_reader_t;

/* path "-" reads stdin.  n_threads <= 0 inflates on the calling thread. */
bgzf_reader_t *bgzf_open(const char *path, int n_threads);
/* The same, reading from virtual offset voff (compressed member offset << 16
 * | offset inside the member, as a BAM index stores it); not for stdin. */
bgzf_reader_t *bgzf_open_at(const char *path, int n_threads, uint64_t voff);
/* Virtual offset of the next byte bgzf_read returns (synchronous readers,
 * n_threads <= 0, only; -1 otherwise). */
int64_t bgzf_tell(const bgzf_reader_t *r);
/* Reads up to n bytes; returns the count (< n only at end of data) or -1 on a
 * malformed / truncated file. */
long bgzf_read(bgzf_reader_t *r, void *dst, size_t n);
void bgzf_close(bgzf_reader_t *r);
const char *bgzf_error(const bgzf_reader_t *r);

#endif
