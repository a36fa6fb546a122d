/* ss_synth.h -- internal helpers of the synthetic generator (host side). */
#ifndef SS_SYNTH_H
#define SS_SYNTH_H

#include "sniper_amd.h"
#include "ss_synth_core.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cdf_tumor / cdf_normal: caller buffers of SS_SYNTH_MAXCDF u32 each. */
int  ss_synth_prepare(const ss_synth_t *s, ss_synth_k_t *k, uint32_t *cdf_tumor,
                      uint32_t *cdf_normal);
void ss_synth_site_depth(const ss_synth_k_t *k, uint64_t site, uint8_t *ref,
                         uint32_t *dt, uint32_t *dn);
void ss_synth_site_reads(const ss_synth_k_t *k, uint64_t site, uint32_t *rt, uint32_t *rn);

#ifdef __cplusplus
}
#endif
#endif
