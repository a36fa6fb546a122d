/* ss_host.h -- internal host-side declarations shared by the C-ABI pieces. */
#ifndef SS_HOST_H
#define SS_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "sniper_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ss_host_model {
    ss_params_t prm;
    double   fk[256];
    double  *coef;          /* [64 << 16], index q<<16 | n<<8 | k */
    double  *lhet;          /* [256 * 256], index n1<<8 | n2      */
    float    q_r;
    int      q_r_int;       /* (int)(q_r + .5)                     */
    int32_t  qadd[1024];
    int32_t  prior[16 * 10];
    int32_t  jprior[16 * 10 * 10];
    uint64_t h_fk, h_coef, h_lhet;
    uint64_t fp_coef, fp_lhet; /* ss_tab_fp_words of coef / lhet at their device word offsets */
    int      pinned;        /* default tables equal a pinned reference run */
    int      source;        /* SS_TABLES_BUILT / _PROCESS / _DISK                */
    void    *shared;        /* the process-wide table entry coef / lhet belong to */
} ss_host_model_t;

extern const unsigned char ss_nt16_table[256];   /* immutable (bam_import.c:23-40) */
extern const int ss_genotype_nt16[10];

int      ss_host_model_build(const ss_params_t *p, ss_host_model_t *m);
void     ss_host_model_free(ss_host_model_t *m);
uint64_t ss_fnv1a64(const void *p, size_t n);

/* Fingerprint of a device table image (ss_kernels.h SS_TAB_* layout, 8-byte
 * words): sum over words of mix(w + word_index * golden); additive, so
 * regions can be summed separately.  Word offsets of the big tables: */
#define SS_FP_COEF_WORD ((uint64_t)0)
#define SS_FP_LHET_WORD ((uint64_t)64 << 16)
uint64_t ss_tab_fp_words(const void *p, size_t nwords, uint64_t first_word);

#ifdef __cplusplus
}
#endif
#endif
