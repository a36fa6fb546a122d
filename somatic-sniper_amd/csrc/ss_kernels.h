/* ss_kernels.h -- internal interface between the C ABI (ss_capi.hip) and the
 * HIP kernels (ss_kernels.hip).  Not installed; plain structs of device
 * pointers passed to the kernels by value. */
#ifndef SS_KERNELS_H
#define SS_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sniper_amd.h"
#include "ss_synth_core.h"

/* Device copy of the model (built on the host by ss_tables.c): every table
 * in ONE allocation, so a kernel needs a single base pointer (SGPR pressure). */
#define SS_TAB_COEF   ((size_t)0)                                 /* f64 [64 << 16]  */
#define SS_TAB_LHET   (SS_TAB_COEF + ((size_t)64 << 16) * 8)      /* f64 [65536]     */
#define SS_TAB_FK     (SS_TAB_LHET + (size_t)65536 * 8)           /* f64 [256]       */
#define SS_TAB_QADD   (SS_TAB_FK + (size_t)256 * 8)               /* i32 [1024]      */
#define SS_TAB_PRIOR  (SS_TAB_QADD + (size_t)1024 * 4)            /* i32 [16 * 10]   */
#define SS_TAB_JPRIOR (SS_TAB_PRIOR + (size_t)160 * 4)            /* i32 [16*10*10]  */
#define SS_TAB_NT16   (SS_TAB_JPRIOR + (size_t)1600 * 4)          /* u8  [256]       */
#define SS_NEAR_MAXN  2048u                                       /* reads per sample the early exit takes */
#define SS_TAB_ESR    (SS_TAB_NT16 + (size_t)256)                 /* f32 [2052]: the early exit's esum bound per c24 */
#define SS_TAB_CMIN   (SS_TAB_ESR + (size_t)2052 * 4)             /* f32 [260]: its coef + lh bound per (rescaled) depth */
#define SS_TAB_BYTES  (SS_TAB_CMIN + (size_t)260 * 4)

#define SS_MF_JOINT 1u
#define SS_MF_LOH   2u
#define SS_MF_GOR   4u
#define SS_MF_FAST  8u   /* SS_TAB_ESR / SS_TAB_CMIN are valid (q_r >= 1): the main kernel's early exit may run */

struct ss_dev_model {
    const uint8_t *tab;      /* SS_TAB_* layout */
    int32_t  q_r_int;
    int32_t  cap_mapQ;       /* clamped to [0, 127]: only min(mapQ & 0x7f, cap) is used */
    int32_t  min_somatic_qual;
    uint32_t flags;          /* SS_MF_* */
};

#define SS_TAB_ACCESSOR(name, T, off)                                                  \
    __host__ __device__ __forceinline__ const T *ss_tab_##name(const ss_dev_model &m) \
    {                                                                                  \
        return reinterpret_cast<const T *>(m.tab + (off));                             \
    }
SS_TAB_ACCESSOR(coef, double, SS_TAB_COEF)
SS_TAB_ACCESSOR(lhet, double, SS_TAB_LHET)
SS_TAB_ACCESSOR(fk, double, SS_TAB_FK)
SS_TAB_ACCESSOR(qadd, int32_t, SS_TAB_QADD)
SS_TAB_ACCESSOR(prior, int32_t, SS_TAB_PRIOR)
SS_TAB_ACCESSOR(jprior, int32_t, SS_TAB_JPRIOR)
SS_TAB_ACCESSOR(nt16, uint8_t, SS_TAB_NT16)
SS_TAB_ACCESSOR(esr, float, SS_TAB_ESR)
SS_TAB_ACCESSOR(cmin, float, SS_TAB_CMIN)
#undef SS_TAB_ACCESSOR

/* Per-launch arguments of the scoring kernels. */
struct ss_score_args {
    /* batch (device) */
    uint64_t        n_sites;
    const uint8_t  *ref;
    const uint32_t *off_t, *off_n;
    const uint32_t *reads_t, *reads_n;
    /* outputs (device) */
    int32_t   *score;
    ss_call_t *calls;
    uint32_t   calls_cap;
    uint32_t  *n_calls;
    ss_glf_t  *glf;
    uint32_t  *n_clamped;
    /* work lists (device; counters zeroed per launch) */
    uint32_t  *deep_list;     /* sites the main kernel's per-lane path does not score: one
                                 segment of deep_seg_cap entries per main-kernel wave, no atomics */
    uint32_t  *deep_segs;     /* [deep_nseg] ids of the main waves that listed sites, compacted */
    uint32_t  *deep_off;      /* [deep_nseg] their first entry in the listed order (ascending) */
    unsigned long long *deep_acc; /* listed segments << 32 | listed entries (zeroed per launch) */
    uint32_t  *wide_next;     /* the group kernel's next chunk of GB listed entries (zeroed per launch) */
    uint32_t   deep_seg_cap;
    uint32_t   deep_nseg;     /* = main-kernel waves */
    uint32_t   deep_cap;      /* deep2 / deep3 list capacity (>= n_sites: cannot overflow) */
    uint32_t  *deep2_list;    /* sites the group kernel cannot sort, any depth (ss_score_deep) */
    uint32_t  *deep2_count;
    uint32_t  *deep_next;     /* ss_score_deep's next chunk of deep2 entries (zeroed per launch) */
    uint32_t  *deep3_list;    /* sites ss_score_deep hands on (ss_score_wild): a read of minq >= 64,
                                 a sample past SS_BINS_MAXN reads, malformed offsets */
    uint32_t  *deep3_count;
    uint32_t  *tri_list;      /* the triage kernel's undecided sites, scored by the main kernel (null:
                                 no triage, the main kernel scores every site) */
    uint32_t  *tri_count;
    uint32_t  *dtri_list;     /* the triage kernel's 64-site blocks past SS_EARLY_MAX_READS mean reads (block
                                 indices), for the deep triage kernel */
    uint32_t  *dtri_count;
    uint32_t  *dsite_list;    /* the triage kernel's undecided sites, for the deep triage's wider test */
    uint32_t  *dsite_count;
    uint32_t  *err;           /* sticky error bits, see SS_KERR_* */
    uint8_t   *grp_rec;       /* the group kernel's fold records: SS_GRP_REC_BYTES per wave */
    ss_dev_model m;
};

#define SS_KERR_DEEP_OVERFLOW  1u   /* a deep list overflowed (cannot happen: sized from the batch) */
#define SS_KERR_MALFORMED      8u   /* decreasing or out-of-range read offsets: the site scored -2 */

/* Launch geometry constants shared with the host. */
#define SS_MAIN_BLOCK      256   /* 4 waves, each 64 sites at a time (lane = site) */
#ifndef SS_TRIAGE_BLOCK
#define SS_TRIAGE_BLOCK    512   /* the triage kernel: 8 waves (lane = site), LDS tables shared */
#endif
#ifndef SS_TRIAGE_WAVES_PER_EU
#define SS_TRIAGE_WAVES_PER_EU 6
#endif
#define SS_TRIAGE_GRID_PER_CU 64 /* triage workgroups per CU (grid-strided 64-site blocks) */
#define SS_TRIAGE_DEEP_BLOCK 256 /* the deep triage kernel: 4 waves (16 lanes per site) */
#define SS_TRIAGE_DEEP_GRID_PER_CU 8
#define SS_MAIN_SITES      64    /* sites per main-kernel wave block           */
#define SS_MAIN_GRID_PER_CU 128  /* main-kernel workgroups per CU: 3 resident (166 VGPRs, 52.5 KB LDS each),
                                    the rest queued as short-lived waves (+5.5% over 16 per CU) */
#define SS_DEEP_BLOCK      512   /* 8 waves, one workgroup per CU (LDS: 19 KB per wave) */
#define SS_WILD_BLOCK      256   /* 4 one-site waves per workgroup, 3 per CU (LDS) */
#define SS_BINS_MAXN       65535u /* reads per sample ss_score_deep takes (16-bit bin counts) */
#ifndef SS_WIDE_BLOCK
#define SS_WIDE_BLOCK      768   /* 12 waves, one workgroup per CU (168 VGPRs: 3 waves per SIMD) */
#endif
#ifndef SS_ROUTE_DEEP
#define SS_ROUTE_DEEP      1024  /* a sample past this many reads: the deep kernel, not the group kernel */
#endif
#ifndef SS_WIDE_MAXSLOTS
#define SS_WIDE_MAXSLOTS   2048  /* reads per sample the group kernel sorts (A/B builds may lower it) */
#endif
#define SS_GRP_REC_MAX     131072 /* fold-record bytes of one group-kernel chunk: 32 sites x 2 x 2048 */
#define SS_GRP_REC_PAD     64    /* pad before and after (a 16-record window may reach past either end) */
#define SS_GRP_REC_BYTES   (SS_GRP_REC_MAX + 2 * SS_GRP_REC_PAD)

/* Launchers (return hipError_t as int). */
int ss_launch_score(const ss_score_args &a, int triage_grid, int triage_deep_grid, int main_grid, int wide_grid,
                    int deep_grid, int wild_grid, hipStream_t s,
                    const hipEvent_t *ev /* 4 events (before main, after main, after wide, after deep + wild) or null */);
/* out3 (zeroed by the caller): fingerprint sums of coef, lhet and the rest (ss_host.h) */
int ss_launch_tab_fingerprint(const uint8_t *tab, unsigned long long *out3, hipStream_t s);
int ss_launch_synth_depth(const ss_synth_k_t &k, uint64_t first, uint64_t n, uint8_t *ref,
                          uint32_t *dt, uint32_t *dn, unsigned long long *sums /* [2], zeroed */, hipStream_t s);
int ss_launch_synth_reads(const ss_synth_k_t &k, uint64_t first, uint64_t n,
                          const uint32_t *off_t, const uint32_t *off_n, uint32_t *rt,
                          uint32_t *rn, hipStream_t s);

#endif
