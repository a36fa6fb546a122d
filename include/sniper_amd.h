/*
 * sniper_amd.h -- C ABI of the MI355X-native SomaticSniper site scorer.
 *
 * This is the drop-in boundary for the reference's per-site callback path:
 *
 *   reference                                        this ABI
 *   ---------------------------------------------------------------------------
 *   bam_sspileup_f / glf_somatic(tid,pos,n1,n2,      ss_score_batch_device()/
 *     pl1,pl2,data,fh)  somatic_sniper.h:42,56;       ss_score_batch_host():
 *     somatic_sniper.c:109 (one call per site,        one call per BATCH of
 *     invoked from sniper_pileup.c:256-258)           sites, results in input order
 *   sniper_maqcns_init/prepare/destroy                ss_ctx_create()/ss_ctx_destroy()
 *     sniper_maqcns.h:23-25, sniper_maqcns.c:102-125  (tables built on the host,
 *     + qAddTableInit/makeSoloPrior/make_joint_prior   uploaded once per device)
 *     somatic_sniper.c:29-77,101-107, main.c:115-127
 *   sniper_maqcns_glfgen + sniper_maqcns_call         ss_out_t.glf / ss_call_t.cns_*
 *     sniper_maqcns.h:26-29                           (optional per-site glf1 export)
 *   pu_data2_t option fields somatic_sniper.h:21-40,  ss_params_t
 *     sniper_maqcns_t fields sniper_maqcns.h:13-21
 *
 * Everything is plain C: pointers + sizes, no C++ or torch types.  Functions
 * return 0 on success or a negative SS_E* code; the library never exits or
 * aborts (the reference exit()s from deep inside, somatic_sniper/main.c).
 *
 * One context per (device, host thread); contexts are independent, so genome
 * shards can be scored concurrently on several GPUs with no communication.
 */
#ifndef SNIPER_AMD_H
#define SNIPER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SS_ABI_VERSION 1

/* ---- error codes ------------------------------------------------------- */
#define SS_OK            0
#define SS_E_INVAL      -1   /* bad argument / malformed batch               */
#define SS_E_HIP        -2   /* a HIP runtime call failed                     */
#define SS_E_NOMEM      -3   /* host or device allocation failed             */
#define SS_E_TABLES     -4   /* host tables differ from the pinned reference,
                                or the device copy no longer matches them     */
#define SS_E_CAPACITY   -5   /* emitted-call buffer overflowed (n_calls > cap)*/
#define SS_E_NODEV      -6   /* no HIP device / device index out of range     */
#define SS_E_CORRUPT    -7   /* debug build: a device buffer's guard band was
                                overwritten (make -C somatic-sniper_amd debug) */

/* ---- packed pileup read ---------------------------------------------------
 * One u32 per NON-DELETED pileup read (bam_pileup1_t with is_del==0 and the
 * read not BAM_FUNMAP; sniper_maqcns.c:144-147).  Deleted reads are dropped on
 * the host; a site whose packed depth is 0 in either sample scores -1 exactly
 * like glf_somatic's depth gate (somatic_sniper.c:127).
 *   bits  0.. 7  mapping quality  (bam1_t.core.qual)
 *   bits  8..15  base quality     (bam1_qual(b)[qpos])
 *   bits 16..19  read base, nt16  (bam1_seqi(bam1_seq(b), qpos); 0 is '=')
 *   bit  20      strand           (bam1_strand(b): BAM_FREVERSE set)
 */
#define SS_READ_PACK(mapq, baseq, nt16, strand)                                  \
    ((uint32_t)((mapq) & 0xffu) | ((uint32_t)((baseq) & 0xffu) << 8) |          \
     ((uint32_t)((nt16) & 0xfu) << 16) | ((uint32_t)((strand) & 1u) << 20))
#define SS_READ_MAPQ(r)   ((r) & 0xffu)
#define SS_READ_BASEQ(r)  (((r) >> 8) & 0xffu)
#define SS_READ_NT16(r)   (((r) >> 16) & 0xfu)
#define SS_READ_STRAND(r) (((r) >> 20) & 1u)

/* ---- model + caller parameters (CLI flags of main.c:70-99) --------------- */
typedef struct ss_params {
    float  theta;             /* -T  maq theta            (default 0.85)  */
    int    n_hap;             /* -N  haplotypes           (default 2)     */
    float  het_rate;          /* -r  het prior            (default 0.001) */
    float  eta;               /*     maq eta, not a flag  (0.03)          */
    int    cap_mapQ;          /*     rms mapQ cap         (60)            */
    int    min_somatic_qual;  /* -Q                       (15)            */
    int    use_priors;        /* !-p                      (1)             */
    int    use_joint_priors;  /* -J (or -s)               (0)             */
    double somatic_rate;      /* -s                       (0.01)          */
    int    include_loh;       /* !-L                      (1)             */
    int    include_gor;       /* !-G                      (1)             */
} ss_params_t;

/* ---- a batch of sites (SoA, CSR reads) ------------------------------------
 * Site i has reference char ref[i] (raw FASTA byte, case kept,
 * somatic_sniper.c:117), tumor reads reads_tumor[off_tumor[i] .. off_tumor[i+1])
 * and normal reads reads_normal[off_normal[i] .. off_normal[i+1]).
 * For ss_score_batch_device every pointer is a device pointer; for
 * ss_score_batch_host every pointer is a host pointer. */
typedef struct ss_batch {
    uint64_t        n_sites;
    const uint8_t  *ref;            /* [n_sites]   */
    const uint32_t *off_tumor;      /* [n_sites+1] */
    const uint32_t *off_normal;     /* [n_sites+1] */
    const uint32_t *reads_tumor;    /* [off_tumor[n_sites]]  packed reads */
    const uint32_t *reads_normal;   /* [off_normal[n_sites]] packed reads */
} ss_batch_t;

/* Per-sample genotype likelihood record, field-for-field glf1_t
 * (samtools-0.1.6/glf.h:4-9) widened to plain bytes. */
typedef struct ss_glf {
    uint8_t  ref_base;     /* nt16 ref base                             */
    uint8_t  max_mapQ;     /* rms mapQ (sniper_maqcns.c:176)            */
    uint8_t  lk[10];       /* AA AC AG AT CC CG CT GG GT TT             */
    uint8_t  min_lk;
    uint8_t  pad;
    uint32_t depth;        /* non-deleted depth, capped at 2^24-1       */
} ss_glf_t;                /* 20 bytes */

/* Variant status codes, allele_util.h:14-20. */
#define SS_WILDTYPE 0
#define SS_GERMLINE 1
#define SS_SOMATIC  2
#define SS_LOH      3
#define SS_UNKNOWN  4

/* One EMITTED site (passes -Q / -L / -G, somatic_sniper.c:225-227): every
 * value sniper_output_t needs except dqstats, which the host computes from its
 * own copy of the reads (only ~1e-4 of sites get here). */
typedef struct ss_call {
    uint32_t site;             /* index in the batch                         */
    int32_t  somatic_score;    /* qPosteriorSum (SSC)                        */
    uint32_t cns_tumor;        /* sniper_glf2cns word, tumor                 */
    uint32_t cns_normal;       /* sniper_glf2cns word, normal                */
    int16_t  joint_cq;         /* joint_consensus_quality (255 if not -J)    */
    uint8_t  snp_q_tumor;      /* tumor variant_allele_quality               */
    uint8_t  snp_q_normal;     /* normal variant_allele_quality              */
    uint8_t  joint_gt_tumor;   /* glfBase[argmin] nt16, 0 if not -J          */
    uint8_t  joint_gt_normal;
    uint8_t  status_tumor;     /* SS_* code                                  */
    uint8_t  status_normal;
    uint8_t  ref_base4;        /* nt16 of the ref char                       */
    uint8_t  flags;            /* SS_CALL_* bits                             */
    uint16_t pad;
} ss_call_t;                   /* 28 bytes */

#define SS_CALL_QADD_CLAMPED 0x01  /* a qAdd index left [0,1024): reference UB */

/* Outputs.  score[i] is exactly glf_somatic's return value for site i:
 *   -1  skipped (ref 'N', or zero non-deleted depth in either sample)
 *   255 scored but not a SNV candidate
 *   else qPosteriorSum of the candidate (emitted or not).
 * calls/n_calls: emitted sites, compacted, in ARBITRARY order on the device
 * path (sort by .site); ss_score_batch_host returns them sorted. */
typedef struct ss_out {
    int32_t   *score;       /* [n_sites], required                          */
    ss_call_t *calls;       /* [calls_cap] or NULL                          */
    uint32_t   calls_cap;
    uint32_t  *n_calls;     /* one counter; zeroed by the call              */
    ss_glf_t  *glf;         /* [n_sites][2] (tumor, normal) or NULL         */
    uint32_t  *n_qadd_clamped; /* optional counter of clamped qAdd indices  */
} ss_out_t;

typedef struct ss_ctx ss_ctx_t;

/* ---- API ------------------------------------------------------------------ */
int         ss_abi_version(void);
const char *ss_strerror(int code);
void        ss_params_default(ss_params_t *p);

/* Build the model tables on the host (bit-exact with sniper_cal_coef /
 * sniper_cal_het, qAddTableInit, makeSoloPrior, make_joint_prior), verify the
 * default-parameter tables against the pinned reference hashes, upload them to
 * HIP device `device`.  The context binds to that device. */
int  ss_ctx_create(const ss_params_t *p, int device, ss_ctx_t **out);
void ss_ctx_destroy(ss_ctx_t *ctx);

/* Score a device-resident batch, asynchronously on `stream` (a hipStream_t,
 * NULL = default stream).  All batch/out pointers are device pointers.
 * Launches of one context share its work lists, so they run one after the
 * other: a launch on another stream than the previous one (or the host path's
 * own stream) first waits for the previous launch on the device.  Use one
 * context per stream for concurrent batches.  No depth limit: sites of any
 * depth are scored.  A batch with more sites than any before it on this
 * context grows the context's work lists first (a new device block; the
 * outgrown one is kept until ss_ctx_destroy): no call here synchronizes the
 * host with the device. */
int  ss_score_batch_device(ss_ctx_t *ctx, const ss_batch_t *batch,
                           const ss_out_t *out, void *stream);

/* Wait for the context's outstanding work and report sticky device-side
 * errors: SS_E_INVAL if a batch had malformed read offsets (a site whose
 * offsets decrease or pass off[n_sites]: it scores -2 and no read is loaded
 * for it).  Clears the sticky bits.  Also re-verifies the context's device
 * tables against the host's (a fingerprint kernel; SS_E_TABLES if they no
 * longer match, as ss_ctx_create checks after the upload), and in the debug
 * build the guard bands around every device buffer (SS_E_CORRUPT).
 * ss_score_batch_host runs this after every batch. */
int  ss_ctx_check(ss_ctx_t *ctx);

/* Score a host batch: stages through pinned buffers, H2D, kernel, D2H, sorts
 * the emitted calls by site.  out->score / calls / glf are host pointers,
 * out->n_calls a host u32.  Synchronous.  Input arrays that live in memory
 * from ss_host_alloc are copied to the device straight from there (no
 * staging copy). */
int  ss_score_batch_host(ss_ctx_t *ctx, const ss_batch_t *batch, const ss_out_t *out);

/* Page-locked host memory for batch arrays (callers that build batches in
 * place, e.g. the CLI's pileup loop); NULL on failure.  No context needed. */
void *ss_host_alloc(size_t bytes);
void  ss_host_free(void *p);

/* Host table inspection (for parity tests): FNV-1a-64 over the raw
 * little-endian doubles of fk[256], coef[64*256*256], lhet[256*256]; q_r. */
int  ss_table_hashes(const ss_ctx_t *ctx, uint64_t *fk, uint64_t *coef,
                     uint64_t *lhet, float *q_r);
/* Build the host tables for `p` without touching a GPU and report their hashes
 * (hashes[0..2] = fk, coef, lhet) and q_r.  The tables are built with this
 * host's libm / x87 exactly as the reference builds them on this host (they are
 * CPU-dependent in the reference too, see DESIGN.md "Tables").
 * ss_model_pinned: 1 if hashes equal a recorded run of the compiled reference.
 * With SS_STRICT_TABLES=1 in the environment, unpinned default tables make
 * ss_model_check / ss_ctx_create fail with SS_E_TABLES. */
int  ss_model_check(const ss_params_t *p, uint64_t hashes[3], float *q_r);
int  ss_model_pinned(const uint64_t hashes[3]);
/* Where the calling thread's latest table set came from: the fk / coef / lhet
 * tables (sniper_maqcns.c:27-100, 0.6 s of x87 work) are built once per
 * process and table parameters, and kept in a disk cache keyed by those
 * parameters and the machine (SS_TABLE_CACHE=<dir>, default
 * ~/.cache/sniper_amd; SS_TABLE_CACHE=off disables it).  A cached blob is
 * verified against its recorded hashes before use.  -1 before any build. */
#define SS_TABLES_BUILT   0
#define SS_TABLES_PROCESS 1
#define SS_TABLES_DISK    2
int  ss_model_last_source(void);
/* Copy of the host tables (for tests): any pointer may be NULL. */
int  ss_table_copy(const ss_ctx_t *ctx, double *fk, double *coef, double *lhet,
                   int *qadd1024, int *prior160, int *jprior1600);

/* ---- deterministic synthetic pileups (bench + parity inputs) -------------
 * Counter-based: every value is a pure function of (seed, shard, site, read),
 * computed by the same integer code on the host and on the device. */
typedef struct ss_synth {
    uint64_t seed;
    uint32_t shard;
    double   lambda_tumor, lambda_normal;  /* Poisson depth means            */
    int      fixed_depth;                  /* 1: depth == lambda exactly     */
    double   p_error;       /* base-call error rate            (0.01)        */
    double   p_nbase;       /* read base N rate                (0.001)       */
    double   p_eq;          /* read base '=' rate              (0)           */
    double   p_iupac;       /* read base IUPAC (M,R,..) rate   (0)           */
    double   p_del;         /* deletion rate (dropped)         (0.01)        */
    double   p_mapq60;      /* P(mapQ == 60)                   (0.9)         */
    int      baseq_lo, baseq_hi;  /* baseQ ~ U[lo,hi]          (2,41)        */
    int      mapq_hi;       /* else mapQ ~ U[0,mapq_hi]        (60)          */
    double   p_wild_qual;   /* P(baseQ/mapQ drawn from U[0,255]) (0)         */
    double   p_somatic;     /* somatic site rate               (1e-4)        */
    double   vaf;           /* tumor VAF at somatic sites      (0.3)         */
    double   p_germline;    /* het germline site rate          (0)           */
    double   p_ref_n;       /* ref char 'N' rate               (0)           */
    double   p_ref_lower;   /* ref char lowercase rate         (0)           */
    double   p_ref_iupac;   /* ref char IUPAC rate             (0)           */
} ss_synth_t;

void ss_synth_default(ss_synth_t *s, double lambda_tumor, double lambda_normal);

/* Host generation.  Two calls: first with reads_* == NULL to get the read
 * counts (written to *n_reads_tumor / *n_reads_normal and the offsets), then
 * with buffers of that size.  Sites are [first_site, first_site + n_sites). */
int  ss_synth_batch_host(const ss_synth_t *s, uint64_t first_site, uint64_t n_sites,
                         uint8_t *ref, uint32_t *off_tumor, uint32_t *off_normal,
                         uint32_t *reads_tumor, uint32_t *reads_normal,
                         uint64_t *n_reads_tumor, uint64_t *n_reads_normal);

/* Device generation into caller-provided device buffers (same bytes as the host
 * generator).  Pass 1 (reads_* NULL) writes ref + offsets and the two totals
 * (host u64s); pass 2 fills the reads.  Synchronous. */
int  ss_synth_batch_device(ss_ctx_t *ctx, const ss_synth_t *s, uint64_t first_site,
                           uint64_t n_sites, uint8_t *ref, uint32_t *off_tumor,
                           uint32_t *off_normal, uint32_t *reads_tumor,
                           uint32_t *reads_normal, uint64_t *n_reads_tumor,
                           uint64_t *n_reads_normal);

/* HIP-event timing of the scoring kernels, recorded on the stream each
 * ss_score_batch_device launch uses.  Enabling clears the log; every launch
 * while enabled appends one set of events (up to 4096 launches).
 * ss_last_kernel_ms: duration of the latest launch (synchronizes on it), -1 if
 * none.  ss_kernel_time_log: durations of all logged launches in ms (waits for
 * them), returns how many were written to ms[0..cap). */
int    ss_set_kernel_timing(ss_ctx_t *ctx, int enable);
double ss_last_kernel_ms(ss_ctx_t *ctx);
int    ss_kernel_time_log(ss_ctx_t *ctx, double *ms, int cap);
/* The same log for one kernel of the launch sequence: SS_KT_MAIN
 * (ss_score_main, as ss_kernel_time_log), SS_KT_WIDE (ss_score_wide),
 * SS_KT_DEEP (ss_score_deep), SS_KT_ALL (the whole launch). */
#define SS_KT_MAIN 0
#define SS_KT_WIDE 1
#define SS_KT_DEEP 2
#define SS_KT_ALL  3
int    ss_kernel_time_log_k(ss_ctx_t *ctx, int kernel, double *ms, int cap);

#ifdef __cplusplus
}
#endif
#endif /* SNIPER_AMD_H */
