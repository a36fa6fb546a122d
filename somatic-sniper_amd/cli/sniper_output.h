/* sniper_output.h -- the classic / VCF / BED writers of bam-somaticsniper
 * (src/lib/sniper/output_classic.c, output_vcf.c, output_bed.c) and the
 * per-sample depth / quality statistics they print (dqstats.c:6-53),
 * computed here from packed reads (include/sniper_amd.h SS_READ_PACK). */
#ifndef SS_SNIPER_OUTPUT_H
#define SS_SNIPER_OUTPUT_H

#include <stdint.h>
#include <stdio.h>

typedef struct {
    uint32_t mean_baseQ[4], mean_mapQ[4], base_occ[4], dp4[4];
    uint32_t total_depth, total_mean_mapQ;
} ss_dqstats_t;

typedef struct {
    int genotype, joint_genotype, joint_consensus_quality, consensus_quality;
    int variant_allele_quality, somatic_score, variant_status;
    ss_dqstats_t dq;
} ss_sample_out_t;

typedef struct {
    const char *seq_name;
    uint32_t pos;
    int ref_base, ref_base4;
    ss_sample_out_t tumor, normal;
} ss_site_out_t;

typedef enum { SS_FMT_CLASSIC = 0, SS_FMT_VCF, SS_FMT_BED } ss_format_t;

/* name -> format; -1 if unknown */
int  ss_format_lookup(const char *name);
const char *ss_format_name(int i);
int  ss_format_count(void);
void ss_write_header(FILE *fh, int fmt, const char *refseq, const char *normal_id, const char *tumor_id);
void ss_write_site(FILE *fh, int fmt, const ss_site_out_t *s);
/* print_mean_quality_values / print_base_count (dqstats.c:55-87) */
void ss_put_masked(FILE *fh, int bases, const uint32_t values[4]);
void ss_dqstats_packed(const uint32_t *reads, uint32_t n, int ref_base4, uint32_t wanted, ss_dqstats_t *q);

#endif
