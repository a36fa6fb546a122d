/* sniper_output.c -- see sniper_output.h.  Field order, separators and
 * number formats follow the reference writers byte for byte. */
#include "sniper_output.h"

#include <string.h>
#include <time.h>

#include "sniper_amd.h"

static const char NT16_CHARS[] = "=ACMGRSVTWYHKDBN";   /* bam_nt16_rev_table */

static const char *FORMAT_NAMES[] = {"classic", "vcf", "bed"};

int ss_format_lookup(const char *name)
{
    for (int i = 0; i < 3; ++i)
        if (strcmp(name, FORMAT_NAMES[i]) == 0) return i;
    return -1;
}
const char *ss_format_name(int i) { return i >= 0 && i < 3 ? FORMAT_NAMES[i] : NULL; }
int ss_format_count(void) { return 3; }

void ss_dqstats_packed(const uint32_t *r, uint32_t n, int ref_base4, uint32_t wanted, ss_dqstats_t *q)
{
    memset(q, 0, sizeof *q);
    for (uint32_t i = 0; i < n; ++i) {
        const int base = (int)SS_READ_NT16(r[i]);
        const uint32_t mq = SS_READ_MAPQ(r[i]), bq = SS_READ_BASEQ(r[i]);
        q->total_depth++;
        q->total_mean_mapQ += mq;
        q->dp4[(base == ref_base4 ? 0 : 2) + SS_READ_STRAND(r[i])]++;
        for (int j = 0; j < 4; ++j) {
            const int bit = 1 << j;
            if ((base & bit) != base) continue;          /* '=' counts for every base, N for none */
            q->base_occ[j]++;
            if (bit & wanted) { q->mean_baseQ[j] += bq; q->mean_mapQ[j] += mq; }
        }
    }
    for (int j = 0; j < 4; ++j)
        if (q->base_occ[j]) {
            q->mean_baseQ[j] = (uint32_t)(q->mean_baseQ[j] / (double)q->base_occ[j] + .499);
            q->mean_mapQ[j] = (uint32_t)(q->mean_mapQ[j] / (double)q->base_occ[j] + .499);
        }
    if (q->total_depth) q->total_mean_mapQ = (uint32_t)(q->total_mean_mapQ / (double)q->total_depth + .499);
}

/* comma list of values[i] for the bases in `bases`, "0" when none
 * (print_mean_quality_values / print_base_count, dqstats.c:55-87) */
void ss_put_masked(FILE *fh, int bases, const uint32_t v[4])
{
    int any = 0;
    for (int i = 0; i < 4; ++i)
        if (bases & (1 << i)) {
            if (any) fputc(',', fh);
            fprintf(fh, "%d", v[i]);
            any = 1;
        }
    if (!any) fputc('0', fh);
}

static void write_classic(FILE *fh, const ss_site_out_t *s)
{
    const ss_sample_out_t *t = &s->tumor, *n = &s->normal;
    fprintf(fh, "%s\t%d\t%c\t%c\t%c\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t", s->seq_name, s->pos + 1,
            s->ref_base, NT16_CHARS[t->genotype], NT16_CHARS[n->genotype], t->somatic_score,
            t->consensus_quality, t->variant_allele_quality, t->dq.total_mean_mapQ, n->consensus_quality,
            n->variant_allele_quality, n->dq.total_mean_mapQ, t->dq.total_depth, n->dq.total_depth);
    const ss_sample_out_t *smp[2] = {t, n};
    for (int k = 0; k < 2; ++k) {
        const ss_sample_out_t *x = smp[k];
        const int alt = ~s->ref_base4 & x->genotype;
        ss_put_masked(fh, s->ref_base4, x->dq.mean_baseQ);
        fputc('\t', fh);
        ss_put_masked(fh, s->ref_base4, x->dq.mean_mapQ);
        fputc('\t', fh);
        ss_put_masked(fh, s->ref_base4, x->dq.base_occ);
        fputc('\t', fh);
        ss_put_masked(fh, alt, x->dq.mean_baseQ);
        fputc('\t', fh);
        ss_put_masked(fh, alt, x->dq.mean_mapQ);
        fputc('\t', fh);
        ss_put_masked(fh, alt, x->dq.base_occ);
        fputc(k == 0 ? '\t' : '\n', fh);
    }
}

static void write_bed(FILE *fh, const ss_site_out_t *s)
{
    fprintf(fh, "%s\t%d\t%d\t%c/%c\t%d\t%d\n", s->seq_name, s->pos, s->pos + 1, s->ref_base,
            NT16_CHARS[s->tumor.genotype], s->tumor.somatic_score, s->tumor.dq.total_depth);
}

static int popcount4(int a) { return (a & 1) + (a >> 1 & 1) + (a >> 2 & 1) + (a >> 3 & 1); }

/* VCF genotype of `gt` against the ref bit and the site's ALT bit set */
static void vcf_gt(FILE *fh, uint32_t ref4, uint32_t alts, uint32_t gt)
{
    const int na = popcount4((int)gt);
    int printed = 0;
    if (gt & ref4) {
        if (na == 1) { fputs("0/0", fh); return; }
        fputc('0', fh);
        printed = 1;
    }
    gt &= ~ref4;
    uint32_t idx = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t bit = 1u << i;
        if (alts & bit) ++idx;
        if (!(gt & bit)) continue;
        if (na == 1) { fprintf(fh, "%u/%u", idx, idx); return; }
        if (printed) fputc('/', fh);
        fprintf(fh, "%u", idx);
        ++printed;
    }
}

static void vcf_int4(FILE *fh, const uint32_t v[4], uint32_t mask)
{
    int c = 0;
    for (int i = 0; i < 4; ++i)
        if (mask & (1u << i)) {
            if (c++) fputc(',', fh);
            fprintf(fh, "%d", v[i]);
        }
}

static void vcf_sample(FILE *fh, int ref4, int alts, const ss_sample_out_t *x)
{
    vcf_gt(fh, (uint32_t)ref4, (uint32_t)alts, (uint32_t)(x->joint_genotype ? x->joint_genotype : x->genotype));
    fputc(':', fh);
    vcf_gt(fh, (uint32_t)ref4, (uint32_t)alts, (uint32_t)x->genotype);
    fprintf(fh, ":%d:%d,%d,%d,%d:%d,%d,%d,%d:%d:", x->dq.total_depth, x->dq.dp4[0], x->dq.dp4[1], x->dq.dp4[2],
            x->dq.dp4[3], x->dq.base_occ[0], x->dq.base_occ[1], x->dq.base_occ[2], x->dq.base_occ[3],
            x->consensus_quality);
    if (x->joint_genotype) fprintf(fh, "%d:", x->joint_consensus_quality);
    else fputs(".:", fh);
    fprintf(fh, "%d:", x->variant_allele_quality);
    vcf_int4(fh, x->dq.mean_baseQ, (uint32_t)x->genotype);
    fputc(':', fh);
    fprintf(fh, "%d:", x->dq.total_mean_mapQ);
    vcf_int4(fh, x->dq.mean_mapQ, (uint32_t)x->genotype);
    fputc(':', fh);
    fprintf(fh, "%d:", x->variant_status);
    if (x->somatic_score >= 0) fprintf(fh, "%d", x->somatic_score);
    else fputc('.', fh);
}

static void write_vcf(FILE *fh, const ss_site_out_t *s)
{
    const int alts = (s->tumor.genotype | s->normal.genotype) & ~s->ref_base4;
    fprintf(fh, "%s\t%d\t.\t%c\t", s->seq_name, s->pos + 1, s->ref_base);
    int n_alt = 0;
    for (int i = 0; i < 4; ++i)
        if (alts & (1 << i)) {
            if (n_alt++) fputc(',', fh);
            fputc(NT16_CHARS[1 << i], fh);
        }
    if (!n_alt) fputc('.', fh);
    fputs("\t.\t.\t.\tGT:IGT:DP:DP4:BCOUNT:GQ:JGQ:VAQ:BQ:MQ:AMQ:SS:SSC\t", fh);
    vcf_sample(fh, s->ref_base4, alts, &s->normal);
    fputc('\t', fh);
    vcf_sample(fh, s->ref_base4, alts, &s->tumor);
    fputc('\n', fh);
}

void ss_write_site(FILE *fh, int fmt, const ss_site_out_t *s)
{
    if (fmt == SS_FMT_VCF) write_vcf(fh, s);
    else if (fmt == SS_FMT_BED) write_bed(fh, s);
    else write_classic(fh, s);
    fflush(fh);
}

static const char *VCF_FIELDS[][4] = {
    {"GT", "1", "String", "Genotype"},
    {"IGT", "1", "String", "Genotype when called independently (only filled if called in joint prior mode)"},
    {"DP", "1", "Integer", "Total read depth"},
    {"DP4", "4", "Integer", "# high-quality ref-forward bases, ref-reverse, alt-forward and alt-reverse bases"},
    {"BCOUNT", "4", "Integer", "Occurrence count for each base at this site (A,C,G,T)"},
    {"GQ", "1", "Integer", "Genotype quality"},
    {"JGQ", "1", "Integer", "Joint genotype quality (only filled if called in join prior mode)"},
    {"VAQ", "1", "Integer", "Variant allele quality"},
    {"BQ", ".", "Integer", "Average base quality"},
    {"MQ", "1", "Integer", "Average mapping quality across all reads"},
    {"AMQ", ".", "Integer", "Average mapping quality for each allele present in the genotype"},
    {"SS", "1", "Integer", "Variant status relative to non-adjacent Normal, 0=wildtype,1=germline,2=somatic,3=LOH,4=unknown"},
    {"SSC", "1", "Integer", "Somatic Score"},
};

void ss_write_header(FILE *fh, int fmt, const char *refseq, const char *normal_id, const char *tumor_id)
{
    if (fmt == SS_FMT_BED) {
        fputs("#CHROM\tSTART\tSTOP\tREF/ALT\tSOMATIC_SCORE\tTUMOR_DEPTH\n", fh);
    } else if (fmt == SS_FMT_VCF) {
        char date[64];
        const time_t now = time(NULL);
        strftime(date, sizeof date, "%Y%m%d", localtime(&now));
        fprintf(fh, "##fileformat=VCFv4.1\n##fileDate=%s\n##phasing=none\n##reference=file://%s\n", date, refseq);
        for (size_t i = 0; i < sizeof VCF_FIELDS / sizeof VCF_FIELDS[0]; ++i)
            fprintf(fh, "##FORMAT=<ID=%s,Number=%s,Type=%s,Description=\"%s\">\n", VCF_FIELDS[i][0],
                    VCF_FIELDS[i][1], VCF_FIELDS[i][2], VCF_FIELDS[i][3]);
        fprintf(fh, "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t%s\t%s\n", normal_id, tumor_id);
    }
}
