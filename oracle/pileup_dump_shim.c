/*
 * pileup_dump_shim.c -- TEST INFRASTRUCTURE (oracle/README.md): linked into
 * the reference's own bam-somaticsniper with -Wl,--wrap=glf_somatic
 * (oracle/ref.mk -> oracle/_ref/bam-somaticsniper-dump).  Before every real
 * glf_somatic call (somatic_sniper.c:109) it writes the site exactly as the
 * native CLI's SS_DUMP_PILEUP hook does (somatic-sniper_amd/cli/sniper_cli.c
 * dump_site): tid, pos, n1, n2, ref char, then the packed non-deleted mapped
 * reads (include/sniper_amd.h SS_READ_PACK) of tumor and normal in pileup
 * order.  The file is named by SS_DUMP_PILEUP.
 */
#include <stdio.h>
#include <stdlib.h>

#include "somatic_sniper.h"
#include "sniper_amd.h"

int __real_glf_somatic(uint32_t tid, uint32_t pos, int n1, int n2, const bam_pileup1_t *pl1,
                       const bam_pileup1_t *pl2, void *data, FILE *snp_fh);

static FILE *g_dump;

static void put_reads(const bam_pileup1_t *pl, int n)
{
    for (int i = 0; i < n; ++i) {
        const bam_pileup1_t *p = pl + i;
        if (p->is_del || (p->b->core.flag & BAM_FUNMAP)) continue;
        fprintf(g_dump, "%x,", SS_READ_PACK(p->b->core.qual, bam1_qual(p->b)[p->qpos],
                                            bam1_seqi(bam1_seq(p->b), p->qpos), bam1_strand(p->b) ? 1 : 0));
    }
}

int __wrap_glf_somatic(uint32_t tid, uint32_t pos, int n1, int n2, const bam_pileup1_t *pl1,
                       const bam_pileup1_t *pl2, void *data, FILE *snp_fh)
{
    pu_data2_t *d = (pu_data2_t *)data;
    if (!g_dump) {
        const char *fn = getenv("SS_DUMP_PILEUP");
        g_dump = fopen(fn ? fn : "pileup.dump", "w");
        if (!g_dump) abort();
    }
    /* the contig cache step of glf_somatic (somatic_sniper.c:112-117); the
     * real call below then finds the cache already filled */
    if (d->fai && (int)tid != d->tid) {
        free(d->ref);
        d->ref = fai_fetch(d->fai, d->h1->target_name[tid], &d->len);
        d->tid = tid;
    }
    const int rb = (d->ref && (int)pos < d->len) ? d->ref[pos] : 'N';
    fprintf(g_dump, "%u\t%u\t%d\t%d\t%d\t", tid, pos, n1, n2, rb);
    put_reads(pl1, n1);
    fputc('\t', g_dump);
    put_reads(pl2, n2);
    fputc('\n', g_dump);
    fflush(g_dump);
    return __real_glf_somatic(tid, pos, n1, n2, pl1, pl2, data, snp_fh);
}
