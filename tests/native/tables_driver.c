/* tables_driver.c -- host-only driver of the library's threaded C parts for
 * the sanitizer builds (make -C somatic-sniper_amd sanitize): the table
 * builder (8 threads over the coef rows, the process-wide and disk caches)
 * and the host synthetic generator.  Test infrastructure, not shipped. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "ss_host.h"
#include "ss_synth.h"

static void *build_one(void *arg)
{
    ss_params_t p;
    uint64_t h[3];
    float qr;
    ss_params_default(&p);
    p.theta = *(float *)arg;
    return (void *)(intptr_t)ss_model_check(&p, h, &qr);
}

/* the nt16 table every context uploads (ss_capi.hip) must hold samtools'
 * bam_nt16_table (bam_import.c:23-40) at every moment, also while other
 * threads build contexts: a reader compares it against the expected bytes
 * until the builders are done (TSan sees any concurrent write) */
static unsigned char expect_nt16[256];
static int builders_done;
static long nt16_bad, nt16_reads;

static void *watch_nt16(void *arg)
{
    (void)arg;
    while (!__atomic_load_n(&builders_done, __ATOMIC_SEQ_CST)) {
        if (memcmp(ss_nt16_table, expect_nt16, 256) != 0) ++nt16_bad;
        ++nt16_reads;
    }
    return NULL;
}

int main(void)
{
    /* concurrent builds of two parameter sets and of the same one, 8 threads */
    float th[8] = {0.85f, 0.9f, 0.85f, 0.9f, 0.85f, 0.85f, 0.9f, 0.85f};
    pthread_t t[8], w;
    int i, bad = 0;
    static const char iupac[] = "=ACMGRSVTWYHKDBN";
    memset(expect_nt16, 15, sizeof expect_nt16);
    for (i = 0; i < 16; ++i) {
        const unsigned char ch = (unsigned char)iupac[i];
        expect_nt16[ch] = (unsigned char)i;
        if (ch >= 'A' && ch <= 'Z') expect_nt16[ch | 0x20] = (unsigned char)i;
    }
    for (i = 0; i < 4; ++i) expect_nt16['0' + i] = (unsigned char)(1 << i);
    pthread_create(&w, NULL, watch_nt16, NULL);
    for (i = 0; i < 8; ++i) pthread_create(&t[i], NULL, build_one, &th[i]);
    for (i = 0; i < 8; ++i) {
        void *rc;
        pthread_join(t[i], &rc);
        bad |= (int)(intptr_t)rc;
    }
    __atomic_store_n(&builders_done, 1, __ATOMIC_SEQ_CST);
    pthread_join(w, NULL);
    if (nt16_bad || memcmp(ss_nt16_table, expect_nt16, 256) != 0) {
        fprintf(stderr, "nt16 table changed under concurrent builds: %ld of %ld reads\n", nt16_bad, nt16_reads);
        bad = 1;
    }
    /* host generator, both passes */
    ss_synth_t s;
    ss_synth_default(&s, 60, 30);
    s.p_somatic = 0.01;
    const uint64_t n = 20000;
    uint8_t *ref = malloc(n);
    uint32_t *ot = malloc(4 * (n + 1)), *on = malloc(4 * (n + 1));
    uint64_t nt = 0, nn = 0;
    bad |= ss_synth_batch_host(&s, 7, n, ref, ot, on, NULL, NULL, &nt, &nn);
    uint32_t *rt = malloc(4 * nt + 4), *rn = malloc(4 * nn + 4);
    bad |= ss_synth_batch_host(&s, 7, n, ref, ot, on, rt, rn, &nt, &nn);
    uint64_t sum = 0;
    for (uint64_t k = 0; k < nt; ++k) sum += rt[k];
    printf("tables+synth ok=%d reads=%llu/%llu sum=%llu\n", bad == 0, (unsigned long long)nt,
           (unsigned long long)nn, (unsigned long long)sum);
    free(ref); free(ot); free(on); free(rt); free(rn);
    return bad != 0;
}
