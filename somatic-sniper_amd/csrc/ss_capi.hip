/*
 * ss_capi.hip -- the C ABI (include/sniper_amd.h): contexts, table upload,
 * batch launches, host-buffer convenience path, device synthetic generator.
 *
 * Memory layout in HBM per context (DESIGN.md "Data layout"):
 *   model   coef 32 MiB + lhet 512 KiB + fk 2 KiB + qadd/prior/jprior/nt16 12 KiB
 *           (read-only, stays resident in L2/MALL after the first batches)
 *   lists   deep site lists + counters (sized from the batch)
 *   host-path staging buffers, grown on demand
 *
 * Contexts are independent (include/sniper_amd.h): nothing here waits for
 * the whole device.  A context waits only for its own work -- its `done`
 * event (the latest launch, whatever stream it went to) and its own stream
 * -- for its launches and copies.  Device memory comes from hipMalloc through
 * a per-device cache of idle blocks (dev_alloc below): nothing is handed back
 * to HIP (hipFree waits for the whole device) while another context of the
 * process lives on that device.  Page-locked staging memory is malloc'd and
 * registered (hipHostRegister / hipHostUnregister) instead of hipHostMalloc /
 * hipHostFree, whose free would wait for the whole device.
 *
 * Every context verifies its device tables after the upload and in each
 * ss_ctx_check (a fingerprint kernel against the host's sums), so tables that
 * stop holding what was uploaded are reported (SS_E_TABLES), never scored.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "sniper_amd.h"
#include "ss_host.h"
#include "ss_kernels.h"
#include "ss_synth.h"

#define SS_EV_PER_LAUNCH 4   /* before main, after main, after wide, after deep */

struct dev_blk;

struct ss_ctx {
    int device;
    int n_cu;
    ss_host_model_t hm;
    /* model on the device */
    uint8_t *d_tab;           /* all tables, SS_TAB_* layout (ss_kernels.h) */
    /* work lists */
    uint32_t *d_counters;     /* [2] err (sticky), [3] scratch n_calls, [4] the deep triage list's count,
                                 [5] deep2 count, [6..7] listed
                                 entries | segments << 32, [8] the group kernel's chunk counter,
                                 [9] the deep kernel's chunk counter, [10] deep3 count,
                                 [11] the triage list's count,
                                 [12..15] the device generator's read totals (2 x u64),
                                 [16..21] the table fingerprint (3 x u64) */
    uint32_t *d_deep_list;
    uint32_t deep_cap;
    uint32_t *d_deep_seg;     /* listed segments' first entries, then their main-wave ids */
    uint8_t *d_grp_rec;       /* the group kernel's per-wave fold-record buffers */
    uint32_t grp_wgs;         /* group-kernel workgroups d_grp_rec holds buffers for */
    /* timing: a pool of events, SS_EV_PER_LAUNCH per launch while enabled */
    int timing;
    std::vector<hipEvent_t> *ev;
    int n_logged;
    hipStream_t last_stream;
    hipEvent_t done;          /* recorded after every launch: the next launch on another stream waits */
    int launched;
    /* host path */
    hipStream_t hstream;
    void *h_stage;  size_t h_stage_sz;     /* pinned */
    void *d_stage;  size_t d_stage_sz;
    /* synth */
    uint32_t *d_cdf;                        /* [2][SS_SYNTH_MAXCDF] */
    void *d_scan_tmp; size_t scan_tmp_sz;
    uint32_t *d_depth_tmp; size_t depth_tmp_n;
    /* device memory (dev_alloc): blocks in use, blocks outgrown but possibly still read */
    std::vector<dev_blk> *blocks, *retired;
    uint64_t fp_expect[3];    /* host fingerprint of the uploaded tables: coef, lhet, the rest */
    float near_esr[2052];     /* SS_TAB_ESR (near_tables) */
    float near_cmin[260];     /* SS_TAB_CMIN */
    int fast_ok;              /* SS_MF_FAST */
    int counted;              /* included in g_live */
};

#define SS_NCOUNTERS 32

#define HIPCHK(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return SS_E_HIP;     \
    } while (0)

extern "C" int ss_abi_version(void) { return SS_ABI_VERSION; }

extern "C" const char *ss_strerror(int code)
{
    switch (code) {
    case SS_OK: return "ok";
    case SS_E_INVAL: return "invalid argument or malformed batch";
    case SS_E_HIP: return "HIP runtime error";
    case SS_E_NOMEM: return "out of memory";
    case SS_E_TABLES: return "model tables differ from the reference (libm mismatch), or the device copy no longer matches the host's";
    case SS_E_CAPACITY: return "capacity exceeded (emitted calls, work lists or pileup depth)";
    case SS_E_NODEV: return "no usable HIP device";
    case SS_E_CORRUPT: return "device memory outside a buffer was overwritten (debug guard bands)";
    default: return "unknown error";
    }
}

/* ---- device memory ---------------------------------------------------------
 * Blocks come from hipMalloc and go back to HIP (hipFree, which waits for the
 * whole device) only when the last context of the process on their device is
 * destroyed.  Until then a block a context no longer needs -- a work list or
 * staging area it outgrew, or everything it held at ss_ctx_destroy -- goes to
 * a per-device cache of idle blocks that later allocations of any context
 * reuse.  So neither a scoring call nor one context's teardown waits for
 * another context's kernels (test_contexts_do_not_wait_for_each_other).
 *
 * A block enters the idle cache only when the device is done with it: at
 * ss_ctx_destroy after the context's own work has completed (ctx_quiesce);
 * a staging area after its stream was synchronized; a work list that grew
 * while launches may still read it stays on the context's retired list until
 * ss_ctx_destroy.
 *
 * Round 4 took device memory from the stream-ordered pool (hipMallocAsync /
 * hipFreeAsync); contexts created while other contexts of the process were
 * being destroyed then lost batches in the CLI's contig-group mode (4 of 25
 * runs).  The cause is NOT established: a standalone
 * stand-in without our kernels (tools/pool_race.hip) did not reproduce it in
 * 160 contexts, and a host wait after every hipMallocAsync (0 of 40 bad) fits
 * a cross-context release inside the runtime's pool and a stream-ordering gap
 * on our side equally well.  This allocator avoids both: no pool, and no
 * block is reused before the device is done with it.
 *
 * Debug build (make debug, -DSS_DEBUG_CANARY): every block carries guard bands
 * of SS_GUARD bytes before and after it, filled with 0xA5 at allocation and
 * checked by ss_ctx_check and ss_ctx_destroy (SS_E_CORRUPT on a difference). */
#ifdef SS_DEBUG_CANARY
#define SS_GUARD ((size_t)4096)
#else
#define SS_GUARD ((size_t)0)
#endif

struct dev_blk {
    void *base;       /* hipMalloc'd address; the user pointer is base + SS_GUARD */
    size_t bytes;     /* usable bytes */
    int device;
};

static std::mutex g_mem_mu;
static std::vector<dev_blk> g_idle;          /* blocks no context uses, any device */
static std::vector<int> g_live;              /* live contexts per device */

static inline void *blk_user(const dev_blk &b) { return (char *)b.base + SS_GUARD; }

static int guards_fill(const dev_blk &b, hipStream_t s)
{
#ifdef SS_DEBUG_CANARY
    if (hipMemsetAsync(b.base, 0xA5, SS_GUARD, s) != hipSuccess ||
        hipMemsetAsync((char *)blk_user(b) + b.bytes, 0xA5, SS_GUARD, s) != hipSuccess)
        return SS_E_HIP;
#else
    (void)b; (void)s;
#endif
    return SS_OK;
}

/* a block of >= bytes on c's device: an idle one of at most twice the size,
 * else a new hipMalloc.  Recorded in c->blocks. */
static int dev_alloc(ss_ctx_t *c, void **p, size_t bytes, hipStream_t s)
{
    const size_t need = (std::max<size_t>(bytes, 16) + 255) & ~(size_t)255;
    dev_blk b = {nullptr, 0, c->device};
    *p = nullptr;
    {
        std::lock_guard<std::mutex> g(g_mem_mu);
        size_t best = g_idle.size();
        for (size_t i = 0; i < g_idle.size(); ++i) {
            const dev_blk &x = g_idle[i];
            if (x.device == c->device && x.bytes >= need && x.bytes / 2 <= need &&
                (best == g_idle.size() || x.bytes < g_idle[best].bytes))
                best = i;
        }
        if (best < g_idle.size()) {
            b = g_idle[best];
            g_idle[best] = g_idle.back();
            g_idle.pop_back();
        }
    }
    if (!b.base) {
        if (hipSetDevice(c->device) != hipSuccess) return SS_E_HIP;
        if (hipMalloc(&b.base, need + 2 * SS_GUARD) != hipSuccess) {
            (void)hipGetLastError();
            return SS_E_NOMEM;
        }
        b.bytes = need;
    }
    c->blocks->push_back(b);
    *p = blk_user(b);
    return guards_fill(b, s);
}

/* p is no longer used by c; `idle_now`: the device is done with it (else it
 * stays on c's retired list until ss_ctx_destroy) */
static void dev_release(ss_ctx_t *c, void *&p, bool idle_now)
{
    if (!p) return;
    auto &v = *c->blocks;
    for (size_t i = 0; i < v.size(); ++i)
        if (blk_user(v[i]) == p) {
            const dev_blk b = v[i];
            v[i] = v.back();
            v.pop_back();
            if (idle_now) {
                std::lock_guard<std::mutex> g(g_mem_mu);
                g_idle.push_back(b);
            } else {
                c->retired->push_back(b);
            }
            break;
        }
    p = nullptr;
}

/* debug build: SS_E_CORRUPT if a guard band of one of c's blocks changed */
static int guards_check(ss_ctx_t *c)
{
#ifdef SS_DEBUG_CANARY
    std::vector<unsigned char> h(2 * SS_GUARD);
    for (auto *list : {c->blocks, c->retired})
        for (const dev_blk &b : *list) {
            if (hipMemcpyAsync(h.data(), b.base, SS_GUARD, hipMemcpyDeviceToHost, c->hstream) != hipSuccess ||
                hipMemcpyAsync(h.data() + SS_GUARD, (char *)blk_user(b) + b.bytes, SS_GUARD, hipMemcpyDeviceToHost,
                               c->hstream) != hipSuccess ||
                hipStreamSynchronize(c->hstream) != hipSuccess)
                return SS_E_HIP;
            for (size_t i = 0; i < h.size(); ++i)
                if (h[i] != 0xA5) {
                    fprintf(stderr, "[sniper_amd] guard band of device block %p (%zu bytes) overwritten at %s%zu\n",
                            blk_user(b), b.bytes, i < SS_GUARD ? "-" : "+",
                            i < SS_GUARD ? SS_GUARD - i : i - SS_GUARD);
                    return SS_E_CORRUPT;
                }
        }
#else
    (void)c;
#endif
    return SS_OK;
}

/* page-locked host memory without hipHostMalloc / hipHostFree (the free
 * synchronizes the device) */
static void *pinned_alloc(size_t bytes)
{
    void *p = nullptr;
    if (posix_memalign(&p, 4096, bytes ? bytes : 1) != 0) return nullptr;
    if (hipHostRegister(p, bytes ? bytes : 1, hipHostRegisterDefault) != hipSuccess) {
        free(p);
        return nullptr;
    }
    return p;
}

static void pinned_free(void *&p)
{
    if (p) {
        hipHostUnregister(p);
        free(p);
    }
    p = nullptr;
}

/* wait for this context's own work only: its latest launch and its stream */
static void ctx_quiesce(ss_ctx_t *c)
{
    if (c->launched && c->done) hipEventSynchronize(c->done);
    if (c->hstream) hipStreamSynchronize(c->hstream);
}

/* float(x) rounded towards -inf */
static float round_down_f(double x)
{
    float f = (float)x;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}

/* The bounds of the early exit (ss_kernels.hip tri_block / trd_block,
 * DESIGN.md 4.0): for a sample whose reference-base group has c of its
 * contributing reads at minq >= 24, and tot contributing reads in all (after
 * the rescale of sniper_maqcns.c:178-182, so tot <= 256),
 *   esr[c]    <= esum[ref]:  24 (m[0] + .. + m[c - 1]) (1 - 2e-4), m[k] = min(fk[0 .. k]);
 *   cmin[tot] <= lh + coef[q << 16 | tot << 8 | k] over q in [4, 63], k in [1, tot]
 *                (the reference's index, OR and all: tot = 256 aliases into
 *                the next q row's n = 0 entries, :195) and lh = -4.343 lhet[..]
 *                (min with 0), less 0.01,
 * so every genotype without the reference base has p >= esr[c] + cmin[tot]
 * (its e sums esum[ref] and other non-negative esums, :184-210).
 * The k-th q >= 24 read of the reference group's walk weighs fk[w] with w <= k
 * (w counts per strand), so its weight is >= m[k] whatever the shape of fk:
 * fk[n] = theta^n (1 - eta) + eta (:72) decreases for theta < 1 but increases
 * for the theta > 1 that -T accepts (main.c:83 has no range check), and then
 * m[k] = fk[0] (w saturates at 255: fk[min(k, 255)]).  The 2e-4 margin covers
 * the float accumulation of esum (<= SS_NEAR_MAXN roundings of 2^-24
 * relative each: 1.2e-4), the 0.01 the float rounding of p; both tables
 * round down.  Enabled only with q_r >= 1 and finite tables. */
static int near_tables(const ss_host_model_t &hm, float esr[2052], float cmin[260])
{
    for (int i = 0; i < 2052; ++i) esr[i] = 0.0f;
    for (int i = 0; i < 260; ++i) cmin[i] = -1e30f;
    if (hm.q_r_int < 1) return 0;
    double F = 0.0, run_min = hm.fk[0];
    for (int k = 0; k < (int)SS_NEAR_MAXN; ++k) {
        run_min = std::min(run_min, hm.fk[k < 255 ? k : 255]);
        F += run_min;
        esr[k + 1] = round_down_f(24.0 * F * (1.0 - 2e-4));
    }
    double lh = 0.0;
    for (int i = 0; i < 65536; ++i) {
        const double v = -4.343 * hm.lhet[i];
        if (!std::isfinite(v)) return 0;
        lh = std::min(lh, v);
    }
    for (int n = 1; n <= 256; ++n) {
        double cm = 1e300;
        for (int q = 4; q < 64; ++q)
            for (int k = 1; k <= n; ++k) {
                const size_t idx = (size_t)q << 16 | (size_t)n << 8 | (size_t)k;
                const double v = hm.coef[idx];
                if (!std::isfinite(v)) return 0;
                cm = std::min(cm, v);
            }
        cmin[n] = round_down_f(cm + lh - 0.01);
    }
    return std::isfinite(F) ? 1 : 0;
}

/* queue the fingerprint of the context's device tables (ss_tab_fingerprint)
 * on the context's stream, after whatever it should check, and its copy to
 * `dst` (3 words; page-locked, so the copy stays asynchronous) */
static int tables_fp_enqueue(ss_ctx_t *c, unsigned long long *dst)
{
    hipStream_t hs = c->hstream;
    unsigned long long *dfp = reinterpret_cast<unsigned long long *>(c->d_counters + 16);
    HIPCHK(hipMemsetAsync(dfp, 0, 3 * sizeof(unsigned long long), hs));
    if (ss_launch_tab_fingerprint(c->d_tab, dfp, hs) != 0) return SS_E_HIP;
    HIPCHK(hipMemcpyAsync(dst, dfp, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, hs));
    return SS_OK;
}

/* compare a completed fingerprint with the host's sums */
static int tables_compare(const ss_ctx_t *c, const unsigned long long fp[3])
{
    if (fp[0] == c->fp_expect[0] && fp[1] == c->fp_expect[1] && fp[2] == c->fp_expect[2]) return SS_OK;
    fprintf(stderr, "[sniper_amd] device %d: the context's device tables no longer match the host's (%s%s%s differ)\n",
            c->device, fp[0] != c->fp_expect[0] ? "coef " : "", fp[1] != c->fp_expect[1] ? "lhet " : "",
            fp[2] != c->fp_expect[2] ? "fk/qAdd/prior/nt16/bounds" : "");
    return SS_E_TABLES;
}

/* fingerprint the context's device tables and compare with the host's sums;
 * the caller's stream order puts this after the upload / the launches it
 * wants checked.  Synchronizes the context's stream. */
static int tables_verify(ss_ctx_t *c)
{
    unsigned long long fp[3] = {0, 0, 0};
    if (int rc = tables_fp_enqueue(c, fp)) return rc;
    HIPCHK(hipStreamSynchronize(c->hstream));
    return tables_compare(c, fp);
}

extern "C" void ss_ctx_destroy(ss_ctx_t *c)
{
    if (!c) return;
    hipSetDevice(c->device);
    ctx_quiesce(c);
    if (c->blocks && c->hstream && guards_check(c) != SS_OK)
        fprintf(stderr, "[sniper_amd] ss_ctx_destroy: device memory corrupted (see above)\n");
    /* the context's work has completed: its blocks are idle now */
    std::vector<dev_blk> trim;
    if (c->blocks) {
        std::lock_guard<std::mutex> g(g_mem_mu);
        for (auto *list : {c->blocks, c->retired})
            for (const dev_blk &b : *list) g_idle.push_back(b);
        if ((size_t)c->device < g_live.size() && c->counted && --g_live[c->device] == 0) {
            /* the process's last context on this device: hand its idle blocks back to HIP */
            for (size_t i = 0; i < g_idle.size();)
                if (g_idle[i].device == c->device) {
                    trim.push_back(g_idle[i]);
                    g_idle[i] = g_idle.back();
                    g_idle.pop_back();
                } else {
                    ++i;
                }
        }
    }
    for (const dev_blk &b : trim) hipFree(b.base);
    delete c->blocks;
    delete c->retired;
    pinned_free(c->h_stage);
    if (c->ev) {
        for (hipEvent_t e : *c->ev) hipEventDestroy(e);
        delete c->ev;
    }
    if (c->hstream) hipStreamDestroy(c->hstream);
    if (c->done) hipEventDestroy(c->done);
    ss_host_model_free(&c->hm);
    free(c);
}

extern "C" int ss_ctx_create(const ss_params_t *p, int device, ss_ctx_t **out)
{
    int ndev = 0, rc;
    if (!p || !out) return SS_E_INVAL;
    *out = nullptr;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SS_E_NODEV;
    if (device < 0 || device >= ndev) return SS_E_NODEV;
    ss_ctx_t *c = (ss_ctx_t *)calloc(1, sizeof(ss_ctx_t));
    if (!c) return SS_E_NOMEM;
    c->device = device;
    c->ev = new std::vector<hipEvent_t>();
    c->blocks = new std::vector<dev_blk>();
    c->retired = new std::vector<dev_blk>();
    {
        std::lock_guard<std::mutex> g(g_mem_mu);
        if (g_live.size() < (size_t)ndev) g_live.resize(ndev, 0);
        ++g_live[device];
        c->counted = 1;
    }
    if ((rc = ss_host_model_build(p, &c->hm)) != SS_OK) { ss_ctx_destroy(c); return rc; }
    if (hipSetDevice(device) != hipSuccess) { ss_ctx_destroy(c); return SS_E_HIP; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { ss_ctx_destroy(c); return SS_E_HIP; }
    c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
        ss_ctx_destroy(c);
        return SS_E_HIP;
    }
    hipStream_t hs = c->hstream;
    c->fast_ok = near_tables(c->hm, c->near_esr, c->near_cmin);
#define TRY(x) do { if ((rc = (x)) != SS_OK) { ss_ctx_destroy(c); return rc; } } while (0)
    TRY(dev_alloc(c, (void **)&c->d_tab, SS_TAB_BYTES, hs));
    {
        struct { size_t off; const void *src; size_t n; } parts[] = {
            {SS_TAB_COEF, c->hm.coef, ((size_t)64 << 16) * sizeof(double)},
            {SS_TAB_LHET, c->hm.lhet, (size_t)65536 * sizeof(double)},
            {SS_TAB_FK, c->hm.fk, 256 * sizeof(double)},
            {SS_TAB_QADD, c->hm.qadd, 1024 * sizeof(int32_t)},
            {SS_TAB_PRIOR, c->hm.prior, 160 * sizeof(int32_t)},
            {SS_TAB_JPRIOR, c->hm.jprior, 1600 * sizeof(int32_t)},
            {SS_TAB_NT16, ss_nt16_table, 256},
            {SS_TAB_ESR, c->near_esr, 2052 * sizeof(float)},
            {SS_TAB_CMIN, c->near_cmin, 260 * sizeof(float)},
        };
        for (auto &pt : parts)
            if (hipMemcpyAsync(c->d_tab + pt.off, pt.src, pt.n, hipMemcpyHostToDevice, hs) != hipSuccess) {
                ss_ctx_destroy(c);
                return SS_E_HIP;
            }
        /* the host's fingerprint of the same image: coef and lhet from the
         * process-wide table entry, the rest assembled here */
        static_assert(SS_TAB_COEF / 8 == SS_FP_COEF_WORD && SS_TAB_LHET / 8 == SS_FP_LHET_WORD, "fingerprint layout");
        std::vector<uint8_t> rest(SS_TAB_BYTES - SS_TAB_FK);
        for (auto &pt : parts)
            if (pt.off >= SS_TAB_FK) memcpy(rest.data() + (pt.off - SS_TAB_FK), pt.src, pt.n);
        c->fp_expect[0] = c->hm.fp_coef;
        c->fp_expect[1] = c->hm.fp_lhet;
        c->fp_expect[2] = ss_tab_fp_words(rest.data(), rest.size() / 8, SS_TAB_FK / 8);
        /* `rest` is pageable and local: the copies above read other buffers */
    }
    TRY(dev_alloc(c, (void **)&c->d_counters, SS_NCOUNTERS * sizeof(uint32_t), hs));
    TRY(dev_alloc(c, (void **)&c->d_deep_seg, 2 * (size_t)c->n_cu * SS_MAIN_GRID_PER_CU * (SS_MAIN_BLOCK / 64) * sizeof(uint32_t), hs));
    TRY(dev_alloc(c, (void **)&c->d_cdf, 2 * SS_SYNTH_MAXCDF * sizeof(uint32_t), hs));
#undef TRY
    /* the tables, lists and counters are complete before any launch can use
     * them, and the tables read back as uploaded */
    if (hipMemsetAsync(c->d_counters, 0, SS_NCOUNTERS * sizeof(uint32_t), hs) != hipSuccess) {
        ss_ctx_destroy(c);
        return SS_E_HIP;
    }
    if ((rc = tables_verify(c)) != SS_OK || (rc = guards_check(c)) != SS_OK) {
        ss_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return SS_OK;
}

extern "C" int ss_table_hashes(const ss_ctx_t *c, uint64_t *fk, uint64_t *coef, uint64_t *lhet,
                               float *q_r)
{
    if (!c) return SS_E_INVAL;
    if (fk) *fk = c->hm.h_fk;
    if (coef) *coef = c->hm.h_coef;
    if (lhet) *lhet = c->hm.h_lhet;
    if (q_r) *q_r = c->hm.q_r;
    return SS_OK;
}

extern "C" int ss_table_copy(const ss_ctx_t *c, double *fk, double *coef, double *lhet,
                             int *qadd, int *prior, int *jprior)
{
    if (!c) return SS_E_INVAL;
    if (fk) memcpy(fk, c->hm.fk, sizeof(c->hm.fk));
    if (coef) memcpy(coef, c->hm.coef, ((size_t)64 << 16) * sizeof(double));
    if (lhet) memcpy(lhet, c->hm.lhet, 65536 * sizeof(double));
    if (qadd) memcpy(qadd, c->hm.qadd, sizeof(c->hm.qadd));
    if (prior) memcpy(prior, c->hm.prior, sizeof(c->hm.prior));
    if (jprior) memcpy(jprior, c->hm.jprior, sizeof(c->hm.jprior));
    return SS_OK;
}

/* the deep list buffer holds five lists of deep_cap entries: the main
 * kernel's per-wave segments (deep), the group kernel's overflow (deep2), the
 * deep kernel's (deep3), the triage kernels' undecided sites (tri) and the
 * triage kernel's sites of deeper blocks (dtri).
 * Grown for a batch larger than any before (by at least half, so a run of
 * growing batches allocates O(log) times); the old list may still be read by
 * the context's previous launch, so it is retired, not reused, until
 * ss_ctx_destroy.  No host or device synchronization. */
static int ensure_deep_cap(ss_ctx_t *c, uint64_t n_sites, hipStream_t s)
{
    if (n_sites <= c->deep_cap) return SS_OK;
    uint64_t cap = std::max<uint64_t>(n_sites, 1u << 16);
    if (c->deep_cap) cap = std::max<uint64_t>(cap, (uint64_t)c->deep_cap + c->deep_cap / 2);
    cap = std::min<uint64_t>(cap, 0xffffffffull);
    if (cap < n_sites) return SS_E_INVAL;
    dev_release(c, *(void **)&c->d_deep_list, false);
    c->deep_cap = 0;
    if (int rc = dev_alloc(c, (void **)&c->d_deep_list, 6 * cap * sizeof(uint32_t), s)) return rc;
    c->deep_cap = (uint32_t)cap;
    return SS_OK;
}

/* The group kernel's fold-record buffers (SS_GRP_REC_BYTES per wave) for a
 * grid of `wgs` workgroups, allocated on first need and grown like the work
 * lists: by at least half each time, up to the full grid of n_cu workgroups
 * (the old buffers are retired, not reused, until ss_ctx_destroy, so a run of
 * slowly growing batches retires O(log n_cu) buffers, not one per batch).  A
 * context that only ever scores small batches holds a few MB, not the 403 MB
 * of a full grid. */
static int ensure_grp_cap(ss_ctx_t *c, uint32_t wgs, hipStream_t s)
{
    if (wgs <= c->grp_wgs) return SS_OK;
    uint32_t want = std::max(wgs, c->grp_wgs + c->grp_wgs / 2);
    want = std::max(std::min(want, (uint32_t)std::max(c->n_cu, 1)), wgs);
    dev_release(c, *(void **)&c->d_grp_rec, false);
    c->grp_wgs = 0;
    if (int rc = dev_alloc(c, (void **)&c->d_grp_rec, (size_t)want * (SS_WIDE_BLOCK / 64) * SS_GRP_REC_BYTES, s))
        return rc;
    c->grp_wgs = want;
    return SS_OK;
}

extern "C" int ss_score_batch_device(ss_ctx_t *c, const ss_batch_t *b, const ss_out_t *o, void *stream)
{
    if (!c || !b || !o || !o->score) return SS_E_INVAL;
    if (b->n_sites == 0) return SS_OK;
    if (b->n_sites >= 0xffffffffull) return SS_E_INVAL;
    if (!b->ref || !b->off_tumor || !b->off_normal || !b->reads_tumor || !b->reads_normal)
        return SS_E_INVAL;
    if (o->calls && !o->n_calls) return SS_E_INVAL;
    HIPCHK(hipSetDevice(c->device));
    /* main kernel: 4 waves per workgroup, one 64-site block per wave per
     * iteration (lane = site), grid-strided; 3 workgroups are resident per CU
     * (166 VGPRs -> 3 waves per SIMD; 52.5 KB of LDS each).
     * Each wave owns a deep-list segment as long as the most blocks it can
     * visit, times 64 sites. */
    const uint64_t site_blocks = (b->n_sites + SS_MAIN_SITES - 1) / SS_MAIN_SITES;
    const uint64_t wpb = SS_MAIN_BLOCK / 64;              /* waves per workgroup */
    uint64_t blocks = (site_blocks + wpb - 1) / wpb;
    const uint64_t max_blocks = (uint64_t)c->n_cu * SS_MAIN_GRID_PER_CU;
    if (blocks > max_blocks) blocks = max_blocks;
    const uint64_t nseg = blocks * (SS_MAIN_BLOCK / 64);
    const uint64_t seg_cap = (site_blocks + nseg - 1) / nseg * SS_MAIN_SITES;
    hipStream_t s = (hipStream_t)stream;
    /* one launch at a time per context (shared work lists and counters) */
    if (c->launched && s != c->last_stream) HIPCHK(hipStreamWaitEvent(s, c->done, 0));
    int rc = ensure_deep_cap(c, nseg * seg_cap, s);
    if (rc) return rc;
    /* group kernel: one 12-wave workgroup per CU, or fewer when the batch
     * could not give every wave a chunk (GB = 32 listed sites per chunk) */
    const uint64_t grp_chunks_max = (b->n_sites + 31u) / 32u;
    const uint64_t wg_need = (grp_chunks_max + SS_WIDE_BLOCK / 64 - 1) / (SS_WIDE_BLOCK / 64);
    const int wide_grid = (int)std::min<uint64_t>((uint64_t)c->n_cu, wg_need);
    if ((rc = ensure_grp_cap(c, (uint32_t)wide_grid, s))) return rc;
    /* counters: deep2, listed segments and entries, the group and deep
     * kernels' next chunks, deep3, the triage list (err is sticky until
     * ss_ctx_check) */
    HIPCHK(hipMemsetAsync(c->d_counters + 4, 0, 9 * sizeof(uint32_t), s));
    if (o->n_calls) HIPCHK(hipMemsetAsync(o->n_calls, 0, sizeof(uint32_t), s));
    ss_score_args a;
    memset(&a, 0, sizeof(a));
    a.n_sites = b->n_sites;
    a.ref = b->ref;
    a.off_t = b->off_tumor;
    a.off_n = b->off_normal;
    a.reads_t = b->reads_tumor;
    a.reads_n = b->reads_normal;
    a.score = o->score;
    a.calls = o->calls;
    a.calls_cap = o->calls ? o->calls_cap : 0;
    a.n_calls = o->n_calls ? o->n_calls : c->d_counters + 3;
    a.glf = o->glf;
    a.n_clamped = o->n_qadd_clamped;
    a.deep_list = c->d_deep_list;
    a.deep_off = c->d_deep_seg;
    a.deep_segs = c->d_deep_seg + (size_t)c->n_cu * SS_MAIN_GRID_PER_CU * (SS_MAIN_BLOCK / 64);
    a.deep_seg_cap = (uint32_t)seg_cap;
    a.deep_nseg = (uint32_t)nseg;
    a.deep_cap = c->deep_cap;
    a.deep2_list = c->d_deep_list + c->deep_cap;
    a.deep2_count = c->d_counters + 5;
    a.deep_next = c->d_counters + 9;
    a.deep3_list = c->d_deep_list + 2 * (size_t)c->deep_cap;
    a.deep3_count = c->d_counters + 10;
    a.deep_acc = reinterpret_cast<unsigned long long *>(c->d_counters + 6);   /* 8-byte aligned */
    a.wide_next = c->d_counters + 8;
    a.grp_rec = c->d_grp_rec;
    /* the triage kernel's early exit writes no glf records and needs the
     * host's bound tables (near_tables) */
    const bool triage = o->glf == nullptr && c->fast_ok;
    a.tri_list = triage ? c->d_deep_list + 3 * (size_t)c->deep_cap : nullptr;
    a.tri_count = c->d_counters + 11;
    a.dtri_list = c->d_deep_list + 4 * (size_t)c->deep_cap;
    a.dtri_count = c->d_counters + 4;
    a.dsite_list = c->d_deep_list + 5 * (size_t)c->deep_cap;
    a.dsite_count = c->d_counters + 12;
    a.err = c->d_counters + 2;
    a.m.tab = c->d_tab;
    a.m.q_r_int = c->hm.q_r_int;
    {   /* only min(mapQ & 0x7f, cap) is ever used (sniper_maqcns.c:173) */
        const int cap = c->hm.prm.cap_mapQ;
        a.m.cap_mapQ = cap < 0 ? 0 : (cap > 127 ? 127 : cap);
    }
    a.m.min_somatic_qual = c->hm.prm.min_somatic_qual;
    a.m.flags = (c->hm.prm.use_joint_priors ? SS_MF_JOINT : 0u) | (c->hm.prm.include_loh ? SS_MF_LOH : 0u) |
                (c->hm.prm.include_gor ? SS_MF_GOR : 0u) | (c->fast_ok ? SS_MF_FAST : 0u);
    const int deep_grid = c->n_cu;                  /* one 8-wave block per CU: LDS */
    const int wild_grid = c->n_cu * 3;              /* 3 blocks (12 one-site waves) per CU: LDS */
    c->last_stream = s;
    const hipEvent_t *evs = nullptr;
    if (c->timing && c->n_logged < 4096) {
        while ((int)c->ev->size() < SS_EV_PER_LAUNCH * (c->n_logged + 1)) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return SS_E_HIP;
            c->ev->push_back(e);
        }
        evs = c->ev->data() + SS_EV_PER_LAUNCH * c->n_logged;
        ++c->n_logged;
    }
    /* triage: 8 waves per workgroup, grid-strided over the 64-site blocks */
    const uint64_t tri_wpb = SS_TRIAGE_BLOCK / 64;
    const int triage_grid = (int)std::min<uint64_t>((site_blocks + tri_wpb - 1) / tri_wpb,
                                                    (uint64_t)c->n_cu * SS_TRIAGE_GRID_PER_CU);
    const int triage_deep_grid = (int)std::min<uint64_t>((site_blocks + 3) / 4,
                                                         (uint64_t)c->n_cu * SS_TRIAGE_DEEP_GRID_PER_CU);
    int e = ss_launch_score(a, triage_grid, triage_deep_grid, (int)blocks, wide_grid, deep_grid, wild_grid, s, evs);
    if (e != 0) return SS_E_HIP;
    HIPCHK(hipEventRecord(c->done, s));
    c->launched = 1;
    return SS_OK;
}

extern "C" int ss_set_kernel_timing(ss_ctx_t *c, int enable)
{
    if (!c) return SS_E_INVAL;
    c->timing = enable ? 1 : 0;
    if (enable) c->n_logged = 0;
    return SS_OK;
}

/* launch i, kernel k: events k .. k+1 (k = 3: the whole launch, events 0 .. 3) */
static double pair_ms(ss_ctx_t *c, int i, int k)
{
    float ms = -1.0f;
    const hipEvent_t *ev = c->ev->data() + SS_EV_PER_LAUNCH * i;
    const hipEvent_t a = k == SS_KT_ALL ? ev[0] : ev[k], b = k == SS_KT_ALL ? ev[3] : ev[k + 1];
    if (hipEventSynchronize(b) != hipSuccess) return -1.0;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.0;
    return ms;
}

extern "C" double ss_last_kernel_ms(ss_ctx_t *c)
{
    if (!c || c->n_logged == 0) return -1.0;
    hipSetDevice(c->device);
    return pair_ms(c, c->n_logged - 1, SS_KT_MAIN);
}

extern "C" int ss_kernel_time_log_k(ss_ctx_t *c, int kernel, double *ms, int cap)
{
    int i, n;
    if (!c || (!ms && cap) || kernel < SS_KT_MAIN || kernel > SS_KT_ALL) return SS_E_INVAL;
    hipSetDevice(c->device);
    n = c->n_logged < cap ? c->n_logged : cap;
    for (i = 0; i < n; ++i) ms[i] = pair_ms(c, i, kernel);
    return n;
}

extern "C" int ss_kernel_time_log(ss_ctx_t *c, double *ms, int cap)
{
    return ss_kernel_time_log_k(c, SS_KT_MAIN, ms, cap);
}

/* waits for this context's own work (its latest launch, its stream), not
 * for other contexts' or the caller's other work on the device; then checks
 * that the device tables still hold what was uploaded (SS_E_TABLES) and, in
 * the debug build, the guard bands (SS_E_CORRUPT) */
extern "C" int ss_ctx_check(ss_ctx_t *c)
{
    uint32_t err = 0;
    int rc;
    if (!c) return SS_E_INVAL;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t hs = c->hstream;
    if (c->launched) HIPCHK(hipStreamWaitEvent(hs, c->done, 0));
    HIPCHK(hipMemcpyAsync(&err, c->d_counters + 2, sizeof(err), hipMemcpyDeviceToHost, hs));
    if ((rc = tables_verify(c)) != SS_OK) return rc;       /* synchronizes hs */
    if ((rc = guards_check(c)) != SS_OK) return rc;
    if (err) {
        HIPCHK(hipMemsetAsync(c->d_counters + 2, 0, sizeof(uint32_t), hs));
        HIPCHK(hipStreamSynchronize(hs));
        return (err & SS_KERR_MALFORMED) ? SS_E_INVAL : SS_E_CAPACITY;
    }
    return SS_OK;
}

/* test hook (not in the public header): overwrite one byte of the context's
 * device tables, so the tests can see ss_ctx_check report it */
extern "C" int ss__test_poke_table(ss_ctx_t *c, uint64_t byte_offset, int value)
{
    /* the debug build maps offsets SS_TAB_BYTES .. +15 to the first bytes of
     * the guard band after the table block */
    if (!c || byte_offset >= SS_TAB_BYTES + (SS_GUARD ? 16 : 0)) return SS_E_INVAL;
    uint8_t *dst = c->d_tab + byte_offset;
    if (byte_offset >= SS_TAB_BYTES)
        for (const dev_blk &b : *c->blocks)
            if (blk_user(b) == c->d_tab) dst = c->d_tab + b.bytes + (byte_offset - SS_TAB_BYTES);
    HIPCHK(hipSetDevice(c->device));
    if (c->launched) HIPCHK(hipStreamWaitEvent(c->hstream, c->done, 0));
    HIPCHK(hipMemsetAsync(dst, value & 0xff, 1, c->hstream));
    HIPCHK(hipStreamSynchronize(c->hstream));
    return SS_OK;
}

/* test hook (not in the public header): the latest launch's routing counts
 * -- out[0] the deep triage's blocks, out[1] the sites the triage kernels
 * left to the main kernel, out[2] the sites the main kernel queued for the
 * group kernel, out[3] for the deep kernel (its two lists) */
extern "C" int ss__test_route_counts(ss_ctx_t *c, uint32_t *out)
{
    uint32_t h[12];
    if (!c || !out) return SS_E_INVAL;
    HIPCHK(hipSetDevice(c->device));
    if (c->launched) HIPCHK(hipStreamWaitEvent(c->hstream, c->done, 0));
    HIPCHK(hipMemcpyAsync(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost, c->hstream));
    HIPCHK(hipStreamSynchronize(c->hstream));
    out[0] = h[4];
    out[1] = h[11];
    out[2] = h[6];
    out[3] = h[5] + h[10];
    return SS_OK;
}

/* ---------------------------------------------------------- host path ---- */
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

/* the host path's staging areas; the previous host call has completed (it
 * synchronizes its stream), so the old areas are free to go */
static int ensure_stage(ss_ctx_t *c, size_t bytes)
{
    if (bytes <= c->h_stage_sz && bytes <= c->d_stage_sz) return SS_OK;
    size_t sz = std::max(bytes, (size_t)1 << 20);
    sz += sz / 4;
    HIPCHK(hipStreamSynchronize(c->hstream));
    pinned_free(c->h_stage);
    c->h_stage_sz = 0;
    dev_release(c, c->d_stage, true);           /* its stream is idle: reusable now */
    c->d_stage_sz = 0;
    if (!(c->h_stage = pinned_alloc(sz))) return SS_E_NOMEM;
    c->h_stage_sz = sz;
    if (int rc = dev_alloc(c, &c->d_stage, sz, c->hstream)) return rc;
    c->d_stage_sz = sz;
    return SS_OK;
}

extern "C" void *ss_host_alloc(size_t bytes) { return pinned_alloc(bytes); }

extern "C" void ss_host_free(void *p) { pinned_free(p); }

/* is [p, p + n) page-locked host memory the device can read directly? */
/* Pageable input -> pinned staging -> device, in pieces: each piece is copied
 * into the staging area by SS_COPY_THREADS threads (default 8) and its H2D is
 * queued at once, so the DMA of one piece runs while the next is copied. */
static int copy_threads()
{
    const char *e = getenv("SS_COPY_THREADS");
    const int t = e && *e ? atoi(e) : 4;
    return t < 1 ? 1 : (t > 64 ? 64 : t);
}

static void par_memcpy(char *dst, const char *src, size_t n, int nthreads)
{
    const size_t min_share = (size_t)4 << 20;
    int t = (int)std::min<size_t>((size_t)nthreads, (n + min_share - 1) / min_share);
    if (t <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t step = ((n + t - 1) / t + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (int i = 1; i < t && (size_t)i * step < n; ++i) {
        const size_t o = (size_t)i * step;
        th.emplace_back(memcpy, dst + o, src + o, std::min(step, n - o));
    }
    memcpy(dst, src, std::min(step, n));
    for (auto &x : th) x.join();
}

static bool pinned_host(const void *p)
{
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();               /* plain pageable memory: not an error */
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

extern "C" int ss_score_batch_host(ss_ctx_t *c, const ss_batch_t *b, const ss_out_t *o)
{
    if (!c || !b || !o || !o->score) return SS_E_INVAL;
    const uint64_t n = b->n_sites;
    if (n == 0) { if (o->n_calls) *o->n_calls = 0; return SS_OK; }
    if (n >= 0xffffffffull) return SS_E_INVAL;
    const uint64_t nt = b->off_tumor[n], nn = b->off_normal[n];
    if (b->off_tumor[0] != 0 || b->off_normal[0] != 0) return SS_E_INVAL;
    const uint32_t cap = o->calls ? o->calls_cap : 0;
    /* one staging area: inputs, then outputs */
    size_t off = 0;
    const size_t o_ref = off;   off = align_up(off + n);
    const size_t o_ot = off;    off = align_up(off + 4 * (n + 1));
    const size_t o_on = off;    off = align_up(off + 4 * (n + 1));
    const size_t o_rt = off;    off = align_up(off + 4 * nt);
    const size_t o_rn = off;    off = align_up(off + 4 * nn);
    const size_t o_sc = off;    off = align_up(off + 4 * n);
    const size_t o_cnt = off;   off = align_up(off + 16);
    const size_t o_calls = off; off = align_up(off + sizeof(ss_call_t) * (size_t)cap);
    const size_t o_glf = off;   off = align_up(off + (o->glf ? sizeof(ss_glf_t) * 2 * n : 0));
    const size_t o_chk = off;   off = align_up(off + 32);     /* err word, table fingerprint */
    const size_t total = off;
    HIPCHK(hipSetDevice(c->device));
    int rc = ensure_stage(c, total);
    if (rc) return rc;
    char *h = (char *)c->h_stage, *d = (char *)c->d_stage;
    hipStream_t s = c->hstream;
    /* inputs already in page-locked memory go to the device directly; the
     * rest through the pinned staging area, one H2D for all of them */
    const struct { const void *src; size_t off, bytes; } in[5] = {
        {b->ref, o_ref, n}, {b->off_tumor, o_ot, 4 * (n + 1)}, {b->off_normal, o_on, 4 * (n + 1)},
        {b->reads_tumor, o_rt, 4 * nt}, {b->reads_normal, o_rn, 4 * nn}};
    const int nthreads = copy_threads();
    const size_t piece = (size_t)64 << 20;
    for (int k = 0; k < 5; ++k) {
        if (!in[k].bytes) continue;
        if (pinned_host(in[k].src)) {
            HIPCHK(hipMemcpyAsync(d + in[k].off, in[k].src, in[k].bytes, hipMemcpyHostToDevice, s));
            continue;
        }
        for (size_t p = 0; p < in[k].bytes; p += piece) {
            const size_t nb = std::min(piece, in[k].bytes - p);
            par_memcpy(h + in[k].off + p, (const char *)in[k].src + p, nb, nthreads);
            HIPCHK(hipMemcpyAsync(d + in[k].off + p, h + in[k].off + p, nb, hipMemcpyHostToDevice, s));
        }
    }
    ss_batch_t db = {n, (const uint8_t *)(d + o_ref), (const uint32_t *)(d + o_ot),
                     (const uint32_t *)(d + o_on), (const uint32_t *)(d + o_rt),
                     (const uint32_t *)(d + o_rn)};
    ss_out_t dout;
    memset(&dout, 0, sizeof(dout));
    dout.score = (int32_t *)(d + o_sc);
    dout.calls = cap ? (ss_call_t *)(d + o_calls) : nullptr;
    dout.calls_cap = cap;
    dout.n_calls = (uint32_t *)(d + o_cnt);
    dout.n_qadd_clamped = (uint32_t *)(d + o_cnt + 4);
    dout.glf = o->glf ? (ss_glf_t *)(d + o_glf) : nullptr;
    HIPCHK(hipMemsetAsync(d + o_cnt, 0, 16, s));
    rc = ss_score_batch_device(c, &db, &dout, s);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(h + o_sc, d + o_sc, o_chk - o_sc, hipMemcpyDeviceToHost, s));
    /* ss_ctx_check's work, queued behind the batch so that one synchronize
     * serves both: the sticky error word and the table fingerprint */
    HIPCHK(hipMemcpyAsync(h + o_chk, c->d_counters + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if ((rc = tables_fp_enqueue(c, reinterpret_cast<unsigned long long *>(h + o_chk + 8)))) return rc;
    HIPCHK(hipStreamSynchronize(s));
    {
        uint32_t err;
        unsigned long long fp[3];
        memcpy(&err, h + o_chk, sizeof err);
        memcpy(fp, h + o_chk + 8, sizeof fp);
        rc = tables_compare(c, fp);
        if (rc == SS_OK) rc = guards_check(c);
        if (rc == SS_OK && err) {
            HIPCHK(hipMemsetAsync(c->d_counters + 2, 0, sizeof(uint32_t), s));
            HIPCHK(hipStreamSynchronize(s));
            rc = (err & SS_KERR_MALFORMED) ? SS_E_INVAL : SS_E_CAPACITY;
        }
    }
    memcpy(o->score, h + o_sc, 4 * n);
    uint32_t ncalls, nclamp;
    memcpy(&ncalls, h + o_cnt, 4);
    memcpy(&nclamp, h + o_cnt + 4, 4);
    if (o->n_calls) *o->n_calls = ncalls;
    if (o->n_qadd_clamped) *o->n_qadd_clamped = nclamp;
    if (cap) {
        const uint32_t k = std::min(ncalls, cap);
        ss_call_t *calls = o->calls;
        memcpy(calls, h + o_calls, sizeof(ss_call_t) * k);
        std::sort(calls, calls + k, [](const ss_call_t &x, const ss_call_t &y) { return x.site < y.site; });
    }
    if (o->glf) memcpy(o->glf, h + o_glf, sizeof(ss_glf_t) * 2 * n);
    if (rc) return rc;
    if (o->calls && ncalls > cap) return SS_E_CAPACITY;
    return SS_OK;
}

/* ------------------------------------------------------ device synth ---- */
extern "C" int ss_synth_batch_device(ss_ctx_t *c, const ss_synth_t *s, uint64_t first,
                                     uint64_t n, uint8_t *ref, uint32_t *off_t, uint32_t *off_n,
                                     uint32_t *rt, uint32_t *rn, uint64_t *n_rt, uint64_t *n_rn)
{
    if (!c || !s || !ref || !off_t || !off_n) return SS_E_INVAL;
    if (n >= 0xffffffffull) return SS_E_INVAL;
    std::vector<uint32_t> cdf(2 * SS_SYNTH_MAXCDF);
    ss_synth_k_t k;
    int rc = ss_synth_prepare(s, &k, cdf.data(), cdf.data() + SS_SYNTH_MAXCDF);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->hstream;
    HIPCHK(hipMemcpyAsync(c->d_cdf, cdf.data(), cdf.size() * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));        /* cdf is a local vector */
    k.cdf_tumor = c->d_cdf;
    k.cdf_normal = c->d_cdf + SS_SYNTH_MAXCDF;
    if (!rt || !rn) {
        /* pass 1: depths -> exclusive scans -> offsets */
        if (c->depth_tmp_n < 2 * (n + 1)) {
            HIPCHK(hipStreamSynchronize(st));
            dev_release(c, *(void **)&c->d_depth_tmp, true);
            c->depth_tmp_n = 0;
            if (int e = dev_alloc(c, (void **)&c->d_depth_tmp, 2 * (n + 1) * 4, st)) return e;
            c->depth_tmp_n = 2 * (n + 1);
        }
        uint32_t *dt = c->d_depth_tmp, *dn = c->d_depth_tmp + (n + 1);
        /* the 64-bit read totals (counters 12..15): the offsets are 32-bit */
        unsigned long long *dsum = reinterpret_cast<unsigned long long *>(c->d_counters + 12);
        HIPCHK(hipMemsetAsync(dt, 0, 2 * (n + 1) * 4, st));
        HIPCHK(hipMemsetAsync(dsum, 0, 2 * sizeof(unsigned long long), st));
        if (ss_launch_synth_depth(k, first, n, ref, dt, dn, dsum, st)) return SS_E_HIP;
        unsigned long long sums[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(sums, dsum, sizeof(sums), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (sums[0] > 0xffffffffull || sums[1] > 0xffffffffull) {
            fprintf(stderr, "[sniper_amd] ss_synth_batch_device: %llu tumor / %llu normal reads do not fit the "
                            "batch's 32-bit offsets; use fewer sites per batch\n", sums[0], sums[1]);
            return SS_E_INVAL;
        }
        size_t need = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, dt, off_t, (int)(n + 1), st));
        if (need > c->scan_tmp_sz) {
            HIPCHK(hipStreamSynchronize(st));
            dev_release(c, c->d_scan_tmp, true);
            c->scan_tmp_sz = 0;
            if (int e = dev_alloc(c, &c->d_scan_tmp, need, st)) return e;
            c->scan_tmp_sz = need;
        }
        size_t sz = c->scan_tmp_sz;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->d_scan_tmp, sz, dt, off_t, (int)(n + 1), st));
        sz = c->scan_tmp_sz;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->d_scan_tmp, sz, dn, off_n, (int)(n + 1), st));
        uint32_t tot[2];
        HIPCHK(hipMemcpyAsync(&tot[0], off_t + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&tot[1], off_n + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (n_rt) *n_rt = tot[0];
        if (n_rn) *n_rn = tot[1];
        return SS_OK;
    }
    if (ss_launch_synth_reads(k, first, n, off_t, off_n, rt, rn, st)) return SS_E_HIP;
    HIPCHK(hipStreamSynchronize(st));
    return SS_OK;
}
