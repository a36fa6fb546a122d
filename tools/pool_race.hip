/*
 * pool_race.hip -- diagnosis tool (GPU box): does device memory of a
 * "context" keep its contents while other threads of the same process create,
 * use and destroy contexts of their own?  No sniper kernel runs here: the
 * contexts are stand-ins with libsniper_amd's allocation pattern
 * (ss_capi.hip: a 34 MB table upload from pageable memory on a non-blocking
 * stream, small counters, work lists, the group kernel's 403 MB record
 * buffers, a staging area grown on first use, everything released at destroy)
 * and a fingerprint kernel that reads the table back.
 *
 *   pool_race MODE THREADS ITERS
 *     MODE  pool   hipMallocAsync / hipFreeAsync on the context's stream
 *                  (libsniper_amd before round 4's switch)
 *           malloc hipMalloc / hipFree (round 4)
 *
 * Every context checks its table twice: right after creation (its own stream
 * synchronized) and again after a random delay, just before it is destroyed.
 * A mismatch prints the region, the first differing offset and what was
 * there.  Output: one summary line per process.
 */
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#define TAB_BYTES ((size_t)34092160)        /* SS_TAB_BYTES */
#define TAB_WORDS (TAB_BYTES / 8)
#define GRP_BYTES ((size_t)256 * 12 * (131072 + 128))
#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(3);                                                                    \
        }                                                                               \
    } while (0)

static int g_pool;
static std::vector<uint64_t> g_host_tab;
static unsigned long long g_host_fp;
static std::atomic<long> g_bad_create{0}, g_bad_late{0}, g_checks{0};
static std::mutex g_print;

__host__ __device__ static inline unsigned long long mix64(unsigned long long x)
{
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__global__ void fp_kernel(const unsigned long long *w, size_t n, unsigned long long *out)
{
    unsigned long long s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += mix64(w[i] + i * 0x9e3779b97f4a7c15ull);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

static void *dalloc(size_t n, hipStream_t s)
{
    void *p = nullptr;
    if (g_pool) CHK(hipMallocAsync(&p, n, s));
    else CHK(hipMalloc(&p, n));
    return p;
}

static void dfree(void *p, hipStream_t s)
{
    if (!p) return;
    if (g_pool) CHK(hipFreeAsync(p, s));
    else { CHK(hipStreamSynchronize(s)); CHK(hipFree(p)); }
}

struct Ctx {
    hipStream_t s;
    void *tab, *cnt, *seg, *cdf, *grp, *stage;
    unsigned long long *fp;
};

static void create(Ctx &c)
{
    CHK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
    c.tab = dalloc(TAB_BYTES, c.s);
    /* the table goes up in the library's seven pieces, from pageable memory */
    const size_t cut[8] = {0, 33554432, 34078720, 34080768, 34084864, 34085504, 34091904, TAB_BYTES};
    for (int k = 0; k < 7; ++k)
        CHK(hipMemcpyAsync((char *)c.tab + cut[k], (const char *)g_host_tab.data() + cut[k], cut[k + 1] - cut[k],
                           hipMemcpyHostToDevice, c.s));
    c.cnt = dalloc(64, c.s);
    c.seg = dalloc((size_t)2 * 256 * 128 * 4 * 4, c.s);
    c.cdf = dalloc(2 * 8192 * 4, c.s);
    c.grp = dalloc(GRP_BYTES, c.s);
    c.stage = nullptr;
    c.fp = (unsigned long long *)dalloc(8, c.s);
    CHK(hipMemsetAsync(c.cnt, 0, 64, c.s));
    CHK(hipStreamSynchronize(c.s));
}

/* 0 = the table reads back intact */
static int check(Ctx &c, const char *when, int tid, int it)
{
    unsigned long long fp = 0;
    CHK(hipMemsetAsync(c.fp, 0, 8, c.s));
    hipLaunchKernelGGL(fp_kernel, dim3(1024), dim3(256), 0, c.s, (const unsigned long long *)c.tab, TAB_WORDS, c.fp);
    CHK(hipGetLastError());
    CHK(hipMemcpyAsync(&fp, c.fp, 8, hipMemcpyDeviceToHost, c.s));
    CHK(hipStreamSynchronize(c.s));
    ++g_checks;
    if (fp == g_host_fp) return 0;
    std::vector<uint64_t> back(TAB_WORDS);
    CHK(hipMemcpyAsync(back.data(), c.tab, TAB_BYTES, hipMemcpyDeviceToHost, c.s));
    CHK(hipStreamSynchronize(c.s));
    size_t first = TAB_WORDS, ndiff = 0, last = 0;
    for (size_t i = 0; i < TAB_WORDS; ++i)
        if (back[i] != g_host_tab[i]) { if (first == TAB_WORDS) first = i; last = i; ++ndiff; }
    std::lock_guard<std::mutex> g(g_print);
    fprintf(stdout, "MISMATCH %s thread %d iter %d tab %p words differ %zu first byte %zu last byte %zu "
                    "(device %016llx host %016llx)\n", when, tid, it, c.tab, ndiff, first * 8, last * 8 + 7,
            first < TAB_WORDS ? (unsigned long long)back[first] : 0ull,
            first < TAB_WORDS ? (unsigned long long)g_host_tab[first] : 0ull);
    fflush(stdout);
    return 1;
}

static void use(Ctx &c, std::mt19937_64 &rng)
{
    /* the host path's staging area, allocated on first use, then a copy in and out */
    const size_t n = ((size_t)1 << 20) + (rng() % (8u << 20));
    c.stage = dalloc(n, c.s);
    std::vector<char> h(n, 7);
    CHK(hipMemcpyAsync(c.stage, h.data(), n, hipMemcpyHostToDevice, c.s));
    CHK(hipMemcpyAsync(h.data(), c.stage, n, hipMemcpyDeviceToHost, c.s));
    CHK(hipStreamSynchronize(c.s));
}

static void destroy(Ctx &c)
{
    CHK(hipStreamSynchronize(c.s));
    void *ps[] = {c.tab, c.cnt, c.seg, c.cdf, c.grp, c.stage, c.fp};
    for (void *p : ps) dfree(p, c.s);
    CHK(hipStreamSynchronize(c.s));
    CHK(hipStreamDestroy(c.s));
}

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: pool_race pool|malloc THREADS ITERS\n"); return 2; }
    g_pool = !strcmp(argv[1], "pool");
    const int T = atoi(argv[2]), iters = atoi(argv[3]);
    g_host_tab.resize(TAB_WORDS);
    std::mt19937_64 r0(12345);
    for (auto &w : g_host_tab) w = r0();
    g_host_fp = 0;
    for (size_t i = 0; i < TAB_WORDS; ++i) g_host_fp += mix64(g_host_tab[i] + i * 0x9e3779b97f4a7c15ull);
    CHK(hipSetDevice(0));
    CHK(hipFree(nullptr));
    std::vector<std::thread> th;
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < T; ++t)
        th.emplace_back([t, iters]() {
            CHK(hipSetDevice(0));
            std::mt19937_64 rng(1000 + t);
            for (int it = 0; it < iters; ++it) {
                Ctx c;
                create(c);
                if (check(c, "after-create", t, it)) ++g_bad_create;
                std::this_thread::sleep_for(std::chrono::microseconds(rng() % 20000));
                use(c, rng);
                std::this_thread::sleep_for(std::chrono::microseconds(rng() % 5000));
                if (check(c, "before-destroy", t, it)) ++g_bad_late;
                destroy(c);
            }
        });
    for (auto &x : th) x.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("mode %s threads %d iters %d contexts %d checks %ld bad_after_create %ld bad_before_destroy %ld (%.1f s)\n",
           argv[1], T, iters, T * iters, g_checks.load(), g_bad_create.load(), g_bad_late.load(), s);
    return (g_bad_create || g_bad_late) ? 1 : 0;
}
