// Round 6 probe: what does one returning same-address atomic per wave cost
// when every wave of a short kernel appends to one list (the triage kernels'
// list appends at 500x)?  Variants: 0 = the atomic append, 1 = a fixed slot
// per wave (no atomic), 2 = the atomic on one of 64 counters (spread).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(512) void append(const uint32_t *off, uint32_t *cnt, uint32_t *lst, uint32_t nblocks,
                                              int variant)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t nwaves = gridDim.x * 8u;
    for (uint32_t blk = blockIdx.x * 8u + wv; blk < nblocks; blk += nwaves) {
        const uint32_t s = blk * 64u + lane;
        const uint32_t breads = off[blk * 64u + 64u] - off[blk * 64u];
        const bool need = breads > 64u * 128u;
        const uint64_t m = __ballot(need);
        if (!m) continue;
        const uint32_t first = (uint32_t)__builtin_ctzll(m);
        uint32_t base = 0;
        if (variant == 1) {
            base = blk * 64u;
        } else {
            uint32_t *c = variant == 2 ? cnt + 16u * (blk & 63u) : cnt;
            if (lane == first) base = atomicAdd(c, (uint32_t)__popcll(m));
            base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)first);
            if (variant == 2) base = (blk & 63u) * (nblocks * 64u / 64u) + base % (nblocks);
        }
        if (need) lst[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = s;
    }
}

int main()
{
    const uint32_t sizes[] = {4096, 16384, 65536, 262144};
    for (uint32_t nb : sizes) {
        const uint32_t n = nb * 64u;
        uint32_t *off, *cnt, *lst;
        hipMalloc(&off, (size_t)(n + 1) * 4);
        hipMalloc(&cnt, 64 * 16 * 4);
        hipMalloc(&lst, (size_t)n * 4 * 2);
        uint32_t *h = (uint32_t *)malloc((size_t)(n + 1) * 4);
        for (uint32_t i = 0; i <= n; ++i) h[i] = i * 1000u;
        hipMemcpy(off, h, (size_t)(n + 1) * 4, hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int v = 0; v < 3; ++v) {
            const int grid = (int)((nb + 7) / 8 < 256 * 64 ? (nb + 7) / 8 : 256 * 64);
            float best = 1e9f;
            for (int it = 0; it < 6; ++it) {
                hipMemset(cnt, 0, 64 * 16 * 4);
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(append, dim3(grid), dim3(512), 0, 0, off, cnt, lst, nb, v);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (it && ms < best) best = ms;
            }
            printf("blocks %u variant %d: %.4f ms (%.2f ns per block)\n", nb, v, best, best * 1e6 / nb);
        }
        hipFree(off);
        hipFree(cnt);
        hipFree(lst);
        free(h);
    }
    return 0;
}
