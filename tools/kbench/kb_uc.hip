// kb_uc.hip -- random 4-byte gathers from a 64 MB table (the C3 margin's
// cold weights) by allocation kind: ordinary device memory (cached in L2
// and the Infinity Cache, 128-byte lines), uncached device memory
// (hipDeviceMallocUncached), and fine-grained memory; plain and
// non-temporal loads.  Whether a cold gather costs a full line is what
// bounds the C3 margin (profiles/r02_kbench_ta.txt: ~60 G lines/s).
//   hipcc --offload-arch=gfx950 -O3 -o kb_uc kb_uc.hip && ./kb_uc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ unsigned mix(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_gather(const float *__restrict__ tab, unsigned nmask, int iters, float *out) {
    const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.0f;
    for (int it = 0; it < iters; ++it) {
        float g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned a = (mix(tid * 2654435761u + (unsigned)(it * 8 + u) * 40503u) >> 3) & nmask;
            g[u] = NT ? __builtin_nontemporal_load(tab + a) : tab[a];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += g[u];
    }
    out[tid] = acc;
}

int main() {
    const size_t n = (size_t)1 << 24;  // 64 MB
    const int grid = 256 * 16, iters = 16;
    const double lanes = (double)grid * 256 * iters * 8;
    float *out;
    CK(hipMalloc(&out, (size_t)grid * 256 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Kind {
        const char *name;
        unsigned flags;  // 0: hipMalloc
    } kinds[] = {{"hipMalloc (coarse, cached)", 0},
                 {"hipDeviceMallocUncached", hipDeviceMallocUncached},
                 {"hipDeviceMallocFinegrained", hipDeviceMallocFinegrained}};
    for (auto &k : kinds) {
        float *tab = nullptr;
        if (k.flags == 0)
            CK(hipMalloc(&tab, n * 4));
        else if (hipExtMallocWithFlags((void **)&tab, n * 4, k.flags) != hipSuccess) {
            printf("%-28s: allocation refused\n", k.name);
            continue;
        }
        CK(hipMemset(tab, 0, n * 4));
        CK(hipDeviceSynchronize());
        for (int nt = 0; nt < 2; ++nt) {
            float best = 1e30f;
            for (int r = 0; r < 6; ++r) {
                CK(hipEventRecord(a));
                if (nt)
                    hipLaunchKernelGGL(k_gather<true>, dim3(grid), dim3(256), 0, 0, tab, (unsigned)(n - 1), iters, out);
                else
                    hipLaunchKernelGGL(k_gather<false>, dim3(grid), dim3(256), 0, 0, tab, (unsigned)(n - 1), iters, out);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (r > 0 && ms < best) best = ms;
            }
            printf("%-28s %s loads: %.3f ms, %.1f G gathers/s\n", k.name, nt ? "nt   " : "plain", best,
                   lanes / (best * 1e-3) / 1e9);
        }
        CK(hipFree(tab));
    }
    // table-size sweep (cached, plain loads): where the random-gather rate
    // falls from the L2 rate to the ~58 G/s plateau
    float *big;
    const size_t nbig = (size_t)1 << 28;  // 1 GiB
    CK(hipMalloc(&big, nbig * 4));
    CK(hipMemset(big, 0, nbig * 4));
    for (size_t mb = 1; mb <= 1024; mb *= 2) {
        const unsigned mask = (unsigned)(mb * 1024 * 1024 / 4 - 1);
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_gather<false>, dim3(grid), dim3(256), 0, 0, big, mask, iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r > 0 && ms < best) best = ms;
        }
        printf("table %5zu MB: %.3f ms, %.1f G gathers/s\n", mb, best, lanes / (best * 1e-3) / 1e9);
    }
    return 0;
}
