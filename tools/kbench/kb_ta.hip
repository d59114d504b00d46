// kb_ta.hip -- what a 4-byte gather instruction costs on gfx950 as a
// function of how many lanes are active and how many distinct addresses
// they carry (the C3 hot margin issues a global load for EVERY entry, the
// ~58% hot ones clamped to w[0]).  Each mode issues the same number of
// wave-level load instructions; time per instruction chip-wide is printed.
//   hipcc --offload-arch=gfx950 -O3 -o kb_ta kb_ta.hip && ./kb_ta
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

// mode 0: every lane a random address in [0, n)
// mode 1: lanes with (hash % 100) < hot_pct clamped to address 0 (all lanes active)
// mode 2: the same lanes exec-masked off (inactive) instead of clamped
// mode 3: every lane address 0
template <int MODE>
__global__ __launch_bounds__(256) void k_ta(const float *__restrict__ tab, unsigned nmask, int iters, int hot_pct,
                                           float *out) {
    const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.0f;
    for (int it = 0; it < iters; ++it) {
        float g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned h = mix(tid * 2654435761u + (unsigned)(it * 8 + u) * 40503u);
            const bool hot = (h % 100u) < (unsigned)hot_pct;
            unsigned a = (h >> 7) & nmask;
            if (MODE == 1 && hot) a = 0;
            if (MODE == 3) a = 0;
            if (MODE == 2) {
                g[u] = 0.0f;
                if (!hot) g[u] = tab[a];
            } else {
                g[u] = tab[a];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += g[u];
    }
    out[tid] = acc;
}

template <int MODE>
double run(const float *tab, unsigned nmask, int iters, int hot, float *out, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_ta<MODE>, dim3(grid), dim3(256), 0, 0, tab, nmask, iters, hot, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_ta<MODE>, dim3(grid), dim3(256), 0, 0, tab, nmask, iters, hot, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5.0;
}

int mall_main();

int main(int argc, char **argv) {
    if (argc > 1 && argv[1][0] == 'm') return mall_main();
    const size_t n = (size_t)1 << 24;  // 64 MB table (C3's weights)
    float *tab, *out;
    CK(hipMalloc(&tab, n * 4));
    CK(hipMemset(tab, 0, n * 4));
    const int grid = 256 * 16;  // 16 waves x 4 per CU... 4,096 workgroups of 4 waves
    CK(hipMalloc(&out, (size_t)grid * 256 * 4));
    const int iters = 64;
    const double instr = (double)grid * 4 * iters * 8;  // wave-level load instructions
    struct {
        const char *name;
        unsigned mask;
    } tabs[] = {{"64 MB table", (unsigned)(n - 1)}, {"64 KB table", (1u << 14) - 1}};
    for (auto &t : tabs) {
        for (int hot : {0, 58}) {
            const double m0 = run<0>(tab, t.mask, iters, hot, out, grid);
            const double m1 = run<1>(tab, t.mask, iters, hot, out, grid);
            const double m2 = run<2>(tab, t.mask, iters, hot, out, grid);
            const double m3 = run<3>(tab, t.mask, iters, hot, out, grid);
            printf("%s hot%%=%d: all-random %.3f ms (%.1f ns/instr chip, %.1f G lanes/s) | clamped %.3f ms | "
                   "masked %.3f ms | all-same %.3f ms\n",
                   t.name, hot, m0, m0 * 1e6 / instr, instr * 64 / m0 / 1e6, m1, m2, m3);
        }
    }
    CK(hipFree(tab));
    CK(hipFree(out));
    return 0;
}

// ---- MALL residency of a gathered table behind a stream (run with "mall")
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream(const v4i *__restrict__ p, size_t n4, int nt, int *out) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const v4i v = nt ? __builtin_nontemporal_load(p + i) : p[i];
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x7fffffff) out[0] = acc;
}

int mall_main() {
    const size_t n = (size_t)1 << 24;  // 64 MB table
    const size_t sbytes = (size_t)2 << 30;  // 2 GiB stream
    float *tab, *out;
    v4i *st;
    CK(hipMalloc(&tab, n * 4));
    CK(hipMemset(tab, 0, n * 4));
    CK(hipMalloc(&st, sbytes));
    CK(hipMemset(st, 1, sbytes));
    const int grid = 256 * 16;
    CK(hipMalloc(&out, (size_t)grid * 256 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto gather = [&]() {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_ta<0>, dim3(grid), dim3(256), 0, 0, tab, (unsigned)(n - 1), 16, 0, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    for (int nt : {-1, 0, 1}) {
        float tot = 0;
        for (int r = 0; r < 6; ++r) {
            if (nt >= 0) hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, st, sbytes / 16, nt, (int *)out);
            const float ms = gather();
            if (r > 0) tot += ms;
        }
        printf("gather 64 MB table (16 iters x 8 per lane): %s -> %.3f ms\n",
               nt < 0 ? "back to back (table warm)" : nt ? "after a 2 GiB nt stream" : "after a 2 GiB plain stream",
               tot / 5);
    }
    return 0;
}
