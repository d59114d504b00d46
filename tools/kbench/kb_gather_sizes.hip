// kb_gather_sizes.hip -- random 4-byte gather rate vs table size on gfx950
// (development tool).  The C3 step gathers weights from a 64 MiB table
// (2^24 features) and residuals from a 50 MB table (12.5M rows): larger than
// one XCD's 4 MB L2, inside the 256 MB Infinity Cache.  Also: the same
// gathers with a row-local index pattern (each wave's 256 indices inside a
// window of `span` floats), the shape of a hot column's chunk.
//
//   hipcc --offload-arch=gfx950 -O3 tools/kbench/kb_gather_sizes.hip -o tools/kbench/kb_gather_sizes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

__global__ __launch_bounds__(256) void g_gather(const int4 *idx, const float *table, float *out, int64_t n4) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n4) return;
    typedef int i4 __attribute__((ext_vector_type(4)));
    const i4 i = __builtin_nontemporal_load(reinterpret_cast<const i4 *>(idx) + t);
    out[t] = table[i.x] + table[i.y] + table[i.z] + table[i.w];
}

__global__ __launch_bounds__(256) void g_flush(const float4 *buf, int64_t n4, float *out) {
    float acc = 0.f;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n4; t += (int64_t)gridDim.x * 256) {
        const float4 v = buf[t];
        acc += v.x + v.y + v.z + v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static uint64_t s_rng = 0x1234567;
static inline uint32_t rnd() {
    s_rng ^= s_rng << 13;
    s_rng ^= s_rng >> 7;
    s_rng ^= s_rng << 17;
    return (uint32_t)(s_rng >> 11);
}

int main() {
    const int64_t n = 64 << 20;  // gathers per launch (256 MiB of indices)
    const int64_t n4 = n / 4;
    std::vector<int> h((size_t)n);
    int *d_idx;
    float *d_tab, *d_out;
    const int64_t max_tab = (int64_t)1 << 28;  // 1 GiB
    CK(hipMalloc(&d_idx, n * 4));
    CK(hipMalloc(&d_tab, max_tab * 4));
    CK(hipMemset(d_tab, 0, max_tab * 4));
    CK(hipMalloc(&d_out, n4 * 4));
    float4 *fb;
    const int64_t fl4 = (int64_t)1 << 26;
    CK(hipMalloc(&fb, fl4 * 16));
    CK(hipMemset(fb, 0, fl4 * 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char *what, int64_t tab, int64_t span) {
        // span == 0: uniform over the table; else wave w's 256 indices lie in
        // [base_w, base_w + span) with base_w ascending through the table
        for (int64_t k = 0; k < n; ++k) {
            if (span == 0) {
                h[(size_t)k] = (int)(rnd() % (uint32_t)tab);
            } else {
                const int64_t wv = k / 256;
                const int64_t base = (wv * 97 * span / 256) % (tab - span);  // bands sweep the table
                h[(size_t)k] = (int)(base + rnd() % (uint32_t)span);
            }
        }
        CK(hipMemcpy(d_idx, h.data(), n * 4, hipMemcpyHostToDevice));
        const unsigned grid = (unsigned)((n4 + 255) / 256);
        hipLaunchKernelGGL(g_gather, dim3(grid), dim3(256), 0, 0, (const int4 *)d_idx, d_tab, d_out, n4);
        double tot = 0;
        const int reps = 5;
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(g_flush, dim3(4096), dim3(256), 0, 0, (const float4 *)fb, fl4, d_out);
            // warm the table into whatever cache holds it (as the step's
            // producer kernel would leave it)
            hipLaunchKernelGGL(g_flush, dim3(4096), dim3(256), 0, 0, (const float4 *)d_tab, tab / 4, d_out);
            CK(hipEventRecord(a, 0));
            hipLaunchKernelGGL(g_gather, dim3(grid), dim3(256), 0, 0, (const int4 *)d_idx, d_tab, d_out, n4);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            tot += ms;
        }
        const double us = tot * 1000.0 / reps;
        printf("%-8s table %9.2f MiB span %9lld: %9.1f us  %7.1f G gathers/s\n", what, tab * 4.0 / (1 << 20),
               (long long)span, us, n / us / 1e3);
        fflush(stdout);
    };
    for (int64_t tab : {(int64_t)1 << 16, (int64_t)1 << 20, (int64_t)1 << 22, (int64_t)12500000, (int64_t)1 << 24,
                        (int64_t)1 << 26, (int64_t)1 << 28})
        run("uniform", tab, 0);
    for (int64_t span : {(int64_t)1024, (int64_t)8192, (int64_t)65536, (int64_t)1 << 20})
        run("banded", 12500000, span);
    return 0;
}
