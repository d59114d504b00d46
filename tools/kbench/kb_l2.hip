// kb_l2.hip -- the C5 dense L2 pass's access pattern (read 1 GiB of
// weights, scale, write them back in place; 16-byte non-temporal loads and
// stores) with ILP float4s per thread in a one-shot grid, to see how much of
// the 6.6 TB/s k_dense_l2 reaches is the load/store issue depth.
//   hipcc --offload-arch=gfx950 -O3 -o kb_l2 kb_l2.hip && ./kb_l2
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

typedef float f4 __attribute__((ext_vector_type(4)));

// ILP float4s per thread, strided by the block so a wave's loads stay
// coalesced: thread t of block b handles b*256*ILP + k*256 + t, k < ILP
template <int ILP>
__global__ __launch_bounds__(256) void k_l2(float *__restrict__ w, int64_t n4, float s) {
    const int64_t base = (int64_t)blockIdx.x * 256 * ILP + threadIdx.x;
    f4 v[ILP];
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
        const int64_t q = base + (int64_t)k * 256;
        v[k] = q < n4 ? __builtin_nontemporal_load(reinterpret_cast<const f4 *>(w) + q) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
        const int64_t q = base + (int64_t)k * 256;
        v[k] = v[k] - s * v[k];
        if (q < n4) __builtin_nontemporal_store(v[k], reinterpret_cast<f4 *>(w) + q);
    }
}

template <int ILP>
float run(float *w, int64_t n4, hipEvent_t a, hipEvent_t b) {
    const unsigned grid = (unsigned)((n4 + 256 * ILP - 1) / (256 * ILP));
    float best = 1e30f;
    for (int r = 0; r < 8; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_l2<ILP>, dim3(grid), dim3(256), 0, 0, w, n4, 1e-7f);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r > 0 && ms < best) best = ms;
    }
    return best;
}

int main() {
    const int64_t D = (int64_t)1 << 28;  // C5: 2^28 weights, 1 GiB
    float *w;
    CK(hipMalloc(&w, D * 4));
    CK(hipMemset(w, 0, D * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double bytes = 2.0 * D * 4;
    const float t1 = run<1>(w, D / 4, a, b), t2 = run<2>(w, D / 4, a, b), t4 = run<4>(w, D / 4, a, b),
                t8 = run<8>(w, D / 4, a, b);
    printf("in-place scale of 1 GiB (read + write, nt 16-B): ILP1 %.1f us %.2f TB/s | ILP2 %.1f us %.2f TB/s | "
           "ILP4 %.1f us %.2f TB/s | ILP8 %.1f us %.2f TB/s\n",
           t1 * 1e3, bytes / (t1 * 1e-3) / 1e12, t2 * 1e3, bytes / (t2 * 1e-3) / 1e12, t4 * 1e3,
           bytes / (t4 * 1e-3) / 1e12, t8 * 1e3, bytes / (t8 * 1e-3) / 1e12);
    return 0;
}
