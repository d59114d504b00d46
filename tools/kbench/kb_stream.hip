// kb_stream.hip -- streaming-read rate of the C4 fused dense kernel's access
// pattern on gfx950: 256 workgroups x 512 threads, workgroup k reads its own
// 4 MiB region (256 rows x 4,096 fp32) 64 KiB (4 rows) at a time, two
// register sets in flight per thread, as k_dense_fused does.  Varies the
// distance between the regions' starts (4 MiB exactly -- every workgroup at
// the same offset modulo any power of two below 4 MiB -- or skewed) and
// plain vs non-temporal loads, to see whether region alignment (channel
// camping) or cache policy costs the kernel its last ~7% of stream rate.
//   hipcc --offload-arch=gfx950 -O3 -o kb_stream kb_stream.hip && ./kb_stream
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

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int kThreads = 512;
constexpr int kSub = 64 * 1024 / 16;    // v4f per 64 KiB sub-chunk
constexpr int kReg = kSub / kThreads;   // 8 per thread
constexpr int kNsub = 64;               // 4 MiB per workgroup

template <bool NT>
__global__ __launch_bounds__(kThreads) void k_stream(const v4f *__restrict__ x, size_t stride_v4, float *out) {
    const v4f *base = x + (size_t)blockIdx.x * stride_v4;
    v4f ra[kReg], rb[kReg];
    v4f acc = {0, 0, 0, 0};
    auto load = [&](int q, v4f *r) {
        const int qc = q < kNsub ? q : kNsub - 1;
#pragma unroll
        for (int p = 0; p < kReg; ++p) {
            const v4f *a = base + (size_t)qc * kSub + p * kThreads + threadIdx.x;
            r[p] = NT ? __builtin_nontemporal_load(a) : *a;
        }
    };
    load(0, ra);
    load(1, rb);
    for (int q = 0; q < kNsub; q += 2) {
#pragma unroll
        for (int p = 0; p < kReg; ++p) acc += ra[p];
        load(q + 2, ra);
#pragma unroll
        for (int p = 0; p < kReg; ++p) acc += rb[p];
        load(q + 3, rb);
    }
    if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[threadIdx.x] = acc.x;
}

int main() {
    const size_t region = (size_t)4 << 20;
    const size_t maxstride = region + ((size_t)1 << 20);
    const size_t bytes = 256 * maxstride;
    v4f *x;
    float *out;
    CK(hipMalloc(&x, bytes));
    CK(hipMemset(x, 0, bytes));
    CK(hipMalloc(&out, 4096));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const size_t skews[] = {0, 256, 4096, 65536, 65536 + 4096, 1 << 20};
    for (int nt = 0; nt < 2; ++nt) {
        for (size_t sk : skews) {
            const size_t stride_v4 = (region + sk) / 16;
            float best = 1e30f;
            for (int r = 0; r < 8; ++r) {
                CK(hipEventRecord(a));
                if (nt)
                    hipLaunchKernelGGL(k_stream<true>, dim3(256), dim3(kThreads), 0, 0, x, stride_v4, out);
                else
                    hipLaunchKernelGGL(k_stream<false>, dim3(256), dim3(kThreads), 0, 0, x, stride_v4, out);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (r > 0 && ms < best) best = ms;
            }
            printf("%s loads, region stride 4 MiB + %7zu B: %.1f us, %.2f TB/s\n", nt ? "nt   " : "plain", sk,
                   best * 1e3, 256.0 * region / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
