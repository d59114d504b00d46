// kb_chain.hip -- latency of a dependent fp32 add chain in ONE wave on gfx950
// (the C1 gradient is 123 serial column sums of ~926 adds, one wave each,
// one wave per SIMD): cycles per add for a register-only chain and for the
// production pattern (16-byte LDS reads, 32 products per wait).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o kb_chain kb_chain.hip && ./kb_chain
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

// register chain: acc = acc + x[k & 7], 8 operands held in registers
__global__ void k_reg(const float *in, float *out, int n, unsigned long long *cyc) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = in[u + threadIdx.x];
    float acc = 0.0f;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int k = 0; k < n; k += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + x[u];
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// production-like: lane 0 sums n products from LDS, 8 x 16-byte reads per wait
__global__ void k_lds(const float *in, float *out, int n, unsigned long long *cyc) {
    __shared__ __attribute__((aligned(16))) float s[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) s[i] = in[i];
    __syncthreads();
    float acc = 0.0f;
    const unsigned long long t0 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) {
        for (int o = 0; o + 32 <= n; o += 32) {
            float4 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) q[u] = *reinterpret_cast<const float4 *>(s + ((o + 4 * u) & 4095));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                acc = acc + q[u].x;
                acc = acc + q[u].y;
                acc = acc + q[u].z;
                acc = acc + q[u].w;
            }
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[1] = t1 - t0;
}

int main() {
    float *in, *out;
    unsigned long long *cyc;
    CK(hipMalloc(&in, 4096 * 4));
    CK(hipMemset(in, 0, 4096 * 4));
    CK(hipMalloc(&out, 4096 * 4));
    CK(hipMalloc(&cyc, 64));
    const int n = 9216;
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_reg, dim3(1), dim3(64), 0, 0, in, out, n, cyc);
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, in, out, n, cyc);
    }
    CK(hipDeviceSynchronize());
    unsigned long long h[2];
    CK(hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost));
    printf("dependent fp32 add chain, one wave: registers %.2f cycles/add; LDS 16-B reads (32 per wait) %.2f cycles/add "
           "(s_memtime/readcyclecounter cycles, n = %d)\n",
           (double)h[0] / n, (double)h[1] / n, n);
    return 0;
}
