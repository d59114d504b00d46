// kb_chain2.hip -- dependent fp32 add chain latency on gfx950, by active
// lanes and interleaving, timed with s_memtime (shader cycles) AND
// s_memrealtime (100 MHz) so the clock is known.  One workgroup of 64 or 256
// threads; the chain is inline asm (v_add_f32 acc, acc, x) so nothing is
// reordered.
//   hipcc --offload-arch=gfx950 -O3 -o kb_chain2 kb_chain2.hip && ./kb_chain2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

#define ADD1(a, x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(x))
#define ADD8(a, x) ADD1(a, x); ADD1(a, x); ADD1(a, x); ADD1(a, x); ADD1(a, x); ADD1(a, x); ADD1(a, x); ADD1(a, x)

// mode 0: every lane; 1: lanes 0-31; 2: lane 0 only; 3: two interleaved
// chains per lane; 4: four interleaved chains per lane; 5: sgpr operand
__global__ void k_chain(const float *in, float *out, int n, int mode, int active_waves,
                        unsigned long long *res) {
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    float x = in[threadIdx.x];
    float a = in[threadIdx.x + 256], b = a, c = a, d = a;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    bool on = wv < active_waves;
    if (mode == 1) on = on && lane < 32;
    if (mode == 2) on = on && lane == 0;
    if (on) {
        if (mode <= 2) {
            for (int k = 0; k < n; k += 64) {
                ADD8(a, x); ADD8(a, x); ADD8(a, x); ADD8(a, x);
                ADD8(a, x); ADD8(a, x); ADD8(a, x); ADD8(a, x);
            }
        } else if (mode == 3) {
            for (int k = 0; k < n; k += 32) {
#pragma unroll
                for (int u = 0; u < 32; ++u) { ADD1(a, x); ADD1(b, x); }
            }
        } else if (mode == 4) {
            for (int k = 0; k < n; k += 32) {
#pragma unroll
                for (int u = 0; u < 32; ++u) { ADD1(a, x); ADD1(b, x); ADD1(c, x); ADD1(d, x); }
            }
        } else if (mode == 5) {
            const float s = __builtin_amdgcn_readfirstlane(__float_as_uint(x)) ? x : x;
            for (int k = 0; k < n; k += 8) {
                asm volatile("v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n"
                             "v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0"
                             : "+v"(a) : "s"(__builtin_amdgcn_readfirstlane(__float_as_uint(s))));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) {
        res[0] = t1 - t0;
        res[1] = r1 - r0;
    }
}

int main() {
    float *in, *out;
    unsigned long long *res;
    CK(hipMalloc(&in, 4096 * 4));
    CK(hipMemset(in, 0, 4096 * 4));
    CK(hipMalloc(&out, 4096 * 4));
    CK(hipMalloc(&res, 64));
    const int n = 1 << 16;
    const char *names[] = {"64 lanes", "32 lanes", "1 lane", "2 chains/lane", "4 chains/lane", "sgpr operand"};
    for (int mode = 0; mode <= 5; ++mode) {
        for (int aw = 1; aw <= 4; aw *= 4) {
            for (int threads = 64; threads <= 1024; threads *= 4) {
                if (aw * 64 > threads) continue;
                unsigned long long h[2] = {0, 0};
                for (int r = 0; r < 3; ++r) {
                    hipLaunchKernelGGL(k_chain, dim3(1), dim3(threads), 0, 0, in, out, n, mode, aw, res);
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(h, res, 16, hipMemcpyDeviceToHost));
                }
                const double cyc = (double)h[0] / n, ns = (double)h[1] * 10.0 / n;
                printf("%-14s threads %4d active waves %d: %.2f cycles/add-step, %.3f ns/add-step, clock %.2f GHz\n",
                       names[mode], threads, aw, cyc, ns, cyc / ns);
            }
        }
    }
    return 0;
}
