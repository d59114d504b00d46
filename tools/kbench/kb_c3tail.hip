// kb_c3tail.hip -- how much of the C3 margin (k_margin_hot, 1.75 ms) is the
// 60 MB tail of the weight table?  Synthetic rows with the entries' rank
// distribution measured on the C3 shard (tools/c3_ranks.py ->
// profiles/r02e_c3_rank_histogram.txt: 63.5% of entries in ranks < 2^14,
// 16.8% in [2^14, 2^18), 7.4% in [2^18, 2^20), 12.3% in [2^20, 2^24)),
// 39 distinct ranks per row, unit values, 12.5M rows; the production
// margin timed as is and with the tail entries remapped into the warm
// range (an upper bound of what a tail product margin could save: the
// tail products would then be read from per-block regions instead of
// gathered).  Development tool only.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I include -I dist-lr_amd/csrc \
//         tools/kbench/kb_c3tail.hip -o tools/kbench/kb_c3tail && ./tools/kbench/kb_c3tail
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../dist-lr_amd/csrc/dlr_kernels.hip"

#define CK(x)                                                                                         \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));          \
            exit(1);                                                                                  \
        }                                                                                             \
    } while (0)

namespace {

struct Rng {
    uint64_t s;
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// remap every column >= 2^20 into [2^14, 2^18) (mode 1) or [0, 2^14) (mode 2)
__global__ void k_remap(int32_t *col, int64_t n, int mode) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t c = col[i];
    if (c >= (1 << 20)) col[i] = mode == 1 ? (1 << 14) + (c & ((1 << 18) - (1 << 14) - 1)) : (c & ((1 << 14) - 1));
}

}  // namespace

int main(int argc, char **argv) {
    const int64_t N = argc > 1 ? atoll(argv[1]) : 12500000;
    const int64_t D = (int64_t)1 << 24;
    const int F = 39;
    // bucket edges and measured probabilities (profiles/r02e_c3_rank_histogram.txt)
    const int64_t edge[8] = {0, 1 << 14, 1 << 18, 1 << 20, 1 << 21, 1 << 22, 1 << 23, 1 << 24};
    const double prob[7] = {0.635, 0.168, 0.074, 0.037, 0.038, 0.035, 0.013};
    double cum[7];
    double acc = 0;
    for (int k = 0; k < 7; ++k) cum[k] = (acc += prob[k]);
    std::vector<int64_t> rp(N + 1);
    std::vector<int32_t> col((size_t)(N * F));
    Rng rng{10};
    for (int64_t i = 0; i < N; ++i) {
        rp[i] = i * F;
        int32_t *r = col.data() + i * F;
        for (int f = 0; f < F; ++f) {
            for (;;) {
                const double u = rng.uni() * acc;
                int k = 0;
                while (k < 6 && u > cum[k]) ++k;
                // within the hot bucket, Zipf-like: rank ~ 2^14 * v^3 (dense at 0)
                const double v = rng.uni();
                const int64_t c = k == 0 ? (int64_t)(v * v * v * (double)(1 << 14))
                                         : edge[k] + (int64_t)(v * (double)(edge[k + 1] - edge[k]));
                bool dup = false;
                for (int g = 0; g < f; ++g) dup |= r[g] == (int32_t)c;
                if (!dup) {
                    r[f] = (int32_t)c;
                    break;
                }
            }
        }
    }
    rp[N] = N * F;
    printf("kb_c3tail: %lld rows x %d entries, D = 2^24, unit values\n", (long long)N, F);
    int64_t *d_rp;
    int32_t *d_col;
    float *d_w, *d_lab, *d_r;
    CK(hipMalloc(&d_rp, (N + 1) * 8));
    CK(hipMalloc(&d_col, (N * F + 64) * 4));
    CK(hipMalloc(&d_w, D * 4));
    CK(hipMalloc(&d_lab, N * 4));
    CK(hipMalloc(&d_r, N * 4));
    CK(hipMemcpy(d_rp, rp.data(), (N + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), N * F * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_col + N * F, 0, 64 * 4));
    CK(hipMemset(d_w, 0, D * 4));
    CK(hipMemset(d_lab, 0, N * 4));
    const dlr::DevBatch bt{d_rp, d_col, nullptr, d_lab, N, N * F};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time_margin = [&](const char *name) {
        for (int k = 0; k < 2; ++k) CK(dlr::launch_margin_hot(bt, d_w, D, d_r, 0));
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(a, 0));
        for (int k = 0; k < reps; ++k) CK(dlr::launch_margin_hot(bt, d_w, D, d_r, 0));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-58s %8.1f us\n", name, ms * 1000.0f / reps);
    };
    time_margin("k_margin_hot, measured rank mix");
    const int64_t n = N * F;
    hipLaunchKernelGGL(k_remap, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d_col, n, 1);
    CK(hipDeviceSynchronize());
    time_margin("k_margin_hot, tail (ranks >= 2^20) remapped to [2^14, 2^18)");
    CK(hipMemcpy(d_col, col.data(), N * F * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_remap, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d_col, n, 2);
    CK(hipDeviceSynchronize());
    time_margin("k_margin_hot, tail remapped into the LDS hot tier");
    return 0;
}
