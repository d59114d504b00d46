// kb_c3tail.hip -- how much of the C3 margin (k_margin_hot, 1.75 ms) is the
// 60 MB tail of the weight table?  Synthetic rows with the entries' rank
// distribution measured on the C3 shard (tools/c3_ranks.py ->
// profiles/r02e_c3_rank_histogram.txt: 63.5% of entries in ranks < 2^14,
// 16.8% in [2^14, 2^18), 7.4% in [2^18, 2^20), 12.3% in [2^20, 2^24)),
// 39 distinct ranks per row, unit values, 12.5M rows; the production
// margin timed as is and with the tail entries remapped into the warm
// range (an upper bound of what a tail product margin could save: the
// tail products would then be read from per-block regions instead of
// gathered); and a variant of it software-pipelined across row blocks.
// Development tool only.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I include -I dist-lr_amd/csrc \
//         tools/kbench/kb_c3tail.hip -o tools/kbench/kb_c3tail && ./tools/kbench/kb_c3tail
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// Persistent hot margin, software-pipelined ACROSS the wave's row blocks
// (a C3 block of 16 rows is one window of ~624 entries): while block i's
// gathers and sums run, block i+1's column window and block i+2's row
// pointers are in flight.  Same products, same in-order sums as
// k_margin_hot.
template <int HOT, int NW, int SEG>
__global__ __launch_bounds__(NW * 64) void k_margin_hot_pipe(dlr::DevBatch bt, const float *__restrict__ w,
                                                           float *__restrict__ resid) {
    constexpr int kWin = 1024, kVec = 4, kT = kWin / (kVec * 64), kChunk = kVec * 64;
    __shared__ __attribute__((aligned(16))) float s_w[HOT];
    __shared__ float s_p[NW][kWin];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x / 64;
    {
        const float4 *src = reinterpret_cast<const float4 *>(w);
        float4 *dst = reinterpret_cast<float4 *>(s_w);
#pragma unroll
        for (int k = 0; k < HOT / 4 / (NW * 64); ++k) dst[k * NW * 64 + threadIdx.x] = src[k * NW * 64 + threadIdx.x];
    }
    __syncthreads();
    float *lds = s_p[wv];
    const int64_t nblk = (bt.rows + NW * SEG - 1) / (NW * SEG);
    struct Blk {
        int64_t row0 = -1, e0 = 0, e1 = 0, a = 0, b = 0;
        float y = 0.0f;
        bool valid = false;
    };
    // the row pointers of block blk (row0 < 0: no block)
    auto ptrs = [&](int64_t blk, Blk &q) {
        q.row0 = -1;
        if (blk >= nblk) return;
        const int64_t row0 = (blk * NW + wv) * SEG;
        if (row0 >= bt.rows) return;
        q.row0 = row0;
        const int64_t my = row0 + lane;
        q.valid = lane < SEG && my < bt.rows;
        const int64_t rlast = min(row0 + SEG, bt.rows);
        q.e0 = bt.row_ptr[row0];
        q.e1 = bt.row_ptr[rlast];
        const int64_t mc = q.valid ? my : row0;
        q.a = bt.row_ptr[mc];
        q.b = bt.row_ptr[mc + 1];
        q.y = bt.label[mc];
    };
    // block q's single window (SEG rows of <= 1024 entries in total)
    auto window = [&](const Blk &q, int4 (&v)[kT]) {
        if (q.row0 < 0) return;
        const int64_t ws = q.e0 & ~int64_t(kVec - 1);
        const int64_t left = q.e1 - ws;
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            if (t * kChunk < left) {
                const int64_t e = ws + t * kChunk + lane * kVec;
                const int64_t ec = e < q.e1 ? e : ws + t * kChunk;
                v[t] = dlr::load_stream(reinterpret_cast<const int4 *>(bt.col + ec));
            }
        }
    };
    Blk cur, nxt, nn;
    int4 iv[kT], nv[kT];
    ptrs(blockIdx.x, cur);
    ptrs(blockIdx.x + gridDim.x, nxt);
    window(cur, iv);
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        if (cur.row0 >= 0) {
            const int64_t ws = cur.e0 & ~int64_t(kVec - 1);
            const int64_t left = cur.e1 - ws;
            float g[kT][kVec];
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                if (t * kChunk < left) {
                    const int64_t e = ws + t * kChunk + lane * kVec;
                    const unsigned i0 = (e >= cur.e0 && e < cur.e1) ? (unsigned)iv[t].x : 0u;
                    const unsigned i1 = (e + 1 >= cur.e0 && e + 1 < cur.e1) ? (unsigned)iv[t].y : 0u;
                    const unsigned i2 = (e + 2 >= cur.e0 && e + 2 < cur.e1) ? (unsigned)iv[t].z : 0u;
                    const unsigned i3 = (e + 3 >= cur.e0 && e + 3 < cur.e1) ? (unsigned)iv[t].w : 0u;
                    const float h0 = s_w[i0 < HOT ? i0 : 0u], h1 = s_w[i1 < HOT ? i1 : 0u];
                    const float h2 = s_w[i2 < HOT ? i2 : 0u], h3 = s_w[i3 < HOT ? i3 : 0u];
                    const float c0 = w[i0 < HOT ? 0u : i0], c1 = w[i1 < HOT ? 0u : i1];
                    const float c2 = w[i2 < HOT ? 0u : i2], c3 = w[i3 < HOT ? 0u : i3];
                    g[t][0] = i0 < HOT ? h0 : c0;
                    g[t][1] = i1 < HOT ? h1 : c1;
                    g[t][2] = i2 < HOT ? h2 : c2;
                    g[t][3] = i3 < HOT ? h3 : c3;
                }
            }
            // behind this block's gathers: the next block's window, the
            // block after's row pointers
            window(nxt, nv);
            ptrs(blk + 2 * (int64_t)gridDim.x, nn);
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                if (t * kChunk < left) {
                    const int o = t * kChunk + lane * kVec;
                    const int64_t e = ws + o;
                    float4 p;
                    p.x = (e >= cur.e0 && e < cur.e1) ? g[t][0] : 0.0f;
                    p.y = (e + 1 >= cur.e0 && e + 1 < cur.e1) ? g[t][1] : 0.0f;
                    p.z = (e + 2 >= cur.e0 && e + 2 < cur.e1) ? g[t][2] : 0.0f;
                    p.w = (e + 3 >= cur.e0 && e + 3 < cur.e1) ? g[t][3] : 0.0f;
                    *reinterpret_cast<float4 *>(lds + o) = p;
                }
            }
            dlr::wave_sync();
            float acc = 0.0f;
            int o = (int)(cur.a - ws);
            const int oe = (int)(cur.b - ws);
            for (; o + 8 <= oe; o += 8) {
                const float x0 = lds[o], x1 = lds[o + 1], x2 = lds[o + 2], x3 = lds[o + 3];
                const float x4 = lds[o + 4], x5 = lds[o + 5], x6 = lds[o + 6], x7 = lds[o + 7];
                acc = acc + x0;
                acc = acc + x1;
                acc = acc + x2;
                acc = acc + x3;
                acc = acc + x4;
                acc = acc + x5;
                acc = acc + x6;
                acc = acc + x7;
            }
            for (; o < oe; ++o) acc = acc + lds[o];
            dlr::wave_sync();
            if (cur.valid) resid[cur.row0 + lane] = dlr::sigmoid_ref(acc) - cur.y;
        } else {
            window(nxt, nv);
            ptrs(blk + 2 * (int64_t)gridDim.x, nn);
        }
        cur = nxt;
        nxt = nn;
#pragma unroll
        for (int t = 0; t < kT; ++t) iv[t] = nv[t];
    }
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
    {
        // the pipelined variant: same grid as launch_margin_hot's default
        // (16,384 hot weights x 16 waves, SEG 16, one workgroup per CU)
        float *d_r2;
        CK(hipMalloc(&d_r2, N * 4));
        int dev = 0, ncu = 256;
        CK(hipGetDevice(&dev));
        CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        const int64_t nb = (N + 16 * 16 - 1) / (16 * 16);
        const unsigned grid = (unsigned)std::min<int64_t>(nb, ncu);
        std::vector<float> w0(D);
        for (int64_t j = 0; j < D; ++j) w0[j] = (float)((j * 2654435761u) % 2001) * 1e-4f - 0.1f;
        CK(hipMemcpy(d_w, w0.data(), D * 4, hipMemcpyHostToDevice));
        CK(dlr::launch_margin_hot(bt, d_w, D, d_r, 0));
        hipLaunchKernelGGL((k_margin_hot_pipe<16384, 16, 16>), dim3(grid), dim3(1024), 0, 0, bt, d_w, d_r2);
        CK(hipDeviceSynchronize());
        std::vector<float> r1(N), r2(N);
        CK(hipMemcpy(r1.data(), d_r, N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r2.data(), d_r2, N * 4, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t i = 0; i < N; ++i) bad += memcmp(&r1[i], &r2[i], 4) != 0;
        printf("pipelined variant vs production: %lld of %lld residuals differ\n", (long long)bad, (long long)N);
        const int reps = 10;
        for (int k = 0; k < 2; ++k) hipLaunchKernelGGL((k_margin_hot_pipe<16384, 16, 16>), dim3(grid), dim3(1024), 0, 0, bt, d_w, d_r2);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int k = 0; k < reps; ++k) hipLaunchKernelGGL((k_margin_hot_pipe<16384, 16, 16>), dim3(grid), dim3(1024), 0, 0, bt, d_w, d_r2);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-58s %8.1f us\n", "k_margin_hot_pipe (next window's columns in flight)", ms * 1000.0f / reps);
        time_margin("k_margin_hot again (same weights)");
    }
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
