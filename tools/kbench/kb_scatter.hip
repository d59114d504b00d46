// kb_scatter.hip -- C2 margin experiment: products formed in COLUMN order
// (w read near-sequentially, column-sorted entries) and scattered to their
// CSR positions, then the margin sums them row by row from a stream (no
// random gathers), against the production gather margin.  Development tool.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I dist-lr_amd/csrc \
//         tools/kbench/kb_scatter.hip -o tools/kbench/kb_scatter && ./tools/kbench/kb_scatter
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

namespace ks {
struct Rng {
    uint64_t s;
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
};

template <typename V>
__device__ __forceinline__ V ld_nt(const V *p) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 x = __builtin_nontemporal_load(reinterpret_cast<const u4 *>(p));
    V out;
    __builtin_memcpy(&out, &x, 16);
    return out;
}

// prod[pos[e]] = fl32(w[col[e]] * val[e]) over column-sorted entries, 4 per thread.
template <bool NTST>
__global__ __launch_bounds__(256) void k_scatter(const uint4 *pos, const int4 *col, const float4 *val,
                                                 const float *__restrict__ w, float *__restrict__ prod, int64_t n4) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n4) return;
    const uint4 p = ld_nt(pos + t);
    const int4 c = ld_nt(col + t);
    const float4 v = ld_nt(val + t);
    const float a = w[c.x] * v.x, b = w[c.y] * v.y, d = w[c.z] * v.z, e = w[c.w] * v.w;
    if constexpr (NTST) {
        __builtin_nontemporal_store(a, prod + p.x);
        __builtin_nontemporal_store(b, prod + p.y);
        __builtin_nontemporal_store(d, prod + p.z);
        __builtin_nontemporal_store(e, prod + p.w);
    } else {
        prod[p.x] = a;
        prod[p.y] = b;
        prod[p.z] = d;
        prod[p.w] = e;
    }
}

// Row sums of the products, in order: a wave owns SEG rows; per window of
// 1,024 entries every lane loads 4 float4s (coalesced), parks them in LDS,
// and lane l < SEG adds its row's run.
template <int SEG>
__global__ __launch_bounds__(256) void k_margin_prod(const int64_t *__restrict__ rp, const float *__restrict__ prod,
                                                     const float *__restrict__ lab, int64_t rows,
                                                     float *__restrict__ resid) {
    constexpr int kW = 1024;
    __shared__ __attribute__((aligned(16))) float s_p[4][kW];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x / 64;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wv) * SEG;
    if (row0 >= rows) return;
    const int64_t my = row0 + lane;
    const bool valid = lane < SEG && my < rows;
    const float y = valid ? lab[my] : 0.0f;
    const int64_t rl = min(row0 + SEG, rows);
    const int64_t e0 = rp[row0], e1 = rp[rl];
    const int64_t a = valid ? rp[my] : e1, b = valid ? rp[my + 1] : e1;
    float *lds = s_p[wv];
    float acc = 0.0f;
    for (int64_t ws = e0 & ~int64_t(3); ws < e1; ws += kW) {
        const int64_t left = e1 - ws;
        float4 v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t * 256 < left) v[t] = ld_nt(reinterpret_cast<const float4 *>(prod + ws + t * 256 + lane * 4));
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t * 256 < left) *reinterpret_cast<float4 *>(lds + t * 256 + lane * 4) = v[t];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int64_t lo = a > ws ? a : ws;
        const int64_t hi = b < ws + kW ? b : ws + kW;
        int o = (int)(lo - ws);
        const int oe = (int)(hi - ws);
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
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (valid) {
        const double e = exp(-(double)acc);
        resid[my] = (float)(1.0 / (1.0 + e)) - y;
    }
}

__global__ __launch_bounds__(256) void k_flush(const float4 *buf, int64_t n4, float *out) {
    float acc = 0.f;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n4; t += (int64_t)gridDim.x * 256) {
        const float4 v = buf[t];
        acc += v.x + v.y + v.z + v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}
}  // namespace ks

using namespace ks;

template <typename F>
static float time_us(int reps, F &&launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) launch(i);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms * 1000.0f / reps;
}

template <typename T>
static T *dup(const std::vector<T> &h, size_t pad = 1024) {
    T *d = nullptr;
    CK(hipMalloc(&d, (h.size() + pad) * sizeof(T)));
    CK(hipMemset(d, 0, (h.size() + pad) * sizeof(T)));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char **argv) {
    const int64_t B = 65536, D = 1000000;
    const int nnz = 50;
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int NB = 24;  // distinct batches cycled (a cold-ish shard: 24 x 39 MB of streams)
    Rng rng{10};
    std::vector<int64_t> rp(B + 1);
    std::vector<int32_t> col;
    std::vector<float> val, lab(B);
    std::vector<int32_t> row;
    for (int64_t i = 0; i < B; ++i) {
        rp[i] = (int64_t)col.size();
        row.clear();
        while ((int)row.size() < nnz) {
            int32_t c = (int32_t)rng.below((uint32_t)D);
            if (std::find(row.begin(), row.end(), c) == row.end()) row.push_back(c);
        }
        std::sort(row.begin(), row.end());
        for (int32_t c : row) {
            col.push_back(c);
            val.push_back((float)(1 + rng.below(10000)) * 1e-4f);
        }
        lab[i] = (float)(rng.below(4) == 0);
    }
    rp[B] = (int64_t)col.size();
    const int64_t E = (int64_t)col.size();
    // column-sorted (stable by row) entries with their CSR positions
    std::vector<uint32_t> cnt(D + 1, 0);
    for (int64_t k = 0; k < E; ++k) ++cnt[col[k] + 1];
    for (int64_t j = 0; j < D; ++j) cnt[j + 1] += cnt[j];
    std::vector<uint32_t> spos(E);
    std::vector<int32_t> scol(E);
    std::vector<float> sval(E);
    for (int64_t k = 0; k < E; ++k) {
        const uint32_t q = cnt[col[k]]++;
        spos[q] = (uint32_t)k;
        scol[q] = col[k];
        sval[q] = val[k];
    }
    std::vector<float> w0(D);
    for (int64_t j = 0; j < D; ++j) w0[j] = (float)rng.below(1 << 24) / (float)(1 << 24);

    // NB copies of the batch (CSR and column-sorted), so streams come from HBM
    std::vector<int64_t> rpb((size_t)NB * B + 1);
    std::vector<int32_t> colb((size_t)NB * E), scolb((size_t)NB * E);
    std::vector<float> valb((size_t)NB * E), svalb((size_t)NB * E);
    std::vector<uint32_t> sposb((size_t)NB * E);
    for (int q = 0; q < NB; ++q) {
        for (int64_t i = 0; i < B; ++i) rpb[(size_t)q * B + i] = q * E + rp[i];
        std::copy(col.begin(), col.end(), colb.begin() + (size_t)q * E);
        std::copy(val.begin(), val.end(), valb.begin() + (size_t)q * E);
        std::copy(scol.begin(), scol.end(), scolb.begin() + (size_t)q * E);
        std::copy(sval.begin(), sval.end(), svalb.begin() + (size_t)q * E);
        for (int64_t k = 0; k < E; ++k) sposb[(size_t)q * E + k] = spos[k] + (uint32_t)(q * E);
    }
    rpb[(size_t)NB * B] = NB * E;
    int64_t *d_rp = dup(rpb);
    int32_t *d_col = dup(colb), *d_scol = dup(scolb);
    float *d_val = dup(valb), *d_sval = dup(svalb), *d_lab = dup(lab), *d_w = dup(w0);
    uint32_t *d_spos = dup(sposb);
    float *d_prod = nullptr, *d_r = nullptr, *d_r2 = nullptr;
    CK(hipMalloc(&d_prod, ((size_t)NB * E + 1024) * 4));
    CK(hipMemset(d_prod, 0, ((size_t)NB * E + 1024) * 4));
    CK(hipMalloc(&d_r, B * 4));
    CK(hipMalloc(&d_r2, B * 4));
    printf("kb_scatter: B=%lld D=%lld nnz=%d E=%lld, %d batch copies\n", (long long)B, (long long)D, nnz, (long long)E, NB);
    const int64_t n4 = E / 4;  // E = 3,276,800: a multiple of 4
    const unsigned g4 = (unsigned)((n4 + 255) / 256);
    auto bt_of = [&](int q) { return dlr::DevBatch{d_rp + (size_t)q * B, d_col, d_val, d_lab, B, E}; };

    float t;
    t = time_us(reps, [&](int i) {
        hipLaunchKernelGGL((dlr::k_margin_residual<16, false>), dim3((B + 63) / 64), dim3(256), 0, 0, bt_of(i % NB), d_w, d_r);
    });
    printf("production gather margin SEG=16      %8.2f us\n", t);
    for (int nts = 0; nts < 2; ++nts) {
        t = time_us(reps, [&](int i) {
            const size_t o = (size_t)(i % NB) * E;
            if (nts)
                hipLaunchKernelGGL(k_scatter<true>, dim3(g4), dim3(256), 0, 0, (const uint4 *)(d_spos + o),
                                   (const int4 *)(d_scol + o), (const float4 *)(d_sval + o), d_w, d_prod, n4);
            else
                hipLaunchKernelGGL(k_scatter<false>, dim3(g4), dim3(256), 0, 0, (const uint4 *)(d_spos + o),
                                   (const int4 *)(d_scol + o), (const float4 *)(d_sval + o), d_w, d_prod, n4);
        });
        printf("scatter products (%s stores)          %8.2f us\n", nts ? "nt   " : "plain", t);
    }
    for (int seg : {16, 32, 64}) {
        t = time_us(reps, [&](int i) {
            const int q = i % NB;
            if (seg == 16)
                hipLaunchKernelGGL(k_margin_prod<16>, dim3((B + 63) / 64), dim3(256), 0, 0, d_rp + (size_t)q * B, d_prod, d_lab, B, d_r2);
            else if (seg == 32)
                hipLaunchKernelGGL(k_margin_prod<32>, dim3((B + 127) / 128), dim3(256), 0, 0, d_rp + (size_t)q * B, d_prod, d_lab, B, d_r2);
            else
                hipLaunchKernelGGL(k_margin_prod<64>, dim3((B + 255) / 256), dim3(256), 0, 0, d_rp + (size_t)q * B, d_prod, d_lab, B, d_r2);
        });
        printf("margin from products SEG=%-2d          %8.2f us\n", seg, t);
    }
    for (int nts = 0; nts < 2; ++nts) {
        t = time_us(reps, [&](int i) {
            const int q = i % NB;
            const size_t o = (size_t)q * E;
            if (nts)
                hipLaunchKernelGGL(k_scatter<true>, dim3(g4), dim3(256), 0, 0, (const uint4 *)(d_spos + o),
                                   (const int4 *)(d_scol + o), (const float4 *)(d_sval + o), d_w, d_prod, n4);
            else
                hipLaunchKernelGGL(k_scatter<false>, dim3(g4), dim3(256), 0, 0, (const uint4 *)(d_spos + o),
                                   (const int4 *)(d_scol + o), (const float4 *)(d_sval + o), d_w, d_prod, n4);
            hipLaunchKernelGGL(k_margin_prod<16>, dim3((B + 63) / 64), dim3(256), 0, 0, d_rp + o / E * B, d_prod, d_lab, B, d_r2);
        });
        printf("scatter (%s) + margin SEG=16       %8.2f us\n", nts ? "nt   " : "plain", t);
    }
    // bitwise check on batch 0
    hipLaunchKernelGGL((dlr::k_margin_residual<16, false>), dim3((B + 63) / 64), dim3(256), 0, 0, bt_of(0), d_w, d_r);
    hipLaunchKernelGGL(k_scatter<false>, dim3(g4), dim3(256), 0, 0, (const uint4 *)d_spos, (const int4 *)d_scol,
                       (const float4 *)d_sval, d_w, d_prod, n4);
    hipLaunchKernelGGL(k_margin_prod<16>, dim3((B + 63) / 64), dim3(256), 0, 0, d_rp, d_prod, d_lab, B, d_r2);
    CK(hipDeviceSynchronize());
    std::vector<float> a(B), b(B);
    CK(hipMemcpy(a.data(), d_r, B * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), d_r2, B * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int64_t i = 0; i < B; ++i) bad += memcmp(&a[i], &b[i], 4) != 0;
    printf("check residuals: %s (%zu of %lld differ)\n", bad ? "MISMATCH" : "bitwise equal", bad, (long long)B);
    return bad ? 1 : 0;
}
