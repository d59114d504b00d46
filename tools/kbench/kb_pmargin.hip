// kb_pmargin.hip -- design microbenchmark: the C2 margin as PRODUCTS BY
// COLUMN SLICE + ROW SUMS FROM LDS, against the production gather margin.
//
// The production margin (k_margin_residual) issues one random 4-byte L2
// request per entry (3.28M per C2 batch) and runs at the L2 request rate.
// Here: pass 1 (one workgroup per 4,096-column slice) stages its slice of w
// in LDS and forms every product of the batch in that slice, written to the
// product array in BLOCK-MAJOR order (64-row block, then slice, then row);
// pass 2 (a wave per 64-row block) copies its block's contiguous products
// into LDS with 16-byte loads and each lane adds its row's products in
// column order through a precomputed slot list.  Same products, same order
// of additions: bitwise the production margins.  Development tool only.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I dist-lr_amd/csrc \
//         tools/kbench/kb_pmargin.hip -o /tmp/kb_pmargin && /tmp/kb_pmargin
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

namespace kb {

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

constexpr int SW = 4096;  // columns per slice
constexpr int RB = 64;    // rows per block
constexpr int CAP = 4096; // products per block (LDS floats per wave)

__device__ __forceinline__ float sig(float z) {
    const double e = exp(-(double)z);
    return (float)(1.0 / (1.0 + e));
}

// pass 1: SPLIT workgroups per slice (all on one XCD: blockIdx % 8 is the
// slice's XCD, so each XCD's L2 serves 1/8 of w).  list entries:
// (lc | blk << 12 | j << 22); product goes to p[pofs[s*nblk + blk] + j].
template <int NT, int SPLIT, int U, int ABL = 0>
__global__ __launch_bounds__(NT) void k_prod(const uint32_t *__restrict__ lbeg, const uint32_t *__restrict__ list,
                                             const float *__restrict__ lval, const uint32_t *__restrict__ pofs,
                                             int nblk, int S, const float *__restrict__ w, int64_t D,
                                             float *__restrict__ p) {
    __shared__ __attribute__((aligned(16))) float s_w[SW];
    __shared__ uint32_t s_po[1024];
    const int x = blockIdx.x, xcd = x & 7, k = x >> 3;
    const int s = (k / SPLIT) * 8 + xcd, part = k % SPLIT;
    if (s >= S) return;  // whole workgroup
    const uint32_t b0 = lbeg[s], b1 = lbeg[s + 1];
    const uint32_t n = b1 - b0, per = (n + SPLIT - 1) / SPLIT;
    const uint32_t c0 = b0 + min(n, per * part), c1 = b0 + min(n, per * (part + 1));
    // everything in flight at once: the slice of w, the block offsets, U entries per thread
    float4 wv[SW / 4 / NT];
#pragma unroll
    for (int u = 0; u < SW / 4 / NT; ++u) {
        const int64_t j = (int64_t)s * SW + 4 * (u * NT + threadIdx.x);
        wv[u] = j + 3 < D ? *reinterpret_cast<const float4 *>(w + j) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    uint32_t po[(1024 + NT - 1) / NT];
#pragma unroll
    for (int u = 0; u < (1024 + NT - 1) / NT; ++u) {
        const int i = u * NT + threadIdx.x;
        po[u] = i < nblk ? pofs[(int64_t)s * nblk + i] : 0u;
    }
    uint32_t pk[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = c0 + u * NT + threadIdx.x;
        const uint32_t ic = i < c1 ? i : b0;
        pk[u] = __builtin_nontemporal_load(list + ic);
        v[u] = __builtin_nontemporal_load(lval + ic);
    }
#pragma unroll
    for (int u = 0; u < SW / 4 / NT; ++u) reinterpret_cast<float4 *>(s_w)[u * NT + threadIdx.x] = wv[u];
#pragma unroll
    for (int u = 0; u < (1024 + NT - 1) / NT; ++u) {
        const int i = u * NT + threadIdx.x;
        if (i < 1024) s_po[i] = po[u];
    }
    __syncthreads();
    for (uint32_t i0 = c0;; i0 += U * NT) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + u * NT + threadIdx.x;
            if (i < c1) {
                const uint32_t lc = pk[u] & (SW - 1), blk = (pk[u] >> 12) & 1023, j = pk[u] >> 22;
                if (ABL == 1)
                    p[i - lbeg[0]] = s_w[lc] * v[u];  // contiguous (list order)
                else if (ABL == 2)
                    p[s_po[blk] + j] = v[u];  // no w gather
                else
                    p[s_po[blk] + j] = s_w[lc] * v[u];
            }
        }
        if (i0 + U * NT >= c1) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + U * NT + u * NT + threadIdx.x;
            const uint32_t ic = i < c1 ? i : b0;
            pk[u] = __builtin_nontemporal_load(list + ic);
            v[u] = __builtin_nontemporal_load(lval + ic);
        }
    }
}

// pass 2: wave per 64-row block.  region [rg[blk], rg[blk+1]) (4-aligned,
// <= CAP), slots qs at qoff[blk]: [k/8][lane][k%8] uint16 (<= QG groups).
template <int QG>
__global__ __launch_bounds__(256) void k_m2(const uint32_t *__restrict__ rg, const uint32_t *__restrict__ qoff,
                                            const uint16_t *__restrict__ qs, const int64_t *__restrict__ row_ptr,
                                            const float *__restrict__ label, int64_t rows,
                                            const float *__restrict__ p, float *__restrict__ resid) {
    __shared__ __attribute__((aligned(16))) float s_reg[4][CAP];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t blk = (int64_t)blockIdx.x * 4 + wv;
    const int64_t r0 = blk * RB;
    if (r0 >= rows) return;
    const uint32_t a = rg[blk], b = rg[blk + 1];
    const uint32_t q0 = qoff[blk], q1 = qoff[blk + 1];
    const int64_t my = r0 + lane;
    const bool valid = my < rows;
    const int64_t mc = valid ? my : r0;
    const int len = valid ? (int)(row_ptr[mc + 1] - row_ptr[mc]) : 0;
    const float y = label[mc];
    float *sr = s_reg[wv];
    const int n4 = (int)((b - a) >> 2);
    const int ngrp = (int)((q1 - q0) >> 9);  // groups of 8 k: 64 lanes x 8 u16
    constexpr int R4 = CAP / 4 / 64;
    float4 rv[R4];
    uint4 qv[QG];
#pragma unroll
    for (int t = 0; t < R4; ++t)
        if (t * 64 < n4) {
            const int tt = t * 64 + lane < n4 ? t * 64 + lane : 0;
            rv[t] = dlr::load_stream(reinterpret_cast<const float4 *>(p + a) + tt);
        }
#pragma unroll
    for (int g = 0; g < QG; ++g)
        if (g < ngrp) qv[g] = dlr::load_stream(reinterpret_cast<const uint4 *>(qs + q0) + g * 64 + lane);
#pragma unroll
    for (int t = 0; t < R4; ++t)
        if (t * 64 < n4 && t * 64 + lane < n4) reinterpret_cast<float4 *>(sr)[t * 64 + lane] = rv[t];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float acc = 0.0f;
#pragma unroll
    for (int g = 0; g < QG; ++g) {
        if (g >= ngrp) break;
        const uint32_t qq[4] = {qv[g].x, qv[g].y, qv[g].z, qv[g].w};
        float x[8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            x[2 * u] = sr[qq[u] & 0xFFFF];
            x[2 * u + 1] = sr[qq[u] >> 16];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float t = acc + x[u];
            acc = (g * 8 + u < len) ? t : acc;
        }
    }
    if (valid) resid[my] = sig(acc) - y;
}

// pass 2 variants: DMA = region copied into LDS by global_load_lds (no
// VGPR staging); HALF = two waves per block (each copies half the region and
// sums 32 rows).
template <int QG, bool DMA, bool HALF>
__global__ __launch_bounds__(256) void k_m2v(const uint32_t *__restrict__ rg, const uint32_t *__restrict__ qoff,
                                             const uint16_t *__restrict__ qs, const int64_t *__restrict__ row_ptr,
                                             const float *__restrict__ label, int64_t rows,
                                             const float *__restrict__ p, float *__restrict__ resid) {
    constexpr int BPW = HALF ? 2 : 4;  // blocks per workgroup
    __shared__ __attribute__((aligned(16))) float s_reg[BPW][CAP];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int sub = HALF ? (wv & 1) : 0;
    const int64_t blk = (int64_t)blockIdx.x * BPW + (HALF ? wv >> 1 : wv);
    const int64_t r0 = blk * RB;
    if (r0 >= rows) return;
    const uint32_t a = rg[blk], b = rg[blk + 1];
    const uint32_t q0 = qoff[blk], q1 = qoff[blk + 1];
    const int rl = HALF ? sub * 32 + (lane & 31) : lane;
    const int64_t my = r0 + rl;
    const bool valid = my < rows && (!HALF || lane < 32);
    const int64_t mc = my < rows ? my : r0;
    const int len = valid ? (int)(row_ptr[mc + 1] - row_ptr[mc]) : 0;
    const float y = label[mc];
    float *sr = s_reg[HALF ? wv >> 1 : wv];
    const int n4 = (int)((b - a) >> 2);
    const int ngrp = (int)((q1 - q0) >> 9);
    constexpr int R4 = CAP / 4 / 64;
    uint4 qv[QG];
    if (DMA) {
#pragma unroll
        for (int t = 0; t < R4; ++t) {
            const int tt = HALF ? 2 * t + sub : t;
            if (tt * 64 < n4) {
                const int e = tt * 64 + lane < n4 ? tt * 64 + lane : tt * 64;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(p + a + 4 * e),
                                                 (__attribute__((address_space(3))) void *)(sr + tt * 256), 16, 0, 0);
            }
        }
    } else {
        float4 rv[R4];
#pragma unroll
        for (int t = 0; t < R4; ++t) {
            const int tt = HALF ? 2 * t + sub : t;
            if (tt * 64 < n4) {
                const int e = tt * 64 + lane < n4 ? tt * 64 + lane : 0;
                rv[t] = dlr::load_stream(reinterpret_cast<const float4 *>(p + a) + e);
            }
        }
#pragma unroll
        for (int t = 0; t < R4; ++t) {
            const int tt = HALF ? 2 * t + sub : t;
            if (tt * 64 < n4 && tt * 64 + lane < n4) reinterpret_cast<float4 *>(sr)[tt * 64 + lane] = rv[t];
        }
    }
#pragma unroll
    for (int g = 0; g < QG; ++g)
        if (g < ngrp) qv[g] = dlr::load_stream(reinterpret_cast<const uint4 *>(qs + q0) + g * 64 + rl);
    if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (HALF) __syncthreads();
    else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    float acc = 0.0f;
#pragma unroll
    for (int g = 0; g < QG; ++g) {
        if (g >= ngrp) break;
        const uint32_t qq[4] = {qv[g].x, qv[g].y, qv[g].z, qv[g].w};
        float x[8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            x[2 * u] = sr[qq[u] & 0xFFFF];
            x[2 * u + 1] = sr[qq[u] >> 16];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float t = acc + x[u];
            acc = (g * 8 + u < len) ? t : acc;
        }
    }
    if (valid) resid[my] = sig(acc) - y;
}

}  // namespace kb

int main(int argc, char **argv) {
    using namespace kb;
    const int64_t B = 65536, D = argc > 1 ? atoll(argv[1]) : 1000000;
    const int nnz = argc > 2 ? atoi(argv[2]) : 50;
    const int NB = argc > 3 ? atoi(argv[3]) : 8;
    const int reps = 200;
    const int64_t nblk = B / RB, S = (D + SW - 1) / SW;
    printf("kb_pmargin: B=%lld D=%lld nnz=%d batches=%d slices=%lld blocks=%lld\n", (long long)B, (long long)D, nnz,
           NB, (long long)S, (long long)nblk);
    const bool xorder = argc > 5 && atoi(argv[5]) != 0;
    std::vector<int64_t> sorder;
    for (int x = 0; x < 8; ++x)
        for (int64_t s = x; s < S; s += 8) sorder.push_back(s);
    Rng rng{10};
    // all batches back to back: CSR (global row_ptr), labels
    const int64_t N = B * NB;
    std::vector<int64_t> rp(N + 1);
    std::vector<int32_t> col;
    std::vector<float> val, lab(N);
    col.reserve(N * nnz);
    val.reserve(N * nnz);
    std::vector<int32_t> row;
    for (int64_t i = 0; i < N; ++i) {
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
    rp[N] = (int64_t)col.size();
    const int64_t E = (int64_t)col.size();
    // product-margin layout per batch
    std::vector<uint32_t> h_lbeg, h_list, h_pofs, h_rg, h_qoff;
    std::vector<float> h_lval;
    std::vector<uint16_t> h_qs;
    std::vector<int64_t> lb_off(NB), pofs_off(NB), rg_off(NB), qo_off(NB), p_cap(NB);
    int64_t pmax = 0;
    for (int bt = 0; bt < NB; ++bt) {
        const int64_t rbase = (int64_t)bt * B;
        // region of each block: entries grouped by slice, then row, then position
        std::vector<uint32_t> rgb(nblk + 1);
        std::vector<uint32_t> cnt((size_t)nblk * S, 0);  // [blk][s]
        for (int64_t r = 0; r < B; ++r)
            for (int64_t e = rp[rbase + r]; e < rp[rbase + r + 1]; ++e) ++cnt[(size_t)(r / RB) * S + col[e] / SW];
        uint32_t acc = 0;
        std::vector<uint32_t> cofs((size_t)nblk * S);  // chunk start (batch-relative p index)
        for (int64_t k = 0; k < nblk; ++k) {
            rgb[k] = acc;
            for (int64_t si = 0; si < S; ++si) {
                // xorder: a region's chunks grouped by the XCD of their slice's workgroup
                const int64_t s = xorder ? sorder[si] : si;
                cofs[(size_t)k * S + s] = acc;
                acc += cnt[(size_t)k * S + s];
            }
            acc = (acc + 3) & ~3u;
            if (acc - rgb[k] > (uint32_t)CAP) { fprintf(stderr, "region too big\n"); return 1; }
        }
        rgb[nblk] = acc;
        p_cap[bt] = acc;
        pmax = std::max<int64_t>(pmax, acc);
        // slot of every entry; slice lists (ordered by blk, then region slot)
        std::vector<uint32_t> fill(cofs);
        std::vector<uint32_t> slot(rp[rbase + B] - rp[rbase]);
        for (int64_t r = 0; r < B; ++r)
            for (int64_t e = rp[rbase + r]; e < rp[rbase + r + 1]; ++e)
                slot[e - rp[rbase]] = fill[(size_t)(r / RB) * S + col[e] / SW]++;
        // lists: per slice, per block, entries in slot order = (row, position) order
        std::vector<uint32_t> lcnt(S + 1, 0);
        for (int64_t e = rp[rbase]; e < rp[rbase + B]; ++e) ++lcnt[col[e] / SW + 1];
        for (int64_t s = 0; s < S; ++s) lcnt[s + 1] += lcnt[s];
        lb_off[bt] = (int64_t)h_lbeg.size();
        const int64_t lbase = (int64_t)h_list.size();
        for (int64_t s = 0; s <= S; ++s) h_lbeg.push_back((uint32_t)(lbase + lcnt[s]));
        h_list.resize(lbase + lcnt[S]);
        h_lval.resize(lbase + lcnt[S]);
        std::vector<uint32_t> lcur(lcnt.begin(), lcnt.end() - 1);
        // iterate rows in order: within a block and slice, (row, position) order
        for (int64_t r = 0; r < B; ++r)
            for (int64_t e = rp[rbase + r]; e < rp[rbase + r + 1]; ++e) {
                const int64_t s = col[e] / SW, blk = r / RB;
                const uint32_t j = slot[e - rp[rbase]] - cofs[(size_t)blk * S + s];
                if (j >= 1024) { fprintf(stderr, "chunk too big\n"); return 1; }
                const uint32_t li = lcur[s]++;
                h_list[lbase + li] = (uint32_t)(col[e] % SW) | (uint32_t)blk << 12 | j << 22;
                h_lval[lbase + li] = val[e];
            }
        // within a slice, entries must be ordered by blk: rows ascend, so yes.
        pofs_off[bt] = (int64_t)h_pofs.size();
        for (int64_t s = 0; s < S; ++s)
            for (int64_t k = 0; k < nblk; ++k) h_pofs.push_back(cofs[(size_t)k * S + s]);
        rg_off[bt] = (int64_t)h_rg.size();
        for (int64_t k = 0; k <= nblk; ++k) h_rg.push_back(rgb[k]);
        qo_off[bt] = (int64_t)h_qoff.size();
        for (int64_t k = 0; k < nblk; ++k) {
            int ml = 0;
            for (int l = 0; l < RB; ++l) ml = std::max<int>(ml, (int)(rp[rbase + k * RB + l + 1] - rp[rbase + k * RB + l]));
            ml = (ml + 7) & ~7;
            h_qoff.push_back((uint32_t)h_qs.size());
            const size_t q0 = h_qs.size();
            h_qs.resize(q0 + (size_t)ml * RB, 0);
            for (int l = 0; l < RB; ++l) {
                const int64_t r = k * RB + l;
                for (int64_t e = rp[rbase + r], kk = 0; e < rp[rbase + r + 1]; ++e, ++kk)
                    h_qs[q0 + (size_t)(kk / 8) * RB * 8 + (size_t)l * 8 + kk % 8] =
                        (uint16_t)(slot[e - rp[rbase]] - rgb[k]);
            }
        }
        h_qoff.push_back((uint32_t)h_qs.size());
    }
    printf("layout: list %zu entries, qs %zu u16 (%.2f per entry), pofs %zu, p max %lld\n", h_list.size(),
           h_qs.size(), (double)h_qs.size() / E, h_pofs.size(), (long long)pmax);
    // device
    auto up = [](const auto &v) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        T *d = nullptr;
        CK(hipMalloc(&d, v.size() * sizeof(T) + 256));
        CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
        return d;
    };
    int64_t *d_rp = up(rp);
    int32_t *d_col = up(col);
    float *d_val = up(val), *d_lab = up(lab);
    uint32_t *d_lbeg = up(h_lbeg), *d_list = up(h_list), *d_pofs = up(h_pofs), *d_rg = up(h_rg),
             *d_qoff = up(h_qoff);
    float *d_lval = up(h_lval);
    uint16_t *d_qs = up(h_qs);
    std::vector<float> hw(D);
    for (int64_t j = 0; j < D; ++j) hw[j] = ((float)rng.below(20001) - 10000.0f) * 1e-4f;
    float *d_w = up(hw);
    float *d_p, *d_r1, *d_r2;
    CK(hipMalloc(&d_p, (pmax + 64) * 4));
    CK(hipMalloc(&d_r1, B * 4));
    CK(hipMalloc(&d_r2, B * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto batch = [&](int bt) {
        dlr::DevBatch b{d_rp + (int64_t)bt * B, d_col, d_val, d_lab + (int64_t)bt * B, B, rp[(bt + 1) * B] - rp[bt * B]};
        return b;
    };
    const int split = argc > 4 ? atoi(argv[4]) : 8;
    auto prod = [&](int bt) {
        const unsigned g = (unsigned)(((S + 7) / 8) * 8 * split);
#define KP(SP, NT, U) \
        if (split == SP) hipLaunchKernelGGL((k_prod<NT, SP, U>), dim3(g), dim3(NT), 0, 0, d_lbeg + lb_off[bt], d_list, \
                           d_lval, d_pofs + pofs_off[bt], (int)nblk, (int)S, d_w, D, d_p);
        KP(1, 1024, 16) KP(2, 512, 16) KP(4, 256, 16) KP(8, 256, 8) KP(16, 256, 4) KP(3, 256, 16) KP(6, 256, 8)
#undef KP
    };
    auto m2 = [&](int bt) {
        hipLaunchKernelGGL(k_m2<8>, dim3((unsigned)(nblk / 4)), dim3(256), 0, 0, d_rg + rg_off[bt], d_qoff + qo_off[bt],
                           d_qs, d_rp + (int64_t)bt * B, d_lab + (int64_t)bt * B, B, d_p, d_r2);
    };
    // correctness, every batch
    int bad = 0;
    for (int bt = 0; bt < NB; ++bt) {
        CK(dlr::launch_margin_residual(batch(bt), d_w, d_r1, 0));
        prod(bt);
        m2(bt);
        CK(hipDeviceSynchronize());
        std::vector<float> a(B), b(B);
        CK(hipMemcpy(a.data(), d_r1, B * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), d_r2, B * 4, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < B; ++i) bad += memcmp(&a[i], &b[i], 4) != 0;
    }
    printf("bitwise mismatches vs production margin: %d\n", bad);
    auto timeit = [&](const char *name, auto fn) {
        for (int k = 0; k < 20; ++k) fn(k % NB);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < reps; ++k) fn(k % NB);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-40s %8.2f us per launch-set\n", name, ms * 1000.0f / reps);
    };
    timeit("production margin (k_margin_residual)", [&](int bt) { (void)dlr::launch_margin_residual(batch(bt), d_w, d_r1, 0); });
    timeit("pass 1 products (k_prod)", [&](int bt) { prod(bt); });
    timeit("pass 2 row sums (k_m2)", [&](int bt) { m2(bt); });
#define M2V(DMA, HALF) [&](int bt) { hipLaunchKernelGGL((k_m2v<8, DMA, HALF>), dim3((unsigned)(nblk / (HALF ? 2 : 4))), dim3(256), 0, 0, \
        d_rg + rg_off[bt], d_qoff + qo_off[bt], d_qs, d_rp + (int64_t)bt * B, d_lab + (int64_t)bt * B, B, d_p, d_r2); }
    timeit("pass 2 variant plain", M2V(false, false));
    timeit("pass 2 variant DMA", M2V(true, false));
    timeit("pass 2 variant 2 waves/block", M2V(false, true));
    timeit("pass 2 variant DMA + 2 waves/block", M2V(true, true));
    {
        // bitwise check of the variants (products from the last pass 1 of batch 0)
        prod(0);
        hipLaunchKernelGGL(k_m2<8>, dim3((unsigned)(nblk / 4)), dim3(256), 0, 0, d_rg + rg_off[0], d_qoff + qo_off[0], d_qs, d_rp, d_lab, B, d_p, d_r1);
        std::vector<float> a(B), b(B);
        CK(hipMemcpy(a.data(), d_r1, B * 4, hipMemcpyDeviceToHost));
        const char *nm[4] = {"plain", "DMA", "half", "DMA+half"};
        for (int v = 0; v < 4; ++v) {
            if (v == 0) M2V(false, false)(0);
            if (v == 1) M2V(true, false)(0);
            if (v == 2) M2V(false, true)(0);
            if (v == 3) M2V(true, true)(0);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(b.data(), d_r2, B * 4, hipMemcpyDeviceToHost));
            printf("variant %s: %s\n", nm[v], memcmp(a.data(), b.data(), B * 4) ? "MISMATCH" : "bitwise equal");
        }
    }
    timeit("pass 1 + pass 2", [&](int bt) { prod(bt); m2(bt); });
    const unsigned g4 = (unsigned)(((S + 7) / 8) * 8);
    timeit("k_prod abl1 contiguous stores", [&](int bt) { hipLaunchKernelGGL((k_prod<1024, 1, 16, 1>), dim3(g4), dim3(1024), 0, 0, d_lbeg + lb_off[bt], d_list, d_lval, d_pofs + pofs_off[bt], (int)nblk, (int)S, d_w, D, d_p); });
    timeit("k_prod abl2 no w gather", [&](int bt) { hipLaunchKernelGGL((k_prod<1024, 1, 16, 2>), dim3(g4), dim3(1024), 0, 0, d_lbeg + lb_off[bt], d_list, d_lval, d_pofs + pofs_off[bt], (int)nblk, (int)S, d_w, D, d_p); });
    return bad != 0;
}
