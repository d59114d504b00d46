// kbench.hip -- kernel-design microbenchmarks for the C2 train step
// (B = 65,536 rows x 50 nnz over D = 1M features).  Development tool only:
// times candidate margin / gradient kernels against the production ones
// (dlr_kernels.hip, included below) and checks them bitwise.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I dist-lr_amd/csrc \
//         tools/kbench/kbench.hip -o tools/kbench/kbench && ./tools/kbench/kbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define DLR_STAMPS 1
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

__device__ __forceinline__ float sig(float z) {
    const double e = exp(-(double)z);
    return (float)(1.0 / (1.0 + e));
}

// ---------------- micro: streams and gathers
__global__ __launch_bounds__(256) void mb_empty(float *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && out[0] == 12345.0f) out[1] = 1.0f;
}

// Streams n4 float4s (grid-stride) to evict L2 and the Infinity Cache.
__global__ __launch_bounds__(256) void mb_flush(const float4 *buf, int64_t n4, float *out) {
    float acc = 0.f;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n4; t += (int64_t)gridDim.x * 256) {
        const float4 v = buf[t];
        acc += v.x + v.y + v.z + v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void mb_stream(const int4 *idx, const float4 *val, float *out, int64_t n4) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n4) return;
    const int4 i = idx[t];
    const float4 v = val[t];
    out[t] = (float)(i.x + i.y + i.z + i.w) + v.x + v.y + v.z + v.w;
}

__global__ __launch_bounds__(256) void mb_gather(const int4 *idx, const float *table, unsigned mask, float *out,
                                                 int64_t n4) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n4) return;
    const int4 i = idx[t];
    out[t] = table[i.x & mask] + table[i.y & mask] + table[i.z & mask] + table[i.w & mask];
}

// Many gathers in flight per lane: G int4 index loads (grid-strided,
// coalesced), then 4G gathers.
template <int G>
__global__ __launch_bounds__(256) void mb_gather_g(const int4 *idx, const float *table, unsigned mask, float *out,
                                                   int64_t n4) {
    const int64_t nth = (int64_t)gridDim.x * 256;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    float s = 0.0f;
    for (int64_t base = t; base < n4; base += nth * G) {
        int4 iv[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t q = base + g * nth;
            iv[g] = q < n4 ? idx[q] : make_int4(0, 0, 0, 0);
        }
        float x[G][4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            x[g][0] = table[iv[g].x & mask];
            x[g][1] = table[iv[g].y & mask];
            x[g][2] = table[iv[g].z & mask];
            x[g][3] = table[iv[g].w & mask];
        }
#pragma unroll
        for (int g = 0; g < G; ++g) s += x[g][0] + x[g][1] + x[g][2] + x[g][3];
    }
    out[t] = s;
}

// Ablation copy of dlr::k_grad_lds (FILL = 8, not fused): ABL bit 0 skips
// the residual gathers (products = values), bit 1 skips the per-column read
// loop (one product per lane), bit 2 runs phase 0 only, bit 3 skips the fill
// waits (garbage residuals; timing only).
template <int ABL>
__global__ __launch_bounds__(1024) void mb_grad_abl(dlr::DevPcsc pc, int64_t D, const float *__restrict__ resid,
                                                    float *__restrict__ w, float *__restrict__ gout, float Bf,
                                                    double Bd, float C) {
    constexpr int R = 8 * 4096, NG = 4, W = 16;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *s_r = smem;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x / 64;
    float *s_p = smem + R + wv * (256 + 8);
    const int P = (ABL & 4) ? 1 : pc.phases;
    const int64_t ng = (D + 63) / 64;
    const int64_t gfirst = (int64_t)blockIdx.x * (W * NG) + wv;
    unsigned bs[NG][2], off[NG][2], cnt[NG][2];
    float acc[NG], wj[NG];
    ushort4 rq[NG][2];
    float4 vq[NG][2];
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t g = gfirst + W * gi;
        const bool gv = g < ng;
        const int64_t gc = gv ? g : ng - 1;
        const int64_t j = g * 64 + lane;
        const bool ok = gv && j < D;
        wj[gi] = w[j < D ? j : D - 1];
        acc[gi] = 0.0f;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int64_t blk = gc * pc.phases + (p < pc.phases ? p : pc.phases - 1);
            bs[gi][p] = pc.base[blk];
            const unsigned hi = pc.ends[blk * 64 + lane];
            const unsigned lo = pc.ends[blk * 64 + (lane ? lane - 1 : 0)];
            off[gi][p] = lane ? lo : 0u;
            cnt[gi][p] = (ok && p < P) ? hi - (lane ? lo : 0u) : 0u;
        }
    }
#pragma unroll
    for (int gi = 0; gi < NG; ++gi)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const unsigned e = bs[gi][p] + lane * 4;
            rq[gi][p] = *reinterpret_cast<const ushort4 *>(pc.row + e);
            vq[gi][p] = *reinterpret_cast<const float4 *>(pc.val + e);
        }
    auto fill = [&](int64_t lo) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const int o = (f * W + wv) * 64 * 4;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(resid + lo + o + lane * 4),
                                             (__attribute__((address_space(3))) void *)(s_r + o), 16, 0, 0);
        }
    };
    if (!(ABL & 8)) fill(0);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        if (p >= P) break;
        if (p > 0) {
            __syncthreads();
            if (!(ABL & 8)) fill((int64_t)p * R);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            if (gfirst + W * gi >= ng) break;
            const ushort4 r4 = rq[gi][p];
            const float4 v4 = vq[gi][p];
            float4 q;
            if (ABL & 1) {
                q = v4;
                q.x += (float)r4.x;
            } else {
                q.x = s_r[r4.x] * v4.x;
                q.y = s_r[r4.y] * v4.y;
                q.z = s_r[r4.z] * v4.z;
                q.w = s_r[r4.w] * v4.w;
            }
            *reinterpret_cast<float4 *>(s_p + lane * 4) = q;
            __builtin_amdgcn_wave_barrier();
            const unsigned o = off[gi][p], c = cnt[gi][p];
            const float *sp = s_p + o;
            float a = acc[gi];
            if (ABL & 2) {
                a = a + sp[0];
            } else {
                float x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = sp[u];
                asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]));
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const bool take = (unsigned)u < c;
                    if (__builtin_amdgcn_ballot_w64(take) == 0) break;
                    const float t = a + x[u];
                    a = take ? t : a;
                }
            }
            acc[gi] = a;
            __builtin_amdgcn_wave_barrier();
        }
    }
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t j = (gfirst + W * gi) * 64 + lane;
        if (gfirst + W * gi >= ng || j >= D) continue;
        const float cw = C * wj[gi];
        const float l2 = cw / Bf;
        gout[j] = (float)((double)acc[gi] / Bd + (double)l2);
    }
}

// LDS random 4-B gathers: 1,024 threads, each NR reads per round from a
// 128 KiB table at LCG addresses.
template <int NR>
__global__ __launch_bounds__(1024) void mb_lds_gather(float *out, int rounds, unsigned mask) {
    extern __shared__ float tab[];
    for (int i = threadIdx.x; i < 32768; i += 1024) tab[i] = (float)i;
    __syncthreads();
    unsigned x = threadIdx.x * 2654435761u + blockIdx.x;
    float acc = 0.f;
    for (int r = 0; r < rounds; ++r) {
        float v[NR];
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            x = x * 1664525u + 1013904223u;
            v[k] = tab[(x >> 8) & mask];
        }
#pragma unroll
        for (int k = 0; k < NR; ++k) acc += v[k];
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

// Dense L2-only update variants (C5's HBM-bound pass), W = 1 formula.
template <bool NT, int U>
__global__ __launch_bounds__(256) void mb_l2(float *__restrict__ w, int64_t n4, float Bf, float lr, float C) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q0 < n4; q0 += stride * U) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = q0 + u * stride;
            if (q < n4) v[u] = NT ? __builtin_nontemporal_load(reinterpret_cast<const f4 *>(w) + q)
                                  : reinterpret_cast<const f4 *>(w)[q];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = q0 + u * stride;
            if (q >= n4) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float cw = C * v[u][k];
                const float l2 = cw / Bf;
                const float st = lr * l2;
                v[u][k] = v[u][k] - st;
            }
            if (NT)
                __builtin_nontemporal_store(v[u], reinterpret_cast<f4 *>(w) + q);
            else
                reinterpret_cast<f4 *>(w)[q] = v[u];
        }
    }
}

// ---------------- K2 candidates
// The production margin kernel with non-temporal loads of the col/val
// stream (so the streamed lines do not evict w from L2).
template <typename IdxT, bool NT>
__device__ __forceinline__ float osd_nt(int64_t e0, int64_t e1, int64_t a, int64_t b, int lane,
                                        const IdxT *__restrict__ idx, const float *__restrict__ val,
                                        const float *__restrict__ table, float *lds) {
    using IV = typename dlr::Vec4<IdxT>::type;
    constexpr int kWin = 1024, kVec = 4, kWave = 64;
    constexpr int kT = kWin / (kVec * kWave);
    constexpr int kChunk = kVec * kWave;
    const int64_t base = e0 & ~int64_t(kVec - 1);
    float acc = 0.0f;
    for (int64_t ws = base; ws < e1; ws += kWin) {
        const int64_t left = e1 - ws;
        IV iv[kT];
        float4 v[kT];
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            if (t * kChunk < left) {
                const int64_t e = ws + t * kChunk + lane * kVec;
                const int64_t ec = e < e1 ? e : ws + t * kChunk;
                if (NT) {
                    typedef int vi4 __attribute__((ext_vector_type(4)));
                    typedef float vf4 __attribute__((ext_vector_type(4)));
                    const vi4 a4 = __builtin_nontemporal_load(reinterpret_cast<const vi4 *>(idx + ec));
                    const vf4 b4 = __builtin_nontemporal_load(reinterpret_cast<const vf4 *>(val + ec));
                    iv[t].x = a4.x; iv[t].y = a4.y; iv[t].z = a4.z; iv[t].w = a4.w;
                    v[t].x = b4.x; v[t].y = b4.y; v[t].z = b4.z; v[t].w = b4.w;
                } else {
                    iv[t] = *reinterpret_cast<const IV *>(idx + ec);
                    v[t] = *reinterpret_cast<const float4 *>(val + ec);
                }
            }
        }
        float g[kT][kVec];
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            if (t * kChunk < left) {
                const int64_t e = ws + t * kChunk + lane * kVec;
                const unsigned i0 = (e >= e0 && e < e1) ? (unsigned)iv[t].x : 0u;
                const unsigned i1 = (e + 1 >= e0 && e + 1 < e1) ? (unsigned)iv[t].y : 0u;
                const unsigned i2 = (e + 2 >= e0 && e + 2 < e1) ? (unsigned)iv[t].z : 0u;
                const unsigned i3 = (e + 3 >= e0 && e + 3 < e1) ? (unsigned)iv[t].w : 0u;
                g[t][0] = table[i0];
                g[t][1] = table[i1];
                g[t][2] = table[i2];
                g[t][3] = table[i3];
            }
        }
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            if (t * kChunk < left) {
                const int o = t * kChunk + lane * kVec;
                const int64_t e = ws + o;
                float4 p;
                p.x = (e >= e0 && e < e1) ? g[t][0] * v[t].x : 0.0f;
                p.y = (e + 1 >= e0 && e + 1 < e1) ? g[t][1] * v[t].y : 0.0f;
                p.z = (e + 2 >= e0 && e + 2 < e1) ? g[t][2] * v[t].z : 0.0f;
                p.w = (e + 3 >= e0 && e + 3 < e1) ? g[t][3] * v[t].w : 0.0f;
                *reinterpret_cast<float4 *>(lds + o) = p;
            }
        }
        dlr::wave_sync();
        const int64_t lo = a > ws ? a : ws;
        const int64_t hi = b < ws + kWin ? b : ws + kWin;
        int o = (int)(lo - ws);
        const int oe = (int)(hi - ws);
        for (; o + 8 <= oe; o += 8) {
            const float x0 = lds[o], x1 = lds[o + 1], x2 = lds[o + 2], x3 = lds[o + 3];
            const float x4 = lds[o + 4], x5 = lds[o + 5], x6 = lds[o + 6], x7 = lds[o + 7];
            acc = acc + x0; acc = acc + x1; acc = acc + x2; acc = acc + x3;
            acc = acc + x4; acc = acc + x5; acc = acc + x6; acc = acc + x7;
        }
        for (; o < oe; ++o) acc = acc + lds[o];
        dlr::wave_sync();
    }
    return acc;
}
template <int SEG, bool NT>
__global__ __launch_bounds__(256) void k2_nt(dlr::DevBatch bt, const float *__restrict__ w, float *__restrict__ resid) {
    __shared__ float s_p[4][1024];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x / 64;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wv) * SEG;
    if (row0 >= bt.rows) return;
    const int64_t my = row0 + lane;
    const bool valid = lane < SEG && my < bt.rows;
    const float y = valid ? bt.label[my] : 0.0f;
    const int64_t rlast = min(row0 + SEG, bt.rows);
    const int64_t e0 = bt.row_ptr[row0], e1 = bt.row_ptr[rlast];
    const int64_t a = valid ? bt.row_ptr[my] : e1, b = valid ? bt.row_ptr[my + 1] : e1;
    const float z = osd_nt<int32_t, NT>(e0, e1, a, b, lane, bt.col, bt.val, w, s_p[wv]);
    if (valid) resid[my] = sig(z) - y;
}

// Lane per row, entries read straight from the row (4 at a time), U in flight.
template <int U>
__global__ __launch_bounds__(256) void k2_lpr(dlr::DevBatch bt, const float *__restrict__ w,
                                              float *__restrict__ resid) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= bt.rows) return;
    const int64_t a = bt.row_ptr[i], b = bt.row_ptr[i + 1];
    const float y = bt.label[i];
    float acc = 0.0f;
    for (int64_t k = a; k < b; k += U) {
        int c[U];
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            c[u] = bt.col[k + u];
            v[u] = bt.val[k + u];
        }
        float g[U];
#pragma unroll
        for (int u = 0; u < U; ++u) g[u] = w[(k + u < b) ? c[u] : 0];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k + u < b) acc = acc + g[u] * v[u];
    }
    resid[i] = sig(acc) - y;
}

// Column-split margin pass: row i's entries in this half are [row_ptr[i],
// row_ptr[i+1]); the sum continues from zin[i] (pass B) and either stores
// the partial (pass A) or finishes sigma - y (pass B).
template <int SEG, bool FIRST, bool LAST>
__global__ __launch_bounds__(256) void k2_split(dlr::DevBatch bt, const float *__restrict__ w,
                                                const float *__restrict__ zin, float *__restrict__ out) {
    __shared__ float s_p[4][1024];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x / 64;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wv) * SEG;
    if (row0 >= bt.rows) return;
    const int64_t my = row0 + lane;
    const bool valid = lane < SEG && my < bt.rows;
    const int64_t rlast = min(row0 + SEG, bt.rows);
    const int64_t e0 = bt.row_ptr[row0], e1 = bt.row_ptr[rlast];
    const int64_t a = valid ? bt.row_ptr[my] : e1, b = valid ? bt.row_ptr[my + 1] : e1;
    const float z0 = (!FIRST && valid) ? zin[my] : 0.0f;
    float z = dlr::ordered_segment_dot<int32_t>(e0, e1, a, b, lane, bt.col, bt.val, w, s_p[wv]);
    // ordered_segment_dot starts from 0: for pass B re-add in order is NOT
    // the same as continuing -- so pass B below uses osd_from instead.
    (void)z0;
    if (valid) out[my] = LAST ? sig(z) - bt.label[my] : z;
}

// ordered segment dot continuing from acc0 (same as dlr::ordered_segment_dot
// but with an initial value): the column-split pass B.
template <int SEG>
__global__ __launch_bounds__(256) void k2_splitB(dlr::DevBatch bt, const float *__restrict__ w,
                                                 const float *__restrict__ zin, float *__restrict__ resid) {
    __shared__ float s_p[4][1024];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x / 64;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wv) * SEG;
    if (row0 >= bt.rows) return;
    const int64_t my = row0 + lane;
    const bool valid = lane < SEG && my < bt.rows;
    const int64_t rlast = min(row0 + SEG, bt.rows);
    const int64_t e0 = bt.row_ptr[row0], e1 = bt.row_ptr[rlast];
    const int64_t a = valid ? bt.row_ptr[my] : e1, b = valid ? bt.row_ptr[my + 1] : e1;
    float acc = valid ? zin[my] : 0.0f;
    // same window loop as the production kernel, summing into acc
    float *lds = s_p[wv];
    const int64_t base = e0 & ~int64_t(3);
    for (int64_t ws = base; ws < e1; ws += 1024) {
        const int64_t left = e1 - ws;
        int4 iv[4];
        float4 v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t * 256 < left) {
                const int64_t e = ws + t * 256 + lane * 4;
                const int64_t ec = e < e1 ? e : ws + t * 256;
                iv[t] = dlr::load_stream(reinterpret_cast<const int4 *>(bt.col + ec));
                v[t] = dlr::load_stream(reinterpret_cast<const float4 *>(bt.val + ec));
            }
        float g[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t * 256 < left) {
                const int64_t e = ws + t * 256 + lane * 4;
                g[t][0] = w[(e >= e0 && e < e1) ? iv[t].x : 0];
                g[t][1] = w[(e + 1 >= e0 && e + 1 < e1) ? iv[t].y : 0];
                g[t][2] = w[(e + 2 >= e0 && e + 2 < e1) ? iv[t].z : 0];
                g[t][3] = w[(e + 3 >= e0 && e + 3 < e1) ? iv[t].w : 0];
            }
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t * 256 < left) {
                const int o = t * 256 + lane * 4;
                const int64_t e = ws + o;
                float4 p;
                p.x = (e >= e0 && e < e1) ? g[t][0] * v[t].x : 0.0f;
                p.y = (e + 1 >= e0 && e + 1 < e1) ? g[t][1] * v[t].y : 0.0f;
                p.z = (e + 2 >= e0 && e + 2 < e1) ? g[t][2] * v[t].z : 0.0f;
                p.w = (e + 3 >= e0 && e + 3 < e1) ? g[t][3] * v[t].w : 0.0f;
                *reinterpret_cast<float4 *>(lds + o) = p;
            }
        dlr::wave_sync();
        const int64_t lo = a > ws ? a : ws;
        const int64_t hi = b < ws + 1024 ? b : ws + 1024;
        for (int o = (int)(lo - ws); o < (int)(hi - ws); ++o) acc = acc + lds[o];
        dlr::wave_sync();
    }
    if (valid) resid[my] = sig(acc) - bt.label[my];
}

// ---------------- K3 candidates
// Lane per column: the column's segment read straight (U entries at a time).
template <int U, bool FUSED>
__global__ __launch_bounds__(256) void k3_lpc(dlr::DevCsc cs, const uint16_t *__restrict__ crow, int64_t D,
                                              const float *__restrict__ resid, float *__restrict__ w,
                                              float *__restrict__ gout, float Bf, double Bd, float lr, float C) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= D) return;
    const uint32_t a = cs.ptr[j], b = cs.ptr[j + 1];
    const float wj = w[j];
    float acc = 0.0f;
    for (uint32_t k = a; k < b; k += U) {
        unsigned r[U];
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            r[u] = crow[k + u];
            v[u] = cs.val[k + u];
        }
        float rr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) rr[u] = resid[r[u]];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k + u < b) acc = acc + rr[u] * v[u];
    }
    const float cw = C * wj;
    const float l2 = cw / Bf;
    const float g = (float)((double)acc / Bd + (double)l2);
    if (FUSED) {
        const float step = lr * g;
        w[j] = wj - step;
    } else {
        gout[j] = g;
    }
}

// K3 with the residual table in LDS: one 1024-thread workgroup per CU,
// rows processed in phases of R rows (R*4 bytes of LDS).  Lane per column;
// each lane prefetches U entries of its column into registers, then per
// phase adds (in order) those whose row falls in the phase.  Columns with
// more than U entries continue from global memory.
template <int U, int NG, bool FUSED>
__global__ __launch_bounds__(1024) void k3_lds(dlr::DevCsc cs, const uint16_t *__restrict__ crow, int64_t D, int64_t B,
                                               int R, int gpw, const float *__restrict__ resid, float *__restrict__ w,
                                               float *__restrict__ gout, float Bf, double Bd, float lr, float C) {
    extern __shared__ __attribute__((aligned(16))) float s_r[];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int64_t g0 = (int64_t)blockIdx.x * gpw;
    unsigned k[NG], b[NG], k0[NG];
    float acc[NG];
    unsigned short rr[NG][U];
    float vv[NG][U];
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t g = g0 + wv + 16 * gi;
        const int64_t j = g * 64 + lane;
        const bool ok = (wv + 16 * gi) < gpw && j < D;
        k[gi] = ok ? cs.ptr[j] : 0u;
        b[gi] = ok ? cs.ptr[j + 1] : 0u;
        k0[gi] = k[gi];
        acc[gi] = 0.0f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = k[gi] + u < b[gi];
            rr[gi][u] = in ? crow[k[gi] + u] : (unsigned short)0;
            vv[gi][u] = in ? cs.val[k[gi] + u] : 0.0f;
        }
    }
    for (int64_t lo = 0; lo < B; lo += R) {
        const int n = (int)min((int64_t)R, B - lo);
        __syncthreads();
        for (int i = threadIdx.x * 4; i < n; i += 4096) {
            if (i + 4 <= n) {
                *reinterpret_cast<float4 *>(s_r + i) = *reinterpret_cast<const float4 *>(resid + lo + i);
            } else {
                for (int q = i; q < n; ++q) s_r[q] = resid[lo + q];
            }
        }
        __syncthreads();
        const unsigned hi = (unsigned)(lo + n);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned e = k0[gi] + u;
                if (e < b[gi] && e >= k[gi] && rr[gi][u] < hi) {
                    acc[gi] = acc[gi] + s_r[rr[gi][u] - (unsigned)lo] * vv[gi][u];
                    k[gi] = e + 1;
                }
            }
            // overflow: entries beyond the prefetched U
            while (k[gi] >= k0[gi] + U && k[gi] < b[gi]) {
                const unsigned r = crow[k[gi]];
                if (r >= hi) break;
                acc[gi] = acc[gi] + s_r[r - (unsigned)lo] * cs.val[k[gi]];
                k[gi] += 1;
            }
        }
    }
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t g = g0 + wv + 16 * gi;
        const int64_t j = g * 64 + lane;
        if ((wv + 16 * gi) >= gpw || j >= D) continue;
        const float wj = w[j];
        const float cw = C * wj;
        const float l2 = cw / Bf;
        const float gr = (float)((double)acc[gi] / Bd + (double)l2);
        if (FUSED) {
            const float step = lr * gr;
            w[j] = wj - step;
        } else {
            gout[j] = gr;
        }
    }
}

// K3 windowed with the residual table in LDS (phases of R rows).  A wave
// owns column groups of 64 (lane = column); per phase and per window of
// kW entries it loads crow/cval entry-parallel (ushort4 + float4), forms
// products for entries whose row is in the phase (others: a sentinel), and
// each lane continues its column's ordered sum from where the previous
// phase stopped, until the sentinel (rows ascend within a column, so the
// in-phase entries are contiguous).
constexpr unsigned kSentinel = 0x7FBADBADu;
__device__ unsigned long long *g_stamp_kb = nullptr;  // diagnostic builds only (MODE 9)
__device__ __forceinline__ void stamp(int slot) {
    if (threadIdx.x == 0) {
        unsigned long long t = __builtin_amdgcn_s_memrealtime();
        g_stamp_kb[blockIdx.x * 8 + slot] = t;
    }
}
template <int NG, int kW, bool FUSED>
__global__ __launch_bounds__(1024) void k3_ldsw(dlr::DevCsc cs, const uint16_t *__restrict__ crow, int64_t D,
                                                int64_t B, int R, int gpw, const float *__restrict__ resid,
                                                float *__restrict__ w, float *__restrict__ gout, float Bf, double Bd,
                                                float lr, float C) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *s_r = smem;                       // R floats
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    float *s_p = smem + R + wv * kW;         // kW floats per wave
    const int64_t g0 = (int64_t)blockIdx.x * gpw;
    unsigned pos[NG], end[NG];
    float acc[NG];
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t j = (g0 + wv + 16 * gi) * 64 + lane;
        const bool ok = (wv + 16 * gi) < gpw && j < D;
        pos[gi] = ok ? cs.ptr[j] : 0u;
        end[gi] = ok ? cs.ptr[j + 1] : 0u;
        acc[gi] = 0.0f;
    }
    for (int64_t lo = 0; lo < B; lo += R) {
        const int n = (int)min((int64_t)R, B - lo);
        __syncthreads();
        for (int i = threadIdx.x * 4; i < n; i += 4096) {
            if (i + 4 <= n) {
                *reinterpret_cast<float4 *>(s_r + i) = *reinterpret_cast<const float4 *>(resid + lo + i);
            } else {
                for (int q = i; q < n; ++q) s_r[q] = resid[lo + q];
            }
        }
        __syncthreads();
        const unsigned ulo = (unsigned)lo, uhi = (unsigned)(lo + n);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            if (wv + 16 * gi >= gpw) break;  // wave-uniform
            const int64_t gcol = (g0 + wv + 16 * gi) * 64;
            if (gcol >= D) break;
            const int64_t jl = min(gcol + 64, D);
            const unsigned e0 = cs.ptr[gcol], e1 = cs.ptr[jl];
            bool open = pos[gi] < end[gi];
            for (unsigned ws = e0 & ~3u; ws < e1; ws += kW) {
                // (1) loads + (2) LDS gathers -> products (sentinel if out of phase)
#pragma unroll
                for (int t = 0; t < kW / 256; ++t) {
                    const unsigned o = t * 256 + lane * 4;
                    if (ws + t * 256 < e1) {
                        const unsigned e = ws + o;
                        const ushort4 r4 = *reinterpret_cast<const ushort4 *>(crow + e);
                        const float4 v4 = *reinterpret_cast<const float4 *>(cs.val + e);
                        float4 p;
                        const unsigned r0 = r4.x, r1 = r4.y, r2 = r4.z, r3 = r4.w;
                        p.x = (r0 >= ulo && r0 < uhi) ? s_r[r0 - ulo] * v4.x : __uint_as_float(kSentinel);
                        p.y = (r1 >= ulo && r1 < uhi) ? s_r[r1 - ulo] * v4.y : __uint_as_float(kSentinel);
                        p.z = (r2 >= ulo && r2 < uhi) ? s_r[r2 - ulo] * v4.z : __uint_as_float(kSentinel);
                        p.w = (r3 >= ulo && r3 < uhi) ? s_r[r3 - ulo] * v4.w : __uint_as_float(kSentinel);
                        *reinterpret_cast<float4 *>(s_p + o) = p;
                    }
                }
                dlr::wave_sync();
                // (3) ordered continuation of this lane's column
                if (open) {
                    unsigned o = pos[gi] > ws ? pos[gi] - ws : 0u;
                    const unsigned oe = min(end[gi], ws + kW) - ws;
                    if (pos[gi] < ws + kW) {
                        float a = acc[gi];
                        for (; o < oe; ++o) {
                            const float x = s_p[o];
                            if (__float_as_uint(x) == kSentinel) {
                                open = false;
                                break;
                            }
                            a = a + x;
                        }
                        acc[gi] = a;
                        pos[gi] = ws + o;
                    }
                }
                dlr::wave_sync();
            }
        }
    }
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t j = (g0 + wv + 16 * gi) * 64 + lane;
        if ((wv + 16 * gi) >= gpw || j >= D) continue;
        const float wj = w[j];
        const float cw = C * wj;
        const float l2 = cw / Bf;
        const float gr = (float)((double)acc[gi] / Bd + (double)l2);
        if (FUSED) {
            const float step = lr * gr;
            w[j] = wj - step;
        } else {
            gout[j] = gr;
        }
    }
}

// K3 "prefetch": every load a wave needs is issued up front -- the first
// window (256 entries) of each of its NG column groups, w, and its share of
// the residual fills -- so the kernel pays about one memory latency; the
// windows stay in registers across the row phases.  Groups with more than
// one window continue through a separate slow path (its own loads), so the
// fast path never waits for the next phase's fill loads.
template <int NG, int FILL, bool FUSED, int MODE = 0>
__global__ __launch_bounds__(1024) void k3_pf(dlr::DevCsc cs, const uint16_t *__restrict__ crow, int64_t D,
                                              int64_t B, int gpw, const float *__restrict__ resid,
                                              float *__restrict__ w, float *__restrict__ gout, float Bf, double Bd,
                                              float lr, float C) {
    constexpr int R = FILL * 4096;
    constexpr int kW = 256;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *s_r = smem;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    float *s_p = smem + R + wv * kW;
    const int64_t g0 = (int64_t)blockIdx.x * gpw;
    unsigned pos[NG], end[NG], ws0[NG], e1[NG];
    float acc[NG], wj[NG];
    bool open[NG];
    ushort4 rq[NG];
    float4 vq[NG];
    // Prologue: every load unconditional (clamped, in-bounds addresses;
    // values selected afterwards) -- a load inside a divergent branch makes
    // the compiler wait for it at the join.
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t gcol = (g0 + wv + 16 * gi) * 64;
        const bool gv = (wv + 16 * gi) < gpw && gcol < D;
        const int64_t gc = gcol < D ? gcol : D;
        const int64_t j = gcol + lane;
        const bool ok = gv && j < D;
        const int64_t jc = j < D ? j : D - 1;
        const unsigned p0 = cs.ptr[jc], p1 = cs.ptr[jc + 1];
        const unsigned e0 = cs.ptr[gc], e1v = cs.ptr[min(gc + 64, D)];
        const float wv_ = w[jc];
        pos[gi] = ok ? p0 : 0u;
        end[gi] = ok ? p1 : 0u;
        e1[gi] = gv ? e1v : 0u;
        ws0[gi] = gv ? (e0 & ~3u) : 0u;
        acc[gi] = 0.0f;
        wj[gi] = wv_;
    }
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const unsigned e = ws0[gi] + lane * 4;
        const bool in = e < e1[gi];
        const unsigned ec = in ? e : (e1[gi] & ~3u);
        const ushort4 r4 = *reinterpret_cast<const ushort4 *>(crow + ec);
        const float4 v4 = *reinterpret_cast<const float4 *>(cs.val + ec);
        rq[gi] = in ? r4 : make_ushort4(0, 0, 0, 0);
        vq[gi] = in ? v4 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 fr[FILL];
    auto fill_load = [&](int64_t lo) {
#pragma unroll
        for (int f = 0; f < FILL; ++f) {
            const int64_t i = lo + (int64_t)(f * 1024 + threadIdx.x) * 4;
            fr[f] = *reinterpret_cast<const float4 *>(resid + i);  // resid padded to a multiple of R
        }
    };
    // products of one 256-entry window (sentinel outside the phase), then
    // each lane continues its column's ordered sum
    auto window = [&](const ushort4 r4, const float4 v4, unsigned ws, unsigned ulo, unsigned uhi, int gi) {
        float4 p;
        const unsigned r0 = r4.x, r1 = r4.y, r2 = r4.z, r3 = r4.w;
        p.x = (r0 >= ulo && r0 < uhi) ? s_r[r0 - ulo] * v4.x : __uint_as_float(kSentinel);
        p.y = (r1 >= ulo && r1 < uhi) ? s_r[r1 - ulo] * v4.y : __uint_as_float(kSentinel);
        p.z = (r2 >= ulo && r2 < uhi) ? s_r[r2 - ulo] * v4.z : __uint_as_float(kSentinel);
        p.w = (r3 >= ulo && r3 < uhi) ? s_r[r3 - ulo] * v4.w : __uint_as_float(kSentinel);
        *reinterpret_cast<float4 *>(s_p + lane * 4) = p;
        dlr::wave_sync();
        if (open[gi] && pos[gi] < ws + kW) {
            unsigned o = pos[gi] - ws;
            const unsigned oe = min(end[gi], ws + kW) - ws;
            float a = acc[gi];
            bool op = true;
            while (op && o < oe) {
                float x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = s_p[min(o + u, (unsigned)kW - 1)];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const bool take = op && (o < oe) && __float_as_uint(x[u]) != kSentinel;
                    if (take) a = a + x[u];
                    op = op && (o >= oe || take);
                    o += take ? 1u : 0u;
                }
            }
            open[gi] = op;
            acc[gi] = a;
            pos[gi] = ws + o;
        }
        dlr::wave_sync();
    };
    if (MODE == 9) stamp(0);
    fill_load(0);
    for (int64_t lo = 0; lo < B; lo += R) {
        __syncthreads();
        if (MODE == 9) stamp(1 + 2 * (int)(lo / R));
#pragma unroll
        for (int f = 0; f < FILL; ++f) *reinterpret_cast<float4 *>(s_r + (f * 1024 + threadIdx.x) * 4) = fr[f];
        if (lo + R < B) fill_load(lo + R);  // next phase's fill in flight during this phase
        __syncthreads();
        const unsigned ulo = (unsigned)lo, uhi = (unsigned)min(lo + R, B);
        if (MODE == 9) stamp(2 + 2 * (int)(lo / R));
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) open[gi] = pos[gi] < end[gi];
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            if ((wv + 16 * gi) >= gpw || (g0 + wv + 16 * gi) * 64 >= D) break;  // wave-uniform
            window(rq[gi], vq[gi], ws0[gi], ulo, uhi, gi);
        }
        // slow path: groups with more than one window (their own loads)
        for (int gi = 0; gi < NG; ++gi) {
            if ((wv + 16 * gi) >= gpw || (g0 + wv + 16 * gi) * 64 >= D) break;
            for (unsigned ws = ws0[gi] + kW; ws < e1[gi]; ws += kW) {
                const unsigned e = ws + lane * 4;
                const bool in = e < e1[gi];
                const ushort4 r4 = in ? *reinterpret_cast<const ushort4 *>(crow + e) : make_ushort4(0, 0, 0, 0);
                const float4 v4 = in ? *reinterpret_cast<const float4 *>(cs.val + e) : make_float4(0.f, 0.f, 0.f, 0.f);
                window(r4, v4, ws, ulo, uhi, gi);
            }
        }
    }
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t j = (g0 + wv + 16 * gi) * 64 + lane;
        if ((wv + 16 * gi) >= gpw || j >= D) continue;
        const float cw = C * wj[gi];
        const float l2 = cw / Bf;
        const float gr = (float)((double)acc[gi] / Bd + (double)l2);
        if (FUSED) {
            const float step = lr * gr;
            w[j] = wj[gi] - step;
        } else {
            gout[j] = gr;
        }
    }
    if (MODE == 9) {
        __syncthreads();
        stamp(5);
    }
}

// Broadcast fill: every workgroup (1024 threads) copies the same R-float
// table into its LDS (FILL float4 per thread), then one lane writes a value.
template <int FILL>
__global__ __launch_bounds__(1024) void mb_fill(const float *__restrict__ tab, float *out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float4 fr[FILL];
#pragma unroll
    for (int f = 0; f < FILL; ++f) fr[f] = *reinterpret_cast<const float4 *>(tab + (f * 1024 + threadIdx.x) * 4);
#pragma unroll
    for (int f = 0; f < FILL; ++f) *reinterpret_cast<float4 *>(smem + (f * 1024 + threadIdx.x) * 4) = fr[f];
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = smem[(blockIdx.x * 977) % (FILL * 4096)];
}
// Writes a fresh table (as the margin kernel writes the residuals).
__global__ __launch_bounds__(256) void mb_write(float *tab, int n, float v) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) tab[i] = v + (float)i;
}

}  // namespace kb

using namespace kb;

template <typename F>
static float time_us(int reps, F &&launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms * 1000.0f / reps;
}

template <typename T>
static T *dup(const std::vector<T> &h, size_t pad = 64) {
    T *d = nullptr;
    CK(hipMalloc(&d, (h.size() + pad) * sizeof(T)));
    CK(hipMemset(d, 0, (h.size() + pad) * sizeof(T)));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

static int cmp_bits(const float *da, const float *db, size_t n, const char *what) {
    std::vector<float> a(n), b(n);
    CK(hipMemcpy(a.data(), da, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), db, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i)
        if (memcmp(&a[i], &b[i], 4) != 0) ++bad;
    printf("  check %-28s %s (%zu of %zu differ)\n", what, bad ? "MISMATCH" : "bitwise equal", bad, n);
    return bad ? 1 : 0;
}

int main(int argc, char **argv) {
    const int64_t B = argc > 1 ? atoll(argv[1]) : 65536;
    const int64_t D = argc > 2 ? atoll(argv[2]) : 1000000;
    const int nnz = argc > 3 ? atoi(argv[3]) : 50;
    const int reps = argc > 4 ? atoi(argv[4]) : 200;
    const bool calib = argc > 5 && strcmp(argv[5], "calib") == 0;
    printf("kbench: B=%lld D=%lld nnz=%d reps=%d%s\n", (long long)B, (long long)D, nnz, reps, calib ? " (calib)" : "");
    if (calib) {
        // PMC calibration: a cold 16-B/lane stream of known bytes (2 GiB
        // buffer, 26 MB windows: never cache-resident) and a 4-B gather of
        // known count from a cold 256 MiB table.
        const size_t big = (size_t)2 << 30;
        char *d_big = nullptr;
        float *d_o = nullptr;
        CK(hipMalloc(&d_big, big));
        CK(hipMemset(d_big, 0, big));
        CK(hipMalloc(&d_o, 64 << 20));
        const size_t win = (size_t)26214400;  // 25 MiB window: idx half + val half
        const int64_t n4 = (int64_t)(win / 2 / 16);
        const int nwin = (int)(big / win);
        for (int k = 0; k < reps; ++k) {
            const char *q = d_big + (size_t)(k % nwin) * win;
            hipLaunchKernelGGL(kb::mb_stream, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, (const int4 *)q,
                               (const float4 *)(q + win / 2), d_o, n4);
        }
        CK(hipDeviceSynchronize());
        printf("calib mb_stream: %d launches, each reads %zu B and writes %lld B\n", reps, win, (long long)(n4 * 4));
        return 0;
    }

    // ---- host data: distinct sorted uniform columns, 4-decimal values
    Rng rng{10};
    std::vector<int64_t> rp(B + 1);
    std::vector<int32_t> col;
    std::vector<float> val;
    std::vector<float> lab(B);
    col.reserve(B * nnz);
    val.reserve(B * nnz);
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
    // CSC (stable by row)
    std::vector<uint32_t> cptr(D + 1, 0);
    for (int64_t k = 0; k < E; ++k) ++cptr[col[k] + 1];
    for (int64_t j = 0; j < D; ++j) cptr[j + 1] += cptr[j];
    std::vector<uint32_t> cur(cptr.begin(), cptr.end() - 1);
    std::vector<uint16_t> crow(E);
    std::vector<float> cval(E);
    for (int64_t i = 0; i < B; ++i)
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
            const uint32_t p = cur[col[k]]++;
            crow[p] = (uint16_t)i;
            cval[p] = val[k];
        }
    std::vector<float> w0(D);
    for (int64_t j = 0; j < D; ++j) w0[j] = (float)rng.below(1 << 24) / (float)(1 << 24);

    int64_t *d_rp = dup(rp);
    int32_t *d_col = dup(col);
    float *d_val = dup(val);
    float *d_lab = dup(lab);
    uint32_t *d_cptr = dup(cptr);
    uint16_t *d_crow = dup(crow);
    float *d_cval = dup(cval);
    float *d_w = dup(w0);
    float *d_w2 = dup(w0);
    float *d_r = nullptr, *d_r2 = nullptr, *d_out = nullptr, *d_g = nullptr, *d_g2 = nullptr;
    CK(hipMalloc(&d_r, B * 4));
    CK(hipMalloc(&d_r2, B * 4));
    CK(hipMalloc(&d_g, D * 4));
    CK(hipMalloc(&d_g2, D * 4));
    CK(hipMalloc(&d_out, (E / 4 + 1024) * 4));
    const dlr::DevBatch bt{d_rp, d_col, d_val, d_lab, B, E};
    const dlr::DevCsc cs{d_cptr, d_crow, d_cval, true};
    const double mb_k2 = (double)E * 8 + B * 8;      // col+val, row_ptr+label
    const double mb_k3 = (double)E * 6 + (D + 1) * 4 + D * 8;  // crow+cval, cptr, w r/w
    printf("entries %lld; K2 bytes %.1f MB, K3 bytes %.1f MB\n", (long long)E, mb_k2 / 1e6, mb_k3 / 1e6);
    auto rate = [](double bytes, float us) { return bytes / (us * 1e-6) / 1e9; };

    // ---- micro
    const int64_t n4 = E / 4;
    const unsigned g4 = (unsigned)((n4 + 255) / 256);
    float t;
    t = time_us(reps, [&] { hipLaunchKernelGGL(mb_empty, dim3(1024), dim3(256), 0, 0, d_out); });
    printf("mb_empty(1024 WG)          %8.2f us\n", t);
    t = time_us(reps, [&] {
        hipLaunchKernelGGL(mb_stream, dim3(g4), dim3(256), 0, 0, (const int4 *)d_col, (const float4 *)d_val, d_out, n4);
    });
    printf("mb_stream col+val          %8.2f us  %7.1f GB/s\n", t, rate(E * 8.0 + n4 * 4.0, t));
    t = time_us(reps, [&] {
        hipLaunchKernelGGL(mb_gather, dim3(g4), dim3(256), 0, 0, (const int4 *)d_col, d_w, 0xFFFFFFFFu, d_out, n4);
    });
    printf("mb_gather w (4 MB table)   %8.2f us  %7.1f Gelem/s\n", t, E / (t * 1e-6) / 1e9);
    t = time_us(reps, [&] {
        hipLaunchKernelGGL(mb_gather, dim3(g4), dim3(256), 0, 0, (const int4 *)d_col, d_w, 0xFFFFu, d_out, n4);
    });
    printf("mb_gather w&0xFFFF (256KB) %8.2f us  %7.1f Gelem/s\n", t, E / (t * 1e-6) / 1e9);
    t = time_us(reps, [&] {
        hipLaunchKernelGGL(mb_gather, dim3(g4), dim3(256), 0, 0, (const int4 *)d_col, d_w, 0x3FFu, d_out, n4);
    });
    printf("mb_gather w&0x3FF (4KB)    %8.2f us  %7.1f Gelem/s\n", t, E / (t * 1e-6) / 1e9);

    for (unsigned mask : {0xFFFFFFFFu, 0xFFFFu, 0x3FFu}) {
        for (int G : {1, 2, 4, 8}) {
            for (int wpc : {8, 16, 32}) {  // waves per CU
                const unsigned grid = 256u * (unsigned)wpc / 4u;
                auto go = [&] {
                    if (G == 1) hipLaunchKernelGGL(mb_gather_g<1>, dim3(grid), dim3(256), 0, 0, (const int4 *)d_col, d_w, mask, d_out, n4);
                    if (G == 2) hipLaunchKernelGGL(mb_gather_g<2>, dim3(grid), dim3(256), 0, 0, (const int4 *)d_col, d_w, mask, d_out, n4);
                    if (G == 4) hipLaunchKernelGGL(mb_gather_g<4>, dim3(grid), dim3(256), 0, 0, (const int4 *)d_col, d_w, mask, d_out, n4);
                    if (G == 8) hipLaunchKernelGGL(mb_gather_g<8>, dim3(grid), dim3(256), 0, 0, (const int4 *)d_col, d_w, mask, d_out, n4);
                };
                t = time_us(reps, go);
                printf("mb_gather_g mask=%08x G=%d waves/CU=%2d %8.2f us  %7.1f Gelem/s\n", mask, G, wpc, t, E / (t * 1e-6) / 1e9);
            }
        }
    }
    {   // HBM-cold stream: walk 26 MB windows of a 2 GiB buffer
        const size_t big = (size_t)2 << 30;
        char *d_big = nullptr;
        CK(hipMalloc(&d_big, big));
        CK(hipMemset(d_big, 1, big));
        const size_t win = (size_t)E * 8;
        const int nwin = (int)(big / win);
        int k = 0;
        t = time_us(reps, [&] {
            const char *p = d_big + (size_t)(k++ % nwin) * win;
            hipLaunchKernelGGL(mb_stream, dim3(g4), dim3(256), 0, 0, (const int4 *)p, (const float4 *)(p + win / 2), d_out, n4 / 2);
        });
        printf("mb_stream cold 26MB windows %8.2f us  %7.1f GB/s\n", t, rate(win + n4 * 2.0, t));
        CK(hipFree(d_big));
    }

    {
        float *tab = nullptr;
        CK(hipMalloc(&tab, 65536 * 4));
        CK(hipMemset(tab, 0, 65536 * 4));
        for (int G : {256, 512, 1024}) {
            t = time_us(reps, [&] { hipLaunchKernelGGL(mb_fill<8>, dim3(G), dim3(1024), 131072, 0, tab, d_out); });
            printf("mb_fill 128KB x %4d WG (static)      %8.2f us\n", G, t);
            t = time_us(reps, [&] {
                hipLaunchKernelGGL(mb_write, dim3(128), dim3(256), 0, 0, tab, 32768, 1.0f);
                hipLaunchKernelGGL(mb_fill<8>, dim3(G), dim3(1024), 131072, 0, tab, d_out);
            });
            printf("mb_write+mb_fill 128KB x %4d WG      %8.2f us\n", G, t);
            t = time_us(reps, [&] { hipLaunchKernelGGL(mb_fill<2>, dim3(G), dim3(1024), 32768, 0, tab, d_out); });
            printf("mb_fill 32KB x %4d WG (static)       %8.2f us\n", G, t);
        }
        t = time_us(reps, [&] { hipLaunchKernelGGL(mb_write, dim3(128), dim3(256), 0, 0, tab, 32768, 1.0f); });
        printf("mb_write alone                        %8.2f us\n", t);
    }

    // ---- K2
    int bad = 0;
    CK(hipMemcpy(d_w, w0.data(), D * 4, hipMemcpyHostToDevice));
    for (int seg : {16, 32, 64}) {
        // each rows-per-wave form of the margin template, launched directly
        const dim3 blk(256);
        auto go = [&] {
            if (seg == 16)
                hipLaunchKernelGGL(dlr::k_margin_residual<16>, dim3((B + 63) / 64), blk, 0, 0, bt, d_w, d_r);
            else if (seg == 32)
                hipLaunchKernelGGL(dlr::k_margin_residual<32>, dim3((B + 127) / 128), blk, 0, 0, bt, d_w, d_r);
            else
                hipLaunchKernelGGL(dlr::k_margin_residual<64>, dim3((B + 255) / 256), blk, 0, 0, bt, d_w, d_r);
        };
        t = time_us(reps, go);
        printf("K2 ref SEG=%-2d               %8.2f us  %7.1f GB/s\n", seg, t, rate(mb_k2, t));
    }
    hipLaunchKernelGGL(dlr::k_margin_residual<16>, dim3((B + 63) / 64), dim3(256), 0, 0, bt, d_w, d_r);
    {   // C5 dense L2 pass variants on a 1 GiB weight vector (2^28 floats)
        const int64_t DW = (int64_t)1 << 28;
        float *wb = nullptr;
        CK(hipMalloc(&wb, DW * 4));
        CK(hipMemset(wb, 0, DW * 4));
        const int64_t n4 = DW / 4;
        const double bytes = 2.0 * DW * 4;
        auto run = [&](const char *nm, auto kern, unsigned grid) {
            const float tt = time_us(20, [&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, wb, n4, 1024.f, 0.2f, 1.0f); });
            printf("L2 pass %-28s grid %6u %9.1f us  %7.1f GB/s\n", nm, grid, tt, bytes / (tt * 1e-6) / 1e9);
        };
        run("nt U1 (production)", mb_l2<true, 1>, 2048);
        run("nt U1", mb_l2<true, 1>, 8192);
        run("nt U4", mb_l2<true, 4>, 2048);
        run("nt U4", mb_l2<true, 4>, 4096);
        run("plain U1", mb_l2<false, 1>, 2048);
        run("plain U4", mb_l2<false, 4>, 2048);
        run("plain U4", mb_l2<false, 4>, 8192);
        run("plain U1 one-shot", mb_l2<false, 1>, (unsigned)((n4 + 255) / 256));
        run("nt U1 one-shot", mb_l2<true, 1>, (unsigned)((n4 + 255) / 256));
        CK(hipFree(wb));
    }
    {   // column-split margin (two passes over half-size w tables) vs one pass, cold shard
        const int64_t NB = 40;
        // host split of the batch: entries with col < D/2 (A) and >= D/2 (B)
        std::vector<int64_t> rpA(B + 1), rpB(B + 1);
        std::vector<int32_t> cA, cB;
        std::vector<float> vA, vB;
        for (int64_t i = 0; i < B; ++i) {
            rpA[i] = (int64_t)cA.size();
            rpB[i] = (int64_t)cB.size();
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                if (col[k] < D / 2) {
                    cA.push_back(col[k]);
                    vA.push_back(val[k]);
                } else {
                    cB.push_back(col[k]);
                    vB.push_back(val[k]);
                }
            }
        }
        rpA[B] = (int64_t)cA.size();
        rpB[B] = (int64_t)cB.size();
        const int64_t EA = (int64_t)cA.size(), EB = (int64_t)cB.size();
        auto mk = [&](const std::vector<int64_t> &rph, const std::vector<int32_t> &ch, const std::vector<float> &vh,
                      int64_t Eh, int64_t **drp, int32_t **dc, float **dv) {
            CK(hipMalloc(dc, (Eh * NB + 1024) * 4));
            CK(hipMalloc(dv, (Eh * NB + 1024) * 4));
            CK(hipMalloc(drp, (B * NB + 1) * 8));
            std::vector<int64_t> big(B * NB + 1);
            for (int64_t q = 0; q < NB; ++q) {
                CK(hipMemcpy(*dc + q * Eh, ch.data(), Eh * 4, hipMemcpyHostToDevice));
                CK(hipMemcpy(*dv + q * Eh, vh.data(), Eh * 4, hipMemcpyHostToDevice));
                for (int64_t i = 0; i < B; ++i) big[q * B + i] = q * Eh + rph[i];
            }
            big[B * NB] = Eh * NB;
            CK(hipMemcpy(*drp, big.data(), big.size() * 8, hipMemcpyHostToDevice));
        };
        int64_t *drA, *drB;
        int32_t *dcA, *dcB;
        float *dvA, *dvB, *dz;
        mk(rpA, cA, vA, EA, &drA, &dcA, &dvA);
        mk(rpB, cB, vB, EB, &drB, &dcB, &dvB);
        CK(hipMalloc(&dz, B * 4));
        int q = 0;
        t = time_us(reps, [&] {
            const dlr::DevBatch ba{drA + (q % NB) * B, dcA, dvA, d_lab, B, EA};
            const dlr::DevBatch bb{drB + (q % NB) * B, dcB, dvB, d_lab, B, EB};
            ++q;
            hipLaunchKernelGGL((k2_split<16, true, false>), dim3((B + 63) / 64), dim3(256), 0, 0, ba, d_w, nullptr, dz);
            hipLaunchKernelGGL((k2_splitB<16>), dim3((B + 63) / 64), dim3(256), 0, 0, bb, d_w, dz, d_r2);
        });
        printf("K2 column-split 2 passes     %8.2f us  %7.1f GB/s\n", t, rate(mb_k2, t));
        bad |= cmp_bits(d_r, d_r2, B, "K2 split vs ref");
        for (int seg : {8, 16, 32}) {
            q = 0;
            t = time_us(reps, [&] {
                const dlr::DevBatch ba{drA + (q % NB) * B, dcA, dvA, d_lab, B, EA};
                ++q;
                if (seg == 8)
                    hipLaunchKernelGGL((k2_split<8, true, false>), dim3((B + 31) / 32), dim3(256), 0, 0, ba, d_w, nullptr, dz);
                else if (seg == 16)
                    hipLaunchKernelGGL((k2_split<16, true, false>), dim3((B + 63) / 64), dim3(256), 0, 0, ba, d_w, nullptr, dz);
                else
                    hipLaunchKernelGGL((k2_split<32, true, false>), dim3((B + 127) / 128), dim3(256), 0, 0, ba, d_w, nullptr, dz);
            });
            printf("K2 half pass A alone SEG=%-2d  %8.2f us\n", seg, t);
        }
    }
    {   // margin over a cold 10M-row shard (HBM-resident stream), plain vs nt
        const int64_t NB = 40;  // batches in the cold shard
        const int64_t EB = E * NB;
        int32_t *bc = nullptr;
        float *bv = nullptr;
        int64_t *brp = nullptr;
        CK(hipMalloc(&bc, (EB + 1024) * 4));
        CK(hipMalloc(&bv, (EB + 1024) * 4));
        CK(hipMalloc(&brp, (B * NB + 1) * 8));
        for (int64_t q = 0; q < NB; ++q) {
            CK(hipMemcpy(bc + q * E, col.data(), E * 4, hipMemcpyHostToDevice));
            CK(hipMemcpy(bv + q * E, val.data(), E * 4, hipMemcpyHostToDevice));
        }
        std::vector<int64_t> brph(B * NB + 1);
        for (int64_t q = 0; q < NB; ++q)
            for (int64_t i = 0; i < B; ++i) brph[q * B + i] = q * E + rp[i];
        brph[B * NB] = EB;
        CK(hipMemcpy(brp, brph.data(), brph.size() * 8, hipMemcpyHostToDevice));
        for (int nt = 0; nt < 2; ++nt) {
            int q = 0;
            t = time_us(reps, [&] {
                const dlr::DevBatch bq{brp + (q % NB) * B, bc, bv, d_lab, B, E};
                ++q;
                if (nt)
                    hipLaunchKernelGGL((k2_nt<16, true>), dim3((B + 63) / 64), dim3(256), 0, 0, bq, d_w, d_r2);
                else
                    hipLaunchKernelGGL((k2_nt<16, false>), dim3((B + 63) / 64), dim3(256), 0, 0, bq, d_w, d_r2);
            });
            printf("K2 cold-shard SEG=16 %s       %8.2f us  %7.1f GB/s\n", nt ? "nt   " : "plain", t, rate(mb_k2, t));
        }
        CK(hipFree(bc));
        CK(hipFree(bv));
        CK(hipFree(brp));
    }
    const unsigned gB = (unsigned)((B + 255) / 256);
    t = time_us(reps, [&] { hipLaunchKernelGGL(k2_lpr<8>, dim3(gB), dim3(256), 0, 0, bt, d_w, d_r2); });
    printf("K2 lane-per-row U=8        %8.2f us  %7.1f GB/s\n", t, rate(mb_k2, t));
    bad |= cmp_bits(d_r, d_r2, B, "K2 lpr8 vs ref");
    t = time_us(reps, [&] { hipLaunchKernelGGL(k2_lpr<16>, dim3(gB), dim3(256), 0, 0, bt, d_w, d_r2); });
    printf("K2 lane-per-row U=16       %8.2f us  %7.1f GB/s\n", t, rate(mb_k2, t));
    bad |= cmp_bits(d_r, d_r2, B, "K2 lpr16 vs ref");

    // ---- K3 (unfused: output g, so repeated launches are idempotent)
    const unsigned gD = (unsigned)((D + 255) / 256);
    const float Bf = (float)B;
    const double Bd = (double)B;
    t = time_us(reps, [&] {
        hipLaunchKernelGGL((dlr::k_grad<uint16_t, false>), dim3(gD), dim3(256), 0, 0, cs, d_crow, D, d_r, d_w, d_g, Bf,
                           Bd, 0.2f, 1.0f);
    });
    printf("K3 ref                     %8.2f us  %7.1f GB/s\n", t, rate(mb_k3, t));
    for (int u : {2, 4, 8}) {
        auto go = [&] {
            if (u == 2)
                hipLaunchKernelGGL((k3_lpc<2, false>), dim3(gD), dim3(256), 0, 0, cs, d_crow, D, d_r, d_w, d_g2, Bf, Bd,
                                   0.2f, 1.0f);
            else if (u == 4)
                hipLaunchKernelGGL((k3_lpc<4, false>), dim3(gD), dim3(256), 0, 0, cs, d_crow, D, d_r, d_w, d_g2, Bf, Bd,
                                   0.2f, 1.0f);
            else
                hipLaunchKernelGGL((k3_lpc<8, false>), dim3(gD), dim3(256), 0, 0, cs, d_crow, D, d_r, d_w, d_g2, Bf, Bd,
                                   0.2f, 1.0f);
        };
        t = time_us(reps, go);
        printf("K3 lane-per-col U=%d        %8.2f us  %7.1f GB/s\n", u, t, rate(mb_k3, t));
        bad |= cmp_bits(d_g, d_g2, D, "K3 lpc vs ref");
    }
    for (int R : {32768, 36864}) {
        const int64_t ngroups = (D + 63) / 64;
        const int G = 256;
        const int gpw = (int)((ngroups + G - 1) / G);
        const int NGn = (gpw + 15) / 16;
        const size_t lds = (size_t)R * 4;
        auto go = [&](int U) {
            if (NGn <= 4 && U == 8)
                hipLaunchKernelGGL((k3_lds<8, 4, false>), dim3(G), dim3(1024), lds, 0, cs, d_crow, D, B, R, gpw, d_r, d_w,
                                   d_g2, Bf, Bd, 0.2f, 1.0f);
            else if (NGn <= 4 && U == 4)
                hipLaunchKernelGGL((k3_lds<4, 4, false>), dim3(G), dim3(1024), lds, 0, cs, d_crow, D, B, R, gpw, d_r, d_w,
                                   d_g2, Bf, Bd, 0.2f, 1.0f);
            else
                printf("NG %d unsupported\n", NGn);
        };
        for (int U : {4, 8}) {
            CK(hipMemset(d_g2, 0, D * 4));
            t = time_us(reps, [&] { go(U); });
            printf("K3 lds R=%d U=%d NG=%d        %8.2f us  %7.1f GB/s\n", R, U, NGn, t, rate(mb_k3, t));
            bad |= cmp_bits(d_g, d_g2, D, "K3 lds vs ref");
        }
    }
    for (int kW : {256, 512}) {
        const int R = kW == 256 ? 36864 : 32768;
        const int64_t ngroups = (D + 63) / 64;
        const int G = 256;
        const int gpw = (int)((ngroups + G - 1) / G);
        const int NGn = (gpw + 15) / 16;
        const size_t lds = (size_t)R * 4 + 16 * kW * 4;
        CK(hipMemset(d_g2, 0, D * 4));
        t = time_us(reps, [&] {
            if (kW == 256)
                hipLaunchKernelGGL((k3_ldsw<4, 256, false>), dim3(G), dim3(1024), lds, 0, cs, d_crow, D, B, R, gpw, d_r,
                                   d_w, d_g2, Bf, Bd, 0.2f, 1.0f);
            else
                hipLaunchKernelGGL((k3_ldsw<4, 512, false>), dim3(G), dim3(1024), lds, 0, cs, d_crow, D, B, R, gpw, d_r,
                                   d_w, d_g2, Bf, Bd, 0.2f, 1.0f);
        });
        printf("K3 ldsw kW=%d R=%d NG=%d    %8.2f us  %7.1f GB/s\n", kW, R, NGn, t, rate(mb_k3, t));
        bad |= cmp_bits(d_g, d_g2, D, "K3 ldsw vs ref");
    }
    {
        const int64_t ngroups = (D + 63) / 64;
        const int G = 256;
        const int gpw = (int)((ngroups + G - 1) / G);
        const size_t lds = (size_t)8 * 4096 * 4 + 16 * 256 * 4;
        CK(hipMemset(d_g2, 0, D * 4));
        t = time_us(reps, [&] {
            hipLaunchKernelGGL((k3_pf<4, 8, false>), dim3(G), dim3(1024), lds, 0, cs, d_crow, D, B, gpw, d_r, d_w, d_g2,
                               Bf, Bd, 0.2f, 1.0f);
        });
        printf("K3 pf NG=4 R=32768           %8.2f us  %7.1f GB/s\n", t, rate(mb_k3, t));
        bad |= cmp_bits(d_g, d_g2, D, "K3 pf vs ref");
        const size_t lds2 = (size_t)1 * 4096 * 4 + 16 * 256 * 4;
        t = time_us(reps, [&] { hipLaunchKernelGGL((k3_pf<4, 1, false, 0>), dim3(G), dim3(1024), lds2, 0, cs, d_crow, D, (int64_t)4096, gpw, d_r, d_w, d_g2, Bf, Bd, 0.2f, 1.0f); });
        printf("K3 pf ablate: B=4096 1 phase %8.2f us\n", t);
        {
            unsigned long long *d_st = nullptr;
            CK(hipMalloc(&d_st, G * 8 * 8));
            CK(hipMemset(d_st, 0, G * 8 * 8));
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_kb), &d_st, sizeof(d_st)));
            for (int it = 0; it < 20; ++it)
                hipLaunchKernelGGL((k3_pf<4, 8, false, 9>), dim3(G), dim3(1024), lds, 0, cs, d_crow, D, B, gpw, d_r, d_w, d_g2, Bf, Bd, 0.2f, 1.0f);
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> st(G * 8);
            CK(hipMemcpy(st.data(), d_st, G * 8 * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (int g = 0; g < G; ++g) t0 = std::min(t0, st[g * 8]);
            // 100 MHz ticks -> us
            const char *nm[6] = {"start", "fill0 in", "ph0 go", "fill1 in", "ph1 go", "end"};
            for (int k = 0; k < 6; ++k) {
                std::vector<double> v;
                for (int g = 0; g < G; ++g) v.push_back((st[g * 8 + k] - t0) * 0.01);
                std::sort(v.begin(), v.end());
                printf("  stamp %-9s min %6.2f med %6.2f p90 %6.2f max %6.2f us\n", nm[k], v[0], v[G / 2], v[G * 9 / 10], v[G - 1]);
            }
        }
    }
    {   // production LDS gradient kernel on a phase-split copy of the batch
        const int fillq = dlr::grad_lds_fill(B);
        const int64_t R = (int64_t)fillq * 4096;
        const int P = (int)((B + R - 1) / R);
        const int64_t ngr = (D + 63) / 64, nblk = ngr * P;
        std::vector<uint32_t> cnt2((size_t)(D * P), 0), pbase((size_t)nblk + 1);
        std::vector<uint8_t> pends((size_t)nblk * 64);
        for (int64_t i = 0; i < B; ++i)
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) ++cnt2[(size_t)col[k] * P + (size_t)(i / R)];
        uint32_t at = 0;
        bool fits = true;
        for (int64_t g = 0; g < ngr; ++g)
            for (int p = 0; p < P; ++p) {
                const int64_t blk = g * P + p;
                pbase[blk] = at;
                uint32_t o = 0;
                for (int l = 0; l < 64; ++l) {
                    const int64_t j = g * 64 + l;
                    if (j < D) {
                        const uint32_t c = cnt2[(size_t)(j * P + p)];
                        cnt2[(size_t)(j * P + p)] = at + o;
                        o += c;
                    }
                    pends[blk * 64 + l] = (uint8_t)o;
                }
                fits = fits && o <= 255;
                at += (o + 3) & ~3u;
            }
        pbase[nblk] = at;
        std::vector<uint16_t> prow(at, 0);
        std::vector<float> pval(at, 0.0f);
        for (int64_t i = 0; i < B; ++i)
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const uint32_t q = cnt2[(size_t)col[k] * P + (size_t)(i / R)]++;
                prow[q] = (uint16_t)(i % R);
                pval[q] = val[k];
            }
        printf("pcsc: P=%d R=%lld entries(padded)=%u fits=%d\n", P, (long long)R, at, (int)fits);
        uint32_t *d_pb = dup(pbase);
        uint8_t *d_pe = dup(pends);
        uint16_t *d_pr = dup(prow, 256);
        float *d_pv = dup(pval, 256);
        float *d_rp = nullptr;
        CK(hipMalloc(&d_rp, P * R * 4));
        CK(hipMemset(d_rp, 0, P * R * 4));
        CK(hipMemcpy(d_rp, d_r, B * 4, hipMemcpyDeviceToDevice));
        const dlr::DevPcsc pc{d_pb, d_pe, d_pr, d_pv, P};
        // the stamp buffer must be set before ANY launch of the stamped kernel
        const int G = (int)((ngr + 63) / 64);
        unsigned long long *d_st = nullptr;
        CK(hipMalloc(&d_st, (size_t)G * 16 * 8));  // dlr_kernels.hip DLR_STAMP: 16 slots per workgroup
        CK(hipMemset(d_st, 0, (size_t)G * 16 * 8));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(dlr::g_stamp), &d_st, sizeof(d_st)));
        CK(hipMemset(d_g2, 0, D * 4));
        t = time_us(reps, [&] { CK(dlr::launch_grad_lds(pc, D, B, d_rp, d_w, d_g2, 0.2f, 1.0f, false, 0)); });
        printf("K3 production lds            %8.2f us  %7.1f GB/s\n", t, rate(mb_k3, t));
        bad |= cmp_bits(d_g, d_g2, D, "K3 production lds vs ref");
        {
            const size_t lds = (size_t)8 * 4096 * 4 + 16 * 264 * 4;
            const unsigned grid = (unsigned)((ngr + 63) / 64);
            auto abl = [&](const char *nm, auto kern) {
                const float ta = time_us(reps, [&] {
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds, 0, pc, D, d_rp, d_w, d_g2, (float)B, (double)B, 1.0f);
                });
                printf("K3 ablation %-32s %8.2f us\n", nm, ta);
            };
            abl("none (copy)", mb_grad_abl<0>);
            abl("no gathers", mb_grad_abl<1>);
            abl("no read loop", mb_grad_abl<2>);
            abl("no gathers, no read loop", mb_grad_abl<3>);
            abl("phase 0 only", mb_grad_abl<4>);
            abl("no fills", mb_grad_abl<8>);
            abl("no fills, no gathers, no loop", mb_grad_abl<11>);
            abl("phase 0 only, no fills/gathers/loop", mb_grad_abl<15>);
            float *d_o = nullptr;
            CK(hipMalloc(&d_o, 256 * 1024 * 4));
            for (unsigned mask : {32767u, 0u}) {
                const int rounds = 64;
                const float tg = time_us(20, [&] {
                    hipLaunchKernelGGL(mb_lds_gather<8>, dim3(256), dim3(1024), 131072, 0, d_o, rounds, mask);
                });
                const double n = 256.0 * 1024 * 8 * rounds;
                printf("LDS gather mask %5u: %8.2f us  %7.1f G/s chip  %5.2f lanes/clk/CU @2.4GHz\n", mask, tg, n / tg * 1e-3,
                       n / 256 / (tg * 1e-6) / 2.4e9);
            }
            CK(hipFree(d_o));
        }
        {   // cold: a 1 GiB stream through L2 / the Infinity Cache before every launch
            const int64_t fl4 = (int64_t)1 << 26;  // float4s = 1 GiB
            float4 *fb = nullptr;
            float *fo = nullptr;
            CK(hipMalloc(&fb, fl4 * 16));
            CK(hipMemset(fb, 0, fl4 * 16));
            CK(hipMalloc(&fo, 1 << 22));
            hipEvent_t ea, eb;
            CK(hipEventCreate(&ea));
            CK(hipEventCreate(&eb));
            double tot = 0;
            const int cr = 20;
            for (int it = 0; it < cr; ++it) {
                hipLaunchKernelGGL(mb_flush, dim3(4096), dim3(256), 0, 0, (const float4 *)fb, fl4, fo);
                CK(hipEventRecord(ea, 0));
                CK(dlr::launch_grad_lds(pc, D, B, d_rp, d_w, d_g2, 0.2f, 1.0f, false, 0));
                CK(hipEventRecord(eb, 0));
                CK(hipEventSynchronize(eb));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, ea, eb));
                tot += ms;
            }
            printf("K3 production lds, cold MALL %8.2f us\n", tot * 1000.0 / cr);
            CK(hipFree(fb));
            CK(hipFree(fo));
        }
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> st((size_t)G * 16);
        CK(hipMemcpy(st.data(), d_st, (size_t)G * 16 * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (int g = 0; g < G; ++g) t0 = std::min(t0, st[g * 16]);
        const char *nm[6] = {"start", "ph0 go", "", "ph0 done", "ph1 go", "end"};
        for (int k : {0, 1, 3, 4, 5}) {
            std::vector<double> v;
            for (int g = 0; g < G; ++g) v.push_back((st[g * 16 + k] - t0) * 0.01);
            std::sort(v.begin(), v.end());
            printf("  stamp %-9s min %6.2f med %6.2f p90 %6.2f max %6.2f us\n", nm[k], v[0], v[G / 2], v[G * 9 / 10], v[G - 1]);
        }
    }
    printf("%s\n", bad ? "SOME CHECKS FAILED" : "all checks bitwise equal");
    return bad;
}
