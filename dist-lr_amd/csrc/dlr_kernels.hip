// dlr_kernels.hip -- gfx950 kernels of the dist-lr hot path.
//
// Parity contract (DESIGN.md "Numerics"): every fp32 sum is
// accumulated in the reference's order with separate multiply and add
// (this file is compiled with -ffp-contract=off; tests/test_abi.py checks
// the ISA has no fused f32 op outside correctly-rounded divisions), so
// results are bitwise equal to src/lr.cc:
//   margin  z_i = sum_j w_j*x_ij, j ascending          (lr.cc:108-112)
//   sigma_i = (float)(1/(1+exp(-(double)z_i)))          (lr.cc:113)
//   r_i     = sigma_i - y_i                             (lr.cc:38)
//   G_j     = sum_i fl32(r_i*x_ij), batch-row order     (lr.cc:35-39)
//   g_j     = fl32((double)G_j/B + (double)(fl32(C*w_j)/(float)B))  (lr.cc:40)
//   update  w_j -= fl32(fl32(lr*g_j)/(float)W)          (main.cc:70-72)
//
// Both hot kernels are one primitive, an ORDERED SEGMENTED DOT: segment s
// (a batch row for the margin, a feature column for the gradient) sums
// fl32(table[idx_k] * val_k) over its entries k in storage order.  A wave
// owns 64 consecutive segments, whose entries are contiguous.  Per window
// of kWin entries the wave (1) loads idx/val ENTRY-parallel with 16-byte
// loads (coalesced, balanced however ragged the segments are), (2) issues
// every table gather of the window at once and forms the products, (3)
// parks the products in LDS, and (4) each lane adds its own segment's
// products in order.  Products do not depend on the order, the additions
// do -- and those stay sequential, so the result is the reference's bits.
//
// Layout (DESIGN.md "Data layout in HBM"): the shard is resident as CSR
// (row_ptr int64, col int32, val fp32, label fp32); each batch also has a
// column-major copy (cptr uint32[D+1], batch-local row uint16/uint32, val
// fp32) built once at load time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

#include "dlr_kernels.h"
#include "dlr_exchange.h"

namespace dlr {

namespace {

constexpr int kWave = 64;
constexpr int kWaves = 4;      // waves per workgroup (independent)
constexpr int kWin = 1024;     // entries per wave per window
constexpr int kVec = 4;        // entries per lane per load
constexpr uint32_t kLongFlag = 0x80000000u;  // DevCsc::ptr bit 31: long column
constexpr uint32_t kPtrMask = 0x7FFFFFFFu;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a
// workgroup-scope release + acquire, which on gfx950 waits vmcnt(0): it
// drains every global load in flight (loads issued early for later phases,
// LDS-DMA prefetches) at every barrier.  LDS-DMA data is published by the
// issuing wave's own s_waitcnt vmcnt before the barrier.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// LDS accesses the compiler cannot see.  A compiler-issued LDS access that
// may alias an in-flight LDS-DMA gets an s_waitcnt vmcnt(0) -- every global
// load in flight drains first.  Callers order these after their DMA with
// explicit vmcnt waits and use the results only after lds_wait*().
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
template <int OFF = 0>
__device__ __forceinline__ float lds_rd32(uint32_t a) {
    float v;
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
    return v;
}
__device__ __forceinline__ void lds_wr128(uint32_t a, v4f v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_wait1(float &a) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a)); }
__device__ __forceinline__ void lds_wait4(float &a, float &b, float &c, float &d) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}

// Bounded waits of the in-launch hand-offs (dlr_kernels.h DevErr).  The
// reference's worker never computes on data it has not received
// (lr.cc:122, 131: kv_->Wait); a wait here that has seen no producer for
// kSpinTicks of the 100 MHz real-time clock records its kind in the
// context's error word -- the host then fails dlr_sync / the next step
// with DLR_E_DEVICE instead of returning weights -- and marks the waiting
// lane dead: its later waits in the launch return at once, so a launch
// whose producer never comes drains after one timeout per wave, not one per
// wait.  The clock is read every 64 polls from the 64th on: a wait whose
// producer comes within 64 polls (nearly every wait of a healthy launch)
// never reads it.
constexpr uint64_t kSpinTicks = 25000000ull;  // 250 ms
struct Spin {
    uint32_t *err;  // the error words (host-mapped; null: none)
    int kind;
    bool dead = false;
    uint64_t t0 = 0;
    __device__ explicit Spin(uint32_t *e, int k) : err(e), kind(k) {}
    // poll k (from 0) of a wait: false = stop polling (dead, or timed out)
    __device__ __forceinline__ bool more(int k) {
        if (dead) return false;
        if ((k & 63) || k == 0) return true;
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if (k == 64) {
            t0 = t;
            return true;
        }
        if (t - t0 < kSpinTicks) return true;
        dead = true;
        if (err) __hip_atomic_store(err + kind, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
    }
};

template <typename T>
struct Vec4;
template <>
struct Vec4<int32_t> {
    using type = int4;
};
template <>
struct Vec4<uint32_t> {
    using type = uint4;
};
template <>
struct Vec4<uint16_t> {
    using type = ushort4;
};

// Non-temporal 16-byte loads for once-read streams: the streamed lines do
// not displace the gathered table (w) from L2 (tools/kbench, cold 10M-row
// shard: margin 22.9 -> 20.8 us).
template <typename V>
__device__ __forceinline__ V load_stream(const V *p) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    static_assert(sizeof(V) == 16 || sizeof(V) == 8, "16- or 8-byte vectors");
    V out;
    if constexpr (sizeof(V) == 16) {
        const u4 x = __builtin_nontemporal_load(reinterpret_cast<const u4 *>(p));
        __builtin_memcpy(&out, &x, 16);
    } else {
        const u2 x = __builtin_nontemporal_load(reinterpret_cast<const u2 *>(p));
        __builtin_memcpy(&out, &x, 8);
    }
    return out;
}

// Sum over this lane's segment [a, b) of fl32(table[idx[k]] * val[k]), in
// k order.  The wave's entries are [e0, e1).  lds: kWin floats of this wave.
// Only lanes < SEG own a segment; all 64 lanes load and gather.
// UNIT: every value is 1.0f and val is not read (one-hot / binary shards:
// fl32(t * 1.0f) == t exactly, so the sums are the same bits).
// acc0: the sum the segment continues (0.0f: a whole segment; the band
// kernel passes a column's sum over the earlier row bands, which continues
// the same sequential chain).
// HOT > 0: table[0, HOT) is also staged in LDS at `hot` (the frequency-
// ordered hot weights); those gathers read LDS, the others read table
// (each lane issues both, with the unused one clamped to index 0: no
// divergent load, and the clamped global lanes share one L1 line).
template <typename IdxT, bool UNIT = false, int HOT = 0>
__device__ __forceinline__ float ordered_segment_dot(int64_t e0, int64_t e1, int64_t a, int64_t b, int lane,
                                                     const IdxT *__restrict__ idx, const float *__restrict__ val,
                                                     const float *__restrict__ table, float *lds,
                                                     float acc0 = 0.0f, const float *hot = nullptr) {
    using IV = typename Vec4<IdxT>::type;
    constexpr int kT = kWin / (kVec * kWave);
    constexpr int kChunk = kVec * kWave;  // entries per (t) step of the wave
    const int64_t base = e0 & ~int64_t(kVec - 1);
    float acc = acc0;
    for (int64_t ws = base; ws < e1; ws += kWin) {
        const int64_t left = e1 - ws;  // wave-uniform
        // (1) index/value loads of the window's chunks that hold entries
        // (wave-uniform skip), branch-free inside a chunk: a lane past the
        // last entry re-reads the chunk's first vector (masked below).
        IV iv[kT];
        float4 v[kT];
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            if (t * kChunk < left) {
                const int64_t e = ws + t * kChunk + lane * kVec;
                const int64_t ec = e < e1 ? e : ws + t * kChunk;
                iv[t] = load_stream(reinterpret_cast<const IV *>(idx + ec));
                if constexpr (UNIT)
                    v[t] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
                else
                    v[t] = load_stream(reinterpret_cast<const float4 *>(val + ec));
            }
        }
        // (2) every gather of the window, then the products.  Entries outside
        // [e0, e1) belong to no segment of this wave: index 0, product 0.
        float g[kT][kVec];
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            if (t * kChunk < left) {
                const int64_t e = ws + t * kChunk + lane * kVec;
                const unsigned i0 = (e >= e0 && e < e1) ? (unsigned)iv[t].x : 0u;
                const unsigned i1 = (e + 1 >= e0 && e + 1 < e1) ? (unsigned)iv[t].y : 0u;
                const unsigned i2 = (e + 2 >= e0 && e + 2 < e1) ? (unsigned)iv[t].z : 0u;
                const unsigned i3 = (e + 3 >= e0 && e + 3 < e1) ? (unsigned)iv[t].w : 0u;
                if constexpr (HOT > 0) {
                    const float h0 = hot[i0 < HOT ? i0 : 0u], h1 = hot[i1 < HOT ? i1 : 0u];
                    const float h2 = hot[i2 < HOT ? i2 : 0u], h3 = hot[i3 < HOT ? i3 : 0u];
                    const float c0 = table[i0 < HOT ? 0u : i0], c1 = table[i1 < HOT ? 0u : i1];
                    const float c2 = table[i2 < HOT ? 0u : i2], c3 = table[i3 < HOT ? 0u : i3];
                    g[t][0] = i0 < HOT ? h0 : c0;
                    g[t][1] = i1 < HOT ? h1 : c1;
                    g[t][2] = i2 < HOT ? h2 : c2;
                    g[t][3] = i3 < HOT ? h3 : c3;
                } else {
                    g[t][0] = table[i0];
                    g[t][1] = table[i1];
                    g[t][2] = table[i2];
                    g[t][3] = table[i3];
                }
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
        wave_sync();
        // (3) this lane's segment, in order; 8 LDS reads in flight per step.
        const int64_t lo = a > ws ? a : ws;
        const int64_t hi = b < ws + kWin ? b : ws + kWin;
        int o = (int)(lo - ws);
        const int oe = (int)(hi - ws);
        if (oe - o >= 64) {
            // a long run (a column of a small-D full batch: C1's 123 columns
            // hold ~900 entries each): 16-byte reads, 32 products per LDS
            // wait, same order.  Rows of a margin never get here (their
            // runs are the row lengths, well under 64 at every config).
            for (; o & 3; ++o) acc = acc + lds[o];
            for (; o + 32 <= oe; o += 32) {
                float4 q[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) q[u] = *reinterpret_cast<const float4 *>(lds + o + 4 * u);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    acc = acc + q[u].x;
                    acc = acc + q[u].y;
                    acc = acc + q[u].z;
                    acc = acc + q[u].w;
                }
            }
        }
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
        wave_sync();
    }
    return acc;
}

// ordered_segment_dot for K segments per lane (short segments: the band
// kernel's (column, band) pairs average ~3.6 entries, so 64 per wave left
// its windows a quarter full).  Lane l owns segments [a[k], b[k]) for
// k < K (empty: a == b), each summed in order from acc[k]; the wave's
// entries are [e0, e1).  Same loads, gathers and products as
// ordered_segment_dot.
// ordered_segments_dot for bands that hold long runs (DLR_LONG_COLUMN=0 in
// band mode: a Zipf-head column puts ~125,000 entries into each 2^20-row
// band, so whole windows are one lane's run and that lane's serial chain is
// the band's critical path).  Same loads, gathers, products and order of
// additions as ordered_segments_dot; the window loop is software-pipelined
// so the chain never waits for memory: while the lanes sum window w, the
// residual gathers of window w+1 and the entry loads of window w+2 are in
// flight (issue order gathers(w+1), loads(w+2): the in-order vmcnt makes
// each stage's wait exact).  Runs of >= 64 products are read 16 bytes at a
// time, 32 per LDS wait.
template <typename IdxT, bool UNIT, int K>
__device__ __forceinline__ void ordered_segments_dot_piped(int64_t e0, int64_t e1, const int64_t (&a)[K],
                                                           const int64_t (&b)[K], float (&acc)[K], int lane,
                                                           const IdxT *__restrict__ idx, const float *__restrict__ val,
                                                           const float *__restrict__ table, float *lds) {
    using IV = typename Vec4<IdxT>::type;
    constexpr int kT = kWin / (kVec * kWave);
    constexpr int kChunk = kVec * kWave;
    const int64_t base = e0 & ~int64_t(kVec - 1);
    struct Win {
        IV iv[kT];
        float4 v[kT];
    };
    // loads: always issued (clamped to the last window): fixed vmcnt counts
    auto load = [&](int64_t ws, Win &w) {
        const int64_t wc = ws < e1 ? ws : base;
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            const int64_t e = wc + t * kChunk + lane * kVec;
            const int64_t ec = e < e1 ? e : base;
            w.iv[t] = load_stream(reinterpret_cast<const IV *>(idx + ec));
            if constexpr (UNIT)
                w.v[t] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
            else
                w.v[t] = load_stream(reinterpret_cast<const float4 *>(val + ec));
        }
    };
    auto gather = [&](int64_t ws, const Win &w, float (&g)[kT][kVec]) {
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            const int64_t e = ws + t * kChunk + lane * kVec;
            g[t][0] = table[(e >= e0 && e < e1) ? (unsigned)w.iv[t].x : 0u];
            g[t][1] = table[(e + 1 >= e0 && e + 1 < e1) ? (unsigned)w.iv[t].y : 0u];
            g[t][2] = table[(e + 2 >= e0 && e + 2 < e1) ? (unsigned)w.iv[t].z : 0u];
            g[t][3] = table[(e + 3 >= e0 && e + 3 < e1) ? (unsigned)w.iv[t].w : 0u];
        }
    };
    Win wa, wb;
    float ga[kT][kVec];
    load(base, wa);
    gather(base, wa, ga);
    load(base + kWin, wb);
    for (int64_t ws = base; ws < e1; ws += kWin) {
        // park window ws's products (its gathers were issued an iteration ago)
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            const int o = t * kChunk + lane * kVec;
            const int64_t e = ws + o;
            float4 p;
            p.x = (e >= e0 && e < e1) ? ga[t][0] * wa.v[t].x : 0.0f;
            p.y = (e + 1 >= e0 && e + 1 < e1) ? ga[t][1] * wa.v[t].y : 0.0f;
            p.z = (e + 2 >= e0 && e + 2 < e1) ? ga[t][2] * wa.v[t].z : 0.0f;
            p.w = (e + 3 >= e0 && e + 3 < e1) ? ga[t][3] * wa.v[t].w : 0.0f;
            *reinterpret_cast<float4 *>(lds + o) = p;
        }
        wave_sync();
        // window ws+1: its entries landed during the previous sums; issue its
        // gathers, then the loads of window ws+2, all in flight under the sums
        wa = wb;
        gather(ws + kWin, wa, ga);
        load(ws + 2 * kWin, wb);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t lo = a[k] > ws ? a[k] : ws;
            const int64_t hi = b[k] < ws + kWin ? b[k] : ws + kWin;
            int o = (int)(lo - ws);
            const int oe = (int)(hi - ws);
            float s = acc[k];
            if (oe - o >= 64) {
                // the run's products 32 at a time, the next 32's reads in
                // flight while these are added (reads past the run are
                // clamped inside the wave's slab and never added)
                for (; o & 3; ++o) s = s + lds[o];
                auto rd = [&](float4(&q)[8], int off) {
                    off = off < kWin - 32 ? off : kWin - 32;
#pragma unroll
                    for (int u = 0; u < 8; ++u) q[u] = *reinterpret_cast<const float4 *>(lds + off + 4 * u);
                };
                auto add = [&](const float4(&q)[8]) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        s = s + q[u].x;
                        s = s + q[u].y;
                        s = s + q[u].z;
                        s = s + q[u].w;
                    }
                };
                const int n32 = (oe - o) >> 5;
                float4 qa[8], qb[8];
                rd(qa, o);
                int g = 0;
                for (; g + 2 <= n32; g += 2, o += 64) {
                    rd(qb, o + 32);
                    add(qa);
                    rd(qa, o + 64);
                    add(qb);
                }
                if (g < n32) {
                    add(qa);
                    o += 32;
                }
            }
            for (; o + 4 <= oe; o += 4) {
                const float x0 = lds[o], x1 = lds[o + 1], x2 = lds[o + 2], x3 = lds[o + 3];
                s = s + x0;
                s = s + x1;
                s = s + x2;
                s = s + x3;
            }
            for (; o < oe; ++o) s = s + lds[o];
            acc[k] = s;
        }
        wave_sync();
    }
}

template <typename IdxT, bool UNIT, int K>
__device__ __forceinline__ void ordered_segments_dot(int64_t e0, int64_t e1, const int64_t (&a)[K],
                                                     const int64_t (&b)[K], float (&acc)[K], int lane,
                                                     const IdxT *__restrict__ idx, const float *__restrict__ val,
                                                     const float *__restrict__ table, float *lds) {
    using IV = typename Vec4<IdxT>::type;
    constexpr int kT = kWin / (kVec * kWave);
    constexpr int kChunk = kVec * kWave;
    const int64_t base = e0 & ~int64_t(kVec - 1);
    for (int64_t ws = base; ws < e1; ws += kWin) {
        const int64_t left = e1 - ws;  // wave-uniform
        IV iv[kT];
        float4 v[kT];
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            if (t * kChunk < left) {
                const int64_t e = ws + t * kChunk + lane * kVec;
                const int64_t ec = e < e1 ? e : ws + t * kChunk;
                iv[t] = load_stream(reinterpret_cast<const IV *>(idx + ec));
                if constexpr (UNIT)
                    v[t] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
                else
                    v[t] = load_stream(reinterpret_cast<const float4 *>(val + ec));
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
        wave_sync();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t lo = a[k] > ws ? a[k] : ws;
            const int64_t hi = b[k] < ws + kWin ? b[k] : ws + kWin;
            int o = (int)(lo - ws);
            const int oe = (int)(hi - ws);
            float s = acc[k];
            for (; o + 4 <= oe; o += 4) {
                const float x0 = lds[o], x1 = lds[o + 1], x2 = lds[o + 2], x3 = lds[o + 3];
                s = s + x0;
                s = s + x1;
                s = s + x2;
                s = s + x3;
            }
            for (; o < oe; ++o) s = s + lds[o];
            acc[k] = s;
        }
        wave_sync();
    }
}

__device__ __forceinline__ float sigmoid_ref(float z) {
    // lr.cc:113: 1. / (1. + exp(-z)) in double (glibc double exp there,
    // OCML's f64 exp here), returned as float.
    const double e = exp(-(double)z);
    return (float)(1.0 / (1.0 + e));
}

// K2: margin + sigmoid + residual.  A wave owns SEG consecutive batch rows
// (lane l < SEG owns row row0 + l); SEG < 64 gives small batches more waves
// to hide latency with (the loads and gathers still use all 64 lanes).
template <int SEG, bool UNIT = false>
__global__ __launch_bounds__(kWaves *kWave) void k_margin_residual(DevBatch bt, const float *__restrict__ w,
                                                                   float *__restrict__ resid) {
    __shared__ float s_p[kWaves][kWin];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wv) * SEG;
    if (row0 >= bt.rows) return;  // wave-uniform
    const int64_t my = row0 + lane;
    const bool valid = lane < SEG && my < bt.rows;
    const float y = valid ? bt.label[my] : 0.0f;
    const int64_t rlast = min(row0 + SEG, bt.rows);
    const int64_t e0 = bt.row_ptr[row0], e1 = bt.row_ptr[rlast];
    const int64_t a = valid ? bt.row_ptr[my] : e1, b = valid ? bt.row_ptr[my + 1] : e1;
    const float z = ordered_segment_dot<int32_t, UNIT>(e0, e1, a, b, lane, bt.col, bt.val, w, s_p[wv]);
    if (valid) resid[my] = sigmoid_ref(z) - y;
}

// K2 for frequency-ordered (relabeled) shards, e.g. BASELINE C3: the HOT
// lowest-numbered -- most frequent -- weights (58% of C3's entries fall in
// the first 8,192 columns) are staged in LDS once per workgroup, so their
// gathers read LDS and only the tail's go to L2.  Persistent workgroups
// (two per CU) loop over blocks of NW*SEG rows; otherwise k_margin_residual
// (same products, same in-order sums: bitwise the same margins).
// ho.off != null: after row i's residual, its hot columns' products
// fl32(r_i * x_ij) go to their product streams (DevHotOut) -- the same
// products k_band_hot forms from the residuals, in the same rounding.
template <int HOT, int NW, int SEG, bool UNIT>
__global__ __launch_bounds__(NW *kWave) void k_margin_hot(DevBatch bt, const float *__restrict__ w,
                                                          float *__restrict__ resid, DevHotOut ho) {
    __shared__ __attribute__((aligned(16))) float s_w[HOT];
    __shared__ float s_p[NW][kWin];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    {
        const float4 *src = reinterpret_cast<const float4 *>(w);
        float4 *dst = reinterpret_cast<float4 *>(s_w);
#pragma unroll
        for (int k = 0; k < HOT / 4 / (NW * kWave); ++k) dst[k * NW * kWave + threadIdx.x] = src[k * NW * kWave + threadIdx.x];
    }
    __syncthreads();
    const int64_t nblk = (bt.rows + NW * SEG - 1) / (NW * SEG);
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int64_t row0 = (blk * NW + wv) * SEG;
        if (row0 >= bt.rows) continue;  // wave-uniform (no barrier in the loop)
        const int64_t my = row0 + lane;
        const bool valid = lane < SEG && my < bt.rows;
        const float y = valid ? bt.label[my] : 0.0f;
        const int64_t rlast = min(row0 + SEG, bt.rows);
        const int64_t e0 = bt.row_ptr[row0], e1 = bt.row_ptr[rlast];
        const int64_t a = valid ? bt.row_ptr[my] : e1, b = valid ? bt.row_ptr[my + 1] : e1;
        const float z = ordered_segment_dot<int32_t, UNIT, HOT>(e0, e1, a, b, lane, bt.col, bt.val, w, s_p[wv],
                                                                 0.0f, s_w);
        if (valid) {
            const float r = sigmoid_ref(z) - y;
            resid[my] = r;
            if (ho.off) {
                const uint32_t t1 = ho.off[my + 1];
                for (uint32_t t = ho.off[my]; t < t1; ++t) ho.buf[ho.dest[t]] = UNIT ? r : r * ho.val[t];
            }
        }
    }
}


__device__ __forceinline__ double softplus(double t) { return t > 0 ? t + log1p(exp(-t)) : log1p(exp(t)); }

// K5: LR::Test / Predict_ (lr.cc:47-63, 100-106): pred = z > 0; correct
// count by wave ballot (integer atomics: order-free), log-loss partial per
// workgroup in a fixed order (deterministic for a fixed grid).
template <bool UNIT>
__global__ __launch_bounds__(kWaves *kWave) void k_predict(DevBatch bt, const float *__restrict__ w,
                                                           unsigned long long *__restrict__ correct,
                                                           double *__restrict__ ll_part) {
    __shared__ float s_p[kWaves][kWin];
    __shared__ double s_ll[kWaves];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wv) * kWave;
    double ll = 0.0;
    if (row0 < bt.rows) {
        const int64_t my = row0 + lane;
        const bool valid = my < bt.rows;
        const int64_t rlast = min(row0 + kWave, bt.rows);
        const int64_t e0 = bt.row_ptr[row0], e1 = bt.row_ptr[rlast];
        const int64_t a = valid ? bt.row_ptr[my] : e1, b = valid ? bt.row_ptr[my + 1] : e1;
        const float z = ordered_segment_dot<int32_t, UNIT>(e0, e1, a, b, lane, bt.col, bt.val, w, s_p[wv]);
        bool hit = false;
        if (valid) {
            const float y = bt.label[my];
            const int pred = z > 0.0f ? 1 : 0;
            hit = pred == (int)y;
            ll = y != 0.0f ? softplus(-(double)z) : softplus((double)z);
        }
        const unsigned long long m = __ballot(hit);
        if (lane == 0 && m) atomicAdd(correct, (unsigned long long)__popcll(m));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ll += __shfl_xor(ll, off);
    if (lane == 0) s_ll[wv] = ll;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < kWaves; ++i) t += s_ll[i];
        ll_part[blockIdx.x] = t;
    }
}

__global__ void k_sum_partials(const double *__restrict__ part, int n, double *__restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < n; ++i) t += part[i];
        *out = t;
    }
}

// K3 (+K4 when FUSED): one lane per feature column, the column's segment
// in batch-row order -> G_j is the reference's sequential fp32 sum; then
// the lr.cc:40 normalisation + L2 term.  FUSED (single rank) applies the
// server update in place: with W == 1, fl32(fl32(lr*g)/1.0f) == fl32(lr*g)
// for every mode (main.cc:71, 81).
template <typename RowT, bool FUSED, bool UNIT = false>
__global__ __launch_bounds__(kWaves *kWave) void k_grad(DevCsc cs, const RowT *__restrict__ crow, int64_t D,
                                                        const float *__restrict__ resid, float *__restrict__ w,
                                                        float *__restrict__ gout, float Bf, double Bd, float lr,
                                                        float C) {
    __shared__ float s_p[kWaves][kWin];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t wid = (int64_t)blockIdx.x * kWaves + wv;
    int64_t j0, jl;
    if (cs.wstart) {  // entry-balanced schedule (frequency-ordered columns are not)
        if (wid >= cs.nwaves) return;  // wave-uniform
        j0 = cs.wstart[wid];
        jl = cs.wstart[wid + 1];
    } else {
        j0 = wid * kWave;
        if (j0 >= D) return;  // wave-uniform
        jl = min(j0 + kWave, D);
    }
    const int64_t j = j0 + lane;
    const bool valid = j < jl;
    const float wj = valid ? w[j] : 0.0f;
    // bit 31 of ptr[j] marks a LONG column: its entries live in the long
    // arrays (k_long_segments / k_long_combine update it), its segment here
    // is empty
    const int64_t e0 = cs.ptr[j0] & kPtrMask, e1 = cs.ptr[jl] & kPtrMask;
    const uint32_t pj = valid ? cs.ptr[j] : 0u;
    const int64_t a = valid ? (int64_t)(pj & kPtrMask) : e1, b = valid ? (int64_t)(cs.ptr[j + 1] & kPtrMask) : e1;
    const float G = ordered_segment_dot<RowT, UNIT>(e0, e1, a, b, lane, crow, cs.val, resid, s_p[wv]);
    if (!valid || (pj & kLongFlag)) return;
    const float cw = C * wj;
    const float l2 = cw / Bf;
    const float g = (float)((double)G / Bd + (double)l2);
    if (FUSED) {
        const float step = lr * g;
        w[j] = wj - step;
    } else {
        gout[j] = g;
    }
}

// ---------------------------------------------------------------------------
// The LDS layout of one batch (DevPcsc: per 64-column group and row phase a
// block of entries, column by column, rows ascending, each block padded to 4
// entries) built ON THE DEVICE from the batch's CSR, for a streamed shard:
// then only the CSR and the block bases cross PCIe (the host's pcsc_fill
// output is ~45% of a C2 batch's bytes).  Same bytes as pcsc_fill:
//   (1) counts per (block, lane) by atomics; (2) a wave per block scans its
//   64 counts into the end offsets and per-lane cursors and zeroes the
//   block's padding; (3) entries scattered at atomically taken cursors --
//   in any order within a (block, lane) run -- then (4) every run sorted by
//   row (runs hold distinct rows: a column appears once per row), which is
//   pcsc_fill's row-ordered layout exactly.
__global__ __launch_bounds__(256) void k_pcsc_count(DevBatch bt, int P, int64_t R, uint32_t *__restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= bt.rows) return;
    const int64_t p = i / R;
    for (int64_t k = bt.row_ptr[i]; k < bt.row_ptr[i + 1]; ++k) {
        const uint32_t c = (uint32_t)bt.col[k];
        atomicAdd(cnt + ((int64_t)(c >> 6) * P + p) * 64 + (c & 63), 1u);
    }
}

__global__ __launch_bounds__(256) void k_pcsc_scan(const uint32_t *__restrict__ base, int64_t pblocks,
                                                   uint32_t *__restrict__ cnt, uint8_t *__restrict__ ends,
                                                   uint16_t *__restrict__ row, float *__restrict__ val) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t blk = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    if (blk >= pblocks) return;  // wave-uniform
    const uint32_t v = cnt[blk * 64 + lane];
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    const uint32_t b0 = base[blk];
    ends[blk * 64 + lane] = (uint8_t)incl;
    cnt[blk * 64 + lane] = b0 + incl - v;  // this lane's cursor
    const uint32_t total = __shfl(incl, 63);
    const uint32_t padded = (total + 3) & ~3u;
    if ((uint32_t)lane < padded - total) {  // the block's padding entries
        row[b0 + total + lane] = 0;
        val[b0 + total + lane] = 0.0f;
    }
}

template <bool UNIT>
__global__ __launch_bounds__(256) void k_pcsc_scatter(DevBatch bt, int P, int64_t R, uint32_t *__restrict__ cur,
                                                      uint16_t *__restrict__ row, float *__restrict__ val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= bt.rows) return;
    const int64_t p = i / R;
    const uint16_t li = (uint16_t)(i - p * R);
    for (int64_t k = bt.row_ptr[i]; k < bt.row_ptr[i + 1]; ++k) {
        const uint32_t c = (uint32_t)bt.col[k];
        const uint32_t pos = atomicAdd(cur + ((int64_t)(c >> 6) * P + p) * 64 + (c & 63), 1u);
        row[pos] = li;
        val[pos] = UNIT ? 1.0f : bt.val[k];
    }
}

__global__ __launch_bounds__(256) void k_pcsc_order(const uint32_t *__restrict__ base, const uint8_t *__restrict__ ends,
                                                    int64_t pblocks, uint16_t *__restrict__ row,
                                                    float *__restrict__ val) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (block, lane)
    if (q >= pblocks * 64) return;
    const int64_t blk = q >> 6;
    const int l = (int)(q & 63);
    const uint32_t b0 = base[blk];
    const uint32_t a = b0 + (l ? ends[q - 1] : 0u), e = b0 + ends[q];
    for (uint32_t x = a + 1; x < e; ++x) {  // insertion sort by row (runs are short)
        const uint16_t r = row[x];
        const float v = val[x];
        uint32_t y = x;
        for (; y > a && row[y - 1] > r; --y) {
            row[y] = row[y - 1];
            val[y] = val[y - 1];
        }
        row[y] = r;
        val[y] = v;
    }
}

// Long columns (classic layout, e.g. Zipf-hot features of a full-shard
// Criteo batch, BASELINE C3): a column with more than DLR_LONG_COLUMN
// entries (default 4,096) would be one lane's serial chain of millions of
// adds.  Its entries are cut into chunks of kLongChunk: each chunk is summed
// sequentially in batch-row order (lane per chunk, direct 16-byte loads),
// then k_long_combine adds the chunk partials in chunk order.  Deterministic
// (fixed chunking), but for these columns not the reference's single
// sequential sum -- DLR_LONG_COLUMN=0 keeps every column bitwise.
//
// One wave per chunk of kLongChunk = 256 entries: entry-parallel 16-byte
// loads (a hot column's rows ascend, so neighbouring lanes' residual
// gathers hit neighbouring lines), each lane adds its 4 products in order,
// the wave adds the 64 lane sums with a fixed xor-shuffle tree (fp add is
// commutative: every lane gets the same bits).  Fixed chunks + fixed tree:
// deterministic, more accurate than one fp32 chain.  (A lane-per-chunk
// sequential version took 5.35 ms on the C3 shard: each lane streamed its
// own region and the rows' locality was lost.)

// Chunk starts are 4-aligned; the low 2 bits of a column's end pointer (the
// next column's first start, or the batch's terminal entry) hold the
// column's padding count.  Valued: padding entries are (row 0, value 0) and
// summed like the others.  UNIT (no value array, every value 1.0f): the
// chunk ends before its padding.
template <typename RowT, bool UNIT = false>
__global__ __launch_bounds__(256) void k_long_segments(const uint32_t *__restrict__ sptr, int64_t nseg,
                                                       const uint32_t *__restrict__ sched,
                                                       const RowT *__restrict__ row, const float *__restrict__ val,
                                                       const float *__restrict__ resid, float *__restrict__ part) {
    using RV = typename Vec4<RowT>::type;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wpb = blockDim.x / kWave;
    const int64_t nw = (int64_t)gridDim.x * wpb;
    for (int64_t k = (int64_t)blockIdx.x * wpb + threadIdx.x / kWave; k < nseg; k += nw) {  // wave-uniform
        const int64_t s = sched ? (int64_t)sched[k] : k;
        const uint32_t a = sptr[s] & ~3u, bn = sptr[s + 1];  // b - a <= kLongChunk (+3 padding)
        const uint32_t b = UNIT ? (bn & ~3u) - (bn & 3u) : bn & ~3u;
        const uint32_t e = a + (uint32_t)lane * 4;  // arrays padded by kLongChunk entries
        const RV r4 = *reinterpret_cast<const RV *>(row + e);
        float4 v4;
        if constexpr (UNIT)
            v4 = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        else
            v4 = *reinterpret_cast<const float4 *>(val + e);
        // gathers unconditional (past the chunk the rows are the next
        // chunk's or padding: valid indices), masked after -- a load in a
        // divergent branch makes the compiler wait at the join
        const float g0 = resid[r4.x], g1 = resid[r4.y], g2 = resid[r4.z], g3 = resid[r4.w];
        const float x0 = e < b ? g0 * v4.x : 0.0f;
        const float x1 = e + 1 < b ? g1 * v4.y : 0.0f;
        const float x2 = e + 2 < b ? g2 * v4.z : 0.0f;
        const float x3 = e + 3 < b ? g3 * v4.w : 0.0f;
        float t = x0 + x1;
        t = t + x2;
        t = t + x3;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t = t + __shfl_xor(t, off);
        if (lane == 0) part[s] = t;
    }
}

// One long column per wave: lane l adds chunk partials l, l+64, ... in
// order, the wave adds the 64 lane sums with the fixed xor-shuffle tree
// (deterministic); then lr.cc:40 and the update (FUSED) or the pushed
// gradient.
// RAW (band layout): gout[j] = G, the column's raw sum; k_band_finalize
// applies lr.cc:40 and the update to every column.
template <bool FUSED, bool RAW = false>
__global__ __launch_bounds__(256) void k_long_combine(const uint32_t *__restrict__ cols,
                                                      const uint32_t *__restrict__ cseg, int64_t ncols,
                                                      const float *__restrict__ part, float *__restrict__ w,
                                                      float *__restrict__ gout, float Bf, double Bd, float lr,
                                                      float C) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t l = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    if (l >= ncols) return;  // wave-uniform
    const uint32_t s0 = cseg[l], s1 = cseg[l + 1];
    float G = 0.0f;
    uint32_t s = s0 + (uint32_t)lane;
    // 32 (then 8) partials in flight per lane, added in the same order: the
    // hottest column's wave (C3: ~20K partials) is the kernel's critical path
    for (; s + 31 * kWave < s1; s += 32 * kWave) {
        float x[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) x[u] = part[s + u * kWave];
#pragma unroll
        for (int u = 0; u < 32; ++u) G = G + x[u];
    }
    for (; s + 7 * kWave < s1; s += 8 * kWave) {
        float x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = part[s + u * kWave];
#pragma unroll
        for (int u = 0; u < 8; ++u) G = G + x[u];
    }
    for (; s < s1; s += kWave) G = G + part[s];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) G = G + __shfl_xor(G, off);
    if (lane != 0) return;
    const uint32_t j = cols[l];
    if (RAW) {
        gout[j] = G;
        return;
    }
    const float wj = w[j];
    const float cw = C * wj;
    const float l2 = cw / Bf;
    const float g = (float)((double)G / Bd + (double)l2);
    if (FUSED) {
        const float step = lr * g;
        w[j] = wj - step;
    } else {
        gout[j] = g;
    }
}

// K3 (+K4), LDS-resident residuals (batches of <= 65,536 rows).  Gathering
// r_i from L2 runs at ~250 G gathers/s chip-wide (tools/kbench: one L2
// request per gathered element), so here every workgroup (1,024 threads, one
// per CU) stages the residuals in LDS -- R = FILL*4,096 rows per phase,
// one or two phases -- and gathers them from LDS instead.  The batch's
// column-major copy is PHASE-SPLIT (DevPcsc): for each group of 64 columns
// and each phase, the block of entries whose row lies in the phase, column
// by column, rows ascending (at most 255 entries: one 256-entry window).
// Column j's entries in phase 0 precede those in phase 1 in batch-row
// order, so summing phase 0's run then phase 1's run IS lr.cc:37's order.
// Every load a wave needs (both phases' windows, its weights, the first
// fill) is issued up front; the next phase's fill is in flight while the
// current phase computes.  Loads are unconditional with clamped addresses
// (a load in a divergent branch makes the compiler wait at the join).
// Diagnostic builds only (tools/kbench defines DLR_STAMPS): per-workgroup
// s_memrealtime stamps at the kernel's phase boundaries.
#ifdef DLR_STAMPS
__device__ unsigned long long *g_stamp = nullptr;
}  // namespace
}  // namespace dlr
// tools/c2_stamps.py (a DLR_STAMPS build of the library): where the stamps go
extern "C" int dlr_debug_stamp_buffer(void *d) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(dlr::g_stamp), &d, sizeof(d));
}
namespace dlr {
namespace {
#define DLR_STAMP(slot)                                                                      \
    do {                                                                                     \
        if (threadIdx.x == 0) g_stamp[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// the same, written by thread tid (another wave's view)
#define DLR_STAMPW(slot, tid)                                                                \
    do {                                                                                     \
        if (threadIdx.x == (tid)) g_stamp[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// k_dense_ref: 64 slots per workgroup, written by one chosen lane
#define DLR_STAMP64(slot, cond)                                                                      \
    do {                                                                                             \
        if (cond) g_stamp[blockIdx.x * 64 + (slot)] = __builtin_amdgcn_s_memrealtime();               \
    } while (0)
#define DLR_STAMP64V(slot, cond, v)                                                                  \
    do {                                                                                             \
        if (cond) g_stamp[blockIdx.x * 64 + (slot)] = (v);                                           \
    } while (0)
// (the margin launch's workgroups: rows 256 + blockIdx.x)
#define DLR_STAMP64M(slot, cond)                                                                     \
    do {                                                                                             \
        if (cond) g_stamp[(256 + blockIdx.x) * 64 + (slot)] = __builtin_amdgcn_s_memrealtime();      \
    } while (0)
#define DLR_STAMP64MV(slot, cond, v)                                                                 \
    do {                                                                                             \
        if (cond) g_stamp[(256 + blockIdx.x) * 64 + (slot)] = (v);                                   \
    } while (0)
// time accumulators (s_memrealtime ticks) of one wave's loop phases
#define DLR_TACC_DECL(v) unsigned long long v = 0
#define DLR_TACC_BEGIN() unsigned long long tacc_t = __builtin_amdgcn_s_memrealtime()
#define DLR_TACC_LAP(v)                                                  \
    do {                                                                 \
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime(); \
        v += tn - tacc_t;                                                \
        tacc_t = tn;                                                     \
    } while (0)
#else
#define DLR_TACC_DECL(v) \
    do {                 \
    } while (0)
#define DLR_TACC_BEGIN() \
    do {                 \
    } while (0)
#define DLR_TACC_LAP(v) \
    do {                \
    } while (0)
#define DLR_STAMP(slot) \
    do {                \
    } while (0)
#define DLR_STAMPW(slot, tid) \
    do {                      \
    } while (0)
#define DLR_STAMP64(slot, cond) \
    do {                        \
    } while (0)
#define DLR_STAMP64V(slot, cond, v) \
    do {                            \
    } while (0)
#define DLR_STAMP64M(slot, cond) \
    do {                         \
    } while (0)
#define DLR_STAMP64MV(slot, cond, v) \
    do {                             \
    } while (0)
#endif
// Timing-only ablations of the stamps build (tools/c2_stamps.py; WRONG
// results): bit 0 no first residual fill, bit 1 no phase-0 window loads,
// bit 2 no pass 1, bit 3 no weight loads.  Always 0 in the product library.
// Bit 4 (a variant, same results): pass 1's product stores write-through
// (sc1), so they leave L2 as they issue instead of in the kernel-end flush.
// k_dense_ref (tools/c4_stamps.py --abl): bit 5 no chain halves (run with
// --lead 0), bit 6 no margin row chains (the stages stream, nothing adds).
#ifndef DLR_ABL
#define DLR_ABL 0
#endif
#ifndef DLR_MG_SLEEP  // the fused margin's poll interval (x 64 cycles)
#define DLR_MG_SLEEP 8
#endif
constexpr int kMgSub = 8;  // sub-counters per phase (DevP2)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#ifndef DLR_GRAD_WAVES  // A/B builds only (make variant VDEFS=...): 16 x 4 in the product
#define DLR_GRAD_WAVES 16
#define DLR_GRAD_NG 4
#endif
constexpr int kGradWaves = DLR_GRAD_WAVES;  // waves per workgroup
constexpr int kGradNG = DLR_GRAD_NG;        // 64-column groups per wave
constexpr int kBlk = 256;       // window = one phase block (<= 255 entries)
constexpr int kBlkPad = kBlk + 8;  // product slab per wave: lane reads at o + [0, 8) never leave it

// ---------------------------------------------------------------------------
// Product margin (LDS-layout batches; dlr_kernels.h DevPm).  The gather
// margin (k_margin_residual) issues one random 4-byte L2 request per entry
// and runs at the L2 request rate (C2: 3.28M per batch, ~21 us).  Here the
// weights are read by SLICE instead: pass 1 -- one workgroup per 4,096-column
// slice, i.e. the columns of one k_grad_lds workgroup, which can run it
// right after its update -- stages the slice's weights in LDS and forms the
// batch's products in the slice, writing them block by block into the
// product array; pass 2 -- a wave per 64-row block -- copies the block's
// products (one contiguous region) into LDS by 16-byte LDS-DMA and each
// lane adds its row's products in column order through a precomputed slot
// list.  Padding slots (chunks are whole 4-slot groups) hold w * 0 or any
// value: no slot list points at them.
// The products are the same fl32(w_j * x_ij) and each row's additions run in
// the same (column) order from +0: bitwise k_margin_residual's residuals.

// Pass 1 of one workgroup: the 4-entry groups [c0, c1) of slice s's list
// (chunks are padded to whole groups: a group is 4 consecutive product
// slots of one chunk, 16-byte aligned), U groups per thread in flight at
// once (the rest in further rounds); one 16-byte store per group.
template <int NT, int U>
struct PmPass1 {
    static constexpr int NPO = (kPmMaxBlocks + NT - 1) / NT;
    uint2 pk[U];  // a group: four 12-bit columns within the slice, block, rank / 4 (DevPm)
    float4 v[U];
    uint32_t po[NPO];
    uint32_t c0 = 0, c1 = 0;
    // group set u of the round starting at g0 (k_grad_rt spreads the sets
    // over its rounds)
    __device__ __forceinline__ void fetch_one(const DevPm &pm, uint32_t g0, int u) {
        // unit values: a dummy load (the list's own words, in range) keeps
        // the instruction count fixed
        const float4 *vp = pm.val ? reinterpret_cast<const float4 *>(pm.val) : reinterpret_cast<const float4 *>(pm.list);
        const uint32_t vs = pm.val ? 0u : 1u;
        const uint32_t g = g0 + u * NT + threadIdx.x;
        const uint32_t gc = g < c1 ? g : c0;
        pk[u] = load_stream(reinterpret_cast<const uint2 *>(pm.list) + gc);
        v[u] = load_stream(vp + (gc >> vs));
    }
    __device__ __forceinline__ void fetch(const DevPm &pm, uint32_t g0) {
#pragma unroll
        for (int u = 0; u < U; ++u) fetch_one(pm, g0, u);
    }
    // The slice's list range and chunk offsets (no dependence on anything):
    // k_grad_lds issues these first, so the fetch() that needs c0 waits for
    // them alone, not for the loads issued in between (vmcnt is in order).
    __device__ __forceinline__ void bounds(const DevPm &pm, int s, int part = 0, int nparts = 1) {
        // vector loads: a scalar load here made the compiler wait for it
        // (lgkmcnt(0)) before issuing anything else of the prologue
        int vz;  // a zero the compiler cannot prove uniform: keeps these loads in VGPRs
        asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
        const uint32_t b0 = pm.lbeg[s + vz] / 4, b1 = pm.lbeg[s + 1 + vz] / 4;
        const uint32_t n = b1 - b0, per = (n + nparts - 1) / nparts;
        c0 = b0 + min(n, per * part);
        c1 = b0 + min(n, per * (part + 1));
        const int64_t nb = pm.nblk;
#pragma unroll
        for (int u = 0; u < NPO; ++u) {
            const int64_t i = u * NT + threadIdx.x;
            po[u] = pm.pofs[(int64_t)s * nb + (i < nb ? i : nb - 1)];
        }
    }
    __device__ __forceinline__ void load(const DevPm &pm, int s, int part = 0, int nparts = 1) {
        bounds(pm, s, part, nparts);
        fetch(pm, c0);
    }
    __device__ __forceinline__ void stage_offsets(uint32_t *s_po) const {
#pragma unroll
        for (int u = 0; u < NPO; ++u) {
            const int i = u * NT + threadIdx.x;
            if (i < kPmMaxBlocks) s_po[i] = po[u];
        }
    }
    // s_w: the slice's weights; s_po: the staged chunk offsets.  A group's
    // slot is its first entry's (block, rank); padding entries (column 0,
    // value 0) fill slots no row reads.
    __device__ __forceinline__ void store(const DevPm &pm, const float *s_w, const uint32_t *s_po,
                                          float *__restrict__ p) {
        const bool unit = pm.val == nullptr;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7FFFFFFF, 0x00020000);
        (void)rs;
        for (uint32_t g0 = c0; g0 < c1; g0 += U * NT) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t g = g0 + u * NT + threadIdx.x;
                if (g < c1) {
                    const uint32_t x = pk[u].x, y = pk[u].y;
                    const uint32_t k = (y >> 16) & (kPmMaxBlocks - 1), j = (y >> 26) * 4;
                    float4 q;
                    q.x = s_w[x & 0xFFFu] * (unit ? 1.0f : v[u].x);
                    q.y = s_w[(x >> 12) & 0xFFFu] * (unit ? 1.0f : v[u].y);
                    q.z = s_w[(x >> 24) | ((y & 0xFu) << 8)] * (unit ? 1.0f : v[u].z);
                    q.w = s_w[(y >> 4) & 0xFFFu] * (unit ? 1.0f : v[u].w);
                    if (DLR_ABL & 16) {  // (stamps-build variant: write-through stores)
                        const u32x4 b = {__float_as_uint(q.x), __float_as_uint(q.y), __float_as_uint(q.z),
                                         __float_as_uint(q.w)};
                        __builtin_amdgcn_raw_buffer_store_b128(b, rs, (int)((s_po[k] + j) * 4u), 0, 16);
                    } else {
                        *reinterpret_cast<float4 *>(p + s_po[k] + j) = q;
                    }
                }
            }
            if (g0 + U * NT < c1) fetch(pm, g0 + U * NT);
        }
    }
};

// Standalone pass 1: SPLIT (pm.split) workgroups per slice, all on the
// slice's XCD (workgroup x runs on XCD x % 8): slice s = (x/8/SPLIT)*8 + x%8,
// so each XCD's L2 serves its 1/8 of w and the region chunks it writes are
// adjacent (a region's chunks are ordered by XCD).
// sl (optional): the slices to form, nsl of them (the exchange overlap forms
// the slices whose weights have landed, group by group).
__device__ __forceinline__ void pm_products_wg(const DevPm &pm, int x, const float *__restrict__ w, int64_t D,
                                               float *__restrict__ p, const uint32_t *__restrict__ sl, int64_t nsl,
                                               float *s_w, uint32_t *s_po) {
    const int xcd = x & 7, k = x >> 3;
    const int i = (k / pm.split) * 8 + xcd, part = k % pm.split;
    if (i >= (sl ? nsl : pm.S)) return;  // whole workgroup
    const int s = sl ? (int)sl[i] : i;
    PmPass1<1024, 4> pp;
    const int64_t j = (int64_t)s * kPmSlice + 4 * threadIdx.x;  // one float4 per thread
    const float4 wv = j + 3 < D ? *reinterpret_cast<const float4 *>(w + j)
                                : make_float4(j < D ? w[j] : 0.f, j + 1 < D ? w[j + 1] : 0.f,
                                              j + 2 < D ? w[j + 2] : 0.f, 0.f);
    pp.load(pm, s, part, pm.split);
    reinterpret_cast<float4 *>(s_w)[threadIdx.x] = wv;
    pp.stage_offsets(s_po);
    __syncthreads();
    pp.store(pm, s_w, s_po, p);
}
__global__ __launch_bounds__(1024) void k_pm_products(DevPm pm, const float *__restrict__ w, int64_t D,
                                                      float *__restrict__ p, const uint32_t *__restrict__ sl,
                                                      int64_t nsl) {
    __shared__ __attribute__((aligned(16))) float s_w[kPmSlice];
    __shared__ uint32_t s_po[kPmMaxBlocks];
    pm_products_wg(pm, blockIdx.x, w, D, p, sl, nsl, s_w, s_po);
}

// Pass 1 of several product-margin WINDOWS in one launch (band mode,
// TrainShard::pmw: the weights are fixed for the whole step): window v's
// workgroups are [v * G, (v + 1) * G), G = the one-window grid (a multiple
// of 8, so k_pm_products' XCD mapping holds inside every window and each
// XCD's L2 serves the same 1/8 of w for all of them); window v's products go
// to p + v * pstride.  One launch instead of one per window: the windows'
// 17 us launches were latency-bound (a thread's dozen entries in one round
// trip), a band's 8 at once stream.
__global__ __launch_bounds__(1024) void k_pm_products_win(const DevPm *__restrict__ views, int64_t G,
                                                          const float *__restrict__ w, int64_t D,
                                                          float *__restrict__ p, int64_t pstride) {
    __shared__ __attribute__((aligned(16))) float s_w[kPmSlice];
    __shared__ uint32_t s_po[kPmMaxBlocks];
    const int64_t v = blockIdx.x / G;
    const DevPm pm = views[v];
    pm_products_wg(pm, (int)(blockIdx.x - v * G), w, D, p + v * pstride, nullptr, 0, s_w, s_po);
}

// Pass 2 of block blk (one wave; lane l owns row 64 blk + l of bt) in the
// wave's kPmCap-float LDS region sr.  SC1: the residuals are stored with sc1
// (device scope), for readers on other CUs in the same launch (the fused
// margin of k_grad_lds below).
template <int QG, bool SC1>
__device__ __forceinline__ void pm_rowsum(const DevPm &pm, const DevBatch &bt, const float *__restrict__ p,
                                          float *resid, int64_t blk, float *sr, int lane) {
    const int64_t r0 = blk * kPmRows;
    // (fixed strides: no dependent load at the head of the hand-off chain)
    const uint32_t a = pm.rstride ? (uint32_t)blk * pm.rstride : pm.rg[blk];
    const uint32_t b = pm.rstride ? a + pm.rstride : pm.rg[blk + 1];
    const uint32_t q0 = pm.qstride ? (uint32_t)blk * pm.qstride : pm.qoff[blk];
    const uint32_t q1 = pm.qstride ? q0 + pm.qstride : pm.qoff[blk + 1];
    const int64_t my = r0 + lane;
    const bool valid = my < bt.rows;
    const int64_t mc = valid ? my : r0;
    const int len = valid ? (int)(bt.row_ptr[mc + 1] - bt.row_ptr[mc]) : 0;
    const float y = bt.label[mc];
    const int n4 = (int)((b - a) >> 2);
    const int ngrp = (int)((q1 - q0) >> 9);
    constexpr int R4 = kPmCap / 4 / kWave;
    // the region (straight into LDS by LDS-DMA: 1 KiB per wave-instruction,
    // lane l's 16 bytes at +16*l; lanes past the region re-copy its start
    // into slots no slot list reads) and the slot lists, all in flight at
    // once (tools/kbench/kb_pmargin.hip: 6.0 -> 5.2 us against staging the
    // region through registers)
#pragma unroll
    for (int t = 0; t < R4; ++t)
        if (t * kWave < n4) {
            const int e = t * kWave + lane < n4 ? t * kWave + lane : 0;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(p + a + 4 * e),
                                             (__attribute__((address_space(3))) void *)(sr + t * 4 * kWave), 16, 0,
                                             0);
        }
    uint4 qv[QG];
#pragma unroll
    for (int g = 0; g < QG; ++g)
        if (g < ngrp) qv[g] = load_stream(reinterpret_cast<const uint4 *>(pm.qs + q0) + g * kWave + lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA copies (not tracked by the compiler)
    wave_sync();
    float acc = 0.0f;
#pragma unroll
    for (int g = 0; g < QG; ++g) {
        if (g >= ngrp) break;  // wave-uniform
        const uint32_t qq[4] = {qv[g].x, qv[g].y, qv[g].z, qv[g].w};
        float x[8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            x[2 * u] = sr[qq[u] & 0xFFFFu];
            x[2 * u + 1] = sr[qq[u] >> 16];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float t = acc + x[u];
            acc = (g * 8 + u < len) ? t : acc;
        }
    }
    if (valid) {
        const float r = sigmoid_ref(acc) - y;
        if (SC1) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(resid, 0, 0x7FFFFFFF, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r), rs, (int)(my * 4), 0, 16);  // sc1
        } else {
            resid[my] = r;
        }
    }
}

// Pass 2: a wave per block.
// NW waves (blocks) per workgroup: 4, or 1 for a small batch (B <= 8,192:
// 128 blocks), whose blocks would otherwise share 32 CUs' memory paths --
// each block pulls ~20 KB (region + slot lists) at once
template <int QG, int NW = 4>
__global__ __launch_bounds__(NW *kWave) void k_pm_margin(DevPm pm, DevBatch bt, const float *__restrict__ p,
                                                         float *__restrict__ resid) {
    __shared__ __attribute__((aligned(16))) float s_reg[NW][kPmCap];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int64_t blk = (int64_t)blockIdx.x * NW + wv;
    if (blk * kPmRows >= bt.rows) return;  // wave-uniform
    pm_rowsum<QG, false>(pm, bt, p, resid, blk, s_reg[wv], lane);
}

// Pass 2 of several windows in one launch (k_pm_products_win's): bt is the
// windows' rows from the first's, window v = rows [v * kPmWinRows, + its
// rows) with its products at p + v * pstride; G = kPmMaxBlocks / 4
// workgroups a window (a wave per 64-row block).
template <int QG>
__global__ __launch_bounds__(256) void k_pm_margin_win(const DevPm *__restrict__ views, DevBatch bt,
                                                       const float *__restrict__ p, int64_t pstride,
                                                       float *__restrict__ resid) {
    __shared__ __attribute__((aligned(16))) float s_reg[4][kPmCap];
    constexpr int64_t G = kPmMaxBlocks / 4, kWinRows = (int64_t)kPmMaxBlocks * kPmRows;
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int64_t v = blockIdx.x / G;
    const int64_t blk = (blockIdx.x - v * G) * 4 + wv;
    DevBatch sub = bt;
    sub.row_ptr = bt.row_ptr + v * kWinRows;
    sub.label = bt.label + v * kWinRows;
    sub.rows = min(kWinRows, bt.rows - v * kWinRows);
    if (blk * kPmRows >= sub.rows) return;  // wave-uniform
    const DevPm pm = views[v];
    pm_rowsum<QG, false>(pm, sub, p + v * pstride, resid + v * kWinRows, blk, s_reg[wv], lane);
}

// PM (with FUSED): after the update, form the NEXT batch's products of this
// workgroup's slice (pm_pass1 below) from the new weights.
// MG (with PM; one rank): this batch's pass 2 (the margin) runs in the same
// launch, first thing (dlr_kernels.h DevP2): wave v of workgroup x sums
// block x + v * grid in LDS that the residual fills use only later, stores
// the residuals with sc1 and adds 1 to its phase's counter (agent scope);
// every workgroup waits for phase p's count before its fill of phase p
// (wave 0 polls with sc1 loads, bounded; the fill is sc1 too).  The grid is
// one workgroup per CU (LDS), so all of them are resident and every block
// is summed; the pass-1 stores into p come after the last phase's wait, so
// after every block's copy of its region.  The launch boundary between the
// margin and the gradient is gone and the gradient's window loads stream
// while the blocks are summed.
// (A double-buffered form -- phases of 16,384 rows in two 64 KB buffers,
// each fill streaming while the previous phase computes -- was measured
// slower: C2 31.2 vs 24.8 us per step, a phase costing nearly what a
// 32,768-row one does; profiles/r05_stamps_c2_db.txt.  Removed in round 6.)
template <int FILL, bool FUSED, bool PM = false, bool MG = false>
__global__ __launch_bounds__(kGradWaves *kWave) void k_grad_lds(DevPcsc pc, int64_t D, int64_t B,
                                                                const float *__restrict__ resid,
                                                                float *__restrict__ w, float *__restrict__ gout,
                                                                float Bf, double Bd, float lr, float C,
                                                                DevPm pn = DevPm{}, float *__restrict__ pm_p = nullptr,
                                                                DevP2 p2 = DevP2{}) {
    constexpr int R = FILL * 4096;      // rows per phase
    constexpr int NPH = 2;              // phases
    constexpr int NG = kGradNG;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *s_r = smem;
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // uniform: scalar block loads
    float *s_p = smem + R + wv * kBlkPad;
    const uint32_t s_r_a = lds_addr(s_r), s_p_a = lds_addr(s_p);
    const int P = pc.phases;
    const int64_t ng = (D + 63) / 64;
    const int64_t gfirst = (int64_t)blockIdx.x * (kGradWaves * NG) + wv;
    PmPass1<kGradWaves * kWave, 4> pm;
    // (MG: workgroups past the slices only sum blocks)
    if (PM && !(DLR_ABL & 4) && (!MG || blockIdx.x < pn.S)) pm.bounds(pn, blockIdx.x);  // first (PmPass1::bounds)
    static_assert(!MG || (PM && FUSED), "the fused margin comes with the fused pass 1");
    if constexpr (MG) {
        DLR_STAMP(11);
        if (blockIdx.x == 0 && wv < 8)  // the next launch's bank: 64 phases x 8 sub-counters
            p2.cnt[(((p2.gen + 1) & 1) * 64 + lane) * kMgSub * 32 + wv * 32] = 0u;
        const int64_t k2 = blockIdx.x + (int64_t)gridDim.x * wv;  // wv < FILL (launch_grad_lds_pm)
        if (k2 < p2.pm.nblk) {  // wave-uniform
            pm_rowsum<8, true>(p2.pm, p2.bt, pm_p, p2.resid, k2, smem + wv * kPmCap, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every residual of the block stored
            // sub-counter k2 % 8 of the phase (each on a line of its own:
            // the adds and the polls spread over 8 lines)
            if (lane == 0 && !(p2.fault == kFaultMgPublish && k2 == 0))
                __hip_atomic_fetch_add(
                    p2.cnt + (((p2.gen & 1) * 64 + (k2 * kPmRows) / R) * kMgSub + (k2 % kMgSub)) * 32, 1u,
                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        DLR_STAMP(12);
        DLR_STAMPW(14, 3 * kWave);  // wave 3's block (the last of a CU's four)
        if (blockIdx.x >= pn.S) return;  // a block-only workgroup (launch_grad_lds_pm): done
        // the other waves' window loads wait for the workgroup's blocks (the
        // blocks' loads have the CU's memory path to themselves: the phases
        // wait for the slowest block; issued at once: 28.0 vs 26.8 us)
        lds_barrier();
    }
    // wave 0 waits until every block of phase p is published (the caller's
    // barrier then holds the other waves' fills); a wait that runs out is
    // reported (Spin)
    // The same poll reads the LATER phases' counters too (lane 8d + s:
    // sub-counter s of phase p + d, d < NPH): the blocks of every phase are
    // summed at the launch's start, so the later phases are nearly always
    // complete when phase p is, and their own polls -- round trips queued
    // behind the windows, fills and pass-1 list loads -- are skipped
    // (mg_done: the phases known complete).
    Spin spin(MG ? p2.err : nullptr, kErrMgPublish);
    int mg_done = 0;
    auto mg_wait = [&](int p) {
        if constexpr (MG) {
            if (wv == 0 && p >= mg_done) {
                constexpr int64_t bpp = R / kPmRows;
                auto want_of = [&](int q) {
                    return (uint32_t)(min<int64_t>(p2.pm.nblk, (q + 1) * bpp) - q * bpp);
                };
                const __amdgpu_buffer_rsrc_t crs =
                    __builtin_amdgcn_make_buffer_rsrc(p2.cnt, 0, 0x7FFFFFFF, 0x00020000);
                // (phases past the last read the last one again)
                const int q = min(p + ((lane >> 3) & (NPH - 1)), P - 1);
                const int off = (int)(((((p2.gen & 1) * 64 + q) * kMgSub + (lane & (kMgSub - 1))) * 32) * 4);
                for (int k = 0; spin.more(k); ++k) {
                    const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(crs, off, 0, 16);
                    uint32_t n[NPH];
#pragma unroll
                    for (int d = 0; d < NPH; ++d) {
                        n[d] = 0;
#pragma unroll
                        for (int i = 0; i < kMgSub; ++i) n[d] += __builtin_amdgcn_readlane(v, d * kMgSub + i);
                    }
                    if (n[0] >= want_of(p)) {
                        int done = p + 1;
#pragma unroll
                        for (int d = 1; d < NPH; ++d)
                            if (done == p + d && p + d < P && n[d] >= want_of(p + d)) done = p + d + 1;
                        mg_done = done;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(DLR_MG_SLEEP);
                }
            }
        }
    };
    // per group: the bases of its phase blocks (blocks gc*P + q are
    // consecutive: P + 1 bases give every block's first entry and its
    // entries rounded up to 4 -- blocks are 4-aligned: a lane's first
    // window slot 4*lane is an entry iff 4*lane < that) -- wave-uniform,
    // all phases up front; per lane: its column's inclusive end offset in
    // the block (<= 255) for the phases in registers (set p & 1; meta) --
    // the column's start is lane - 1's end (a lane shuffle at its use, so
    // that no arithmetic waits for the load where it is issued)
    constexpr int RS = 2;
    auto rs = [](int p) { return p & 1; };
    unsigned sb[NG][NPH + 1], hb[NG][RS];
    float acc[NG], wj[NG];
    ushort4 rq[NG][RS];
    float4 vq[NG][RS];
    // (the bases first, and straight into SGPRs: the windows' addresses
    // need them at once, and a base left in a VGPR made the compiler wait
    // for every load in flight where the next phase's windows are issued)
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t g = gfirst + kGradWaves * gi;
        const int64_t gc = g < ng ? g : ng - 1;
#pragma unroll
        for (int q = 0; q <= NPH; ++q) sb[gi][q] = pc.base[gc * P + (q < P ? q : P)];
    }
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
#pragma unroll
        for (int q = 0; q <= NPH; ++q) sb[gi][q] = __builtin_amdgcn_readfirstlane(sb[gi][q]);
        const int64_t j = (gfirst + kGradWaves * gi) * 64 + lane;
        wj[gi] = (DLR_ABL & 8) ? 0.0f : w[j < D ? j : D - 1];
        acc[gi] = 0.0f;
    }
    auto bs_of = [&](int gi, int p) { return sb[gi][p]; };
    auto nblk_of = [&](int gi, int p) { return sb[gi][p + 1] - sb[gi][p]; };
    auto meta = [&](int p) {
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            const int64_t g = gfirst + kGradWaves * gi;
            const int64_t blk = (g < ng ? g : ng - 1) * P + (p < P ? p : P - 1);
            hb[gi][rs(p)] = pc.ends[blk * 64 + lane];
        }
    };
    meta(0);
    meta(1);
    auto windows = [&](int p, int g0 = 0, int g1 = NG) {
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            if (gi < g0 || gi >= g1) continue;
            if ((DLR_ABL & 2) && p == 0) {
                rq[gi][0] = ushort4{0, 0, 0, 0};
                vq[gi][0] = make_float4(0.f, 0.f, 0.f, 0.f);
                continue;
            }
            // lanes past the block re-read its last 4 entries: the wave's
            // addresses then span the block only (the next blocks' lines are
            // not pulled into this CU), and a duplicate address costs nothing
            const unsigned nb4 = nblk_of(gi, p);
            const unsigned e = bs_of(gi, p) + min((unsigned)lane * 4, nb4 ? nb4 - 4 : 0u);  // padded: in bounds
            // (plain loads: non-temporal ones measured slower, 19.4 vs 16.6 us
            // for the gradient alone -- the kernel is latency-bound)
            rq[gi][rs(p)] = *reinterpret_cast<const ushort4 *>(pc.row + e);
            vq[gi][rs(p)] = *reinterpret_cast<const float4 *>(pc.val + e);
        }
    };
    // Residual fills by LDS-DMA (no VGPRs): each wave-instruction copies
    // 1 KiB -- lane l's 16 bytes land at the wave-uniform base + 16*l.
    // (MG: the residuals were stored in this launch by other CUs, through
    // p2.resid.  Plain loads: no CU reads a residual line before its block
    // is published -- the launch starts with this XCD's L2 and every L1
    // holding no residual line (the kernel-start acquire), the blocks' sc1
    // stores have reached memory before their counter moved, and a line
    // belongs to one block -- so the first read of a line, and every later
    // hit on it, sees the stored values.)
    const float *rsrc = MG ? p2.resid : resid;
    auto fill = [&](int64_t lo) {
#pragma unroll
        for (int f = 0; f < R / (kGradWaves * kWave * 4); ++f) {  // FILL with 16 waves
            const int o = (f * kGradWaves + wv) * kWave * 4;  // floats; this wave's 1 KiB slot
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(rsrc + lo + o + lane * 4),
                (__attribute__((address_space(3))) void *)(s_r + o), 16, 0, 0);
        }
    };
    // Group gi's products and column sums of phase p (residuals at LDS
    // address sra); false when the wave has no group gi.
    auto group = [&](int gi, int p, uint32_t sra) -> bool {
        if (gfirst + kGradWaves * gi >= ng) return false;  // wave-uniform
        // products of the block's entries only: the window's other slots
        // (the next blocks' entries) are never read, so those lanes skip
        // their residual gathers (LDS bank cycles) and the slab write
        // (LDS through lds_* asm: the pass-1 loads stay in flight)
        if ((unsigned)lane * 4 < nblk_of(gi, p)) {
            const ushort4 r4 = rq[gi][rs(p)];
            const float4 v4 = vq[gi][rs(p)];
            float g0 = lds_rd32(sra + 4u * r4.x), g1 = lds_rd32(sra + 4u * r4.y);
            float g2 = lds_rd32(sra + 4u * r4.z), g3 = lds_rd32(sra + 4u * r4.w);
            lds_wait4(g0, g1, g2, g3);
            const v4f q = {g0 * v4.x, g1 * v4.y, g2 * v4.z, g3 * v4.w};
            lds_wr128(s_p_a + 16u * lane, q);
        }
        // the slab is complete: a wave's LDS operations complete in issue
        // order, so the reads below follow the slab writes without a wait
        // this lane's column: cnt products in order from off.  The first
        // eight are read at immediate offsets from s_p + o (the slab is
        // padded, so no clamping) and added while any lane still has one
        // (a wave-uniform exit: the sum stops at the wave's largest count,
        // ~5 at C2's 1.6 entries per column and phase); the rare longer
        // runs continue in a general loop.  Per product: compare, add,
        // select.  Not the bound: the SQ counters put VALU issue at <= ~20%
        // busy (profiles/r02f_c2_sq_counters.txt); the kernel is bound by
        // its chain of dependent memory phases (tools/c2_stamps.py).
        const unsigned hi = hb[gi][rs(p)];
        // (the shuffle outside the lane test: inside it, lane 0 -- the
        // source of lane 1's start -- would be inactive)
        const unsigned up = (unsigned)__shfl_up((int)hi, 1);
        const unsigned o = lane ? up : 0u;
        const bool cok = p < P && (gfirst + kGradWaves * gi) * 64 + lane < D;
        const unsigned c = cok ? hi - o : 0u;
        const uint32_t sp = s_p_a + 4u * o;
        float a = acc[gi];
        // all eight reads issue together (one LDS round trip)
        float x[8];
        x[0] = lds_rd32<0>(sp), x[1] = lds_rd32<4>(sp), x[2] = lds_rd32<8>(sp), x[3] = lds_rd32<12>(sp);
        x[4] = lds_rd32<16>(sp), x[5] = lds_rd32<20>(sp), x[6] = lds_rd32<24>(sp), x[7] = lds_rd32<28>(sp);
        lds_wait4(x[0], x[1], x[2], x[3]);
        lds_wait4(x[4], x[5], x[6], x[7]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool take = (unsigned)u < c;
            if (__builtin_amdgcn_ballot_w64(take) == 0) break;  // wave-uniform
            const float t = a + x[u];
            a = take ? t : a;
        }
        for (unsigned k = 8; __builtin_amdgcn_ballot_w64(k < c) != 0; ++k) {
            float xv = lds_rd32(s_p_a + 4u * min(o + k, (unsigned)kBlk - 1));
            lds_wait1(xv);
            if (k < c) a = a + xv;
        }
        acc[gi] = a;
        wave_sync();
        return true;
    };
    // All NG groups of phase p, software-pipelined (the wave has all of
    // them; 24.6 vs 25.0 us against group() in turn): per group one LDS round trip -- the slab write, its
    // reads and the next group's residual gathers issued together, then a
    // wait for all but those 4 gathers (LDS returns in order; an older
    // scalar load in the count only makes the wait stricter).  The same
    // products and the same additions as group(): bitwise.
    auto group_pipe = [&](int p, uint32_t sra, auto &&hooks) {
        unsigned o[NG], c[NG];
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            const unsigned hi = hb[gi][rs(p)];
            const unsigned up = (unsigned)__shfl_up((int)hi, 1);
            o[gi] = lane ? up : 0u;
            c[gi] = (p < P && (gfirst + kGradWaves * gi) * 64 + lane < D) ? hi - o[gi] : 0u;
        }
        float g[2][4], x[8];
        auto gath = [&](int gi, float(&gg)[4]) {
            // every lane (lanes past the block gather its last entries'
            // rows: in range, their products land in slab slots no run reads)
            const ushort4 r4 = rq[gi][rs(p)];
            gg[0] = lds_rd32(sra + 4u * r4.x), gg[1] = lds_rd32(sra + 4u * r4.y);
            gg[2] = lds_rd32(sra + 4u * r4.z), gg[3] = lds_rd32(sra + 4u * r4.w);
        };
        gath(0, g[0]);
        lds_wait4(g[0][0], g[0][1], g[0][2], g[0][3]);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            hooks(gi);
            float(&gc)[4] = g[gi & 1];
            const float4 v4 = vq[gi][rs(p)];
            const v4f q = {gc[0] * v4.x, gc[1] * v4.y, gc[2] * v4.z, gc[3] * v4.w};
            lds_wr128(s_p_a + 16u * lane, q);
            const uint32_t sp = s_p_a + 4u * o[gi];
            x[0] = lds_rd32<0>(sp), x[1] = lds_rd32<4>(sp), x[2] = lds_rd32<8>(sp), x[3] = lds_rd32<12>(sp);
            x[4] = lds_rd32<16>(sp), x[5] = lds_rd32<20>(sp), x[6] = lds_rd32<24>(sp), x[7] = lds_rd32<28>(sp);
            if (gi + 1 < NG) {
                float(&gn)[4] = g[(gi + 1) & 1];
                gath(gi + 1, gn);
                asm volatile("s_waitcnt lgkmcnt(4)"
                             : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                               "+v"(x[7]));
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                               "+v"(x[7]));
            }
            float a = acc[gi];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const bool take = (unsigned)u < c[gi];
                if (__builtin_amdgcn_ballot_w64(take) == 0) break;  // wave-uniform
                const float t = a + x[u];
                a = take ? t : a;
            }
            for (unsigned k = 8; __builtin_amdgcn_ballot_w64(k < c[gi]) != 0; ++k) {
                float xv = lds_rd32(s_p_a + 4u * min(o[gi] + k, (unsigned)kBlk - 1));
                lds_wait1(xv);  // (lgkmcnt(0): the next group's gathers land too)
                if (k < c[gi]) a = a + xv;
            }
            acc[gi] = a;
            if (gi + 1 < NG) {
                float(&gn)[4] = g[(gi + 1) & 1];
                lds_wait4(gn[0], gn[1], gn[2], gn[3]);
            }
        }
    };
    // Phase 0's windows and the first fill are issued up front.  (Wave 0's
    // poll returns behind its own window loads -- vmcnt is in order -- but
    // polling first was no faster: 26.96 us, profiles/r04mg.)
    DLR_STAMP(0);
    windows(0);
    if constexpr (MG) {
        mg_wait(0);
        lds_barrier();  // and this workgroup's pass-2 regions are read
        DLR_STAMP(13);
    }
    if (!(DLR_ABL & 1)) fill(0);
    DLR_STAMP(8);
#ifdef DLR_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DLR_STAMP(9);
#endif
    DLR_STAMP(10);
    bool listed = false;  // (wave-uniform) this wave issued its share of the pass-1 list
    int nsets = 0;        // the list's group sets issued (phase 1: one before each group)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        if (p >= P) break;  // uniform
        if (p > 0) {
            DLR_STAMP(2);
            mg_wait(p);
            lds_barrier();  // every wave is done reading the previous phase
            DLR_STAMP(3);
            fill((int64_t)p * R);  // resid is padded to P*R floats
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA fill (not tracked by the compiler)
        lds_barrier();
        DLR_STAMP(1 + 3 * p);
        // The loads issued between phase p's groups (VMEM only), after the
        // first group's compiler-placed waits so that they do not delay
        // phase 0's start: in phase 0, phase 1's windows group by group
        // (2 before group 1, then one per group: 25.16 vs 25.24 us at once);
        // in phase 1, the next batch's pass-1 list, one of its four group
        // sets before each group (25.3 vs 25.7 at once, vs 26.5 in phase 0:
        // profiles/r05_c2_issue_order.txt).  A one-phase batch issues the
        // whole list in phase 0.
        auto hooks = [&](int gi) {
            if (p == 0 && gi >= 1) {
                asm volatile("" ::: "memory");
                if (P > 1) {
                    if (gi == 1)
                        windows(1, 0, 2);
                    else
                        windows(1, gi, gi + 1);
                } else if (gi == 1 && PM && !(DLR_ABL & 4)) {
                    pm.fetch(pn, pm.c0);
                    listed = true;
                }
                asm volatile("" ::: "memory");
            }
            if (p == 1 && PM && !(DLR_ABL & 4)) {
                asm volatile("" ::: "memory");
                pm.fetch_one(pn, pm.c0, gi);
                nsets = gi + 1;
                asm volatile("" ::: "memory");
            }
        };
        // a wave with all NG groups software-pipelines them -- group gi +
        // 1's residual gathers in flight with group gi's slab reads and
        // adds, the slab rewritten after the reads are issued: a wave's LDS
        // operations complete in issue order (24.6 vs 25.0 us in turn)
        if (gfirst + kGradWaves * (NG - 1) < ng) {
            group_pipe(p, s_r_a, hooks);
        } else {
#pragma unroll
            for (int gi = 0; gi < NG; ++gi) {
                hooks(gi);
                if (!group(gi, p, s_r_a)) break;
            }
        }
    }
    // a wave with no column group left the loop before issuing its share of
    // the pass-1 list (every thread takes part in pass 1)
    if (PM && !(DLR_ABL & 4) && !listed) {
        if (P > 1) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (u >= nsets) pm.fetch_one(pn, pm.c0, u);
        } else {
            pm.fetch(pn, pm.c0);
        }
    }
#ifdef DLR_STAMPS
    __syncthreads();
    DLR_STAMP(5);
#endif
    if (PM) lds_barrier();  // every wave is done with s_r: pass 1 reuses it
    // lr.cc:40 divides by B; for a power-of-two B a product with the exact
    // reciprocal IS that correctly rounded quotient (C2: B = 65,536), and the
    // f64 division sequence x 4 groups x 4 waves per SIMD costs ~1 us here
    auto update = [&](auto pow2) {
        constexpr bool P2 = decltype(pow2)::value;
        const float rBf = P2 ? 1.0f / Bf : 0.0f;
        const double rBd = P2 ? 1.0 / Bd : 0.0;
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            const int64_t j = (gfirst + kGradWaves * gi) * 64 + lane;
            if (gfirst + kGradWaves * gi >= ng || j >= D) continue;
            const float cw = C * wj[gi];
            const float l2 = P2 ? cw * rBf : cw / Bf;
            const float g = (float)((P2 ? (double)acc[gi] * rBd : (double)acc[gi] / Bd) + (double)l2);
            if (FUSED) {
                const float step = lr * g;
                const float wn = wj[gi] - step;
                w[j] = wn;
                if (PM) smem[(wv + kGradWaves * gi) * 64 + lane] = wn;  // column j - kPmSlice*blockIdx.x
            } else {
                gout[j] = g;
            }
        }
    };
    if ((B & (B - 1)) == 0)
        update(std::true_type{});
    else
        update(std::false_type{});
    if (PM) {
        pm.stage_offsets(reinterpret_cast<uint32_t *>(smem + kPmSlice));
        lds_barrier();
        DLR_STAMP(6);
        if (!(DLR_ABL & 4)) pm.store(pn, smem, reinterpret_cast<const uint32_t *>(smem + kPmSlice), pm_p);
    }
#ifdef DLR_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    DLR_STAMP(7);
#endif
}

// ---------------------------------------------------------------------------
// Row-round gradient (RT; product-margin batches, dlr_kernels.h DevRt).
// k_grad_lds stages the residuals of a whole 32,768-row phase before it can
// multiply anything (its column-major windows span the phase), so each CU
// waits for two 128 KB fills in turn and every phase ends at a barrier.
// Here the workgroup of slice s reads its entries in ROW order -- pass 1's
// list order -- so the batch is consumed in rounds of kRtRows rows: round
// t needs only rows [t*R, (t+1)*R) of the residuals (32 KB).  Every round's
// entries (one 4-entry group per thread, at a fixed stride: no offsets to
// load first) are in flight from the start, the residuals of rounds t+1 and
// t+2 while round t computes.  Each entry's product fl32(r_i * x_ij) goes to
// its slot in the slice's column-major order in LDS; after the last round
// each lane adds its column's run of products in order (rows ascending)
// from +0: the same products and the same additions as lr.cc:35-39, bitwise
// k_grad_lds's sums.  The update and the fused pass 1 are k_grad_lds's.
template <typename F, int... I>
__device__ __forceinline__ void unroll_seq(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

// MG (with PM; one rank): this batch's pass 2 runs at the start of the
// launch, as in k_grad_lds MG: wave v < 5 of workgroup x sums block
// x + grid * v in the product area (not yet in use), stores its residuals
// with sc1 and counts them per round; the round's entries are loaded
// meanwhile, and wave 0 waits for every round's blocks before any residual
// load (plain loads of lines no CU read before their block was published).
template <bool FUSED, bool PM, bool UNIT, bool MG = false>
__global__ __launch_bounds__(kGradWaves *kWave) void k_grad_rt(DevRt rt, int64_t D, const float *__restrict__ resid,
                                                               float *__restrict__ w, float *__restrict__ gout,
                                                               float Bf, double Bd, float lr, float C,
                                                               DevPm pn = DevPm{}, float *__restrict__ pm_p = nullptr,
                                                               DevP2 p2 = DevP2{}) {
    constexpr int NT = kGradWaves * kWave;
    constexpr int NG = kGradNG;
    constexpr int kSink = 16;  // the sink slot kRtCap and the chain's unclamped reads past a run
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *s_prod = smem;
    float *s_r = smem + kRtCap + kSink;
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int s = blockIdx.x;
    const int64_t ng = (D + 63) / 64;
    const int64_t gfirst = (int64_t)s * (kGradWaves * NG) + wv;
    DLR_STAMP(0);
    const int T = rt.rounds;
    static_assert(!MG || (PM && FUSED), "the fused margin comes with the fused pass 1");
    if constexpr (MG) {
        if (blockIdx.x == 0 && wv < 8)  // the next launch's bank (DevP2)
            p2.cnt[(((p2.gen + 1) & 1) * 64 + lane) * kMgSub * 32 + wv * 32] = 0u;
        const int64_t k2 = blockIdx.x + (int64_t)gridDim.x * wv;  // wv < kRtRegions (launch_grad_rt)
        if (wv < kRtRegions && k2 < p2.pm.nblk) {  // wave-uniform
            pm_rowsum<8, true>(p2.pm, p2.bt, pm_p, p2.resid, k2, smem + wv * kPmCap, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every residual of the block stored
            if (lane == 0 && !(p2.fault == kFaultMgPublish && k2 == 0))
                __hip_atomic_fetch_add(
                    p2.cnt + (((p2.gen & 1) * 64 + (k2 * kPmRows) / kRtRows) * kMgSub + (k2 % kMgSub)) * 32, 1u,
                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        lds_barrier();  // the regions are read: the product area is free
    }
    const float *rsrc = MG ? p2.resid : resid;
    // (MG) wave kPoller waits until every round's blocks are published; the
    // caller's barrier holds the other waves' residual loads.  (The last
    // wave, which sums no block, polling instead: measured no faster.)
    constexpr int kPoller = 0;
    static_assert(kPoller == 0 || kPoller >= kRtRegions, "the poller sums no block");
    auto mg_wait_all = [&]() {
        if constexpr (MG) {
            if (wv == kPoller) {
                Spin spin(p2.err, kErrMgPublish);
                const __amdgpu_buffer_rsrc_t crs =
                    __builtin_amdgcn_make_buffer_rsrc(p2.cnt, 0, 0x7FFFFFFF, 0x00020000);
                constexpr int64_t bpr = kRtRows / kPmRows;
                // lane 8d + s: sub-counter s of round d (rounds past the last
                // read the last one again)
                const int q = min((lane >> 3) & (kRtMaxRounds - 1), T - 1);
                const int off = (int)(((((p2.gen & 1) * 64 + q) * kMgSub + (lane & (kMgSub - 1))) * 32) * 4);
                for (int k = 0; spin.more(k); ++k) {
                    const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(crs, off, 0, 16);
                    bool all = true;
#pragma unroll
                    for (int d = 0; d < kRtMaxRounds; ++d) {
                        uint32_t n = 0;
#pragma unroll
                        for (int i = 0; i < kMgSub; ++i) n += __builtin_amdgcn_readlane(v, d * kMgSub + i);
                        const uint32_t want = d < T ? (uint32_t)(min<int64_t>(p2.pm.nblk, (d + 1) * bpr) - d * bpr) : 0u;
                        all = all && n >= want;
                    }
                    if (all) break;
                    __builtin_amdgcn_s_sleep(DLR_MG_SLEEP);
                }
            }
        }
    };
    // residuals: three register sets, always indexed by compile-time
    // constants (rounds are unrolled by unroll_seq; a runtime-indexed set
    // goes to scratch).  Native vectors: a float4 struct copied to LDS goes
    // through a stack temporary.
    struct Rnd {
        v4f r0, r1;  // rows 4*tid and 4*(tid + NT) of the round
    };
    Rnd rr[3];
    auto issue = [&](int t, Rnd &x) __attribute__((always_inline)) {
        const v4f *src = reinterpret_cast<const v4f *>(rsrc + (int64_t)t * kRtRows);
        x.r0 = src[threadIdx.x];
        x.r1 = src[NT + threadIdx.x];
    };
    // round t's entries: thread i takes group i of (s, t) if i < cap / 4
    const unsigned ngrp = (unsigned)rt.cap / 4;
    const bool mine = threadIdx.x < ngrp;
    const uint4 *gq4 = reinterpret_cast<const uint4 *>(rt.gq);
    const float4 *val4 = reinterpret_cast<const float4 *>(rt.val);
    uint4 eq[kRtMaxRounds];
    float4 ev[kRtMaxRounds];
    const bool no_entries = MG && wv == kPoller && (unsigned)(wv * kWave) >= ngrp;  // (wave-uniform)
    auto entries = [&](auto tc) __attribute__((always_inline)) {
        constexpr int t = decltype(tc)::value;
        if (t >= T) return;  // uniform
        if (no_entries) return;  // (never read: no thread of the wave is `mine`)
        const int64_t g = ((int64_t)s * T + t) * ngrp + (mine ? threadIdx.x : 0u);
        eq[t] = load_stream(gq4 + g);
        ev[t] = UNIT ? make_float4(1.f, 1.f, 1.f, 1.f) : load_stream(val4 + g);
    };
    // the memory pipeline is in order: what round 0 needs first, then the
    // rest of the first rounds; rounds 4+ are issued four rounds ahead
    // (MG: the entries first, then -- after every round's blocks are
    // published -- the residuals)
    if constexpr (MG) {
        entries(std::integral_constant<int, 0>{});
        entries(std::integral_constant<int, 1>{});
        entries(std::integral_constant<int, 2>{});
        entries(std::integral_constant<int, 3>{});
        mg_wait_all();
        lds_barrier();
        issue(0, rr[0]);
        if (T > 1) issue(1, rr[1]);
        if (T > 2) issue(2, rr[2]);
    } else {
        issue(0, rr[0]);
        entries(std::integral_constant<int, 0>{});
        if (T > 1) issue(1, rr[1]);
        entries(std::integral_constant<int, 1>{});
        if (T > 2) issue(2, rr[2]);
        entries(std::integral_constant<int, 2>{});
        entries(std::integral_constant<int, 3>{});
    }
    // this lane's columns (as k_grad_lds): weights and column-major runs
    float wj[NG];
    unsigned cb[NG], ce[NG];
    const uint16_t *cs = rt.cend + (int64_t)s * kPmSlice;
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        const int64_t j = (gfirst + kGradWaves * gi) * 64 + lane;
        wj[gi] = w[j < D ? j : D - 1];
        const int c = (wv + kGradWaves * gi) * 64 + lane;
        ce[gi] = cs[c];
        const unsigned p = cs[c ? c - 1 : 0];
        cb[gi] = c ? p : 0u;
    }
    PmPass1<NT, 4> pm;
    if (PM) pm.bounds(pn, s);
    DLR_STAMP(1);
    auto products = [&](const uint4 &q, const float4 &v, const float *br, uint32_t row0) __attribute__((always_inline)) {
        const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
        const float vv[4] = {v.x, v.y, v.z, v.w};
        float r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = br[(qq[u] >> 16) - row0];
#pragma unroll
        for (int u = 0; u < 4; ++u) s_prod[qq[u] & 0xFFFFu] = UNIT ? r[u] : r[u] * vv[u];
    };
    auto round = [&](auto tc) __attribute__((always_inline)) {
        constexpr int t = decltype(tc)::value;
        if (t >= T) return;  // uniform
        Rnd &x = rr[t % 3];
        float *br = s_r + (t & 1) * kRtRows;
        // buffer t & 1 was last read in round t - 2: every wave has passed
        // round t - 1's barrier since
        reinterpret_cast<v4f *>(br)[threadIdx.x] = x.r0;
        reinterpret_cast<v4f *>(br)[NT + threadIdx.x] = x.r1;
        lds_barrier();
        DLR_STAMP(2 + t);
        if (mine) products(eq[t], ev[t], br, (uint32_t)t * kRtRows);
        if (t + 3 < T) issue(t + 3, x);
        if constexpr (t + 4 < kRtMaxRounds) entries(std::integral_constant<int, t + 4>{});
        // the next batch's pass-1 list, one group set per round from round 4
        // (all at once stalls the issue of the round loads behind it)
        if constexpr (t >= 4) {
            if (PM) pm.fetch_one(pn, pm.c0, t - 4);
        }
    };
    unroll_seq(round, std::make_integer_sequence<int, kRtMaxRounds>{});
    if (PM) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (4 + u >= T) pm.fetch_one(pn, pm.c0, u);  // the sets the rounds did not issue
    }
    lds_barrier();  // every product is in s_prod
    DLR_STAMP(10);
    float acc[NG];
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        acc[gi] = 0.0f;
        if (gfirst + kGradWaves * gi >= ng) break;  // wave-uniform
        const unsigned o = cb[gi], c = ce[gi] - cb[gi];
        const float *sp = s_prod + o;
        float a = 0.0f;
        float x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = sp[u];  // o + 7 < kRtCap + kSink
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool take = (unsigned)u < c;
            if (__builtin_amdgcn_ballot_w64(take) == 0) break;  // wave-uniform
            const float tt = a + x[u];
            a = take ? tt : a;
        }
        for (unsigned k = 8; __builtin_amdgcn_ballot_w64(k < c) != 0; ++k) {
            const float xv = s_prod[min(o + k, (unsigned)(kRtCap + kSink - 1))];
            if (k < c) a = a + xv;
        }
        acc[gi] = a;
    }
    DLR_STAMP(11);
    if (PM) lds_barrier();  // every wave is done with s_prod: pass 1 reuses it
    auto update = [&](auto pow2) {
        constexpr bool P2 = decltype(pow2)::value;
        const float rBf = P2 ? 1.0f / Bf : 0.0f;
        const double rBd = P2 ? 1.0 / Bd : 0.0;
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            const int64_t j = (gfirst + kGradWaves * gi) * 64 + lane;
            if (gfirst + kGradWaves * gi >= ng || j >= D) continue;
            const float cw = C * wj[gi];
            const float l2 = P2 ? cw * rBf : cw / Bf;
            const float g = (float)((P2 ? (double)acc[gi] * rBd : (double)acc[gi] / Bd) + (double)l2);
            if (FUSED) {
                const float step = lr * g;
                const float wn = wj[gi] - step;
                w[j] = wn;
                if (PM) smem[(wv + kGradWaves * gi) * 64 + lane] = wn;
            } else {
                gout[j] = g;
            }
        }
    };
    const int64_t Bi = (int64_t)Bd;
    if ((Bi & (Bi - 1)) == 0)
        update(std::true_type{});
    else
        update(std::false_type{});
    if (PM) {
        pm.stage_offsets(reinterpret_cast<uint32_t *>(smem + kPmSlice));
        lds_barrier();
        DLR_STAMP(12);
        pm.store(pn, smem, reinterpret_cast<const uint32_t *>(smem + kPmSlice), pm_p);
    }
#ifdef DLR_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    DLR_STAMP(13);
#endif
}

// ---------------------------------------------------------------------------
// Touched-column layout (huge D, small batches: BASELINE C5, 2^28 features,
// B = 1,024).  The batch's column-major copy lists only the columns the
// batch touches (cols[s], ascending) -- a per-batch array over all D would
// not fit.  The reference still applies the L2 term to EVERY weight every
// step (lr.cc:40 runs j over all D; for an untouched column G_j = +0, so
// g_j = fl32(fl32(C*w_j)/(float)B) exactly), so the step is:
//   K3t  touched columns: ordered gradient (as k_grad), g or the new w
//   K4d  a streaming pass over all D applying the L2-only update
//   K4s  scatter of the touched columns' new weights (overwrites K4d's)
// K4d reads and writes 8 bytes per weight: it is the HBM-bound kernel here.

// K3t: segment s = column cols[s].  FUSED (one rank): out[s] = new w of the
// column (w - fl32(lr*g)); else out[s] = g (this rank's pushed gradient).
template <typename RowT, bool FUSED, bool UNIT = false>
__global__ __launch_bounds__(kWaves *kWave) void k_grad_touched(DevCsc cs, const RowT *__restrict__ crow,
                                                                const uint32_t *__restrict__ cols, int64_t ncols,
                                                                const float *__restrict__ resid,
                                                                const float *__restrict__ w, float *__restrict__ out,
                                                                float Bf, double Bd, float lr, float C) {
    __shared__ float s_p[kWaves][kWin];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t s0 = ((int64_t)blockIdx.x * kWaves + wv) * kWave;
    if (s0 >= ncols) return;  // wave-uniform
    const int64_t sg = s0 + lane;
    const bool valid = sg < ncols;
    const int64_t sl = min(s0 + kWave, ncols);
    const int64_t e0 = cs.ptr[s0], e1 = cs.ptr[sl];
    const int64_t a = valid ? (int64_t)cs.ptr[sg] : e1, b = valid ? (int64_t)cs.ptr[sg + 1] : e1;
    const float G = ordered_segment_dot<RowT, UNIT>(e0, e1, a, b, lane, crow, cs.val, resid, s_p[wv]);
    if (!valid) return;
    const float wj = w[cols[sg]];
    const float cw = C * wj;
    const float l2 = cw / Bf;
    const float g = (float)((double)G / Bd + (double)l2);
    if (FUSED) {
        const float step = lr * g;
        out[sg] = wj - step;
    } else {
        out[sg] = g;
    }
}

// ---------------------------------------------------------------------------
// Row-band layout (classic layout, large batches: BASELINE C3's full-shard
// batch of 12.5M rows).  A short column's residual gathers hit random rows
// of the whole batch -- a 50 MB residual array, far beyond an XCD's 4 MB L2,
// so every gather went to the Infinity Cache (~60 G gathers/s).  Here the
// batch's rows are cut into bands of 2^k rows (DevBand) and the short
// columns are summed band by band, one launch per band in band order: a
// launch gathers only from its band's slice of the residuals (L2-resident).
// Column j's entries in band s precede those in band s+1 in batch-row
// order, so continuing j's running sum (gacc[j], +0 before the first band)
// band after band IS lr.cc:37's sequential order: bitwise the classic
// kernel's result.  Each column appears at most once per band, so a launch
// has no write conflicts; the kernel boundary orders the bands.
template <typename RowT, bool UNIT = false, bool LONGRUN = false>
__global__ __launch_bounds__(kWaves *kWave) void k_grad_band(DevBand bd, const RowT *__restrict__ brow,
                                                             const float *__restrict__ resid,
                                                             float *__restrict__ gacc, bool skip_hot) {
    __shared__ float s_p[kWaves][kWin];
    constexpr int K = kBandPairsPerLane;
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t wid = (int64_t)blockIdx.x * kWaves + wv;
    if (wid >= bd.nwaves) return;  // wave-uniform
    // every access but the residual gathers is non-temporal: the pairs'
    // columns and pointers (37 MB per band at C3) and the running sums (a
    // 64 MB array) must not evict the band's residual slice from L2
    // (bit 31: a hot pair's own wave, k_band_hot's when skip_hot)
    const uint32_t w0 = __builtin_nontemporal_load(bd.wstart + wid);
    if (skip_hot && (w0 >> 31)) return;
    const int64_t s0 = w0 & 0x7FFFFFFFu, sl = __builtin_nontemporal_load(bd.wstart + wid + 1) & 0x7FFFFFFFu;
    const int64_t e0 = __builtin_nontemporal_load(bd.ptr + s0), e1 = __builtin_nontemporal_load(bd.ptr + sl);
    // lane l owns pairs s0 + l + 64k
    int64_t a[K], b[K];
    float acc[K];
    uint32_t j[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t sg = s0 + lane + (int64_t)k * kWave;
        const bool valid = sg < sl;
        j[k] = valid ? __builtin_nontemporal_load(bd.cols + sg) : 0u;
        a[k] = valid ? (int64_t)__builtin_nontemporal_load(bd.ptr + sg) : e1;
        b[k] = valid ? (int64_t)__builtin_nontemporal_load(bd.ptr + sg + 1) : e1;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = s0 + lane + (int64_t)k * kWave < sl ? __builtin_nontemporal_load(gacc + j[k]) : 0.0f;
    if constexpr (LONGRUN)
        ordered_segments_dot_piped<RowT, UNIT, K>(e0, e1, a, b, acc, lane, brow, bd.val, resid, s_p[wv]);
    else
        ordered_segments_dot<RowT, UNIT, K>(e0, e1, a, b, acc, lane, brow, bd.val, resid, s_p[wv]);
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (s0 + lane + (int64_t)k * kWave < sl) __builtin_nontemporal_store(acc[k], gacc + j[k]);
}

// Bounded polls (Spin): a hand-off whose producer never comes ends after
// kSpinTicks and is reported -- the host fails the step -- instead of
// hanging the GPU.
// LDS hand-off words between the waves of one half (no s_barrier: the two
// halves run at their own pace).  A producer's data writes (or, for LDS-DMA,
// its covering vmcnt wait) complete before the word is written; a consumer
// reads the data only after it has seen the word.
__device__ __forceinline__ uint32_t ctl_read(const uint32_t *p) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}
__device__ __forceinline__ void ctl_write(uint32_t *p, uint32_t v) {
    asm volatile("s_waitcnt lgkmcnt(0)\n ds_write_b32 %0, %1\n s_waitcnt lgkmcnt(0)" ::"v"(lds_addr(p)), "v"(v)
                 : "memory");
}
__device__ __forceinline__ void ctl_wait_ge(const uint32_t *p, uint32_t v, Spin &sp) {
    for (int k = 0; (int32_t)(ctl_read(p) - v) < 0 && sp.more(k); ++k) __builtin_amdgcn_s_sleep(0);
}
// The per-stage / per-slot hand-offs: a plain ds_write (a wave's LDS
// operations complete in order, so the data it stored before -- or the
// LDS-DMA its vmcnt wait covered -- lands first), and polls that return the
// value seen, so a consumer that is behind its producer (the usual case)
// skips the next polls: one LDS round trip per hand-off instead of three.
__device__ __forceinline__ void ctl_post(uint32_t *p, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t ctl_poll(const uint32_t *p, uint32_t v, Spin &sp) {
    uint32_t x = ctl_read(p);
    for (int k = 0; (int32_t)(x - v) < 0 && sp.more(k); ++k) {
        __builtin_amdgcn_s_sleep(0);
        x = ctl_read(p);
    }
    return x;
}
// min of the counters p[0], p[1] (N = 2) or p[0..2] (N = 3; p 16-byte aligned)
template <int N>
__device__ __forceinline__ uint32_t ctl_read_min(const uint32_t *p) {
    if constexpr (N == 2) {
        uint2 v;
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
        return min(v.x, v.y);
    } else {
        u32x4 v;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
        return min(min(v.x, v.y), v.z);
    }
}
template <int N>
__device__ __forceinline__ uint32_t ctl_poll_min(const uint32_t *p, uint32_t v, Spin &sp) {
    uint32_t x = ctl_read_min<N>(p);
    for (int k = 0; (int32_t)(x - v) < 0 && sp.more(k); ++k) {
        __builtin_amdgcn_s_sleep(0);
        x = ctl_read_min<N>(p);
    }
    return x;
}

// HOT columns of a band (REFERENCE order, band mode): a column whose chain
// over a full-shard batch is ~10^6 adds (C3's Zipf heads: ~130,000 entries
// per 2^20-row band) is the critical path of its band's launch -- one lane
// of k_grad_band adds it while the launch's other work is long done.  The
// layout builder gives each such (column, band) pair a wave of its own,
// marked in bit 31 of its wstart entry; k_grad_band skips those waves
// (skip_hot) and k_band_hot runs them beside it, one 256-thread workgroup
// per hot pair holding a CU by itself (dynamic LDS: nothing else fits
// beside it, the chain's SIMD is not shared):
//   wave 0    the chain: gacc[j] + the pair's products in entry order, 256
//             at a time from a 16-chunk LDS ring (16-byte broadcast reads,
//             the next 32 in flight while 32 are added, across chunks);
//   waves 1-2 the products: lane l of the 128 forms entries 256c + l and
//             256c + 128 + l of chunk c -- the rows loaded 16 chunks ahead,
//             the residual gathers (L2: the band's slice) eight ahead -- and
//             stores fl32(r * x) into the ring.
// The same products added in the same order from the same start: bitwise
// k_grad_band's sum.  Hand-offs through LDS counters (as K6r's); waits
// bounded.
constexpr int kHotChunk = 256;
constexpr int kHotRing = 16;
constexpr size_t kHotLds = 150 * 1024;  // requested: the workgroup holds its CU alone
template <typename RowT, bool UNIT>
__global__ __launch_bounds__(256) void k_band_hot(DevBand bd, const uint32_t *__restrict__ hw,
                                                  const RowT *__restrict__ brow, const float *__restrict__ resid,
                                                  float *__restrict__ gacc, uint32_t *err, int fault) {
    extern __shared__ __attribute__((aligned(16))) float hsm[];
    float *ring = hsm;                                                    // [kHotRing][kHotChunk]
    uint32_t *ctl = reinterpret_cast<uint32_t *>(hsm + kHotRing * kHotChunk);  // helper 1, helper 2, chain
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    Spin spin(err, kErrHotLds);
    if (threadIdx.x < 4) ctl[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t wid = hw[blockIdx.x];
    const int64_t s0 = bd.wstart[wid] & 0x7FFFFFFFu;
    const uint32_t j = bd.cols[s0];
    const int64_t e0 = bd.ptr[s0], e1 = bd.ptr[s0 + 1];
    const int64_t n = e1 - e0;
    const int64_t nch = (n + kHotChunk - 1) / kHotChunk;
    if (wv == 0) {
        float acc = __builtin_nontemporal_load(gacc + j);
        uint32_t pk = 0;  // chunks both helpers are known to have stored
        auto rd = [&](v4f(&d)[8], const float *q) {
#pragma unroll
            for (int u = 0; u < 8; ++u) d[u] = *reinterpret_cast<const v4f *>(q + 4 * u);
        };
        auto add = [&](const v4f(&d)[8]) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                acc = acc + d[u].x;
                acc = acc + d[u].y;
                acc = acc + d[u].z;
                acc = acc + d[u].w;
            }
        };
        // full chunks: the next 32 products' reads in flight while 32 are
        // added, across chunk boundaries once the helpers have stored the
        // next chunk; the last (partial) chunk one by one
        const int64_t nfull = n / kHotChunk;
        v4f da[8], db[8];
        if (nfull > 0) {
            pk = ctl_poll_min<2>(ctl, 1u, spin);
            rd(da, ring);
        }
        for (int64_t c = 0; c < nfull; ++c) {
            const float *q = ring + (c % kHotRing) * kHotChunk;
#pragma unroll 1
            for (int k = 0; k < kHotChunk - 64; k += 64) {
                rd(db, q + k + 32);
                add(da);
                rd(da, q + k + 64);
                add(db);
            }
            rd(db, q + kHotChunk - 32);
            add(da);
            const bool more = c + 1 < nfull;
            if (more && (int32_t)(pk - ((uint32_t)c + 2)) < 0) pk = ctl_poll_min<2>(ctl, (uint32_t)c + 2, spin);
            rd(da, more ? ring + ((c + 1) % kHotRing) * kHotChunk : q);  // (after the last: a re-read, unused)
            add(db);
            if (lane == 0) ctl_post(ctl + 2, (uint32_t)c + 1);
        }
        if (nfull < nch) {
            const int64_t c = nfull;
            if ((int32_t)(pk - ((uint32_t)c + 1)) < 0) pk = ctl_poll_min<2>(ctl, (uint32_t)c + 1, spin);
            const float *q = ring + (c % kHotRing) * kHotChunk;
            const int cnt = (int)(n - c * kHotChunk);
            for (int k = 0; k < cnt; ++k) acc = acc + q[k];
        }
        if (lane == 0) __builtin_nontemporal_store(acc, gacc + j);
        return;
    }
    if (wv > 2) return;
    // helpers: chunk c's entries 256c + hl, 256c + 128 + hl (hl: 0..127)
    const int hl = (wv - 1) * kWave + lane;
    uint32_t *mine = ctl + (wv - 1);
    uint32_t ck = 0;  // chunks the chain is known to have added
    auto ent = [&](int64_t c, int h) { return min<int64_t>(e0 + c * kHotChunk + 128 * h + hl, e1 - 1); };
    constexpr int RA = 16, GA = 8;  // rows RA chunks ahead, gathers GA (32 / 16 measured no better)
    uint32_t rw[RA][2];
    float vl[RA][2], g[GA][2];
    auto load_rows = [&](int64_t c, int d) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t e = ent(c < nch ? c : 0, h);
            rw[d][h] = (uint32_t)__builtin_nontemporal_load(brow + e);
            vl[d][h] = UNIT ? 1.0f : __builtin_nontemporal_load(bd.val + e);
        }
    };
#pragma unroll
    for (int d = 0; d < RA; ++d) load_rows(d, d);
#pragma unroll
    for (int d = 0; d < GA; ++d) {
        g[d][0] = resid[rw[d][0]];
        g[d][1] = resid[rw[d][1]];
    }
    for (int64_t c0 = 0; c0 < nch; c0 += RA) {
#pragma unroll
        for (int d = 0; d < RA; ++d) {
            const int64_t c = c0 + d;
            if (c < nch) {
                // chunk c's gathers landed GA chunks ago; issue chunk c + GA's
                // (its rows landed RA - GA chunks ago), then chunk c + RA's rows
                const float p0 = g[d % GA][0] * vl[d][0], p1 = g[d % GA][1] * vl[d][1];
                g[d % GA][0] = resid[rw[(d + GA) % RA][0]];
                g[d % GA][1] = resid[rw[(d + GA) % RA][1]];
                load_rows(c + RA, d);
                if (c >= kHotRing && (int32_t)(ck - (uint32_t)(c - kHotRing + 1)) < 0)
                    ck = ctl_poll(ctl + 2, (uint32_t)(c - kHotRing + 1), spin);
                float *q = ring + (c % kHotRing) * kHotChunk;
                q[hl] = p0;
                q[128 + hl] = p1;
                if (lane == 0 && fault != kFaultHotRing) ctl_post(mine, (uint32_t)c + 1);
            }
        }
    }
}

// Hot-column product stream (REFERENCE order, band mode; DevHotOut /
// DevHotChain).  k_band_hot forms a hot column's products from residuals
// it gathers band by band -- random L2 reads on the chain's critical path,
// slowest beside the next band's margin -- and is launched once per band, so
// its chain restarts at every band.  Here the margin kernel writes each hot
// product as it computes the row's residual (k_margin_hot, ho), into the
// column's stream in batch-row order, and after each band's margin a flag
// publishes the band (launch_flag_store).  ONE launch per step then runs
// every hot column's chain over all bands: wave 1 streams the column's
// products into a 32-chunk LDS ring by LDS-DMA (a band's chunks once its flag
// is up; sc1 loads, and no band segment shares a chunk -- or a cache line --
// with the next, so no line is read before its band is published), and wave
// 0 adds them in order from +0, 32 per LDS wait, the next 32 in flight.  The
// same products added in the same order: bitwise k_band_hot's (and the
// oracle's) sums; the chain never waits on a gather.
constexpr int kHcRing = 32;  // chunks of kHotChunkF floats in a ring
constexpr int kHcLA = 8;     // chunks a loader keeps in flight
// hot columns per workgroup: chain waves 0..kHcCols-1 (one per SIMD), their
// loaders waves kHcCols..2*kHcCols-1 (a loader's few instructions share its
// chain's SIMD); a ring each.  One workgroup per CU (kHotLds).
constexpr int kHcCols = 4;
static_assert(kHcCols * (kHcRing * kHotChunkF * 4 + 16) <= (int)kHotLds, "the rings fit the workgroup's LDS");
static_assert(kHotChunkF == kHotChunk, "one chunk size for both hot kernels");
__global__ __launch_bounds__(1) void k_flag_store(uint32_t *flag, uint32_t seq) {
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(2 * kHcCols * kWave) void k_hot_chain(DevHotChain hc, float *__restrict__ gacc) {
    extern __shared__ __attribute__((aligned(16))) float hsm[];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int pr = wv % kHcCols;  // this wave's (chain, loader) pair
    float *ring = hsm + pr * kHcRing * kHotChunkF;  // [kHcRing][kHotChunkF]
    // per pair: [0] chunks landed, [1] chunks added, [2] bands whose flag the
    // loader has seen (bit 31: it gave up at that band)
    uint32_t *ctl = reinterpret_cast<uint32_t *>(hsm + kHcCols * kHcRing * kHotChunkF) + 4 * pr;
    if (threadIdx.x < 4 * kHcCols) reinterpret_cast<uint32_t *>(hsm + kHcCols * kHcRing * kHotChunkF)[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t h = (int64_t)blockIdx.x * kHcCols + pr;
    if (h >= hc.nh) return;  // wave-uniform (no barrier after this point)
    const uint2 *seg = hc.seg + h * hc.nbands;
    // a launch after the first continues where the one before stopped
    // (state[h]: the first band not added, the chain's sum so far)
    int64_t s0 = 0;
    float acc0 = 0.0f;
    if (hc.b0 > 0) {
        const uint2 st = hc.state[h];
        s0 = st.x;
        acc0 = __uint_as_float(st.y);
    }
    if (s0 >= hc.b1) return;  // (wave-uniform; state stays as it is)
    const bool last = hc.final_launch != 0;
    Spin spin(hc.err, kErrHotLds);
    if (wv >= kHcCols) {
        // the loader: chunk g of the column's stream (bands in order) into
        // ring slot g % kHcRing; landed chunks are posted in order
        const __amdgpu_buffer_rsrc_t frs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(hc.flag), 0, 0x7FFFFFFF, 0x00020000);
        uint32_t g = 0, landed = 0, ck = 0;  // chunks issued, posted landed, known consumed
        for (int64_t s = s0; s < hc.b1; ++s) {
            const uint2 sg = seg[s];
            const uint32_t nch = (sg.y + kHotChunkF - 1) / kHotChunkF;
            if (nch > 0) {
                // the band's products are published -- or, after `giveup`
                // ticks without them, the rest is left to the next launch
                // (counted in stats).  The engine queues a launch after the
                // margins of its last band, so a flag is up by the time its
                // launch runs unless the margins run BEHIND it on the same
                // hardware queue -- which then cannot happen -- or kernels
                // run one at a time
                bool up = false;
                uint64_t t0 = 0;
                for (int k = 0;; ++k) {
                    const uint32_t f = __builtin_amdgcn_raw_buffer_load_b32(frs, (int)(s * 4), 0, 16);
                    if ((int32_t)(__builtin_amdgcn_readfirstlane(f) - hc.seq) >= 0) {
                        up = true;
                        break;
                    }
                    const uint64_t t = __builtin_amdgcn_s_memrealtime();
                    if (k == 0) t0 = t;
                    if (t - t0 > hc.giveup) break;
                    __builtin_amdgcn_s_sleep(8);
                }
                if (!up) {
                    // (the final launch runs after every margin: a flag
                    // it does not see is an error)
                    if (last && hc.err && lane == 0)
                        __hip_atomic_store(hc.err + kErrHotFlag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (!last && hc.stats && lane == 0)
                        __hip_atomic_fetch_add(hc.stats + kStatHotGiveUps, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                    if (lane == 0) ctl_post(ctl + 2, 0x80000000u | (uint32_t)(s - s0));
                    break;
                }
            }
            if (lane == 0) ctl_post(ctl + 2, (uint32_t)(s - s0 + 1));
            for (uint32_t c = 0; c < nch; ++c, ++g) {
                if (g >= (uint32_t)kHcRing && (int32_t)(ck - (g - kHcRing + 1)) < 0)
                    ck = ctl_poll(ctl + 1, g - kHcRing + 1, spin);  // the slot's last chunk was added
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(hc.buf + sg.x + (size_t)c * kHotChunkF + 4 * lane),
                    (__attribute__((address_space(3))) void *)(ring + (g % kHcRing) * kHotChunkF), 16, 0, 16);
                if (g + 1 - landed > (uint32_t)kHcLA) {
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // = kHcLA: chunk g - 8 has landed
                    landed = g + 1 - kHcLA;
                    if (lane == 0 && hc.fault != kFaultHotRing) ctl_post(ctl, landed);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the band's chunks (before the next flag poll)
            landed = g;
            if (lane == 0 && hc.fault != kFaultHotRing) ctl_post(ctl, landed);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives its wave
        return;
    }
    // the chain: the column's products in stream order, from +0 (or the
    // first launch's sum)
    float acc = acc0;
    uint32_t pk = 0, g = 0, bk = 0;  // chunks known landed, chunks added, loader's band word
    auto rd = [&](v4f(&d)[8], const float *q) {
#pragma unroll
        for (int u = 0; u < 8; ++u) d[u] = *reinterpret_cast<const v4f *>(q + 4 * u);
    };
    auto add = [&](const v4f(&d)[8]) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            acc = acc + d[u].x;
            acc = acc + d[u].y;
            acc = acc + d[u].z;
            acc = acc + d[u].w;
        }
    };
    v4f da[8], db[8];
    int64_t s = s0;
    for (; s < hc.b1; ++s) {
        // the loader is past band s's flag, or gave up before it
        const uint32_t want = (uint32_t)(s - s0 + 1);
        if ((bk & 0x7FFFFFFFu) < want && !(bk & 0x80000000u)) {
            bk = ctl_read(ctl + 2);
            for (int k = 0; (bk & 0x7FFFFFFFu) < want && !(bk & 0x80000000u) && spin.more(k); ++k) {
                __builtin_amdgcn_s_sleep(1);
                bk = ctl_read(ctl + 2);
            }
        }
        if ((bk & 0x7FFFFFFFu) < want) break;  // gave up here: the next launch adds the rest
        const uint2 sg = seg[s];
        const uint32_t nfull = sg.y / kHotChunkF, rem = sg.y % kHotChunkF;
        if (nfull > 0) {
            if ((int32_t)(pk - (g + 1)) < 0) pk = ctl_poll(ctl, g + 1, spin);
            rd(da, ring + (g % kHcRing) * kHotChunkF);
        }
        for (uint32_t c = 0; c < nfull; ++c, ++g) {
            const float *q = ring + (g % kHcRing) * kHotChunkF;
#pragma unroll 1
            for (int k = 0; k < kHotChunkF - 64; k += 64) {
                rd(db, q + k + 32);
                add(da);
                rd(da, q + k + 64);
                add(db);
            }
            rd(db, q + kHotChunkF - 32);
            add(da);
            const bool more = c + 1 < nfull;
            if (more && (int32_t)(pk - (g + 2)) < 0) pk = ctl_poll(ctl, g + 2, spin);
            rd(da, more ? ring + ((g + 1) % kHcRing) * kHotChunkF : q);  // (after the last: a re-read, unused)
            add(db);
            if (lane == 0) ctl_post(ctl + 1, g + 1);
        }
        if (rem > 0) {
            if ((int32_t)(pk - (g + 1)) < 0) pk = ctl_poll(ctl, g + 1, spin);
            const float *q = ring + (g % kHcRing) * kHotChunkF;
            for (uint32_t k = 0; k < rem; ++k) acc = acc + q[k];
            if (lane == 0) ctl_post(ctl + 1, g + 1);
            ++g;
        }
    }
    if (lane == 0) {
        if (s >= hc.nbands) gacc[hc.cols[h]] = acc;
        hc.state[h] = make_uint2((uint32_t)s, __float_as_uint(acc));
    }
}

// Long columns in ROW PHASES (band mode).  The chunked long path gathers
// each chunk's residuals from wherever its rows lie: a sparse long column's
// 256-entry chunk spans up to ~1M rows, so its gathers miss L2.  Here the
// batch's rows are cut into phases of kLPhase rows; one 1,024-thread
// workgroup per phase stages the phase's residuals in LDS (64 KB), then its
// waves sum the phase's pieces (<= 64 entries of one column each; lane per
// piece, products parked in LDS, in batch-row order: ordered_segment_dot
// with the LDS residuals as the table) into part[slot].  k_long_combine then
// adds a column's piece partials with its fixed tree.  Deterministic; for
// these columns not the single sequential sum (DLR_LONG_COLUMN=0 keeps
// every column sequential and bitwise).  Pieces keep every lane's serial
// chain <= 64 adds: a hot column's ~2,000 entries per phase would
// otherwise be one lane's chain while its wave's other lanes idle.
// A wave's tasks are software-pipelined three deep: while it sums task i
// (LDS work), the entry window of task i+1, the piece pointers of task i+2
// and the task bounds of task i+3 are already in flight -- each a
// dependent load of the one before, which the unpipelined loop waited for
// in turn (three round trips per ~1,000-entry task).  Loads are
// unconditional (clamped to the wave's last task), so the compiler's
// in-order vmcnt accounting waits for exactly the stage it needs.  Same
// sums in the same order as before.
template <bool UNIT>
struct LPWindow {
    ushort4 iv[kWin / (kVec * kWave)];
    float4 v[kWin / (kVec * kWave)];
};
// The window's loads are unclamped (the phase rows carry kLPWinPad entries
// of padding) and its entries outside [e0, e1) are gathered and multiplied
// like the others: their products land in slab slots no piece of this task
// reads, and every row index is phase-local (< kLPhase), so the gathers stay
// inside the staged residuals.
template <bool UNIT>
__device__ __forceinline__ void lp_load_window(LPWindow<UNIT> &w, uint32_t base, int lane,
                                               const uint16_t *__restrict__ row, const float *__restrict__ val) {
    constexpr int kT = kWin / (kVec * kWave);
#pragma unroll
    for (int t = 0; t < kT; ++t) {
        const uint32_t e = base + t * (kVec * kWave) + lane * kVec;
        w.iv[t] = load_stream(reinterpret_cast<const ushort4 *>(row + e));
        if constexpr (UNIT)
            w.v[t] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        else
            w.v[t] = load_stream(reinterpret_cast<const float4 *>(val + e));
    }
}
// gathers (from the phase's LDS residuals), products, ordered piece sums of
// the window [ws, ws + kWin)
template <bool UNIT, int K>
__device__ __forceinline__ void lp_window_sums(const LPWindow<UNIT> &w, uint32_t ws, const uint32_t (&a)[K],
                                               const uint32_t (&b)[K], float (&acc)[K], int lane, const float *s_r,
                                               float *lds) {
    constexpr int kT = kWin / (kVec * kWave);
    constexpr int kChunk = kVec * kWave;
    float g[kT][kVec];
#pragma unroll
    for (int t = 0; t < kT; ++t) {
        g[t][0] = s_r[w.iv[t].x];
        g[t][1] = s_r[w.iv[t].y];
        g[t][2] = s_r[w.iv[t].z];
        g[t][3] = s_r[w.iv[t].w];
    }
#pragma unroll
    for (int t = 0; t < kT; ++t) {
        const int o = t * kChunk + lane * kVec;
        float4 p;
        if constexpr (UNIT) {  // fl32(r * 1.0f) == r
            p = make_float4(g[t][0], g[t][1], g[t][2], g[t][3]);
        } else {
            p.x = g[t][0] * w.v[t].x;
            p.y = g[t][1] * w.v[t].y;
            p.z = g[t][2] * w.v[t].z;
            p.w = g[t][3] * w.v[t].w;
        }
        *reinterpret_cast<float4 *>(lds + o) = p;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t lo = a[k] > ws ? a[k] : ws;
        const uint32_t hi = b[k] < ws + kWin ? b[k] : ws + kWin;
        int o = (int)(lo - ws);
        const int oe = hi > lo ? (int)(hi - ws) : o;
        float sum = acc[k];
        // a piece is <= 63 entries: 16 LDS reads in flight per wait, then 4,
        // then 1 (the chain's adds stay in order)
        for (; o + 16 <= oe; o += 16) {
            float x[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) x[u] = lds[o + u];
#pragma unroll
            for (int u = 0; u < 16; ++u) sum = sum + x[u];
        }
        for (; o + 4 <= oe; o += 4) {
            const float x0 = lds[o], x1 = lds[o + 1], x2 = lds[o + 2], x3 = lds[o + 3];
            sum = sum + x0;
            sum = sum + x1;
            sum = sum + x2;
            sum = sum + x3;
        }
        for (; o < oe; ++o) sum = sum + lds[o];
        acc[k] = sum;
    }
    wave_sync();
}

template <bool UNIT>
__global__ __launch_bounds__(kLPWaves *kWave) void k_long_phase(DevLPhase lp, const float *__restrict__ resid,
                                                                float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *s_r = smem;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    float *slab = smem + kLPhase + wv * kWin;
    const int64_t p = blockIdx.x;
    {
        const float4 *src = reinterpret_cast<const float4 *>(resid + p * kLPhase);
        float4 *dst = reinterpret_cast<float4 *>(s_r);
#pragma unroll
        for (int k = 0; k < kLPhase / 4 / (kLPWaves * kWave); ++k)
            dst[k * kLPWaves * kWave + threadIdx.x] = src[k * kLPWaves * kWave + threadIdx.x];
    }
    __syncthreads();
    const PhaseDesc d = lp.desc[p];
    const uint2 *ps = lp.ps + d.ptr;
    const uint32_t *ws = lp.ws + d.ws;
    const uint16_t *row = lp.row + d.ent;
    const float *val = UNIT ? nullptr : lp.val + d.ent;
    constexpr int K = kBandPairsPerLane;  // pieces per lane: s0 + lane + 64k
    const int nt = (int)d.ntasks;
    const int mine = nt > wv ? (nt - wv + kLPWaves - 1) / kLPWaves : 0;  // this wave's tasks
    if (mine == 0) return;                                                // wave-uniform
    const int last = wv + (mine - 1) * kLPWaves;
    auto task_of = [&](int i) { return i < mine ? wv + i * kLPWaves : last; };
    // stage 0: task bounds (every lane loads both; uniform values)
    auto load_bounds = [&](int i, uint32_t &w0, uint32_t &w1) {
        const int t = task_of(i);
        w0 = ws[t];
        w1 = ws[t + 1];
    };
    // stage 1: piece pointers and slots; e1 = ptr[sl]
    auto load_meta = [&](uint32_t s0, uint32_t sl, uint32_t (&a)[K], uint32_t (&b)[K], uint32_t (&slot)[K],
                         uint32_t &e1) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t q = s0 + lane + k * kWave;
            const uint32_t qc = q < sl ? q : sl;
            const uint2 pa = ps[qc];  // used unconditionally: the load is not sunk under the select
            a[k] = pa.x;
            b[k] = ps[q < sl ? q + 1 : sl].x;
            slot[k] = q < sl ? pa.y : lp.npart + lane;  // idle lanes store to the sink
        }
        e1 = ps[sl].x;
    };
    uint32_t w0, w1;  // bounds of task i + 2 (in flight)
    uint32_t s0c, slc, a[K], b[K], slot[K], e1v;            // task i
    uint32_t s0n, sln, an[K], bn[K], slotn[K], e1n;         // task i + 1 (in flight)
    LPWindow<UNIT> win;
    // prologue
    load_bounds(0, w0, w1);
    s0c = __builtin_amdgcn_readfirstlane(w0);
    slc = __builtin_amdgcn_readfirstlane(w1);
    load_meta(s0c, slc, a, b, slot, e1v);
    load_bounds(1, w0, w1);
    uint32_t e0c = __builtin_amdgcn_readfirstlane(a[0]), e1c = __builtin_amdgcn_readfirstlane(e1v);
    lp_load_window<UNIT>(win, e0c & ~uint32_t(kVec - 1), lane, row, val);
    s0n = __builtin_amdgcn_readfirstlane(w0);
    sln = __builtin_amdgcn_readfirstlane(w1);
    load_meta(s0n, sln, an, bn, slotn, e1n);
    load_bounds(2, w0, w1);
    for (int i = 0; i < mine; ++i) {
        // 1. task i + 1's bounds of entries -> its window
        const uint32_t e0x = __builtin_amdgcn_readfirstlane(an[0]), e1x = __builtin_amdgcn_readfirstlane(e1n);
        LPWindow<UNIT> wnext;
        lp_load_window<UNIT>(wnext, e0x & ~uint32_t(kVec - 1), lane, row, val);
        // 2. task i + 2's bounds -> its pointers; task i + 3's bounds
        const uint32_t s0x = __builtin_amdgcn_readfirstlane(w0), slx = __builtin_amdgcn_readfirstlane(w1);
        uint32_t ax[K], bx[K], slotx[K], e1y;
        load_meta(s0x, slx, ax, bx, slotx, e1y);
        load_bounds(i + 3, w0, w1);
        // 3. task i
        float acc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = 0.0f;
        const uint32_t base = e0c & ~uint32_t(kVec - 1);
        lp_window_sums<UNIT, K>(win, base, a, b, acc, lane, s_r, slab);
        for (uint32_t wst = base + kWin; wst < e1c; wst += kWin) {  // rare: a task past one window
            LPWindow<UNIT> wx;
            lp_load_window<UNIT>(wx, wst, lane, row, val);
            lp_window_sums<UNIT, K>(wx, wst, a, b, acc, lane, s_r, slab);
        }
        // unconditional stores (idle lanes into the sink): a fixed count of
        // stores keeps the next waits exact (vmcnt counts stores on gfx9)
#pragma unroll
        for (int k = 0; k < K; ++k) part[slot[k]] = acc[k];
        // rotate
        s0c = s0n;
        slc = sln;
        e0c = e0x;
        e1c = e1x;
        win = wnext;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            a[k] = an[k];
            b[k] = bn[k];
            slot[k] = slotn[k];
            an[k] = ax[k];
            bn[k] = bx[k];
            slotn[k] = slotx[k];
        }
        s0n = s0x;
        sln = slx;
        e1n = e1y;
    }
}

// After the bands (and the long columns' combine, RAW into gacc): lr.cc:40
// and the update (FUSED) or the pushed gradient, for every column -- an
// untouched column has G = +0 there, as in k_grad.
// Four columns per thread (16-byte loads and stores; gacc, read once, with
// non-temporal loads); a scalar tail when D % 4 != 0.  Per column the same
// arithmetic as k_grad's epilogue.
__device__ __forceinline__ float finalize_one(float G, float wj, float Bf, double Bd, float C) {
    const float cw = C * wj;
    const float l2 = cw / Bf;
    return (float)((double)G / Bd + (double)l2);
}

template <bool FUSED>
__global__ __launch_bounds__(256) void k_band_finalize(const float *__restrict__ gacc, float *__restrict__ w,
                                                       float *__restrict__ gout, int64_t D, float Bf, double Bd,
                                                       float lr, float C) {
    const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (j >= D) return;
    if (j + 4 <= D) {
        const float4 G = load_stream(reinterpret_cast<const float4 *>(gacc + j));
        const float4 wj = *reinterpret_cast<const float4 *>(w + j);
        float4 g;
        g.x = finalize_one(G.x, wj.x, Bf, Bd, C);
        g.y = finalize_one(G.y, wj.y, Bf, Bd, C);
        g.z = finalize_one(G.z, wj.z, Bf, Bd, C);
        g.w = finalize_one(G.w, wj.w, Bf, Bd, C);
        if (FUSED) {
            float4 nw;
            nw.x = wj.x - lr * g.x;
            nw.y = wj.y - lr * g.y;
            nw.z = wj.z - lr * g.z;
            nw.w = wj.w - lr * g.w;
            *reinterpret_cast<float4 *>(w + j) = nw;
        } else {
            *reinterpret_cast<float4 *>(gout + j) = g;
        }
        return;
    }
    for (int64_t k = j; k < D; ++k) {
        const float wj = w[k];
        const float g = finalize_one(gacc[k], wj, Bf, Bd, C);
        if (FUSED) {
            const float step = lr * g;
            w[k] = wj - step;
        } else {
            gout[k] = g;
        }
    }
}

// (server_apply, l2_only_update: dlr_exchange.h, shared with the host)

// K4d: every weight gets the L2-only update of the W ranks; touched columns
// are overwritten afterwards by K4s.  16-byte non-temporal loads and stores
// (every byte is touched once), one float4 per thread: a one-shot grid
// streams at 6.0 TB/s where a 2048-block grid-stride loop reached 4.9
// (profiles/r01_kbench_l2.txt).
__global__ __launch_bounds__(256) void k_dense_l2(float *__restrict__ w, int64_t D, RankSizes rs, float lr,
                                                  float C, int mode) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int64_t n4 = D / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
        f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(w) + q);
        v.x = l2_only_update(v.x, rs, lr, C, mode);
        v.y = l2_only_update(v.y, rs, lr, C, mode);
        v.z = l2_only_update(v.z, rs, lr, C, mode);
        v.w = l2_only_update(v.w, rs, lr, C, mode);
        __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(w) + q);
    }
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < (D & 3)) w[n4 * 4 + t] = l2_only_update(w[n4 * 4 + t], rs, lr, C, mode);
}

// The pushed vector of an untouched column: g_j = fl32(fl32(C*w_j)/(float)B)
// (lr.cc:40 with G_j = +0), for the parameter-server topology's full push.
__global__ __launch_bounds__(256) void k_l2_fill(float *__restrict__ g, const float *__restrict__ w, int64_t D,
                                                 float Bf, float C) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= D) return;
    const float cw = C * w[j];
    g[j] = cw / Bf;
}

// K4s: w[cols[s]] = newv[s] for s < n (cols[s] == UINT32_MAX: skip).
__global__ __launch_bounds__(256) void k_scatter(float *__restrict__ w, const uint32_t *__restrict__ cols,
                                                 const float *__restrict__ newv, int64_t n) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint32_t c = cols[s];
    if (c != 0xFFFFFFFFu) w[c] = newv[s];
}

// Sparse exchange merge (world > 1, touched layout).  The all-gathered
// lists: rank r's block of `stride` words = [count | cols[cap] | g[cap]].
// Entry (r, s) owns its column iff no lower rank touched it; the owner
// computes the column's new weight from all W pushes (a rank that did not
// touch it pushed the L2 term) in rank order, and writes (col, newv) for
// K4s; non-owners write col = UINT32_MAX.
__global__ __launch_bounds__(256) void k_sparse_merge(const uint32_t *__restrict__ lists, int64_t cap, int64_t stride,
                                                      const float *__restrict__ w, RankSizes rs, float lr, float C,
                                                      int mode, uint32_t *__restrict__ out_cols,
                                                      float *__restrict__ out_newv) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)rs.W * cap) return;
    const int r = (int)(idx / cap);
    uint32_t c;
    float v;
    if (sparse_merge_entry(lists, cap, stride, w, rs, lr, C, mode, r, idx - (int64_t)r * cap, &c, &v)) {
        out_cols[idx] = c;
        out_newv[idx] = v;
    } else {
        out_cols[idx] = 0xFFFFFFFFu;
    }
}

// ---------------------------------------------------------------------------
// K6: dense rows (BASELINE C4, 4,096 features; and the reference's own dense
// representation).  GEMV-shaped and HBM-bound (0.5 flop/byte): no MFMA --
// its f32 MFMA would also reorder the sums.  Batch row i is shard row
// (first + i) mod N (NextBatch's wrap, data_iter.h:49-52).

// Shard row of batch row i: (first + i) mod N without a 64-bit division
// (first < N; a batch wraps ceil(B/N) times at most).
__device__ __forceinline__ int64_t wrap_row(int64_t r, int64_t N) {
    while (r >= N) r -= N;
    return r;
}

// K6a: lane per batch row; z = sum_j w_j*x_ij sequential fp32, j ascending
// (lr.cc:108-112), then sigma - y.  VEC4 (D % 4 == 0): 16-byte loads along
// the row, 8 in flight; w is wave-uniform (scalar loads).
template <bool VEC4>
__global__ __launch_bounds__(256) void k_dense_margin(DevDense dd, int64_t first, int64_t B,
                                                      const float *__restrict__ w, float *__restrict__ resid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const int64_t row = wrap_row(first + i, dd.N);
    const float *__restrict__ x = dd.X + row * dd.D;
    float acc = 0.0f;
    int64_t j = 0;
    if (VEC4) {
        constexpr int U = 8;
        for (; j + 4 * U <= dd.D; j += 4 * U) {
            float4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) xv[u] = *reinterpret_cast<const float4 *>(x + j + 4 * u);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float4 wv = *reinterpret_cast<const float4 *>(w + j + 4 * u);
                acc = acc + wv.x * xv[u].x;
                acc = acc + wv.y * xv[u].y;
                acc = acc + wv.z * xv[u].z;
                acc = acc + wv.w * xv[u].w;
            }
        }
    }
    for (; j < dd.D; ++j) acc = acc + w[j] * x[j];
    resid[i] = sigmoid_ref(acc) - dd.label[row];
}

// K6b, reference order: lane per column, G_j = sum over the batch rows in
// order of fl32(r_i*x_ij) (lr.cc:35-39); 8 rows' loads in flight.  Only
// D/64 waves: for parity-scale batches (DLR_DENSE_GRAD).
template <bool FUSED>
__global__ __launch_bounds__(256) void k_dense_grad_seq(DevDense dd, int64_t first, int64_t B,
                                                        const float *__restrict__ resid, float *__restrict__ w,
                                                        float *__restrict__ gout, float Bf, double Bd, float lr,
                                                        float C) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= dd.D) return;
    constexpr int U = 8;
    float acc = 0.0f;
    for (int64_t i = 0; i < B; i += U) {
        float xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t ii = i + u < B ? i + u : B - 1;
            xv[u] = dd.X[wrap_row(first + ii, dd.N) * dd.D + j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u < B) acc = acc + resid[i + u] * xv[u];
    }
    const float wj = w[j];
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

// K6b, reference order at C4's scale ("chain"; D % 4 == 0): lr.cc:35-39's
// per-column chain G_j = (((+0 + p_0j) + p_1j) + ...) over the batch rows in
// order, p_ij = fl32(r_i * x_ij) -- bitwise k_dense_grad_seq -- but with the
// chain as the ONLY work of its lane.  A column's 65,536 dependent adds are
// the floor (~4 cycles each), so everything else moves off the chain lane:
// workgroup = kChainCols columns (256 workgroups at D = 4,096: every CU),
//   waves 1-3  stream the batch rows' kChainCols-column segments (64 B) and
//              the residuals into an LDS ring by LDS-DMA, kChainAhead slots of
//              kChainRows rows in flight, and turn each landed slot into the
//              products, transposed: s_p[column][row];
//   wave 0     lane c runs column c's chain over the slot with one 16-byte
//              LDS read per 4 rows (stride kChainPad: conflict-free).
// One workgroup barrier per slot hands slot t's products to the chain while
// the helpers transform slot t + 1.  Rows past B get +0 products: G starts
// at +0 and a round-to-nearest sum is -0 only if both addends are, so G is
// never -0 and adding +0 leaves it unchanged.  Workgroups 2m, 2m+1 (the two
// halves of a 128-byte row line) run on one XCD (blockIdx % 8) when the grid
// is a multiple of 16, so the line is fetched into one L2 once.
constexpr int kChainCols = 16;
template <int R>
struct ChainCfg {
    static constexpr int kRing = R == 128 ? 8 : 6;        // staging slots
    static constexpr int kAhead = kRing - 1;               // slots in flight
    static constexpr int kPad = R + 4;                     // s_p column stride (floats): conflict-free 16-B reads
    static constexpr int kXI = R * kChainCols * 4 / 1024;  // 1 KiB LDS-DMA instructions per slot (x)
    // wave h (1..3) issues x blocks h-1, h+2, ... and wave 3 also the residuals
    static constexpr int count(int h) { return (kXI - (h - 1) + 2) / 3 + (h == 3 ? 1 : 0); }
    static constexpr size_t kLds = ((size_t)kRing * (R * kChainCols + 256) + 2 * kChainCols * kPad) * 4;
};

template <bool FUSED, int R>
__global__ __launch_bounds__(256) void k_dense_grad_chain(DevDense dd, int64_t first, int64_t B,
                                                          const float *__restrict__ resid, float *__restrict__ w,
                                                          float *__restrict__ gout, float Bf, double Bd, float lr,
                                                          float C) {
    using Cfg = ChainCfg<R>;
    constexpr int NS = Cfg::kRing, A = Cfg::kAhead, PAD = Cfg::kPad;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *s_x = smem;                                    // ring x [row][col]
    float *s_r = s_x + NS * R * kChainCols;               // ring r (256 per slot)
    float *s_p = s_r + NS * 256;                          // 2 x [col][PAD]
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    unsigned cg = blockIdx.x;
    if ((gridDim.x & 15) == 0) {
        const unsigned k = blockIdx.x >> 3;
        cg = ((k >> 1) << 4) | ((blockIdx.x & 7) << 1) | (k & 1);
    }
    const int64_t c0 = (int64_t)cg * kChainCols;
    const int64_t nslot = (B + R - 1) / R;
    const int64_t col = min(c0 + 4 * (lane & 3), dd.D - 4);
    // LDS-DMA of slot t (clamped past the last slot: the wait counts stay fixed)
    auto issue = [&](int64_t t) {
        const int64_t ts = t < nslot ? t : nslot - 1;
        const int ring = (int)(t % NS);
        if (wv >= 1) {
            const int64_t r0 = wrap_row(first + ts * R, dd.N);  // uniform; rows past it wrap at most once when N >= R
#pragma unroll
            for (int blk = wv - 1; blk < Cfg::kXI; blk += 3) {  // 16 rows per instruction
                const int64_t i = min(ts * R + blk * 16 + (lane >> 2), B - 1) - ts * R;
                int64_t row = r0 + i;
                if (dd.N >= R) {
                    if (row >= dd.N) row -= dd.N;
                } else {
                    row = wrap_row(row, dd.N);
                }
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(dd.X + row * dd.D + col),
                                                 (__attribute__((address_space(3))) void *)(s_x + (ring * R + blk * 16) * kChainCols),
                                                 16, 0, 0);
            }
        }
        if (wv == 3) {
            // resid is allocated to a multiple of 4 floats (+4): quads in bounds
            const int64_t q = min(ts * R + 4 * (lane & (R / 4 - 1)), (B - 1) & ~int64_t(3));
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(resid + q),
                                             (__attribute__((address_space(3))) void *)(s_r + ring * 256), 16, 0, 0);
        }
    };
    // helpers (waves 1, 2): the products of slot t into s_p[t & 1],
    // transposed; R groups of 4 rows x 4 columns, R / 128 per lane.  The
    // staged bytes are read with asm ds_read_b128 (and s_p written with asm):
    // a compiler-issued LDS access that may alias an in-flight LDS-DMA gets
    // an s_waitcnt vmcnt(0), which would drain the whole ring every slot (the
    // explicit waits below order these after their slot's DMA).
    auto transform = [&](int64_t t) {
        if (wv < 1 || wv > 2) return;
        const int ring = (int)(t % NS);
#pragma unroll
        for (int h = 0; h < R / 128; ++h) {
            const int g = h * 128 + (wv - 1) * kWave + lane;
            const int k = g >> 2, q = g & 3;
            const uint32_t xr = lds_addr(s_x + (ring * R + 4 * k) * kChainCols + 4 * q);
            const uint32_t ra = lds_addr(s_r + ring * 256 + 4 * k);
            v4f x4v[4], r4v;
            asm volatile("ds_read_b128 %0, %1" : "=v"(r4v) : "v"(ra));
            asm volatile("ds_read_b128 %0, %1" : "=v"(x4v[0]) : "v"(xr));
            asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(x4v[1]) : "v"(xr));
            asm volatile("ds_read_b128 %0, %1 offset:128" : "=v"(x4v[2]) : "v"(xr));
            asm volatile("ds_read_b128 %0, %1 offset:192" : "=v"(x4v[3]) : "v"(xr));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r4v), "+v"(x4v[0]), "+v"(x4v[1]), "+v"(x4v[2]), "+v"(x4v[3]));
            static_assert(kChainCols * 4 == 64, "row stride of the staged slot");
            const float rr[4] = {r4v.x, r4v.y, r4v.z, r4v.w};
            float p[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const bool ok = t * R + 4 * k + u < B;
                p[u][0] = ok ? rr[u] * x4v[u].x : 0.0f;
                p[u][1] = ok ? rr[u] * x4v[u].y : 0.0f;
                p[u][2] = ok ? rr[u] * x4v[u].z : 0.0f;
                p[u][3] = ok ? rr[u] * x4v[u].w : 0.0f;
            }
            const uint32_t pd = lds_addr(s_p + (int)(t & 1) * kChainCols * PAD + 4 * q * PAD + 4 * k);
            const v4f o0 = {p[0][0], p[1][0], p[2][0], p[3][0]}, o1 = {p[0][1], p[1][1], p[2][1], p[3][1]};
            const v4f o2 = {p[0][2], p[1][2], p[2][2], p[3][2]}, o3 = {p[0][3], p[1][3], p[2][3], p[3][3]};
            asm volatile("ds_write_b128 %0, %1" ::"v"(pd), "v"(o0) : "memory");
            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(pd), "v"(o1), "n"(PAD * 4) : "memory");
            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(pd), "v"(o2), "n"(PAD * 8) : "memory");
            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(pd), "v"(o3), "n"(PAD * 12) : "memory");
        }
    };
    float acc = 0.0f;
    // chain: the slot's rows as blocks of 8 16-byte reads (asm: the compiler
    // kept only one read in flight), block b+1 in flight while block b is added
    const uint32_t pc = lds_addr(s_p + (lane & (kChainCols - 1)) * PAD);
    auto rd8 = [&](v4f (&d)[8], uint32_t a) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(d[0]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(d[1]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(d[2]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:48" : "=v"(d[3]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(d[4]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:80" : "=v"(d[5]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:96" : "=v"(d[6]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:112" : "=v"(d[7]) : "v"(a));
    };
    auto add8 = [&](const v4f (&d)[8]) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            acc = acc + d[u].x;
            acc = acc + d[u].y;
            acc = acc + d[u].z;
            acc = acc + d[u].w;
        }
    };
#define DLR_CHAIN_WAIT(N, d)                                                                                   \
    asm volatile("s_waitcnt lgkmcnt(" #N ")"                                                                  \
                 : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]))
    auto chain = [&](int64_t t) {
        const uint32_t ps = pc + (uint32_t)((t & 1) * kChainCols * PAD * 4);
        v4f a[8], b[8];
        rd8(a, ps);
#pragma unroll
        for (int blk = 0; blk < R / 32; blk += 2) {
            rd8(b, ps + 128 * (blk + 1));
            DLR_CHAIN_WAIT(8, a);
            add8(a);
            if (blk + 2 < R / 32) {
                rd8(a, ps + 128 * (blk + 2));
                DLR_CHAIN_WAIT(8, b);
            } else {
                DLR_CHAIN_WAIT(0, b);
            }
            add8(b);
        }
    };
#undef DLR_CHAIN_WAIT
    for (int64_t t = 0; t < A; ++t) issue(t);
    for (int64_t t = 0; t <= nslot; ++t) {
        if (t < nslot) {  // uniform: slot t's own loads have landed (A - 1 later slots still in flight)
            if (wv == 1)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Cfg::count(1) * (A - 1)) : "memory");
            else if (wv == 2)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Cfg::count(2) * (A - 1)) : "memory");
            else if (wv == 3)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Cfg::count(3) * (A - 1)) : "memory");
        }
        // slot t staged for every helper; s_p[t & 1] no longer read by the chain
        lds_barrier();
        if (wv == 0) {
            if (t > 0) chain(t - 1);
        } else if (t < nslot) {
            transform(t);
            issue(t + A);  // into the ring slot transformed in the previous iteration
        }
    }
    if (wv != 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives its wave
        return;
    }
    const int64_t j = c0 + lane;
    if (lane >= kChainCols || j >= dd.D) return;
    const float wj = w[j];
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

// K6b, blocked: workgroup (k, c) sums batch rows [k*R, (k+1)*R) of columns
// [c*1024, (c+1)*1024) -- per column sequential in row order, 4 columns per
// lane (16-byte loads along the row: every row read once, coalesced) --
// into part[k][j]; k_dense_combine then adds the chunk partials in chunk
// order.  Deterministic; a different (blocked) order than lr.cc:37.
constexpr int kDenseChunk = 256;
template <bool VEC4>
__global__ __launch_bounds__(256) void k_dense_grad_blocked(DevDense dd, int64_t first, int64_t B,
                                                            const float *__restrict__ resid, int64_t Dp,
                                                            float *__restrict__ part) {
    const int64_t k = blockIdx.x;
    const int64_t i0 = k * kDenseChunk, i1 = min(i0 + kDenseChunk, B);
    constexpr int U = 8;
    if (VEC4) {
        const int64_t j = ((int64_t)blockIdx.y * blockDim.x + threadIdx.x) * 4;
        if (j >= dd.D) return;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int64_t i = i0; i < i1; i += U) {
            float4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t ii = i + u < i1 ? i + u : i1 - 1;
                xv[u] = *reinterpret_cast<const float4 *>(dd.X + wrap_row(first + ii, dd.N) * dd.D + j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (i + u < i1) {
                    const float r = resid[i + u];
                    acc.x = acc.x + r * xv[u].x;
                    acc.y = acc.y + r * xv[u].y;
                    acc.z = acc.z + r * xv[u].z;
                    acc.w = acc.w + r * xv[u].w;
                }
            }
        }
        *reinterpret_cast<float4 *>(part + k * Dp + j) = acc;
    } else {
        const int64_t j = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
        if (j >= dd.D) return;
        float acc = 0.0f;
        for (int64_t i = i0; i < i1; ++i) acc = acc + resid[i] * dd.X[wrap_row(first + i, dd.N) * dd.D + j];
        part[k * Dp + j] = acc;
    }
}

// K6 fused (DLR_DENSE_GRAD=fused): margin AND the blocked gradient partials
// in ONE pass over X.  The two-kernel path reads every batch row twice from
// HBM (the gradient needs a row's residual, which exists only after the
// whole row is summed); here workgroup k owns the same 256-row chunk as
// k_dense_grad_blocked and streams it through LDS four rows (one
// "sub-chunk") at a time, so each row is read from HBM once and used twice
// from LDS.  Two wave roles, one sub-chunk apart, so the margin and the
// gradient run side by side (one wave of each per SIMD):
//   margin   waves 0-3, sub-chunk t: wave i takes row i; lane l sums the
//            columns 256u + 4l .. +3, u = 0, 1, ..., in order (LDS reads
//            conflict-free), then the 64 lane partials combine by the
//            xor-butterfly tree: z is a fixed blocked order, not
//            lr.cc:108-112's single chain (the same tolerance regime as the
//            blocked gradient);
//   gradient waves 4-7, sub-chunk t - 1: column quad g sums r_i * x_i in
//            row order, continuing across the chunk's sub-chunks -- exactly
//            k_dense_grad_blocked's per-chunk order -- into part[k].
// Staging: every thread holds the next two sub-chunks in registers (16-byte
// loads, 128 KiB per CU in flight) and writes one into the LDS buffer the
// step has just freed (register staging: the compiler's waits are per
// register, where LDS-DMA pieces make it drain every load before each LDS
// read).  k_dense_combine then adds the chunk partials and applies the
// update.  Instantiated for D = 512, 1,024, 2,048 and 4,096 (BASELINE C4).
// (v4f: the staging registers, SROA-friendly)
constexpr int kFuseRows = 4;       // rows per sub-chunk: one margin wave each
constexpr int kFuseThreads = 512;  // 4 margin + 4 gradient waves


template <int DQ>  // D / 4
__global__ __launch_bounds__(kFuseThreads) void k_dense_fused(DevDense dd, int64_t first, int64_t B,
                                                              const float *__restrict__ w, int64_t Dp,
                                                              float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) float fsm[];
    constexpr int64_t D = 4 * DQ;
    constexpr int d4 = DQ;                                   // float4 per row
    constexpr int nreg = kFuseRows * d4 / kFuseThreads;      // float4 per thread per sub-chunk
    static_assert(nreg >= 1 && kFuseRows * d4 % kFuseThreads == 0, "D % 512 == 0");
    float *s_x = fsm;                                        // 2 buffers x kFuseRows x D
    float *s_w = fsm + (size_t)2 * kFuseRows * D;            // D
    float *s_zp = s_w + D;                                   // kFuseRows x 64 margin partials
    float *s_r = s_zp + kFuseRows * 64;                      // 2 x kFuseRows residuals
    float *s_lab = s_r + 2 * kFuseRows;                      // the chunk's labels (kDenseChunk)
    int64_t *s_roff = reinterpret_cast<int64_t *>(s_lab + kDenseChunk);  // row offsets (kDenseChunk + kFuseRows)
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wv = tid / kWave;
    const int gt = tid - 256;                                // gradient thread (waves 4-7)
    const int64_t k = blockIdx.x;
    const int64_t i0 = k * kDenseChunk, i1 = min(i0 + kDenseChunk, B);
    const int nsub = (int)((i1 - i0 + kFuseRows - 1) / kFuseRows);
    // sub-chunk q's float4 f = p * kFuseThreads + tid into registers RG
    // (past the last sub-chunk: the last one again, never used -- every step
    // issues the same loads, so the compiler's vmcnt waits stay exact)
#define DLR_FUSE_LOAD(q, RG)                                                                                   \
    {                                                                                                          \
        const int qc_ = min((q), nsub - 1);                                                                    \
        _Pragma("unroll") for (int p = 0; p < nreg; ++p)                                                       \
            RG[p] = __builtin_nontemporal_load(                                                                \
                reinterpret_cast<const v4f *>(dd.X + s_roff[qc_ * kFuseRows + fri[p]] + fc[p]));                \
    }
#define DLR_FUSE_STORE(q, RG)                                                                                  \
    {                                                                                                          \
        float *sbuf_ = s_x + (size_t)((q) & 1) * kFuseRows * D;                                                \
        _Pragma("unroll") for (int p = 0; p < nreg; ++p)                                                       \
            *reinterpret_cast<v4f *>(sbuf_ + (size_t)(p * kFuseThreads + tid) * 4) = RG[p];                    \
    }
    // gradient threads: column quads g = gt, gt + 256, ...
    constexpr int kMaxQ = (d4 + 255) / 256;
    const int nq = gt < 0 ? 0 : (d4 + 255 - gt) / 256;
    float4 acc[kMaxQ];
#pragma unroll
    for (int u = 0; u < kMaxQ; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    // one step: margin of sub-chunk t (t < nsub) and gradient of t - 1 (t >= 1)
    auto step = [&](int t) {
        if (wv < kFuseRows) {
            if (t < nsub) {
                const float *buf = s_x + (size_t)(t & 1) * kFuseRows * D;
                const int i = wv;
                const float *x = buf + (size_t)i * D + lane * 4;
                const float *ww = s_w + lane * 4;
                float z = 0.0f;
#pragma unroll 4
                for (int64_t u = 0; u < D; u += 256) {
                    const float4 xv = *reinterpret_cast<const float4 *>(x + u);
                    const float4 wq = *reinterpret_cast<const float4 *>(ww + u);
                    z = z + wq.x * xv.x;
                    z = z + wq.y * xv.y;
                    z = z + wq.z * xv.z;
                    z = z + wq.w * xv.w;
                }
                // the 64 lane partials by the xor-butterfly tree (every
                // lane ends with the same z): off the serial lane-0 chain
                // that every step's closing barrier waited for
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) z = z + __shfl_xor(z, off);
                const int64_t row = i0 + (int64_t)t * kFuseRows + i;
                if (lane == 0 && row < i1) s_r[(t & 1) * kFuseRows + i] = sigmoid_ref(z) - s_lab[t * kFuseRows + i];
            }
        } else if (t >= 1) {
            const int q = t - 1;
            const float *buf = s_x + (size_t)(q & 1) * kFuseRows * D;
            const int nr = (int)min<int64_t>(kFuseRows, i1 - (i0 + (int64_t)q * kFuseRows));
            for (int i = 0; i < nr; ++i) {
                const float r = s_r[(q & 1) * kFuseRows + i];
                const float *x = buf + (size_t)i * D;
#pragma unroll
                for (int u = 0; u < kMaxQ; ++u) {
                    if (u < nq) {
                        const float4 xv = *reinterpret_cast<const float4 *>(x + (size_t)(gt + 256 * u) * 4);
                        acc[u].x = acc[u].x + r * xv.x;
                        acc[u].y = acc[u].y + r * xv.y;
                        acc[u].z = acc[u].z + r * xv.z;
                        acc[u].w = acc[u].w + r * xv.w;
                    }
                }
            }
        }
    };
    for (int64_t j = tid * 4; j < D; j += 4 * kFuseThreads)
        *reinterpret_cast<float4 *>(s_w + j) = *reinterpret_cast<const float4 *>(w + j);
    if (tid < kDenseChunk && i0 + tid < i1) s_lab[tid] = dd.label[wrap_row(first + i0 + tid, dd.N)];
    // shard offset of each of the chunk's rows (NextBatch's wrap,
    // data_iter.h:49-52; rows past the chunk end repeat its last row), and
    // this thread's (row, column) of each staged float4
    for (int ii = tid; ii < kDenseChunk + kFuseRows; ii += kFuseThreads) {
        const int64_t r = min(i0 + ii, i1 - 1);
        s_roff[ii] = wrap_row(first + r, dd.N) * D;
    }
    int fri[nreg], fc[nreg];
#pragma unroll
    for (int p = 0; p < nreg; ++p) {
        const int f = p * kFuseThreads + tid;
        fri[p] = f / d4;
        fc[p] = (f - fri[p] * d4) * 4;
    }
    __syncthreads();
    v4f ra[nreg], rb[nreg];
    DLR_FUSE_LOAD(0, ra)
    DLR_FUSE_LOAD(1, rb)
    DLR_FUSE_STORE(0, ra)
    DLR_FUSE_LOAD(2, ra)
    __syncthreads();
    // step t reads buffers t & 1 (margin) and (t - 1) & 1 (gradient); then
    // sub-chunk t + 1 goes into buffer (t + 1) & 1 -- the gradient's, now
    // free -- and its register set is refilled with t + 3
    for (int t = 0; t <= nsub; t += 2) {
        step(t);
        lds_barrier();
        DLR_FUSE_STORE(t + 1, rb)
        DLR_FUSE_LOAD(t + 3, rb)
        lds_barrier();
        if (t + 1 <= nsub) {  // uniform
            step(t + 1);
            lds_barrier();
            DLR_FUSE_STORE(t + 2, ra)
            DLR_FUSE_LOAD(t + 4, ra)
            lds_barrier();
        }
    }
#undef DLR_FUSE_LOAD
#undef DLR_FUSE_STORE
#pragma unroll
    for (int u = 0; u < kMaxQ; ++u)
        if (u < nq) *reinterpret_cast<float4 *>(part + k * Dp + (int64_t)(gt + 256 * u) * 4) = acc[u];
}

// Chunk partials of 16 columns per workgroup: the 256 threads stage up to
// 256 chunks x 16 columns in LDS with one round of 16-byte loads (every
// workgroup's loads in flight at once: a single memory round trip per tile,
// where a lane-per-column loop waited ~4), then lane t < 16 adds its column's
// partials in chunk order from LDS.  Same order as before.
template <bool FUSED>
__global__ __launch_bounds__(256) void k_dense_combine(const float *__restrict__ part, int64_t nchunks, int64_t Dp,
                                                       int64_t D, float *__restrict__ w, float *__restrict__ gout,
                                                       float Bf, double Bd, float lr, float C) {
    constexpr int CT = 16, KT = 256;
    __shared__ __attribute__((aligned(16))) float s_t[KT][CT];
    const int t = threadIdx.x;
    const int64_t j0 = (int64_t)blockIdx.x * CT;
    const int64_t jq = j0 + 4 * (t % 4);  // this thread's column quad (Dp is a multiple of 4)
    float G = 0.0f;
    for (int64_t k0 = 0; k0 < nchunks; k0 += KT) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = k0 + t / 4 + 64 * u;
            v[u] = (k < nchunks && jq < Dp) ? *reinterpret_cast<const float4 *>(part + k * Dp + jq)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();  // the previous tile is consumed
#pragma unroll
        for (int u = 0; u < 4; ++u) *reinterpret_cast<float4 *>(&s_t[t / 4 + 64 * u][4 * (t % 4)]) = v[u];
        __syncthreads();
        if (t < CT) {
            const int kn = (int)min<int64_t>(KT, nchunks - k0);
            int k = 0;
            for (; k + 8 <= kn; k += 8) {
                float x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = s_t[k + u][t];
#pragma unroll
                for (int u = 0; u < 8; ++u) G = G + x[u];
            }
            for (; k < kn; ++k) G = G + s_t[k][t];
        }
    }
    const int64_t j = j0 + t;
    if (t >= CT || j >= D) return;
    const float wj = w[j];
    const float cw = C * wj;
    const float l2 = cw / Bf;
    const float g = (float)((double)G / Bd + (double)l2);
    if (FUSED) {
        const float step = lr * g;
        w[j] = wj - step;
    } else {
        gout[j] = g;
    }
}

// ---------------------------------------------------------------------------
// K6r: the dense step in the REFERENCE order as one launch (C4's default).
// lr.cc's arithmetic is two families of serial fp32 chains: every margin z_i
// is a chain over the columns in order (lr.cc:108-112), every gradient G_j a
// chain over the batch rows in order (lr.cc:35-39), and a row can enter the
// column chains only once its own chain is done.  A column chain of
// B = 65,536 dependent adds is the floor (8.3 cycles each on gfx950,
// profiles/r04_kbench_chain2.txt: ~0.23 ms), so the step keeps every column
// chain busy from its first row to its last.  One 512-thread workgroup per
// CU, two independent halves (no workgroup barrier after the start: each
// half hands off through LDS counters):
//
//   chain half (waves 0-3; workgroup b < D/16 owns columns [16b, 16b + 16)):
//     wave 0    lane c runs column c's chain over each slot's products (LDS,
//               16-byte reads, 256 rows per slot) -- its only work;
//     waves 1-2 load slot t's 256 rows x 16 columns into registers (six
//               slots in flight: the rows were read from HBM moments ago by
//               the margin halves and come back from the Infinity Cache),
//               form fl32(r_i * x_ij) and store them transposed;
//     wave 3    loads the residuals of slot t+3 once its margins are
//               published (sc1: written by other CUs); workgroup 0's also
//               publishes the margins' LIMIT, `lead` slots past its own
//               progress, so the rows the chains re-read are still in the
//               Infinity Cache;
//   margin half (waves 4-7): claims units of 64 batch rows in row order from
//     a queue (rows finish in order, and any resident subset of workgroups
//     drains it), waits for the limit before it starts a unit (holding only
//     later units: no chain waits on it), streams the unit's rows through a
//     7-stage LDS ring, 64 columns a stage, by LDS-DMA (waves 4-6, six stages
//     in flight) while lane i of wave 7 runs row i's chain in column order;
//     publishes sigma - y with sc1 stores and one agent-scope add to the
//     slot's counter (MI355X_MICROARCH.md, inter-workgroup hand-off, the sc1
//     row).
//
// X in HBM (a resident shard, dense_ref_tiled): tiles of 64 rows x 64
// columns, 16 KiB each, chunk-major inside (16-byte chunk k of the tile's
// rows 0..63, then chunk k + 1), the tiles of a 64-row block in column
// order -- a margin stage is ONE contiguous 16 KiB read whose LDS image the
// compute lanes read without bank conflicts (lane = row, 16 bytes apart),
// and a chain slot reads 1 KiB runs.  (Row-major X, a streamed batch: the
// same kernel with per-row addresses.)  The weights are written only by the
// chain epilogue, after its last slot: by then every unit -- every read of
// w -- is done.  Counters and the queue are monotonic over launches
// (sy.seq), so nothing is reset between steps.  Every wait is bounded
// (Spin): a launch whose producers never come drains and reports the wait
// that ran out (DevErr) instead of hanging the GPU, and the host fails the
// step.  The grid never exceeds what is resident at once (dense_ref_ok).
// X is read once from HBM (the margins) and once from the Infinity Cache
// (the chains).
constexpr int kRefCols = 16;      // columns per chain half
constexpr int kRefSlot = 256;     // batch rows per chain slot
constexpr int kRefUnit = 64;      // batch rows per margin unit (one lane each) = rows of a tile
constexpr int kRefStage = 64;     // columns per margin stage = columns of a tile
constexpr int kRefChunks = kRefStage / 4;  // 16-byte chunks of a tile row
constexpr int kRefRing = 7;       // margin stages in the LDS ring (6 in flight)
constexpr int kRefLA = kRefRing - 1;
constexpr int kRefPad = kRefSlot + 4;
constexpr int kRefHD = 6;         // chain slots whose rows a helper has in flight
constexpr int kRefThreads = 512;
constexpr uint32_t kRefNone = 0xFFFFFFFFu;
// LDS (floats): chain products [2][16][kRefPad], residuals [2][256], the
// margin ring [7][64 x 64 + 256 (the stage's 64 weights, in a 1 KiB area)],
// then 16 words of hand-off counters / unit ids
constexpr int kRefSlotF = kRefUnit * kRefStage + 256;
constexpr int kRefOffR = 2 * kRefCols * kRefPad;
constexpr int kRefOffRing = kRefOffR + 2 * kRefSlot;
constexpr int kRefOffCtl = kRefOffRing + kRefRing * kRefSlotF;
constexpr size_t kRefLds = (size_t)(kRefOffCtl + 16) * 4;
static_assert(kRefLds <= 160 * 1024, "one workgroup per CU");
// control words (uint32 at kRefOffCtl): chain half -- helper 1 / 2 slots
// done, chain slots done, residual slots staged; margin half -- loader 0..2
// stages landed, compute stages done, unit ids published, unit ids [4]
// (unit k's id in [k & 3], valid once ids > k)
enum { kCtlH0 = 0, kCtlH1, kCtlChain, kCtlR, kCtlL0, kCtlL1, kCtlL2, kCtlComp, kCtlIds, kCtlUnit };

// Shard row (first + i) mod N of batch row i: the launch needs B <= N
// (dense_ref_ok), so first + i < 2N and one subtraction wraps it
// (data_iter.h:49-52; no 64-bit division in the kernel).
__device__ __forceinline__ int64_t ref_row(int64_t first, int64_t i, int64_t N) {
    const int64_t r = first + i;
    return r >= N ? r - N : r;
}

// Float offset in X of 16-byte chunk k (columns 4k .. 4k + 3) of shard row
// `row`: tiled (above) or row-major.
template <bool TILED>
__device__ __forceinline__ int64_t ref_xoff(int64_t row, int64_t k, int64_t D) {
    if constexpr (TILED)
        return ((((row >> 6) * (D / kRefStage) + (k >> 4)) * kRefChunks + (k & 15)) * kRefUnit + (row & 63)) * 4;
    else
        return row * D + 4 * k;
}


// A margin stage in its ring slot: chunk k of rows 0..63 at k * 1 KiB + row *
// 16 (the tile's own image), the stage's 64 weights at 16 KiB.  ref_rd8<S>:
// set S (chunks 4S .. 4S + 3, 16 columns) of the lane's row (a = slot + 16 *
// lane) and their weights (wa = slot, uniform: every lane reads the same 16
// bytes, an LDS broadcast) -- eight reads, so that two sets in flight stay
// within lgkmcnt's 15.
template <int S>
__device__ __forceinline__ void ref_rd8(v4f (&d)[4], v4f (&wq)[4], uint32_t a, uint32_t wa) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d[0]) : "v"(a), "n"((4 * S + 0) * 1024));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d[1]) : "v"(a), "n"((4 * S + 1) * 1024));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d[2]) : "v"(a), "n"((4 * S + 2) * 1024));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d[3]) : "v"(a), "n"((4 * S + 3) * 1024));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(wq[0]) : "v"(wa), "n"(16384 + (4 * S + 0) * 16));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(wq[1]) : "v"(wa), "n"(16384 + (4 * S + 1) * 16));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(wq[2]) : "v"(wa), "n"(16384 + (4 * S + 2) * 16));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(wq[3]) : "v"(wa), "n"(16384 + (4 * S + 3) * 16));
}
#define DLR_REF_WAIT(N, d, e)                                                                                 \
    asm volatile("s_waitcnt lgkmcnt(" #N ")"                                                                 \
                 : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(e[0]), "+v"(e[1]), "+v"(e[2]), "+v"(e[3]))

// fl32(w_c * x_c) of a set's 16 columns
__device__ __forceinline__ void ref_products(float (&p)[16], const v4f (&x)[4], const v4f (&wq)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        p[4 * m + 0] = wq[m].x * x[m].x;
        p[4 * m + 1] = wq[m].y * x[m].y;
        p[4 * m + 2] = wq[m].z * x[m].z;
        p[4 * m + 3] = wq[m].w * x[m].w;
    }
}
// z += p0; n0 = w0 * x0; z += p1; ... : a set's adds in order (each waits
// for the last: the row chain), the next set's products issued in their
// shadow.  v_add_f32 / v_mul_f32 round as the C operators do (-ffp-contract
// =off: never fused).
#define DLR_REF_ADDMUL4(z, p, n, w4, x4)                                                               \
    asm volatile("v_add_f32 %0, %0, %5\n v_mul_f32 %1, %9, %13\n"                                     \
                 "v_add_f32 %0, %0, %6\n v_mul_f32 %2, %10, %14\n"                                    \
                 "v_add_f32 %0, %0, %7\n v_mul_f32 %3, %11, %15\n"                                    \
                 "v_add_f32 %0, %0, %8\n v_mul_f32 %4, %12, %16"                                       \
                 : "+v"(z), "=&v"(n[0]), "=&v"(n[1]), "=&v"(n[2]), "=&v"(n[3])                         \
                 : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(w4.x), "v"(w4.y), "v"(w4.z), "v"(w4.w), \
                   "v"(x4.x), "v"(x4.y), "v"(x4.z), "v"(x4.w))
// Set S of the stage's four (data of set s in buffer s % 3, products of set
// s in pp[s & 1]): wait for set S + 1's reads (set S + 2's still in flight),
// issue set S + 3's into set S's buffer (its products were formed in set
// S - 1), then add set S's products while forming set S + 1's.
template <int S>
__device__ __forceinline__ void ref_set(float &z, v4f (&xd)[3][4], v4f (&wd)[3][4], float (&pp)[2][16], uint32_t a,
                                        uint32_t wa) {
    constexpr int NS = kRefChunks / 4;
    constexpr int N1 = (S + 1) % 3, N3 = S % 3;
    if constexpr (S + 1 < NS) {
        if constexpr (S + 2 < NS)
            DLR_REF_WAIT(8, xd[N1], wd[N1]);
        else
            DLR_REF_WAIT(0, xd[N1], wd[N1]);
    }
    if constexpr (S + 3 < NS) ref_rd8<S + 3>(xd[N3], wd[N3], a, wa);
    float(&pc)[16] = pp[S & 1];
    if constexpr (S + 1 < NS) {
        float(&pn)[16] = pp[(S + 1) & 1];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            float *pcm = pc + 4 * m, *pnm = pn + 4 * m;
            DLR_REF_ADDMUL4(z, pcm, pnm, wd[N1][m], xd[N1][m]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) z = z + pc[k];
    }
}

// The queue position (claims so far) at the start of launch seq: every
// launch makes nunits successful claims and one failed claim per margin half.
__device__ __forceinline__ uint32_t ref_base(const DevRefSync &sy, int64_t nunits) {
    return sy.seq * (uint32_t)(nunits + sy.mgrid);
}

// The chain half of workgroup blockIdx.x (< D / 16).
template <bool FUSED, bool TILED>
__device__ __forceinline__ void ref_chain_half(const DevDense &dd, int64_t first, int64_t B, float *w,
                                               float *__restrict__ gout, float *resid, const DevRefSync &sy,
                                               float Bf, double Bd, float lr, float C, float *rsm, int wv,
                                               int lane) {
    const int64_t D = dd.D, N = dd.N;
    const int64_t nslot = (B + kRefSlot - 1) / kRefSlot;
    const int64_t nunits = (B + kRefUnit - 1) / kRefUnit;
    const int nstripes = (int)(D / kRefCols);
    float *s_p = rsm;            // [2][kRefCols][kRefPad]
    float *s_r = rsm + kRefOffR; // [2][kRefSlot]
    uint32_t *ctl = reinterpret_cast<uint32_t *>(rsm + kRefOffCtl);
    unsigned cg = blockIdx.x;
    if ((nstripes & 15) == 0 && (int)gridDim.x == nstripes) {  // stripes 2m, 2m+1 (one 128-byte line of a row) on one XCD
        const unsigned k = blockIdx.x >> 3;
        cg = ((k >> 1) << 4) | ((blockIdx.x & 7) << 1) | (k & 1);
    }
    const int64_t c0 = (int64_t)cg * kRefCols;
    Spin spin(sy.err, kErrRefLds);
    // helpers: lane hl in [0, 128); its load v (0..7) is chunk v >> 1 of
    // the stripe for slot row r = 128 (v & 1) + hl -- a wave reads 64
    // consecutive rows of one chunk (1 KiB of a tile)
    const int hl = (wv - 1) * kWave + lane;
    auto load = [&](int64_t t, v4f (&x)[8]) {
        const int64_t tc = t < nslot ? t : nslot - 1;  // past the end: the last slot again (never used)
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            const int64_t i = min<int64_t>(tc * kRefSlot + 128 * (v & 1) + hl, B - 1);
            x[v] = __builtin_nontemporal_load(
                reinterpret_cast<const v4f *>(dd.X + ref_xoff<TILED>(ref_row(first, i, N), c0 / 4 + (v >> 1), D)));
        }
    };
    auto transform = [&](int64_t t, const v4f (&x)[8]) {
        const float *sr = s_r + (t & 1) * kRefSlot;
        float *sp = s_p + (t & 1) * kRefCols * kRefPad;
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            const int r = 128 * (v & 1) + hl, cc = v >> 1;
            const bool ok = t * kRefSlot + r < B;  // rows past B: +0 (never -0 in a sum from +0)
            const float rr = sr[r];
            sp[(4 * cc + 0) * kRefPad + r] = ok ? rr * x[v].x : 0.0f;
            sp[(4 * cc + 1) * kRefPad + r] = ok ? rr * x[v].y : 0.0f;
            sp[(4 * cc + 2) * kRefPad + r] = ok ? rr * x[v].z : 0.0f;
            sp[(4 * cc + 3) * kRefPad + r] = ok ? rr * x[v].w : 0.0f;
        }
    };
    if (wv == 0) {
        // the chain: slot t once both helpers have stored it
        float acc = 0.0f;
        uint32_t hk = 0;  // slots both helpers are known to have stored
        DLR_TACC_DECL(t_cw);
        DLR_TACC_DECL(t_ca);
        DLR_STAMP64V(60, lane == 0, __builtin_amdgcn_s_memtime());  // shader clock: the clock under load
        DLR_STAMP64V(61, lane == 0, __builtin_amdgcn_s_memrealtime());
        // 256 products a slot, 32 at a time: the next 32's reads -- across
        // the slot boundary too, once the helpers have stored the next slot
        // -- in flight while these are added
        const int cl = lane & (kRefCols - 1);
        auto sp_of = [&](int64_t t) { return s_p + (t & 1) * kRefCols * kRefPad + cl * kRefPad; };
        auto rd = [&](v4f(&d)[8], const float *q) {
#pragma unroll
            for (int u = 0; u < 8; ++u) d[u] = *reinterpret_cast<const v4f *>(q + 4 * u);
        };
        auto add = [&](const v4f(&d)[8]) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                acc = acc + d[u].x;
                acc = acc + d[u].y;
                acc = acc + d[u].z;
                acc = acc + d[u].w;
            }
        };
        v4f da[8], db[8];
        {
            DLR_TACC_BEGIN();
            hk = ctl_poll_min<2>(ctl + kCtlH0, 1u, spin);
            DLR_TACC_LAP(t_cw);
        }
        rd(da, sp_of(0));
        for (int64_t t = 0; t < nslot; ++t) {
            DLR_TACC_BEGIN();
            const float *sp = sp_of(t);
#pragma unroll 1
            for (int k = 0; k < kRefSlot - 64; k += 64) {
                rd(db, sp + k + 32);
                add(da);
                rd(da, sp + k + 64);
                add(db);
            }
            rd(db, sp + kRefSlot - 32);
            add(da);
            const bool more = t + 1 < nslot;
            if (more && (int32_t)(hk - ((uint32_t)t + 2)) < 0) {
                DLR_TACC_LAP(t_ca);
                hk = ctl_poll_min<2>(ctl + kCtlH0, (uint32_t)t + 2, spin);
                DLR_TACC_LAP(t_cw);
            }
            rd(da, more ? sp_of(t + 1) : sp);  // (after the last slot: a re-read, unused)
            add(db);
            if (lane == 0) ctl_post(ctl + kCtlChain, (uint32_t)t + 1);
            DLR_TACC_LAP(t_ca);
            DLR_STAMP64(2 + (int)(t >> 4), lane == 0 && (t & 15) == 0 && t < 16 * 40);
        }
        DLR_STAMP64(50, lane == 0);
        DLR_STAMP64V(62, lane == 0, __builtin_amdgcn_s_memtime());
        DLR_STAMP64V(63, lane == 0, __builtin_amdgcn_s_memrealtime());
        DLR_STAMP64V(52, lane == 0, t_cw);
        DLR_STAMP64V(53, lane == 0, t_ca);
        const int64_t j = c0 + lane;
        if (lane >= kRefCols || j >= D) return;
        const float wj = w[j];
        const float cw = C * wj;
        const float l2 = cw / Bf;
        const float g = (float)((double)acc / Bd + (double)l2);
        if (FUSED) {
            const float stepv = lr * g;
            w[j] = wj - stepv;
        } else {
            gout[j] = g;
        }
        return;
    }
    if (wv <= 2) {
        // helpers: slot t needs its residuals staged and the products buffer
        // of slot t - 2 consumed by the chain
        // (kRefHD slots' loads in flight: the re-read rows come from the
        // Infinity Cache, microseconds away under the margins' stream)
        uint32_t *mine = ctl + (wv == 1 ? kCtlH0 : kCtlH1);
        uint32_t rk = 0, ck = 0;  // residual slots known staged, chain slots known done
        DLR_TACC_DECL(t_hr);
        DLR_TACC_DECL(t_hc);
        DLR_TACC_DECL(t_hx);
        v4f x[kRefHD][8];
#pragma unroll
        for (int d = 0; d < kRefHD; ++d) load(d, x[d]);
        for (int64_t t0 = 0; t0 < nslot; t0 += kRefHD) {
#pragma unroll
            for (int d = 0; d < kRefHD; ++d) {
                const int64_t t = t0 + d;
                if (t < nslot) {
                    DLR_TACC_BEGIN();
                    if ((int32_t)(rk - ((uint32_t)t + 1)) < 0) rk = ctl_poll(ctl + kCtlR, (uint32_t)t + 1, spin);
                    DLR_TACC_LAP(t_hr);
                    if (t >= 2 && (int32_t)(ck - ((uint32_t)t - 1)) < 0) ck = ctl_poll(ctl + kCtlChain, (uint32_t)t - 1, spin);
                    DLR_TACC_LAP(t_hc);
                    transform(t, x[d]);
                    if (lane == 0) ctl_post(mine, (uint32_t)t + 1);
                    load(t + kRefHD, x[d]);
                    DLR_TACC_LAP(t_hx);
                }
            }
        }
        DLR_STAMP64V(54, lane == 0 && wv == 1, t_hr);
        DLR_STAMP64V(55, lane == 0 && wv == 1, t_hc);
        DLR_STAMP64V(56, lane == 0 && wv == 1, t_hx);
        return;
    }
    // wave 3: the residuals.  Its view of the margins: every slot <= ready
    // is published.  Waiting for a slot polls its counter from ONE lane, a
    // microsecond apart (hundreds of CUs polling flat out take HBM bandwidth
    // from the margins they wait for); once it is published, one 64-lane
    // poll of the next 64 counters extends `ready`, so while the margins run
    // ahead a round trip is paid once per 64 slots.  Global loads and stores
    // go through the buffer path with sc1 (aux 16): L2-coherent, and tracked
    // by the compiler's waits.
    auto slot_target = [&](int64_t t) -> uint32_t {
        const int64_t rows = min<int64_t>(kRefSlot, B - t * kRefSlot);
        const uint32_t units = (uint32_t)((rows + kRefUnit - 1) / kRefUnit);
        return units * (sy.seq + 1);
    };
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(sy.slot_cnt, 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(resid, 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(sy.limit, 0, 0x7FFFFFFF, 0x00020000);
    const bool leader = blockIdx.x == 0 && sy.lead > 0;
    const uint32_t qbase = ref_base(sy, nunits);
    auto publish_limit = [&](int64_t t) {
        const int64_t lim = min<int64_t>(nunits, (t + sy.lead) * (kRefSlot / kRefUnit));
        if (lane == 0) __builtin_amdgcn_raw_buffer_store_b32(qbase + (uint32_t)lim, lrs, 0, 0, 16);
    };
    int64_t ready = -1;
    Spin gspin(sy.err, kErrRefSlot);
    DLR_TACC_DECL(t_rp);
    DLR_TACC_DECL(t_rh);
    auto poll_from = [&](int64_t t0) {
        const uint32_t want0 = slot_target(t0);
        for (int k = 0;; ++k) {
            const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(crs, (int)(t0 * 4), 0, 16);
            if (v >= want0 || !gspin.more(k)) break;
            __builtin_amdgcn_s_sleep(32);
        }
        const int64_t sl = min<int64_t>(t0 + lane, nslot - 1);
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(crs, (int)(sl * 4), 0, 16);
        const bool ok = t0 + lane >= nslot || v >= slot_target(sl);
        const unsigned long long bad = ~__ballot(ok) | 1ull << 63;  // (lane 63: not counted past it)
        const int first_bad = __ffsll((long long)bad) - 1;
        ready = t0 + max(first_bad, 1) - 1;  // t0 itself is published (or the bounded wait ran out)
    };
    auto r_issue = [&](int64_t t, v4f &rv) {
        const int64_t tc = t < nslot ? t : nslot - 1;  // past the end: a load of a published slot, unused
        if (tc > ready) {
            DLR_TACC_BEGIN();
            poll_from(tc);
            DLR_TACC_LAP(t_rp);
        }
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rrs, (int)((tc * kRefSlot + 4 * lane) * 4), 0, 16);
        __builtin_memcpy(&rv, &q, 16);
    };
    // slot t's residuals into s_r[t & 1] once both helpers are done with
    // slot t - 2 (the same buffer)
    uint32_t hk = 0;  // slots both helpers are known to have stored
    auto r_store = [&](int64_t t, const v4f &rv) {
        DLR_TACC_BEGIN();
        if (t >= 2 && (int32_t)(hk - ((uint32_t)t - 1)) < 0) hk = ctl_poll_min<2>(ctl + kCtlH0, (uint32_t)t - 1, spin);
        DLR_TACC_LAP(t_rh);
        *reinterpret_cast<v4f *>(s_r + (t & 1) * kRefSlot + 4 * lane) = rv;
        if (lane == 0) ctl_post(ctl + kCtlR, (uint32_t)t + 1);
    };
    v4f ra, rb, rc;
    if (leader) publish_limit(0);
    r_issue(0, ra);
    r_issue(1, rb);
    r_issue(2, rc);
    auto step = [&](int64_t t, v4f &rv) {  // slot t staged, slot t + 3 issued into its registers
        r_store(t, rv);
        r_issue(t + 3, rv);
        if (leader) publish_limit(t);
    };
    for (int64_t t = 0; t < nslot; t += 3) {
        step(t, ra);
        if (t + 1 < nslot) step(t + 1, rb);
        if (t + 2 < nslot) step(t + 2, rc);
    }
    DLR_STAMP64V(57, lane == 0, t_rp);
    DLR_STAMP64V(58, lane == 0, t_rh);
}

// The margin half (the workgroup's waves 4-7; mw = wave - 4).  wr: read-only
// here (the chains update w after every margin is published).
template <bool TILED>
__device__ __forceinline__ void ref_margin_half(const DevDense &dd, int64_t first, int64_t B,
                                                const float *__restrict__ wr, float *resid, const DevRefSync &sy,
                                                float *rsm, int mw, int lane) {
    const int64_t D = dd.D, N = dd.N;
    const int64_t nunits = (B + kRefUnit - 1) / kRefUnit;
    float *ring = rsm + kRefOffRing;  // [kRefRing][kRefSlotF]
    uint32_t *ctl = reinterpret_cast<uint32_t *>(rsm + kRefOffCtl);
    uint32_t *s_unit = ctl + kCtlUnit;  // [4]
    const int spu = (int)(D / kRefStage);  // stages per unit (>= 8)
    const uint32_t base = ref_base(sy, nunits);
    Spin spin(sy.err, kErrRefLds);
    if (mw < 3) {
        // loaders: stage g of this half's unit sequence into ring[g % 7]:
        // chunk q of the unit's 64 rows per LDS-DMA instruction (1 KiB; lane
        // l: row l), and loader 1 the stage's 64 weights too.  Stage g is
        // published (kCtlL0 + lw) once this loader's pieces of it have
        // landed; stage g + 6 goes into the slot stage g - 1 used, once the
        // compute is past it.
        const int lw = mw;                    // loader 0..2: chunks lw, lw + 3, ...
        const int npieces = lw == 2 ? 5 : 6;  // of the 16 + 1 (6 + 5 + 5, and loader 1 the weights)
        uint32_t compk = 0;  // stages the compute is known to be past
        int kc = -1;         // the unit whose id uc is
        uint32_t uc = kRefNone;
        auto issue = [&](int k, int sg, int ri, int g) {
            if (g >= kRefRing && (int32_t)(compk - (uint32_t)(g - kRefRing + 1)) < 0)
                compk = ctl_poll(ctl + kCtlComp, (uint32_t)(g - kRefRing + 1), spin);
            if (k != kc) {
                ctl_wait_ge(ctl + kCtlIds, (uint32_t)k + 1, spin);
                uc = ctl_read(s_unit + (k & 3));
                kc = k;
            }
            const uint32_t u = uc;
            const int64_t i = min((int64_t)(u == kRefNone ? 0 : u) * kRefUnit + lane, B - 1);
            const int64_t row = ref_row(first, i, N);
            float *dst = ring + (size_t)ri * kRefSlotF;
            for (int q = lw; q < kRefChunks; q += 3)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(dd.X +
                                                                     ref_xoff<TILED>(row, sg * kRefChunks + q, D)),
                    (__attribute__((address_space(3))) void *)(dst + q * 256), 16, 0, 0);
            if (lw == 1)  // the stage's weights (lanes 16..63 again into the rest of the 1 KiB area)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(wr + (int64_t)sg * kRefStage + 4 * (lane & 15)),
                    (__attribute__((address_space(3))) void *)(dst + kRefUnit * kRefStage), 16, 0, 0);
            return u;
        };
        // issue stages [0, 6) first; then per stage g: wait for g (the five
        // later stages still in flight), publish it, issue g + 6 (whose ring
        // slot frees when the compute is past g - 1: by then it is usually
        // adding g)
        int ka = 0, sa = 0, ria = 0;  // the next stage to issue
        auto issue_next = [&](int g) {
            const uint32_t u = issue(ka, sa, ria, g);
            if (++sa == spu) {
                sa = 0;
                ++ka;
            }
            if (++ria == kRefRing) ria = 0;
            return u;
        };
        for (int g = 0; g < kRefLA; ++g) issue_next(g);
        uint32_t *mine = ctl + kCtlL0 + lw;
        DLR_TACC_DECL(t_issue);
        DLR_TACC_DECL(t_land);
        for (int g = 0, k = 0, sg = 0;; ++g) {
            if (sg == 0) {  // a new unit: stop at the end of the sequence
                ctl_wait_ge(ctl + kCtlIds, (uint32_t)k + 1, spin);
                if (ctl_read(s_unit + (k & 3)) == kRefNone) break;
            }
            DLR_TACC_BEGIN();
            if (npieces == 6)
                asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(25)" ::: "memory");
            DLR_TACC_LAP(t_land);
            if (lane == 0) ctl_post(mine, (uint32_t)g + 1);
            issue_next(g + kRefLA);
            DLR_TACC_LAP(t_issue);
            if (++sg == spu) {
                sg = 0;
                ++k;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives its wave
        DLR_STAMP64MV(56 + 2 * lw, lane == 0 && lw < 2, t_issue);
        DLR_STAMP64MV(57 + 2 * lw, lane == 0 && lw < 2, t_land);
        return;
    }
    // compute wave (wave 7: its SIMD's other wave is the chain half's
    // mostly idle wave 3, not the column chain): lane i runs row i's chain;
    // the weights come with the stage (w is read-only until the chain
    // epilogue, after every margin)
    const __amdgpu_buffer_rsrc_t rres = __builtin_amdgcn_make_buffer_rsrc(resid, 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(sy.limit, 0, 0x7FFFFFFF, 0x00020000);
    // claims: unit ids in row order; after the first failed claim none more
    // (so every margin half fails exactly once and the head advances by
    // nunits + mgrid per launch).  The atomic's address is made
    // non-uniform-looking so the compiler's atomic optimizer (a wave scan
    // that waits for the result at once) leaves it alone: the result is
    // used only at the end of the unit.
    bool claiming = true;
    Spin lspin(sy.err, kErrRefLimit);
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    auto claim_issue = [&]() -> uint32_t {
        return __hip_atomic_fetch_add(sy.head + vz, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto claim_finish = [&](uint32_t raw) -> uint32_t {
        const uint32_t u = raw - base;
        if (u >= (uint32_t)nunits) {
            claiming = false;
            return kRefNone;
        }
        return u;
    };
    if (lane == 0) {
        const uint32_t u0 = claim_finish(claim_issue());
        const uint32_t u1 = claiming ? claim_finish(claim_issue()) : kRefNone;
        ctl_write(s_unit + 0, u0);
        ctl_write(s_unit + 1, u1);
        ctl_write(ctl + kCtlIds, 2u);
    }
    DLR_STAMP64M(1, lane == 0);
    DLR_TACC_DECL(t_wait);
    DLR_TACC_DECL(t_comp);
    float z = 0.0f, y = 0.0f;
    int64_t urow = -1;  // batch row of this lane in the current unit (-1: none)
    uint32_t pend = 0;  // lane 0: the raw claim issued at the start of the unit
    bool have_pend = false;
    uint32_t lk = 0;  // stages all three loaders are known to have landed
    uint32_t u = kRefNone;
    for (int g = 0, k = 0, sg = 0, ri = 0;; ++g) {
        if (sg == 0) {
            u = ctl_read(s_unit + (k & 3));
            if (u == kRefNone) break;
            // the margins' limit: start unit u only once the chains are
            // within `lead` slots of it (every unit this half still holds is
            // later: nothing a chain waits for is held here)
            if (sy.lead > 0 && lane == 0)
                for (int s = 0;; ++s) {
                    const uint32_t lim = __builtin_amdgcn_raw_buffer_load_b32(lrs, 0, 0, 16);
                    if ((int32_t)(lim - (base + u)) > 0 || !lspin.more(s)) break;
                    __builtin_amdgcn_s_sleep(16);
                }
            DLR_STAMP64M(22 + k, lane == 0 && k < 20);
            urow = (int64_t)u * kRefUnit + lane < B ? (int64_t)u * kRefUnit + lane : -1;
            if (urow >= 0) y = dd.label[ref_row(first, urow, N)];
            z = 0.0f;
            have_pend = lane == 0 && claiming;
            if (have_pend) pend = claim_issue();  // the unit after the next one
        }
        // stage g landed: every loader's pieces of it
        DLR_TACC_BEGIN();
        if ((int32_t)(lk - ((uint32_t)g + 1)) < 0) lk = ctl_poll_min<3>(ctl + kCtlL0, (uint32_t)g + 1, spin);
        DLR_TACC_LAP(t_wait);
        if (!(DLR_ABL & 64)) {
            // the stage's 64 columns in order, 4 sets of 16: set S's adds
            // interleaved with set S + 1's products (ref_set), set S + 2's
            // reads in flight
            const uint32_t wa = lds_addr(ring) + (uint32_t)ri * (kRefSlotF * 4);
            const uint32_t a = wa + 16 * lane;
            v4f xd[3][4], wd[3][4];
            float pp[2][16];
            ref_rd8<0>(xd[0], wd[0], a, wa);
            ref_rd8<1>(xd[1], wd[1], a, wa);
            DLR_REF_WAIT(8, xd[0], wd[0]);
            ref_products(pp[0], xd[0], wd[0]);
            ref_rd8<2>(xd[2], wd[2], a, wa);
            ref_set<0>(z, xd, wd, pp, a, wa);
            ref_set<1>(z, xd, wd, pp, a, wa);
            ref_set<2>(z, xd, wd, pp, a, wa);
            ref_set<3>(z, xd, wd, pp, a, wa);
        }
        DLR_TACC_LAP(t_comp);
        if (sg == spu - 1) {
            if (urow >= 0) {
                const float r = sigmoid_ref(z) - y;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r), rres, (int)(urow * 4), 0, 16);  // sc1
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every residual of the unit stored
            if (lane == 0) {
                if (!(sy.fault == kFaultRefPublish && u == 0))
                    __hip_atomic_fetch_add(sy.slot_cnt + (u / (kRefSlot / kRefUnit)), 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                // the next-but-one unit, before the stage count that lets the
                // loaders reach it
                ctl_write(s_unit + ((k + 2) & 3), have_pend ? claim_finish(pend) : kRefNone);
                ctl_write(ctl + kCtlIds, (uint32_t)k + 3);
            }
            DLR_STAMP64M(2 + k, lane == 0 && k < 20);
            DLR_STAMP64MV(42 + k, lane == 0 && k < 20, (unsigned long long)u);
        }
        if (lane == 0) ctl_post(ctl + kCtlComp, (uint32_t)g + 1);  // ring slot ri free
        if (++sg == spu) {
            sg = 0;
            ++k;
        }
        if (++ri == kRefRing) ri = 0;
    }
    DLR_STAMP64MV(60, lane == 0, t_wait);
    DLR_STAMP64MV(61, lane == 0, t_comp);
    DLR_STAMP64M(63, lane == 0);
}

// grid: max(D / 16, margin halves) workgroups; workgroup b runs the chain
// half of stripe b (b < D / 16) and a margin half (b < sy.mgrid)
template <bool FUSED, bool TILED>
__global__ __launch_bounds__(kRefThreads) void k_dense_ref(DevDense dd, int64_t first, int64_t B,
                                                           const float *__restrict__ wr, float *w,
                                                           float *__restrict__ gout, float *resid, DevRefSync sy,
                                                           float Bf, double Bd, float lr, float C) {
    extern __shared__ __attribute__((aligned(16))) float rsm[];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint32_t *ctl = reinterpret_cast<uint32_t *>(rsm + kRefOffCtl);
    if (threadIdx.x < 16) ctl[threadIdx.x] = threadIdx.x >= kCtlUnit ? kRefNone : 0u;
    DLR_STAMP64(0, threadIdx.x == 0);
    __syncthreads();  // the only workgroup barrier: the halves go their own ways
    if (wv < 4) {
        if (!(DLR_ABL & 32) && (int)blockIdx.x < (int)(dd.D / kRefCols))
            ref_chain_half<FUSED, TILED>(dd, first, B, w, gout, resid, sy, Bf, Bd, lr, C, rsm, wv, lane);
    } else if ((int)blockIdx.x < sy.mgrid) {
        ref_margin_half<TILED>(dd, first, B, wr, resid, sy, rsm, wv - 4, lane);
    }
}

// The tiled image of a row-major N x D shard (dense_ref_tiled): workgroup
// (S, R0) writes tile S of the 64-row blocks R0, R0 + gridDim.y, ...; thread
// t its chunks t + 256 m, in image order (rows past N: zeros).  No divisions
// (test_abi's FMA census).
__global__ __launch_bounds__(256) void k_dense_tile(const float *__restrict__ src, float *__restrict__ dst, int64_t N,
                                                    int64_t D, int64_t nR) {
    const int64_t nS = D / kRefStage, S = blockIdx.x;
    for (int64_t R = blockIdx.y; R < nR; R += gridDim.y) {
        float *tile = dst + (R * nS + S) * (kRefUnit * kRefStage);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int q = (int)threadIdx.x + 256 * m, i = q & 63, k = q >> 6;
            const int64_t row = R * kRefUnit + i;
            v4f v = {0.0f, 0.0f, 0.0f, 0.0f};
            if (row < N) v = *reinterpret_cast<const v4f *>(src + row * D + (S * kRefChunks + k) * 4);
            *reinterpret_cast<v4f *>(tile + 4 * q) = v;
        }
    }
}
#undef DLR_REF_WAIT

// K5 dense: LR::Test on dense rows (lr.cc:47-63, 100-106); counts and
// log-loss partials as k_predict.
template <bool VEC4>
__global__ __launch_bounds__(kWaves *kWave) void k_dense_predict(DevDense dd, const float *__restrict__ w,
                                                                 unsigned long long *__restrict__ correct,
                                                                 double *__restrict__ ll_part) {
    __shared__ double s_ll[kWaves];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double ll = 0.0;
    bool hit = false;
    if (i < dd.N) {
        const float *__restrict__ x = dd.X + i * dd.D;
        float z = 0.0f;
        int64_t j = 0;
        if (VEC4)
            for (; j + 4 <= dd.D; j += 4) {
                const float4 xv = *reinterpret_cast<const float4 *>(x + j);
                const float4 wv4 = *reinterpret_cast<const float4 *>(w + j);
                z = z + wv4.x * xv.x;
                z = z + wv4.y * xv.y;
                z = z + wv4.z * xv.z;
                z = z + wv4.w * xv.w;
            }
        for (; j < dd.D; ++j) z = z + w[j] * x[j];
        const float y = dd.label[i];
        hit = (z > 0.0f ? 1 : 0) == (int)y;
        ll = y != 0.0f ? softplus(-(double)z) : softplus((double)z);
    }
    const unsigned long long m = __ballot(hit);
    if (lane == 0 && m) atomicAdd(correct, (unsigned long long)__popcll(m));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ll += __shfl_xor(ll, off);
    if (lane == 0) s_ll[wv] = ll;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < kWaves; ++q) t += s_ll[q];
        ll_part[blockIdx.x] = t;
    }
}

// K4 for world > 1: this rank owns keys [kb, kb+n) ("serves" them, the
// role of KVStoreDistServer::DataHandle, main.cc:57-84).  recv holds the W
// ranks' pushed gradients for the owned range, rank-major.
__global__ __launch_bounds__(256) void k_merge_update(const float *__restrict__ recv, int W, int64_t chunk,
                                                      int64_t n, float *__restrict__ w_own, float lr, int mode) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    w_own[i] = server_apply(w_own[i], recv + i, chunk, W, lr, mode, false);
}

inline unsigned grid_for(int64_t n, int per_block) { return (unsigned)((n + per_block - 1) / per_block); }

}  // namespace

// Rows per wave for the margin: aim for about one window of entries per
// wave (fewer, longer-running waves for short rows; more for long rows).
int margin_seg(const DevBatch &bt) {
    if (bt.rows <= 0) return 64;
    const double avg = (double)bt.nnz / (double)bt.rows;
    if (avg * 64 <= kWin) return 64;
    if (avg * 32 <= kWin) return 32;
    return 16;
}

hipError_t launch_margin_residual(const DevBatch &bt, const float *w, float *resid, hipStream_t s) {
    if (bt.rows <= 0) return hipSuccess;
    const dim3 blk(kWaves * kWave);
    const bool unit = bt.val == nullptr;  // unit-valued shard: no value array
#define DLR_MR(SEG)                                                                                              \
    case SEG:                                                                                                    \
        if (unit)                                                                                                \
            hipLaunchKernelGGL((k_margin_residual<SEG, true>), dim3(grid_for(bt.rows, kWaves * SEG)), blk, 0, s, bt, \
                               w, resid);                                                                        \
        else                                                                                                     \
            hipLaunchKernelGGL((k_margin_residual<SEG, false>), dim3(grid_for(bt.rows, kWaves * SEG)), blk, 0, s,    \
                               bt, w, resid);                                                                    \
        break;
    switch (margin_seg(bt)) {
        DLR_MR(16)
        DLR_MR(32)
        DLR_MR(64)
        default:
            return hipErrorInvalidValue;
    }
#undef DLR_MR
    return hipGetLastError();
}

template <int HOT, int NW>
hipError_t launch_mh(const DevBatch &bt, const float *w, float *resid, unsigned cap, hipStream_t s,
                     const DevHotOut &ho) {
    const bool unit = bt.val == nullptr;
#define DLR_MH(SEG)                                                                                            \
    case SEG: {                                                                                                \
        const unsigned grid = std::min<unsigned>(grid_for(bt.rows, NW * SEG), cap);                            \
        if (unit)                                                                                              \
            hipLaunchKernelGGL((k_margin_hot<HOT, NW, SEG, true>), dim3(grid), dim3(NW * kWave), 0, s, bt, w,   \
                               resid, ho);                                                                     \
        else                                                                                                   \
            hipLaunchKernelGGL((k_margin_hot<HOT, NW, SEG, false>), dim3(grid), dim3(NW * kWave), 0, s, bt, w,  \
                               resid, ho);                                                                     \
        break;                                                                                                 \
    }
    switch (margin_seg(bt)) {
        DLR_MH(16)
        DLR_MH(32)
        DLR_MH(64)
        default:
            return hipErrorInvalidValue;
    }
#undef DLR_MH
    return hipGetLastError();
}

hipError_t launch_margin_hot(const DevBatch &bt, const float *w, int64_t D, float *resid, hipStream_t s,
                             int reserve, const DevHotOut &ho) {
    if (bt.rows <= 0) return hipSuccess;
    static const int ncu_all = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n = 256;
        return n > 0 ? n : 256;
    }();
    // reserve: CUs left to the band-hot chains running beside this launch
    // (its persistent workgroups would otherwise take every CU's LDS)
    const int ncu = std::max(ncu_all / 2, ncu_all - std::max(0, reserve));
    // 24,576 (below) or 16,384 hot weights x 16 waves, one workgroup per CU,
    // when D allows (C3 margin 1.749 ms with 16,384, round 2), else 8,192 x
    // 8, two per CU (1.779 ms).  Also
    // measured on C3: 16,384 x 8 (2.01 ms), 24,576 x 8 (2.00), 4,096 x 8
    // (2.04), 2,048 x 8 (1.87), 8,192 x 4 (1.79), 4,096 x 4 (2.22).
    // (a compacted-cold-gather variant -- ballot + list of the cold entries
    // -- measured slower: 1.90 vs 1.76 ms, profiles/r02_c3_margin_ab.txt)
    // 24,576 x 16 (LDS: exactly 160 KiB) since the rare-column order: C3
    // margin 1.579 vs 1.601 ms for 16,384 x 16 (profiles/r03j_bench_c3_*.json)
    if (D >= 24576) return launch_mh<24576, 16>(bt, w, resid, (unsigned)ncu, s, ho);
    if (D >= 16384) return launch_mh<16384, 16>(bt, w, resid, (unsigned)ncu, s, ho);
    return launch_mh<kMarginHot, kMarginHotWaves>(bt, w, resid, (unsigned)ncu * 2, s, ho);
}

int predict_grid(int64_t rows) { return rows <= 0 ? 0 : (int)grid_for(rows, kWaves * kWave); }

hipError_t launch_predict(const DevBatch &bt, const float *w, unsigned long long *correct, double *ll_part,
                          double *ll_out, hipStream_t s) {
    const int grid = predict_grid(bt.rows);
    if (grid > 0 && bt.val == nullptr)
        hipLaunchKernelGGL(k_predict<true>, dim3(grid), dim3(kWaves * kWave), 0, s, bt, w, correct, ll_part);
    else if (grid > 0)
        hipLaunchKernelGGL(k_predict<false>, dim3(grid), dim3(kWaves * kWave), 0, s, bt, w, correct, ll_part);
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, s, ll_part, grid, ll_out);
    return hipGetLastError();
}

hipError_t launch_pcsc_build(const DevBatch &bt, const uint32_t *base, int P, int64_t R, int64_t pblocks,
                             uint32_t *scratch, uint8_t *ends, uint16_t *row, float *val, hipStream_t s) {
    if (bt.rows <= 0 || pblocks <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(scratch, 0, (size_t)pblocks * 64 * 4, s);
    if (e != hipSuccess) return e;
    const unsigned gr = grid_for(bt.rows, 256);
    hipLaunchKernelGGL(k_pcsc_count, dim3(gr), dim3(256), 0, s, bt, P, R, scratch);
    hipLaunchKernelGGL(k_pcsc_scan, dim3(grid_for(pblocks * kWave, 256)), dim3(256), 0, s, base, pblocks, scratch, ends,
                       row, val);
    if (bt.val == nullptr)
        hipLaunchKernelGGL(k_pcsc_scatter<true>, dim3(gr), dim3(256), 0, s, bt, P, R, scratch, row, val);
    else
        hipLaunchKernelGGL(k_pcsc_scatter<false>, dim3(gr), dim3(256), 0, s, bt, P, R, scratch, row, val);
    hipLaunchKernelGGL(k_pcsc_order, dim3(grid_for(pblocks * 64, 256)), dim3(256), 0, s, base, ends, pblocks, row, val);
    return hipGetLastError();
}

hipError_t launch_grad(const DevCsc &cs, int64_t D, const float *resid, float *w, float *gout, int64_t B, float lr,
                       float C, bool fused, hipStream_t s) {
    if (D <= 0) return hipSuccess;
    const unsigned grid = cs.wstart ? (unsigned)((cs.nwaves + kWaves - 1) / kWaves) : grid_for(D, kWaves * kWave);
    if (grid == 0) return hipSuccess;
    const dim3 blk(kWaves * kWave);
    const float Bf = (float)B;
    const double Bd = (double)B;
#define DLR_G(RT, F, U)                                                                                          \
    hipLaunchKernelGGL((k_grad<RT, F, U>), dim3(grid), blk, 0, s, cs, static_cast<const RT *>(cs.row), D, resid, w, \
                       gout, Bf, Bd, lr, C)
#define DLR_GU(RT, F)      \
    if (cs.val == nullptr) \
        DLR_G(RT, F, true);  \
    else                   \
        DLR_G(RT, F, false);
    if (cs.row16) {
        if (fused) {
            DLR_GU(uint16_t, true)
        } else {
            DLR_GU(uint16_t, false)
        }
    } else {
        if (fused) {
            DLR_GU(uint32_t, true)
        } else {
            DLR_GU(uint32_t, false)
        }
    }
#undef DLR_GU
#undef DLR_G
    return hipGetLastError();
}

int grad_lds_fill(int64_t B) {
    if (B <= 4096) return 1;
    if (B <= 8192) return 2;
    if (B <= 16384) return 4;
    return 8;
}

// Batches of more than 16,384 rows: two phases of 32,768 rows in one buffer
// (k_grad_lds, "A double-buffered form").
int64_t grad_lds_phase_rows(int64_t B) { return (int64_t)grad_lds_fill(B) * 4096; }

namespace {
// The kernel form of a layout: FILL = its rows per phase / 4,096; one or
// two phases.
bool grad_lds_form_ok(const DevPcsc &pc) {
    return (pc.fill == 1 || pc.fill == 2 || pc.fill == 4 || pc.fill == 8) && pc.phases >= 1 && pc.phases <= 2;
}
// residual floats in LDS
size_t grad_lds_rrows(int fill) { return (size_t)fill * 4096; }
}  // namespace

hipError_t launch_grad_lds(const DevPcsc &pc, int64_t D, int64_t B, const float *resid, float *w, float *gout,
                           float lr, float C, bool fused, hipStream_t s) {
    if (D <= 0) return hipSuccess;
    const int64_t ng = (D + 63) / 64;
    const unsigned grid = (unsigned)((ng + kGradWaves * kGradNG - 1) / (kGradWaves * kGradNG));
    const dim3 blk(kGradWaves * kWave);
    const float Bf = (float)B;
    const double Bd = (double)B;
    if (!grad_lds_form_ok(pc)) return hipErrorInvalidValue;
    const int fill = pc.fill;
    const size_t lds = grad_lds_rrows(fill) * 4 + (size_t)kGradWaves * kBlkPad * 4;
#define DLR_GL(F)                                                                                                   \
    case F:                                                                                                         \
        if (fused)                                                                                                  \
            hipLaunchKernelGGL((k_grad_lds<F, true>), dim3(grid), blk, lds, s, pc, D, B, resid, w, gout, Bf, Bd, lr, \
                               C);                                                                                  \
        else                                                                                                        \
            hipLaunchKernelGGL((k_grad_lds<F, false>), dim3(grid), blk, lds, s, pc, D, B, resid, w, gout, Bf, Bd,    \
                               lr, C);                                                                              \
        break;
    switch (fill) {
        DLR_GL(1)
        DLR_GL(2)
        DLR_GL(4)
        DLR_GL(8)
        default:
            return hipErrorInvalidValue;
    }
#undef DLR_GL
    return hipGetLastError();
}

hipError_t launch_pm_products(const DevPm &pm, const float *w, int64_t D, float *p, hipStream_t s,
                              const uint32_t *slices, int64_t nslices) {
    const int64_t n = slices ? nslices : pm.S;
    if (n <= 0) return hipSuccess;
    if (pm.nblk > kPmMaxBlocks || pm.split < 1) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(((n + 7) / 8) * 8 * pm.split);
    hipLaunchKernelGGL(k_pm_products, dim3(grid), dim3(1024), 0, s, pm, w, D, p, slices, n);
    return hipGetLastError();
}

hipError_t launch_pm_windows(const DevPm *views, const DevPm &pm0, int64_t nwin, const DevBatch &bt,
                             const float *w, int64_t D, float *p, int64_t pstride, float *resid, hipStream_t s) {
    constexpr int64_t kWinRows = (int64_t)kPmMaxBlocks * kPmRows;
    if (nwin <= 0 || bt.rows <= 0) return hipSuccess;
    if (pm0.split < 1 || pstride % 64 != 0 || (nwin - 1) * kWinRows >= bt.rows || nwin * kWinRows < bt.rows)
        return hipErrorInvalidValue;
    const int64_t G = ((pm0.S + 7) / 8) * 8 * pm0.split;
    hipLaunchKernelGGL(k_pm_products_win, dim3((unsigned)(nwin * G)), dim3(1024), 0, s, views, G, w, D, p, pstride);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)(nwin * (kPmMaxBlocks / 4)));
    if (pm0.groups <= 4)
        hipLaunchKernelGGL((k_pm_margin_win<4>), grid, dim3(256), 0, s, views, bt, p, pstride, resid);
    else if (pm0.groups <= 8)
        hipLaunchKernelGGL((k_pm_margin_win<8>), grid, dim3(256), 0, s, views, bt, p, pstride, resid);
    else if (pm0.groups <= kPmMaxGroups)
        hipLaunchKernelGGL((k_pm_margin_win<kPmMaxGroups>), grid, dim3(256), 0, s, views, bt, p, pstride, resid);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

namespace {
int device_cus();
}  // namespace

hipError_t launch_pm_margin(const DevPm &pm, const DevBatch &bt, const float *p, float *resid, hipStream_t s) {
    if (bt.rows <= 0) return hipSuccess;
    if ((bt.rows + kPmRows - 1) / kPmRows != pm.nblk) return hipErrorInvalidValue;
    // one block per workgroup while the blocks fit the device's CUs twice
    const bool one = pm.nblk <= 2 * (int64_t)device_cus();
    const dim3 grid((unsigned)(one ? pm.nblk : (pm.nblk + 3) / 4)), blk(one ? kWave : 4 * kWave);
#define DLR_PMM(G)                                                                   \
    if (one)                                                                         \
        hipLaunchKernelGGL((k_pm_margin<G, 1>), grid, blk, 0, s, pm, bt, p, resid); \
    else                                                                             \
        hipLaunchKernelGGL((k_pm_margin<G, 4>), grid, blk, 0, s, pm, bt, p, resid);
    if (pm.groups <= 4) {
        DLR_PMM(4)
    } else if (pm.groups <= 8) {
        DLR_PMM(8)
    } else if (pm.groups <= kPmMaxGroups) {
        DLR_PMM(kPmMaxGroups)
    } else {
        return hipErrorInvalidValue;
    }
#undef DLR_PMM
    return hipGetLastError();
}

namespace {
// The one-launch step's kernel for a fill (a workgroup of every grid
// size it may take must fit beside the others: they wait for each other).
const void *grad_lds_mg_fn(int fill) {
    switch (fill) {
        case 1: return reinterpret_cast<const void *>(&k_grad_lds<1, true, true, true>);
        case 2: return reinterpret_cast<const void *>(&k_grad_lds<2, true, true, true>);
        case 4: return reinterpret_cast<const void *>(&k_grad_lds<4, true, true, true>);
        case 8: return reinterpret_cast<const void *>(&k_grad_lds<8, true, true, true>);
        default: return nullptr;
    }
}
size_t grad_lds_pm_lds(int fill) {
    return std::max(grad_lds_rrows(fill) * 4 + (size_t)kGradWaves * kBlkPad * 4, (size_t)(kPmSlice + kPmMaxBlocks) * 4);
}

// CUs of the current device (cached per device; 0 if the runtime cannot say)
int device_cus() {
    static int ncu[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (!ncu[dev] && hipDeviceGetAttribute(&ncu[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        (void)hipGetLastError();
        ncu[dev] = 0;
    }
    return ncu[dev];
}

// The MG launch's workgroups: one per slice, or more when that evens the
// blocks out over the CUs (C2: 1,024 blocks on 256 workgroups, 4 each, not
// 245 with up to 5: 26.6 vs 26.9 us); the extra workgroups only sum blocks.
int64_t grad_lds_mg_grid(int64_t nblk, int64_t grid) {
    const int64_t even = (nblk + 3) / 4;
    if (even > grid && even <= device_cus()) return even;
    return grid;
}
}  // namespace

// Workgroups of kernel fn (`threads` threads, `lds` bytes of dynamic LDS)
// that one CU holds at once, from the kernel's own attributes and gfx950's
// per-CU budgets (MI355X_MICROARCH.md, "Register files" and "Residency"):
// VGPRs 512 per lane per SIMD, allocated in granules of 8; at most 8 waves
// per SIMD and 32 per CU; SGPRs 800 per SIMD in granules of 16 plus 16 per
// wave (taken at the 112-register ceiling of a wave, since the attributes
// do not report SGPRs); a workgroup's waves spread over the 4 SIMDs; LDS
// 160 KiB per CU (static + dynamic).  The runtime's occupancy query is
// consulted too and the LOWER answer wins when it answers >= 1 -- it can
// say one block per CU too many near the SGPR steps (the guide's table);
// an answer of 0 (seen with hipSuccess: DESIGN.md 2.1) is not taken.
int resident_per_cu(const void *fn, int threads, size_t lds, int *query) {
    if (query) *query = -1;
    if (!fn || threads < 1) return 0;
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, fn) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    int dev = 0, cu_lds = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cu_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (threads > a.maxThreadsPerBlock) return 0;
    const int waves = (threads + kWave - 1) / kWave;
    const int per_simd = (waves + 3) / 4;  // a workgroup's waves on its busiest SIMD
    const int valloc = ((std::max(a.numRegs, 1) + 7) / 8) * 8;
    const int simd_waves = std::min({8, 512 / valloc, 800 / (112 + 16)});
    int n = std::min(simd_waves / per_simd, 32 / waves);
    const size_t need = a.sharedSizeBytes + lds;
    if (need > 0) n = std::min<int64_t>(n, (int64_t)cu_lds / (int64_t)need);
    int q = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, fn, threads, lds);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        q = -1;
    }
    if (query) *query = q;
    if (q >= 1) n = std::min(n, q);
    return std::max(n, 0);
}

int resident_grid(const void *fn, int threads, size_t lds) { return resident_per_cu(fn, threads, lds, nullptr) * device_cus(); }

// Whether batch b's pass 2 may run in its gradient's launch: the shape
// fits, and every workgroup of the launch is resident at once -- each one
// waits for blocks summed by the others, so one that is not resident
// would leave the resident ones waiting (D = 2^21 at B =
// 65,536 has 512 slices on 256 CUs; such batches take k_pm_margin).
bool grad_lds_mg_ok(const DevPm &cur, int64_t D, int64_t B, int phases, int fill) {
    const int64_t grid = (D + kPmSlice - 1) / kPmSlice;
    DevPcsc form{};
    form.phases = phases;
    form.fill = fill;
    if (!grad_lds_form_ok(form)) return false;
    // (wave v < the workgroup's pass-2 regions sums block x + grid * v)
    const int64_t regions = (int64_t)grad_lds_rrows(fill) / kPmCap;
    if (!(D > 0 && cur.groups <= 8 && cur.nblk == (B + kPmRows - 1) / kPmRows && cur.nblk <= grid * regions &&
          (int64_t)phases * fill * 4096 >= B))
        return false;
    static int cap[64][9] = {};  // per device and fill (cached: the check runs every step)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    int &c = cap[dev][fill];
    if (c == 0) c = resident_grid(grad_lds_mg_fn(fill), kGradWaves * kWave, grad_lds_pm_lds(fill));
    return c > 0 && grad_lds_mg_grid(cur.nblk, grid) <= c;
}

hipError_t launch_grad_lds_pm(const DevPcsc &pc, int64_t D, int64_t B, const float *resid, float *w, float lr,
                              float C, const DevPm &next, float *p, hipStream_t s, const DevP2 *mg) {
    if (D <= 0) return hipSuccess;
    const int64_t ng = (D + 63) / 64;
    const unsigned grid = (unsigned)((ng + kGradWaves * kGradNG - 1) / (kGradWaves * kGradNG));
    static_assert(kGradWaves * kGradNG * 64 == kPmSlice, "a gradient workgroup's columns are one slice");
    if ((int64_t)grid != next.S || next.nblk > kPmMaxBlocks) return hipErrorInvalidValue;
    if (!grad_lds_form_ok(pc)) return hipErrorInvalidValue;
    if (mg && (!grad_lds_mg_ok(mg->pm, D, B, pc.phases, pc.fill) || mg->bt.rows != B || !mg->cnt || !mg->resid))
        return hipErrorInvalidValue;
    // MG: every workgroup resident at once (grad_lds_mg_ok checked it)
    const unsigned mgrid = mg ? (unsigned)grad_lds_mg_grid(mg->pm.nblk, grid) : grid;
    const dim3 blk(kGradWaves * kWave);
    const float Bf = (float)B;
    const double Bd = (double)B;
    const int fill = pc.fill;
    const size_t lds = grad_lds_pm_lds(fill);
#define DLR_GLP(F)                                                                                                \
    case F:                                                                                                       \
        if (mg)                                                                                                   \
            hipLaunchKernelGGL((k_grad_lds<F, true, true, true>), dim3(mgrid), blk, lds, s, pc, D, B, resid, w,   \
                               nullptr, Bf, Bd, lr, C, next, p, *mg);                                             \
        else                                                                                                      \
            hipLaunchKernelGGL((k_grad_lds<F, true, true>), dim3(grid), blk, lds, s, pc, D, B, resid, w, nullptr, \
                               Bf, Bd, lr, C, next, p);                                                           \
        break;
    switch (fill) {
        DLR_GLP(1)
        DLR_GLP(2)
        DLR_GLP(4)
        DLR_GLP(8)
        default:
            return hipErrorInvalidValue;
    }
#undef DLR_GLP
    return hipGetLastError();
}

namespace {
size_t grad_rt_lds() {
    return std::max((size_t)(kRtCap + 16 + 2 * kRtRows) * 4, (size_t)(kPmSlice + kPmMaxBlocks) * 4);
}
const void *grad_rt_mg_fn(bool unit) {
    return unit ? reinterpret_cast<const void *>(&k_grad_rt<true, true, true, true>)
                : reinterpret_cast<const void *>(&k_grad_rt<true, true, false, true>);
}
}  // namespace

// Whether batch b's pass 2 may run in its row-round gradient's launch: a
// batch of >= 2 rounds (C2 at B = 16,384: 15.2 vs 16.6 us per step; at one
// round, B = 8,192, the separate pass 2 is faster: 13.9 vs 14.9,
// profiles/r05_c2_rt_mg.txt), every block has a summing wave (wave v <
// kRtRegions of workgroup x sums block x + grid * v) and every workgroup of
// the launch is resident at once.
bool grad_rt_mg_ok(const DevPm &cur, int64_t D, int64_t B, int rounds, bool unit) {
    const int64_t grid = (D + kPmSlice - 1) / kPmSlice;
    if (!(D > 0 && cur.groups <= 8 && cur.nblk == (B + kPmRows - 1) / kPmRows && cur.nblk <= grid * kRtRegions &&
          rounds >= 2 && rounds <= kRtMaxRounds && (int64_t)rounds * kRtRows >= B))
        return false;
    static int cap[64][2] = {};  // per device and value kind (cached: the check runs every step)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    int &c = cap[dev][unit];
    if (c == 0) c = resident_grid(grad_rt_mg_fn(unit), kGradWaves * kWave, grad_rt_lds());
    return c > 0 && grid <= c;
}

hipError_t launch_grad_rt(const DevRt &rt, int64_t D, int64_t B, const float *resid, float *w, float *gout, float lr,
                          float C, bool fused, const DevPm *next, float *p, hipStream_t s, const DevP2 *mg) {
    if (D <= 0) return hipSuccess;
    if (rt.rounds < 1 || rt.rounds > kRtMaxRounds || (next && !fused) || (mg && !next)) return hipErrorInvalidValue;
    if (mg && (!grad_rt_mg_ok(mg->pm, D, B, rt.rounds, rt.val == nullptr) || mg->bt.rows != B || !mg->cnt ||
               !mg->resid))
        return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((D + kPmSlice - 1) / kPmSlice);
    static_assert(kGradWaves * kGradNG * 64 == kPmSlice, "a gradient workgroup's columns are one slice");
    if (next && ((int64_t)grid != next->S || next->nblk > kPmMaxBlocks)) return hipErrorInvalidValue;
    const dim3 blk(kGradWaves * kWave);
    const float Bf = (float)B;
    const double Bd = (double)B;
    const size_t lds = grad_rt_lds();
    const bool unit = rt.val == nullptr;
    if (mg) {
        if (unit)
            hipLaunchKernelGGL((k_grad_rt<true, true, true, true>), dim3(grid), blk, lds, s, rt, D, resid, w, gout, Bf,
                               Bd, lr, C, *next, p, *mg);
        else
            hipLaunchKernelGGL((k_grad_rt<true, true, false, true>), dim3(grid), blk, lds, s, rt, D, resid, w, gout,
                               Bf, Bd, lr, C, *next, p, *mg);
        return hipGetLastError();
    }
#define DLR_GRT(F, PMX, U)                                                                                     \
    hipLaunchKernelGGL((k_grad_rt<F, PMX, U>), dim3(grid), blk, lds, s, rt, D, resid, w, gout, Bf, Bd, lr, C, \
                       next ? *next : DevPm{}, p)
    if (next) {
        if (unit)
            DLR_GRT(true, true, true);
        else
            DLR_GRT(true, true, false);
    } else if (fused) {
        if (unit)
            DLR_GRT(true, false, true);
        else
            DLR_GRT(true, false, false);
    } else {
        if (unit)
            DLR_GRT(false, false, true);
        else
            DLR_GRT(false, false, false);
    }
#undef DLR_GRT
    return hipGetLastError();
}

hipError_t launch_grad_touched(const DevCsc &cs, const uint32_t *cols, int64_t ncols, const float *resid,
                               const float *w, float *out, int64_t B, float lr, float C, bool fused, hipStream_t s) {
    if (ncols <= 0) return hipSuccess;
    const unsigned grid = grid_for(ncols, kWaves * kWave);
    const dim3 blk(kWaves * kWave);
    const float Bf = (float)B;
    const double Bd = (double)B;
#define DLR_GT1(RT, F, U)                                                                                         \
    hipLaunchKernelGGL((k_grad_touched<RT, F, U>), dim3(grid), blk, 0, s, cs, static_cast<const RT *>(cs.row), cols, \
                       ncols, resid, w, out, Bf, Bd, lr, C)
#define DLR_GT(RT, F)          \
    if (cs.val == nullptr)     \
        DLR_GT1(RT, F, true);  \
    else                       \
        DLR_GT1(RT, F, false);
    if (cs.row16) {
        if (fused) {
            DLR_GT(uint16_t, true)
        } else {
            DLR_GT(uint16_t, false)
        }
    } else {
        if (fused) {
            DLR_GT(uint32_t, true)
        } else {
            DLR_GT(uint32_t, false)
        }
    }
#undef DLR_GT
#undef DLR_GT1
    return hipGetLastError();
}

hipError_t launch_dense_l2(float *w, int64_t D, const RankSizes &rs, float lr, float C, int mode, hipStream_t s) {
    if (D <= 0) return hipSuccess;
    const int64_t work = std::max<int64_t>(D / 4, 4);
    const unsigned grid = (unsigned)std::min<int64_t>((work + 255) / 256, int64_t(1) << 30);
    hipLaunchKernelGGL(k_dense_l2, dim3(grid), dim3(256), 0, s, w, D, rs, lr, C, mode);
    return hipGetLastError();
}

hipError_t launch_l2_fill(float *g, const float *w, int64_t D, float Bf, float C, hipStream_t s) {
    if (D <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_l2_fill, dim3(grid_for(D, 256)), dim3(256), 0, s, g, w, D, Bf, C);
    return hipGetLastError();
}

hipError_t launch_scatter(float *w, const uint32_t *cols, const float *newv, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter, dim3(grid_for(n, 256)), dim3(256), 0, s, w, cols, newv, n);
    return hipGetLastError();
}

hipError_t launch_sparse_merge(const uint32_t *lists, int64_t cap, int64_t stride, const float *w,
                               const RankSizes &rs, float lr, float C, int mode, uint32_t *out_cols, float *out_newv,
                               hipStream_t s) {
    const int64_t n = (int64_t)rs.W * cap;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sparse_merge, dim3(grid_for(n, 256)), dim3(256), 0, s, lists, cap, stride, w, rs, lr, C,
                       mode, out_cols, out_newv);
    return hipGetLastError();
}

hipError_t launch_grad_long(const DevLong &lg, int64_t B, const float *resid, float *w, float *gout, float *part,
                            float lr, float C, bool fused, hipStream_t s, float *graw) {
    if (lg.ncols <= 0) return hipSuccess;
    const unsigned sgrid = (unsigned)std::min<int64_t>((lg.nseg + 3) / 4, 256 * 16);  // a wave per chunk
#define DLR_LS(RT, U)                                                                                      \
    hipLaunchKernelGGL((k_long_segments<RT, U>), dim3(sgrid), dim3(256), 0, s, lg.sptr, lg.nseg, lg.sched, \
                       static_cast<const RT *>(lg.row), lg.val, resid, part)
    if (lg.row16 && lg.val == nullptr)
        DLR_LS(uint16_t, true);
    else if (lg.row16)
        DLR_LS(uint16_t, false);
    else if (lg.val == nullptr)
        DLR_LS(uint32_t, true);
    else
        DLR_LS(uint32_t, false);
#undef DLR_LS
    const float Bf = (float)B;
    const double Bd = (double)B;
    const unsigned cgrid = grid_for(lg.ncols, 4);  // a wave per long column
    if (graw)
        hipLaunchKernelGGL((k_long_combine<false, true>), dim3(cgrid), dim3(256), 0, s, lg.cols, lg.cseg, lg.ncols,
                           part, w, graw, Bf, Bd, lr, C);
    else if (fused)
        hipLaunchKernelGGL(k_long_combine<true>, dim3(cgrid), dim3(256), 0, s, lg.cols, lg.cseg, lg.ncols, part, w,
                           gout, Bf, Bd, lr, C);
    else
        hipLaunchKernelGGL(k_long_combine<false>, dim3(cgrid), dim3(256), 0, s, lg.cols, lg.cseg, lg.ncols, part, w,
                           gout, Bf, Bd, lr, C);
    return hipGetLastError();
}

hipError_t launch_grad_band(const DevBand &bd, const float *resid, float *gacc, hipStream_t s, bool longrun,
                            bool skip_hot) {
    if (bd.nwaves <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((bd.nwaves + kWaves - 1) / kWaves);
    const dim3 blk(kWaves * kWave);
#define DLR_GB(RT, U, L)                                                                                     \
    hipLaunchKernelGGL((k_grad_band<RT, U, L>), dim3(grid), blk, 0, s, bd, static_cast<const RT *>(bd.row), resid, \
                       gacc, skip_hot)
#define DLR_GBL(RT, U)      \
    if (longrun)            \
        DLR_GB(RT, U, true); \
    else                    \
        DLR_GB(RT, U, false);
    if (bd.row16 && bd.val == nullptr) {
        DLR_GBL(uint16_t, true)
    } else if (bd.row16) {
        DLR_GBL(uint16_t, false)
    } else if (bd.val == nullptr) {
        DLR_GBL(uint32_t, true)
    } else {
        DLR_GBL(uint32_t, false)
    }
#undef DLR_GBL
#undef DLR_GB
    return hipGetLastError();
}

hipError_t launch_band_hot(const DevBand &bd, const uint32_t *hw, int64_t nhot, const float *resid, float *gacc,
                           hipStream_t s, uint32_t *err, int fault) {
    if (nhot <= 0) return hipSuccess;
#define DLR_BH(RT, U)                                                                                                \
    hipLaunchKernelGGL((k_band_hot<RT, U>), dim3((unsigned)nhot), dim3(256), kHotLds, s, bd, hw,                       \
                       static_cast<const RT *>(bd.row), resid, gacc, err, fault)
    if (bd.row16 && bd.val == nullptr)
        DLR_BH(uint16_t, true);
    else if (bd.row16)
        DLR_BH(uint16_t, false);
    else if (bd.val == nullptr)
        DLR_BH(uint32_t, true);
    else
        DLR_BH(uint32_t, false);
#undef DLR_BH
    return hipGetLastError();
}

hipError_t launch_flag_store(uint32_t *flag, uint32_t seq, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_store, dim3(1), dim3(1), 0, s, flag, seq);
    return hipGetLastError();
}

int hot_chain_grid(int64_t nh) { return (int)((nh + kHcCols - 1) / kHcCols); }

hipError_t launch_hot_chain(const DevHotChain &hc, float *gacc, hipStream_t s) {
    if (hc.nh <= 0) return hipSuccess;
    // 150 KB of LDS requested (the ring needs 32 KB): the workgroup holds its
    // CU alone, so nothing shares the chain's SIMD (as k_band_hot)
    hipLaunchKernelGGL(k_hot_chain, dim3((unsigned)hot_chain_grid(hc.nh)), dim3(2 * kHcCols * kWave), kHotLds, s, hc,
                       gacc);
    return hipGetLastError();
}

hipError_t launch_long_phase(const DevLPhase &lp, const uint32_t *cols, const uint32_t *cseg, int64_t ncols,
                             const float *resid, float *part, float *graw, hipStream_t s) {
    if (ncols <= 0 || lp.nph <= 0) return hipSuccess;
    const size_t lds = (size_t)(kLPhase + kLPWaves * kWin) * 4;
    if (lp.val == nullptr)
        hipLaunchKernelGGL(k_long_phase<true>, dim3((unsigned)lp.nph), dim3(kLPWaves * kWave), lds, s, lp, resid,
                           part);
    else
        hipLaunchKernelGGL(k_long_phase<false>, dim3((unsigned)lp.nph), dim3(kLPWaves * kWave), lds, s, lp, resid,
                           part);
    hipLaunchKernelGGL((k_long_combine<false, true>), dim3(grid_for(ncols, 4)), dim3(256), 0, s, cols, cseg, ncols,
                       part, nullptr, graw, 1.0f, 1.0, 0.0f, 0.0f);
    return hipGetLastError();
}

hipError_t launch_band_finalize(const float *gacc, float *w, float *gout, int64_t D, int64_t B, float lr, float C,
                                bool fused, hipStream_t s) {
    if (D <= 0) return hipSuccess;
    const float Bf = (float)B;
    const double Bd = (double)B;
    if (fused)
        hipLaunchKernelGGL(k_band_finalize<true>, dim3(grid_for((D + 3) / 4, 256)), dim3(256), 0, s, gacc, w, gout, D, Bf, Bd,
                           lr, C);
    else
        hipLaunchKernelGGL(k_band_finalize<false>, dim3(grid_for((D + 3) / 4, 256)), dim3(256), 0, s, gacc, w, gout, D, Bf, Bd,
                           lr, C);
    return hipGetLastError();
}

hipError_t launch_dense_margin(const DevDense &dd, int64_t first, int64_t B, const float *w, float *resid,
                               hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (dd.D % 4 == 0)
        hipLaunchKernelGGL(k_dense_margin<true>, dim3(grid_for(B, 256)), dim3(256), 0, s, dd, first, B, w, resid);
    else
        hipLaunchKernelGGL(k_dense_margin<false>, dim3(grid_for(B, 256)), dim3(256), 0, s, dd, first, B, w, resid);
    return hipGetLastError();
}

int64_t dense_chunks(int64_t B) { return (B + kDenseChunk - 1) / kDenseChunk; }

bool dense_fused_ok(int64_t D) { return D == 512 || D == 1024 || D == 2048 || D == 4096; }

hipError_t launch_dense_fused(const DevDense &dd, int64_t first, int64_t B, const float *w, float *part,
                              hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (!dense_fused_ok(dd.D)) return hipErrorInvalidValue;
    const size_t lds = ((size_t)2 * kFuseRows * dd.D + dd.D + kFuseRows * 66 + kDenseChunk) * 4 +
                       (size_t)(kDenseChunk + kFuseRows) * 8 + 16;
    const dim3 g((unsigned)dense_chunks(B)), blk(kFuseThreads);
    switch (dd.D) {
        case 512: hipLaunchKernelGGL(k_dense_fused<128>, g, blk, lds, s, dd, first, B, w, dd.D, part); break;
        case 1024: hipLaunchKernelGGL(k_dense_fused<256>, g, blk, lds, s, dd, first, B, w, dd.D, part); break;
        case 2048: hipLaunchKernelGGL(k_dense_fused<512>, g, blk, lds, s, dd, first, B, w, dd.D, part); break;
        default: hipLaunchKernelGGL(k_dense_fused<1024>, g, blk, lds, s, dd, first, B, w, dd.D, part); break;
    }
    return hipGetLastError();
}

hipError_t launch_dense_combine(const float *part, int64_t D, int64_t B, float *w, float *gout, float lr, float C,
                                bool fused, hipStream_t s) {
    const int64_t nch = dense_chunks(B);
    const int64_t Dp = (D + 3) & ~int64_t(3);
    const float Bf = (float)B;
    const double Bd = (double)B;
    if (fused)
        hipLaunchKernelGGL(k_dense_combine<true>, dim3(grid_for(D, 16)), dim3(256), 0, s, part, nch, Dp, D, w, gout, Bf,
                           Bd, lr, C);
    else
        hipLaunchKernelGGL(k_dense_combine<false>, dim3(grid_for(D, 16)), dim3(256), 0, s, part, nch, Dp, D, w, gout,
                           Bf, Bd, lr, C);
    return hipGetLastError();
}

// K6r's workgroups hand off to each other (chain slots wait for margin
// units, margin units for the chains' limit): the launch is at most what
// is resident at once -- D / 16 chain halves, and the margin halves capped
// to that capacity (dense_ref_cap, queried per device: one 512-thread
// workgroup with kRefLds per CU).
static int dense_ref_cap() {
    static int cap[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (cap[dev] == 0) {
        const void *fn = reinterpret_cast<const void *>(&k_dense_ref<true, true>);
        cap[dev] = std::min(256, resident_grid(fn, kRefThreads, kRefLds));
    }
    return cap[dev];
}
bool dense_ref_ok(int64_t D, int64_t N, int64_t B) {
    return D % kRefStage == 0 && D >= 512 && D / kRefCols <= dense_ref_cap() && B <= N && B < ((int64_t)1 << 31);
}
int64_t dense_ref_resid(int64_t B) { return (B + kRefSlot - 1) / kRefSlot * kRefSlot + 4; }
int64_t dense_ref_sync_words(int64_t B) { return (B + kRefSlot - 1) / kRefSlot + 96; }
int dense_ref_grid(int64_t D, int64_t B) {
    return (int)std::max<int64_t>(D / kRefCols, std::min<int64_t>(dense_ref_cap(), (B + kRefUnit - 1) / kRefUnit));
}

hipError_t launch_dense_ref(const DevDense &dd, int64_t first, int64_t B, float *w, float *gout, float *resid,
                            const DevRefSync &sy_in, float lr, float C, bool fused, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (!dense_ref_ok(dd.D, dd.N, B) || first < 0 || first >= dd.N) return hipErrorInvalidValue;
    DevRefSync sy = sy_in;
    sy.mgrid = (int)std::min<int64_t>(dense_ref_cap(), (B + kRefUnit - 1) / kRefUnit);
    const unsigned grid = (unsigned)std::max<int64_t>(dd.D / kRefCols, sy.mgrid);
    const float Bf = (float)B;
    const double Bd = (double)B;
#define DLR_REF(F, T)                                                                                              \
    hipLaunchKernelGGL((k_dense_ref<F, T>), dim3(grid), dim3(kRefThreads), kRefLds, s, dd, first, B, w, w, gout, resid, \
                       sy, Bf, Bd, lr, C)
    if (fused && dd.tiled)
        DLR_REF(true, true);
    else if (fused)
        DLR_REF(true, false);
    else if (dd.tiled)
        DLR_REF(false, true);
    else
        DLR_REF(false, false);
#undef DLR_REF
    return hipGetLastError();
}

int64_t dense_ref_tiled_floats(int64_t N, int64_t D) { return (N + kRefUnit - 1) / kRefUnit * kRefUnit * D; }

hipError_t launch_dense_tile(const float *src, float *dst, int64_t N, int64_t D, hipStream_t s) {
    if (D % kRefStage != 0 || N <= 0) return hipErrorInvalidValue;
    const int64_t nR = (N + kRefUnit - 1) / kRefUnit;
    hipLaunchKernelGGL(k_dense_tile, dim3((unsigned)(D / kRefStage), (unsigned)std::min<int64_t>(nR, 4096)), dim3(256), 0,
                       s, src, dst, N, D, nR);
    return hipGetLastError();
}

hipError_t launch_dense_grad(const DevDense &dd, int64_t first, int64_t B, const float *resid, float *w, float *gout,
                             float *part, bool blocked, float lr, float C, bool fused, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    const float Bf = (float)B;
    const double Bd = (double)B;
    if (!blocked && dd.D % 4 == 0) {
        const unsigned grid = (unsigned)((dd.D + kChainCols - 1) / kChainCols);
#define DLR_CH(R)                                                                                                   \
    if (fused)                                                                                                      \
        hipLaunchKernelGGL((k_dense_grad_chain<true, R>), dim3(grid), dim3(256), ChainCfg<R>::kLds, s, dd, first, B, \
                           resid, w, gout, Bf, Bd, lr, C);                                                          \
    else                                                                                                            \
        hipLaunchKernelGGL((k_dense_grad_chain<false, R>), dim3(grid), dim3(256), ChainCfg<R>::kLds, s, dd, first,   \
                           B, resid, w, gout, Bf, Bd, lr, C);
        DLR_CH(256)  // (256 rows per staging slot; 128 measured no faster)
#undef DLR_CH
        return hipGetLastError();
    }
    if (!blocked) {
        if (fused)
            hipLaunchKernelGGL(k_dense_grad_seq<true>, dim3(grid_for(dd.D, 256)), dim3(256), 0, s, dd, first, B, resid,
                               w, gout, Bf, Bd, lr, C);
        else
            hipLaunchKernelGGL(k_dense_grad_seq<false>, dim3(grid_for(dd.D, 256)), dim3(256), 0, s, dd, first, B,
                               resid, w, gout, Bf, Bd, lr, C);
        return hipGetLastError();
    }
    const int64_t nch = dense_chunks(B);
    const int64_t Dp = (dd.D + 3) & ~int64_t(3);
    if (dd.D % 4 == 0)
        hipLaunchKernelGGL(k_dense_grad_blocked<true>, dim3((unsigned)nch, grid_for(dd.D / 4, 256)), dim3(256), 0, s,
                           dd, first, B, resid, Dp, part);
    else
        hipLaunchKernelGGL(k_dense_grad_blocked<false>, dim3((unsigned)nch, grid_for(dd.D, 256)), dim3(256), 0, s,
                           dd, first, B, resid, Dp, part);
    if (fused)
        hipLaunchKernelGGL(k_dense_combine<true>, dim3(grid_for(dd.D, 16)), dim3(256), 0, s, part, nch, Dp, dd.D, w,
                           gout, Bf, Bd, lr, C);
    else
        hipLaunchKernelGGL(k_dense_combine<false>, dim3(grid_for(dd.D, 16)), dim3(256), 0, s, part, nch, Dp, dd.D,
                           w, gout, Bf, Bd, lr, C);
    return hipGetLastError();
}

hipError_t launch_dense_predict(const DevDense &dd, const float *w, unsigned long long *correct, double *ll_part,
                                double *ll_out, hipStream_t s) {
    const int grid = predict_dense_grid(dd.N);
    if (grid > 0) {
        if (dd.D % 4 == 0)
            hipLaunchKernelGGL(k_dense_predict<true>, dim3(grid), dim3(kWaves * kWave), 0, s, dd, w, correct,
                               ll_part);
        else
            hipLaunchKernelGGL(k_dense_predict<false>, dim3(grid), dim3(kWaves * kWave), 0, s, dd, w, correct,
                               ll_part);
    }
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, s, ll_part, grid, ll_out);
    return hipGetLastError();
}

int predict_dense_grid(int64_t rows) { return rows <= 0 ? 0 : (int)grid_for(rows, kWaves * kWave); }

hipError_t launch_merge_update(const float *recv, int W, int64_t chunk, int64_t n, float *w_own, float lr, int mode,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_merge_update, dim3(grid_for(n, 256)), dim3(256), 0, s, recv, W, chunk, n, w_own, lr, mode);
    return hipGetLastError();
}

}  // namespace dlr
