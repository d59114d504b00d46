// dlr_kernels.hip -- gfx950 kernels of the dist-lr hot path.
//
// Parity contract (DESIGN.md "Numerics"): every fp32 sum is
// accumulated in the reference's order with separate multiply and add
// (this file is compiled with -ffp-contract=off; tests check the ISA has no
// v_fma in these kernels), so results are bitwise equal to src/lr.cc:
//   margin  z_i = sum_j w_j*x_ij, j ascending          (lr.cc:108-112)
//   sigma_i = (float)(1/(1+exp(-(double)z_i)))          (lr.cc:113)
//   r_i     = sigma_i - y_i                             (lr.cc:38)
//   G_j     = sum_i fl32(r_i*x_ij), batch-row order     (lr.cc:35-39)
//   g_j     = fl32((double)G_j/B + (double)(fl32(C*w_j)/(float)B))  (lr.cc:40)
//   update  w_j -= fl32(fl32(lr*g_j)/(float)W)          (main.cc:70-72)
//
// Layout (DESIGN.md "Data layout in HBM"): the shard is resident as CSR
// (row_ptr int64, col int32, val fp32, label fp32); each batch also has a
// column-major copy (cptr uint32[D+1], batch-local row uint16/uint32, val
// fp32) built once at load time, so the per-column gradient sums run in
// batch-row order without atomics.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dlr_kernels.h"

namespace dlr {

namespace {

constexpr int kWave = 64;
constexpr int kMarginWaves = 4;    // waves per workgroup
constexpr int kMarginWin = 1024;   // CSR entries staged per wave per window

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// z for the row owned by this lane.  One wave owns 64 consecutive batch
// rows; their CSR entries are contiguous, so the wave stages them through
// LDS in windows with 16-byte coalesced loads and every lane then walks its
// own row in column order (the reference's summation order).
__device__ __forceinline__ float wave_row_margin(const DevBatch &bt, const float *__restrict__ w, int64_t row0,
                                                 int lane, int32_t *s_col, float *s_val, bool valid, int64_t my) {
    const int64_t rlast = min(row0 + kWave, bt.rows);
    const int64_t e0 = bt.row_ptr[row0];
    const int64_t e1 = bt.row_ptr[rlast];
    const int64_t a = valid ? bt.row_ptr[my] : e1;
    const int64_t b = valid ? bt.row_ptr[my + 1] : e1;
    float z = 0.0f;
    for (int64_t ws = e0 & ~int64_t(3); ws < e1; ws += kMarginWin) {
#pragma unroll
        for (int t = 0; t < kMarginWin / (4 * kWave); ++t) {
            const int o = (t * kWave + lane) * 4;
            const int64_t g = ws + o;
            if (g < e1) {
                const int4 c = *reinterpret_cast<const int4 *>(bt.col + g);
                const float4 v = *reinterpret_cast<const float4 *>(bt.val + g);
                *reinterpret_cast<int4 *>(s_col + o) = c;
                *reinterpret_cast<float4 *>(s_val + o) = v;
            }
        }
        wave_sync();
        const int64_t lo = a > ws ? a : ws;
        const int64_t hi = b < ws + kMarginWin ? b : ws + kMarginWin;
        int o = (int)(lo - ws);
        const int oe = (int)(hi - ws);
        for (; o + 4 <= oe; o += 4) {
            const float w0 = w[s_col[o]], w1 = w[s_col[o + 1]], w2 = w[s_col[o + 2]], w3 = w[s_col[o + 3]];
            const float p0 = w0 * s_val[o];
            z = z + p0;
            const float p1 = w1 * s_val[o + 1];
            z = z + p1;
            const float p2 = w2 * s_val[o + 2];
            z = z + p2;
            const float p3 = w3 * s_val[o + 3];
            z = z + p3;
        }
        for (; o < oe; ++o) {
            const float p = w[s_col[o]] * s_val[o];
            z = z + p;
        }
        wave_sync();
    }
    return z;
}

__device__ __forceinline__ float sigmoid_ref(float z) {
    // lr.cc:113: 1. / (1. + exp(-z)) in double (glibc double exp there,
    // OCML's correctly-rounded-to-<1ulp f64 exp here), returned as float.
    const double e = exp(-(double)z);
    return (float)(1.0 / (1.0 + e));
}

__global__ __launch_bounds__(kMarginWaves *kWave) void k_margin_residual(DevBatch bt, const float *__restrict__ w,
                                                                         float *__restrict__ resid) {
    __shared__ int32_t s_col[kMarginWaves][kMarginWin];
    __shared__ float s_val[kMarginWaves][kMarginWin];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t row0 = ((int64_t)blockIdx.x * kMarginWaves + wv) * kWave;
    if (row0 >= bt.rows) return;  // wave-uniform
    const int64_t my = row0 + lane;
    const bool valid = my < bt.rows;
    const float z = wave_row_margin(bt, w, row0, lane, s_col[wv], s_val[wv], valid, my);
    if (valid) {
        const float s = sigmoid_ref(z);
        resid[my] = s - bt.label[my];
    }
}

__device__ __forceinline__ double softplus(double t) { return t > 0 ? t + log1p(exp(-t)) : log1p(exp(t)); }

// LR::Test / Predict_ (lr.cc:47-63, 100-106): pred = z > 0; correct count by
// wave ballot (integer atomics: order-free), log-loss partial per workgroup
// in a fixed shuffle order (deterministic for a fixed grid).
__global__ __launch_bounds__(kMarginWaves *kWave) void k_predict(DevBatch bt, const float *__restrict__ w,
                                                                 unsigned long long *__restrict__ correct,
                                                                 double *__restrict__ ll_part) {
    __shared__ int32_t s_col[kMarginWaves][kMarginWin];
    __shared__ float s_val[kMarginWaves][kMarginWin];
    __shared__ double s_ll[kMarginWaves];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t row0 = ((int64_t)blockIdx.x * kMarginWaves + wv) * kWave;
    double ll = 0.0;
    if (row0 < bt.rows) {
        const int64_t my = row0 + lane;
        const bool valid = my < bt.rows;
        const float z = wave_row_margin(bt, w, row0, lane, s_col[wv], s_val[wv], valid, my);
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
        for (int i = 0; i < kMarginWaves; ++i) t += s_ll[i];
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

// K3 (+K4 when FUSED): one thread per feature column j walks the batch's
// column-major segment in batch-row order, so G_j is the reference's
// sequential fp32 sum; then the lr.cc:40 normalisation + L2 term.  FUSED
// (world == 1) applies the server update in place: with W == 1,
// fl32(fl32(lr*g)/1.0f) == fl32(lr*g) for every mode (main.cc:71, 81).
template <typename RowT, bool FUSED>
__global__ __launch_bounds__(256) void k_grad(DevCsc cs, const RowT *__restrict__ crow, int64_t D,
                                              const float *__restrict__ resid, float *__restrict__ w,
                                              float *__restrict__ gout, float Bf, double Bd, float lr, float C) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= D) return;
    const uint32_t s = cs.ptr[j], e = cs.ptr[j + 1];
    float G = 0.0f;
    for (uint32_t k = s; k < e; ++k) {
        const float p = resid[crow[k]] * cs.val[k];
        G = G + p;
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

// K4 for world > 1: this rank owns keys [kb, kb+n) ("serves" them, the
// role of KVStoreDistServer::DataHandle, main.cc:57-84).  recv holds the W
// ranks' pushed gradients for the owned range, rank-major.
__global__ __launch_bounds__(256) void k_merge_update(const float *__restrict__ recv, int W, int64_t chunk,
                                                      int64_t n, float *__restrict__ w_own, float lr, int mode) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float wi = w_own[i];
    const float Wf = (float)W;
    if (mode == 2) {  // async: each push applied in rank order (main.cc:80-82)
        for (int r = 0; r < W; ++r) {
            const float step = lr * recv[(int64_t)r * chunk + i];
            wi = wi - step;
        }
    } else if (mode == 1) {  // sync as written: last push only (main.cc:71)
        const float step = lr * recv[(int64_t)(W - 1) * chunk + i];
        wi = wi - step / Wf;
    } else {  // sync mean: merged = ((0 + g_0) + g_1) + ... (main.cc:59-65)
        float m = 0.0f;
        for (int r = 0; r < W; ++r) m = m + recv[(int64_t)r * chunk + i];
        const float step = lr * m;
        wi = wi - step / Wf;
    }
    w_own[i] = wi;
}

inline unsigned grid_for(int64_t n, int per_block) { return (unsigned)((n + per_block - 1) / per_block); }

}  // namespace

hipError_t launch_margin_residual(const DevBatch &bt, const float *w, float *resid, hipStream_t s) {
    if (bt.rows <= 0) return hipSuccess;
    const unsigned grid = grid_for(bt.rows, kMarginWaves * kWave);
    hipLaunchKernelGGL(k_margin_residual, dim3(grid), dim3(kMarginWaves * kWave), 0, s, bt, w, resid);
    return hipGetLastError();
}

int predict_grid(int64_t rows) { return rows <= 0 ? 0 : (int)grid_for(rows, kMarginWaves * kWave); }

hipError_t launch_predict(const DevBatch &bt, const float *w, unsigned long long *correct, double *ll_part,
                          double *ll_out, hipStream_t s) {
    const int grid = predict_grid(bt.rows);
    if (grid > 0)
        hipLaunchKernelGGL(k_predict, dim3(grid), dim3(kMarginWaves * kWave), 0, s, bt, w, correct, ll_part);
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, s, ll_part, grid, ll_out);
    return hipGetLastError();
}

hipError_t launch_grad(const DevCsc &cs, int64_t D, const float *resid, float *w, float *gout, int64_t B, float lr,
                       float C, bool fused, hipStream_t s) {
    if (D <= 0) return hipSuccess;
    const unsigned grid = grid_for(D, 256);
    const float Bf = (float)B;
    const double Bd = (double)B;
    if (cs.row16) {
        const uint16_t *r = static_cast<const uint16_t *>(cs.row);
        if (fused)
            hipLaunchKernelGGL((k_grad<uint16_t, true>), dim3(grid), dim3(256), 0, s, cs, r, D, resid, w, gout, Bf,
                               Bd, lr, C);
        else
            hipLaunchKernelGGL((k_grad<uint16_t, false>), dim3(grid), dim3(256), 0, s, cs, r, D, resid, w, gout, Bf,
                               Bd, lr, C);
    } else {
        const uint32_t *r = static_cast<const uint32_t *>(cs.row);
        if (fused)
            hipLaunchKernelGGL((k_grad<uint32_t, true>), dim3(grid), dim3(256), 0, s, cs, r, D, resid, w, gout, Bf,
                               Bd, lr, C);
        else
            hipLaunchKernelGGL((k_grad<uint32_t, false>), dim3(grid), dim3(256), 0, s, cs, r, D, resid, w, gout, Bf,
                               Bd, lr, C);
    }
    return hipGetLastError();
}

hipError_t launch_merge_update(const float *recv, int W, int64_t chunk, int64_t n, float *w_own, float lr, int mode,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_merge_update, dim3(grid_for(n, 256)), dim3(256), 0, s, recv, W, chunk, n, w_own, lr, mode);
    return hipGetLastError();
}

}  // namespace dlr
