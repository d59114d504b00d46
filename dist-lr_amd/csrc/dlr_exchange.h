// dlr_exchange.h -- the data-parallel exchange's rules, ONE source for the
// HIP kernels (dlr_kernels.hip: k_merge_update, k_dense_l2, k_sparse_merge)
// and the host (dlr_engine.cpp: the step's collective plan, and the C-ABI's
// host-side merges that tests/test_dist_gloo.py drives across processes).
//
// Replaces KVStoreDistServer::DataHandle (src/main.cc:57-84) and the
// KVWorker Push/Pull key layout (main.cc:98-101, lr.cc:116-132): rank r owns
// keys [r * chunk, (r + 1) * chunk) (dlr_key_range), merges the W ranks'
// pushes of them in rank order, and every rank pulls the merged weights.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

#include "dlr_kernels.h"

#ifdef __HIPCC__
#define DLR_HD __host__ __device__ __forceinline__
#else
#define DLR_HD inline
#endif

namespace dlr {

// The server update of one weight given the W ranks' pushes g_r, g_r at
// g[r * stride] (main.cc:57-84).  mode 0 (sync mean): merged = ((0 + g_0)
// + g_1) + ... in rank order (main.cc:59-65's buffer), w -= fl32(lr *
// merged) / W; mode 1 (sync as written): only the last push, w -=
// fl32(lr * g_{W-1}) / W (main.cc:71); mode 2 (async): each push applied in
// rank order, w -= fl32(lr * g_r) (main.cc:80-82).  single: one rank, w -=
// fl32(lr * g_0) -- the same bits as mode 0 with W = 1.
DLR_HD float server_apply(float wj, const float *g, int64_t stride, int W, float lr, int mode, bool single) {
    if (single) {
        const float step = lr * g[0];
        return wj - step;
    }
    const float Wf = (float)W;
    if (mode == 2) {
        for (int r = 0; r < W; ++r) {
            const float step = lr * g[(int64_t)r * stride];
            wj = wj - step;
        }
        return wj;
    }
    if (mode == 1) {
        const float step = lr * g[(int64_t)(W - 1) * stride];
        return wj - step / Wf;
    }
    float m = 0.0f;
    for (int r = 0; r < W; ++r) m = m + g[(int64_t)r * stride];
    const float step = lr * m;
    return wj - step / Wf;
}

// The update of a weight no rank touched (touched layout): every push is
// rank r's L2 term l2_r = fl32(fl32(C * w) / (float)B_r) (lr.cc:40 with
// G_j = +0), merged as server_apply.
// (server_apply's arithmetic written out: no per-rank array, which the
// streaming L2 pass would index dynamically)
DLR_HD float l2_only_update(float wj, const RankSizes &rs, float lr, float C, int mode) {
    const float cw = C * wj;
    if (rs.W == 1) {
        const float l2 = cw / rs.Bf[0];
        const float step = lr * l2;
        return wj - step;
    }
    const float Wf = (float)rs.W;
    if (mode == 2) {
        for (int r = 0; r < rs.W; ++r) {
            const float l2 = cw / rs.Bf[r];
            const float step = lr * l2;
            wj = wj - step;
        }
        return wj;
    }
    if (mode == 1) {
        const float l2 = cw / rs.Bf[rs.W - 1];
        const float step = lr * l2;
        return wj - step / Wf;
    }
    float m = 0.0f;
    for (int r = 0; r < rs.W; ++r) m = m + cw / rs.Bf[r];
    const float step = lr * m;
    return wj - step / Wf;
}

// Sparse exchange (touched layout): rank r's all-gathered block of
// `stride` words is [count | cols[cap] | g[cap]] (cols ascending).  The
// entry (r, s) OWNS its column iff no lower rank touched it; the owner
// merges all W pushes in rank order (a rank that did not touch the column
// pushed its L2 term).  Returns false for a non-owner (or s >= count).
DLR_HD int64_t find_sorted(const uint32_t *cols, int64_t n, uint32_t c) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cols[mid] < c)
            lo = mid + 1;
        else
            hi = mid;
    }
    return (lo < n && cols[lo] == c) ? lo : -1;
}
DLR_HD bool sparse_merge_entry(const uint32_t *lists, int64_t cap, int64_t stride, const float *w,
                               const RankSizes &rs, float lr, float C, int mode, int r, int64_t s, uint32_t *col,
                               float *newv) {
    const int W = rs.W;
    const uint32_t *blk = lists + (int64_t)r * stride;
    if (s >= (int64_t)blk[0]) return false;
    const uint32_t c = blk[1 + s];
    for (int q = 0; q < r; ++q) {
        const uint32_t *bq = lists + (int64_t)q * stride;
        if (find_sorted(bq + 1, bq[0], c) >= 0) return false;
    }
    const float wj = w[c];
    const float cw = C * wj;
    float g[kMaxRanks];
    for (int q = 0; q < W; ++q) {
        const uint32_t *bq = lists + (int64_t)q * stride;
        const int64_t k = q == r ? s : find_sorted(bq + 1, bq[0], c);
        if (k >= 0) {
            const uint32_t bits = bq[1 + cap + k];
            float v;
            __builtin_memcpy(&v, &bits, 4);
            g[q] = v;
        } else {
            g[q] = cw / rs.Bf[q];
        }
    }
    *col = c;
    *newv = server_apply(wj, g, 1, W, lr, mode, false);
    return true;
}

// The collectives of ONE world > 1 training step, in the order every rank
// issues them (dlr_train_step): a function of the protocol, D, W and the
// exchange form only -- never of the rank or the data -- so the ranks'
// RCCL calls pair up.
//   key range (dense / LDS / classic / band layouts): ALL_TO_ALL of the
//     pushed gradient's key ranges (chunk words per peer), the rank-ordered
//     merge of the owned range, then the pull: ALL_GATHER of the merged
//     ranges (chunk words a rank), or -- the all-gather in pieces overlapped
//     with the next batch's pass 1 -- ALL_GATHER_PART k of `pieces`
//     (offset k * sub, count min(sub, chunk - offset) of every rank's range);
//   touched (huge D): ALL_GATHER of each rank's [count | cols | g] block
//     (1 + 2 * cap words), merged on every rank alike.
enum ExchangeProtocol { kXKeyRange = 0, kXTouched = 1 };
enum CollKind { kCollAllToAll = 1, kCollAllGather = 2, kCollAllGatherPart = 3 };
struct CollOp {
    int64_t kind, words, off, count;
};
inline std::vector<CollOp> exchange_plan(int protocol, int64_t D, int W, int pieces, int64_t cap) {
    std::vector<CollOp> ops;  // (W = 1: the same ops, through a one-rank communicator)
    if (W < 1) return ops;
    const int64_t chunk = (D + W - 1) / W;
    if (protocol == kXTouched) {
        ops.push_back({kCollAllGather, 1 + 2 * cap, 0, 0});
        return ops;
    }
    ops.push_back({kCollAllToAll, chunk, 0, 0});
    if (pieces <= 1) {  // (0: no overlap; 1: the overlap with one plain all-gather)
        ops.push_back({kCollAllGather, chunk, 0, 0});
        return ops;
    }
    const int64_t sub = (chunk + pieces - 1) / pieces;
    for (int k = 0; k < pieces; ++k) {
        const int64_t off = k * sub;
        ops.push_back({kCollAllGatherPart, chunk, off, off < chunk ? std::min(sub, chunk - off) : 0});
    }
    return ops;
}

}  // namespace dlr
