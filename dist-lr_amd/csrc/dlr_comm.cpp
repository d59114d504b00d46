// dlr_comm.cpp -- RCCL and in-process loopback transports (dlr_comm.h).
#include "dlr_comm.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace dlr {

namespace {

bool hip_ok(hipError_t e, const char *what, std::string &err) {
    if (e == hipSuccess) return true;
    err = std::string(what) + ": " + hipGetErrorString(e);
    return false;
}

bool nccl_ok(ncclResult_t r, const char *what, std::string &err) {
    if (r == ncclSuccess) return true;
    err = std::string(what) + ": " + ncclGetErrorString(r);
    return false;
}

// ------------------------------------------------------------------ RCCL

class RcclComm final : public Comm {
public:
    RcclComm(ncclComm_t c, int world, int rank) : comm_(c), world_(world), rank_(rank) {}
    ~RcclComm() override {
        if (!aborted_) ncclCommDestroy(comm_);
    }
    void abort(const std::string &) override {
        if (!aborted_) (void)ncclCommAbort(comm_);  // frees the communicator; peers' RCCL calls error out
        aborted_ = true;
    }
    int world() const override { return world_; }
    int rank() const override { return rank_; }
    const char *kind() const override { return "rccl"; }
    bool all_reduce_i64(int64_t *d, size_t n, bool max, hipStream_t s, std::string &err) override {
        if (aborted_) return nccl_ok(ncclInvalidUsage, "aborted communicator", err);
        return nccl_ok(ncclAllReduce(d, d, n, ncclInt64, max ? ncclMax : ncclSum, comm_, s), "ncclAllReduce", err);
    }
    bool all_gather(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) override {
        if (aborted_) return nccl_ok(ncclInvalidUsage, "aborted communicator", err);
        return nccl_ok(ncclAllGather(send, recv, words, ncclUint32, comm_, s), "ncclAllGather", err);
    }
    bool all_to_all(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) override {
        if (aborted_) return nccl_ok(ncclInvalidUsage, "aborted communicator", err);
        return nccl_ok(ncclAllToAll(send, recv, words, ncclUint32, comm_, s), "ncclAllToAll", err);
    }
    bool all_gather_part(void *buf, size_t chunk, size_t off, size_t count, hipStream_t s,
                         std::string &err) override {
        if (aborted_) return nccl_ok(ncclInvalidUsage, "aborted communicator", err);
        if (world_ == 1 || count == 0) return true;
        // point to point: the piece of every peer's block, strided by chunk
        uint32_t *b = static_cast<uint32_t *>(buf);
        if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
        bool ok = true;
        for (int q = 0; q < world_ && ok; ++q) {
            if (q == rank_) continue;
            ok = nccl_ok(ncclSend(b + (size_t)rank_ * chunk + off, count, ncclUint32, q, comm_, s), "ncclSend", err) &&
                 nccl_ok(ncclRecv(b + (size_t)q * chunk + off, count, ncclUint32, q, comm_, s), "ncclRecv", err);
        }
        const bool ended = nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err);
        return ok && ended;
    }
    int count() const {
        int n = 0;
        return ncclCommCount(comm_, &n) == ncclSuccess ? n : -1;
    }

private:
    ncclComm_t comm_;
    int world_, rank_;
    bool aborted_ = false;
};

}  // namespace

bool rccl_unique_id(void *out, std::string &err) {
    ncclUniqueId id;
    if (!nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId", err)) return false;
    static_assert(sizeof(id) <= 128, "DLR_UNIQUE_ID_BYTES");
    memcpy(out, &id, sizeof(id));
    return true;
}

Comm *make_rccl_comm(int world, int rank, const void *unique_id, std::string &err) {
    ncclUniqueId id;
    if (world > 1) {
        memcpy(&id, unique_id, sizeof(id));
    } else if (!nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId", err)) {
        return nullptr;
    }
    ncclComm_t c = nullptr;
    if (!nccl_ok(ncclCommInitRank(&c, world, id, rank), "ncclCommInitRank", err)) return nullptr;
    auto *rc = new RcclComm(c, world, rank);
    // the communicator's own rank count (reported by bench.py as rccl_nranks)
    if (rc->count() != world) {
        err = "ncclCommCount disagrees with the world size";
        delete rc;
        return nullptr;
    }
    return rc;
}

// ------------------------------------------------------------------ loopback

// Seconds a loopback rank waits for its peers at a collective before the
// group is declared broken: DLR_LOOPBACK_TIMEOUT_S (default 1,800 -- long
// enough for W ranks building large layouts one after another on one GPU;
// a rank that FAILS releases its peers at once through abort()).
int loop_timeout_s() {
    const char *v = getenv("DLR_LOOPBACK_TIMEOUT_S");
    const int s = v ? atoi(v) : 0;
    return s > 0 ? s : 1800;
}

struct LoopGroup {
    explicit LoopGroup(int w) : W(w), timeout_s(loop_timeout_s()), send((size_t)w, nullptr), recv((size_t)w, nullptr) {}
    const int W;
    const int timeout_s;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;  // a rank timed out or aborted: every later barrier fails at once
    std::string why;      // ... and why
    std::vector<const void *> send;
    std::vector<void *> recv;
    std::atomic<int> refs{0};

    void abort(const std::string &reason) {
        std::lock_guard<std::mutex> lk(mu);
        if (!broken) why = reason;
        broken = true;
        cv.notify_all();
    }

    // Generation barrier over the W ranks (each rank is one host thread).
    bool barrier(std::string &err) {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) {
            err = "loopback group: a peer failed earlier (" + why + ")";
            return false;
        }
        const uint64_t g = gen;
        if (++arrived == W) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(timeout_s), [&] { return gen != g || broken; })) {
            broken = true;
            why = "peers did not reach a collective within " + std::to_string(timeout_s) + " s";
            cv.notify_all();
        }
        if (gen != g) return true;  // released by the last arriver (an abort after that does not undo it)
        err = "loopback group: " + why;
        return false;
    }
};

namespace {

class LoopbackComm final : public Comm {
public:
    LoopbackComm(LoopGroup *g, int rank) : g_(g), rank_(rank) { g_->refs.fetch_add(1); }
    ~LoopbackComm() override {
        if (g_->refs.fetch_sub(1) == 1) delete g_;
    }
    int world() const override { return g_->W; }
    int rank() const override { return rank_; }
    const char *kind() const override { return "loopback"; }
    void abort(const std::string &why) override { g_->abort("rank " + std::to_string(rank_) + ": " + why); }

    bool all_reduce_i64(int64_t *d, size_t n, bool max, hipStream_t s, std::string &err) override {
        const int W = g_->W;
        if (!publish(d, d, s, err)) return false;
        std::vector<int64_t> all((size_t)W * n);
        bool ok = true;
        for (int q = 0; q < W && ok; ++q)
            ok = hip_ok(hipMemcpyAsync(all.data() + (size_t)q * n, g_->send[(size_t)q], n * 8, hipMemcpyDeviceToHost, s),
                        "loopback all_reduce (gather)", err);
        ok = ok && hip_ok(hipStreamSynchronize(s), "loopback all_reduce", err);
        if (!g_->barrier(err) || !ok) return false;  // every rank has read every buffer
        std::vector<int64_t> r(all.begin(), all.begin() + (ptrdiff_t)n);
        for (int q = 1; q < W; ++q)  // rank order
            for (size_t i = 0; i < n; ++i) {
                const int64_t v = all[(size_t)q * n + i];
                r[i] = max ? std::max(r[i], v) : r[i] + v;
            }
        return hip_ok(hipMemcpyAsync(d, r.data(), n * 8, hipMemcpyHostToDevice, s), "loopback all_reduce (scatter)",
                      err) &&
               hip_ok(hipStreamSynchronize(s), "loopback all_reduce", err);
    }

    bool all_gather(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) override {
        const size_t bytes = words * 4;
        if (!publish(send, recv, s, err)) return false;
        bool ok = true;
        for (int q = 0; q < g_->W && ok; ++q) {
            char *dst = static_cast<char *>(recv) + (size_t)q * bytes;
            if (dst == g_->send[(size_t)q] || bytes == 0) continue;  // in place
            ok = hip_ok(hipMemcpyAsync(dst, g_->send[(size_t)q], bytes, hipMemcpyDeviceToDevice, s),
                        "loopback all_gather", err);
        }
        return finish(ok, s, err);
    }

    bool all_gather_part(void *buf, size_t chunk, size_t off, size_t count, hipStream_t s,
                         std::string &err) override {
        if (!publish(buf, buf, s, err)) return false;
        bool ok = true;
        for (int q = 0; q < g_->W && ok && count; ++q) {
            if (q == rank_) continue;
            const size_t at = ((size_t)q * chunk + off) * 4;
            ok = hip_ok(hipMemcpyAsync(static_cast<char *>(buf) + at, static_cast<const char *>(g_->send[(size_t)q]) + at,
                                       count * 4, hipMemcpyDeviceToDevice, s),
                        "loopback all_gather_part", err);
        }
        return finish(ok, s, err);
    }

    bool all_to_all(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) override {
        const size_t bytes = words * 4;
        if (!publish(send, recv, s, err)) return false;
        bool ok = true;
        for (int q = 0; q < g_->W && ok && bytes; ++q)
            ok = hip_ok(hipMemcpyAsync(static_cast<char *>(recv) + (size_t)q * bytes,
                                       static_cast<const char *>(g_->send[(size_t)q]) + (size_t)rank_ * bytes, bytes,
                                       hipMemcpyDeviceToDevice, s),
                        "loopback all_to_all", err);
        return finish(ok, s, err);
    }

private:
    // This rank's buffers are complete (stream drained) and visible to the
    // peers once every rank has passed the barrier.
    bool publish(const void *send, void *recv, hipStream_t s, std::string &err) {
        if (!hip_ok(hipStreamSynchronize(s), "loopback collective", err)) return false;
        g_->send[(size_t)rank_] = send;
        g_->recv[(size_t)rank_] = recv;
        return g_->barrier(err);
    }
    // The copies out of the peers' buffers are done before any rank reuses
    // its send buffer.
    bool finish(bool ok, hipStream_t s, std::string &err) {
        ok = ok && hip_ok(hipStreamSynchronize(s), "loopback collective", err);
        std::string berr;
        const bool b = g_->barrier(berr);
        if (ok && !b) err = berr;
        return ok && b;
    }

    LoopGroup *g_;
    int rank_;
};

}  // namespace

LoopGroup *make_loop_group(int world) { return new LoopGroup(world); }

Comm *make_loopback_comm(LoopGroup *g, int rank) { return new LoopbackComm(g, rank); }

}  // namespace dlr
