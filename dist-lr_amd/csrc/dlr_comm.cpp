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
#include <thread>
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

// rec (tests, make_rccl_recorder): no communicator -- every RCCL call the
// transport would make is appended to *rec as a line instead (the calls'
// arguments as RCCL would get them: counts, peers, buffer offsets in words).
class RcclComm final : public Comm {
public:
    RcclComm(ncclComm_t c, int world, int rank, std::string *rec = nullptr)
        : comm_(c), world_(world), rank_(rank), rec_(rec) {}
    ~RcclComm() override {
        if (rec_) return;
        if (abort_req_.load())
            abort_now();
        else
            ncclCommDestroy(comm_);
    }
    // Any thread: flags the communicator.  Its driving thread aborts it
    // (abort_now) at the next collective or wait: ncclCommAbort on a
    // communicator another thread is using would free it under that
    // thread.
    void abort(const std::string &why) override {
        {
            std::lock_guard<std::mutex> g(mu_);
            if (why_.empty()) why_ = why;
        }
        abort_req_.store(true);
    }
    bool wait(hipStream_t s, std::string &err) override {
        // poll the stream; a flagged communicator is aborted here, which
        // makes its pending collective kernels return, then the stream drains
        for (int spin = 0;; ++spin) {
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) return hip_ok(e, "hipStreamQuery", err);
            if (abort_req_.load()) abort_now();
            if (spin > 2000) std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        return !flagged(err);
    }
    int world() const override { return world_; }
    int rank() const override { return rank_; }
    const char *kind() const override { return "rccl"; }
    bool all_reduce_i64(int64_t *d, size_t n, bool max, hipStream_t s, std::string &err) override {
        if (flagged(err)) return false;
        if (rec_) return log("ncclAllReduce int64 count=" + std::to_string(n) + (max ? " max" : " sum"));
        return nccl_ok(ncclAllReduce(d, d, n, ncclInt64, max ? ncclMax : ncclSum, comm_, s), "ncclAllReduce", err);
    }
    bool all_gather(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) override {
        if (flagged(err)) return false;
        if (rec_) return log("ncclAllGather uint32 count=" + std::to_string(words));
        return nccl_ok(ncclAllGather(send, recv, words, ncclUint32, comm_, s), "ncclAllGather", err);
    }
    bool all_to_all(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) override {
        if (flagged(err)) return false;
        if (rec_) return log("ncclAllToAll uint32 count=" + std::to_string(words));
        return nccl_ok(ncclAllToAll(send, recv, words, ncclUint32, comm_, s), "ncclAllToAll", err);
    }
    bool all_gather_part(void *buf, size_t chunk, size_t off, size_t count, hipStream_t s,
                         std::string &err) override {
        if (flagged(err)) return false;
        if (world_ == 1 || count == 0) return true;
        // point to point: the piece of every peer's block, strided by chunk
        uint32_t *b = static_cast<uint32_t *>(buf);
        if (rec_) {
            log("ncclGroupStart");
            for (int q = 0; q < world_; ++q) {
                if (q == rank_) continue;
                log("ncclSend uint32 count=" + std::to_string(count) + " peer=" + std::to_string(q) +
                    " at=" + std::to_string((size_t)rank_ * chunk + off));
                log("ncclRecv uint32 count=" + std::to_string(count) + " peer=" + std::to_string(q) +
                    " at=" + std::to_string((size_t)q * chunk + off));
            }
            return log("ncclGroupEnd");
        }
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
    bool log(const std::string &line) {
        *rec_ += line;
        *rec_ += '\n';
        return true;
    }
    // the driving thread: a flagged communicator is aborted, the call fails
    bool flagged(std::string &err) {
        if (!abort_req_.load()) return false;
        abort_now();
        std::lock_guard<std::mutex> g(mu_);
        err = "RCCL communicator aborted (" + why_ + ")";
        return true;
    }
    void abort_now() {
        if (!aborted_.exchange(true)) (void)ncclCommAbort(comm_);
    }

    ncclComm_t comm_;
    int world_, rank_;
    std::string *rec_;
    std::atomic<bool> abort_req_{false}, aborted_{false};
    std::mutex mu_;
    std::string why_;
};

}  // namespace

Comm *make_rccl_recorder(int world, int rank, std::string *log) { return new RcclComm(nullptr, world, rank, log); }

bool issue(Comm &comm, const CollOp &op, const void *send, void *recv, hipStream_t s, std::string &err) {
    switch (op.kind) {
        case kCollAllToAll:
            return comm.all_to_all(send, recv, (size_t)op.words, s, err);
        case kCollAllGather:
            return comm.all_gather(send, recv, (size_t)op.words, s, err);
        case kCollAllGatherPart:
            return comm.all_gather_part(recv, (size_t)op.words, (size_t)op.off, (size_t)op.count, s, err);
        default:
            err = "unknown collective in the exchange plan";
            return false;
    }
}

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
    LoopGroup(int w, bool a)
        : W(w), async(a), timeout_s(loop_timeout_s()), send((size_t)w, nullptr), recv((size_t)w, nullptr),
          ev_send((size_t)w, nullptr), ev_done((size_t)w, nullptr) {}
    const int W;
    const bool async;
    const int timeout_s;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;  // a rank timed out or aborted: every later barrier fails at once
    std::string why;      // ... and why
    std::vector<const void *> send;
    std::vector<void *> recv;
    // async: rank q's events -- its send buffer is produced (recorded on its
    // stream before the collective's first barrier), its copies out of the
    // peers' buffers are done (before the second)
    std::vector<hipEvent_t> ev_send, ev_done;
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
        for (hipEvent_t e : {g_->ev_send[(size_t)rank_], g_->ev_done[(size_t)rank_]})
            if (e) (void)hipEventDestroy(e);
        if (g_->refs.fetch_sub(1) == 1) delete g_;
    }
    int world() const override { return g_->W; }
    int rank() const override { return rank_; }
    const char *kind() const override { return "loopback"; }
    void abort(const std::string &why) override { g_->abort("rank " + std::to_string(rank_) + ": " + why); }

    bool all_reduce_i64(int64_t *d, size_t n, bool max, hipStream_t s, std::string &err) override {
        // load-time agreement on host values: always synchronous
        const int W = g_->W;
        if (!publish_sync(d, d, s, err)) return false;
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
            ok = after(q, s, err) && hip_ok(hipMemcpyAsync(dst, g_->send[(size_t)q], bytes, hipMemcpyDeviceToDevice, s),
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
            ok = after(q, s, err) &&
                 hip_ok(hipMemcpyAsync(static_cast<char *>(buf) + at, static_cast<const char *>(g_->send[(size_t)q]) + at,
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
            ok = after(q, s, err) &&
                 hip_ok(hipMemcpyAsync(static_cast<char *>(recv) + (size_t)q * bytes,
                                       static_cast<const char *>(g_->send[(size_t)q]) + (size_t)rank_ * bytes, bytes,
                                       hipMemcpyDeviceToDevice, s),
                        "loopback all_to_all", err);
        return finish(ok, s, err);
    }

private:
    bool events(std::string &err) {
        for (hipEvent_t *e : {&g_->ev_send[(size_t)rank_], &g_->ev_done[(size_t)rank_]})
            if (!*e && !hip_ok(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate", err)) return false;
        return true;
    }
    // sync: this rank's buffers are complete (stream drained) and visible
    // to the peers once every rank has passed the barrier
    bool publish_sync(const void *send, void *recv, hipStream_t s, std::string &err) {
        if (!hip_ok(hipStreamSynchronize(s), "loopback collective", err)) return false;
        g_->send[(size_t)rank_] = send;
        g_->recv[(size_t)rank_] = recv;
        return g_->barrier(err);
    }
    // async: the buffers are published with the event that marks them
    // produced on this rank's stream; nothing waits for the GPU here
    bool publish(const void *send, void *recv, hipStream_t s, std::string &err) {
        if (!g_->async) return publish_sync(send, recv, s, err);
        if (!events(err) ||
            !hip_ok(hipEventRecord(g_->ev_send[(size_t)rank_], s), "loopback collective (record)", err))
            return false;
        g_->send[(size_t)rank_] = send;
        g_->recv[(size_t)rank_] = recv;
        return g_->barrier(err);
    }
    // async: this stream's copies out of rank q's buffer start after q produced it
    bool after(int q, hipStream_t s, std::string &err) {
        if (!g_->async || q == rank_) return true;
        return hip_ok(hipStreamWaitEvent(s, g_->ev_send[(size_t)q], 0), "loopback collective (wait)", err);
    }
    // The copies out of the peers' buffers are done before any rank reuses
    // its send buffer: sync -- both streams drained behind a barrier; async
    // -- every rank's stream waits on every copier's event
    bool finish(bool ok, hipStream_t s, std::string &err) {
        if (!g_->async) {
            ok = ok && hip_ok(hipStreamSynchronize(s), "loopback collective", err);
            std::string berr;
            const bool b = g_->barrier(berr);
            if (ok && !b) err = berr;
            return ok && b;
        }
        ok = ok && hip_ok(hipEventRecord(g_->ev_done[(size_t)rank_], s), "loopback collective (record)", err);
        std::string berr;
        const bool b = g_->barrier(berr);
        if (ok && !b) err = berr;
        ok = ok && b;
        for (int q = 0; q < g_->W && ok; ++q)
            if (q != rank_)
                ok = hip_ok(hipStreamWaitEvent(s, g_->ev_done[(size_t)q], 0), "loopback collective (wait)", err);
        return ok;
    }

    LoopGroup *g_;
    int rank_;
};

}  // namespace

LoopGroup *make_loop_group(int world, bool async) { return new LoopGroup(world, async); }

Comm *make_loopback_comm(LoopGroup *g, int rank) { return new LoopbackComm(g, rank); }

}  // namespace dlr
