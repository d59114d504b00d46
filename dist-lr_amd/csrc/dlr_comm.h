// dlr_comm.h -- the exchange transport of one rank (internal, not ABI).
//
// Replaces ps-lite's KVWorker::Push/Pull + Postoffice::Barrier
// (src/lr.cc:116-132, src/main.cc:150) for the data-parallel exchange.
// Two transports behind one interface, both driving the SAME engine code
// (key-range all-to-all, rank-ordered merge, in-place all-gather, touched
// lists):
//   * RcclComm     -- RCCL over xGMI, one process (or thread) per GPU: the
//                     product path;
//   * LoopbackComm -- W contexts of ONE process on ONE device linked by an
//                     in-process group: device-to-device copies between the
//                     contexts' buffers behind host barriers.  RCCL refuses
//                     two ranks on one device, so this is what runs the
//                     world > 1 engine path on a single GPU (tests, and
//                     bin/distlr's DISTLR_TOPOLOGY=group).
// Every call is collective: all ranks call it in the same order.  Buffers
// are device pointers; `words` counts 4-byte words (floats / uint32) per
// rank (all_gather) or per peer (all_to_all).  On failure the call returns
// false and sets err.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <string>

#include "dlr_exchange.h"

namespace dlr {

class Comm {
public:
    virtual ~Comm() = default;
    virtual int world() const = 0;
    virtual int rank() const = 0;
    virtual const char *kind() const = 0;
    // In-place all-reduce of n int64 (max or sum).
    virtual bool all_reduce_i64(int64_t *d, size_t n, bool max, hipStream_t s, std::string &err) = 0;
    // recv[q * words ..] = rank q's send[0 .. words); send may alias
    // recv + rank * words (in place).
    virtual bool all_gather(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) = 0;
    // recv[q * words ..] = rank q's send[rank * words ..).
    virtual bool all_to_all(const void *send, void *recv, size_t words, hipStream_t s, std::string &err) = 0;
    // One piece of an in-place all-gather whose rank blocks are `chunk`
    // words apart: buf[q * chunk + off, + count) = rank q's same words, for
    // every rank q (the caller's own block is already in place).  Pieces of
    // one gather may be issued one after another so that work on the pieces
    // that have landed overlaps the rest (the exchange / next-margin overlap).
    virtual bool all_gather_part(void *buf, size_t chunk, size_t off, size_t count, hipStream_t s,
                                 std::string &err) = 0;
    // A rank that will not reach its next collective (it failed) releases
    // its peers: their pending and later collectives fail with `why`
    // instead of waiting (loopback).  RCCL: callable from any thread (the
    // in-process topology of bin/distlr aborts every rank's communicator
    // from the failing rank's thread): it only flags the communicator; the
    // thread that drives it aborts it (ncclCommAbort) at its next
    // collective or stream wait (wait below), which also makes its
    // stuck collective kernels exit.
    virtual void abort(const std::string &why) = 0;
    // Waits for stream s (the engine's waits on streams that carry this
    // transport's collectives).  RCCL: polls, and aborts the communicator
    // when abort() was called -- a plain hipStreamSynchronize would never
    // return behind a collective whose peer died.
    virtual bool wait(hipStream_t s, std::string &err) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e == hipSuccess) return true;
        err = std::string("hipStreamSynchronize: ") + hipGetErrorString(e);
        return false;
    }
};

// One collective of a step's plan (dlr_exchange.h exchange_plan) on a
// transport -- how dlr_train_step and dlr_rccl_trace issue every step
// collective: ALL_TO_ALL send -> recv (op.words per peer); ALL_GATHER send
// (op.words) -> recv; ALL_GATHER_PART in place on recv (rank blocks op.words
// apart, op.count words at op.off of each).
bool issue(Comm &comm, const CollOp &op, const void *send, void *recv, hipStream_t s, std::string &err);

// RCCL communicator for rank `rank` of `world` (unique_id: the 128-byte
// ncclUniqueId from rank 0; ignored and generated locally when world == 1).
Comm *make_rccl_comm(int world, int rank, const void *unique_id, std::string &err);

// TEST ONLY: rank `rank` of a `world`-rank RCCL transport with no
// communicator, whose every RCCL call is appended to *log as a line instead
// (dlr_rccl_trace).  No GPU, no RCCL initialisation.
Comm *make_rccl_recorder(int world, int rank, std::string *log);

// ncclGetUniqueId into out (DLR_UNIQUE_ID_BYTES).
bool rccl_unique_id(void *out, std::string &err);

// In-process group of `world` loopback ranks; make_loopback_comm(g, r) is
// rank r's endpoint.  The group is reference-counted by its endpoints.
// async (default; DLR_LOOPBACK_SYNC=1 turns it off): the data collectives
// are STREAM-ORDERED like RCCL's -- a rank's copies out of a peer's buffer
// wait on the event the peer recorded after producing it, and the peer's
// stream waits on the copiers' events before it may overwrite it; the host
// threads meet only to exchange buffers and events (they never wait for
// GPU work), so a rank's next kernels queue up behind the collective as
// they would over RCCL.  sync: every collective drains both streams behind
// host barriers.
struct LoopGroup;
LoopGroup *make_loop_group(int world, bool async);
Comm *make_loopback_comm(LoopGroup *g, int rank);

}  // namespace dlr
