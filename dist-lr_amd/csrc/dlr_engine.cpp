// dlr_engine.cpp -- device engine of libdistlr_amd: one context per GPU/rank.
//
// Replaces, for the LR hot path:
//   LR::Train / PullWeight_ / PushGradient_   src/lr.cc:28-45, 116-132
//   KVStoreDistServer::DataHandle             src/main.cc:41-96
//   DataIter per-epoch re-parse + copies      include/data_iter.h:16-55, main.cc:158-159
// Weights stay resident and replicated; with world > 1 each rank serves one
// key range: all-to-all of the pushed gradients (rank r receives every
// rank's slice of its range), rank-ordered merge + SGD on the range, then
// an in-place all-gather of the updated weights (the "pull").
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <numeric>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "dlr_comm.h"
#include "dlr_exchange.h"
#include "dlr_internal.h"
#include "dlr_kernels.h"

namespace {

constexpr int kTimers = 5;  // 0 margin, 1 gradient, 2 update, 3 exchange, 4 step
constexpr int kXPiecesMax = 16;  // pieces of the overlapped all-gather (exchange_overlapped), at most
constexpr int64_t kPad = 64;  // padding entries after col/val (16-B tail loads)

struct DeviceBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// One array of a STREAMED sparse shard (DLR_RESIDENCY_STREAM: the shard and
// its column-major copies stay in page-locked host memory; each batch's
// slice of every array is copied into one of two device slots on the copy
// stream).  beg/end: the batch's element range; pad: elements copied past
// it (the kernels' padded tail loads).  Before batch b runs, the shard's
// pointer field is bound to slot - beg[b] (element-wise), so the views the
// kernels get (field + the batch's own offset) land in the slot.
struct StreamArr {
    void **field = nullptr;
    size_t es = 0, pad = 0;
    std::vector<int64_t> beg, end;
    std::shared_ptr<void> keep;  // the host array, page-locked
    const char *host = nullptr;
    bool registered = false;
    void *slot[2] = {nullptr, nullptr};
    size_t cap = 0;  // elements per slot
};

struct TrainShard {
    bool loaded = false;
    // every value is 1.0f (one-hot / binary features): no value arrays are
    // stored and the kernels' UNIT variants run (dlr_kernels.h DevBatch)
    bool unit = false;
    int64_t n_rows = 0, nnz = 0, B = 0;
    std::vector<dlr::BatchSpan> plan;
    // shard CSR
    int64_t *row_ptr = nullptr;
    int32_t *col = nullptr;
    float *val = nullptr;
    float *label = nullptr;
    // materialised wrap batch (rows (start+i) mod N)
    int64_t wrap_batch = -1;
    int64_t *w_row_ptr = nullptr;
    int32_t *w_col = nullptr;
    float *w_val = nullptr;
    float *w_label = nullptr;
    // per-batch column-major copy: phase-split for the LDS gradient kernel
    // (pcsc) when every batch qualifies, else the classic layout
    bool pcsc = false;
    int phases = 1;
    int64_t pblocks = 0;          // groups * phases
    uint32_t *pbase = nullptr;    // n_batches x (pblocks + 1)
    uint8_t *pends = nullptr;     // n_batches x pblocks x 64
    uint16_t *prow = nullptr;     // entries (batch-relative offsets poff)
    float *pval = nullptr;
    std::vector<int64_t> poff;    // entry offset of each batch (+ total)
    // streamed shards: only the block bases are streamed; the batch's ends /
    // rows / values are built on the device from its CSR before its gradient
    // (dlr_kernels.h launch_pcsc_build) into these one-batch buffers
    bool gpu_pcsc = false;
    int64_t pR = 0;
    uint8_t *gends = nullptr;
    uint16_t *grow = nullptr;
    float *gval = nullptr;
    uint32_t *gscratch = nullptr;
    // product margin (pcsc batches; dlr_kernels.h DevPm): batch b's slice
    // list offsets at b*(pmS+1) of pm_lbeg, its list/values at pmo_list[b],
    // chunk offsets at pmo_pofs[b], regions and slot-list offsets at pmo_rg[b]
    // (rg, qoff), slot lists at pmo_qs[b]; pm_p holds one batch's products.
    // pm_fused: the fused k_grad_lds forms the next batch's products.
    // pm_mg: (one rank, pm_fused) the fused k_grad_lds also runs this
    // batch's pass 2 (DevP2): pm_cnt its hand-off counters, pm_gen the
    // launches so far.
    bool pm = false, pm_fused = false, pm_mg = false;
    // the one-launch step (pm_mg) or K6r (dref) would have been used, but
    // this context's in-launch wait ran out before (dlr_ctx::mg_demoted)
    bool mg_demoted = false;
    // band mode (classic layout, batches of >= 2^21 rows: C2 at B = -1): the
    // margin as the product margin over WINDOWS of kPmWinRows rows (pass 1 +
    // pass 2 per window; the weights do not change inside the step); the
    // DevPm arrays are the windows', window w of batch b at index
    // pmw_first[b] + w
    // pmw_views: every window's DevPm (device memory, for the multi-window
    // launches); pm_p then holds pmw_slots windows' products, pm_pstride
    // floats apart (a band's windows: one pass-1 and one pass-2 launch)
    bool pmw = false;
    std::vector<int64_t> pmw_first;
    dlr::DevPm *pmw_views = nullptr;
    int64_t pmw_slots = 1, pm_pstride = 0;
    uint32_t *pm_cnt = nullptr;
    uint32_t pm_gen = 0;
    int64_t pmS = 0;
    int pm_groups = 0, pm_split = 1;
    uint32_t *pm_lbeg = nullptr, *pm_list = nullptr, *pm_pofs = nullptr, *pm_rg = nullptr, *pm_qoff = nullptr;
    float *pm_val = nullptr, *pm_p = nullptr;
    uint16_t *pm_qs = nullptr;
    std::vector<int64_t> pmo_list, pmo_pofs, pmo_rg, pmo_qs;
    std::vector<uint32_t> pm_rstride, pm_qstride;  // per span (DevPm)
    // row-round gradient (dlr_kernels.h DevRt) of every product-margin batch:
    // gq / val at rtoff[b] (pmS * rt_rounds * rt_cap[b] entries), cend at
    // b*pmS*kPmSlice; rt_rounds rounds per batch
    bool rt = false;
    int rt_rounds = 0;
    uint32_t *rt_gq = nullptr;
    float *rt_val = nullptr;
    uint16_t *rt_cend = nullptr;
    std::vector<int64_t> rtoff;
    std::vector<uint32_t> rt_cap;
    // world > 1: the exchange / next-margin overlap (dlr_train_step).  The
    // in-place all-gather of the updated weights runs in xpieces pieces on
    // the exchange stream; after piece k the next batch's pass 1 forms the
    // slices whose weights have all landed.  xslices: slice ids grouped by
    // the piece that completes them (group 0: inside this rank's own key
    // range, ready after the merge; group k + 1: after piece k), group g at
    // [xgofs[g], xgofs[g + 1]).
    uint32_t *xslices = nullptr;
    std::vector<int64_t> xgofs;
    int64_t xsub = 0;  // words per piece of a rank's key range
    int xpieces = 1;   // pieces (dlr_set_exchange_pieces at load, agreed over the ranks)
    bool xauto = true; // the piece count was left to auto_pieces
    // touched-column layout (huge D, small batches): per batch the touched
    // columns tcols[tcoff[b] .. +tncols[b]), segment pointers in cptr at
    // tpoff[b] (tncols[b]+1 entries), entries at coff[b] in crow/cval
    bool touched = false;
    uint32_t *tcols = nullptr;
    std::vector<int64_t> tcoff, tncols, tpoff;
    int64_t tcap = 0;           // max touched columns of a batch (all ranks)
    // long columns of the classic layout (per batch: lcoff cols, lsoff
    // segments, leoff entries; cseg/sptr have one extra entry per batch)
    bool any_long = false;
    uint32_t *lsched = nullptr;  // long chunks by first row (lsoff offsets, one pad entry per batch)
    uint32_t *lcols = nullptr, *lcseg = nullptr, *lsptr = nullptr;
    void *lrow = nullptr;
    float *lval = nullptr, *lpart = nullptr;
    std::vector<int64_t> lcoff, lsoff, leoff;
    // dense shard (dlr_load_train_dense): X row-major n_rows x D
    bool dense = false, dblocked = false, dfused = false;
    float *dX = nullptr, *dpart = nullptr;
    bool dtiled = false;  // dX is K6r's tiled image (dense_ref_tiled_floats), not row-major
    // reference order, large batches: the banded one-launch step (K6r,
    // k_dense_ref) and its hand-off words (dlr_kernels.h DevRefSync)
    bool dref = false;
    uint32_t *dref_sync = nullptr;
    uint32_t dref_seq = 0;
    int dref_lead = 0;
    // streamed dense shard (DLR_RESIDENCY_STREAM): X stays in the caller's
    // host memory (registered, pinned in place); each batch's rows and labels
    // are staged into one of two device slots on the copy stream
    bool streamed = false, host_registered = false;
    const float *hX = nullptr;
    float *sx[2] = {nullptr, nullptr}, *sl[2] = {nullptr, nullptr};
    int64_t sb[2] = {-1, -1};  // batch held by each slot (dense or sparse streaming)
    // streamed sparse shard: every per-batch array (StreamArr)
    bool sparse_stream = false;
    std::vector<StreamArr> sarr;
    // coalesced staging of a streamed sparse shard: batch b's slices of
    // every streamed array packed back to back (256-B aligned) in one
    // page-locked buffer at sboff[b] (sbsz[b] bytes), array a of batch b at
    // soff[b * sarr.size() + a] -- one H2D copy per batch into sslot[0|1]
    char *shost = nullptr;
    std::vector<size_t> sboff, sbsz, soff;
    void *sslot[2] = {nullptr, nullptr};
    bool row16 = false;
    uint32_t *cptr = nullptr;   // n_batches x (D+1)
    void *crow = nullptr;
    float *cval = nullptr;
    std::vector<int64_t> coff;  // entry offset of each batch
    // classic layout: entry-balanced wave schedules (DevCsc::wstart), per batch
    // wsoff[b] .. wsoff[b+1]-1 in wsched (column starts, then D)
    uint32_t *wsched = nullptr;
    std::vector<int64_t> wsoff;
    // row-band layout of the classic copy's short columns (large batches,
    // dlr_kernels.hip "Row-band layout"): band_shift > 0 replaces
    // cptr/crow/cval/wsched; band k of batch b is bands[bfirst[b] + k]
    struct Band {
        int64_t pair, ptr, ent, ws, nwaves;  // offsets into bcols, bptr, brow/bval, bws
        int64_t hw = 0, nhot = 0;            // the band's hot waves (k_band_hot): bhw[hw .. hw + nhot)
    };
    int64_t max_hot = 0;  // the most hot waves of a band (CUs the pipelined margin leaves them)
    // hot-column product stream (band mode, REFERENCE; dlr_kernels.h
    // DevHotOut / DevHotChain): per batch b, its hot columns hs_cols[hsco[b]
    // .. + hs_nh[b]), their (start, count) per band hs_seg[hsso[b] ..], the
    // per-row hot entry lists hs_off[hsoo[b] ..] (B_b + 1, absolute into
    // hs_dest / hs_val); one stream buffer and per-band flags for the shard
    bool hs = false;
    std::vector<int64_t> hs_nh, hsco, hsso, hsoo;
    uint32_t *hs_cols = nullptr, *hs_off = nullptr, *hs_dest = nullptr, *hs_flag = nullptr;
    uint2 *hs_seg = nullptr, *hs_state = nullptr;
    float *hs_val = nullptr, *hs_buf = nullptr;
    uint32_t hs_seq = 0;
    int64_t hs_bytes = 0;
    int band_shift = 0;
    bool band_longrun = false;  // band mode without the long-column split: runs of 10^5 entries in a band
    // margin with the hot (lowest, frequency-ordered) weights in LDS
    bool margin_hot = false;
    std::vector<Band> bands;
    std::vector<int64_t> bfirst;
    uint32_t *bcols = nullptr, *bptr = nullptr, *bws = nullptr, *bhw = nullptr;
    void *brow = nullptr;
    float *bval = nullptr;
    float *gacc = nullptr;  // D running column sums
    // band mode: long columns in row phases (dlr_kernels.h DevLPhase); batch
    // b's phases are lpdesc[b * lnph ..], its columns lcols/lcseg as above
    int64_t lnph = 0;
    dlr::PhaseDesc *lpdesc = nullptr;
    int64_t lnpart = 0;
    uint32_t *lpptr = nullptr, *lpslot = nullptr, *lpws = nullptr;
    uint16_t *lprow = nullptr;
    float *lpval = nullptr;
    // some sum of this shard is reordered (DLR_ORDER_FAST actually applied:
    // long columns, blocked / fused dense gradients); dlr_summation_order
    bool fast = false;
    // world > 1: the pieced all-gather overlapped with the next batch's pass 1
    // (exchange_overlapped), AGREED over the ranks at load / by the
    // collective dlr_set_exchange_overlap -- the two forms are different
    // collective sequences
    bool xpieced = false;
    int64_t bytes = 0;
};

// What the column-major builders read of a CSR shard (the caller's arrays,
// or the same rows with relabeled columns).
struct CsrView {
    int64_t n_rows;
    const int64_t *row_ptr;
    const int32_t *col;
    const float *val;
};

struct TestShard {
    bool loaded = false;
    bool dense = false;
    float *dX = nullptr;
    int64_t n_rows = 0, nnz = 0;
    int64_t *row_ptr = nullptr;
    int32_t *col = nullptr;
    float *val = nullptr;  // null: unit values (TrainShard::unit)
    float *label = nullptr;
    int grid = 0;
    int64_t bytes = 0;
};

}  // namespace

struct dlr_ctx {
    int device = 0, rank = 0, world = 1;
    int64_t D = 0, chunk = 0, Dpad = 0;
    hipStream_t stream = nullptr;
    dlr::Comm *comm = nullptr;  // exchange transport (RCCL, or an in-process loopback group); null: none
    float *w = nullptr;      // Dpad (replicated weights)
    float *g = nullptr;      // Dpad (this rank's pushed gradient), world > 1
    float *recv = nullptr;   // world x chunk, world > 1
    float *resid = nullptr;  // max batch rows
    int64_t resid_cap = 0;
    unsigned long long *correct = nullptr;
    double *ll = nullptr;       // [0] total, [1..] partials
    int64_t ll_cap = 0;
    unsigned long long *h_correct = nullptr;  // pinned
    double *h_ll = nullptr;                   // pinned
    // in-launch hand-off errors (dlr_kernels.h DevErr): kErrWords words of
    // host-mapped memory the kernels store to when a bounded wait runs out
    // (h_err: host view, d_err: device view); checked by check_device
    uint32_t *h_err = nullptr, *d_err = nullptr;
    // ... followed by kStatWords event counters the kernels add to (DevStat;
    // d_stat = d_err + kErrWords), and the host's own (dlr_stage_counters)
    uint32_t *d_stat = nullptr;
    int64_t hcount[DLR_COUNTERS] = {};
    int fault = dlr::kFaultNone;  // dlr_set_fault (tests; cleared by every load)
    // the loads' tuning (dlr_tuning): set by dlr_set_tuning, else taken from
    // the environment at each load (load_tuning)
    dlr_tuning tune{};
    bool tune_set = false;
    // an in-launch wait of this context's one-launch step (kErrMgPublish) or
    // K6r (kErrRef*) ran out: the device did not hold the whole grid (another
    // process's work, CowaitScope) -- later loads use the separate launches
    bool mg_demoted = false, dref_demoted = false;
    TrainShard train;
    TestShard test;
    // exchange / next-margin overlap (TrainShard::xslices): asked for unless
    // dlr_set_exchange_overlap(0) (the loaded shard's agreed form:
    // TrainShard::xpieced); its stream and events
    bool xoverlap = true;
    // summation order of the next loaded training shard (DLR_ORDER_*)
    int order = DLR_ORDER_REFERENCE;
    hipStream_t xstream = nullptr;
    hipEvent_t ev_xmerged = nullptr;
    hipEvent_t ev_xpiece[kXPiecesMax] = {};
    // pieces of the next loaded shard's overlapped all-gather (0: auto,
    // auto_pieces)
    int xpieces = 0;
    // product margin: the batch whose products pm_p holds, formed from the
    // CURRENT weights by the last step's fused gradient (-1: none; every
    // entry point that changes w or the shard resets it)
    int64_t pm_ready = -1;
    // touched-layout step buffers: newv (world 1: new weights of the touched
    // columns); sparse exchange (world > 1): send block [count|cols|g],
    // all-gathered blocks, merged (col, new weight) per entry
    float *newv = nullptr;
    uint32_t *xsend = nullptr, *xrecv = nullptr, *xcols = nullptr;
    float *xnewv = nullptr;
    int64_t xcap = 0;
    dlr::RankSizes rs{};
    // residency of the next dense training shard, and the streamed shard's
    // copy stream + slot events (created on first use)
    // column relabeling of Zipf-skewed sparse shards: perm[j] = the internal
    // id of column j (frequency order); empty = identity.  Device weights,
    // gradients and shard columns are internal; every D-length host boundary
    // (weights, pushed gradients) and the test shard's columns are mapped.
    std::vector<int32_t> perm;
    int residency = DLR_RESIDENCY_AUTO;
    hipStream_t cstream = nullptr;
    // band mode, pipelined (band_step_pipelined): the bands' gradient stream,
    // one event per band's margins, the step start and the bands' end
    hipStream_t gstream = nullptr;
    std::vector<hipEvent_t> ev_band;
    hipEvent_t ev_bstart = nullptr, ev_bdone = nullptr;
    // ... and the hot pairs' stream (k_band_hot, band after band)
    hipStream_t hstream = nullptr;
    hipEvent_t ev_hdone = nullptr;
    hipEvent_t ev_hmargins = nullptr;  // after a step's last margin (the final hot-chain launch waits on it)
    hipEvent_t ev_ready[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
    std::vector<void *> allocs;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_pending;
    size_t ev_next = 0;
    double t_ms[kTimers] = {0};
    int64_t t_n[kTimers] = {0};
    std::string err;
};

namespace {

int fail(dlr_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    dlr::set_error(msg);
    return code;
}

#define HIPC(c, expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return fail((c), DLR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));             \
    } while (0)

// A collective of the context's transport (dlr_comm.h); bool result.
// One collective of the step's plan (dlr::issue)
#define XCHGC(c, op, send, recv, s)                                                                       \
    do {                                                                                                  \
        std::string e_;                                                                                   \
        if (!dlr::issue(*(c)->comm, *(op), (send), (recv), (s), e_))                                      \
            return fail((c), DLR_E_RCCL, std::string((c)->comm->kind()) + " " + e_);                      \
    } while (0)
#define COMMC(c, expr)                                                                                  \
    do {                                                                                                \
        std::string e_;                                                                                 \
        if (!(c)->comm->expr) return fail((c), DLR_E_RCCL, std::string((c)->comm->kind()) + " " + e_);  \
    } while (0)

// Waits for a stream that may carry this rank's collectives: through the
// transport (an aborted RCCL communicator makes its stuck kernels return
// instead of blocking here forever, dlr_comm.h), else hipStreamSynchronize.
int wait_stream(dlr_ctx *c, hipStream_t s, const char *who) {
    if (!c->comm) {
        HIPC(c, hipStreamSynchronize(s));
        return DLR_OK;
    }
    std::string err;
    if (!c->comm->wait(s, err)) return fail(c, DLR_E_RCCL, std::string(who) + ": " + err);
    return DLR_OK;
}

// The hand-off errors the context's kernels have recorded (sticky until the
// next load): a bounded wait inside a launch ran out, so the launch computed
// on data that never arrived -- the step fails instead of returning weights
// (lr.cc:122, 131: the reference's worker waits until its data is there).
// Reads host memory only: the caller has synchronized for a definitive
// answer, or (dlr_train_step) sees what earlier steps recorded.
int check_device(dlr_ctx *c, const char *who) {
    if (!c->h_err) return DLR_OK;
    static const char *what[dlr::kErrWords] = {
        "the fused margin's blocks of a phase were never all published (k_grad_lds, one-launch step)",
        "a chain slot's margin units were never published (k_dense_ref)",
        "the column chains' limit never reached a margin unit (k_dense_ref)",
        "a hand-off between the waves of a workgroup never came (k_dense_ref)",
        "a hand-off between the waves of a workgroup never came (k_band_hot / k_hot_chain)",
        "a band's hot-column products were never published (k_hot_chain)",
        "unknown", "unknown"};
    std::string msg;
    for (int k = 0; k < dlr::kErrWords; ++k) {
        if (__atomic_load_n(c->h_err + k, __ATOMIC_ACQUIRE) == 0u) continue;
        msg += msg.empty() ? "" : "; ";
        msg += what[k];
        if (k == dlr::kErrMgPublish) c->mg_demoted = true;
        if (k == dlr::kErrRefSlot || k == dlr::kErrRefLimit || k == dlr::kErrRefLds) c->dref_demoted = true;
    }
    if (msg.empty()) return DLR_OK;
    return fail(c, DLR_E_DEVICE, std::string(who) + ": in-launch wait ran out: " + msg +
                                     " -- the weights are not the reference's; reload the shard" +
                                     (c->mg_demoted || c->dref_demoted
                                          ? " (this context's later loads run those steps in separate launches)"
                                          : ""));
}

void clear_device_errors(dlr_ctx *c) {
    if (c->h_err)
        for (int k = 0; k < dlr::kErrWords; ++k) __atomic_store_n(c->h_err + k, 0u, __ATOMIC_RELEASE);
}

// dlr_stage_counters' counts start again with each loaded shard
void clear_counters(dlr_ctx *c) {
    if (c->h_err)
        for (int k = 0; k < dlr::kStatWords; ++k) __atomic_store_n(c->h_err + dlr::kErrWords + k, 0u, __ATOMIC_RELEASE);
    for (int64_t &v : c->hcount) v = 0;
}

// CO-WAITING LAUNCHES.  The one-launch step (k_grad_lds / k_grad_rt MG),
// K6r (k_dense_ref) and the hot chains (k_hot_chain beside their band's
// margins) have workgroups that wait INSIDE the GPU for data other
// workgroups produce; they are sized to what the device holds at once
// (resident_grid).  Two such grids from different streams -- two contexts
// in one process (loopback ranks, engines on threads), or one context's
// streams -- could each hold part of the CUs and wait for the rest.  So
// every co-waiting launch (or launch sequence) of this process is queued
// after the previous one of ANOTHER stream: under a process-wide lock, the
// stream waits on an event recorded on that stream, and the lock is held
// until the sequence is queued.  A context that keeps to one stream adds no
// API call (the common case: one engine per process).  Other PROCESSES are
// not covered: their launches are bounded by the in-launch waits (250 ms,
// DLR_E_DEVICE), after which this context stops using the one-launch step
// (mg_demoted).
struct CowaitOrder {
    std::mutex mu;
    hipStream_t last[64] = {};  // per device: the stream of the last co-waiting sequence
    hipEvent_t ev[64] = {};
};
CowaitOrder &cowait_order() {
    static CowaitOrder *o = new CowaitOrder;  // (never destroyed: contexts may outlive static destructors)
    return *o;
}

class CowaitScope {
  public:
    CowaitScope(dlr_ctx *c, hipStream_t s) : c_(c), s_(s), lk_(cowait_order().mu) {}
    CowaitScope(const CowaitScope &) = delete;
    CowaitScope &operator=(const CowaitScope &) = delete;
    // order s after the last co-waiting sequence of another stream
    hipError_t begin() {
        CowaitOrder &o = cowait_order();
        const int d = c_->device;
        if (d < 0 || d >= 64) return hipErrorInvalidDevice;
        if (o.last[d] && o.last[d] != s_) {
            if (!o.ev[d]) {
                const hipError_t e = hipEventCreateWithFlags(&o.ev[d], hipEventDisableTiming);
                if (e != hipSuccess) return e;
            }
            hipError_t e = hipEventRecord(o.ev[d], o.last[d]);
            if (e == hipSuccess) e = hipStreamWaitEvent(s_, o.ev[d], 0);
            if (e != hipSuccess) return e;
            ++c_->hcount[DLR_COUNT_COWAIT_SERIALISED];
        }
        o.last[d] = s_;
        return hipSuccess;
    }

  private:
    dlr_ctx *c_;
    hipStream_t s_;
    std::lock_guard<std::mutex> lk_;
};

// a destroyed stream is no longer anyone's predecessor
void cowait_forget(dlr_ctx *c) {
    CowaitOrder &o = cowait_order();
    std::lock_guard<std::mutex> lk(o.mu);
    if (c->device < 0 || c->device >= 64) return;
    hipStream_t &l = o.last[c->device];
    if (l && (l == c->stream || l == c->hstream || l == c->gstream)) l = nullptr;
}

// The tuning a load uses (dlr_tuning): the context's own, or the
// environment's at this load.
void load_tuning(dlr_ctx *c) {
    if (!c->tune_set) dlr_tuning_from_env(&c->tune);
}
// a tuning field: its value, or `def` when DLR_AUTO
inline int64_t tv(int64_t v, int64_t def) { return v == DLR_AUTO ? def : v; }

int dev_alloc(dlr_ctx *c, void **p, size_t bytes) {
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, DLR_E_NOMEM, "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
    }
    c->allocs.push_back(*p);
    return DLR_OK;
}

void dev_free(dlr_ctx *c, void *p) {
    if (!p) return;
    auto it = std::find(c->allocs.begin(), c->allocs.end(), p);
    if (it != c->allocs.end()) c->allocs.erase(it);
    (void)hipFree(p);
}

// Every setup copy/memset is ordered on the context's own stream: it is a
// non-blocking stream, so null-stream operations (hipMemset/hipMemcpy) would
// NOT be ordered before the kernels that follow.  The copy is synchronous
// (pageable source), so `src` may be freed on return.
template <typename T>
int upload(dlr_ctx *c, T **dst, const T *src, size_t n, size_t pad = 0) {
    int rc = dev_alloc(c, (void **)dst, (n + pad) * sizeof(T));
    if (rc) return rc;
    if (n) HIPC(c, hipMemcpyAsync(*dst, src, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    if (pad) HIPC(c, hipMemsetAsync(*dst + n, 0, pad * sizeof(T), c->stream));
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    return DLR_OK;
}

// A shard array: uploaded (resident), or -- for a streamed sparse shard --
// kept page-locked in host memory with its per-batch element ranges
// rng(b) = [beg, end) and two device slots (StreamArr).  The host copy is
// made here, so src may be freed on return.
using RangeFn = std::function<std::pair<int64_t, int64_t>(int64_t)>;
template <typename T>
int place(dlr_ctx *c, T **field, const T *src, size_t n, size_t pad, const RangeFn &rng);

void free_train(dlr_ctx *c) {
    TrainShard &t = c->train;
    // a reload frees what the last steps' kernels and copies may still read
    // (hipFree alone is not relied on to order them)
    for (hipStream_t s : {c->stream, c->cstream, c->gstream, c->hstream, c->xstream})
        if (s) (void)hipStreamSynchronize(s);
    if (t.sparse_stream) {
        if (c->cstream) (void)hipStreamSynchronize(c->cstream);
        for (StreamArr &a : t.sarr) {
            if (a.registered) (void)hipHostUnregister(const_cast<char *>(a.host));
            dev_free(c, a.slot[0]);
            dev_free(c, a.slot[1]);
            *a.field = nullptr;  // the bound view pointed into a slot
        }
        if (t.shost) (void)hipHostFree(t.shost);
        dev_free(c, t.sslot[0]);
        dev_free(c, t.sslot[1]);
    }
    if (t.streamed) {
        if (c->cstream) (void)hipStreamSynchronize(c->cstream);
        if (t.host_registered) (void)hipHostUnregister(const_cast<float *>(t.hX));
        for (void *p : {(void *)t.sx[0], (void *)t.sx[1], (void *)t.sl[0], (void *)t.sl[1]}) dev_free(c, p);
    }
    for (void *p : {(void *)t.row_ptr, (void *)t.col, (void *)t.val, (void *)t.label, (void *)t.w_row_ptr,
                    (void *)t.w_col, (void *)t.w_val, (void *)t.w_label, (void *)t.cptr, t.crow, (void *)t.cval,
                    (void *)t.pbase, (void *)t.pends, (void *)t.prow, (void *)t.pval, (void *)t.gends, (void *)t.grow,
                    (void *)t.gval, (void *)t.gscratch, (void *)t.tcols,
                    (void *)t.lcols, (void *)t.lcseg, (void *)t.lsptr, t.lrow, (void *)t.lval, (void *)t.lpart, (void *)t.lsched,
                    (void *)t.dX, (void *)t.dpart, (void *)t.wsched, (void *)t.bcols, (void *)t.bptr,
                    (void *)t.bws, (void *)t.bhw, (void *)t.hs_cols, (void *)t.hs_off, (void *)t.hs_dest,
                    (void *)t.hs_flag, (void *)t.hs_seg, (void *)t.hs_state, (void *)t.hs_val, (void *)t.hs_buf, t.brow, (void *)t.bval, (void *)t.gacc, (void *)t.lpdesc, (void *)t.lpptr,
                    (void *)t.lpslot, (void *)t.lpws, (void *)t.lprow, (void *)t.lpval, (void *)t.pm_lbeg,
                    (void *)t.pm_list, (void *)t.pm_pofs, (void *)t.pm_rg, (void *)t.pm_qoff, (void *)t.pm_val,
                    (void *)t.pm_p, (void *)t.pm_qs, (void *)t.xslices, (void *)t.rt_gq, (void *)t.rt_val,
                    (void *)t.rt_cend, (void *)t.dref_sync, (void *)t.pm_cnt, (void *)t.pmw_views})
        dev_free(c, p);
    t = TrainShard();
    c->pm_ready = -1;
    c->fault = dlr::kFaultNone;  // (test knob: one shard at most)
    clear_device_errors(c);      // nothing of the old shard runs any more
    clear_counters(c);
}

template <typename T>
int place(dlr_ctx *c, T **field, const T *src, size_t n, size_t pad, const RangeFn &rng) {
    TrainShard &t = c->train;
    if (!t.sparse_stream) return upload(c, field, src, n, pad);
    const int64_t nb = (int64_t)t.plan.size();
    StreamArr a;
    a.field = reinterpret_cast<void **>(field);
    a.es = sizeof(T);
    a.pad = pad;
    a.beg.resize((size_t)nb);
    a.end.resize((size_t)nb);
    size_t cap = 1;
    for (int64_t b = 0; b < nb; ++b) {
        const std::pair<int64_t, int64_t> r = rng(b);
        a.beg[(size_t)b] = r.first;
        a.end[(size_t)b] = std::max(r.first, r.second);
        if (a.end[(size_t)b] > a.beg[(size_t)b]) cap = std::max(cap, (size_t)(a.end[(size_t)b] - a.beg[(size_t)b]) + pad);
    }
    auto *hv = new std::vector<T>(n + pad);  // zero tail: the padded reads of the last batch
    if (n) std::copy(src, src + n, hv->begin());
    a.keep = std::shared_ptr<void>(hv, [](void *p) { delete static_cast<std::vector<T> *>(p); });
    a.host = reinterpret_cast<const char *>(hv->data());
    hipError_t e = hipHostRegister(const_cast<char *>(a.host), (n + pad) * sizeof(T), hipHostRegisterDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, DLR_E_HIP, std::string("dlr_load_train: hipHostRegister (streamed shard): ") + hipGetErrorString(e));
    }
    a.registered = true;
    a.cap = cap;
    *field = nullptr;
    t.sarr.push_back(std::move(a));
    StreamArr &sa = t.sarr.back();
    for (int k = 0; k < 2; ++k) {
        const int rc = dev_alloc(c, &sa.slot[k], cap * sizeof(T));
        if (rc) return rc;
    }
    t.bytes += (int64_t)(2 * cap * sizeof(T));
    return DLR_OK;
}

void free_touched_bufs(dlr_ctx *c) {
    for (void *p : {(void *)c->newv, (void *)c->xsend, (void *)c->xrecv, (void *)c->xcols, (void *)c->xnewv})
        dev_free(c, p);
    c->newv = c->xnewv = nullptr;
    c->xsend = c->xrecv = c->xcols = nullptr;
    c->xcap = 0;
}

void free_test(dlr_ctx *c) {
    TestShard &t = c->test;
    for (void *p : {(void *)t.row_ptr, (void *)t.col, (void *)t.val, (void *)t.label, (void *)t.dX}) dev_free(c, p);
    t = TestShard();
}

// ---- timing: pairs of events around each launch, harvested on demand
void time_begin(dlr_ctx *c, hipEvent_t *a) {
    *a = nullptr;
    if (!c->timing) return;
    if (c->ev_next + 2 > c->ev_pool.size()) {
        for (int i = 0; i < 256; ++i) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return;
            c->ev_pool.push_back(e);
        }
    }
    *a = c->ev_pool[c->ev_next++];
    (void)hipEventRecord(*a, c->stream);
}

void time_end(dlr_ctx *c, int which, hipEvent_t a) {
    if (!c->timing || !a) return;
    hipEvent_t b = c->ev_pool[c->ev_next++];
    (void)hipEventRecord(b, c->stream);
    c->ev_pending.push_back({which, {a, b}});
}

void harvest(dlr_ctx *c) {
    if (c->ev_pending.empty()) return;
    (void)hipStreamSynchronize(c->stream);
    for (auto &p : c->ev_pending) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, p.second.first, p.second.second) == hipSuccess) {
            c->t_ms[p.first] += ms;
            c->t_n[p.first] += 1;
        }
    }
    c->ev_pending.clear();
    c->ev_next = 0;
}

// Load-time collectives (all ranks call dlr_load_train together): max of
// an int64 over ranks, and an all-gather of one float per rank.
// In-place max or sum of an int64 vector over the ranks (through a device
// buffer: both transports reduce device memory).
int coll_reduce_i64(dlr_ctx *c, int64_t *v, size_t n, bool max) {
    if (!c->comm || n == 0) return DLR_OK;
    int64_t *d = nullptr;
    int rc = dev_alloc(c, (void **)&d, n * 8);
    if (rc) return rc;
    std::string err;
    hipError_t e = hipMemcpyAsync(d, v, n * 8, hipMemcpyHostToDevice, c->stream);
    const bool ok = e == hipSuccess && c->comm->all_reduce_i64(d, n, max, c->stream, err);
    if (ok) e = hipMemcpyAsync(v, d, n * 8, hipMemcpyDeviceToHost, c->stream);
    // through the transport: a peer's abort ends the wait
    const int wrc = wait_stream(c, c->stream, "coll_reduce_i64");
    dev_free(c, d);
    if (wrc) return wrc;
    if (e != hipSuccess) return fail(c, DLR_E_HIP, std::string("coll_reduce_i64: ") + hipGetErrorString(e));
    if (!ok) return fail(c, DLR_E_RCCL, std::string(c->comm->kind()) + " " + err);
    return DLR_OK;
}

int coll_max_i64(dlr_ctx *c, int64_t *v) { return coll_reduce_i64(c, v, 1, true); }

// Sum of an int64 vector over the ranks, in place.
int coll_sum_i64(dlr_ctx *c, std::vector<int64_t> &v) { return coll_reduce_i64(c, v.data(), v.size(), false); }

int coll_gather_f32(dlr_ctx *c, float v, std::vector<float> &out) {
    const int W = c->comm ? c->world : 1;
    out.assign((size_t)W, v);
    if (!c->comm) return DLR_OK;
    float *d = nullptr;
    int rc = dev_alloc(c, (void **)&d, (size_t)(W + 1) * 4);
    if (rc) return rc;
    std::string err;
    hipError_t e = hipMemcpyAsync(d + W, &v, 4, hipMemcpyHostToDevice, c->stream);
    const bool ok = e == hipSuccess && c->comm->all_gather(d + W, d, 1, c->stream, err);
    if (ok) e = hipMemcpyAsync(out.data(), d, (size_t)W * 4, hipMemcpyDeviceToHost, c->stream);
    const int wrc = wait_stream(c, c->stream, "coll_gather_f32");
    dev_free(c, d);
    if (wrc) return wrc;
    if (e != hipSuccess) return fail(c, DLR_E_HIP, std::string("coll_gather_f32: ") + hipGetErrorString(e));
    if (!ok) return fail(c, DLR_E_RCCL, std::string(c->comm->kind()) + " " + err);
    return DLR_OK;
}

// Load-time agreement: every rank runs the same number of steps
// with the same collectives, so a rank whose own arguments are bad, or
// whose batch count differs from its peers', must not leave the others
// waiting in a collective.  Each rank contributes its local error flag and
// batch count; all ranks fail together.  Called by every rank exactly once
// per load, before any other load-time collective.
int coll_agree_load(dlr_ctx *c, const char *who, int local_rc, const std::string &local_msg, int64_t nb) {
    if (!c->comm) return local_rc ? fail(c, local_rc, local_msg) : DLR_OK;
    int64_t v[3] = {local_rc ? 1 : 0, nb, -nb};
    int rc = coll_reduce_i64(c, v, 3, true);
    if (rc) return rc;
    if (local_rc) return fail(c, local_rc, local_msg);
    if (v[0]) return fail(c, DLR_E_ARG, std::string(who) + ": another rank rejected its shard");
    if (v[1] != -v[2])
        return fail(c, DLR_E_ARG, std::string(who) + ": ranks have different batch counts per epoch (" +
                                      std::to_string(-v[2]) + " .. " + std::to_string(v[1]) +
                                      "); synchronous data parallelism needs equal shards (INTEGRATION.md)");
    return DLR_OK;
}

// Every rank must load with the same summation order (dlr_set_summation_order):
// a rank summing differently would hold different weights after the merge;
// and with the same exchange piece count (dlr_set_exchange_pieces): the
// pieces are collectives.
int coll_agree_order(dlr_ctx *c, const char *who) {
    int64_t v[4] = {c->order, -(int64_t)c->order, c->xpieces, -(int64_t)c->xpieces};
    int rc = coll_reduce_i64(c, v, 4, true);
    if (rc) return rc;
    if (v[0] != -v[1])
        return fail(c, DLR_E_ARG, std::string(who) + ": the ranks asked for different summation orders");
    if (v[2] != -v[3])
        return fail(c, DLR_E_ARG, std::string(who) + ": the ranks asked for different exchange piece counts");
    return DLR_OK;
}

// The pieced all-gather (exchange_overlapped) only where EVERY rank can and
// wants to run it: its RCCL send/recv groups and the plain all-gather's
// ncclAllGather would not pair up.  Collective.
int coll_agree_pieced(dlr_ctx *c) {
    TrainShard &t = c->train;
    t.xpieced = false;
    if (!c->comm) return DLR_OK;
    // auto with one piece: no overlap -- pass 1 of this rank's own range is
    // all it would hide (1/W of pass 1, under a microsecond at C2) and it
    // costs a second pass-1 launch and a cross-stream wait (the loopback
    // estimate, profiles/r05_loopback_c2_w*.json: 0.151 vs 0.122 ms per
    // step at W = 2); the plain all-gather and the next margin's pass 1
    const bool want = t.pm && c->xoverlap && !t.sparse_stream && !(t.xauto && t.xpieces == 1);
    int64_t v = want ? -1 : 0;  // max(-x) = -min(x)
    int rc = coll_max_i64(c, &v);
    if (rc) return rc;
    t.xpieced = v == -1;
    return DLR_OK;
}

// The collectives of this context's world > 1 step (dlr_exchange.h
// exchange_plan: the same on every rank), consumed in order by
// dlr_train_step -- each collective's sizes come from the plan, and a step
// that would issue another sequence fails instead of leaving the peers in
// an unmatched collective.
struct StepPlan {
    std::vector<dlr::CollOp> ops;
    size_t k = 0;
    const dlr::CollOp *next(int64_t kind) { return k < ops.size() && ops[k].kind == kind ? &ops[k++] : nullptr; }
};
StepPlan step_plan(const dlr_ctx *c) {
    const TrainShard &t = c->train;
    StepPlan p;
    p.ops = t.touched ? dlr::exchange_plan(dlr::kXTouched, c->D, c->world, 0, c->xcap)
                      : dlr::exchange_plan(dlr::kXKeyRange, c->D, c->world, t.xpieced ? t.xpieces : 0, 0);
    return p;
}
#define PLANC(c, op)                                                                                \
    do {                                                                                            \
        if (!(op)) return fail((c), DLR_E_STATE, "dlr_train_step: the exchange left its plan"); \
    } while (0)

inline int64_t pid(const std::vector<int32_t> &p, int64_t j) { return p.empty() ? j : (int64_t)p[(size_t)j]; }

// Frequency order of the columns of a sparse training shard, summed over
// the ranks (every rank gets the same numbering): internal id k = the k-th
// most frequent column (ties by id).  Returned empty (identity) unless
// DLR_RELABEL=1 forces it or (default) the counts are Zipf-skewed -- the top
// 1% of columns hold over half of the entries, as C3's hashed fields do --
// when the hot weights then share cache lines in the margin's gathers.  A
// pure renaming: every sum keeps its order, results are bitwise unchanged.
int column_order(dlr_ctx *c, const dlr_dataset &ds, std::vector<int32_t> &np) {
    np.clear();
    const int64_t mode = c->tune.relabel;  // DLR_AUTO, 0 off, 1 on
    const int64_t D = c->D;
    int64_t want = (mode == 1 || (mode < 0 && D >= 65536)) && D <= ((int64_t)1 << 25) ? 1 : 0;
    int rc;
    if ((rc = coll_max_i64(c, &want))) return rc;  // ranks agree before any collective below
    if (!want) return DLR_OK;
    std::vector<int64_t> cnt((size_t)D, 0);
    {
        const int nt = std::max(1, std::min(8, dlr::default_threads()));
        std::vector<std::vector<int32_t>> part((size_t)nt);
        std::vector<std::thread> th;
        const int64_t nnz = (int64_t)ds.col.size();
        for (int k = 0; k < nt; ++k)
            th.emplace_back([&, k] {
                std::vector<int32_t> &pc = part[(size_t)k];
                pc.assign((size_t)D, 0);
                for (int64_t e = nnz * k / nt; e < nnz * (k + 1) / nt; ++e) ++pc[(size_t)ds.col[(size_t)e]];
            });
        for (auto &x : th) x.join();
        for (auto &pc : part)
            for (int64_t j = 0; j < D; ++j) cnt[(size_t)j] += pc[(size_t)j];
    }
    if ((rc = coll_sum_i64(c, cnt))) return rc;
    std::vector<uint64_t> key((size_t)D);
    int64_t total = 0;
    for (int64_t j = 0; j < D; ++j) {
        total += cnt[(size_t)j];
        const uint64_t cj = (uint64_t)std::min<int64_t>(cnt[(size_t)j], ((int64_t)1 << 38) - 1);
        key[(size_t)j] = ((((uint64_t)1 << 38) - 1 - cj) << 25) | (uint64_t)j;  // count desc, id asc
    }
    std::sort(key.begin(), key.end());
    if (mode < 0) {  // auto: relabel only skewed shards
        const int64_t top = std::max<int64_t>(1, D / 100);
        int64_t hot = 0;
        for (int64_t k = 0; k < top; ++k) hot += cnt[(size_t)(key[(size_t)k] & (((uint64_t)1 << 25) - 1))];
        if (2 * hot <= total) return DLR_OK;
    }
    // The rare columns (the 60 MB tail of C3's table: each seen a few times)
    // miss L2 in the margin's gathers whatever their order among equals; in
    // order of FIRST OCCURRENCE (row-major, this rank's shard) instead of id,
    // the rare columns that rows close together introduce sit on the same
    // cache lines (relabel_tail 0: by id).
    const int64_t tail_mode = tv(c->tune.relabel_tail, 2);  // 0 by id, 1 by first occurrence among equal counts, 2 by it alone
    if (tail_mode > 0) {
        const int64_t kRare = tv(c->tune.relabel_rare, 16);
        // -first, reduced by max over the ranks: every rank numbers alike
        std::vector<int64_t> first((size_t)D, -INT64_MAX);
        const int64_t nnz = (int64_t)ds.col.size();
        for (int64_t e = nnz - 1; e >= 0; --e) first[(size_t)ds.col[(size_t)e]] = -e;
        if ((rc = coll_reduce_i64(c, first.data(), first.size(), true))) return rc;
        for (auto &f : first) f = -f;
        int64_t k0 = 0;
        while (k0 < D && cnt[(size_t)(key[(size_t)k0] & (((uint64_t)1 << 25) - 1))] > kRare) ++k0;
        // the hot-weight margin stages ids [0, kMarginHot) in LDS as the
        // hottest: keep them in count order even on a shard with few
        // columns above kRare
        k0 = std::max<int64_t>(k0, std::min<int64_t>(D, dlr::kMarginHot));
        // [k0, D): counts <= kRare, descending; within each count, by first occurrence
        auto cid = [&](uint64_t kk) { return (int64_t)(kk & (((uint64_t)1 << 25) - 1)); };
        std::stable_sort(key.begin() + k0, key.end(), [&](uint64_t a, uint64_t b) {
            const int64_t ca = cnt[(size_t)cid(a)], cb = cnt[(size_t)cid(b)];
            if (tail_mode == 1 && ca != cb) return ca > cb;
            return first[(size_t)cid(a)] < first[(size_t)cid(b)];
        });
    }
    np.assign((size_t)D, 0);
    for (int64_t k = 0; k < D; ++k) np[(size_t)(key[(size_t)k] & (((uint64_t)1 << 25) - 1))] = (int32_t)k;
    return DLR_OK;
}

// Re-express the device weights and a loaded sparse test shard's columns in
// a new column numbering (load time only).
int change_perm(dlr_ctx *c, std::vector<int32_t> &&np) {
    if (np == c->perm) return DLR_OK;
    const int64_t D = c->D;
    std::vector<float> oldw((size_t)D), neww((size_t)D);
    HIPC(c, hipMemcpyAsync(oldw.data(), c->w, (size_t)D * 4, hipMemcpyDeviceToHost, c->stream));
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    for (int64_t j = 0; j < D; ++j) neww[(size_t)pid(np, j)] = oldw[(size_t)pid(c->perm, j)];
    c->pm_ready = -1;
    HIPC(c, hipMemcpyAsync(c->w, neww.data(), (size_t)D * 4, hipMemcpyHostToDevice, c->stream));
    TestShard &t = c->test;
    if (t.loaded && !t.dense && t.nnz > 0) {
        std::vector<int32_t> inv;
        if (!c->perm.empty()) {
            inv.assign((size_t)D, 0);
            for (int64_t j = 0; j < D; ++j) inv[(size_t)c->perm[(size_t)j]] = (int32_t)j;
        }
        std::vector<int32_t> col((size_t)t.nnz);
        HIPC(c, hipMemcpyAsync(col.data(), t.col, (size_t)t.nnz * 4, hipMemcpyDeviceToHost, c->stream));
        if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
        for (auto &x : col) x = (int32_t)pid(np, inv.empty() ? x : inv[(size_t)x]);
        HIPC(c, hipMemcpyAsync(t.col, col.data(), (size_t)t.nnz * 4, hipMemcpyHostToDevice, c->stream));
    }
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    c->perm = std::move(np);
    return DLR_OK;
}

// Long columns of one batch, built beside the classic copy (see
// dlr_kernels.hip "Long columns").
template <typename RowT>
struct LongBatch {
    std::vector<uint32_t> cols, cseg, sptr;
    std::vector<RowT> row;
    std::vector<float> val;
};

// Builds the column-major copy of every batch: a stable counting sort by
// column of the batch's entries taken in batch-row order, so each column's
// segment lists its rows in the order lr.cc:37 visits them.  Columns with
// more than long_min entries (0: none) go to `lb` in chunks of kLongChunk
// (4-aligned starts); their pointer entry carries kLongFlag and their
// segment in the classic copy is empty.  unit: no values are written (cval
// and the long values stay empty).
template <typename RowT>
void build_csc(const CsrView &ds, const std::vector<dlr::BatchSpan> &plan, int64_t D,
               const std::vector<int64_t> &coff, std::vector<uint32_t> &cptr, std::vector<RowT> &crow,
               std::vector<float> &cval, int64_t long_min, std::vector<LongBatch<RowT>> &lb, bool unit,
               int nthreads) {
    const int64_t nb = (int64_t)plan.size();
    const int64_t N = ds.n_rows;
    lb.assign((size_t)nb, LongBatch<RowT>());
    std::vector<std::thread> th;
    nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, nb));
    for (int t = 0; t < nthreads; ++t) {
        th.emplace_back([&, t] {
            std::vector<uint32_t> cnt((size_t)D + 1);
            std::vector<uint8_t> is_long;
            for (int64_t b = t; b < nb; b += nthreads) {
                const dlr::BatchSpan &sp = plan[(size_t)b];
                LongBatch<RowT> &L = lb[(size_t)b];
                std::fill(cnt.begin(), cnt.end(), 0u);
                for (int64_t i = 0; i < sp.rows; ++i) {
                    const int64_t r = (sp.first_row + i) % N;
                    for (int64_t k = ds.row_ptr[(size_t)r]; k < ds.row_ptr[(size_t)r + 1]; ++k)
                        ++cnt[(size_t)ds.col[(size_t)k] + 1];
                }
                bool any_long = false;
                if (long_min > 0) {
                    is_long.assign((size_t)D, 0);
                    for (int64_t j = 0; j < D; ++j)
                        if ((int64_t)cnt[(size_t)j + 1] > long_min) {
                            is_long[(size_t)j] = 1;
                            any_long = true;
                        }
                }
                uint32_t *ptr = cptr.data() + (size_t)b * (size_t)(D + 1);
                ptr[0] = 0;
                uint32_t lat = 0;  // long-array cursor
                uint32_t pad = 0;  // padding entries of the previous long column
                for (int64_t j = 0; j < D; ++j) {
                    const uint32_t c = cnt[(size_t)j + 1];
                    if (any_long && is_long[(size_t)j]) {
                        ptr[j + 1] = ptr[j];
                        L.cols.push_back((uint32_t)j);
                        L.cseg.push_back((uint32_t)L.sptr.size());
                        // a start is 4-aligned; its low bits carry the previous
                        // column's padding count (DevLong)
                        for (uint32_t o = 0; o < c; o += dlr::kLongChunk) L.sptr.push_back((lat + o) | (o ? 0u : pad));
                        cnt[(size_t)j + 1] = lat;  // long cursor
                        pad = ((c + 3) & ~3u) - c;
                        lat += (c + 3) & ~3u;
                    } else {
                        ptr[j + 1] = ptr[j] + c;
                    }
                }
                // every batch ends its cseg / sptr lists with one terminal
                // entry (the per-batch offsets rely on it).  A chunk ends
                // where the next begins: a column's last chunk also covers
                // its <= 3 padding entries (row 0, value 0), whose products
                // are +-0 and leave a sum unchanged.
                L.cseg.push_back((uint32_t)L.sptr.size());
                L.sptr.push_back(lat | pad);
                if (any_long) {
                    L.row.assign((size_t)lat + dlr::kLongChunk, 0);
                    if (!unit) L.val.assign((size_t)lat + dlr::kLongChunk, 0.0f);
                }
                // cursors: short columns in the classic copy, long ones in L
                for (int64_t j = 0; j < D; ++j)
                    if (!(any_long && is_long[(size_t)j])) cnt[(size_t)j + 1] = ptr[j];
                RowT *rr = crow.data() + coff[(size_t)b];
                float *vv = unit ? nullptr : cval.data() + coff[(size_t)b];
                for (int64_t i = 0; i < sp.rows; ++i) {
                    const int64_t r = (sp.first_row + i) % N;
                    for (int64_t k = ds.row_ptr[(size_t)r]; k < ds.row_ptr[(size_t)r + 1]; ++k) {
                        const int32_t cj = ds.col[(size_t)k];
                        const uint32_t pos = cnt[(size_t)cj + 1]++;
                        if (any_long && is_long[(size_t)cj]) {
                            L.row[pos] = (RowT)i;
                            if (!unit) L.val[pos] = ds.val[(size_t)k];
                        } else {
                            rr[pos] = (RowT)i;
                            if (!unit) vv[pos] = ds.val[(size_t)k];
                        }
                    }
                }
                for (int64_t j = 0; j < D; ++j)
                    if (any_long && is_long[(size_t)j]) ptr[j] |= 0x80000000u;
            }
        });
    }
    for (auto &x : th) x.join();
}

// Row-band copy (DevBand) of the classic copy's short columns: for each
// batch and each band of 2^shift rows, the (column, segment) pairs of the
// short columns with entries in the band, columns ascending, entries in
// batch-row order; each band's entries start 4-aligned.  Built from the
// classic copy (whose column segments are already in row order) in
// parallel over column ranges; `ws` gets each band's entry-balanced wave
// schedule (as the classic one: <= 64 pairs, ~kWin entries per wave).
// entries of a band wave's window (dlr_kernels.hip kWin): the schedule's
// wave size
constexpr int64_t kWinEntries = 1024;
template <typename RowT>
struct BandBuild {
    std::vector<uint32_t> cols, ptr, ws, hw;
    std::vector<RowT> row;
    std::vector<float> val;
    std::vector<TrainShard::Band> bands;
    std::vector<int64_t> bfirst;
    int64_t max_pair = 0;  // entries of the longest (column, band) pair
};

template <typename RowT>
void build_bands(const std::vector<uint32_t> &cptr, const std::vector<RowT> &crow, const std::vector<float> &cval,
                 const std::vector<int64_t> &coff, int64_t nb, int64_t D, int64_t B, int shift, bool unit,
                 int nthreads, int64_t hot_min, BandBuild<RowT> &out) {
    const int64_t nbands = (B + ((int64_t)1 << shift) - 1) >> shift;
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, D / 4096 + 1));
    out.bfirst.assign((size_t)nb + 1, 0);
    int64_t pair_at = 0, ptr_at = 0, ent_at = 0, ws_at = 0;
    std::vector<int64_t> np((size_t)nt * (size_t)nbands), ne((size_t)nt * (size_t)nbands);
    for (int64_t b = 0; b < nb; ++b) {
        const uint32_t *cp = cptr.data() + (size_t)b * (size_t)(D + 1);
        const RowT *rr = crow.data() + coff[(size_t)b];
        const float *vv = unit ? nullptr : cval.data() + coff[(size_t)b];
        auto lo = [&](int k) { return D * k / nt; };
        // pass 1: pairs and entries per (thread range, band)
        std::fill(np.begin(), np.end(), 0);
        std::fill(ne.begin(), ne.end(), 0);
        {
            std::vector<std::thread> th;
            for (int k = 0; k < nt; ++k)
                th.emplace_back([&, k] {
                    int64_t *P = np.data() + (size_t)k * (size_t)nbands, *E = ne.data() + (size_t)k * (size_t)nbands;
                    for (int64_t j = lo(k); j < lo(k + 1); ++j) {
                        if (cp[j] & 0x80000000u) continue;  // long column
                        const uint32_t a = cp[j] & 0x7FFFFFFFu, e = cp[j + 1] & 0x7FFFFFFFu;
                        int64_t last = -1;
                        for (uint32_t q = a; q < e; ++q) {
                            const int64_t s = (int64_t)rr[q] >> shift;
                            if (s != last) ++P[s], last = s;
                            ++E[s];
                        }
                    }
                });
            for (auto &x : th) x.join();
        }
        // band-major offsets (thread ranges ascend in column order)
        std::vector<int64_t> po((size_t)nt * (size_t)nbands), eo((size_t)nt * (size_t)nbands);
        const size_t bb0 = out.bands.size();
        for (int64_t s = 0; s < nbands; ++s) {
            TrainShard::Band bd{pair_at, ptr_at, ent_at, 0, 0};
            int64_t p = 0, e = 0;
            for (int k = 0; k < nt; ++k) {
                po[(size_t)k * nbands + s] = p;
                eo[(size_t)k * nbands + s] = e;
                p += np[(size_t)k * nbands + s];
                e += ne[(size_t)k * nbands + s];
            }
            out.bands.push_back(bd);
            pair_at += p;
            ptr_at += p + 1;
            ent_at += (e + 3) & ~int64_t(3);
        }
        out.cols.resize((size_t)pair_at);
        out.ptr.resize((size_t)ptr_at);
        out.row.resize((size_t)ent_at + 64, 0);
        if (!unit) out.val.resize((size_t)ent_at + 64, 0.0f);
        // pass 2: fill
        {
            std::vector<std::thread> th;
            for (int k = 0; k < nt; ++k)
                th.emplace_back([&, k] {
                    std::vector<int64_t> pc((size_t)nbands), ec((size_t)nbands);
                    for (int64_t s = 0; s < nbands; ++s) {
                        pc[(size_t)s] = po[(size_t)k * nbands + s];
                        ec[(size_t)s] = eo[(size_t)k * nbands + s];
                    }
                    for (int64_t j = lo(k); j < lo(k + 1); ++j) {
                        if (cp[j] & 0x80000000u) continue;
                        const uint32_t a = cp[j] & 0x7FFFFFFFu, e = cp[j + 1] & 0x7FFFFFFFu;
                        int64_t last = -1;
                        for (uint32_t q = a; q < e; ++q) {
                            const int64_t s = (int64_t)rr[q] >> shift;
                            const TrainShard::Band &bd = out.bands[bb0 + (size_t)s];
                            if (s != last) {
                                out.cols[(size_t)(bd.pair + pc[(size_t)s])] = (uint32_t)j;
                                out.ptr[(size_t)(bd.ptr + pc[(size_t)s])] = (uint32_t)ec[(size_t)s];
                                ++pc[(size_t)s];
                                last = s;
                            }
                            const size_t o = (size_t)(bd.ent + ec[(size_t)s]++);
                            out.row[o] = rr[q];
                            if (!unit) out.val[o] = vv[q];
                        }
                    }
                });
            for (auto &x : th) x.join();
        }
        // terminal pointers and wave schedules
        for (int64_t s = 0; s < nbands; ++s) {
            TrainShard::Band &bd = out.bands[bb0 + (size_t)s];
            int64_t p = 0, e = 0;
            for (int k = 0; k < nt; ++k) p += np[(size_t)k * nbands + s], e += ne[(size_t)k * nbands + s];
            out.ptr[(size_t)(bd.ptr + p)] = (uint32_t)e;
            bd.ws = ws_at;
            const uint32_t *pp = out.ptr.data() + bd.ptr;
            // a HOT column's pair (hot_min > 0: >= hot_min entries in the
            // batch) gets a wave of its own, marked in bit 31 of its start
            // (k_band_hot's; k_grad_band skips it when launched beside it)
            auto hot = [&](int64_t q) {
                if (hot_min <= 0) return false;
                const uint32_t j = out.cols[(size_t)(bd.pair + q)];
                return (int64_t)(cp[j + 1] & 0x7FFFFFFFu) - (int64_t)(cp[j] & 0x7FFFFFFFu) >= hot_min;
            };
            bd.hw = (int64_t)out.hw.size();
            out.ws.push_back(0);
            int64_t acc = 0;
            int cols = 0;
            bool prev_hot = false;
            for (int64_t q = 0; q < p; ++q) {
                const int64_t cq = (int64_t)pp[q + 1] - (int64_t)pp[q];
                out.max_pair = std::max(out.max_pair, cq);
                const bool hq = hot(q);
                if (cols > 0 && (hq || prev_hot || cols == 64 * dlr::kBandPairsPerLane || acc + cq > kWinEntries)) {
                    out.ws.push_back((uint32_t)q);
                    acc = 0;
                    cols = 0;
                }
                if (hq) {
                    out.ws.back() |= 0x80000000u;
                    out.hw.push_back((uint32_t)((int64_t)out.ws.size() - 1 - ws_at));
                }
                prev_hot = hq;
                acc += cq;
                ++cols;
            }
            out.ws.push_back((uint32_t)p);
            bd.nwaves = p > 0 ? (int64_t)out.ws.size() - ws_at - 1 : 0;
            bd.nhot = (int64_t)out.hw.size() - bd.hw;
            ws_at = (int64_t)out.ws.size();
        }
        out.bfirst[(size_t)b + 1] = (int64_t)out.bands.size();
    }
}

// The hot-column product stream (TrainShard::hs) of every batch, from the
// classic copy (each column's entries in batch-row order): a column with >=
// hot_min entries in the batch is HOT (the same ones build_bands marks);
// its stream holds its products band by band, each band's segment starting
// at a multiple of kHotChunkF floats (no chunk -- no cache line -- holds two
// bands); row i's list gets one (stream slot, value) per hot entry.  Off
// (DLR_HOT_STREAM=0, no hot column, or more than hs_max_cols() in a batch: the
// per-band k_band_hot launches instead).
// (the hot stream's chains: kHcCols per CU.  C3 has 39 columns of ~1.55M
// entries, 39 of ~724K, 273 more of >= 2^17: at most 40 / 78 / 128 / 256
// of them in the stream, 5.70 / 5.71 / 5.72 / 6.53 ms per step -- the
// margin's hot-product writes grow with them, the band kernels' chains
// shrink; profiles/r05_c3_hot_stream_max.txt)
// A band flag not seen for this long ends a k_hot_chain launch that is not
// the step's last (the next one goes on; counted, DLR_COUNT_HOT_GIVEUPS):
// far above the ~0.1-0.3 ms between flags when the margins run beside it,
// far below the 250 ms error bound
constexpr uint32_t kHsGiveUpTicks = 2000000;  // 20 ms at 100 MHz
// bands of a step's first hot-chain launch (band_step_pipelined)
// (C3, same box: 1 band 5.72-5.73 ms, 2 bands 5.72-5.73, 3 bands 5.77-5.78,
// 4 bands 5.79-5.81; profiles/r06_c3_hot_first_group.txt)
#ifndef DLR_HS_FIRST  // (A/B builds only: make variant VDEFS=-DDLR_HS_FIRST=n)
#define DLR_HS_FIRST 2
#endif
constexpr int64_t kHsFirstGroup = DLR_HS_FIRST;
// rows of a window of the band-mode product margin (TrainShard::pmw): the
// product margin's 1,024 blocks of 64 rows
constexpr int64_t kPmWinRows = (int64_t)dlr::kPmMaxBlocks * dlr::kPmRows;
static int64_t hs_max_cols(const dlr_ctx *c) { return std::max<int64_t>(1, tv(c->tune.hot_stream_max, 64)); }

bool hot_stream_wanted(const dlr_ctx *c) { return tv(c->tune.hot_stream, 1) != 0; }
// The smallest threshold >= hot_min that leaves at most hs_max_cols() hot
// columns in every batch (dlr::hot_chain_grid: kHcCols chains per CU).
int64_t hot_stream_threshold(const dlr_ctx *c, const std::vector<uint32_t> &cptr, int64_t nb, int64_t D,
                             int64_t hot_min) {
    const int64_t maxc = hs_max_cols(c);
    int64_t thr = hot_min;
    for (int64_t b = 0; b < nb; ++b) {
        const uint32_t *cp = cptr.data() + (size_t)b * (size_t)(D + 1);
        std::vector<int64_t> big;
        for (int64_t j = 0; j < D; ++j) {
            const int64_t n = (int64_t)(cp[j + 1] & 0x7FFFFFFFu) - (int64_t)(cp[j] & 0x7FFFFFFFu);
            if (n >= hot_min) big.push_back(n);
        }
        if ((int64_t)big.size() > maxc) {
            std::nth_element(big.begin(), big.begin() + maxc, big.end(), std::greater<int64_t>());
            thr = std::max(thr, big[(size_t)maxc] + 1);  // the (maxc + 1)-th largest is not hot
        }
    }
    return thr;
}
template <typename RowT>
int build_hot_stream(dlr_ctx *c, const std::vector<uint32_t> &cptr, const std::vector<RowT> &crow,
                     const std::vector<float> &cval, int64_t hot_min, int shift) {
    TrainShard &t = c->train;
    if (!hot_stream_wanted(c)) return DLR_OK;
    const int64_t nb = (int64_t)t.plan.size(), D = c->D;
    std::vector<std::vector<uint32_t>> hot((size_t)nb);
    int64_t any = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const uint32_t *cp = cptr.data() + (size_t)b * (size_t)(D + 1);
        for (int64_t j = 0; j < D; ++j)
            if ((int64_t)(cp[j + 1] & 0x7FFFFFFFu) - (int64_t)(cp[j] & 0x7FFFFFFFu) >= hot_min && !(cp[j] & 0x80000000u))
                hot[(size_t)b].push_back((uint32_t)j);
        if ((int64_t)hot[(size_t)b].size() > hs_max_cols(c)) return DLR_OK;
        any += (int64_t)hot[(size_t)b].size();
    }
    if (any == 0) return DLR_OK;
    std::vector<uint32_t> cols, off, dest;
    std::vector<float> val;
    std::vector<uint2> seg;
    t.hs_nh.assign((size_t)nb, 0);
    t.hsco.assign((size_t)nb + 1, 0);
    t.hsso.assign((size_t)nb + 1, 0);
    t.hsoo.assign((size_t)nb + 1, 0);
    int64_t buf_need = 0, max_bands = 1;
    for (int64_t b = 0; b < nb; ++b) {
        const uint32_t *cp = cptr.data() + (size_t)b * (size_t)(D + 1);
        const RowT *rr = crow.data() + t.coff[(size_t)b];
        const float *vv = t.unit ? nullptr : cval.data() + t.coff[(size_t)b];
        const int64_t rows = t.plan[(size_t)b].rows;
        const int64_t nbands = (rows + ((int64_t)1 << shift) - 1) >> shift;
        max_bands = std::max(max_bands, nbands);
        const std::vector<uint32_t> &H = hot[(size_t)b];
        const int64_t nh = (int64_t)H.size();
        t.hs_nh[(size_t)b] = nh;
        // segments: per (column, band) count, then padded starts
        std::vector<uint2> sg((size_t)(nh * nbands), uint2{0, 0});
        for (int64_t h = 0; h < nh; ++h) {
            const uint32_t j = H[(size_t)h];
            for (uint32_t q = cp[j] & 0x7FFFFFFFu; q < (cp[j + 1] & 0x7FFFFFFFu); ++q)
                ++sg[(size_t)(h * nbands + ((int64_t)rr[q] >> shift))].y;
        }
        int64_t at = 0;
        for (uint2 &x : sg) {
            x.x = (uint32_t)at;
            at += (x.y + dlr::kHotChunkF - 1) / dlr::kHotChunkF * dlr::kHotChunkF;
        }
        if (at >= ((int64_t)1 << 32)) return fail(c, DLR_E_ARG, "dlr_load_train: hot-column stream too large");
        buf_need = std::max(buf_need, at);
        // per-row lists: counts, offsets, then (slot, value) per hot entry
        std::vector<uint32_t> cnt((size_t)rows + 1, 0);
        for (int64_t h = 0; h < nh; ++h) {
            const uint32_t j = H[(size_t)h];
            for (uint32_t q = cp[j] & 0x7FFFFFFFu; q < (cp[j + 1] & 0x7FFFFFFFu); ++q) ++cnt[(size_t)rr[q] + 1];
        }
        const size_t o0 = off.size(), d0 = dest.size();
        if (d0 + (size_t)std::accumulate(cnt.begin(), cnt.end(), (uint64_t)0) >= ((size_t)1 << 32))
            return fail(c, DLR_E_ARG, "dlr_load_train: too many hot entries");
        off.resize(o0 + (size_t)rows + 1);
        uint32_t run = (uint32_t)d0;
        for (int64_t i = 0; i <= rows; ++i) {
            run += cnt[(size_t)i];
            off[o0 + (size_t)i] = run;  // (cnt[0] == 0: off[o0] = d0)
        }
        dest.resize(off[o0 + (size_t)rows]);
        if (!t.unit) val.resize(dest.size());
        std::vector<uint32_t> fillp(off.begin() + (int64_t)o0, off.end() - 1);
        for (int64_t h = 0; h < nh; ++h) {
            const uint32_t j = H[(size_t)h];
            std::vector<uint32_t> rank((size_t)nbands, 0);
            for (uint32_t q = cp[j] & 0x7FFFFFFFu; q < (cp[j + 1] & 0x7FFFFFFFu); ++q) {
                const int64_t i = (int64_t)rr[q], sb = i >> shift;
                const uint32_t slot = sg[(size_t)(h * nbands + sb)].x + rank[(size_t)sb]++;
                const uint32_t k = fillp[(size_t)i]++;
                dest[k] = slot;
                if (!t.unit) val[k] = vv[q];
            }
        }
        t.hsco[(size_t)b + 1] = t.hsco[(size_t)b] + nh;
        t.hsso[(size_t)b + 1] = t.hsso[(size_t)b] + nh * nbands;
        t.hsoo[(size_t)b] = (int64_t)o0;
        t.hsoo[(size_t)b + 1] = (int64_t)off.size();
        cols.insert(cols.end(), H.begin(), H.end());
        seg.insert(seg.end(), sg.begin(), sg.end());
    }
    int r;
    if ((r = upload(c, &t.hs_cols, cols.data(), cols.size()))) return r;
    if ((r = upload(c, &t.hs_seg, seg.data(), seg.size()))) return r;
    if ((r = upload(c, &t.hs_off, off.data(), off.size()))) return r;
    if ((r = upload(c, &t.hs_dest, dest.data(), dest.size(), 1))) return r;
    if (!t.unit && (r = upload(c, &t.hs_val, val.data(), val.size(), 1))) return r;
    if ((r = dev_alloc(c, (void **)&t.hs_buf, (size_t)(buf_need + dlr::kHotChunkF) * 4))) return r;
    std::vector<uint32_t> zero((size_t)max_bands, 0);
    if ((r = upload(c, &t.hs_flag, zero.data(), zero.size()))) return r;
    int64_t nh_max = 1;
    for (int64_t x : t.hs_nh) nh_max = std::max(nh_max, x);
    if ((r = dev_alloc(c, (void **)&t.hs_state, (size_t)nh_max * 8))) return r;
    t.hs_seq = 0;
    t.hs = true;
    t.hs_bytes = (int64_t)((cols.size() + off.size() + dest.size() + val.size()) * 4 + seg.size() * 8 +
                           (buf_need + dlr::kHotChunkF) * 4);
    return DLR_OK;
}

// Long columns of every batch regrouped in row phases of kLPhase rows
// (band mode): from the chunked long arrays (LongBatch, rows ascending per
// column), for each batch and phase the entries of each long column with a
// row in the phase (phase-local uint16 rows), columns in long-column order,
// each phase's entries starting 4-aligned.  A column's entries in a phase
// are cut into PIECES of <= kPiece consecutive entries (a lane sums one
// piece in row order); piece partials are numbered column-major -- column
// l's pieces, phase by phase, from cseg[l] -- so k_long_combine adds each
// column's partials in row order.  Per phase an entry-balanced wave
// schedule over the pieces (<= 64 pieces, ~kWin entries per wave).
// DLR_LONG_PIECE overrides the piece size (1..1024; default 63: a wave's
// pieces then start 63 floats apart in its LDS product slab, one bank
// apart, where 64-entry pieces put every summing lane on the same bank --
// C3 long phases 427 -> 333 us; tools/lp_ab.sh sweeps 31..127)
int64_t long_piece(const dlr_tuning &tu) {
    const int64_t v = tv(tu.long_piece, 63);
    return v >= 1 && v <= 1024 ? v : 63;
}
struct LPhaseBuild {
    std::vector<dlr::PhaseDesc> desc;
    std::vector<uint32_t> ptr, slot, ws, cseg;
    std::vector<uint16_t> row;
    std::vector<float> val;
    int64_t maxpart = 0;
};

template <typename RowT>
void build_long_phases(const std::vector<LongBatch<RowT>> &lb, int64_t B, bool unit, int64_t kPiece,
                       LPhaseBuild &out) {
    const int64_t nph = (B + dlr::kLPhase - 1) / dlr::kLPhase;
    for (const LongBatch<RowT> &L : lb) {
        const int64_t nl = (int64_t)L.cols.size();
        std::vector<int64_t> cnt((size_t)(nph * nl), 0);  // [p][l]
        std::vector<int64_t> a((size_t)nl), e((size_t)nl);
        for (int64_t l = 0; l < nl; ++l) {
            a[(size_t)l] = L.sptr[L.cseg[(size_t)l]] & ~3u;
            const uint32_t nx = L.sptr[L.cseg[(size_t)l + 1]];
            e[(size_t)l] = (int64_t)(nx & ~3u) - (int64_t)(nx & 3u);
            for (int64_t q = a[(size_t)l]; q < e[(size_t)l]; ++q)
                ++cnt[(size_t)(((int64_t)L.row[(size_t)q] / dlr::kLPhase) * nl + l)];
        }
        // piece slots: column-major
        std::vector<int64_t> cs((size_t)nl + 1, 0), pslot((size_t)(nph * nl));
        for (int64_t l = 0; l < nl; ++l) {
            int64_t n = cs[(size_t)l];
            for (int64_t p = 0; p < nph; ++p) {
                pslot[(size_t)(p * nl + l)] = n;
                n += (cnt[(size_t)(p * nl + l)] + kPiece - 1) / kPiece;
            }
            cs[(size_t)l + 1] = n;
        }
        std::vector<int64_t> cur((size_t)(nph * nl));
        for (int64_t p = 0; p < nph; ++p) {
            dlr::PhaseDesc d{(int64_t)out.ptr.size(), (int64_t)out.row.size(), (int64_t)out.ws.size(), 0};
            int64_t at = 0, np = 0, acc = 0;
            int pieces = 0;
            out.ws.push_back(0);
            for (int64_t l = 0; l < nl; ++l) {
                const int64_t c = cnt[(size_t)(p * nl + l)];
                cur[(size_t)(p * nl + l)] = d.ent + at;
                for (int64_t o = 0; o < c; o += kPiece) {
                    const int64_t n = std::min(kPiece, c - o);
                    if (pieces == 64 * dlr::kBandPairsPerLane || (pieces > 0 && acc + n > 1024)) {
                        out.ws.push_back((uint32_t)np);
                        acc = 0;
                        pieces = 0;
                    }
                    out.ptr.push_back((uint32_t)(at + o));
                    out.slot.push_back((uint32_t)(pslot[(size_t)(p * nl + l)] + o / kPiece));
                    acc += n;
                    ++pieces;
                    ++np;
                }
                at += c;
            }
            out.ptr.push_back((uint32_t)at);
            out.slot.push_back(0);  // keeps slot indexed like ptr
            out.ws.push_back((uint32_t)np);
            d.ntasks = np > 0 ? (int64_t)out.ws.size() - d.ws - 1 : 0;
            out.desc.push_back(d);
            out.row.resize((size_t)(d.ent + ((at + 3) & ~int64_t(3))), 0);
        }
        if (!unit) out.val.resize(out.row.size(), 0.0f);
        for (int64_t l = 0; l < nl; ++l)
            for (int64_t q = a[(size_t)l]; q < e[(size_t)l]; ++q) {
                const int64_t r = (int64_t)L.row[(size_t)q];
                const size_t o = (size_t)cur[(size_t)((r / dlr::kLPhase) * nl + l)]++;
                out.row[o] = (uint16_t)(r % dlr::kLPhase);
                if (!unit) out.val[o] = L.val[(size_t)q];
            }
        for (int64_t l = 0; l <= nl; ++l) out.cseg.push_back((uint32_t)cs[(size_t)l]);
        out.maxpart = std::max(out.maxpart, cs[(size_t)nl]);
    }
}

// Phase-split column-major copy (DevPcsc, dlr_kernels.h) of every batch.
// Rows of batch b fall in phases of R rows; for each 64-column group and
// phase, a block lists the entries of the group's columns whose row is in
// the phase, column by column, in batch-row order (a stable counting sort
// of the batch taken in row order, as lr.cc:37 visits it).  Returns false
// (layout not applicable) if some block would exceed 255 entries.
struct PcscBuild {
    int P = 1;
    int64_t R = 0, groups = 0, pblocks = 0;
    std::vector<int64_t> size;  // padded entries per batch
};

template <typename Fn>
void for_batches(int64_t nb, int nthreads, Fn fn) {
    std::vector<std::thread> th;
    std::atomic<int64_t> next{0};
    nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, nb));
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([&] {
            for (int64_t b; (b = next.fetch_add(1)) < nb;) fn(b);
        });
    for (auto &x : th) x.join();
}

// After every streamed array is placed: pack each batch's slices of all of
// them into one page-locked buffer (batch-major), so staging a batch is ONE
// H2D copy ("coalesced CSR upload of each minibatch"), and replace the
// per-array host copies and device slots by two batch-sized slots.
int coalesce_stream(dlr_ctx *c, int nthreads) {
    TrainShard &t = c->train;
    if (tv(c->tune.stream_coalesce, 1) == 0) return DLR_OK;  // one copy per array and batch
    const size_t nb = t.plan.size(), na = t.sarr.size();
    t.soff.assign(nb * na, 0);
    t.sbsz.assign(nb, 0);
    t.sboff.assign(nb + 1, 0);
    size_t maxs = 256;
    for (size_t b = 0; b < nb; ++b) {
        size_t o = 0;
        for (size_t k = 0; k < na; ++k) {
            const StreamArr &a = t.sarr[k];
            o = (o + 255) & ~(size_t)255;
            t.soff[b * na + k] = o;
            if (a.end[b] > a.beg[b]) o += ((size_t)(a.end[b] - a.beg[b]) + a.pad) * a.es;
        }
        t.sbsz[b] = o;
        t.sboff[b + 1] = t.sboff[b] + ((o + 255) & ~(size_t)255);
        maxs = std::max(maxs, o);
    }
    HIPC(c, hipHostMalloc((void **)&t.shost, std::max<size_t>(t.sboff[nb], 256), hipHostMallocDefault));
    for_batches((int64_t)nb, nthreads, [&](int64_t b) {
        for (size_t k = 0; k < na; ++k) {
            const StreamArr &a = t.sarr[k];
            if (a.end[(size_t)b] <= a.beg[(size_t)b]) continue;
            memcpy(t.shost + t.sboff[(size_t)b] + t.soff[(size_t)b * na + k], a.host + (size_t)a.beg[(size_t)b] * a.es,
                   ((size_t)(a.end[(size_t)b] - a.beg[(size_t)b]) + a.pad) * a.es);
        }
    });
    for (StreamArr &a : t.sarr) {  // the array-major copies and slots are no longer needed
        if (a.registered) (void)hipHostUnregister(const_cast<char *>(a.host));
        a.registered = false;
        a.keep.reset();
        a.host = nullptr;
        for (int k = 0; k < 2; ++k) {
            t.bytes -= (int64_t)(a.cap * a.es);
            dev_free(c, a.slot[k]);
            a.slot[k] = nullptr;
        }
    }
    for (int k = 0; k < 2; ++k) {
        const int rc = dev_alloc(c, &t.sslot[k], maxs);
        if (rc) return rc;
    }
    t.bytes += (int64_t)(2 * maxs);
    return DLR_OK;
}


// Counts of (column, phase) for batch sp; cnt has D*P entries.
void pcsc_count(const CsrView &ds, const dlr::BatchSpan &sp, const PcscBuild &pb, std::vector<uint32_t> &cnt) {
    std::fill(cnt.begin(), cnt.end(), 0u);
    const int64_t N = ds.n_rows;
    for (int64_t i = 0; i < sp.rows; ++i) {
        const int64_t r = (sp.first_row + i) % N;
        const int64_t p = i / pb.R;
        for (int64_t k = ds.row_ptr[(size_t)r]; k < ds.row_ptr[(size_t)r + 1]; ++k)
            ++cnt[(size_t)ds.col[(size_t)k] * pb.P + (size_t)p];
    }
}

bool pcsc_plan(const CsrView &ds, const std::vector<dlr::BatchSpan> &plan, int64_t D, PcscBuild &pb,
               int nthreads) {
    const int64_t nb = (int64_t)plan.size();
    pb.size.assign((size_t)nb, 0);
    std::atomic<bool> ok{true};
    for_batches(nb, nthreads, [&](int64_t b) {
        if (!ok) return;
        std::vector<uint32_t> cnt((size_t)(D * pb.P));
        pcsc_count(ds, plan[(size_t)b], pb, cnt);
        int64_t total = 0;
        for (int64_t g = 0; g < pb.groups && ok; ++g)
            for (int p = 0; p < pb.P; ++p) {
                uint32_t blen = 0;
                for (int64_t j = g * 64; j < std::min(D, g * 64 + 64); ++j) blen += cnt[(size_t)(j * pb.P + p)];
                if (blen > 255) {
                    ok = false;
                    break;
                }
                total += (blen + 3) & ~3u;
            }
        pb.size[(size_t)b] = total;
    });
    return ok;
}

void pcsc_fill(const CsrView &ds, const std::vector<dlr::BatchSpan> &plan, int64_t D, const PcscBuild &pb,
               const std::vector<int64_t> &poff, std::vector<uint32_t> &base, std::vector<uint8_t> &ends,
               std::vector<uint16_t> &row, std::vector<float> &val, int nthreads) {
    const int64_t nb = (int64_t)plan.size();
    const int64_t N = ds.n_rows;
    for_batches(nb, nthreads, [&](int64_t b) {
        const dlr::BatchSpan &sp = plan[(size_t)b];
        std::vector<uint32_t> cnt((size_t)(D * pb.P));
        pcsc_count(ds, sp, pb, cnt);
        uint32_t *bs = base.data() + (size_t)b * (size_t)(pb.pblocks + 1);
        uint8_t *en = ends.data() + (size_t)b * (size_t)pb.pblocks * 64;
        uint16_t *rr = row.data() + poff[(size_t)b];
        float *vv = val.data() + poff[(size_t)b];
        // block bases, per-column end offsets, and cursors (reusing cnt)
        uint32_t at = 0;
        for (int64_t g = 0; g < pb.groups; ++g)
            for (int p = 0; p < pb.P; ++p) {
                const int64_t blk = g * pb.P + p;
                bs[blk] = at;
                uint32_t o = 0;
                for (int l = 0; l < 64; ++l) {
                    const int64_t j = g * 64 + l;
                    if (j < D) {
                        const uint32_t c = cnt[(size_t)(j * pb.P + p)];
                        cnt[(size_t)(j * pb.P + p)] = at + o;  // cursor
                        o += c;
                    }
                    en[blk * 64 + l] = (uint8_t)o;
                }
                at += (o + 3) & ~3u;
            }
        bs[pb.pblocks] = at;
        for (int64_t i = 0; i < sp.rows; ++i) {
            const int64_t r = (sp.first_row + i) % N;
            const int64_t p = i / pb.R;
            for (int64_t k = ds.row_ptr[(size_t)r]; k < ds.row_ptr[(size_t)r + 1]; ++k) {
                const uint32_t pos = cnt[(size_t)ds.col[(size_t)k] * pb.P + (size_t)p]++;
                rr[pos] = (uint16_t)(i - p * pb.R);
                vv[pos] = ds.val[(size_t)k];
            }
        }
    });
}

// Product-margin layout of one batch (dlr_kernels.h DevPm).  Returns false
// when the batch does not fit it (a region over kPmCap products, a chunk
// over kPmMaxChunk, a row over 8 * kPmMaxGroups entries).
struct PmBatch {
    std::vector<uint32_t> lbeg, list, pofs, rg, qoff;
    std::vector<float> val;
    std::vector<uint16_t> qs;
    int groups = 0;
    uint32_t rstride = 0, qstride = 0;  // DevPm: fixed region / slot-list strides (0: none)
    int64_t maxslice = 0;
    // the row-round gradient's view of the same batch (dlr_kernels.h DevRt);
    // empty when a slice holds more than kRtCap entries
    std::vector<uint32_t> gq;
    std::vector<float> rval;
    std::vector<uint16_t> cend;
    uint32_t rtcap = 0;  // entries per (slice, round)
};

// DevRt arrays of one product-margin batch, from its (unpacked) list words
// (column | block << 12 | rank << 22), each entry's batch row and value (list
// order): slots in column-major order within each slice, column runs, and
// the entries of each (slice, round) at a fixed stride (o.rtcap) so that a
// workgroup computes where its rounds are without loading anything first.
void rt_batch(const std::vector<uint32_t> &words, const std::vector<uint16_t> &rows, const std::vector<float> &vals,
              const std::vector<uint32_t> &slice_n, const std::vector<uint32_t> &cnt, int64_t S, int64_t nblk,
              int64_t R, PmBatch &o) {
    const int64_t T = (R + dlr::kRtRows - 1) / dlr::kRtRows;
    const bool unit = vals.empty();
    std::vector<uint32_t> gq(words.size(), 0), rb((size_t)(S * (T + 1)));
    o.cend.assign((size_t)(S * dlr::kPmSlice), 0);
    std::vector<uint32_t> cur(dlr::kPmSlice);
    uint32_t cap = 4;
    auto drop = [&] {
        o.gq.clear();
        o.rval.clear();
        o.cend.clear();
        o.rtcap = 0;
    };
    for (int64_t q = 0; q < S; ++q) {
        const uint32_t l0 = slice_n[(size_t)q], l1 = slice_n[(size_t)q + 1];
        auto real = [&](uint32_t li) {
            const uint32_t wd = words[li];
            return (wd >> 22) < cnt[(size_t)(((wd >> 12) & 1023u) * S + q)];
        };
        std::fill(cur.begin(), cur.end(), 0u);
        for (uint32_t li = l0; li < l1; ++li)
            if (real(li)) ++cur[words[li] & 0xFFFu];
        uint32_t at = 0;
        uint16_t *ce = o.cend.data() + (size_t)q * dlr::kPmSlice;
        for (int c = 0; c < dlr::kPmSlice; ++c) {
            const uint32_t n = cur[(size_t)c];
            cur[(size_t)c] = at;
            at += n;
            ce[c] = (uint16_t)std::min<uint32_t>(at, 0xFFFFu);
        }
        if (at > (uint32_t)dlr::kRtCap) return drop();  // does not fit LDS
        // list order is (block, row, column): each column's slots take its
        // rows in ascending order
        for (uint32_t li = l0; li < l1; ++li) {
            const uint32_t row = rows[li];
            gq[li] = row << 16 | (real(li) ? cur[words[li] & 0xFFFu]++ : (uint32_t)dlr::kRtCap);
        }
        // round t starts at the chunk of block t * kRtRows / 64
        uint32_t li = l0;
        int64_t k = 0;
        for (int64_t t = 0; t <= T; ++t) {
            const int64_t kt = std::min<int64_t>(nblk, t * (dlr::kRtRows / dlr::kPmRows));
            for (; k < kt; ++k) li += (cnt[(size_t)(k * S + q)] + 3) & ~3u;
            rb[(size_t)(q * (T + 1) + t)] = li;
            if (t > 0) cap = std::max(cap, li - rb[(size_t)(q * (T + 1) + t - 1)]);
        }
    }
    if (cap > (uint32_t)dlr::kRtMaxRound) return drop();  // one 4-entry group per thread and round
    // (slice, round) q * T + t holds its entries at [(q * T + t) * cap, + cap):
    // the round's list entries, then sinks (row t * kRtRows, slot kRtCap)
    o.rtcap = cap;
    o.gq.assign((size_t)(S * T * cap), 0);
    if (!unit) o.rval.assign((size_t)(S * T * cap), 0.0f);
    for (int64_t q = 0; q < S; ++q)
        for (int64_t t = 0; t < T; ++t) {
            const uint32_t a = rb[(size_t)(q * (T + 1) + t)], b = rb[(size_t)(q * (T + 1) + t + 1)];
            const size_t d = (size_t)((q * T + t) * cap);
            for (uint32_t e = 0; e < cap; ++e) {
                const bool in = a + e < b;
                o.gq[d + e] = in ? gq[a + e] : (uint32_t)(t * dlr::kRtRows) << 16 | (uint32_t)dlr::kRtCap;
                if (!unit) o.rval[d + e] = in ? vals[a + e] : 0.0f;
            }
        }
}

bool pm_batch(const CsrView &ds, const dlr::BatchSpan &sp, int64_t D, bool unit, bool rt, PmBatch &o) {
    const int64_t N = ds.n_rows, R = sp.rows;
    const int64_t S = (D + dlr::kPmSlice - 1) / dlr::kPmSlice, nblk = (R + dlr::kPmRows - 1) / dlr::kPmRows;
    if (nblk > dlr::kPmMaxBlocks) return false;
    // a region's chunks in the order of their slice's XCD (workgroup s runs
    // on XCD s % 8): each XCD's pass-1 stores land in adjacent chunks
    std::vector<int64_t> sorder;
    for (int x = 0; x < 8; ++x)
        for (int64_t q = x; q < S; q += 8) sorder.push_back(q);
    auto row_of = [&](int64_t i) { return (sp.first_row + i) % N; };
    std::vector<uint32_t> cnt((size_t)(nblk * S), 0), slice_n((size_t)S + 1, 0);
    for (int64_t i = 0; i < R; ++i) {
        const int64_t r = row_of(i), k = i / dlr::kPmRows;
        if (ds.row_ptr[r + 1] - ds.row_ptr[r] > 8 * dlr::kPmMaxGroups) return false;
        for (int64_t e = ds.row_ptr[r]; e < ds.row_ptr[r + 1]; ++e) ++cnt[(size_t)(k * S + ds.col[e] / dlr::kPmSlice)];
    }
    // chunks padded to whole 4-slot groups (pass 1 stores 16 bytes per group).
    // Regions at a FIXED stride (the batch's largest region) when that costs
    // at most 1/8 more space than packing them -- uniform rows (C2) -- so
    // pass 2 needs no offset load (DevPm::rstride)
    uint32_t rmax = 0;
    uint64_t rsum = 0;
    for (int64_t k = 0; k < nblk; ++k) {
        uint32_t n = 0;
        for (int64_t q = 0; q < S; ++q) n += (cnt[(size_t)(k * S + q)] + 3) & ~3u;
        rmax = std::max(rmax, n);
        rsum += n;
    }
    o.rstride = (uint64_t)rmax * (uint64_t)nblk * 8 <= rsum * 9 ? rmax : 0u;
    std::vector<uint32_t> cofs((size_t)(nblk * S));
    o.rg.assign((size_t)nblk + 1, 0);
    uint32_t at = 0;
    for (int64_t k = 0; k < nblk; ++k) {
        if (o.rstride) at = (uint32_t)k * o.rstride;
        o.rg[(size_t)k] = at;
        for (int64_t q : sorder) {
            const uint32_t n = (cnt[(size_t)(k * S + q)] + 3) & ~3u;
            if (n > (uint32_t)dlr::kPmMaxChunk) return false;
            cofs[(size_t)(k * S + q)] = at;
            at += n;
            slice_n[(size_t)q + 1] += n;
        }
        if (at - o.rg[(size_t)k] > (uint32_t)dlr::kPmCap) return false;
    }
    o.rg[(size_t)nblk] = o.rstride ? (uint32_t)nblk * o.rstride : at;
    for (int64_t q = 0; q < S; ++q) {
        o.maxslice = std::max<int64_t>(o.maxslice, slice_n[(size_t)q + 1]);
        slice_n[(size_t)q + 1] += slice_n[(size_t)q];
    }
    o.lbeg.assign(slice_n.begin(), slice_n.end());
    const size_t E = slice_n[(size_t)S];
    o.list.assign(E, 0);
    if (!unit) o.val.assign(E, 0.0f);
    o.pofs.assign((size_t)(S * nblk), 0);
    for (int64_t q = 0; q < S; ++q)
        for (int64_t k = 0; k < nblk; ++k) o.pofs[(size_t)(q * nblk + k)] = cofs[(size_t)(k * S + q)];
    // padding entries: column 0, value 0, the group's block and rank (and,
    // for the row-round gradient, the block's first row)
    std::vector<uint16_t> lrow(rt ? E : 0);
    for (int64_t q = 0; q < S; ++q) {
        uint32_t li = slice_n[(size_t)q];
        for (int64_t k = 0; k < nblk; ++k) {
            const uint32_t n = cnt[(size_t)(k * S + q)], np = (n + 3) & ~3u;
            for (uint32_t j = n; j < np; ++j) {
                o.list[li + j] = (uint32_t)k << 12 | j << 22;
                if (rt) lrow[li + j] = (uint16_t)(k * dlr::kPmRows);
            }
            li += np;
        }
    }
    // entries: slice q's list holds block k's chunk at its padded offset
    std::vector<uint32_t> lcur((size_t)(nblk * S));
    for (int64_t q = 0; q < S; ++q) {
        uint32_t li = slice_n[(size_t)q];
        for (int64_t k = 0; k < nblk; ++k) {
            lcur[(size_t)(k * S + q)] = li;
            li += (cnt[(size_t)(k * S + q)] + 3) & ~3u;
        }
    }
    std::vector<uint32_t> fill(cofs);
    o.qoff.assign((size_t)nblk + 1, 0);
    o.qs.clear();
    o.groups = 0;
    // slot lists at a fixed stride too (the batch's most groups; a block's
    // extra groups are zeros its rows never take)
    std::vector<int> gblk((size_t)nblk);
    for (int64_t k = 0; k < nblk; ++k) {
        const int64_t i0 = k * dlr::kPmRows, i1 = std::min(R, i0 + dlr::kPmRows);
        int64_t ml = 0;
        for (int64_t i = i0; i < i1; ++i) ml = std::max(ml, ds.row_ptr[row_of(i) + 1] - ds.row_ptr[row_of(i)]);
        gblk[(size_t)k] = (int)((ml + 7) / 8);
        o.groups = std::max(o.groups, gblk[(size_t)k]);
    }
    o.qstride = o.rstride ? (uint32_t)o.groups * 512u : 0u;
    for (int64_t k = 0; k < nblk; ++k) {
        const int64_t i0 = k * dlr::kPmRows, i1 = std::min(R, i0 + dlr::kPmRows);
        const int g = o.qstride ? o.groups : gblk[(size_t)k];
        const size_t q0 = o.qs.size();
        o.qoff[(size_t)k] = (uint32_t)q0;
        o.qs.resize(q0 + (size_t)g * 512, 0);
        for (int64_t i = i0; i < i1; ++i) {
            const int64_t r = row_of(i), l = i - i0;
            for (int64_t e = ds.row_ptr[r], kk = 0; e < ds.row_ptr[r + 1]; ++e, ++kk) {
                const int64_t q = ds.col[e] / dlr::kPmSlice;
                const uint32_t slot = fill[(size_t)(k * S + q)]++;
                const uint32_t j = slot - cofs[(size_t)(k * S + q)];
                const uint32_t li = lcur[(size_t)(k * S + q)]++;
                o.list[li] = (uint32_t)(ds.col[e] % dlr::kPmSlice) | (uint32_t)k << 12 | j << 22;
                if (rt) lrow[li] = (uint16_t)i;
                if (!unit) o.val[li] = ds.val[e];
                o.qs[q0 + (size_t)(kk / 8) * 512 + (size_t)l * 8 + (size_t)(kk % 8)] = (uint16_t)(slot - o.rg[(size_t)k]);
            }
        }
    }
    o.qoff[(size_t)nblk] = (uint32_t)o.qs.size();
    if (rt) rt_batch(o.list, lrow, o.val, slice_n, cnt, S, nblk, R, o);
    // pack the entries in groups of four (dlr_kernels.h DevPm)
    for (size_t g = 0; g < E / 4; ++g) {
        const uint32_t *e = o.list.data() + 4 * g;
        const uint32_t k = (e[0] >> 12) & 1023u, j4 = (e[0] >> 22) / 4;
        const uint32_t c0 = e[0] & 0xFFFu, c1 = e[1] & 0xFFFu, c2 = e[2] & 0xFFFu, c3 = e[3] & 0xFFFu;
        o.list[2 * g] = c0 | c1 << 12 | (c2 & 0xFFu) << 24;
        o.list[2 * g + 1] = c2 >> 8 | c3 << 4 | k << 16 | j4 << 26;
    }
    o.list.resize(E / 2);
    return true;
}

// The block bases alone (pcsc_fill's first half), for a streamed shard
// whose layout is built on the device.
void pcsc_bases(const CsrView &ds, const std::vector<dlr::BatchSpan> &plan, int64_t D, const PcscBuild &pb,
                std::vector<uint32_t> &base, int nthreads) {
    const int64_t nb = (int64_t)plan.size();
    for_batches(nb, nthreads, [&](int64_t b) {
        std::vector<uint32_t> cnt((size_t)(D * pb.P));
        pcsc_count(ds, plan[(size_t)b], pb, cnt);
        uint32_t *bs = base.data() + (size_t)b * (size_t)(pb.pblocks + 1);
        uint32_t at = 0;
        for (int64_t g = 0; g < pb.groups; ++g)
            for (int p = 0; p < pb.P; ++p) {
                bs[g * pb.P + p] = at;
                uint32_t o = 0;
                for (int64_t j = g * 64; j < std::min(D, g * 64 + 64); ++j) o += cnt[(size_t)(j * pb.P + p)];
                at += (o + 3) & ~3u;
            }
        bs[pb.pblocks] = at;
    });
}

// Touched-column copy of one batch: the batch's entries sorted by (column,
// batch row) -- a stable sort of the batch in row order, so each column's
// segment lists its rows in the order lr.cc:37 visits them.
struct TouchedBatch {
    std::vector<uint32_t> cols, ptr;
    std::vector<uint32_t> row;
    std::vector<float> val;
};

void touched_batch(const CsrView &ds, const dlr::BatchSpan &sp, TouchedBatch &tb) {
    const int64_t N = ds.n_rows;
    struct E {
        uint32_t col, row;
        float val;
    };
    std::vector<E> es;
    for (int64_t i = 0; i < sp.rows; ++i) {
        const int64_t r = (sp.first_row + i) % N;
        for (int64_t k = ds.row_ptr[(size_t)r]; k < ds.row_ptr[(size_t)r + 1]; ++k)
            es.push_back({(uint32_t)ds.col[(size_t)k], (uint32_t)i, ds.val[(size_t)k]});
    }
    std::stable_sort(es.begin(), es.end(), [](const E &a, const E &b) { return a.col < b.col; });
    tb.cols.clear();
    tb.ptr.clear();
    tb.row.resize(es.size());
    tb.val.resize(es.size());
    for (size_t k = 0; k < es.size(); ++k) {
        if (k == 0 || es[k].col != es[k - 1].col) {
            tb.cols.push_back(es[k].col);
            tb.ptr.push_back((uint32_t)k);
        }
        tb.row[k] = es[k].row;
        tb.val[k] = es[k].val;
    }
    tb.ptr.push_back((uint32_t)es.size());
}

// True when every value is exactly 1.0f (one-hot / binary features, e.g.
// a9a and Criteo-style hashed fields): fl32(t * 1.0f) == t, so the UNIT
// kernels that never read values give the same bits.  DLR_UNIT_VALUES=0
// keeps the value arrays (A/B and tests).
bool unit_values(const dlr_ctx *c, const std::vector<float> &val) {
    if (tv(c->tune.unit_values, 1) == 0 || val.empty()) return false;
    const size_t n = val.size();
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)dlr::default_threads(), n >> 20));
    std::atomic<bool> all{true};
    std::vector<std::thread> th;
    for (int k = 0; k < nt; ++k)
        th.emplace_back([&, k] {
            const uint32_t *v = reinterpret_cast<const uint32_t *>(val.data());
            for (size_t e = n * k / nt; e < n * (k + 1) / nt; e += 4096) {
                if (!all.load(std::memory_order_relaxed)) return;
                const size_t end = std::min(n * (k + 1) / nt, e + 4096);
                uint32_t acc = 0;
                for (size_t i = e; i < end; ++i) acc |= v[i] ^ 0x3F800000u;
                if (acc) {
                    all = false;
                    return;
                }
            }
        });
    for (auto &x : th) x.join();
    return all;
}

dlr::DevBatch batch_view(const dlr_ctx *c, int64_t b) {
    const TrainShard &t = c->train;
    const dlr::BatchSpan &sp = t.plan[(size_t)b];
    const int64_t nnz = t.coff[(size_t)b + 1] - t.coff[(size_t)b];  // upper bound (aligned)
    if (b == t.wrap_batch) return {t.w_row_ptr, t.w_col, t.w_val, t.w_label, sp.rows, nnz};
    return {t.row_ptr + sp.first_row, t.col, t.val, t.label + sp.first_row, sp.rows, nnz};
}

dlr::DevPm pm_view(const dlr_ctx *c, int64_t b) {
    const TrainShard &t = c->train;
    dlr::DevPm v{};
    v.lbeg = t.pm_lbeg + b * (t.pmS + 1);
    v.list = t.pm_list + t.pmo_list[(size_t)b] / 2;  // two words per group of four entries
    v.val = t.pm_val ? t.pm_val + t.pmo_list[(size_t)b] : nullptr;
    v.pofs = t.pm_pofs + t.pmo_pofs[(size_t)b];
    v.rg = t.pm_rg + t.pmo_rg[(size_t)b];
    v.qoff = t.pm_qoff + t.pmo_rg[(size_t)b];
    v.qs = t.pm_qs + t.pmo_qs[(size_t)b];
    v.S = t.pmS;
    v.nblk = t.pmo_rg[(size_t)b + 1] - t.pmo_rg[(size_t)b] - 1;
    v.groups = t.pm_groups;
    v.split = t.pm_split;
    v.rstride = t.pm_rstride[(size_t)b];
    v.qstride = t.pm_qstride[(size_t)b];
    return v;
}

// Streamed dense shard: copy batch b's rows (wrapping to row 0 as
// data_iter.h:49-52 does) and labels into slot s, after the kernels that
// last read the slot are done (ev_free[s]); ev_ready[s] marks the copy.
hipError_t stage_dense(dlr_ctx *c, int64_t b, int s) {
    TrainShard &t = c->train;
    const int64_t D = c->D, N = t.n_rows;
    hipError_t e = hipStreamWaitEvent(c->cstream, c->ev_free[s], 0);
    int64_t row = t.plan[(size_t)b].first_row, off = 0, left = t.plan[(size_t)b].rows;
    while (e == hipSuccess && left > 0) {
        const int64_t n = std::min(left, N - row);
        e = hipMemcpyAsync(t.sx[s] + off * D, t.hX + row * D, (size_t)(n * D) * 4, hipMemcpyHostToDevice, c->cstream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(t.sl[s] + off, t.label + row, (size_t)n * 4, hipMemcpyDeviceToDevice, c->cstream);
        off += n;
        left -= n;
        row = 0;
    }
    if (e == hipSuccess) e = hipEventRecord(c->ev_ready[s], c->cstream);
    t.sb[s] = e == hipSuccess ? b : -1;
    return e;
}

// Streamed sparse shard: copy batch b's slice of every array into slot s
// after the kernels that last read the slot are done (ev_free[s]).
hipError_t stage_sparse(dlr_ctx *c, int64_t b, int s) {
    TrainShard &t = c->train;
    hipError_t e = hipStreamWaitEvent(c->cstream, c->ev_free[s], 0);
    if (t.shost) {
        if (e == hipSuccess && t.sbsz[(size_t)b] > 0)  // the batch's slices, one coalesced copy
            e = hipMemcpyAsync(t.sslot[s], t.shost + t.sboff[(size_t)b], t.sbsz[(size_t)b], hipMemcpyHostToDevice,
                               c->cstream);
    } else {
        for (StreamArr &a : t.sarr) {
            if (e != hipSuccess) break;
            const int64_t beg = a.beg[(size_t)b], end = a.end[(size_t)b];
            if (end <= beg) continue;
            e = hipMemcpyAsync(a.slot[s], a.host + (size_t)beg * a.es, ((size_t)(end - beg) + a.pad) * a.es,
                               hipMemcpyHostToDevice, c->cstream);
        }
    }
    if (e == hipSuccess) e = hipEventRecord(c->ev_ready[s], c->cstream);
    t.sb[s] = e == hipSuccess ? b : -1;
    return e;
}

// Before batch b's kernels: its slices are (being) staged, the engine
// stream waits for them, and every streamed array's pointer is bound to
// the slot (slot - beg[b] elements: the views add the batch's offsets).
hipError_t sparse_batch(dlr_ctx *c, int64_t b) {
    TrainShard &t = c->train;
    int s = t.sb[0] == b ? 0 : t.sb[1] == b ? 1 : -1;
    hipError_t e = hipSuccess;
    if (s < 0) {
        s = (int)(b & 1);
        e = stage_sparse(c, b, s);
    }
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_ready[s], 0);
    const size_t na = t.sarr.size();
    for (size_t k = 0; k < na; ++k) {
        const StreamArr &a = t.sarr[k];
        char *base = t.shost ? static_cast<char *>(t.sslot[s]) + t.soff[(size_t)b * na + k]
                             : static_cast<char *>(a.slot[s]);
        void *p = base - (ptrdiff_t)((size_t)a.beg[(size_t)b] * a.es);
        memcpy(a.field, &p, sizeof p);
    }
    return e;
}

// After batch b's last kernel: release its slot and start staging the next
// batch into the other one (it overlaps this step's remaining work).
hipError_t sparse_batch_done(dlr_ctx *c, int64_t b) {
    TrainShard &t = c->train;
    const int s = t.sb[0] == b ? 0 : 1;
    hipError_t e = hipEventRecord(c->ev_free[s], c->stream);
    const int64_t nx = (b + 1) % (int64_t)t.plan.size();
    if (e == hipSuccess && t.sb[0] != nx && t.sb[1] != nx) e = stage_sparse(c, nx, s ^ 1);
    return e;
}

// A streamed shard's LDS layout for batch b, built on the device from the
// batch's CSR (just staged) and its streamed block bases.
hipError_t build_layout(dlr_ctx *c, int64_t b) {
    const TrainShard &t = c->train;
    if (!t.gpu_pcsc) return hipSuccess;
    return dlr::launch_pcsc_build(batch_view(c, b), t.pbase + (size_t)b * (size_t)(t.pblocks + 1), t.phases, t.pR,
                                  t.pblocks, t.gscratch, t.gends, t.grow, t.gval, c->stream);
}

// Batch b's rows as the dense kernels see them: the resident shard (rows
// from plan.first_row, wrapping), or the slot b is staged in (rows 0..B-1;
// the engine stream waits for its copy).
hipError_t dense_batch(dlr_ctx *c, int64_t b, dlr::DevDense *dd, int64_t *first) {
    TrainShard &t = c->train;
    if (!t.streamed) {
        *dd = {t.dX, t.label, t.n_rows, c->D, t.dtiled};
        *first = t.plan[(size_t)b].first_row;
        return hipSuccess;
    }
    int s = t.sb[0] == b ? 0 : t.sb[1] == b ? 1 : -1;
    hipError_t e = hipSuccess;
    if (s < 0) {
        s = (int)(b & 1);
        e = stage_dense(c, b, s);
    }
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_ready[s], 0);
    *dd = {t.sx[s], t.sl[s], t.plan[(size_t)b].rows, c->D};
    *first = 0;
    return e;
}

// After the last kernel that reads batch b's slot: release the slot and
// start copying the next batch into the other one (it overlaps this step's
// remaining work and the next margin's wait is only for what is left).
hipError_t dense_batch_done(dlr_ctx *c, int64_t b) {
    TrainShard &t = c->train;
    if (!t.streamed) return hipSuccess;
    const int s = t.sb[0] == b ? 0 : 1;
    hipError_t e = hipEventRecord(c->ev_free[s], c->stream);
    const int64_t nx = (b + 1) % (int64_t)t.plan.size();
    if (e == hipSuccess && t.sb[0] != nx && t.sb[1] != nx) e = stage_dense(c, nx, s ^ 1);
    return e;
}

// The windowed product margin (TrainShard::pmw) of rows [r0, r1) of batch b
// (r0 a multiple of kPmWinRows): per window, pass 1 from the current
// weights, then pass 2 into resid.  Same products and order as every margin:
// bitwise.
hipError_t launch_pm_windows(dlr_ctx *c, int64_t b, int64_t r0, int64_t r1) {
    const TrainShard &t = c->train;
    const dlr::DevBatch all = batch_view(c, b);
    r1 = std::min(r1, all.rows);
    hipError_t e = hipSuccess;
    for (int64_t wr0 = r0; e == hipSuccess && wr0 < r1; wr0 += t.pmw_slots * kPmWinRows) {
        const int64_t wi = t.pmw_first[(size_t)b] + wr0 / kPmWinRows;
        dlr::DevBatch sub = all;
        sub.row_ptr = all.row_ptr + wr0;
        sub.label = all.label + wr0;
        sub.rows = std::min(t.pmw_slots * kPmWinRows, r1 - wr0);
        const int64_t nwin = (sub.rows + kPmWinRows - 1) / kPmWinRows;
        e = dlr::launch_pm_windows(t.pmw_views + wi, pm_view(c, wi), nwin, sub, c->w, c->D, t.pm_p, t.pm_pstride,
                                   c->resid + wr0, c->stream);
    }
    return e;
}

// Whether batch b's pass 2 runs inside its fused gradient launch (one rank,
// k_grad_lds MG): launch_margin then forms only the products, if missing.
bool pm_mg_ok(const dlr_ctx *c, int64_t b) {
    const TrainShard &t = c->train;
    if (!t.pm_mg || c->comm || !t.pcsc) return false;
    if (t.rt)  // the row-round gradient (k_grad_rt MG)
        return dlr::grad_rt_mg_ok(pm_view(c, b), c->D, t.plan[(size_t)b].rows, t.rt_rounds, t.rt_val == nullptr);
    return dlr::grad_lds_mg_ok(pm_view(c, b), c->D, t.plan[(size_t)b].rows, t.phases, (int)(t.pR / 4096));
}

// rowsum_only (dlr_stage_time): the product margin's pass 2 alone, on
// whatever products pm_p holds (the same work; the residuals are not used).
// mg_next: the caller's next launch is batch b's fused gradient (one rank),
// which then runs the product margin's pass 2 itself when pm_mg_ok.
hipError_t launch_margin(dlr_ctx *c, int64_t b, bool rowsum_only = false, bool mg_next = false) {
    const TrainShard &t = c->train;
    if (t.dense) {
        dlr::DevDense dd;
        int64_t first;
        hipError_t e = dense_batch(c, b, &dd, &first);
        if (e != hipSuccess) return e;
        if (t.dref) return hipSuccess;  // one launch with the gradient (launch_gradient)
        if (t.dfused) return dlr::launch_dense_fused(dd, first, t.plan[(size_t)b].rows, c->w, t.dpart, c->stream);
        return dlr::launch_dense_margin(dd, first, t.plan[(size_t)b].rows, c->w, c->resid, c->stream);
    }
    if (t.pm) {
        // products of batch b from the current weights: made by the previous
        // step's fused gradient when it guessed b, else pass 1 now
        if (c->pm_ready != b && !rowsum_only) {
            const hipError_t e = dlr::launch_pm_products(pm_view(c, b), c->w, c->D, t.pm_p, c->stream);
            if (e != hipSuccess) return e;
        }
        if (mg_next && pm_mg_ok(c, b)) return hipSuccess;  // pass 2 runs in the gradient's launch (launch_gradient)
        c->pm_ready = -1;  // this step changes the weights
        return dlr::launch_pm_margin(pm_view(c, b), batch_view(c, b), t.pm_p, c->resid, c->stream);
    }
    if (t.margin_hot) return dlr::launch_margin_hot(batch_view(c, b), c->w, c->D, c->resid, c->stream);
    if (t.pmw) return launch_pm_windows(c, b, 0, t.plan[(size_t)b].rows);
    return dlr::launch_margin_residual(batch_view(c, b), c->w, c->resid, c->stream);
}

dlr::DevPcsc pcsc_view(const dlr_ctx *c, int64_t b) {
    const TrainShard &t = c->train;
    if (t.gpu_pcsc)  // built on the device for the current batch
        return {t.pbase + (size_t)b * (size_t)(t.pblocks + 1), t.gends, t.grow, t.gval, t.phases, (int)(t.pR / 4096)};
    return {t.pbase + (size_t)b * (size_t)(t.pblocks + 1), t.pends + (size_t)b * (size_t)t.pblocks * 64,
            t.prow + t.poff[(size_t)b], t.pval + t.poff[(size_t)b], t.phases, (int)(t.pR / 4096)};
}

dlr::DevCsc csc_view(const dlr_ctx *c, int64_t b) {
    const TrainShard &t = c->train;
    const size_t esz = t.row16 ? 2 : 4;
    const size_t po = t.touched ? (size_t)t.tpoff[(size_t)b] : (size_t)b * (size_t)(c->D + 1);
    dlr::DevCsc cs{t.cptr + po, (const char *)t.crow + esz * (size_t)t.coff[(size_t)b],
                   t.cval ? t.cval + t.coff[(size_t)b] : nullptr, t.row16};
    if (t.wsched) {
        cs.wstart = t.wsched + t.wsoff[(size_t)b];
        cs.nwaves = t.wsoff[(size_t)b + 1] - t.wsoff[(size_t)b] - 1;
    }
    return cs;
}

// The long columns of batch b (classic layout, §3's chunked option): in row
// phases (band mode: raw sums into gacc) or in chunks.
hipError_t launch_long_columns(dlr_ctx *c, int64_t b, int64_t B, float *gout, float lr, float C, bool fused) {
    const TrainShard &t = c->train;
    const size_t bb = (size_t)b;
    const size_t esz = t.row16 ? 2 : 4;
    const int64_t nl = t.any_long ? t.lcoff[bb + 1] - t.lcoff[bb] : 0;
    if (nl <= 0) return hipSuccess;
    if (t.lnph > 0) {
        dlr::DevLPhase lp{t.lpdesc + b * t.lnph, reinterpret_cast<const uint2 *>(t.lpptr), t.lpws, t.lprow, t.lpval,
                          t.lnph, (uint32_t)t.lnpart};
        return dlr::launch_long_phase(lp, t.lcols + t.lcoff[bb], t.lcseg + (t.lcoff[bb] + (int64_t)b), nl, c->resid,
                                      t.lpart, t.gacc, c->stream);
    }
    dlr::DevLong lg{t.lcols + t.lcoff[bb], t.lcseg + (t.lcoff[bb] + (int64_t)b), t.lsptr + t.lsoff[bb],
                    (const char *)t.lrow + esz * (size_t)t.leoff[bb], t.lval ? t.lval + t.leoff[bb] : nullptr, nl,
                    t.lsoff[bb + 1] - t.lsoff[bb] - 1, t.row16};
    if (t.lsched) lg.sched = t.lsched + t.lsoff[bb];
    return dlr::launch_grad_long(lg, B, c->resid, c->w, gout, t.lpart, lr, C, fused, c->stream,
                                 t.band_shift ? t.gacc : nullptr);
}

hipError_t launch_gradient(dlr_ctx *c, int64_t b, int64_t B, float *gout, float lr, float C, bool fused) {
    TrainShard &t = c->train;
    if (t.dense) {
        dlr::DevDense dd;
        int64_t first;
        hipError_t e = dense_batch(c, b, &dd, &first);
        if (e == hipSuccess && t.dref) {
            const int64_t nw = dlr::dense_ref_sync_words(B);
            const dlr::DevRefSync sy{t.dref_sync, t.dref_sync + nw - 64, t.dref_sync + nw - 32, t.dref_seq,
                                     t.dref_lead, 0, c->d_err, c->fault};
            CowaitScope cw(c, c->stream);
            e = cw.begin();
            if (e == hipSuccess)
                e = dlr::launch_dense_ref(dd, first, B, c->w, gout, c->resid, sy, lr, C, fused, c->stream);
            if (e == hipSuccess) ++c->train.dref_seq;
        } else if (e == hipSuccess)
            e = t.dfused ? dlr::launch_dense_combine(t.dpart, c->D, B, c->w, gout, lr, C, fused, c->stream)
                         : dlr::launch_dense_grad(dd, first, B, c->resid, c->w, gout, t.dpart, t.dblocked, lr, C, fused,
                                                  c->stream);
        if (e == hipSuccess) e = dense_batch_done(c, b);
        return e;
    }
    if (t.pcsc && t.rt) {
        const dlr::DevRt rt{t.rt_gq + t.rtoff[(size_t)b], t.rt_val ? t.rt_val + t.rtoff[(size_t)b] : nullptr,
                            t.rt_cend + (size_t)b * (size_t)t.pmS * dlr::kPmSlice, (int)t.rt_cap[(size_t)b],
                            t.rt_rounds};
        if (t.pm_fused && fused) {
            const int64_t nx = (b + 1) % (int64_t)t.plan.size();
            const dlr::DevPm next = pm_view(c, nx);
            if (pm_mg_ok(c, b)) {  // this batch's pass 2 in the same launch
                const dlr::DevP2 mg{pm_view(c, b), batch_view(c, b), c->resid, t.pm_cnt, t.pm_gen, c->d_err, c->fault};
                CowaitScope cw(c, c->stream);
                hipError_t e = cw.begin();
                if (e == hipSuccess)
                    e = dlr::launch_grad_rt(rt, c->D, B, c->resid, c->w, nullptr, lr, C, true, &next, t.pm_p, c->stream,
                                            &mg);
                if (e == hipSuccess) {
                    ++t.pm_gen;
                    c->pm_ready = nx;
                }
                return e;
            }
            const hipError_t e =
                dlr::launch_grad_rt(rt, c->D, B, c->resid, c->w, nullptr, lr, C, true, &next, t.pm_p, c->stream);
            if (e == hipSuccess) c->pm_ready = nx;
            return e;
        }
        return dlr::launch_grad_rt(rt, c->D, B, c->resid, c->w, gout, lr, C, fused, nullptr, nullptr, c->stream);
    }
    if (t.pcsc) {
        if (t.pm_fused && fused) {
            // the update, then the next batch's products from the new weights
            const int64_t nx = (b + 1) % (int64_t)t.plan.size();
            if (pm_mg_ok(c, b)) {
                const dlr::DevP2 mg{pm_view(c, b), batch_view(c, b), c->resid, t.pm_cnt, t.pm_gen, c->d_err, c->fault};
                CowaitScope cw(c, c->stream);
                hipError_t e = cw.begin();
                if (e == hipSuccess)
                    e = dlr::launch_grad_lds_pm(pcsc_view(c, b), c->D, B, c->resid, c->w, lr, C, pm_view(c, nx), t.pm_p,
                                                c->stream, &mg);
                if (e == hipSuccess) {
                    ++t.pm_gen;
                    c->pm_ready = nx;
                }
                return e;
            }
            const hipError_t e = dlr::launch_grad_lds_pm(pcsc_view(c, b), c->D, B, c->resid, c->w, lr, C,
                                                         pm_view(c, nx), t.pm_p, c->stream);
            if (e == hipSuccess) c->pm_ready = nx;
            return e;
        }
        return dlr::launch_grad_lds(pcsc_view(c, b), c->D, B, c->resid, c->w, gout, lr, C, fused, c->stream);
    }
    const size_t bb = (size_t)b;
    const size_t esz = t.row16 ? 2 : 4;
    hipError_t e = hipSuccess;
    if (t.band_shift) {
        // short columns band by band into gacc, the long columns' raw sums
        // into gacc, then the update of every column
        e = hipMemsetAsync(t.gacc, 0, (size_t)c->D * 4, c->stream);
        for (int64_t k = t.bfirst[bb]; e == hipSuccess && k < t.bfirst[bb + 1]; ++k) {
            const TrainShard::Band &bd = t.bands[(size_t)k];
            dlr::DevBand dv{t.bcols + bd.pair, t.bptr + bd.ptr, t.bws + bd.ws, (const char *)t.brow + esz * (size_t)bd.ent,
                            t.bval ? t.bval + bd.ent : nullptr, bd.nwaves, t.row16};
            e = dlr::launch_grad_band(dv, c->resid, t.gacc, c->stream, t.band_longrun);
        }
    } else {
        e = dlr::launch_grad(csc_view(c, b), c->D, c->resid, c->w, gout, B, lr, C, fused, c->stream);
    }
    if (e == hipSuccess) e = launch_long_columns(c, b, B, gout, lr, C, fused);
    if (e == hipSuccess && t.band_shift)
        e = dlr::launch_band_finalize(t.gacc, c->w, gout, c->D, B, lr, C, fused, c->stream);
    return e;
}

// Band mode (row bands; BASELINE C3), pipelined: a band's short-column
// gradient needs only the residuals of the band's own rows, so the margin
// runs band by band on the engine stream and each band's gradient kernel
// runs on a second stream as soon as its rows' margins exist, beside the
// next band's margin (the margin waits on fabric misses of the cold
// weights, the band kernel on L2 hits of its residual slice).  The long
// columns' phases need every residual: they follow the last margin on the
// engine stream; the update waits for both.  Same kernels, same sums:
// bitwise the sequential order.  False when the bands do not map onto the
// rows one to one (the caller then runs margin and gradient in sequence).
bool band_pipeline_ok(const dlr_ctx *c, int64_t b) {
    const TrainShard &t = c->train;
    if (tv(c->tune.band_pipeline, 1) == 0 || !t.band_shift || t.touched || t.dense || t.pcsc || t.sparse_stream) return false;
    const int64_t rows = t.plan[(size_t)b].rows, BR = (int64_t)1 << t.band_shift;
    return t.bfirst[(size_t)b + 1] - t.bfirst[(size_t)b] == (rows + BR - 1) / BR;
}

hipError_t band_step_pipelined(dlr_ctx *c, int64_t b, int64_t B, float *gout, float lr, float C, bool fused) {
    TrainShard &t = c->train;
    const size_t bb = (size_t)b;
    const int64_t nbands = t.bfirst[bb + 1] - t.bfirst[bb];
    hipError_t e = hipSuccess;
    if (!c->gstream) {
        e = hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_bstart, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_bdone, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    const bool hot = t.bhw != nullptr;
    // the hot columns' chains: ONE k_hot_chain launch over every band (the
    // hot-column product stream: the margins write the products, a flag per
    // band publishes them), or k_band_hot per band
    const bool hs = hot && t.hs;
    const int64_t nh = hs ? t.hs_nh[bb] : 0;
    // with hot chains beside it, the persistent margin leaves their CUs
    // (leaving 32-96 more to the other columns' band kernel measured no
    // better)
    const int margin_reserve = hs ? dlr::hot_chain_grid(nh) : hot ? (int)t.max_hot : 0;
    if (hot && !c->hstream) {
        e = hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_hdone, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_hmargins, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    while ((int64_t)c->ev_band.size() < nbands) {
        hipEvent_t ev;
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
        c->ev_band.push_back(ev);
    }
    const size_t esz = t.row16 ? 2 : 4;
    const dlr::DevBatch all = batch_view(c, b);
    const int64_t BR = (int64_t)1 << t.band_shift;
    // the hot chains wait inside the GPU for the margins beside them: the
    // whole step is one co-waiting sequence (CowaitScope; everything below
    // starts after the engine stream's first operation and joins it at the
    // end)
    std::optional<CowaitScope> cw;
    if (hs) {
        cw.emplace(c, c->stream);
        if ((e = cw->begin()) != hipSuccess) return e;
    }
    // the running sums are cleared on the engine stream (so the long-column
    // phases below are ordered after it too); the bands' stream starts
    // after that and everything queued before this step
    e = hipMemsetAsync(t.gacc, 0, (size_t)c->D * 4, c->stream);
    if (e == hipSuccess) e = hipEventRecord(c->ev_bstart, c->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->gstream, c->ev_bstart, 0);
    if (e == hipSuccess && hot) e = hipStreamWaitEvent(c->hstream, c->ev_bstart, 0);
    dlr::DevHotOut ho{};
    dlr::DevHotChain hc{};
    int64_t hc_end = kHsFirstGroup;  // the band after which the next chain launch is queued
    if (hs) {
        ++t.hs_seq;
        hc = dlr::DevHotChain{t.hs_cols + t.hsco[bb], t.hs_seg + t.hsso[bb], t.hs_buf, t.hs_flag, nh, nbands,
                              t.hs_seq, c->d_err, c->fault, t.hs_state, 0, 0, kHsGiveUpTicks, c->d_stat};
        ho = dlr::DevHotOut{t.hs_off + t.hsoo[bb], t.hs_dest, t.hs_val, t.hs_buf};
    }
    for (int64_t k = 0; e == hipSuccess && k < nbands; ++k) {
        const int64_t r0 = k * BR, r1 = std::min(all.rows, r0 + BR);
        dlr::DevBatch sub = all;
        sub.row_ptr = all.row_ptr + r0;
        sub.label = all.label + r0;
        sub.rows = r1 - r0;
        sub.nnz = all.rows > 0 ? all.nnz * sub.rows / all.rows : 0;  // the margin's rows-per-wave heuristic
        dlr::DevHotOut hk = ho;
        if (hk.off) hk.off += r0;  // the band's rows
        e = t.margin_hot ? dlr::launch_margin_hot(sub, c->w, c->D, c->resid + r0, c->stream, margin_reserve, hk)
            : t.pmw      ? launch_pm_windows(c, b, r0, r1)
                         : dlr::launch_margin_residual(sub, c->w, c->resid + r0, c->stream);
        if (e == hipSuccess && hs) e = dlr::launch_flag_store(t.hs_flag + k, t.hs_seq, c->stream);
        // the hot chains of bands [hc.b1, k + 1), queued after their margins
        // (DevHotChain): two launches, the first bands', then the rest's
        // (and the final one below)
        // after the last margin.  The host queues a band's launches ~4x
        // faster than the GPU runs its margin, and a chain adds a band ~3x
        // slower than the margins make one: the first launch is queued before
        // band 0's margin ends and the second long before the first's chains
        // end -- one launch boundary a step (C3: 5.72 ms; geometric groups,
        // 6 launches: 5.95 ms, each boundary a sync of chains of unequal
        // band lengths)
        if (e == hipSuccess && hs && (k + 1 == hc_end || k + 1 == nbands)) {
            hc.b0 = hc.b1;
            hc.b1 = k + 1;
            e = dlr::launch_hot_chain(hc, t.gacc, c->hstream);
            ++c->hcount[DLR_COUNT_HOT_CHAIN_LAUNCHES];
            hc_end = nbands;
        }
        if (e == hipSuccess) e = hipEventRecord(c->ev_band[(size_t)k], c->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->gstream, c->ev_band[(size_t)k], 0);
        const TrainShard::Band &bd = t.bands[(size_t)(t.bfirst[bb] + k)];
        const dlr::DevBand dv{t.bcols + bd.pair, t.bptr + bd.ptr, t.bws + bd.ws, (const char *)t.brow + esz * (size_t)bd.ent,
                              t.bval ? t.bval + bd.ent : nullptr, bd.nwaves, t.row16};
        if (e == hipSuccess) e = dlr::launch_grad_band(dv, c->resid, t.gacc, c->gstream, t.band_longrun, hot);
        // the hot pairs: their chains continue band after band on their own
        // stream, beside the next band's margin and the other columns
        if (e == hipSuccess && hot && !hs) e = hipStreamWaitEvent(c->hstream, c->ev_band[(size_t)k], 0);
        if (e == hipSuccess && hot && !hs) e = dlr::launch_band_hot(dv, t.bhw + bd.hw, bd.nhot, c->resid, t.gacc, c->hstream, c->d_err, c->fault);
    }
    // the final chain launch, ordered after the last margin by an event:
    // empty unless a launch above gave up on a flag (kernels run one at a
    // time, e.g. under counter collection, in an order the streams do not
    // fix) -- then it adds the rest; only it reports a missing flag
    if (e == hipSuccess && hs) {
        e = hipEventRecord(c->ev_hmargins, c->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->hstream, c->ev_hmargins, 0);
        if (e == hipSuccess) {
            dlr::DevHotChain fin = hc;
            fin.b0 = nbands;
            fin.b1 = nbands;
            fin.final_launch = 1;
            e = dlr::launch_hot_chain(fin, t.gacc, c->hstream);
            ++c->hcount[DLR_COUNT_HOT_CHAIN_LAUNCHES];
        }
    }
    if (e == hipSuccess) e = hipEventRecord(c->ev_bdone, c->gstream);
    if (e == hipSuccess && hot) e = hipEventRecord(c->ev_hdone, c->hstream);
    // the long columns' raw sums go to their own gacc entries (disjoint from
    // the short columns' the bands write)
    if (e == hipSuccess) e = launch_long_columns(c, b, B, gout, lr, C, fused);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_bdone, 0);
    if (e == hipSuccess && hot) e = hipStreamWaitEvent(c->stream, c->ev_hdone, 0);
    if (e == hipSuccess) e = dlr::launch_band_finalize(t.gacc, c->w, gout, c->D, B, lr, C, fused, c->stream);
    return e;
}

// The product margin's arrays (DevPm, and the row-round gradient's DevRt
// when allow_rt) for `spans` -- a shard's batches (their index is the
// batch's), or the 65,536-row WINDOWS of band-mode batches (TrainShard::
// pmw) -- uploaded back to back; built = false (nothing uploaded) when a
// span does not fit them or they would not leave the residency headroom
// (force: DLR_PM=1, that is an error).  slots: spans whose products pm_p
// holds at once (TrainShard::pm_pstride apart).
int build_pm(dlr_ctx *c, const CsrView &src, const std::vector<dlr::BatchSpan> &spans, bool allow_rt, bool force,
             int nthreads, int64_t &resid_need, int64_t &csc_bytes, bool &built, int64_t slots = 1) {
    TrainShard &t = c->train;
    const int64_t ns = (int64_t)spans.size(), D = c->D;
    const int64_t S = (D + dlr::kPmSlice - 1) / dlr::kPmSlice;
    int rc;
    built = false;
    std::vector<PmBatch> pm((size_t)ns);
    std::atomic<bool> ok{true};
    // the row-round gradient: by default for batches of <= 2 rounds
    // (C2 at B = 8,192: 7.5 vs 10.0 us for k_grad_lds); at 8 rounds
    // (B = 65,536) k_grad_lds is faster.  row_rounds 1
    // takes it for every batch that fits, 0 never.
    const int64_t rte = c->tune.row_rounds;
    int64_t maxrows = 0;
    for (const dlr::BatchSpan &sp : spans) maxrows = std::max(maxrows, sp.rows);
    const int64_t rounds = (maxrows + dlr::kRtRows - 1) / dlr::kRtRows;
    const bool want_rt = allow_rt && rounds <= dlr::kRtMaxRounds &&
                         (rte != DLR_AUTO ? rte != 0 : rounds <= 2);
    for_batches(ns, nthreads, [&](int64_t b) {
        if (ok && !pm_batch(src, spans[(size_t)b], D, t.unit, want_rt, pm[(size_t)b])) ok = false;
    });
    bool rt_fits = want_rt;
    if (ok) {
        // only where it leaves the headroom the residency choice keeps
        // (8 GiB): else the gather margin, which needs no extra arrays.
        // The row-round arrays are optional (k_grad_lds needs none of
        // them): they are counted separately and dropped if only they
        // do not fit.
        int64_t need = 0, need_rt = 0;
        for (const PmBatch &q : pm) {
            need += (int64_t)(q.list.size() * 4 + q.val.size() * 4 + q.pofs.size() * 4 + q.rg.size() * 8 +
                              q.qs.size() * 2 + q.lbeg.size() * 4);
            need_rt += (int64_t)(q.gq.size() * 4 + q.rval.size() * 4 + q.cend.size() * 2);
        }
        size_t fr = 0, tot = 0;
        HIPC(c, hipMemGetInfo(&fr, &tot));
        const double head = (double)((size_t)8 << 30);
        if ((double)need + head > (double)fr) {
            ok = false;
            if (force)
                return fail(c, DLR_E_NOMEM, "dlr_load_train: DLR_PM=1 but the product margin's arrays (" +
                                                std::to_string((long long)(need >> 20)) + " MiB) do not fit");
        }
        rt_fits = rt_fits && (double)(need + need_rt) + head <= (double)fr;
        if (!rt_fits)
            for (PmBatch &q : pm) {
                std::vector<uint32_t>().swap(q.gq);
                std::vector<float>().swap(q.rval);
                std::vector<uint16_t>().swap(q.cend);
            }
    }
    if (ok) {
        t.pmS = S;
        t.pmo_list.assign((size_t)ns + 1, 0);
        t.pmo_pofs.assign((size_t)ns + 1, 0);
        t.pmo_rg.assign((size_t)ns + 1, 0);
        t.pmo_qs.assign((size_t)ns + 1, 0);
        t.pm_rstride.clear();
        t.pm_qstride.clear();
        int64_t pcap = 0, maxslice = 0;
        for (int64_t b = 0; b < ns; ++b) {
            const PmBatch &q = pm[(size_t)b];
            t.pmo_list[(size_t)b + 1] = t.pmo_list[(size_t)b] + (int64_t)q.list.size() * 2;  // entries
            t.pmo_pofs[(size_t)b + 1] = t.pmo_pofs[(size_t)b] + (int64_t)q.pofs.size();
            t.pmo_rg[(size_t)b + 1] = t.pmo_rg[(size_t)b] + (int64_t)q.rg.size();
            t.pmo_qs[(size_t)b + 1] = t.pmo_qs[(size_t)b] + (int64_t)q.qs.size();
            pcap = std::max<int64_t>(pcap, q.rg.back());
            maxslice = std::max(maxslice, q.maxslice);
            t.pm_groups = std::max(t.pm_groups, q.groups);
            t.pm_rstride.push_back(q.rstride);
            t.pm_qstride.push_back(q.qstride);
        }
        t.pm_split = (int)std::min<int64_t>(16, std::max<int64_t>(1, (maxslice + 16383) / 16384));
        if (c->tune.pm_split != DLR_AUTO)  // pass-1 workgroups per slice (separate pass)
            t.pm_split = std::max(t.pm_split, (int)std::min<int64_t>(16, std::max<int64_t>(1, c->tune.pm_split)));
        // one device array per member: the batches' parts back to back
        // (offsets off[b] / div elements), each batch's host part
        // released once copied, so the host peak stays ~1x the layout
        auto cat_upload = [&](auto member, auto **dst, const std::vector<int64_t> &off, int64_t div,
                              size_t pad) -> int {
            using V = std::remove_reference_t<decltype(pm[0].*member)>;
            V v((size_t)(off.back() / div));
            for (int64_t b = 0; b < ns; ++b) {
                V &src = pm[(size_t)b].*member;
                std::copy(src.begin(), src.end(), v.begin() + off[(size_t)b] / div);
                V().swap(src);
            }
            return upload(c, dst, v.data(), v.size(), pad);
        };
        std::vector<int64_t> lboff((size_t)ns + 1);
        for (int64_t b = 0; b <= ns; ++b) lboff[(size_t)b] = b * (S + 1);
        const int64_t lbeg_n = lboff.back();
        if ((rc = cat_upload(&PmBatch::lbeg, &t.pm_lbeg, lboff, 1, 0))) return rc;
        if ((rc = cat_upload(&PmBatch::list, &t.pm_list, t.pmo_list, 2, 64))) return rc;  // 2 words / 4 entries
        if (!t.unit && (rc = cat_upload(&PmBatch::val, &t.pm_val, t.pmo_list, 1, 64))) return rc;
        if ((rc = cat_upload(&PmBatch::pofs, &t.pm_pofs, t.pmo_pofs, 1, 0))) return rc;
        if ((rc = cat_upload(&PmBatch::rg, &t.pm_rg, t.pmo_rg, 1, 0))) return rc;
        if ((rc = cat_upload(&PmBatch::qoff, &t.pm_qoff, t.pmo_rg, 1, 0))) return rc;
        if ((rc = cat_upload(&PmBatch::qs, &t.pm_qs, t.pmo_qs, 1, 8))) return rc;
        bool rt_all = rt_fits;
        for (const PmBatch &q : pm) rt_all = rt_all && !q.gq.empty();
        if (rt_all) {
            std::vector<int64_t> ceoff((size_t)ns + 1);
            t.rtoff.assign((size_t)ns + 1, 0);
            t.rt_cap.assign((size_t)ns, 0);
            for (int64_t b = 0; b < ns; ++b) {
                t.rtoff[(size_t)b + 1] = t.rtoff[(size_t)b] + (int64_t)pm[(size_t)b].gq.size();
                t.rt_cap[(size_t)b] = pm[(size_t)b].rtcap;
            }
            for (int64_t b = 0; b <= ns; ++b) ceoff[(size_t)b] = b * S * dlr::kPmSlice;
            if ((rc = cat_upload(&PmBatch::gq, &t.rt_gq, t.rtoff, 1, 0))) return rc;
            if (!t.unit && (rc = cat_upload(&PmBatch::rval, &t.rt_val, t.rtoff, 1, 0))) return rc;
            if ((rc = cat_upload(&PmBatch::cend, &t.rt_cend, ceoff, 1, 0))) return rc;
            t.rt = true;
            t.rt_rounds = (int)rounds;
            resid_need = std::max(resid_need, (int64_t)t.rt_rounds * dlr::kRtRows);
            csc_bytes += (int64_t)(t.rtoff.back() * (t.unit ? 4 : 8) + ceoff.back() * 2);
        } else {
            for (PmBatch &q : pm) {  // release the unused row-round host arrays now
                std::vector<uint32_t>().swap(q.gq);
                std::vector<float>().swap(q.rval);
                std::vector<uint16_t>().swap(q.cend);
            }
        }
        t.pm_pstride = (pcap + 64 + 63) / 64 * 64;
        const size_t pbytes = (size_t)t.pm_pstride * (size_t)std::max<int64_t>(1, slots) * 4;
        if ((rc = dev_alloc(c, (void **)&t.pm_p, pbytes))) return rc;
        HIPC(c, hipMemsetAsync(t.pm_p, 0, pbytes, c->stream));
        csc_bytes += (int64_t)(lbeg_n * 4 + t.pmo_list.back() * (t.unit ? 2 : 6) +
                               t.pmo_pofs.back() * 4 + t.pmo_rg.back() * 8 + t.pmo_qs.back() * 2 + t.pm_pstride * std::max<int64_t>(1, slots) * 4);
        built = true;
    }
    return DLR_OK;
}

}  // namespace

extern "C" {

int dlr_exchange_plan(int protocol, int64_t D, int world, int pieces, int64_t cap, int64_t *ops, int max_ops) {
    if (D <= 0 || world < 1 || world > dlr::kMaxRanks || pieces < 0 || pieces > kXPiecesMax || cap < 0 ||
        max_ops < 0 || (max_ops > 0 && !ops) || (protocol != DLR_EXCHANGE_KEY_RANGE && protocol != DLR_EXCHANGE_TOUCHED))
        return fail(nullptr, DLR_E_ARG, "dlr_exchange_plan: bad argument");
    const std::vector<dlr::CollOp> plan = dlr::exchange_plan(
        protocol == DLR_EXCHANGE_TOUCHED ? dlr::kXTouched : dlr::kXKeyRange, D, world, pieces, cap);
    for (size_t k = 0; k < plan.size() && (int)k < max_ops; ++k) {
        ops[4 * k] = plan[k].kind;
        ops[4 * k + 1] = plan[k].words;
        ops[4 * k + 2] = plan[k].off;
        ops[4 * k + 3] = plan[k].count;
    }
    return (int)plan.size();
}

int dlr_merge_range(const float *recv, int world, int64_t chunk, int64_t n, float *w_own, float lr, int mode) {
    if (!recv || !w_own || world < 1 || n < 0 || chunk < n || mode < 0 || mode > 2)
        return fail(nullptr, DLR_E_ARG, "dlr_merge_range: bad argument");
    for (int64_t i = 0; i < n; ++i) w_own[i] = dlr::server_apply(w_own[i], recv + i, chunk, world, lr, mode, false);
    return DLR_OK;
}

int dlr_merge_touched(const uint32_t *lists, int world, int64_t cap, const float *batch_rows, float *w, int64_t D,
                      float lr, float C, int mode) {
    if (!lists || !batch_rows || !w || world < 1 || world > dlr::kMaxRanks || cap < 0 || D <= 0 || mode < 0 ||
        mode > 2)
        return fail(nullptr, DLR_E_ARG, "dlr_merge_touched: bad argument");
    dlr::RankSizes rs{};
    rs.W = world;
    for (int r = 0; r < world; ++r) rs.Bf[r] = batch_rows[r];
    const int64_t stride = 1 + 2 * cap;
    for (int r = 0; r < world; ++r) {
        const uint32_t n = lists[(int64_t)r * stride];
        if ((int64_t)n > cap) return fail(nullptr, DLR_E_ARG, "dlr_merge_touched: count above cap");
        for (uint32_t s = 0; s < n; ++s)
            if (lists[(int64_t)r * stride + 1 + s] >= (uint64_t)D)
                return fail(nullptr, DLR_E_ARG, "dlr_merge_touched: column out of range");
    }
    // the engine's order: the owners' new weights from the OLD weights
    // (k_sparse_merge), the L2-only update of all D (k_dense_l2), then the
    // owners' weights over it (k_scatter)
    std::vector<std::pair<uint32_t, float>> out;
    for (int r = 0; r < world; ++r)
        for (int64_t s = 0; s < cap; ++s) {
            uint32_t col;
            float v;
            if (dlr::sparse_merge_entry(lists, cap, stride, w, rs, lr, C, mode, r, s, &col, &v)) out.push_back({col, v});
        }
    for (int64_t j = 0; j < D; ++j) w[j] = dlr::l2_only_update(w[j], rs, lr, C, mode);
    for (const auto &cv : out) w[cv.first] = cv.second;
    return DLR_OK;
}

int64_t dlr_rccl_trace(int protocol, int64_t D, int world, int rank, int pieces, int64_t cap, int steps, char *out,
                       int64_t size) {
    if (D <= 0 || world < 1 || world > dlr::kMaxRanks || rank < 0 || rank >= world || pieces < 0 ||
        pieces > kXPiecesMax || cap < 0 || steps < 0 || size < 0 || (size > 0 && !out) ||
        (protocol != DLR_EXCHANGE_KEY_RANGE && protocol != DLR_EXCHANGE_TOUCHED))
        return fail(nullptr, DLR_E_ARG, "dlr_rccl_trace: bad argument");
    std::string log;
    std::unique_ptr<dlr::Comm> comm(dlr::make_rccl_recorder(world, rank, &log));
    const std::vector<dlr::CollOp> plan = dlr::exchange_plan(
        protocol == DLR_EXCHANGE_TOUCHED ? dlr::kXTouched : dlr::kXKeyRange, D, world, pieces, cap);
    for (int st = 0; st < steps; ++st)
        for (const dlr::CollOp &op : plan) {
            std::string err;
            if (!dlr::issue(*comm, op, nullptr, nullptr, nullptr, err))
                return fail(nullptr, DLR_E_RCCL, "dlr_rccl_trace: " + err);
        }
    if (size > 0) {
        const size_t n = std::min<size_t>(log.size(), (size_t)size - 1);
        memcpy(out, log.data(), n);
        out[n] = '\0';
    }
    return (int64_t)log.size() + 1;
}

const char *dlr_last_error(const dlr_ctx *ctx) { return ctx ? ctx->err.c_str() : dlr::thread_error(); }

int dlr_get_unique_id(void *id_out) {
    if (!id_out) return DLR_E_ARG;
    std::string err;
    if (!dlr::rccl_unique_id(id_out, err)) return fail(nullptr, DLR_E_RCCL, err);
    return DLR_OK;
}

namespace {
// One rank's context on `device`; takes ownership of `comm` (may be null).
int create_ctx(int device, int rank, int world, int64_t D, dlr::Comm *comm, dlr_ctx **out) {
    std::unique_ptr<dlr::Comm> own(comm);
    *out = nullptr;
    auto c = std::make_unique<dlr_ctx>();
    c->device = device;
    c->rank = rank;
    c->world = world;
    c->D = D;
    c->chunk = (D + world - 1) / world;
    c->Dpad = c->chunk * world;
    if (const char *r = getenv("DLR_RESIDENCY"))  // default for dlr_set_residency
        c->residency = strcmp(r, "stream") == 0 ? DLR_RESIDENCY_STREAM
                       : strcmp(r, "device") == 0 ? DLR_RESIDENCY_DEVICE
                                                  : DLR_RESIDENCY_AUTO;
    HIPC(c.get(), hipSetDevice(device));
    HIPC(c.get(), hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    int rc;
    if ((rc = dev_alloc(c.get(), (void **)&c->w, (size_t)c->Dpad * 4))) return rc;
    HIPC(c.get(), hipMemsetAsync(c->w, 0, (size_t)c->Dpad * 4, c->stream));
    if ((rc = dev_alloc(c.get(), (void **)&c->correct, 64))) return rc;
    HIPC(c.get(), hipHostMalloc((void **)&c->h_correct, 64, hipHostMallocDefault));
    HIPC(c.get(), hipHostMalloc((void **)&c->h_ll, 64, hipHostMallocDefault));
    HIPC(c.get(), hipHostMalloc((void **)&c->h_err, (dlr::kErrWords + dlr::kStatWords) * 4,
                                hipHostMallocMapped | hipHostMallocCoherent));
    HIPC(c.get(), hipHostGetDevicePointer((void **)&c->d_err, c->h_err, 0));
    c->d_stat = c->d_err + dlr::kErrWords;
    clear_device_errors(c.get());
    clear_counters(c.get());
    // Gradient + receive buffers serve both the exchange and the
    // host-exchange (worker/server) entry points.
    if ((rc = dev_alloc(c.get(), (void **)&c->g, (size_t)c->Dpad * 4))) return rc;
    if ((rc = dev_alloc(c.get(), (void **)&c->recv, (size_t)c->Dpad * 4))) return rc;
    HIPC(c.get(), hipMemsetAsync(c->g, 0, (size_t)c->Dpad * 4, c->stream));
    HIPC(c.get(), hipStreamSynchronize(c->stream));
    c->comm = own.release();
    *out = c.release();
    return DLR_OK;
}
}  // namespace

int dlr_create(int device, int rank, int world, const void *unique_id, int64_t D, dlr_ctx **out) {
    if (!out || D <= 0 || world <= 0 || rank < 0 || rank >= world || (world > 1 && !unique_id))
        return fail(nullptr, DLR_E_ARG, "dlr_create: bad argument");
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return fail(nullptr, DLR_E_HIP, "dlr_create: hipSetDevice(" + std::to_string(device) + ") failed");
    }
    dlr::Comm *comm = nullptr;
    const char *force = getenv("DLR_FORCE_COLLECTIVES");
    if (world > 1 || (force && strcmp(force, "1") == 0)) {
        std::string err;
        comm = dlr::make_rccl_comm(world, rank, unique_id, err);
        if (!comm) return fail(nullptr, DLR_E_RCCL, err);
    }
    return create_ctx(device, rank, world, D, comm, out);
}

int dlr_create_group(int device, int world, int64_t D, dlr_ctx **out) {
    if (!out || D <= 0 || world <= 0 || world > dlr::kMaxRanks)
        return fail(nullptr, DLR_E_ARG, "dlr_create_group: bad argument");
    for (int r = 0; r < world; ++r) out[r] = nullptr;
    const char *ls = getenv("DLR_LOOPBACK_SYNC");  // "1": host-synchronous collectives (A/B)
    dlr::LoopGroup *g = dlr::make_loop_group(world, !(ls && strcmp(ls, "1") == 0));
    std::vector<dlr::Comm *> comms((size_t)world);
    for (int r = 0; r < world; ++r) comms[(size_t)r] = dlr::make_loopback_comm(g, r);  // endpoints own g
    for (int r = 0; r < world; ++r) {
        dlr::Comm *cm = comms[(size_t)r];
        comms[(size_t)r] = nullptr;
        const int rc = create_ctx(device, r, world, D, cm, &out[r]);
        if (rc) {
            for (auto *x : comms) delete x;
            for (int q = 0; q < r; ++q) {
                dlr_destroy(out[q]);
                out[q] = nullptr;
            }
            return rc;
        }
    }
    return DLR_OK;
}

int dlr_comm_info(const dlr_ctx *c, int *nranks, int *transport) {
    if (!c) return DLR_E_ARG;
    if (nranks) *nranks = c->comm ? c->comm->world() : 0;
    if (transport)
        *transport = !c->comm ? DLR_TRANSPORT_NONE
                     : strcmp(c->comm->kind(), "rccl") == 0 ? DLR_TRANSPORT_RCCL
                                                            : DLR_TRANSPORT_LOOPBACK;
    return DLR_OK;
}

int dlr_comm_abort(dlr_ctx *c, const char *why) {
    if (!c) return DLR_E_ARG;
    if (c->comm) c->comm->abort(why ? why : "aborted");
    return DLR_OK;
}

void dlr_destroy(dlr_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    cowait_forget(ctx);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->cstream) (void)hipStreamSynchronize(ctx->cstream);
    if (ctx->gstream) (void)hipStreamSynchronize(ctx->gstream);
    if (ctx->hstream) (void)hipStreamSynchronize(ctx->hstream);
    if (ctx->xstream) (void)hipStreamSynchronize(ctx->xstream);
    free_train(ctx);  // unregisters a streamed shard's host rows
    delete ctx->comm;  // RCCL: ncclCommDestroy; loopback: drops the group reference
    for (void *p : ctx->allocs) (void)hipFree(p);
    for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->h_correct) (void)hipHostFree(ctx->h_correct);
    if (ctx->h_ll) (void)hipHostFree(ctx->h_ll);
    if (ctx->h_err) (void)hipHostFree(ctx->h_err);
    for (int k = 0; k < 2; ++k) {
        if (ctx->ev_ready[k]) (void)hipEventDestroy(ctx->ev_ready[k]);
        if (ctx->ev_free[k]) (void)hipEventDestroy(ctx->ev_free[k]);
    }
    for (hipEvent_t e : ctx->ev_band) (void)hipEventDestroy(e);
    if (ctx->ev_bstart) (void)hipEventDestroy(ctx->ev_bstart);
    if (ctx->ev_bdone) (void)hipEventDestroy(ctx->ev_bdone);
    if (ctx->gstream) (void)hipStreamDestroy(ctx->gstream);
    if (ctx->ev_hdone) (void)hipEventDestroy(ctx->ev_hdone);
    if (ctx->ev_hmargins) (void)hipEventDestroy(ctx->ev_hmargins);
    if (ctx->hstream) (void)hipStreamDestroy(ctx->hstream);
    if (ctx->ev_xmerged) (void)hipEventDestroy(ctx->ev_xmerged);
    for (hipEvent_t e : ctx->ev_xpiece)
        if (e) (void)hipEventDestroy(e);
    if (ctx->xstream) (void)hipStreamDestroy(ctx->xstream);
    if (ctx->cstream) (void)hipStreamDestroy(ctx->cstream);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int dlr_set_weights(dlr_ctx *c, const float *w, int64_t D) {
    if (!c || !w || D != c->D) return fail(c, DLR_E_ARG, "dlr_set_weights: D mismatch");
    HIPC(c, hipSetDevice(c->device));
    std::vector<float> tmp;
    if (!c->perm.empty()) {  // internal column order
        tmp.resize((size_t)D);
        for (int64_t j = 0; j < D; ++j) tmp[(size_t)c->perm[(size_t)j]] = w[j];
        w = tmp.data();
    }
    c->pm_ready = -1;
    HIPC(c, hipMemcpyAsync(c->w, w, (size_t)D * 4, hipMemcpyHostToDevice, c->stream));
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    return DLR_OK;
}

int dlr_get_weights(dlr_ctx *c, float *w, int64_t D) {
    if (!c || !w || D != c->D) return fail(c, DLR_E_ARG, "dlr_get_weights: D mismatch");
    HIPC(c, hipSetDevice(c->device));
    if (c->perm.empty()) {
        HIPC(c, hipMemcpyAsync(w, c->w, (size_t)D * 4, hipMemcpyDeviceToHost, c->stream));
        if (int rc = wait_stream(c, c->stream, "dlr_get_weights")) return rc;
        return check_device(c, "dlr_get_weights");
    }
    std::vector<float> tmp((size_t)D);
    HIPC(c, hipMemcpyAsync(tmp.data(), c->w, (size_t)D * 4, hipMemcpyDeviceToHost, c->stream));
    if (int rc = wait_stream(c, c->stream, "dlr_get_weights")) return rc;
    if (int rc = check_device(c, "dlr_get_weights")) return rc;
    for (int64_t j = 0; j < D; ++j) w[j] = tmp[(size_t)c->perm[(size_t)j]];
    return DLR_OK;
}

// TrainShard::xslices for this rank: slice s (columns [4096 s, 4096 s +
// 4096) of the padded key space) is complete once every key range it
// overlaps has delivered its part -- this rank's own part at once, rank q's
// part [q chunk, q chunk + o] with piece o / xsub.
int build_overlap_groups(dlr_ctx *c) {
    TrainShard &t = c->train;
    const int64_t S = t.pmS, chunk = c->chunk, W = c->world;
    t.xsub = (chunk + t.xpieces - 1) / t.xpieces;
    std::vector<std::vector<uint32_t>> g((size_t)t.xpieces + 1);
    for (int64_t s = 0; s < S; ++s) {
        const int64_t a = s * dlr::kPmSlice, b = std::min((s + 1) * dlr::kPmSlice, c->D);
        int grp = 0;
        for (int64_t q = a / chunk; q < W && q * chunk < b; ++q) {
            if (q == c->rank) continue;
            const int64_t last = std::min(b, (q + 1) * chunk) - 1 - q * chunk;  // last word of q's part
            grp = std::max(grp, (int)(last / t.xsub) + 1);
        }
        g[(size_t)grp].push_back((uint32_t)s);
    }
    std::vector<uint32_t> all;
    t.xgofs.assign(1, 0);
    for (auto &v : g) {
        all.insert(all.end(), v.begin(), v.end());
        t.xgofs.push_back((int64_t)all.size());
    }
    return upload(c, &t.xslices, all.data(), all.size());
}

// The default piece count of the overlapped all-gather from the key range
// one rank owns (the same on every rank: D and W only).  Each piece is a
// collective with its own latency -- grouped RCCL sends and receives to
// every peer, tens of microseconds -- so a piece must carry enough of the
// range to be bandwidth-bound: one piece per 4 MiB of the range, 1 to 4.
// C2 (D = 1M: 4 MB of weights, <= 2 MB a rank at W >= 2) gets ONE piece,
// and then (coll_agree_pieced) no overlap at all: the plain in-place
// ncclAllGather, not W - 1 sends and receives per piece against a 28 us
// step.  An explicit dlr_set_exchange_pieces(1) keeps
// the overlap with one ncclAllGather (exchange_overlapped).
static int auto_pieces(int64_t chunk) {
    const int64_t bytes = chunk * 4;
    return (int)std::max<int64_t>(1, std::min<int64_t>(4, bytes / ((int64_t)4 << 20)));
}

// world > 1, product margin: the all-gather of the merged weights in pieces
// on the exchange stream, the next batch's pass 1 slice group by slice group
// on the engine stream as their weights land (the exchange
// overlapped with the next batch's margin).  Ends with the engine stream
// past every piece.
int exchange_overlapped(dlr_ctx *c, int64_t b, StepPlan &xp) {
    TrainShard &t = c->train;
    if (!c->xstream) {
        HIPC(c, hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking));
        HIPC(c, hipEventCreateWithFlags(&c->ev_xmerged, hipEventDisableTiming));
        for (hipEvent_t &e : c->ev_xpiece) HIPC(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const int64_t nx = (b + 1) % (int64_t)t.plan.size();
    const dlr::DevPm pm = pm_view(c, nx);
    HIPC(c, hipEventRecord(c->ev_xmerged, c->stream));
    HIPC(c, hipStreamWaitEvent(c->xstream, c->ev_xmerged, 0));
    auto pass1 = [&](int grp) -> hipError_t {
        const int64_t n = t.xgofs[(size_t)grp + 1] - t.xgofs[(size_t)grp];
        return dlr::launch_pm_products(pm, c->w, c->D, t.pm_p, c->stream, t.xslices + t.xgofs[(size_t)grp], n);
    };
    HIPC(c, pass1(0));  // inside this rank's own key range: ready now
    if (t.xpieces == 1) {
        // one piece: the plain in-place all-gather (one collective), then
        // pass 1 of every other slice
        const dlr::CollOp *op = xp.next(dlr::kCollAllGather);
        PLANC(c, op);
        XCHGC(c, op, c->w + (int64_t)c->rank * op->words, c->w, c->xstream);
        HIPC(c, hipEventRecord(c->ev_xpiece[0], c->xstream));
        HIPC(c, hipStreamWaitEvent(c->stream, c->ev_xpiece[0], 0));
        HIPC(c, pass1(1));
        c->pm_ready = nx;
        return DLR_OK;
    }
    for (int k = 0; k < t.xpieces; ++k) {
        const dlr::CollOp *op = xp.next(dlr::kCollAllGatherPart);
        PLANC(c, op);
        XCHGC(c, op, nullptr, c->w, c->xstream);
        HIPC(c, hipEventRecord(c->ev_xpiece[k], c->xstream));
        HIPC(c, hipStreamWaitEvent(c->stream, c->ev_xpiece[k], 0));
        HIPC(c, pass1(k + 1));
    }
    c->pm_ready = nx;
    return DLR_OK;
}

int dlr_load_train(dlr_ctx *c, const dlr_dataset *ds, int64_t batch_size, int64_t *n_batches) {
    if (!c) return fail(c, DLR_E_ARG, "dlr_load_train: bad argument");
    HIPC(c, hipSetDevice(c->device));
    load_tuning(c);
    {
        std::string msg;
        if (!ds)
            msg = "dlr_load_train: bad argument";
        else if (ds->D != c->D)
            msg = "dlr_load_train: dataset D != context D";
        else if (batch_size == 0)
            msg = "dlr_load_train: batch_size 0 (reference never terminates)";
        else if (ds->n_rows <= 0)
            msg = "dlr_load_train: empty shard (reference never terminates)";
        const int64_t nb = msg.empty() ? dlr_num_batches(ds->n_rows, batch_size) : 0;
        int rc = coll_agree_load(c, "dlr_load_train", msg.empty() ? DLR_OK : DLR_E_ARG, msg, nb);
        if (rc || (rc = coll_agree_order(c, "dlr_load_train"))) return rc;
    }
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    if (c->xstream)  // the pieced all-gather's stream carries collectives too
        if (int rc_ = wait_stream(c, c->xstream, __func__)) return rc_;
    free_train(c);
    TrainShard &t = c->train;
    t.xpieces = c->xpieces ? c->xpieces : auto_pieces(c->chunk);
    t.xauto = c->xpieces == 0;
    t.n_rows = ds->n_rows;
    t.nnz = (int64_t)ds->col.size();
    t.B = batch_size < 0 ? ds->n_rows : batch_size;
    if (t.B > INT32_MAX) return fail(c, DLR_E_ARG, "dlr_load_train: batch too large");
    t.plan = dlr::plan_batches(ds->n_rows, batch_size);
    const int64_t nb = (int64_t)t.plan.size();
    const int64_t D = c->D;
    // Per-batch entry counts (every batch has exactly B rows).
    t.coff.assign((size_t)nb + 1, 0);
    for (int64_t b = 0; b < nb; ++b) {
        const dlr::BatchSpan &sp = t.plan[(size_t)b];
        int64_t e;
        if (sp.contiguous) {
            e = ds->row_ptr[(size_t)(sp.first_row + sp.rows)] - ds->row_ptr[(size_t)sp.first_row];
        } else {
            e = 0;
            for (int64_t i = 0; i < sp.rows; ++i) {
                const int64_t r = (sp.first_row + i) % ds->n_rows;
                e += ds->row_ptr[(size_t)r + 1] - ds->row_ptr[(size_t)r];
            }
        }
        if (e > (int64_t)UINT32_MAX) return fail(c, DLR_E_ARG, "dlr_load_train: batch has > 2^32 entries");
        // 4-entry aligned batch bases: the kernels load entries 4 at a time.
        t.coff[(size_t)b + 1] = (t.coff[(size_t)b] + e + 3) & ~int64_t(3);
    }
    // Layout: the touched-column copy when the batches touch few of the D
    // columns (per-batch arrays over all D would dominate); decided
    // collectively, since it also picks the exchange (sparse all-gather vs
    // key-range all-to-all).  DLR_GRAD_KERNEL=touched forces it.
    int rc;
    const int64_t gk = c->tune.grad_layout;  // DLR_AUTO or a DLR_LAYOUT_*
    {
        const int64_t epb = std::max<int64_t>(1, t.coff[(size_t)nb] / std::max<int64_t>(1, nb));
        int64_t want = gk == DLR_LAYOUT_TOUCHED ? 1 : (gk != DLR_AUTO ? 0 : (D > 8 * epb ? 1 : 0));
        if ((rc = coll_max_i64(c, &want))) return rc;
        t.touched = want != 0;
        if (c->comm && c->world > dlr::kMaxRanks)
            return fail(c, DLR_E_ARG, "dlr_load_train: more than 16 ranks");
    }
    const double cptr_bytes = (double)nb * (double)(D + 1) * 4.0;
    if (!t.touched && cptr_bytes > 64.0 * (1ull << 30))
        return fail(c, DLR_E_NOMEM, "dlr_load_train: per-batch column pointers would need " +
                                        std::to_string((long long)(cptr_bytes / (1 << 20))) + " MiB");
    // Column numbering (frequency order for skewed shards; identity otherwise)
    // and the shard's columns in it.
    std::vector<int32_t> mapped;
    {
        std::vector<int32_t> np;
        if (!t.touched && (rc = column_order(c, *ds, np))) return rc;
        if ((rc = change_perm(c, std::move(np)))) return rc;
        // DLR_MARGIN_HOT=0|1 forces the LDS hot-weight margin (it needs D >=
        // kMarginHot); default: on for frequency-ordered shards
        const int64_t mh = c->tune.margin_hot;
        t.margin_hot = D >= dlr::kMarginHot && (mh != DLR_AUTO ? mh != 0 : !c->perm.empty());
        if (!c->perm.empty()) {
            mapped.resize(ds->col.size());
            const int nt = dlr::default_threads();
            std::vector<std::thread> th;
            for (int k = 0; k < nt; ++k)
                th.emplace_back([&, k] {
                    const size_t n = mapped.size();
                    for (size_t e = n * k / nt; e < n * (k + 1) / nt; ++e) mapped[e] = c->perm[(size_t)ds->col[e]];
                });
            for (auto &x : th) x.join();
        }
    }
    const CsrView src{ds->n_rows, ds->row_ptr.data(), c->perm.empty() ? ds->col.data() : mapped.data(),
                      ds->val.data()};
    t.unit = unit_values(c, ds->val);
    // Row bands (classic layout, DLR_BAND_ROWS: rows per band, rounded down
    // to a power of two; 0 = off; default 2^20 rows, a 4 MB residual slice,
    // for batches of >= 2 bands); the long columns then go in row phases.
    const bool brs = c->tune.band_rows != DLR_AUTO;  // forced
    const int64_t band_rows = tv(c->tune.band_rows, (int64_t)1 << 20);
    int shift = 0;
    while (band_rows > 0 && ((int64_t)2 << shift) <= band_rows) ++shift;
    const bool band = !t.touched && band_rows > 0 && shift > 0 &&
                      (brs ? t.B > ((int64_t)1 << shift) : t.B >= ((int64_t)2 << shift));
    // REFERENCE order: half-size bands (2^19 rows) by default -- the hot
    // columns' chains (k_band_hot) start after the first band's margin and
    // sync at each band boundary (C3: 7.0-7.3 ms vs 7.2-7.5 with 2^20, 7.4
    // with 2^18, 8.2 with 2^21; profiles/r04br*)
    if (band && !brs && c->order == DLR_ORDER_REFERENCE) shift -= 1;
    // Residency (K1, data_iter.h:40-55's batches): resident in HBM, or --
    // DLR_RESIDENCY_STREAM, or AUTO when the shard would not leave 8 GiB of
    // HBM free -- kept in page-locked host memory and staged batch by batch
    // into two device slots on the copy stream (every array below goes
    // through place()).  A band-mode batch (>= 2^21 rows) is one huge step:
    // streaming it per batch buys nothing, so it stays resident.
    {
        const double est = (double)t.nnz * (t.unit ? 10.0 : 16.0) + (double)t.n_rows * 16.0 +
                           (t.touched ? 0.0 : (double)nb * (double)(D + 1) * 4.0);
        bool stream = c->residency == DLR_RESIDENCY_STREAM;
        if (c->residency == DLR_RESIDENCY_AUTO) {
            size_t fr = 0, tot = 0;
            HIPC(c, hipMemGetInfo(&fr, &tot));
            stream = !band && est + (double)((size_t)8 << 30) > (double)fr;
        }
        // only an explicit STREAM request can fail here; every rank learns
        // of a failure on any rank (no rank is left waiting in a later load
        // collective)
        int64_t bad = stream && band ? 1 : 0;
        if ((rc = coll_max_i64(c, &bad))) return rc;
        if (bad)
            return fail(c, DLR_E_ARG, stream && band ? "dlr_load_train: a band-mode batch (>= 2^21 rows) cannot be "
                                                       "streamed per batch"
                                                     : "dlr_load_train: another rank cannot stream its band-mode batch");
        t.sparse_stream = stream;
        if (stream) {
            if (!c->cstream) HIPC(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
            for (int k = 0; k < 2; ++k) {
                if (!c->ev_ready[k]) HIPC(c, hipEventCreateWithFlags(&c->ev_ready[k], hipEventDisableTiming));
                if (!c->ev_free[k]) HIPC(c, hipEventCreateWithFlags(&c->ev_free[k], hipEventDisableTiming));
                HIPC(c, hipEventRecord(c->ev_free[k], c->stream));
            }
        }
    }
    // Shard CSR (no value array for a unit-valued shard).  Streamed: batch
    // b's rows [first, first + B) (the wrapping batch is materialised below
    // and stays resident).
    auto csr_rows = [&](int64_t extra) -> RangeFn {
        return [&, extra](int64_t b) -> std::pair<int64_t, int64_t> {
            const dlr::BatchSpan &sp = t.plan[(size_t)b];
            if (!sp.contiguous) return {0, 0};
            return {sp.first_row, sp.first_row + sp.rows + extra};
        };
    };
    const RangeFn csr_entries = [&](int64_t b) -> std::pair<int64_t, int64_t> {
        const dlr::BatchSpan &sp = t.plan[(size_t)b];
        if (!sp.contiguous) return {0, 0};
        return {ds->row_ptr[(size_t)sp.first_row] & ~int64_t(3), ds->row_ptr[(size_t)(sp.first_row + sp.rows)]};
    };
    if ((rc = place(c, &t.row_ptr, ds->row_ptr.data(), (size_t)t.n_rows + 1, 0, csr_rows(1)))) return rc;
    if ((rc = place(c, &t.col, src.col, (size_t)t.nnz, kPad, csr_entries))) return rc;
    if (!t.unit && (rc = place(c, &t.val, ds->val.data(), (size_t)t.nnz, kPad, csr_entries))) return rc;
    {
        std::vector<float> lab(ds->label.begin(), ds->label.end());
        if ((rc = place(c, &t.label, lab.data(), lab.size(), 0, csr_rows(0)))) return rc;
    }
    // Materialise the (at most one) wrapping batch.
    for (int64_t b = 0; b < nb; ++b) {
        const dlr::BatchSpan &sp = t.plan[(size_t)b];
        if (sp.contiguous) continue;
        t.wrap_batch = b;
        std::vector<int64_t> rp((size_t)sp.rows + 1);
        std::vector<int32_t> cc;
        std::vector<float> vv, ll((size_t)sp.rows);
        cc.reserve((size_t)(t.coff[(size_t)b + 1] - t.coff[(size_t)b]));
        vv.reserve(cc.capacity());
        rp[0] = 0;
        for (int64_t i = 0; i < sp.rows; ++i) {
            const int64_t r = (sp.first_row + i) % ds->n_rows;
            for (int64_t k = ds->row_ptr[(size_t)r]; k < ds->row_ptr[(size_t)r + 1]; ++k) {
                cc.push_back(src.col[(size_t)k]);
                vv.push_back(ds->val[(size_t)k]);
            }
            rp[(size_t)i + 1] = (int64_t)cc.size();
            ll[(size_t)i] = (float)ds->label[(size_t)r];
        }
        if ((rc = upload(c, &t.w_row_ptr, rp.data(), rp.size()))) return rc;
        if ((rc = upload(c, &t.w_col, cc.data(), cc.size(), kPad))) return rc;
        if (!t.unit && (rc = upload(c, &t.w_val, vv.data(), vv.size(), kPad))) return rc;
        if ((rc = upload(c, &t.w_label, ll.data(), ll.size()))) return rc;
        break;  // NextBatch wraps at most once per epoch
    }
    // Column-major copy of every batch: phase-split (LDS gradient kernel)
    // when the batch is small enough for LDS-resident residuals and every
    // phase block fits one window; else the classic layout.
    // DLR_GRAD_KERNEL=classic|lds forces a choice (lds still needs to fit).
    const int nthreads = dlr::default_threads();
    const bool force_classic = t.touched || gk == DLR_LAYOUT_CLASSIC;
    int64_t csc_bytes = 0;
    int64_t resid_need = t.B;
    PcscBuild pb;
    if (!force_classic && t.B <= 65536 && D <= (int64_t)1 << 31) {
        pb.R = dlr::grad_lds_phase_rows(t.B);
        pb.P = (int)((t.B + pb.R - 1) / pb.R);
        pb.groups = (D + 63) / 64;
        pb.pblocks = pb.groups * pb.P;
        t.pcsc = pb.P <= 4 && pcsc_plan(src, t.plan, D, pb, nthreads);
    }
    if (gk == DLR_LAYOUT_LDS && !t.pcsc)
        return fail(c, DLR_E_ARG, "dlr_load_train: DLR_GRAD_KERNEL=lds but the batches do not fit the LDS layout");
    if (t.pcsc) {
        t.phases = pb.P;
        t.pR = pb.R;
        t.pblocks = pb.pblocks;
        t.poff.assign((size_t)nb + 1, 0);
        for (int64_t b = 0; b < nb; ++b) t.poff[(size_t)b + 1] = t.poff[(size_t)b] + pb.size[(size_t)b];
        const int64_t total = t.poff[(size_t)nb];
        std::vector<uint32_t> base((size_t)nb * (size_t)(pb.pblocks + 1));
        t.gpu_pcsc = t.sparse_stream && tv(c->tune.stream_device_layout, 1) != 0;
        if (t.gpu_pcsc) {
            pcsc_bases(src, t.plan, D, pb, base, nthreads);
            const int64_t pbk = pb.pblocks;
            const RangeFn r_base = [&](int64_t b) { return std::make_pair(b * (pbk + 1), (b + 1) * (pbk + 1)); };
            if ((rc = place(c, &t.pbase, base.data(), base.size(), 0, r_base))) return rc;
            int64_t maxsz = 0;
            for (int64_t b = 0; b < nb; ++b) maxsz = std::max(maxsz, pb.size[(size_t)b]);
            t.pR = pb.R;
            if ((rc = dev_alloc(c, (void **)&t.gends, (size_t)pbk * 64))) return rc;
            if ((rc = dev_alloc(c, (void **)&t.grow, (size_t)(maxsz + 256) * 2))) return rc;
            if ((rc = dev_alloc(c, (void **)&t.gval, (size_t)(maxsz + 256) * 4))) return rc;
            if ((rc = dev_alloc(c, (void **)&t.gscratch, (size_t)pbk * 64 * 4))) return rc;
            HIPC(c, hipMemsetAsync(t.grow, 0, (size_t)(maxsz + 256) * 2, c->stream));  // padded window reads
            HIPC(c, hipMemsetAsync(t.gval, 0, (size_t)(maxsz + 256) * 4, c->stream));
            csc_bytes = (int64_t)(pbk * 64 * 5 + (maxsz + 256) * 6);
            t.bytes += csc_bytes;  // one batch's device-built layout (streamed: not in the slots)
            resid_need = (int64_t)pb.P * pb.R;
        }
        if (!t.gpu_pcsc) {
            std::vector<uint8_t> ends((size_t)nb * (size_t)pb.pblocks * 64);
            std::vector<uint16_t> prow((size_t)total, 0);
            std::vector<float> pval((size_t)total, 0.0f);
            pcsc_fill(src, t.plan, D, pb, t.poff, base, ends, prow, pval, nthreads);
            const int64_t pbk = pb.pblocks;
            const RangeFn r_base = [&](int64_t b) { return std::make_pair(b * (pbk + 1), (b + 1) * (pbk + 1)); };
            const RangeFn r_ends = [&](int64_t b) { return std::make_pair(b * pbk * 64, (b + 1) * pbk * 64); };
            const RangeFn r_ent = [&](int64_t b) { return std::make_pair(t.poff[(size_t)b], t.poff[(size_t)b + 1]); };
            if ((rc = place(c, &t.pbase, base.data(), base.size(), 0, r_base))) return rc;
            if ((rc = place(c, &t.pends, ends.data(), ends.size(), 0, r_ends))) return rc;
            if ((rc = place(c, &t.prow, prow.data(), prow.size(), 256, r_ent))) return rc;
            if ((rc = place(c, &t.pval, pval.data(), pval.size(), 256, r_ent))) return rc;
            csc_bytes = (int64_t)(base.size() * 4 + ends.size() + (total + 256) * 6);
            resid_need = (int64_t)pb.P * pb.R;  // the fills read whole phases
        }
        // Product margin (dlr_kernels.hip "Product margin"): resident shards
        // whose batches fit it, with enough column slices to fill the GPU
        // (DLR_PM=0 off, =1 on whenever the batches fit).
        const int64_t pme = c->tune.product_margin;  // DLR_AUTO, 0 off, 1 required
        const int64_t S = (D + dlr::kPmSlice - 1) / dlr::kPmSlice;
        if (!t.sparse_stream && pme != 0 && (pme == 1 || S >= 128)) {
            bool built = false;
            if ((rc = build_pm(c, src, t.plan, true, pme == 1, nthreads, resid_need, csc_bytes, built)))
                return rc;
            if (built) {
                t.pm = true;
                t.pm_fused = !c->comm && tv(c->tune.pm_fused, 1) != 0;
                // the margin inside the gradient launch (pm_in_gradient 0: its
                // own launch, k_pm_margin)
                t.pm_mg = t.pm_fused && tv(c->tune.pm_in_gradient, 1) != 0;
                t.mg_demoted = t.pm_mg && c->mg_demoted;
                if (t.mg_demoted) t.pm_mg = false;
                // ... only if every batch's launch is resident at once
                // (grad_lds_mg_ok / grad_rt_mg_ok; otherwise pass 2 runs in
                // k_pm_margin)
                for (int64_t b = 0; t.pm_mg && b < nb; ++b)
                    t.pm_mg = t.rt ? dlr::grad_rt_mg_ok(pm_view(c, b), c->D, t.plan[(size_t)b].rows, t.rt_rounds,
                                                        t.rt_val == nullptr)
                                   : dlr::grad_lds_mg_ok(pm_view(c, b), c->D, t.plan[(size_t)b].rows, t.phases,
                                                         (int)(t.pR / 4096));
                if (t.pm_mg) {
                    const size_t cb = (size_t)dlr::DevP2::kMgCntWords * 4;
                    if ((rc = dev_alloc(c, (void **)&t.pm_cnt, cb))) return rc;
                    HIPC(c, hipMemsetAsync(t.pm_cnt, 0, cb, c->stream));
                    t.pm_gen = 0;
                }
                if (c->comm && (rc = build_overlap_groups(c))) return rc;
            } else if (pme == 1) {
                return fail(c, DLR_E_ARG, "dlr_load_train: DLR_PM=1 but the batches do not fit the product margin");
            }
        }
    } else if (t.touched) {
        t.row16 = t.B <= 65536;
        std::vector<TouchedBatch> tbs((size_t)nb);
        for_batches(nb, nthreads, [&](int64_t b) { touched_batch(src, t.plan[(size_t)b], tbs[(size_t)b]); });
        t.tcoff.assign((size_t)nb + 1, 0);
        t.tpoff.assign((size_t)nb + 1, 0);
        t.tncols.assign((size_t)nb, 0);
        int64_t cap = 1;
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t n = (int64_t)tbs[(size_t)b].cols.size();
            t.tncols[(size_t)b] = n;
            t.tcoff[(size_t)b + 1] = t.tcoff[(size_t)b] + n;
            t.tpoff[(size_t)b + 1] = t.tpoff[(size_t)b] + n + 1;
            cap = std::max(cap, n);
        }
        if ((rc = coll_max_i64(c, &cap))) return rc;
        t.tcap = cap;
        const int64_t total = t.coff[(size_t)nb];
        std::vector<uint32_t> tcols((size_t)t.tcoff[(size_t)nb]), tptr((size_t)t.tpoff[(size_t)nb]);
        std::vector<float> cval((size_t)total, 0.0f);
        std::vector<uint32_t> crow32;
        std::vector<uint16_t> crow16;
        if (t.row16)
            crow16.assign((size_t)total, 0);
        else
            crow32.assign((size_t)total, 0);
        for (int64_t b = 0; b < nb; ++b) {
            const TouchedBatch &tb = tbs[(size_t)b];
            std::copy(tb.cols.begin(), tb.cols.end(), tcols.begin() + t.tcoff[(size_t)b]);
            std::copy(tb.ptr.begin(), tb.ptr.end(), tptr.begin() + t.tpoff[(size_t)b]);
            const size_t o = (size_t)t.coff[(size_t)b];
            std::copy(tb.val.begin(), tb.val.end(), cval.begin() + o);
            for (size_t k = 0; k < tb.row.size(); ++k) {
                if (t.row16)
                    crow16[o + k] = (uint16_t)tb.row[k];
                else
                    crow32[o + k] = tb.row[k];
            }
        }
        tbs.clear();
        const RangeFn r_cols = [&](int64_t b) { return std::make_pair(t.tcoff[(size_t)b], t.tcoff[(size_t)b + 1]); };
        const RangeFn r_ptr = [&](int64_t b) { return std::make_pair(t.tpoff[(size_t)b], t.tpoff[(size_t)b + 1]); };
        const RangeFn r_ent = [&](int64_t b) { return std::make_pair(t.coff[(size_t)b], t.coff[(size_t)b + 1]); };
        if ((rc = place(c, &t.tcols, tcols.data(), tcols.size(), 64, r_cols))) return rc;
        if ((rc = place(c, &t.cptr, tptr.data(), tptr.size(), 0, r_ptr))) return rc;
        if (t.row16) {
            if ((rc = place(c, (uint16_t **)&t.crow, crow16.data(), crow16.size(), kPad, r_ent))) return rc;
        } else {
            if ((rc = place(c, (uint32_t **)&t.crow, crow32.data(), crow32.size(), kPad, r_ent))) return rc;
        }
        if (!t.unit && (rc = place(c, &t.cval, cval.data(), cval.size(), kPad, r_ent))) return rc;
        csc_bytes = (int64_t)(tcols.size() * 4 + tptr.size() * 4 +
                              (total + kPad) * ((t.row16 ? 2 : 4) + (t.unit ? 0 : 4)));
        // step buffers and every rank's batch size (L2 term of its pushes)
        free_touched_bufs(c);
        std::vector<float> bs;
        if ((rc = coll_gather_f32(c, (float)t.B, bs))) return rc;
        c->rs.W = (int)bs.size();
        for (int r = 0; r < c->rs.W; ++r) c->rs.Bf[r] = bs[(size_t)r];
        if ((rc = dev_alloc(c, (void **)&c->newv, (size_t)cap * 4))) return rc;
        if (c->comm) {
            const int64_t stride = 1 + 2 * cap;
            if ((rc = dev_alloc(c, (void **)&c->xsend, (size_t)stride * 4))) return rc;
            if ((rc = dev_alloc(c, (void **)&c->xrecv, (size_t)stride * 4 * c->world))) return rc;
            if ((rc = dev_alloc(c, (void **)&c->xcols, (size_t)cap * 4 * c->world))) return rc;
            if ((rc = dev_alloc(c, (void **)&c->xnewv, (size_t)cap * 4 * c->world))) return rc;
        }
        c->xcap = cap;
    } else {
        t.row16 = t.B <= 65536;
        const int64_t total = t.coff[(size_t)nb];
        if (total >= (int64_t)1 << 31) return fail(c, DLR_E_ARG, "dlr_load_train: a batch has >= 2^31 entries");
        std::vector<uint32_t> cptr((size_t)nb * (size_t)(D + 1));
        std::vector<float> cval(t.unit ? 0 : (size_t)total);
        // Long columns (more than long_min entries in a batch; 0 = none):
        // only under DLR_ORDER_FAST are they summed in a fixed chunked /
        // phase order instead of the reference's single sequential chain
        // (DESIGN.md 3).  FAST's threshold: 2,048 in band mode (C3's
        // 2^21+-row batches, ~10^6-entry chains; 2,048 measured best of
        // 512..16,384, profiles/r03t_*), otherwise 2^17; DLR_LONG_COLUMN
        // overrides the FAST threshold (A/B) and never changes the
        // reference order.
        const int64_t lm = c->tune.long_column;
        const int64_t long_min = c->order != DLR_ORDER_FAST ? 0 : lm != DLR_AUTO ? lm : band ? 2048 : ((int64_t)1 << 17);
        int64_t lbytes = 0;
        auto finish_long = [&](auto &lb) -> int {
            // concatenate the batches' long columns
            using RowT = typename std::decay_t<decltype(lb[0].row)>::value_type;
            t.lcoff.assign((size_t)nb + 1, 0);
            t.lsoff.assign((size_t)nb + 1, 0);
            t.leoff.assign((size_t)nb + 1, 0);
            int64_t maxseg = 0;
            for (int64_t b = 0; b < nb; ++b) {
                t.lcoff[(size_t)b + 1] = t.lcoff[(size_t)b] + (int64_t)lb[(size_t)b].cols.size();
                t.lsoff[(size_t)b + 1] = t.lsoff[(size_t)b] + (int64_t)lb[(size_t)b].sptr.size();
                t.leoff[(size_t)b + 1] = t.leoff[(size_t)b] + (int64_t)lb[(size_t)b].row.size();
                maxseg = std::max<int64_t>(maxseg, (int64_t)lb[(size_t)b].sptr.size());
            }
            t.any_long = t.lcoff[(size_t)nb] > 0;
            if (!t.any_long) return DLR_OK;
            if (band) {
                LPhaseBuild ph;
                build_long_phases(lb, t.B, t.unit, long_piece(c->tune), ph);
                std::vector<uint32_t> cols;
                for (auto &L : lb) {
                    cols.insert(cols.end(), L.cols.begin(), L.cols.end());
                    L = {};
                }
                int r;
                t.lnph = (t.B + dlr::kLPhase - 1) / dlr::kLPhase;
                if ((r = upload(c, &t.lcols, cols.data(), cols.size()))) return r;
                if ((r = upload(c, &t.lcseg, ph.cseg.data(), ph.cseg.size()))) return r;
                if ((r = upload(c, &t.lpdesc, ph.desc.data(), ph.desc.size()))) return r;
                {  // (piece pointer, partial slot) pairs, one 8-byte load per piece
                    std::vector<uint32_t> ps(ph.ptr.size() * 2);
                    for (size_t q = 0; q < ph.ptr.size(); ++q) {
                        ps[2 * q] = ph.ptr[q];
                        ps[2 * q + 1] = ph.slot[q];
                    }
                    if ((r = upload(c, &t.lpptr, ps.data(), ps.size()))) return r;
                }
                if ((r = upload(c, &t.lpws, ph.ws.data(), ph.ws.size()))) return r;
                // a full window of padding: k_long_phase loads whole windows unclamped
                if ((r = upload(c, &t.lprow, ph.row.data(), ph.row.size(), (size_t)dlr::kLPWinPad))) return r;
                if (!t.unit && (r = upload(c, &t.lpval, ph.val.data(), ph.val.size(), (size_t)dlr::kLPWinPad)))
                    return r;
                if (ph.maxpart > (int64_t)UINT32_MAX - 64) return fail(c, DLR_E_ARG, "too many long-column pieces");
                t.lnpart = ph.maxpart;
                if ((r = dev_alloc(c, (void **)&t.lpart, (size_t)(ph.maxpart + 64) * 4))) return r;
                lbytes = (int64_t)(cols.size() * 4 + ph.cseg.size() * 4 + ph.desc.size() * sizeof(dlr::PhaseDesc) +
                                   (ph.ptr.size() * 2 + ph.ws.size()) * 4 + (ph.row.size() + dlr::kLPWinPad) * (t.unit ? 2 : 6) +
                                   ph.maxpart * 4);
                resid_need = std::max(resid_need, t.lnph * (int64_t)dlr::kLPhase);
                return DLR_OK;
            }
            std::vector<uint32_t> cols, cseg, sptr, sched;
            std::vector<RowT> row;
            std::vector<float> val;
            for (auto &L : lb) {
                // chunk schedule: by first row (stable), padded to sptr's length
                const size_t ns = L.sptr.empty() ? 0 : L.sptr.size() - 1;
                std::vector<uint32_t> order(ns);
                for (size_t k = 0; k < ns; ++k) order[k] = (uint32_t)k;
                std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
                    return L.row[L.sptr[x] & ~3u] < L.row[L.sptr[y] & ~3u];
                });
                sched.insert(sched.end(), order.begin(), order.end());
                if (!L.sptr.empty()) sched.push_back(0);
                cols.insert(cols.end(), L.cols.begin(), L.cols.end());
                cseg.insert(cseg.end(), L.cseg.begin(), L.cseg.end());
                sptr.insert(sptr.end(), L.sptr.begin(), L.sptr.end());
                row.insert(row.end(), L.row.begin(), L.row.end());
                val.insert(val.end(), L.val.begin(), L.val.end());
                L = {};
            }
            int r;
            const RangeFn r_cols = [&](int64_t b) { return std::make_pair(t.lcoff[(size_t)b], t.lcoff[(size_t)b + 1]); };
            const RangeFn r_cseg = [&](int64_t b) {
                return std::make_pair(t.lcoff[(size_t)b] + b, t.lcoff[(size_t)b + 1] + b + 1);
            };
            const RangeFn r_seg = [&](int64_t b) { return std::make_pair(t.lsoff[(size_t)b], t.lsoff[(size_t)b + 1]); };
            const RangeFn r_ent = [&](int64_t b) { return std::make_pair(t.leoff[(size_t)b], t.leoff[(size_t)b + 1]); };
            if ((r = place(c, &t.lcols, cols.data(), cols.size(), 0, r_cols))) return r;
            if ((r = place(c, &t.lcseg, cseg.data(), cseg.size(), 0, r_cseg))) return r;
            if ((r = place(c, &t.lsptr, sptr.data(), sptr.size(), 0, r_seg))) return r;
            if (tv(c->tune.long_sched, 1) != 0 &&
                (r = place(c, &t.lsched, sched.data(), sched.size(), 0, r_seg)))
                return r;
            if ((r = place(c, (RowT **)&t.lrow, row.data(), row.size(), dlr::kLongChunk, r_ent))) return r;
            if (!t.unit && (r = place(c, &t.lval, val.data(), val.size(), dlr::kLongChunk, r_ent))) return r;
            if ((r = dev_alloc(c, (void **)&t.lpart, (size_t)maxseg * 4))) return r;
            lbytes = (int64_t)(cols.size() * 4 + cseg.size() * 4 + sptr.size() * 4 + row.size() * sizeof(RowT) +
                               val.size() * 4);
            return DLR_OK;
        };
        auto classic = [&](auto &crow, auto &lb) -> int {
            using RowT = typename std::decay_t<decltype(crow)>::value_type;
            build_csc(src, t.plan, D, t.coff, cptr, crow, cval, long_min, lb, t.unit, nthreads);
            int r;
            if ((r = finish_long(lb))) return r;
            if (!band) {
                const RangeFn r_ent = [&](int64_t b) { return std::make_pair(t.coff[(size_t)b], t.coff[(size_t)b + 1]); };
                if ((r = place(c, (RowT **)&t.crow, crow.data(), crow.size(), kPad, r_ent))) return r;
                return DLR_OK;
            }
            BandBuild<RowT> bb;
            // REFERENCE order: the hot columns' pairs run in k_band_hot
            // (DLR_BAND_HOT: entries in the batch that make a column hot;
            // 0 = none)
            int64_t hot_min = long_min == 0 ? tv(c->tune.band_hot, (int64_t)1 << 17) : 0;
            // with the hot-column product stream: at most hs_max_cols() hot
            // columns a batch (the hottest; the others' chains run in
            // k_grad_band, band by band)
            if (hot_min > 0 && t.margin_hot && hot_stream_wanted(c))
                hot_min = hot_stream_threshold(c, cptr, nb, D, hot_min);
            build_bands(cptr, crow, cval, t.coff, nb, D, t.B, shift, t.unit, nthreads, hot_min, bb);
            t.band_shift = shift;
            // the software-pipelined band kernel only where a pair spans
            // windows (REFERENCE order keeps long runs in the bands: C3's
            // Zipf heads); with every wave one window (C2 at B = -1: ~25
            // entries a pair) its prefetches of the next two windows are
            // clamped re-reads -- 3x the loads, 2x the gathers
            t.band_longrun = long_min == 0 && bb.max_pair > kWinEntries;
            t.bands = std::move(bb.bands);
            t.bfirst = std::move(bb.bfirst);
            if ((r = upload(c, &t.bcols, bb.cols.data(), bb.cols.size(), 64))) return r;
            if ((r = upload(c, &t.bptr, bb.ptr.data(), bb.ptr.size()))) return r;
            if ((r = upload(c, &t.bws, bb.ws.data(), bb.ws.size()))) return r;
            if (!bb.hw.empty() && (r = upload(c, &t.bhw, bb.hw.data(), bb.hw.size()))) return r;
            for (const TrainShard::Band &x : t.bands) t.max_hot = std::max(t.max_hot, x.nhot);
            if (hot_min > 0 && t.margin_hot && (r = build_hot_stream(c, cptr, crow, cval, hot_min, shift))) return r;
            csc_bytes += t.hs_bytes;
            if ((r = upload(c, (RowT **)&t.brow, bb.row.data(), bb.row.size(), kPad))) return r;
            if (!t.unit && (r = upload(c, &t.bval, bb.val.data(), bb.val.size(), kPad))) return r;
            if ((r = dev_alloc(c, (void **)&t.gacc, (size_t)D * 4))) return r;
            csc_bytes += (int64_t)((bb.cols.size() + bb.ptr.size() + bb.ws.size()) * 4 +
                                   (bb.row.size() + kPad) * (sizeof(RowT) + (t.unit ? 0 : 4)) + D * 4);
            return DLR_OK;
        };
        if (t.row16) {
            std::vector<uint16_t> crow((size_t)total);
            std::vector<LongBatch<uint16_t>> lb;
            if ((rc = classic(crow, lb))) return rc;
        } else {
            std::vector<uint32_t> crow((size_t)total);
            std::vector<LongBatch<uint32_t>> lb;
            if ((rc = classic(crow, lb))) return rc;
        }
        if (!band) {
            const RangeFn r_ptr = [&](int64_t b) { return std::make_pair(b * (D + 1), (b + 1) * (D + 1)); };
            const RangeFn r_ent = [&](int64_t b) { return std::make_pair(t.coff[(size_t)b], t.coff[(size_t)b + 1]); };
            if ((rc = place(c, &t.cptr, cptr.data(), cptr.size(), 0, r_ptr))) return rc;
            if (!t.unit && (rc = place(c, &t.cval, cval.data(), cval.size(), kPad, r_ent))) return rc;
        }
        // Entry-balanced wave schedule: a wave takes consecutive columns until
        // it has 64 or about one window (kWin entries) of them -- a column
        // order with runs of long columns (frequency order) would otherwise
        // give some waves 64 x thousands of entries.
        if (!band) {
            std::vector<std::vector<uint32_t>> ws((size_t)nb);
            for_batches(nb, nthreads, [&](int64_t b) {
                const uint32_t *cp = cptr.data() + (size_t)b * (size_t)(D + 1);
                std::vector<uint32_t> &v = ws[(size_t)b];
                v.reserve((size_t)(D / 64 + 16));
                v.push_back(0);
                int64_t acc = 0;
                int cols = 0;
                for (int64_t j = 0; j < D; ++j) {
                    const int64_t cj = (int64_t)(cp[j + 1] & 0x7FFFFFFFu) - (int64_t)(cp[j] & 0x7FFFFFFFu);
                    if (cols == 64 || (cols > 0 && acc + cj > 1024)) {
                        v.push_back((uint32_t)j);
                        acc = 0;
                        cols = 0;
                    }
                    acc += cj;
                    ++cols;
                }
                v.push_back((uint32_t)D);
            });
            t.wsoff.assign((size_t)nb + 1, 0);
            for (int64_t b = 0; b < nb; ++b) t.wsoff[(size_t)b + 1] = t.wsoff[(size_t)b] + (int64_t)ws[(size_t)b].size();
            std::vector<uint32_t> all;
            all.reserve((size_t)t.wsoff[(size_t)nb]);
            for (auto &v : ws) all.insert(all.end(), v.begin(), v.end());
            const RangeFn r_ws = [&](int64_t b) { return std::make_pair(t.wsoff[(size_t)b], t.wsoff[(size_t)b + 1]); };
            if ((rc = place(c, &t.wsched, all.data(), all.size(), 0, r_ws))) return rc;
            csc_bytes += (int64_t)all.size() * 4;
        }
        if (!band)
            csc_bytes += (int64_t)(cptr.size() * 4 + (total + kPad) * ((t.row16 ? 2 : 4) + (t.unit ? 0 : 4)));
        csc_bytes += lbytes;
        // the windowed product margin (band mode, no hot-weight margin)
        const int64_t pme = c->tune.product_margin;
        const int64_t S = (D + dlr::kPmSlice - 1) / dlr::kPmSlice;
        if (band && !t.margin_hot && ((int64_t)1 << shift) % kPmWinRows == 0 && pme != 0 && (pme == 1 || S >= 128)) {
            std::vector<dlr::BatchSpan> spans;
            t.pmw_first.assign((size_t)nb + 1, 0);
            for (int64_t b = 0; b < nb; ++b) {
                const dlr::BatchSpan &sp = t.plan[(size_t)b];
                for (int64_t r0 = 0; r0 < sp.rows; r0 += kPmWinRows) {
                    const int64_t f = (sp.first_row + r0) % t.n_rows, n = std::min(kPmWinRows, sp.rows - r0);
                    spans.push_back(dlr::BatchSpan{f, n, f + n <= t.n_rows});
                }
                t.pmw_first[(size_t)b + 1] = (int64_t)spans.size();
            }
            bool built = false;
            // a band's windows share a launch (launch_pm_windows)
            const int64_t slots = std::min<int64_t>(16, std::max<int64_t>(1, ((int64_t)1 << shift) / kPmWinRows));
            if ((rc = build_pm(c, src, spans, false, pme == 1, nthreads, resid_need, csc_bytes,
                               built, slots)))
                return rc;
            t.pmw = built;
            if (built) {
                t.pmw_slots = slots;
                std::vector<dlr::DevPm> views(spans.size());
                for (size_t i = 0; i < spans.size(); ++i) views[i] = pm_view(c, (int64_t)i);
                if ((rc = upload(c, &t.pmw_views, views.data(), views.size(), 0))) return rc;
            }
            if (!built && pme == 1)
                return fail(c, DLR_E_ARG, "dlr_load_train: DLR_PM=1 but the batches' windows do not fit the product margin");
        }
    }
    // Residual buffer (padded to whole LDS phases for the LDS kernel).
    if (c->resid_cap < resid_need) {
        dev_free(c, c->resid);
        c->resid = nullptr;
        if ((rc = dev_alloc(c, (void **)&c->resid, (size_t)resid_need * 4))) return rc;
        HIPC(c, hipMemsetAsync(c->resid, 0, (size_t)resid_need * 4, c->stream));
        if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
        c->resid_cap = resid_need;
    }
    if (t.sparse_stream && (rc = coalesce_stream(c, nthreads))) return rc;
    // streamed: the slots (counted by place()); resident: the shard arrays
    if (!t.sparse_stream)
        t.bytes = (int64_t)((t.n_rows + 1) * 8 + (t.nnz + kPad) * (t.unit ? 4 : 8) + t.n_rows * 4) + csc_bytes;
    t.fast = t.any_long;  // only long columns reorder a sparse sum (DLR_ORDER_FAST)
    if ((rc = coll_agree_pieced(c))) return rc;
    t.loaded = true;
    if (n_batches) *n_batches = nb;
    return DLR_OK;
}

int dlr_load_test(dlr_ctx *c, const dlr_dataset *ds) {
    if (!c || !ds) return fail(c, DLR_E_ARG, "dlr_load_test: bad argument");
    if (ds->D != c->D) return fail(c, DLR_E_ARG, "dlr_load_test: dataset D != context D");
    HIPC(c, hipSetDevice(c->device));
    if (!c->train.loaded) load_tuning(c);  // (else the training shard's)
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    free_test(c);
    TestShard &t = c->test;
    t.n_rows = ds->n_rows;
    t.nnz = (int64_t)ds->col.size();
    int rc;
    std::vector<int32_t> mapped;  // the training shard's column numbering
    if (!c->perm.empty()) {
        mapped.resize(ds->col.size());
        for (size_t e = 0; e < mapped.size(); ++e) mapped[e] = c->perm[(size_t)ds->col[e]];
    }
    if ((rc = upload(c, &t.row_ptr, ds->row_ptr.data(), (size_t)t.n_rows + 1))) return rc;
    if ((rc = upload(c, &t.col, c->perm.empty() ? ds->col.data() : mapped.data(), (size_t)t.nnz, kPad))) return rc;
    if (!unit_values(c, ds->val) && (rc = upload(c, &t.val, ds->val.data(), (size_t)t.nnz, kPad))) return rc;
    std::vector<float> lab(ds->label.begin(), ds->label.end());
    if ((rc = upload(c, &t.label, lab.data(), lab.size()))) return rc;
    t.grid = dlr::predict_grid(t.n_rows);
    if (c->ll_cap < t.grid + 1) {
        dev_free(c, c->ll);
        c->ll = nullptr;
        if ((rc = dev_alloc(c, (void **)&c->ll, (size_t)(t.grid + 1) * 8))) return rc;
        c->ll_cap = t.grid + 1;
    }
    t.bytes = (int64_t)((t.n_rows + 1) * 8 + (t.nnz + kPad) * 8 + t.n_rows * 4);
    t.loaded = true;
    return DLR_OK;
}

int dlr_load_train_dense(dlr_ctx *c, const dlr_dense *ds, int64_t batch_size, int64_t *n_batches) {
    if (!c) return fail(c, DLR_E_ARG, "dlr_load_train_dense: bad argument");
    HIPC(c, hipSetDevice(c->device));
    load_tuning(c);
    {
        std::string msg;
        if (!ds)
            msg = "dlr_load_train_dense: bad argument";
        else if (ds->D != c->D)
            msg = "dlr_load_train_dense: dataset D != context D";
        else if (batch_size == 0)
            msg = "dlr_load_train_dense: batch_size 0 (reference never terminates)";
        else if (ds->n_rows <= 0)
            msg = "dlr_load_train_dense: empty shard (reference never terminates)";
        const int64_t nb = msg.empty() ? dlr_num_batches(ds->n_rows, batch_size) : 0;
        int rc = coll_agree_load(c, "dlr_load_train_dense", msg.empty() ? DLR_OK : DLR_E_ARG, msg, nb);
        if (rc || (rc = coll_agree_order(c, "dlr_load_train_dense"))) return rc;
    }
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    if (c->xstream)  // the pieced all-gather's stream carries collectives too
        if (int rc_ = wait_stream(c, c->xstream, __func__)) return rc_;
    free_train(c);
    free_touched_bufs(c);
    int rc;
    if ((rc = change_perm(c, {}))) return rc;  // dense rows are in the original column order
    TrainShard &t = c->train;
    t.dense = true;
    t.n_rows = ds->n_rows;
    t.B = batch_size < 0 ? ds->n_rows : batch_size;
    t.plan = dlr::plan_batches(ds->n_rows, batch_size);
    const int64_t D = c->D;
    // Summation order (dlr_set_summation_order): REFERENCE --
    // the row chains and column chains of lr.cc:108-112 / 35-39 (banded for
    // large batches, launch_dense_step); FAST -- for batch rows x D > 2^24
    // the fused one-pass kernel where D allows (C4), else the two-pass
    // blocked sums (DLR_DENSE_GRAD=blocked|fused picks a FAST variant).
    const int64_t dg = c->tune.dense_grad;  // FAST order: DLR_AUTO, 0 chain, 1 blocked, 2 fused
    const bool big = t.B * D > ((int64_t)1 << 24);
    if (c->order == DLR_ORDER_FAST) {
        t.dfused = dg != DLR_AUTO ? dg == 2 : (big && dlr::dense_fused_ok(D));
        if (t.dfused && !dlr::dense_fused_ok(D))
            return fail(c, DLR_E_ARG, "dlr_load_train_dense: the fused dense gradient needs D in {512, 1024, 2048, 4096}");
        t.dblocked = t.dfused || (dg != DLR_AUTO ? dg == 1 : big);
    } else {
        // the banded reference-order launch (k_dense_ref) for large batches;
        // DLR_DENSE_REF=1|0 forces it on (where D allows) / off (A/B: the
        // margin kernel, then the column-chain kernel -- the same order)
        const int64_t dr = c->tune.dense_ref;
        t.dref = dlr::dense_ref_ok(D, ds->n_rows, t.B) && (dr != DLR_AUTO ? dr != 0 : big);
        t.mg_demoted = t.dref && c->dref_demoted;
        if (t.mg_demoted) t.dref = false;
        // how far (in 256-row slots) the margins may run ahead of the column
        // chains: the rows the chains re-read stay in the Infinity Cache
        // (DLR_DENSE_REF_LEAD: A/B; 0 = no limit)
        t.dref_lead = (int)tv(c->tune.dense_ref_lead, 64);
    }
    t.fast = t.dblocked;
    // Residency: device-resident unless asked to stream, or (auto) the rows
    // would not leave room in HBM (20M x 4096 fp32 = 328 GB
    // on one 288 GB GPU).  Streamed rows are staged per batch over PCIe.
    const size_t xbytes = ds->X.size() * 4;
    const size_t slot_bytes = (size_t)(t.B * D) * 4;
    bool stream = c->residency == DLR_RESIDENCY_STREAM;
    if (c->residency == DLR_RESIDENCY_AUTO) {
        size_t fr = 0, tot = 0;
        HIPC(c, hipMemGetInfo(&fr, &tot));
        const size_t reserve = ((size_t)8 << 30) + 4 * slot_bytes;
        stream = xbytes + reserve > fr;
    }
    if (stream) {
        t.streamed = true;
        t.hX = ds->X.data();
        hipError_t e = hipHostRegister(const_cast<float *>(t.hX), xbytes, hipHostRegisterDefault);
        if (e == hipSuccess)
            t.host_registered = true;
        else if (e == hipErrorHostMemoryAlreadyRegistered)
            (void)hipGetLastError();
        else
            return fail(c, DLR_E_HIP, std::string("dlr_load_train_dense: hipHostRegister: ") + hipGetErrorString(e));
        if (!c->cstream) HIPC(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
        for (int k = 0; k < 2; ++k) {
            if (!c->ev_ready[k]) HIPC(c, hipEventCreateWithFlags(&c->ev_ready[k], hipEventDisableTiming));
            if (!c->ev_free[k]) HIPC(c, hipEventCreateWithFlags(&c->ev_free[k], hipEventDisableTiming));
            if ((rc = dev_alloc(c, (void **)&t.sx[k], slot_bytes + 64))) return rc;
            if ((rc = dev_alloc(c, (void **)&t.sl[k], (size_t)t.B * 4 + 64))) return rc;
            HIPC(c, hipEventRecord(c->ev_free[k], c->stream));
        }
    } else if (t.dref) {
        // K6r's tiled image (64 x 64 tiles, dlr_kernels.hip): the rows staged
        // row-major, transformed on the device
        float *tmp = nullptr;
        if ((rc = upload(c, &tmp, ds->X.data(), ds->X.size(), 64))) return rc;
        const int64_t nf = dlr::dense_ref_tiled_floats(ds->n_rows, D);
        if ((rc = dev_alloc(c, (void **)&t.dX, (size_t)nf * 4 + 64))) {
            dev_free(c, tmp);
            return rc;
        }
        hipError_t e = dlr::launch_dense_tile(tmp, t.dX, ds->n_rows, D, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        dev_free(c, tmp);
        if (e != hipSuccess) return fail(c, DLR_E_HIP, std::string("dlr_load_train_dense: tiling: ") + hipGetErrorString(e));
        t.dtiled = true;
    } else if ((rc = upload(c, &t.dX, ds->X.data(), ds->X.size(), 64))) {
        return rc;
    }
    {
        std::vector<float> lab(ds->label.begin(), ds->label.end());
        if ((rc = upload(c, &t.label, lab.data(), lab.size()))) return rc;
    }
    if (t.dblocked &&
        (rc = dev_alloc(c, (void **)&t.dpart, (size_t)dlr::dense_chunks(t.B) * (size_t)((D + 3) & ~int64_t(3)) * 4)))
        return rc;
    // residuals: whole 4-row quads + 4 (the reference-order gradient reads
    // them 16 bytes at a time); the banded launch reads whole 256-row slots
    const int64_t rneed = t.dref ? dlr::dense_ref_resid(t.B) : ((t.B + 3) & ~int64_t(3)) + 4;
    if (t.dref) {
        const int64_t nw = dlr::dense_ref_sync_words(t.B);
        if ((rc = dev_alloc(c, (void **)&t.dref_sync, (size_t)nw * 4))) return rc;
        HIPC(c, hipMemsetAsync(t.dref_sync, 0, (size_t)nw * 4, c->stream));
        t.dref_seq = 0;
    }
    if (c->resid_cap < rneed) {
        dev_free(c, c->resid);
        c->resid = nullptr;
        if ((rc = dev_alloc(c, (void **)&c->resid, (size_t)rneed * 4))) return rc;
        c->resid_cap = rneed;
    }
    t.bytes = (int64_t)(ds->X.size() * 4 + ds->label.size() * 4);
    t.loaded = true;
    if (n_batches) *n_batches = (int64_t)t.plan.size();
    return DLR_OK;
}

int dlr_load_test_dense(dlr_ctx *c, const dlr_dense *ds) {
    if (!c || !ds) return fail(c, DLR_E_ARG, "dlr_load_test_dense: bad argument");
    if (ds->D != c->D) return fail(c, DLR_E_ARG, "dlr_load_test_dense: dataset D != context D");
    if (!c->perm.empty())
        return fail(c, DLR_E_STATE,
                    "dlr_load_test_dense: the loaded sparse training shard uses relabeled columns (DLR_RELABEL=0 "
                    "keeps the original order)");
    HIPC(c, hipSetDevice(c->device));
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    free_test(c);
    TestShard &t = c->test;
    t.dense = true;
    t.n_rows = ds->n_rows;
    int rc;
    if ((rc = upload(c, &t.dX, ds->X.data(), ds->X.size(), 64))) return rc;
    std::vector<float> lab(ds->label.begin(), ds->label.end());
    if ((rc = upload(c, &t.label, lab.data(), lab.size()))) return rc;
    t.grid = dlr::predict_dense_grid(t.n_rows);
    if (c->ll_cap < t.grid + 1) {
        dev_free(c, c->ll);
        c->ll = nullptr;
        if ((rc = dev_alloc(c, (void **)&c->ll, (size_t)(t.grid + 1) * 8))) return rc;
        c->ll_cap = t.grid + 1;
    }
    t.bytes = (int64_t)(ds->X.size() * 4 + ds->label.size() * 4);
    t.loaded = true;
    return DLR_OK;
}

int dlr_train_step(dlr_ctx *c, int64_t b, float lr, float C, int mode) {
    if (!c) return fail(c, DLR_E_ARG, "dlr_train_step: null context");
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_step: no training shard loaded");
    if (b < 0 || b >= (int64_t)c->train.plan.size()) return fail(c, DLR_E_ARG, "dlr_train_step: batch out of range");
    if (mode < 0 || mode > 2) return fail(c, DLR_E_ARG, "dlr_train_step: bad mode");
    if (int rc = check_device(c, "dlr_train_step")) return rc;  // what earlier steps recorded
    HIPC(c, hipSetDevice(c->device));
    struct {
        int64_t rows;
    } const bt{c->train.plan[(size_t)b].rows};
    if (bt.rows > c->resid_cap) return fail(c, DLR_E_STATE, "dlr_train_step: residual buffer too small");
    hipEvent_t t_step, t0;
    time_begin(c, &t_step);
    if (c->train.sparse_stream) {
        HIPC(c, sparse_batch(c, b));  // binds the batch's slot (the views below)
        HIPC(c, build_layout(c, b));
    }
    const bool piped = band_pipeline_ok(c, b);  // margin and band gradients interleaved (band mode)
    if (!piped) {
        time_begin(c, &t0);
        HIPC(c, launch_margin(c, b, false, !c->comm));
        time_end(c, 0, t0);
    }
    if (piped) {
        // the margin, the gradient and (one rank) the update: one timed stage
        time_begin(c, &t0);
        HIPC(c, band_step_pipelined(c, b, bt.rows, c->comm ? c->g : nullptr, lr, C, !c->comm));
        time_end(c, 1, t0);
        if (c->comm) {
            StepPlan xp = step_plan(c);
            const dlr::CollOp *a2a = xp.next(dlr::kCollAllToAll);
            PLANC(c, a2a);
            time_begin(c, &t0);
            XCHGC(c, a2a, c->g, c->recv, c->stream);
            time_end(c, 3, t0);
            int64_t kb, ke;
            dlr_key_range(c->D, c->world, c->rank, &kb, &ke);
            time_begin(c, &t0);
            HIPC(c, dlr::launch_merge_update(c->recv, c->world, c->chunk, ke - kb, c->w + kb, lr, mode, c->stream));
            time_end(c, 2, t0);
            const dlr::CollOp *ag = xp.next(dlr::kCollAllGather);
            PLANC(c, ag);
            time_begin(c, &t0);
            XCHGC(c, ag, c->w + (int64_t)c->rank * ag->words, c->w, c->stream);
            time_end(c, 3, t0);
        }
    } else if (c->train.touched) {
        // touched columns (ordered gradient), then the dense L2 pass over
        // all D, then the touched columns' new weights (dlr_kernels.hip
        // "Touched-column layout").
        const TrainShard &t = c->train;
        const int64_t n = t.tncols[(size_t)b];
        const uint32_t *cols = t.tcols + t.tcoff[(size_t)b];
        const dlr::DevCsc cs = csc_view(c, b);
        if (!c->comm) {
            time_begin(c, &t0);
            HIPC(c, dlr::launch_grad_touched(cs, cols, n, c->resid, c->w, c->newv, bt.rows, lr, C, true, c->stream));
            time_end(c, 1, t0);
            time_begin(c, &t0);
            HIPC(c, dlr::launch_dense_l2(c->w, c->D, c->rs, lr, C, mode, c->stream));
            HIPC(c, dlr::launch_scatter(c->w, cols, c->newv, n, c->stream));
            time_end(c, 2, t0);
        } else {
            // sparse exchange: all-gather every rank's [count | cols | g]
            const int64_t cap = c->xcap, stride = 1 + 2 * cap;
            time_begin(c, &t0);
            HIPC(c, dlr::launch_grad_touched(cs, cols, n, c->resid, c->w, (float *)(c->xsend + 1 + cap), bt.rows,
                                             0.0f, C, false, c->stream));
            time_end(c, 1, t0);
            HIPC(c, hipMemsetD32Async(c->xsend, (int)n, 1, c->stream));
            HIPC(c, hipMemcpyAsync(c->xsend + 1, cols, (size_t)n * 4, hipMemcpyDeviceToDevice, c->stream));
            StepPlan xp = step_plan(c);
            const dlr::CollOp *ag = xp.next(dlr::kCollAllGather);
            PLANC(c, ag);
            if (ag->words != stride) return fail(c, DLR_E_STATE, "dlr_train_step: touched block size");
            time_begin(c, &t0);
            XCHGC(c, ag, c->xsend, c->xrecv, c->stream);
            time_end(c, 3, t0);
            time_begin(c, &t0);
            HIPC(c, dlr::launch_sparse_merge(c->xrecv, cap, stride, c->w, c->rs, lr, C, mode, c->xcols, c->xnewv,
                                             c->stream));
            HIPC(c, dlr::launch_dense_l2(c->w, c->D, c->rs, lr, C, mode, c->stream));
            HIPC(c, dlr::launch_scatter(c->w, c->xcols, c->xnewv, (int64_t)c->world * cap, c->stream));
            time_end(c, 2, t0);
        }
    } else if (!c->comm) {
        time_begin(c, &t0);
        HIPC(c, launch_gradient(c, b, bt.rows, nullptr, lr, C, true));
        time_end(c, 1, t0);
    } else {
        time_begin(c, &t0);
        HIPC(c, launch_gradient(c, b, bt.rows, c->g, lr, C, false));
        time_end(c, 1, t0);
        StepPlan xp = step_plan(c);
        const dlr::CollOp *a2a = xp.next(dlr::kCollAllToAll);
        PLANC(c, a2a);
        time_begin(c, &t0);
        XCHGC(c, a2a, c->g, c->recv, c->stream);
        time_end(c, 3, t0);
        int64_t kb, ke;
        dlr_key_range(c->D, c->world, c->rank, &kb, &ke);
        time_begin(c, &t0);
        HIPC(c, dlr::launch_merge_update(c->recv, c->world, c->chunk, ke - kb, c->w + kb, lr, mode, c->stream));
        time_end(c, 2, t0);
        time_begin(c, &t0);
        if (c->train.xpieced) {
            // (the exchange interval then includes the next batch's pass 1)
            int rc = exchange_overlapped(c, b, xp);
            if (rc) return rc;
        } else {
            const dlr::CollOp *ag = xp.next(dlr::kCollAllGather);
            PLANC(c, ag);
            XCHGC(c, ag, c->w + (int64_t)c->rank * ag->words, c->w, c->stream);
        }
        time_end(c, 3, t0);
    }
    if (c->train.sparse_stream) HIPC(c, sparse_batch_done(c, b));
    if (c->train.mg_demoted) ++c->hcount[DLR_COUNT_MG_DEMOTED];
    time_end(c, 4, t_step);
    return DLR_OK;
}

int dlr_train_epoch(dlr_ctx *c, float lr, float C, int mode) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_epoch: no training shard loaded");
    for (int64_t b = 0; b < (int64_t)c->train.plan.size(); ++b) {
        int rc = dlr_train_step(c, b, lr, C, mode);
        if (rc) return rc;
    }
    // the epoch's success is definitive: its last step's in-launch waits
    // are known to have completed
    return dlr_sync(c);
}

int dlr_worker_gradient(dlr_ctx *c, int64_t b, float C, float *grad_out, int64_t D) {
    if (!c || !grad_out || D != c->D) return fail(c, DLR_E_ARG, "dlr_worker_gradient: bad argument");
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_worker_gradient: no training shard loaded");
    if (b < 0 || b >= (int64_t)c->train.plan.size())
        return fail(c, DLR_E_ARG, "dlr_worker_gradient: batch out of range");
    HIPC(c, hipSetDevice(c->device));
    struct {
        int64_t rows;
    } const bt{c->train.plan[(size_t)b].rows};
    if (c->train.sparse_stream) {
        HIPC(c, sparse_batch(c, b));
        HIPC(c, build_layout(c, b));
    }
    HIPC(c, launch_margin(c, b));
    if (c->train.touched) {
        // full pushed vector: the L2 term everywhere, the touched columns' g
        const TrainShard &t = c->train;
        const int64_t n = t.tncols[(size_t)b];
        const uint32_t *cols = t.tcols + t.tcoff[(size_t)b];
        HIPC(c, dlr::launch_grad_touched(csc_view(c, b), cols, n, c->resid, c->w, c->newv, bt.rows, 0.0f, C, false,
                                         c->stream));
        HIPC(c, dlr::launch_l2_fill(c->g, c->w, c->D, (float)bt.rows, C, c->stream));
        HIPC(c, dlr::launch_scatter(c->g, cols, c->newv, n, c->stream));
    } else {
        HIPC(c, launch_gradient(c, b, bt.rows, c->g, 0.0f, C, false));
    }
    if (c->train.sparse_stream) HIPC(c, sparse_batch_done(c, b));
    if (c->perm.empty()) {
        HIPC(c, hipMemcpyAsync(grad_out, c->g, (size_t)D * 4, hipMemcpyDeviceToHost, c->stream));
        if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
        return check_device(c, "dlr_worker_gradient");
    }
    std::vector<float> tmp((size_t)D);
    HIPC(c, hipMemcpyAsync(tmp.data(), c->g, (size_t)D * 4, hipMemcpyDeviceToHost, c->stream));
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    if (int rc = check_device(c, "dlr_worker_gradient")) return rc;
    for (int64_t j = 0; j < D; ++j) grad_out[j] = tmp[(size_t)c->perm[(size_t)j]];
    return DLR_OK;
}

int dlr_server_apply(dlr_ctx *c, const float *grads, int W, int64_t D, float lr, int mode) {
    if (!c || !grads || W <= 0 || D != c->D || mode < 0 || mode > 2)
        return fail(c, DLR_E_ARG, "dlr_server_apply: bad argument");
    HIPC(c, hipSetDevice(c->device));
    std::vector<float> tmp;
    if (!c->perm.empty()) {  // the pushes in the internal column order
        tmp.resize((size_t)W * (size_t)D);
        for (int r = 0; r < W; ++r)
            for (int64_t j = 0; j < D; ++j)
                tmp[(size_t)r * (size_t)D + (size_t)c->perm[(size_t)j]] = grads[(size_t)r * (size_t)D + (size_t)j];
        grads = tmp.data();
    }
    float *buf = nullptr;
    int rc = dev_alloc(c, (void **)&buf, (size_t)W * (size_t)D * 4);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(buf, grads, (size_t)W * (size_t)D * 4, hipMemcpyHostToDevice, c->stream);
    c->pm_ready = -1;
    if (e == hipSuccess) e = dlr::launch_merge_update(buf, W, D, D, c->w, lr, mode, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dev_free(c, buf);
    if (e != hipSuccess) return fail(c, DLR_E_HIP, std::string("dlr_server_apply: ") + hipGetErrorString(e));
    return DLR_OK;
}

int dlr_predict(dlr_ctx *c, int64_t *correct, int64_t *n_rows, double *logloss) {
    if (!c) return DLR_E_ARG;
    if (!c->test.loaded) return fail(c, DLR_E_STATE, "dlr_predict: no test shard loaded");
    HIPC(c, hipSetDevice(c->device));
    const TestShard &t = c->test;
    HIPC(c, hipMemsetAsync(c->correct, 0, 8, c->stream));
    if (t.dense) {
        HIPC(c, dlr::launch_dense_predict({t.dX, t.label, t.n_rows, c->D}, c->w, c->correct, c->ll + 1, c->ll,
                                          c->stream));
    } else {
        const dlr::DevBatch bt{t.row_ptr, t.col, t.val, t.label, t.n_rows, t.nnz};
        HIPC(c, dlr::launch_predict(bt, c->w, c->correct, c->ll + 1, c->ll, c->stream));
    }
    HIPC(c, hipMemcpyAsync(c->h_correct, c->correct, 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(c->h_ll, c->ll, 8, hipMemcpyDeviceToHost, c->stream));
    if (int rc = wait_stream(c, c->stream, "dlr_predict")) return rc;
    if (int rc = check_device(c, "dlr_predict")) return rc;
    if (correct) *correct = (int64_t)*c->h_correct;
    if (n_rows) *n_rows = t.n_rows;
    if (logloss) *logloss = *c->h_ll;
    return DLR_OK;
}

int dlr_sync(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    HIPC(c, hipSetDevice(c->device));
    if (int rc = wait_stream(c, c->stream, "dlr_sync")) return rc;
    if (c->cstream) HIPC(c, hipStreamSynchronize(c->cstream));  // a streamed shard's batch copies
    return check_device(c, "dlr_sync");
}

int dlr_timing(dlr_ctx *c, int enable) {
    if (!c) return DLR_E_ARG;
    HIPC(c, hipSetDevice(c->device));
    harvest(c);
    c->timing = enable != 0;
    // Pre-create the events so recording never allocates inside a timed region.
    while (c->timing && c->ev_pool.size() < 16384) {
        hipEvent_t e;
        HIPC(c, hipEventCreate(&e));
        c->ev_pool.push_back(e);
    }
    for (int i = 0; i < kTimers; ++i) {
        c->t_ms[i] = 0;
        c->t_n[i] = 0;
    }
    return DLR_OK;
}

int dlr_kernel_time(dlr_ctx *c, int which, double *total_ms, int64_t *launches) {
    if (!c || which < 0 || which >= kTimers) return DLR_E_ARG;
    HIPC(c, hipSetDevice(c->device));
    harvest(c);
    if (total_ms) *total_ms = c->t_ms[which];
    if (launches) *launches = c->t_n[which];
    return DLR_OK;
}

int dlr_stage_time(dlr_ctx *c, int stage, int64_t first, int64_t count, float lr, float C, double *avg_ms) {
    if (!c || count <= 0 || stage < 0 || stage > 2) return fail(c, DLR_E_ARG, "dlr_stage_time: bad argument");
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_stage_time: no training shard loaded");
    const TrainShard &t = c->train;
    if (stage == DLR_STAGE_UPDATE && !t.touched)
        return fail(c, DLR_E_ARG, "dlr_stage_time: the update stage is separate only in the touched layout");
    if (t.streamed || t.sparse_stream)
        return fail(c, DLR_E_STATE, "dlr_stage_time: streamed shard (kernel stages wait on batch copies)");
    HIPC(c, hipSetDevice(c->device));
    harvest(c);
    const bool was = c->timing;
    c->timing = false;
    hipEvent_t a, b;
    HIPC(c, hipEventCreate(&a));
    HIPC(c, hipEventCreate(&b));
    const int64_t nb = (int64_t)t.plan.size();
    hipError_t e = hipEventRecord(a, c->stream);
    for (int64_t k = 0; k < count && e == hipSuccess; ++k) {
        const int64_t bb = (first + k) % nb;
        const int64_t rows = t.plan[(size_t)bb].rows;
        if (stage == DLR_STAGE_MARGIN) {
            // product margin: pass 2 alone -- in the training step pass 1 runs
            // inside the previous step's gradient (counted there); nothing
            // when pass 2 runs in the gradient's launch too (pm_mg_ok)
            e = launch_margin(c, bb, t.pm_fused, !c->comm);
        } else if (t.touched) {
            const int64_t n = t.tncols[(size_t)bb];
            const uint32_t *cols = t.tcols + t.tcoff[(size_t)bb];
            if (stage == DLR_STAGE_GRADIENT)
                e = dlr::launch_grad_touched(csc_view(c, bb), cols, n, c->resid, c->w, c->newv, rows, lr, C, true,
                                             c->stream);
            else {
                e = dlr::launch_dense_l2(c->w, c->D, c->rs, lr, C, 0, c->stream);
                if (e == hipSuccess) e = dlr::launch_scatter(c->w, cols, c->newv, n, c->stream);
            }
        } else {
            e = launch_gradient(c, bb, rows, c->comm ? c->g : nullptr, lr, C, !c->comm);
        }
    }
    if (e == hipSuccess) e = hipEventRecord(b, c->stream);
    if (e == hipSuccess) e = hipEventSynchronize(b);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    c->timing = was;
    c->pm_ready = -1;  // the stages ran without their partners
    if (e != hipSuccess) return fail(c, DLR_E_HIP, std::string("dlr_stage_time: ") + hipGetErrorString(e));
    if (avg_ms) *avg_ms = (double)ms / (double)count;
    return check_device(c, "dlr_stage_time");
}

int dlr_stage_counters(dlr_ctx *c, int64_t *out, int n) {
    if (!c || !out || n < 0 || n > DLR_COUNTERS) return fail(c, DLR_E_ARG, "dlr_stage_counters: bad argument");
    HIPC(c, hipSetDevice(c->device));
    for (hipStream_t s : {c->stream, c->gstream, c->hstream})
        if (s) HIPC(c, hipStreamSynchronize(s));
    int64_t v[DLR_COUNTERS];
    for (int k = 0; k < DLR_COUNTERS; ++k) v[k] = c->hcount[k];
    if (c->h_err)
        v[DLR_COUNT_HOT_GIVEUPS] =
            (int64_t)__atomic_load_n(c->h_err + dlr::kErrWords + dlr::kStatHotGiveUps, __ATOMIC_ACQUIRE);
    for (int k = 0; k < n; ++k) out[k] = v[k];
    return DLR_OK;
}

int dlr_set_fault(dlr_ctx *c, int fault) {
    if (!c || fault < dlr::kFaultNone || fault > dlr::kFaultHotRing)
        return fail(c, DLR_E_ARG, "dlr_set_fault: bad fault");
    c->fault = fault;
    return DLR_OK;
}

void dlr_tuning_default(dlr_tuning *t) {
    if (!t) return;
    int64_t *f = reinterpret_cast<int64_t *>(t);
    for (size_t k = 0; k < sizeof(dlr_tuning) / sizeof(int64_t); ++k) f[k] = DLR_AUTO;
}

// The environment's tuning: each DLR_* variable the header names, parsed
// as the engine always has (a numeric value, or 0 / any other value for a
// switch; names for the layout and the dense gradient).
void dlr_tuning_from_env(dlr_tuning *t) {
    if (!t) return;
    dlr_tuning_default(t);
    auto num = [](const char *name, int64_t &f) {
        if (const char *e = getenv(name)) f = atoll(e);
    };
    auto on_off = [](const char *name, int64_t &f) {  // "0" off, any other value on
        if (const char *e = getenv(name)) f = strcmp(e, "0") == 0 ? 0 : 1;
    };
    if (const char *e = getenv("DLR_GRAD_KERNEL"))
        t->grad_layout = strcmp(e, "classic") == 0 ? DLR_LAYOUT_CLASSIC
                         : strcmp(e, "lds") == 0   ? DLR_LAYOUT_LDS
                         : strcmp(e, "touched") == 0 ? DLR_LAYOUT_TOUCHED
                                                     : DLR_AUTO;
    if (const char *e = getenv("DLR_PM"))  // "0" off, "1" required, else automatic
        t->product_margin = strcmp(e, "0") == 0 ? 0 : strcmp(e, "1") == 0 ? 1 : DLR_AUTO;
    on_off("DLR_PM_FUSED", t->pm_fused);
    on_off("DLR_PM_MG", t->pm_in_gradient);
    num("DLR_PM_SPLIT", t->pm_split);
    on_off("DLR_GRAD_RT", t->row_rounds);
    num("DLR_BAND_ROWS", t->band_rows);
    on_off("DLR_BAND_PIPE", t->band_pipeline);
    num("DLR_BAND_HOT", t->band_hot);
    on_off("DLR_HOT_STREAM", t->hot_stream);
    num("DLR_HOT_STREAM_MAX", t->hot_stream_max);
    if (const char *e = getenv("DLR_MARGIN_HOT")) t->margin_hot = atoi(e) != 0 ? 1 : 0;
    num("DLR_LONG_COLUMN", t->long_column);
    num("DLR_LONG_PIECE", t->long_piece);
    on_off("DLR_LONG_SCHED", t->long_sched);
    num("DLR_RELABEL", t->relabel);
    num("DLR_RELABEL_TAIL", t->relabel_tail);
    num("DLR_RELABEL_RARE", t->relabel_rare);
    on_off("DLR_UNIT_VALUES", t->unit_values);
    on_off("DLR_STREAM_COALESCE", t->stream_coalesce);
    on_off("DLR_STREAM_DEVICE_LAYOUT", t->stream_device_layout);
    if (const char *e = getenv("DLR_DENSE_GRAD"))
        t->dense_grad = strcmp(e, "fused") == 0 ? 2 : strcmp(e, "blocked") == 0 ? 1 : 0;
    on_off("DLR_DENSE_REF", t->dense_ref);
    num("DLR_DENSE_REF_LEAD", t->dense_ref_lead);
}

int dlr_set_tuning(dlr_ctx *c, const dlr_tuning *t) {
    if (!c) return fail(c, DLR_E_ARG, "dlr_set_tuning: null context");
    if (t) {
        if (t->grad_layout != DLR_AUTO && (t->grad_layout < DLR_LAYOUT_CLASSIC || t->grad_layout > DLR_LAYOUT_TOUCHED))
            return fail(c, DLR_E_ARG, "dlr_set_tuning: grad_layout");
        if (t->band_rows != DLR_AUTO && (t->band_rows < 0 || (t->band_rows & (t->band_rows - 1)) != 0))
            return fail(c, DLR_E_ARG, "dlr_set_tuning: band_rows must be 0 or a power of two");
        if (t->dense_grad != DLR_AUTO && (t->dense_grad < 0 || t->dense_grad > 2))
            return fail(c, DLR_E_ARG, "dlr_set_tuning: dense_grad");
        c->tune = *t;
    }
    c->tune_set = t != nullptr;
    return DLR_OK;
}

int dlr_get_tuning(dlr_ctx *c, dlr_tuning *t) {
    if (!c || !t) return fail(c, DLR_E_ARG, "dlr_get_tuning: bad argument");
    if (!c->tune_set && !c->train.loaded) dlr_tuning_from_env(&c->tune);
    *t = c->tune;
    return DLR_OK;
}

int dlr_set_residency(dlr_ctx *c, int mode) {
    if (!c || mode < DLR_RESIDENCY_AUTO || mode > DLR_RESIDENCY_STREAM)
        return fail(c, DLR_E_ARG, "dlr_set_residency: bad mode");
    c->residency = mode;
    return DLR_OK;
}

int dlr_train_residency(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_residency: no training shard loaded");
    return c->train.streamed || c->train.sparse_stream ? DLR_RESIDENCY_STREAM : DLR_RESIDENCY_DEVICE;
}

int dlr_train_relabeled(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    return c->perm.empty() ? 0 : 1;
}

int dlr_train_unit_values(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_unit_values: no training shard loaded");
    return c->train.unit ? 1 : 0;
}

int dlr_train_product_margin(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_product_margin: no training shard loaded");
    return c->train.pm ? (c->train.pm_fused ? (c->train.pm_mg ? 3 : 2) : 1) : c->train.pmw ? 1 : 0;
}

int dlr_train_pm_strided(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_pm_strided: no training shard loaded");
    const TrainShard &t = c->train;
    if (!t.pm && !t.pmw) return 0;
    size_t n = 0;
    for (uint32_t r : t.pm_rstride) n += r != 0;
    return n == 0 ? 0 : n == t.pm_rstride.size() ? 1 : 2;
}

int dlr_train_row_rounds(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_row_rounds: no training shard loaded");
    return c->train.pcsc && c->train.rt ? c->train.rt_rounds : 0;
}

int dlr_train_hot_columns(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_hot_columns: no training shard loaded");
    const TrainShard &t = c->train;
    int64_t n = 0;
    for (int64_t x : t.hs_nh) n = std::max(n, x);
    return t.hs ? (int)n : 0;
}

int dlr_train_band_rows(dlr_ctx *c) {
    if (!c || !c->train.loaded) return 0;
    return c->train.band_shift ? 1 << c->train.band_shift : 0;
}

int dlr_train_layout(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_train_layout: no training shard loaded");
    return c->train.touched ? DLR_LAYOUT_TOUCHED : c->train.pcsc ? DLR_LAYOUT_LDS : DLR_LAYOUT_CLASSIC;
}

int dlr_set_exchange_overlap(dlr_ctx *c, int on) {
    if (!c) return DLR_E_ARG;
    HIPC(c, hipSetDevice(c->device));
    if (int rc_ = wait_stream(c, c->stream, __func__)) return rc_;
    c->xoverlap = on != 0;
    c->pm_ready = -1;  // products formed under the other setting are not assumed
    // with a shard loaded the ranks re-agree now (collective): every rank's
    // next step must issue the same collectives
    if (c->train.loaded) return coll_agree_pieced(c);
    return DLR_OK;
}

int dlr_exchange_overlap(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    return c->comm && c->train.loaded && c->train.xpieced ? 1 : 0;
}

int dlr_set_exchange_pieces(dlr_ctx *c, int pieces) {
    if (!c || pieces < 0 || pieces > kXPiecesMax)
        return fail(c, DLR_E_ARG, "dlr_set_exchange_pieces: pieces must be 0 (auto) or in [1, 16]");
    c->xpieces = pieces;  // the next load's (the ranks agree there)
    return DLR_OK;
}

int dlr_exchange_pieces(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    return c->comm && c->train.loaded && c->train.xpieced ? c->train.xpieces : 0;
}

int dlr_set_summation_order(dlr_ctx *c, int order) {
    if (!c || (order != DLR_ORDER_REFERENCE && order != DLR_ORDER_FAST))
        return fail(c, DLR_E_ARG, "dlr_set_summation_order: bad order");
    c->order = order;
    return DLR_OK;
}

int dlr_summation_order(dlr_ctx *c) {
    if (!c) return DLR_E_ARG;
    if (!c->train.loaded) return fail(c, DLR_E_STATE, "dlr_summation_order: no training shard loaded");
    return c->train.fast ? DLR_ORDER_FAST : DLR_ORDER_REFERENCE;
}

int dlr_memory_info(dlr_ctx *c, int64_t *train_bytes, int64_t *test_bytes) {
    if (!c) return DLR_E_ARG;
    if (train_bytes) *train_bytes = c->train.loaded ? c->train.bytes : 0;
    if (test_bytes) *test_bytes = c->test.loaded ? c->test.bytes : 0;
    return DLR_OK;
}

int dlr_stream_bytes(dlr_ctx *c, int64_t *mean_bytes, int64_t *max_bytes) {
    if (!c) return DLR_E_ARG;
    const TrainShard &t = c->train;
    if (!t.loaded) return fail(c, DLR_E_STATE, "dlr_stream_bytes: no training shard loaded");
    double sum = 0.0;
    int64_t mx = 0;
    const size_t nb = t.plan.size();
    for (size_t b = 0; b < nb && (t.streamed || t.sparse_stream); ++b) {
        int64_t n = 0;  // exactly what stage_dense / stage_sparse copy host -> device for batch b
        if (t.streamed) {
            n = t.plan[b].rows * c->D * 4;
        } else if (t.shost) {
            n = (int64_t)t.sbsz[b];
        } else {
            for (const StreamArr &a : t.sarr)
                if (a.end[b] > a.beg[b]) n += (int64_t)(((size_t)(a.end[b] - a.beg[b]) + a.pad) * a.es);
        }
        sum += (double)n;
        mx = std::max(mx, n);
    }
    if (mean_bytes) *mean_bytes = nb ? (int64_t)(sum / (double)nb + 0.5) : 0;
    if (max_bytes) *max_bytes = mx;
    return DLR_OK;
}

}  // extern "C"
