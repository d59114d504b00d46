// dlr_kernels.h -- launchers of the gfx950 kernels (dlr_kernels.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace dlr {

// One batch as CSR: rows [0, rows) with row_ptr[i] absolute offsets into
// col/val (row_ptr may point into the middle of the shard's array).
// val == nullptr (here and in DevCsc / DevLong): a unit-valued shard, every
// value 1.0f (one-hot / binary features), so no value array is stored.
struct DevBatch {
    const int64_t *row_ptr;
    const int32_t *col;
    const float *val;
    const float *label;
    int64_t rows;
    int64_t nnz;  // entries of the batch (row_ptr[rows] - row_ptr[0])
};

// One batch column-major: entries of column j are [ptr[j], ptr[j+1]) in
// batch-row order; row holds batch-local row indices (uint16 when the batch
// has <= 65536 rows, else uint32).
struct DevCsc {
    const uint32_t *ptr;
    const void *row;
    const float *val;
    bool row16;
    // classic layout: wave k sums columns [wstart[k], wstart[k+1]) -- at most
    // 64 columns and about one window of entries (built at load); null:
    // 64 consecutive columns per wave
    const uint32_t *wstart = nullptr;
    int64_t nwaves = 0;
};

// Long columns of one batch (classic layout): ncols columns cols[] (their
// ptr entries in DevCsc carry bit 31), column l's chunks are segments
// [cseg[l], cseg[l+1]); segment s spans entries [sptr[s], sptr[s+1]) of
// row/val (4-aligned starts; at most kLongChunk entries + 3 padding; the
// arrays are padded by kLongChunk entries).  The low 2 bits of a column's
// end pointer (the next start, or the batch's terminal entry) hold the
// column's padding count.
constexpr int kLongChunk = 256;
struct DevLong {
    const uint32_t *cols;
    const uint32_t *cseg;
    const uint32_t *sptr;
    const void *row;
    const float *val;
    int64_t ncols, nseg;
    bool row16;
    // chunks in order of their first row (null: chunk order): the chunks in
    // flight at once then gather from a narrow band of the residuals
    const uint32_t *sched = nullptr;
};

// One batch column-major, PHASE-SPLIT for the LDS-resident gradient
// kernel: rows fall in phases of R = fill*4,096 rows (grad_lds_phase_rows:
// one phase of <= 16,384 rows, or up to two of 32,768).
// For 64-column group g and phase p, block (g*phases + p) holds the entries
// of those columns whose row is in the phase, column by column, rows
// ascending; base[blk] is its first entry (4-aligned), ends[blk*64 + l] the
// inclusive end offset of column 64g+l within the block (block <= 255
// entries).  row is the phase-local row (uint16).  base has
// groups*phases+1 entries; row/val are padded by >= 256 entries.
struct DevPcsc {
    const uint32_t *base;
    const uint8_t *ends;
    const uint16_t *row;
    const float *val;
    int phases;
    int fill;  // R / 4,096
};

// Short columns of one batch in ROW BANDS of 2^k rows (classic layout, large
// batches): for one band, the (column, segment) pairs of the short columns
// with entries in the band, columns ascending; pair s is column cols[s] with
// entries [ptr[s], ptr[s+1]) of row/val (batch-local rows, ascending).  Wave
// k sums pairs [wstart[k], wstart[k+1]) (<= 64 * kBandPairsPerLane pairs,
// ~one window of entries).  row/val are padded by >= 64 entries.
#ifndef DLR_BAND_K  // A/B builds only (make variant VDEFS=-DDLR_BAND_K=n)
#define DLR_BAND_K 4
#endif
constexpr int kBandPairsPerLane = DLR_BAND_K;
struct DevBand {
    const uint32_t *cols;
    const uint32_t *ptr;
    const uint32_t *wstart;
    const void *row;
    const float *val;
    int64_t nwaves;
    bool row16;
};

// Long columns of one batch in ROW PHASES of kLPhase rows (band mode):
// phase p's entries (phase-local rows, ascending per column) are cut into
// PIECES of <= 64 consecutive entries of one column; piece s of the phase
// spans [ps[desc[p].ptr + s].x, ps[... + s + 1].x) of row/val offset by
// desc[p].ent, and its partial goes to part[ps[desc[p].ptr + s].y]; waves
// take pieces [ws[desc[p].ws + t], ... + t + 1) (<= 64 pieces, ~one window
// of entries).
constexpr int kLPhase = 16384;  // rows per phase (64 KB of residuals in LDS)
constexpr int kLPWaves = 16;    // waves per workgroup (one workgroup per phase)
constexpr int kLPWinPad = 1024; // padding entries after the phase rows (one unclamped window)
struct PhaseDesc {
    int64_t ptr, ent, ws, ntasks;
};
struct DevLPhase {
    const PhaseDesc *desc;
    const uint2 *ps;  // (entry pointer, partial slot) per piece
    const uint32_t *ws;
    const uint16_t *row;
    const float *val;
    int64_t nph;
    uint32_t npart;  // partials; part[npart, npart + 64) is a write sink for idle lanes
};

// In-launch hand-off errors.  The one-launch kernels (k_grad_lds MG,
// k_dense_ref, k_band_hot) hand data between workgroups or waves through
// counters; every wait is bounded (dlr_kernels.hip Spin).  A wait that runs
// out sets word [kind] of the context's error words (host-mapped, zero when
// healthy), which the engine turns into DLR_E_DEVICE.
enum DevErr {
    kErrMgPublish = 0,  // k_grad_lds MG: a phase's margin blocks were never all published
    kErrRefSlot = 1,    // k_dense_ref: a chain slot's margin units were never published
    kErrRefLimit = 2,   // k_dense_ref: the chains' limit never reached a margin unit
    kErrRefLds = 3,     // k_dense_ref: a hand-off between the waves of a workgroup
    kErrHotLds = 4,     // k_band_hot / k_hot_chain: a hand-off between the waves of a workgroup
    kErrHotFlag = 5,    // k_hot_chain (last launch of a step): a band's hot products were never published
    kErrWords = 8
};
// Event counters the kernels keep beside the error words (same host-mapped
// array, words kErrWords + k): cumulative since the shard was loaded,
// reported by dlr_stage_counters.
enum DevStat {
    kStatHotGiveUps = 0,  // k_hot_chain: a column's launch stopped at a band flag (the next launch went on)
    kStatWords = 8
};
// Test-only fault injection (dlr_set_fault): a producer that never comes.
enum DevFault {
    kFaultNone = 0,
    kFaultMgPublish = 1,   // k_grad_lds MG: margin block 0 never adds to its counter
    kFaultRefPublish = 2,  // k_dense_ref: margin unit 0 never adds to its slot's counter
    kFaultHotRing = 3      // k_band_hot / k_hot_chain: the product / loader waves never post a chunk
};

// The largest grid of `threads`-thread workgroups with `lds` bytes of
// dynamic LDS that is resident at once on the current device when nothing
// else runs on it (workgroups per CU x CUs) for kernel `fn`; 0 if its
// attributes cannot be read.  resident_per_cu: per CU, from the kernel's
// attributes and gfx950's budgets, capped by the runtime's occupancy query
// when that answers >= 1 (*query: its answer, -1 on error).
int resident_grid(const void *fn, int threads, size_t lds);
int resident_per_cu(const void *fn, int threads, size_t lds, int *query);

// PRODUCT MARGIN of one batch (dlr_kernels.hip "Product margin"; LDS-layout
// batches).  The batch's rows fall in blocks of kPmRows; its columns in
// slices of kPmSlice (the columns of one k_grad_lds workgroup).  Every
// product fl32(w_j * x_ij) of the batch has a slot in the product array p:
// block k's products fill its REGION [rg[k], rg[k+1]) (4-aligned, <=
// kPmCap), one chunk per slice (chunks ordered by the XCD of their slice's
// workgroup; each padded to a multiple of 4 slots), rows ascending within a
// chunk.  Pass 1 (workgroup = slice s) forms slice s's products: entries
// [lbeg[s], lbeg[s+1]) (multiples of 4) of val and, in groups of four, of
// list -- two words per group: the four columns within the slice (12 bits
// each, bits 0-47), the block k (bits 48-57) and the group's rank in its
// chunk / 4 (bits 58-63); the chunk of block k starts at p[pofs[s*nblk + k]];
// padding entries (column 0, value 0) complete each chunk's last group.
// Pass 2 (wave = block)
// copies its region into LDS and each lane adds its row's products in
// column order through its slot list: qs[qoff[k] + (i/8)*512 + lane*8 + i%8]
// = region slot of the row's i-th entry (qoff[k+1] - qoff[k] = 512 * groups).
constexpr int kPmSlice = 4096;
constexpr int kPmRows = 64;
constexpr int kPmCap = 4096;
constexpr int kPmMaxGroups = 16;  // rows of up to 128 entries
constexpr int kPmMaxChunk = 256;  // slots (rank / 4 in 6 bits)
constexpr int kPmMaxBlocks = 1024;
struct DevPm {
    const uint32_t *lbeg;  // S + 1, relative to list/val
    const uint32_t *list;  // 2 words per group of 4 entries
    const float *val;      // null: unit values
    const uint32_t *pofs;  // S x nblk
    const uint32_t *rg;    // nblk + 1
    const uint32_t *qoff;  // nblk + 1, relative to qs
    const uint16_t *qs;
    int64_t S, nblk;
    int groups;            // max slot groups of a block (8 entries each)
    int split;             // pass-1 workgroups per slice (standalone pass)
    // fixed strides (0: none): block k's region at k * rstride, its slot
    // lists at k * qstride -- pass 2 then issues its region copy and slot
    // list loads at once, without loading rg / qoff first
    uint32_t rstride = 0, qstride = 0;
};

// The product margin's pass 2 run INSIDE the fused gradient (k_grad_lds MG,
// one rank): batch bt's blocks (pm) are summed at the launch's start and
// published per gradient phase: phase p's blocks done are counted in 8
// sub-counters cnt[((bank * 64 + p) * 8 + s) * 32] (block k in s = k % 8;
// one 128-byte line each), bank = gen & 1, which is zero when launch gen
// starts (each launch zeroes the other bank for the next; both zero when
// cnt is allocated), so gen must go up by exactly one per launch.
struct DevP2 {
    DevPm pm;
    DevBatch bt;
    float *resid;
    uint32_t *cnt;  // kMgCntWords words
    static constexpr int64_t kMgCntWords = 2 * 64 * 8 * 32;
    uint32_t gen;
    uint32_t *err = nullptr;  // DevErr words
    int fault = 0;            // kFaultMgPublish: block 0 is never published (tests)
};

// ROW-ROUND gradient (RT) of a product-margin batch (dlr_kernels.hip
// "Row-round gradient").  Round t covers batch rows [t * kRtRows, (t + 1) *
// kRtRows).  The entries of slice s in round t are gq / val [(s * rounds +
// t) * cap, + cap), in pass 1's order (64-row blocks ascending, rows
// ascending within a block): gq = batch row << 16 | slot, where slot is the
// entry's place in the slice's COLUMN-MAJOR order (columns ascending, rows
// ascending within a column); padding entries (the rest of each (slice,
// round) and each chunk's padding) carry the round's first row and slot
// kRtCap, a sink.  cend[s * kPmSlice + c] = the end of local column c's run
// in column-major order (its start is the previous column's end).
constexpr int kRtRows = 8192;       // rows per round: 32 KB of residuals in LDS
constexpr int kRtMaxRounds = 8;     // batches of up to 65,536 rows
constexpr int kRtCap = 20480;       // entries of one slice (their products live in LDS)
constexpr int kRtRegions = kRtCap / 4096;  // pass-2 regions (kPmCap floats) in the product area (MG)
constexpr int kRtMaxRound = 4096;   // entries of one (slice, round): a 4-entry group per thread
struct DevRt {
    const uint32_t *gq;
    const float *val;  // null: unit values
    const uint16_t *cend;
    int cap;     // entries per (slice, round), a multiple of 4
    int rounds;
};

// Dense rows (row-major N x D fp32, or K6r's tiled image: tiled) and 0/1
// labels as floats.
struct DevDense {
    const float *X;
    const float *label;
    int64_t N, D;
    bool tiled = false;
};

// K6r (k_dense_ref) hand-off state, device words of the loaded shard
// (zeroed at load): per chain slot of 256 rows the count of its 64-row
// margin units published, and the margin unit queue head; both monotonic
// over the launches of the shard (seq = launches so far).
struct DevRefSync {
    uint32_t *slot_cnt;
    uint32_t *head;
    uint32_t *limit;  // the margins' limit in queue positions, published by chain workgroup 0
    uint32_t seq;
    int lead;         // slots the margins may run ahead of the chains (0: no limit)
    int mgrid;        // margin workgroups (set by launch_dense_ref)
    uint32_t *err = nullptr;  // DevErr words
    int fault = 0;            // kFaultRefPublish (tests)
};

// Batch size of every rank (the L2 term of rank r's push is
// fl32(C*w)/(float)B_r); at most kMaxRanks ranks.
constexpr int kMaxRanks = 16;
struct RankSizes {
    float Bf[kMaxRanks];
    int W;
};

hipError_t launch_margin_residual(const DevBatch &bt, const float *w, float *resid, hipStream_t s);
// HOT-COLUMN PRODUCT STREAM (REFERENCE order, band mode; dlr_kernels.hip
// "Hot-column product stream").  The margin kernel, right after row i's
// residual r_i, writes fl32(r_i * x_ij) of each of the row's entries in a
// HOT column j (one with a chain of ~10^6 adds) to that column's stream in
// buf: entries t in [off[i], off[i+1]) of dest/val (val null: unit values)
// go to buf[dest[t]].  A column's stream holds its products in batch-row
// order, band by band, each band's segment starting at a multiple of
// kHotChunk floats.  off/dest/val indexed from the margin's first row (the
// caller offsets off like row_ptr).
struct DevHotOut {
    const uint32_t *off = nullptr;  // null: no hot products
    const uint32_t *dest = nullptr;
    const float *val = nullptr;
    float *buf = nullptr;
};
// The margin kernel of a band publishes the band's hot products: after it,
// flag[band] = seq (agent scope).
hipError_t launch_flag_store(uint32_t *flag, uint32_t seq, hipStream_t s);
// The hot columns' chains of one batch over bands [b0, b1) (a workgroup
// per 4 hot columns, persistent over its bands): the column's products
// streamed from buf in order, band s once flag[s] >= seq; chain sum from +0
// in batch-row order, continued across launches through state[h] (the
// first band not added, the sum so far; every launch writes it); the sum
// stored to gacc[cols[h]] by the launch that adds the last band.  seg: per
// (column h, band s) the segment's (start, count) in buf, h-major.
// The engine queues the launch for bands [b0, b1) after the margin of band
// b1 - 1 (two launches: the first bands', then the rest), so the flags a launch
// waits on come from margins queued BEFORE it: beside it on another
// hardware queue, or ahead of it when the streams share one.  A flag not
// up within `giveup` ticks (100 MHz) ends such a launch (stats[
// kStatHotGiveUps] += 1 per column; a later launch adds the rest, the same
// chain, the same bits).  Then a FINAL launch (final = 1, b0 = b1 =
// nbands) that the stream orders after the last margin by an event: empty
// when the chains are done (the usual case), it adds what a launch gave up
// on -- kernels run one at a time, as counter collection runs them, in
// whatever order across streams -- and only it records kErrHotFlag.
struct DevHotChain {
    const uint32_t *cols;
    const uint2 *seg;
    const float *buf;
    const uint32_t *flag;
    int64_t nh, nbands;
    uint32_t seq;
    uint32_t *err;
    int fault;
    uint2 *state;  // nh: (first band not added, the sum's bits)
    int64_t b0, b1;
    uint32_t giveup;
    uint32_t *stats;  // host-mapped counters (kStat*), or null
    int final_launch = 0;  // ordered after every margin: a missing flag is an error
};
constexpr int kHotChunkF = 256;  // floats of one stream chunk (a band segment starts at a multiple)
hipError_t launch_hot_chain(const DevHotChain &hc, float *gacc, hipStream_t s);
int hot_chain_grid(int64_t nh);  // workgroups (= CUs) of that launch
// The same margins with w[0, kMarginHot) staged in LDS (frequency-ordered
// shards; needs D >= kMarginHot); ho: the hot columns' products too.
constexpr int kMarginHot = 8192;
constexpr int kMarginHotWaves = 8;
hipError_t launch_margin_hot(const DevBatch &bt, const float *w, int64_t D, float *resid, hipStream_t s,
                             int reserve, const DevHotOut &ho);
inline hipError_t launch_margin_hot(const DevBatch &bt, const float *w, int64_t D, float *resid, hipStream_t s,
                                    int reserve = 0) {
    return launch_margin_hot(bt, w, D, resid, s, reserve, DevHotOut{});
}
int predict_grid(int64_t rows);
hipError_t launch_predict(const DevBatch &bt, const float *w, unsigned long long *correct, double *ll_part,
                          double *ll_out, hipStream_t s);
hipError_t launch_grad(const DevCsc &cs, int64_t D, const float *resid, float *w, float *gout, int64_t B, float lr,
                       float C, bool fused, hipStream_t s);
// Long columns: chunk sums (part[nseg] scratch), then the ordered combine
// and the update (fused) / pushed gradient (gout).
// graw != null (band layout): the long columns' raw sums G go to graw[j]
// and k_band_finalize applies the update.
hipError_t launch_grad_long(const DevLong &lg, int64_t B, const float *resid, float *w, float *gout, float *part,
                            float lr, float C, bool fused, hipStream_t s, float *graw = nullptr);
// Row bands: one launch per band, in band order, continuing gacc (zeroed
// before the first band); then the update of every column from gacc.
// longrun: the band holds runs of >= 64 entries of one column (band mode
// without the long-column split, DLR_LONG_COLUMN=0): 16-byte LDS reads.
hipError_t launch_grad_band(const DevBand &bd, const float *resid, float *gacc, hipStream_t s, bool longrun = false,
                            bool skip_hot = false);
// The band's hot pairs (waves marked in bit 31 of wstart; hw: their nhot wave
// ids): one workgroup each, beside launch_grad_band(..., skip_hot = true) of
// the same band (dlr_kernels.hip k_band_hot; bitwise the same sums).
hipError_t launch_band_hot(const DevBand &bd, const uint32_t *hw, int64_t nhot, const float *resid, float *gacc,
                           hipStream_t s, uint32_t *err = nullptr, int fault = 0);
// Long columns in row phases: piece partials part[slot], then the fixed
// combine of each column's partials [cseg[l], cseg[l+1]) into graw[j].
hipError_t launch_long_phase(const DevLPhase &lp, const uint32_t *cols, const uint32_t *cseg, int64_t ncols,
                             const float *resid, float *part, float *graw, hipStream_t s);
hipError_t launch_band_finalize(const float *gacc, float *w, float *gout, int64_t D, int64_t B, float lr, float C,
                                bool fused, hipStream_t s);
int grad_lds_fill(int64_t B);
// Rows per phase of the LDS layout for batches of up to B rows.
int64_t grad_lds_phase_rows(int64_t B);
// The LDS layout (DevPcsc row/val/ends) of one batch built on the device
// from its CSR and block bases (streamed shards); scratch: pblocks*64 uint32.
hipError_t launch_pcsc_build(const DevBatch &bt, const uint32_t *base, int P, int64_t R, int64_t pblocks,
                             uint32_t *scratch, uint8_t *ends, uint16_t *row, float *val, hipStream_t s);  // float4 fills per thread = rows per phase / 4,096
hipError_t launch_grad_lds(const DevPcsc &pc, int64_t D, int64_t B, const float *resid, float *w, float *gout,
                           float lr, float C, bool fused, hipStream_t s);
// Product margin: pass 1 (the products of pm's batch from w), pass 2 (the
// margins, sigmoid and residuals of bt's rows from those products).
// slices (optional): form only these nslices slices (device array).
hipError_t launch_pm_products(const DevPm &pm, const float *w, int64_t D, float *p, hipStream_t s,
                              const uint32_t *slices = nullptr, int64_t nslices = 0);
hipError_t launch_pm_margin(const DevPm &pm, const DevBatch &bt, const float *p, float *resid, hipStream_t s);
// Pass 1 + pass 2 of nwin consecutive windows of kPmMaxBlocks * kPmRows rows
// (band mode, TrainShard::pmw) in two launches: views[v] is window v's DevPm
// (device memory), pm0 a host copy of views[0] (S, split, groups: the same
// for every window), bt the windows' rows from the first's, window v's
// products at p + v * pstride (pstride a multiple of 64 floats).
hipError_t launch_pm_windows(const DevPm *views, const DevPm &pm0, int64_t nwin, const DevBatch &bt,
                             const float *w, int64_t D, float *p, int64_t pstride, float *resid, hipStream_t s);
// k_grad_lds (fused update) that also forms the products of the NEXT batch
// (next: its product-margin view) from the weights it has just updated:
// pass 1 for free in the gradient's workgroups (slice s = workgroup s).
// mg != null: this batch's pass 2 too, in the same launch (DevP2; resid is
// then mg->resid, written by the launch; p holds this batch's products);
// grad_lds_mg_ok says whether the batch's shape allows it.
bool grad_lds_mg_ok(const DevPm &cur, int64_t D, int64_t B, int phases, int fill);
hipError_t launch_grad_lds_pm(const DevPcsc &pc, int64_t D, int64_t B, const float *resid, float *w, float lr,
                              float C, const DevPm &next, float *p, hipStream_t s, const DevP2 *mg = nullptr);
// The row-round gradient (DevRt): the update (fused) or the pushed gradient
// (gout); next != null (fused only): also the next batch's products, as
// launch_grad_lds_pm.  resid must hold rounds * kRtRows floats.
// mg (one rank, with next): batch b's pass 2 in the same launch, as
// launch_grad_lds_pm; grad_rt_mg_ok says whether the batch's shape allows it.
hipError_t launch_grad_rt(const DevRt &rt, int64_t D, int64_t B, const float *resid, float *w, float *gout, float lr,
                          float C, bool fused, const DevPm *next, float *p, hipStream_t s, const DevP2 *mg = nullptr);
bool grad_rt_mg_ok(const DevPm &cur, int64_t D, int64_t B, int rounds, bool unit);
// Touched-column layout (dlr_kernels.hip "Touched-column layout"): cs.ptr
// spans the ncols touched columns cols[] of the batch.
hipError_t launch_grad_touched(const DevCsc &cs, const uint32_t *cols, int64_t ncols, const float *resid,
                               const float *w, float *out, int64_t B, float lr, float C, bool fused, hipStream_t s);
hipError_t launch_dense_l2(float *w, int64_t D, const RankSizes &rs, float lr, float C, int mode, hipStream_t s);
hipError_t launch_l2_fill(float *g, const float *w, int64_t D, float Bf, float C, hipStream_t s);
hipError_t launch_scatter(float *w, const uint32_t *cols, const float *newv, int64_t n, hipStream_t s);
hipError_t launch_sparse_merge(const uint32_t *lists, int64_t cap, int64_t stride, const float *w,
                               const RankSizes &rs, float lr, float C, int mode, uint32_t *out_cols, float *out_newv,
                               hipStream_t s);
// K6 dense (dlr_kernels.hip "K6: dense rows"): batch rows (first+i) mod N.
hipError_t launch_dense_margin(const DevDense &dd, int64_t first, int64_t B, const float *w, float *resid,
                               hipStream_t s);
int64_t dense_chunks(int64_t B);  // row chunks of the blocked gradient (part: chunks x roundup4(D) floats)
hipError_t launch_dense_grad(const DevDense &dd, int64_t first, int64_t B, const float *resid, float *w, float *gout,
                             float *part, bool blocked, float lr, float C, bool fused, hipStream_t s);
// K6 fused (DLR_DENSE_GRAD=fused): margin + blocked gradient partials in
// one pass over X (part: dense_chunks(B) x D), then the combine + update.
bool dense_fused_ok(int64_t D);  // D in {512, 1024, 2048, 4096}
hipError_t launch_dense_fused(const DevDense &dd, int64_t first, int64_t B, const float *w, float *part,
                              hipStream_t s);
hipError_t launch_dense_combine(const float *part, int64_t D, int64_t B, float *w, float *gout, float lr, float C,
                                bool fused, hipStream_t s);
// K6r: the reference-order dense step as one banded launch (margins +
// column chains + update).  D % 128 == 0, 512 <= D <= 4096, B <= N (the
// shard, or the streamed slot).  resid: whole 256-row slots (+4).  sync
// words: dense_ref_sync_words(B) (zeroed).
bool dense_ref_ok(int64_t D, int64_t N, int64_t B);
int64_t dense_ref_sync_words(int64_t B);
int64_t dense_ref_resid(int64_t B);
int dense_ref_grid(int64_t D, int64_t B);  // workgroups of the launch
// K6r's tiled image of a resident shard (64 x 64 tiles, chunk-major; rows
// padded to a multiple of 64): its size in floats, and the transform from
// the row-major rows.
int64_t dense_ref_tiled_floats(int64_t N, int64_t D);
hipError_t launch_dense_tile(const float *src, float *dst, int64_t N, int64_t D, hipStream_t s);
hipError_t launch_dense_ref(const DevDense &dd, int64_t first, int64_t B, float *w, float *gout, float *resid,
                            const DevRefSync &sy, float lr, float C, bool fused, hipStream_t s);
int predict_dense_grid(int64_t rows);
hipError_t launch_dense_predict(const DevDense &dd, const float *w, unsigned long long *correct, double *ll_part,
                                double *ll_out, hipStream_t s);
hipError_t launch_merge_update(const float *recv, int W, int64_t chunk, int64_t n, float *w_own, float lr, int mode,
                               hipStream_t s);

}  // namespace dlr
