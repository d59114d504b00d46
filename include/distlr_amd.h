/*
 * distlr_amd.h -- C-ABI of the MI355X-native dist-lr training engine.
 *
 * This is the drop-in boundary for dist-lr's logistic-regression hot path
 * (future-xy/dist-lr, reference at /root/reference).  Plain C types only:
 * pointers, sizes, status codes.  No exceptions, no C++ or torch types cross
 * it.  Every entry point names the reference interface it replaces.
 *
 * Conventions
 *   - Return value: 0 = OK, < 0 = error (DLR_E_*).  dlr_last_error(ctx)
 *     returns a message for the calling thread's last failure (ctx may be
 *     NULL for failures that have no context yet).
 *   - A dlr_ctx is one GPU = one rank, driven by exactly one host thread.
 *   - The caller owns every host array it passes; the library owns device
 *     buffers, datasets and contexts it returns (free with *_free/_destroy).
 *   - Host-only entry points (parsing, batching, init, formatting, key
 *     ranges) never touch a GPU and are safe without one.
 */
#ifndef DISTLR_AMD_H_
#define DISTLR_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLR_OK 0
#define DLR_E_ARG (-1)      /* bad argument / shape mismatch            */
#define DLR_E_IO (-2)       /* file cannot be opened / written          */
#define DLR_E_PARSE (-3)    /* input the reference would hit UB on      */
#define DLR_E_HIP (-4)      /* HIP runtime error                        */
#define DLR_E_RCCL (-5)     /* RCCL error                               */
#define DLR_E_NOMEM (-6)    /* host or device allocation failed         */
#define DLR_E_STATE (-7)    /* call out of order (e.g. no data loaded)  */
#define DLR_E_DEVICE (-8)   /* an in-launch hand-off never came (below) */

/* Server update semantics (main.cc:41-96, KVStoreDistServer::DataHandle). */
#define DLR_MODE_SYNC_MEAN 0  /* intended sync merge: w -= fl32(lr*sum_r g_r)/W, sum in rank order */
#define DLR_MODE_SYNC_LAST 1  /* what main.cc:71 does: only the last push (rank W-1) is applied /W */
#define DLR_MODE_ASYNC 2      /* main.cc:79-84 per push, pushes applied in rank order           */

typedef struct dlr_dataset dlr_dataset; /* host CSR shard (DataIter's storage) */
typedef struct dlr_dense dlr_dense;     /* host dense shard (DataIter's own N x D layout) */
typedef struct dlr_ctx dlr_ctx;         /* one GPU engine context (one rank)   */

/* ------------------------------------------------------------------ */
/* Host: reference parsing semantics (include/util.h, src/util.cc)      */
/* ------------------------------------------------------------------ */

/* replaces distlr::ToInt  -- src/util.cc:20-36 */
int dlr_to_int(const char *str);
/* replaces distlr::ToFloat -- src/util.cc:42-63 (digit accumulation, no sign/exponent) */
float dlr_to_float(const char *str);
/* replaces distlr::Split  -- src/util.cc:6-18; fields written NUL-separated
 * into out; returns the field count, or DLR_E_ARG if cap is too small. */
int dlr_split(const char *line, char separator, char *out, int cap);

/* ------------------------------------------------------------------ */
/* Host: datasets (include/data_iter.h, include/sample.h)              */
/* ------------------------------------------------------------------ */

/* replaces distlr::DataIter::DataIter(filename, num_feature_dim) --
 * include/data_iter.h:16-35.  Parses a libsvm text shard into CSR with the
 * reference's exact semantics (label = ToInt(tok0)==1; feature[ToInt(idx)-1]
 * = ToFloat(val), last duplicate wins; a blank line reuses the previous
 * token as its label).  Inputs the reference has undefined behaviour on
 * (index outside [1,D], token without ':') return DLR_E_PARSE with the line
 * number in the message.  nthreads <= 0 picks a default. */
int dlr_dataset_load_libsvm(const char *path, int64_t num_feature_dim, int nthreads, dlr_dataset **out);

/* Builds a dataset from caller CSR arrays (0-based ascending distinct
 * columns per row; label 0/1).  Arrays are copied. */
int dlr_dataset_from_csr(int64_t n_rows, int64_t num_feature_dim, const int64_t *row_ptr,
                         const int32_t *col, const float *val, const int32_t *label, dlr_dataset **out);

/* Seeded synthetic generator producing gen_data.py-shaped data
 * (examples/gen_data.py:18-45 layout; see DESIGN.md "Synthetic data").
 * value_mode 0: binary values "1"; 1: 4-decimal values in (0,1], held as
 * ToFloat of their text so a written+reparsed file is bitwise identical.
 * stream selects an independent row stream (part k of train, test, ...). */
typedef struct dlr_gen_spec {
    int64_t n_rows;
    int64_t num_feature_dim;
    int32_t nnz_per_row;    /* distinct uniform columns per row (<= D)   */
    int32_t value_mode;     /* 0 binary, 1 four-decimal real             */
    uint64_t seed;          /* data seed (planted model + rows)          */
    uint64_t stream;        /* row stream id                             */
    double positive_frac;   /* target fraction of +1 labels              */
    double label_noise;     /* fraction of flipped labels                */
    int32_t nthreads;       /* <= 0: default                             */
} dlr_gen_spec;
int dlr_dataset_generate(const dlr_gen_spec *spec, dlr_dataset **out);

/* Criteo-shaped hashed categorical rows (BASELINE C3): `fields` fields, each
 * drawing a value from Zipf(zipf_s) over [1, cardinality], hashed with
 * splitmix64(field, value) mod num_feature_dim; duplicates within a row
 * collapse, columns ascending, values 1.  Labels from a planted model. */
typedef struct dlr_hashed_spec {
    int64_t n_rows;
    int64_t num_feature_dim;
    int32_t fields;
    int32_t nthreads;       /* <= 0: default                             */
    int64_t cardinality;    /* values per field                          */
    double zipf_s;
    uint64_t seed;
    uint64_t stream;
    double positive_frac;
    double label_noise;
} dlr_hashed_spec;
int dlr_dataset_generate_hashed(const dlr_hashed_spec *spec, dlr_dataset **out);

/* Writes a dataset as libsvm text ("+1 idx:val ...", 1-based indices). */
int dlr_dataset_write_libsvm(const dlr_dataset *ds, const char *path, int value_mode);

/* Binary CSR cache: the parsed shard's four arrays with a checksum, so a
 * large text shard is parsed once (SURVEY 8(f) ingest).  Loading verifies
 * the checksum and the CSR invariants (DLR_E_PARSE otherwise). */
int dlr_dataset_save_binary(const dlr_dataset *ds, const char *path);
int dlr_dataset_load_binary(const char *path, dlr_dataset **out);

int dlr_dataset_info(const dlr_dataset *ds, int64_t *n_rows, int64_t *nnz, int64_t *num_feature_dim);
/* Borrowed views of the CSR arrays (valid until dlr_dataset_free). */
int dlr_dataset_view(const dlr_dataset *ds, const int64_t **row_ptr, const int32_t **col, const float **val,
                     const int32_t **label);
void dlr_dataset_free(dlr_dataset *ds);

/* Dense shards (BASELINE C4: wide dense inputs; also the reference's own
 * representation, data_iter.h:28).  Row-major N x D fp32 + 0/1 labels. */
/* Densifies a CSR dataset (what DataIter does per line, data_iter.h:28-31). */
int dlr_dense_from_dataset(const dlr_dataset *ds, dlr_dense **out);
/* Copies caller arrays X[n_rows * D] (row-major) and label[n_rows]. */
int dlr_dense_from_array(int64_t n_rows, int64_t num_feature_dim, const float *X, const int32_t *label,
                         dlr_dense **out);
/* Seeded dense rows: every feature a 4-decimal value in (0,1] (ToFloat of
 * its text, like dlr_dataset_generate's value_mode 1), planted-model labels. */
typedef struct dlr_dense_spec {
    int64_t n_rows;
    int64_t num_feature_dim;
    uint64_t seed;
    uint64_t stream;
    double positive_frac;
    double label_noise;
    int32_t nthreads;       /* <= 0: default */
    int32_t reserved;
} dlr_dense_spec;
int dlr_dense_generate(const dlr_dense_spec *spec, dlr_dense **out);
int dlr_dense_info(const dlr_dense *ds, int64_t *n_rows, int64_t *num_feature_dim);
int dlr_dense_view(const dlr_dense *ds, const float **X, const int32_t **label);
void dlr_dense_free(dlr_dense *ds);

/* replaces DataIter::NextBatch/HasNext batching -- include/data_iter.h:40-59:
 * ceil(N/B) batches per epoch (B < 0 means N); batch b holds rows
 * (b*B + i) mod N, i in [0,B) (the last batch wraps to row 0). */
int64_t dlr_num_batches(int64_t n_rows, int64_t batch_size);
int dlr_batch_rows(int64_t n_rows, int64_t batch_size, int64_t batch, int64_t *rows_out);

/* ------------------------------------------------------------------ */
/* Host: model helpers (include/lr.h, src/lr.cc)                       */
/* ------------------------------------------------------------------ */

/* replaces LR::InitWeight_ -- src/lr.cc:92-98: srand(random_state);
 * w_j = (float)rand()/(float)RAND_MAX.  glibc's TYPE_3 additive generator is
 * restated here (thread-safe, no global state). */
int dlr_init_weight(int random_state, float *w, int64_t num_feature_dim);

/* replaces LR::SaveModel's text -- src/lr.cc:73-82: "D\n", each weight in
 * default ostream format followed by ' ', then "\n".  Writes at most cap
 * bytes; *needed receives the full length. */
int dlr_format_model(const float *w, int64_t num_feature_dim, char *out, int64_t cap, int64_t *needed);

/* Key-range ownership for the data-parallel exchange: rank r "serves" keys
 * [begin, end) (the role of ps-lite's server key ranges, main.cc:98-101).
 * Ranges are equal-sized chunks of ceil(D/world) (the last may be short or
 * empty). */
int dlr_key_range(int64_t num_feature_dim, int world, int rank, int64_t *begin, int64_t *end);

/* The collectives ONE world > 1 training step issues, in order -- the same
 * on every rank (dlr_train_step issues exactly these, through RCCL or the
 * loopback group; replaces KVWorker::Push/Pull, lr.cc:116-132).
 * protocol DLR_EXCHANGE_KEY_RANGE (dense, LDS, classic and band layouts:
 * ALL_TO_ALL of every rank's pushed key ranges, the owned range merged,
 * then ALL_GATHER -- or, pieces > 1, ALL_GATHER_PART per piece -- of the
 * merged ranges) or DLR_EXCHANGE_TOUCHED (huge D: ALL_GATHER of each rank's
 * [count | cols | g] block of 1 + 2 * touched_cap words).  ops[4k .. 4k+3]
 * = (kind, words, offset, count): ALL_TO_ALL / ALL_GATHER move `words` per
 * rank; ALL_GATHER_PART moves words [offset, offset + count) of every
 * rank's `words`-word block.  Returns the op count (at most max_ops are
 * written) or < 0.  Host only. */
#define DLR_EXCHANGE_KEY_RANGE 0
#define DLR_EXCHANGE_TOUCHED 1
#define DLR_COLL_ALL_TO_ALL 1
#define DLR_COLL_ALL_GATHER 2
#define DLR_COLL_ALL_GATHER_PART 3
int dlr_exchange_plan(int protocol, int64_t num_feature_dim, int world, int pieces, int64_t touched_cap,
                      int64_t *ops, int max_ops);
/* The server side of the exchange on the HOST, from the same source as the
 * kernels (dist-lr_amd/csrc/dlr_exchange.h), for transports other than this
 * engine's (tests drive it over torch.distributed gloo).
 * dlr_merge_range: KVStoreDistServer::DataHandle (main.cc:57-84) on the
 * owned keys: w_own[i] updated from the world ranks' pushes recv[r * chunk
 * + i], r = 0 .. world-1, in rank order (k_merge_update), i < n.
 * dlr_merge_touched: the touched-list exchange's update of all D weights
 * (k_sparse_merge, k_dense_l2, k_scatter): lists = the world all-gathered
 * [count | cols[cap] | g bits[cap]] blocks (rank-major, 1 + 2 * cap uint32
 * each), batch_rows[r] = rank r's batch size (its L2 term's divisor). */
int dlr_merge_range(const float *recv, int world, int64_t chunk, int64_t n, float *w_own, float learning_rate,
                    int mode);
int dlr_merge_touched(const uint32_t *lists, int world, int64_t cap, const float *batch_rows, float *w,
                      int64_t num_feature_dim, float learning_rate, float C, int mode);
/* TEST ONLY (no GPU, no RCCL): the RCCL calls rank `rank` of `world` makes
 * for `steps` training steps -- dlr_exchange_plan's collectives issued the
 * way dlr_train_step issues them, through the RCCL transport with each RCCL
 * call recorded as a text line (name, count, peer, buffer offset) instead
 * of made.  Writes at most size bytes to out; returns the full length or
 * < 0.  Every rank's trace must pair up with the others' (same
 * collectives and counts; each ncclSend to q matched by q's ncclRecv). */
int64_t dlr_rccl_trace(int protocol, int64_t num_feature_dim, int world, int rank, int pieces, int64_t touched_cap,
                       int steps, char *out, int64_t size);

/* ------------------------------------------------------------------ */
/* Device engine (gfx950)                                              */
/* ------------------------------------------------------------------ */

/* RCCL bootstrap: rank 0 calls this and hands the 128 bytes to the others
 * (replaces ps-lite's scheduler rendezvous, main.cc:173 ps::Start). */
#define DLR_UNIQUE_ID_BYTES 128
int dlr_get_unique_id(void *id_out);

/* Creates the context of one rank on HIP device `device`.  world == 1 needs
 * no unique id (NULL); with the environment variable DLR_FORCE_COLLECTIVES=1
 * a world-1 context still runs the RCCL exchange path (a 1-rank
 * communicator), for testing it on one GPU.  Replaces the worker-side construction in RunWorker
 * (main.cc:135-138: KVWorker + LR) and the server (main.cc:116-122): with
 * replicated weights each rank also serves its key range. */
int dlr_create(int device, int rank, int world, const void *unique_id, int64_t num_feature_dim, dlr_ctx **out);
/* Creates `world` ranks' contexts, out[0..world), all on HIP device `device`
 * and linked by an in-process LOOPBACK group instead of RCCL (RCCL refuses
 * two ranks on one device): the collectives of dlr_load_train* and
 * dlr_train_step become device-to-device copies between the contexts'
 * buffers behind host barriers.  Everything else -- key ranges, the
 * rank-ordered merge, the in-place all-gather, the touched-list exchange --
 * is the same engine code as over RCCL.  Replaces ps-lite's W workers + 1
 * server sharing one machine (examples/local.sh:34-49) when there are more
 * workers than GPUs.  Each context must be driven by its own host thread
 * (every collective blocks until all ranks arrive; a rank missing for 300 s
 * fails the group).  world <= 16. */
int dlr_create_group(int device, int world, int64_t num_feature_dim, dlr_ctx **out);
/* The context's exchange transport: *nranks = ranks of its communicator (the
 * RCCL communicator's own count, ncclCommCount) or 0 without one;
 * *transport = DLR_TRANSPORT_*. */
#define DLR_TRANSPORT_NONE 0
#define DLR_TRANSPORT_RCCL 1
#define DLR_TRANSPORT_LOOPBACK 2
/* A rank that has failed and will not reach its next collective releases its
 * peers (the parameter-server topology's ParamServer::Abort for the rank
 * groups): their pending and later collectives fail with `why` instead of
 * waiting -- loopback groups at once, RCCL by ncclCommAbort (this context's
 * communicator is unusable afterwards).  No-op without a transport. */
int dlr_comm_abort(dlr_ctx *ctx, const char *why);
int dlr_comm_info(const dlr_ctx *ctx, int *nranks, int *transport);
void dlr_destroy(dlr_ctx *ctx);
const char *dlr_last_error(const dlr_ctx *ctx);

/* Weights: the initial push (main.cc:141-148) and PullWeight_ (lr.cc:116-124). */
int dlr_set_weights(dlr_ctx *ctx, const float *w, int64_t num_feature_dim);
int dlr_get_weights(dlr_ctx *ctx, float *w, int64_t num_feature_dim);

/* K1: makes the shard resident in HBM with its batch plan for batch_size
 * (DataIter + NextBatch, data_iter.h:16-59): CSR for the margin kernel and a
 * per-batch column-major copy for the deterministic gradient.  Replaces the
 * per-epoch re-parse + dense copies of main.cc:158-159.  *n_batches receives
 * the batches per epoch. */
int dlr_load_train(dlr_ctx *ctx, const dlr_dataset *ds, int64_t batch_size, int64_t *n_batches);
/* Test shard (LR::Test's NextBatch(-1), lr.cc:49). */
int dlr_load_test(dlr_ctx *ctx, const dlr_dataset *ds);
/* The dense counterparts (K6: GEMV-shaped margin and gradient kernels,
 * HBM-bound, off MFMA).  Summation order (dlr_set_summation_order): under
 * DLR_ORDER_REFERENCE (default) every margin is lr.cc:108-112's row chain
 * and every gradient lr.cc:35-39's column chain -- for large batches (C4) as
 * one banded launch that runs the row chains of one band of rows beside the
 * column chains of the bands before it; under DLR_ORDER_FAST, for batch
 * rows x D > 2^24, one FUSED pass over X (D in {512, 1024, 2048, 4096}: the
 * margin in a fixed blocked order, per-256-row-chunk gradient partials) or
 * two passes with the blocked gradient (DLR_DENSE_GRAD=blocked|fused picks
 * among these FAST variants only). */
int dlr_load_train_dense(dlr_ctx *ctx, const dlr_dense *ds, int64_t batch_size, int64_t *n_batches);
int dlr_load_test_dense(dlr_ctx *ctx, const dlr_dense *ds);

/* K1 -- residency of the next training shard (replaces DataIter's
 * per-batch copies, data_iter.h:40-55; SURVEY 8(d) C4: 20M x 4096 fp32 is
 * 328 GB, more than one GPU's HBM).  DEVICE uploads the shard once; STREAM
 * keeps it in page-locked host memory and copies each batch into one of two
 * device slots on a copy stream while the previous batch computes --
 * PCIe-bound.  Dense shards stream the caller's rows in place (registered:
 * the dlr_dense must outlive the loaded shard); sparse shards stream a
 * page-locked, batch-major copy of their CSR and per-batch column-major
 * slices, each batch staged by ONE copy (every
 * layout except band mode, whose one >= 2^21-row batch is not worth
 * streaming: DLR_E_ARG).  AUTO (default) streams only when the shard would
 * not leave 8 GiB of HBM free.  Results are bitwise identical either way.
 * dlr_train_residency reports what the loaded shard uses. */
#define DLR_RESIDENCY_AUTO 0
#define DLR_RESIDENCY_DEVICE 1
#define DLR_RESIDENCY_STREAM 2
int dlr_set_residency(dlr_ctx *ctx, int mode);
int dlr_train_residency(dlr_ctx *ctx);

/* TUNING of the loads (one struct instead of scattered switches).  The
 * engine picks layouts and kernel forms itself at dlr_load_train* time;
 * each field below can force one choice (DLR_AUTO = the engine's pick).
 * None of them changes the arithmetic order (DLR_ORDER_REFERENCE stays
 * bitwise the oracle's whatever is forced), only the layout and kernels
 * doing it.  Unless dlr_set_tuning was called, every load takes the fields
 * from the environment variable named beside each (dlr_tuning_from_env),
 * so A/B runs need no code.
 *   grad_layout          DLR_GRAD_KERNEL  classic|lds|touched -> DLR_LAYOUT_*
 *   product_margin       DLR_PM           0 off; 1 required (the load fails
 *                                         if the batches do not fit it)
 *   pm_fused             DLR_PM_FUSED     0: the next batch's pass 1 in its own launch
 *   pm_in_gradient       DLR_PM_MG        0: pass 2 in its own launch (no
 *                                         one-launch step)
 *   pm_split             DLR_PM_SPLIT     pass-1 workgroups per slice (separate pass 1)
 *   row_rounds           DLR_GRAD_RT      0 never / 1 whenever the batch fits
 *                                         the row-round gradient (auto: <= 2 rounds)
 *   band_rows            DLR_BAND_ROWS    rows per band (power of two; 0 off)
 *   band_pipeline        DLR_BAND_PIPE    0: margin, then the bands' gradient
 *   band_hot             DLR_BAND_HOT     entries that make a column hot (0 none)
 *   hot_stream           DLR_HOT_STREAM   0: hot columns in k_band_hot
 *   hot_stream_max       DLR_HOT_STREAM_MAX  most streamed hot columns a batch (64)
 *   margin_hot           DLR_MARGIN_HOT   0/1: the LDS hot-weight margin
 *   long_column          DLR_LONG_COLUMN  FAST order: entries of a long column
 *   long_piece           DLR_LONG_PIECE   FAST order: entries per long piece (63)
 *   long_sched           DLR_LONG_SCHED   0: long chunks in chunk order
 *   relabel              DLR_RELABEL      0/1: frequency order of the columns
 *   relabel_tail         DLR_RELABEL_TAIL 0 id, 1, 2 (default) first occurrence
 *   relabel_rare         DLR_RELABEL_RARE count below which a column is rare (16)
 *   unit_values          DLR_UNIT_VALUES  0: keep the value array of an all-1 shard
 *   stream_coalesce      DLR_STREAM_COALESCE  0: one copy per streamed array
 *   stream_device_layout DLR_STREAM_DEVICE_LAYOUT  0: stream the host-built layout
 *   dense_grad           DLR_DENSE_GRAD   FAST order: 0 chain, 1 blocked, 2 fused
 *                                         (fused|blocked in the environment)
 *   dense_ref            DLR_DENSE_REF    0/1: K6r, the one-launch dense step
 *   dense_ref_lead       DLR_DENSE_REF_LEAD  K6r margin lead in slots (64; 0 none)
 * Process-level switches stay in the environment (read at dlr_create*):
 * DLR_RESIDENCY (dlr_set_residency's default), DLR_FORCE_COLLECTIVES (RCCL
 * at one rank), DLR_LOOPBACK_SYNC and DLR_LOOPBACK_TIMEOUT_S (loopback
 * group). */
#define DLR_AUTO (-1)
typedef struct dlr_tuning {
    int64_t grad_layout, product_margin, pm_fused, pm_in_gradient, pm_split, row_rounds;
    int64_t band_rows, band_pipeline, band_hot, hot_stream, hot_stream_max, margin_hot;
    int64_t long_column, long_piece, long_sched;
    int64_t relabel, relabel_tail, relabel_rare, unit_values;
    int64_t stream_coalesce, stream_device_layout;
    int64_t dense_grad, dense_ref, dense_ref_lead;
} dlr_tuning;
/* Every field DLR_AUTO. */
void dlr_tuning_default(dlr_tuning *t);
/* DLR_AUTO, then each field whose environment variable is set. */
void dlr_tuning_from_env(dlr_tuning *t);
/* The tuning of the context's later loads (t = NULL: back to the
 * environment at each load, the default); dlr_get_tuning: the tuning the
 * last load used (or the set one, before any load). */
int dlr_set_tuning(dlr_ctx *ctx, const dlr_tuning *t);
int dlr_get_tuning(dlr_ctx *ctx, dlr_tuning *t);

/* Summation order of the next training shard's sums (applies at the next
 * dlr_load_train / dlr_load_train_dense; every rank must ask for the same
 * order, else the load fails on every rank).
 *   DLR_ORDER_REFERENCE (default): every margin is summed in column order
 *     (lr.cc:108-112) and every gradient column in batch-row order
 *     (lr.cc:35-39) -- results bitwise those of the reference's arithmetic
 *     (the oracle), on every layout and at every size.
 *   DLR_ORDER_FAST: where the reference order is a serial chain of 10^5 -
 *     10^6 dependent adds (C3's Zipf-hot columns in full-shard batches, C4's
 *     65,536-row column sums), a fixed reordering: long sparse columns
 *     summed in row-phase pieces combined by a fixed tree (DLR_LONG_COLUMN
 *     sets the entry threshold), dense gradients by 256-row chunks (and, in
 *     the fused dense pass, each margin by 64 lane partials combined by a
 *     butterfly).  Deterministic; within the north-star tolerance (DESIGN.md
 *     §3 states what each option measured).
 * dlr_summation_order reports what the LOADED shard's kernels use:
 * DLR_ORDER_FAST only if some sum of it is actually reordered (e.g. a FAST
 * request on a shard with no long column is still the reference order). */
#define DLR_ORDER_REFERENCE 0
#define DLR_ORDER_FAST 1
int dlr_set_summation_order(dlr_ctx *ctx, int order);
int dlr_summation_order(dlr_ctx *ctx);

/* One step of LR::Train's loop body (lr.cc:30-43) plus the server update
 * (main.cc:57-84) for batch `batch` of the loaded shard: margin + sigmoid +
 * residual (K2), segmented Xᵀr gradient + L2 (K3), key-range exchange over
 * RCCL (world > 1), fused SGD update (K4).  Enqueued on the context's stream;
 * returns without waiting.  lr/C are the server learning rate
 * (LEARNING_RATE, main.cc:27) and LR's C (lr.h:10). */
int dlr_train_step(dlr_ctx *ctx, int64_t batch, float learning_rate, float C, int mode);
/* All batches of one epoch in order (LR::Train, lr.cc:28-45); ends with
 * dlr_sync, so DLR_OK means the epoch's kernels completed without a device
 * error. */
int dlr_train_epoch(dlr_ctx *ctx, float learning_rate, float C, int mode);

/* Parameter-server topology without RCCL (several contexts on one GPU, or a
 * host-side exchange): the worker half and the server half of one step.
 * dlr_worker_gradient: LR::Train's pushed vector for `batch` (lr.cc:34-43:
 * K2 + K3 unfused, normalised + L2), copied to grad_out[D]; blocks.
 * dlr_server_apply: KVStoreDistServer::DataHandle's update (main.cc:57-84)
 * of the W pushes grads[W*D] (rank-major) to this context's weights (K4);
 * blocks. */
int dlr_worker_gradient(dlr_ctx *ctx, int64_t batch, float C, float *grad_out, int64_t num_feature_dim);
int dlr_server_apply(dlr_ctx *ctx, const float *grads, int num_workers, int64_t num_feature_dim, float learning_rate,
                     int mode);

/* LR::Test (lr.cc:47-63): counts (z > 0) == label over the test shard (K5);
 * *logloss receives the summed log-loss (our addition; NULL to skip).
 * Blocks until done. */
int dlr_predict(dlr_ctx *ctx, int64_t *correct, int64_t *n_rows, double *logloss);

/* Waits for all work on the context's stream.
 *
 * In-launch hand-offs.  Some kernels hand data between workgroups of one
 * launch (the one-launch C2 step: rows summed by one CU, their residuals
 * used by all; K6r: margins -> column chains) or between the waves of one
 * workgroup.  Like the reference's worker, which waits until its pulled data
 * is there (lr.cc:122, 131), a consumer never proceeds on data whose
 * producer has not published it -- but a wait is bounded (250 ms), so a
 * producer that never comes cannot hang the GPU: the wait records what it
 * waited for, and dlr_sync, dlr_get_weights, dlr_predict,
 * dlr_worker_gradient, dlr_stage_time and every later dlr_train_step return
 * DLR_E_DEVICE (dlr_last_error names the hand-off) until the next
 * dlr_load_train*.  Launches whose workgroups wait for each other are never
 * larger than what the device holds at once (they fall back to separate
 * launches), so a healthy run never sees it. */
int dlr_sync(dlr_ctx *ctx);

/* TEST ONLY: withhold one producer of the next steps' in-launch hand-offs
 * (0 = none; 1 = the one-launch step's margin block 0 never publishes; 2 =
 * K6r's margin unit 0 never publishes; 3 = k_band_hot's product waves never
 * post) -- the steps must then fail with DLR_E_DEVICE. */
int dlr_set_fault(dlr_ctx *ctx, int fault);

/* Per-kernel timing with HIP events on the context's stream.  enable=1
 * starts recording (clears totals); dlr_kernel_time returns the summed
 * milliseconds and launch count of kernel `which` (0 margin, 1 gradient,
 * 2 update/merge, 3 exchange, 4 step total) since enabling; syncs first. */
int dlr_timing(dlr_ctx *ctx, int enable);
int dlr_kernel_time(dlr_ctx *ctx, int which, double *total_ms, int64_t *launches);
/* Average duration of ONE kernel stage over `count` consecutive launches on
 * batches first, first+1, ... (mod the epoch), between a single HIP-event
 * pair on the context's stream -- the per-launch event overhead of
 * dlr_timing is gone, so the figure is comparable with rocprofv3's kernel
 * durations.  stage: DLR_STAGE_MARGIN (K2), DLR_STAGE_GRADIENT (K3 with the
 * fused single-rank update, or the pushed gradient when world > 1; for the
 * touched layout the touched-column gradient), DLR_STAGE_UPDATE (the
 * touched layout's dense L2 pass + scatter).  The stages run without their
 * partners, so the weights end up changed: use after the measured run.
 * Blocks. */
#define DLR_STAGE_MARGIN 0
#define DLR_STAGE_GRADIENT 1
#define DLR_STAGE_UPDATE 2
int dlr_stage_time(dlr_ctx *ctx, int stage, int64_t first_batch, int64_t count, float learning_rate, float C,
                   double *avg_ms);

/* Event counts of the steps since the training shard was loaded (n <= 
 * DLR_COUNTERS entries into out; syncs the context's streams first):
 *   DLR_COUNT_HOT_CHAIN_LAUNCHES  k_hot_chain launches queued (C3's hot
 *                                 columns: three per step -- two after the
 *                                 margins of their last band, and a final
 *                                 one ordered after the last margin, empty
 *                                 unless a launch gave up);
 *   DLR_COUNT_HOT_GIVEUPS         hot chains that stopped at a band flag not
 *                                 up within 20 ms and left the band to a
 *                                 later launch (same bits, but the step ran
 *                                 serialised behind that wait; 0 in a
 *                                 healthy run);
 *   DLR_COUNT_COWAIT_SERIALISED   co-waiting launches (one-launch step, K6r,
 *                                 hot chains) that another context's
 *                                 co-waiting launch in this process was
 *                                 queued ahead of on another stream, so the
 *                                 launch was ordered after it;
 *   DLR_COUNT_MG_DEMOTED          steps run with a separate pass-2 launch
 *                                 because an earlier one-launch step of this
 *                                 context ran out of its in-launch wait.
 * The reference has no such counters: they report how this engine met
 * lr.cc:122/131's "wait until the data is there". */
#define DLR_COUNT_HOT_CHAIN_LAUNCHES 0
#define DLR_COUNT_HOT_GIVEUPS 1
#define DLR_COUNT_COWAIT_SERIALISED 2
#define DLR_COUNT_MG_DEMOTED 3
#define DLR_COUNTERS 4
int dlr_stage_counters(dlr_ctx *ctx, int64_t *out, int n);

/* Column-major layout the loaded training shard uses for the gradient
 * (chosen by dlr_load_train; DLR_GRAD_KERNEL=classic|lds|touched forces
 * one): the LDS-resident-residual layout for batches of <= 65,536 rows,
 * the touched-column layout when batches touch few of the D columns
 * (huge D), else the classic layout.  Returns a DLR_LAYOUT_* value or < 0. */
#define DLR_LAYOUT_CLASSIC 0
#define DLR_LAYOUT_LDS 1
#define DLR_LAYOUT_TOUCHED 2
int dlr_train_layout(dlr_ctx *ctx);

/* Rows per band when the classic layout's short columns are summed in ROW
 * BANDS (large batches such as BASELINE C3's 12.5M-row full-shard batch:
 * each band's residual slice stays in an XCD's L2), else 0.  Bitwise the
 * same sums as without bands (each column's running sum continues from band
 * to band in batch-row order).  DLR_BAND_ROWS=<rows> (a power of two; 0 =
 * off) overrides the default of 2^20 rows for batches of >= 2^21 rows.
 * Under DLR_ORDER_FAST the long columns of a band-mode batch are summed per
 * row phase of 16,384 rows and the phase partials combined by a fixed tree
 * (deterministic; within 1e-5 of the single sequential sum); under
 * DLR_ORDER_REFERENCE every column is one chain in batch-row order. */
int dlr_train_band_rows(dlr_ctx *ctx);

/* 1 when the loaded sparse training shard's columns are relabeled in
 * frequency order (Zipf-skewed shards such as BASELINE C3: the hot weights
 * then share cache lines in the margin's gathers), else 0.  Chosen at load
 * over the ranks' summed column counts (DLR_RELABEL=0|1 forces it).  A pure
 * renaming: every sum keeps its order and results are bitwise unchanged;
 * weights, pushed gradients and test shards keep the original numbering at
 * this API (a dense test shard cannot be loaded beside a relabeled one). */
int dlr_train_relabeled(dlr_ctx *ctx);

/* 1 when every value of the loaded sparse training shard is exactly 1.0f
 * (one-hot / binary features: a9a, Criteo-style hashed fields, BASELINE C1,
 * C3, C5), else 0.  Such a shard stores no value arrays (4 bytes per entry
 * less in HBM and per pass) and its kernels never read values:
 * fl32(t * 1.0f) == t, so results are bitwise those of the valued path.
 * Decided at load; DLR_UNIT_VALUES=0 keeps the value arrays.  A test shard
 * is checked the same way on its own. */
int dlr_train_unit_values(dlr_ctx *ctx);

/* The margin of the loaded sparse training shard: 0 = gathers (one weight
 * read per entry), 1 = PRODUCT MARGIN with a separate pass 1, 2 = product
 * margin with pass 1 inside the previous step's gradient (one rank), 3 = as
 * 2 and pass 2 inside the step's own gradient launch (one rank, LDS-phase
 * gradient, rows of <= 64 entries: the launch sums the batch's rows first and
 * hands the residuals to the gradient's phases through device-scope counters;
 * DLR_PM_MG=0 keeps it a launch of its own; a shard whose launch would have
 * more workgroups than the device holds at once -- they wait for each other
 * -- gets 2).  The
 * product margin (LDS-layout batches, >= 128 column slices of 4,096; resident
 * shards) forms every product fl32(w_j * x_ij) by column slice from LDS-staged
 * weights, then sums each row's products in column order from LDS: bitwise
 * the gather margin.  DLR_PM=0 turns it off, DLR_PM=1 on for any batches that
 * fit; DLR_PM_FUSED=0 keeps pass 1 separate.  Replaces lr.cc:108-114's
 * Sigmoid_ dot product for these shards (same arithmetic).  Band-mode
 * batches (>= 2^21 rows, e.g. a full-shard batch) without the hot-weight
 * margin run it over windows of 65,536 rows (pass 1 and pass 2 per window:
 * reported as 1). */
int dlr_train_product_margin(dlr_ctx *ctx);
/* The product margin's region layout of the loaded shard: 1 when every
 * batch (or window) keeps its regions and slot lists at fixed strides
 * (uniform rows: pass 2 then loads no offsets first), 0 when none does
 * (packed: ragged rows), 2 when some do; 0 without the product margin.
 * Either way the same products and sums. */
int dlr_train_pm_strided(dlr_ctx *ctx);

/* Band mode, REFERENCE order: the hot columns (>= DLR_BAND_HOT entries in a
 * batch, default 2^17: C3's Zipf heads) whose chains run from the HOT-COLUMN
 * PRODUCT STREAM -- the margin kernel writes each hot product fl32(r_i *
 * x_ij) as it computes r_i, and ONE launch per step adds every hot column's
 * products in batch-row order over all bands (k_hot_chain) -- returns the
 * most hot columns of a batch; 0 when the hot chains run per band from
 * gathered residuals (k_band_hot: DLR_HOT_STREAM=0, more than 64 hot
 * columns, or no LDS hot-weight margin) or there are none.  Same products,
 * same order: lr.cc:35-39's sums either way. */
int dlr_train_hot_columns(dlr_ctx *ctx);

/* The gradient kernel of a product-margin shard: the number of 8,192-row
 * rounds of the ROW-ROUND gradient (k_grad_rt: the batch read in pass 1's
 * row-major order, products transposed into column order in LDS; default
 * for batches of <= 2 rounds, DLR_GRAD_RT), or 0 for the phase-split LDS
 * gradient (k_grad_lds) / any other layout.  Same arithmetic either way
 * (lr.cc:35-40, bitwise). */
int dlr_train_row_rounds(dlr_ctx *ctx);

/* World > 1 with the product margin: the exchange overlapped with the next
 * batch's margin (BASELINE north_star).  The in-place all-gather of the
 * merged weights (lr.cc:122's Pull) runs in pieces (dlr_set_exchange_pieces)
 * on a second stream --
 * RCCL grouped send/recv of each rank's piece, or device copies on the
 * loopback group -- and the next batch's pass 1 forms each 4,096-column
 * slice as soon as every weight in it has landed (the slices of this rank's
 * own key range right after the merge).  The step's results are unchanged
 * (the same products; tests/test_gpu_pm.py).  On by default;
 * dlr_set_exchange_overlap(ctx, 0) uses the plain all-gather and forms the
 * products at the next margin.  The ranks AGREE on it (the two forms are
 * different collective sequences): at load, the pieced form is used only if
 * every rank has the product margin and asks for it; called with a shard
 * loaded, dlr_set_exchange_overlap is collective (every rank calls it at the
 * same point of its step sequence).  dlr_exchange_overlap reports 1 when the
 * loaded shard's steps use it. */
int dlr_set_exchange_overlap(dlr_ctx *ctx, int on);
int dlr_exchange_overlap(dlr_ctx *ctx);

/* Pieces of that all-gather, 1 .. 16, or 0 (default) = auto: one piece per
 * 4 MiB of the key range a rank owns, 1 to 4 -- and when that is one piece
 * (C2 at any W), no overlap: the plain all-gather, then the next margin's
 * pass 1 (one own-range slice group is all one piece could hide).  More
 * pieces start the next margin's slices earlier, each piece costs a
 * collective's latency; an explicit 1 is one in-place all-gather with the
 * own-range pass 1 beside it.
 * A load-time setting: it applies to the next dlr_load_train, where the
 * ranks must agree on it (DLR_E_ARG otherwise).  dlr_exchange_pieces: the
 * loaded shard's piece count, 0 when its steps do not piece the gather. */
int dlr_set_exchange_pieces(dlr_ctx *ctx, int pieces);
int dlr_exchange_pieces(dlr_ctx *ctx);

/* Device bytes resident for the loaded shards (for reporting). */
int dlr_memory_info(dlr_ctx *ctx, int64_t *train_bytes, int64_t *test_bytes);

/* Host -> device bytes staged per training batch of a STREAMED shard (K1):
 * the mean and the maximum over the epoch's batches of exactly what one
 * batch's copies move (dense: the batch's rows; sparse: the coalesced slices
 * -- the CSR and block bases, not the column-major layout built on the
 * device).  0 / 0 for a device-resident shard.  For bench's PCIe figure. */
int dlr_stream_bytes(dlr_ctx *ctx, int64_t *mean_bytes, int64_t *max_bytes);

#ifdef __cplusplus
}
#endif

#endif /* DISTLR_AMD_H_ */
