// lr.cc -- the drop-in distlr::LR / distlr::KVWorker (include/distlr/lr.h)
// over the C-ABI.  Mirrors src/lr.cc's behaviour:
//   LR ctor + InitWeight_  lr.cc:13-17, 92-98   (glibc rand restated)
//   Train                  lr.cc:28-45           (GPU steps, K2..K4)
//   Test                   lr.cc:47-63           (GPU K5 + the same print)
//   GetWeight / SaveModel / DebugInfo lr.cc:65-90 (last PULLED weights)
#include "distlr/lr.h"

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <ctime>
#include <mutex>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <stdexcept>
#include <string>

#include "distlr_amd.h"

namespace distlr {

namespace {
void check(int rc, dlr_ctx *ctx, const char *what) {
    if (rc < 0) throw std::runtime_error(std::string(what) + ": " + dlr_last_error(ctx));
}
}  // namespace

// ------------------------------------------------------------------ ParamServer

struct ParamServer::State {
    std::mutex mu;
    std::condition_variable cv;
    dlr_ctx *ctx = nullptr;
    int64_t D = 0;
    float lr = 0;
    int mode = DLR_MODE_SYNC_MEAN;
    std::vector<float> grads;  // W x D, rank-major
    int arrived = 0;
    uint64_t generation = 0;
    bool initialised = false;
    std::string failure;  // set once a step failed (or a worker aborted): every Push then throws
};

ParamServer::ParamServer(int device, int num_workers, float learning_rate, bool sync_mode, int64_t D)
    : st_(new State), num_workers_(num_workers) {
    st_->D = D;
    st_->lr = learning_rate;
    const char *m = getenv("DISTLR_SYNC_MERGE");
    st_->mode = !sync_mode ? DLR_MODE_ASYNC
                           : ((m && std::string(m) == "last") ? DLR_MODE_SYNC_LAST : DLR_MODE_SYNC_MEAN);
    st_->grads.assign((size_t)num_workers * (size_t)D, 0.0f);
    check(dlr_create(device, 0, 1, nullptr, D, &st_->ctx), nullptr, "ParamServer: dlr_create");
}

ParamServer::~ParamServer() {
    dlr_destroy(st_->ctx);
    delete st_;
}

void ParamServer::Init(const std::vector<float> &w) {
    std::lock_guard<std::mutex> g(st_->mu);
    if (st_->initialised) return;
    check(dlr_set_weights(st_->ctx, w.data(), st_->D), st_->ctx, "ParamServer::Init");
    st_->initialised = true;
}

void ParamServer::Pull(std::vector<float> &w) {
    std::lock_guard<std::mutex> g(st_->mu);
    if (!st_->initialised) throw std::logic_error("ParamServer::Pull before Init (main.cc:86 CHECK)");
    w.resize((size_t)st_->D);
    check(dlr_get_weights(st_->ctx, w.data(), st_->D), st_->ctx, "ParamServer::Pull");
}

void ParamServer::Push(int rank, const std::vector<float> &grad) {
    std::unique_lock<std::mutex> lk(st_->mu);
    if (!st_->failure.empty()) throw std::runtime_error(st_->failure);
    std::copy(grad.begin(), grad.end(), st_->grads.begin() + (size_t)rank * (size_t)st_->D);
    const uint64_t gen = st_->generation;
    if (++st_->arrived == num_workers_) {
        // The last arrival applies the step.  On failure every waiting
        // worker is released with the same error instead of blocking forever
        // (the reference's server CHECK-aborts the process, main.cc:49).
        const int rc = dlr_server_apply(st_->ctx, st_->grads.data(), num_workers_, st_->D, st_->lr, st_->mode);
        if (rc < 0) st_->failure = std::string("ParamServer::Push: ") + dlr_last_error(st_->ctx);
        st_->arrived = 0;
        ++st_->generation;
        st_->cv.notify_all();
    } else {
        st_->cv.wait(lk, [&] { return st_->generation != gen || !st_->failure.empty(); });
    }
    if (!st_->failure.empty()) throw std::runtime_error(st_->failure);
}

void ParamServer::Abort(const std::string &why) {
    std::lock_guard<std::mutex> g(st_->mu);
    if (st_->failure.empty()) st_->failure = why;
    st_->cv.notify_all();
}

// ------------------------------------------------------------------ KVWorker

KVWorker::KVWorker(int device, int rank, ParamServer *ps, float learning_rate, bool sync_mode,
                   int64_t num_feature_dim)
    : ps_(ps), rank_(rank), world_(ps->num_workers()), learning_rate_(learning_rate), sync_mode_(sync_mode) {
    check(dlr_create(device, 0, 1, nullptr, num_feature_dim, &ctx_), nullptr, "dlr_create");
}

KVWorker::KVWorker(int device, int rank, int world, const void *unique_id, float learning_rate, bool sync_mode,
                   int64_t num_feature_dim)
    : rank_(rank), world_(world), learning_rate_(learning_rate), sync_mode_(sync_mode) {
    check(dlr_create(device, rank, world, unique_id, num_feature_dim, &ctx_), nullptr, "dlr_create");
}

KVWorker::KVWorker(dlr_ctx *ctx, int rank, int world, float learning_rate, bool sync_mode)
    : ctx_(ctx), rank_(rank), world_(world), learning_rate_(learning_rate), sync_mode_(sync_mode) {}

std::vector<KVWorker *> KVWorker::Group(int device, int world, float learning_rate, bool sync_mode,
                                        int64_t num_feature_dim) {
    std::vector<dlr_ctx *> ctx((size_t)world, nullptr);
    check(dlr_create_group(device, world, num_feature_dim, ctx.data()), nullptr, "dlr_create_group");
    std::vector<KVWorker *> out;
    for (int r = 0; r < world; ++r) out.push_back(new KVWorker(ctx[(size_t)r], r, world, learning_rate, sync_mode));
    return out;
}

KVWorker::~KVWorker() { dlr_destroy(ctx_); }

void KVWorker::Abort(const std::string &why) {
    if (ps_)
        ps_->Abort(why);
    else
        (void)dlr_comm_abort(ctx_, why.c_str());
}

int KVWorker::mode() const {
    if (!sync_mode_) return DLR_MODE_ASYNC;
    const char *m = getenv("DISTLR_SYNC_MERGE");  // "last": main.cc:71 as written
    return (m && std::string(m) == "last") ? DLR_MODE_SYNC_LAST : DLR_MODE_SYNC_MEAN;
}

// ------------------------------------------------------------------ LR

LR::LR(int num_feature_dim, float learning_rate, float C, int random_state)
    : num_feature_dim_(num_feature_dim), learning_rate_(learning_rate), C_(C), random_state_(random_state) {
    InitWeight_();
}

void LR::InitWeight_() {
    weight_.assign((size_t)num_feature_dim_, 0.0f);
    check(dlr_init_weight(random_state_, weight_.data(), num_feature_dim_), nullptr, "dlr_init_weight");
}

void LR::SetKVWorker(KVWorker *kv) {
    if (kv_ && kv_ != kv) delete kv_;
    kv_ = kv;
    // The initial push (main.cc:141-148): every rank holds the same
    // InitWeight_ result, so each sets its replica directly.
    if (!kv_) return;
    if (kv_->ps() && rank_ == 0) kv_->ps()->Init(weight_);
    check(dlr_set_weights(kv_->ctx(), weight_.data(), num_feature_dim_), kv_->ctx(), "dlr_set_weights");
}

void LR::SetRank(int rank) { rank_ = rank; }

KVWorker *LR::GetKVWorker() { return kv_; }

std::vector<float> LR::GetWeight() { return weight_; }

void LR::PullWeight_() {
    if (kv_->ps()) {  // parameter-server topology: the server holds the truth
        kv_->ps()->Pull(weight_);
        check(dlr_set_weights(kv_->ctx(), weight_.data(), num_feature_dim_), kv_->ctx(), "dlr_set_weights");
        return;
    }
    check(dlr_get_weights(kv_->ctx(), weight_.data(), num_feature_dim_), kv_->ctx(), "dlr_get_weights");
}

namespace {
// The shard's rows starting at row k, wrapping (row i of the result is row
// (k + i) mod N): batch m of it is NextBatch's m-th batch after k rows were
// consumed (data_iter.h:40-55), so a partially consumed DataIter trains the
// same rows in the same order as lr.cc:29-30's loop.
std::shared_ptr<Shard> rotated_shard(const Shard &sh, int64_t k) {
    const int64_t n = sh.rows();
    const int64_t *rp;
    const int32_t *col;
    const float *val;
    const int32_t *lab;
    dlr_dataset_view(sh.get(), &rp, &col, &val, &lab);
    std::vector<int64_t> rp2((size_t)n + 1, 0);
    std::vector<int32_t> col2, lab2((size_t)n);
    std::vector<float> val2;
    col2.reserve((size_t)rp[n]);
    val2.reserve((size_t)rp[n]);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t r = (k + i) % n;
        col2.insert(col2.end(), col + rp[r], col + rp[r + 1]);
        val2.insert(val2.end(), val + rp[r], val + rp[r + 1]);
        rp2[(size_t)i + 1] = (int64_t)col2.size();
        lab2[(size_t)i] = lab[r];
    }
    dlr_dataset *ds = nullptr;
    check(dlr_dataset_from_csr(n, sh.feature_dim(), rp2.data(), col2.data(), val2.data(), lab2.data(), &ds), nullptr,
          "LR::Train: dlr_dataset_from_csr");
    return std::make_shared<Shard>(ds);
}
}  // namespace

void LR::Train(DataIter &iter, int /*num_iter*/, int batch_size) {
    if (!kv_) throw std::logic_error("LR::Train: SetKVWorker first");
    if (!iter.HasNext()) return;  // lr.cc:29: nothing left in this round
    std::shared_ptr<Shard> sh = iter.shard();
    const int64_t n = sh->rows();
    if (n == 0) throw std::runtime_error("LR::Train: empty shard (the reference never terminates)");
    if (batch_size == 0) throw std::runtime_error("LR::Train: batch_size 0 (the reference never terminates)");
    const int64_t bs = batch_size < 0 ? n : batch_size;
    // A DataIter that NextBatch already advanced k rows (lr.cc:29-30 trains
    // what is left of the round): batches of bs rows from row k on, wrapping
    // to row 0, ceil((n - k) / bs) of them, as NextBatch would hand them out;
    // trained from the shard rotated by k rows.
    // The cache is keyed on the caller's shard (kept alive in train_src) and
    // the rotation, never on a rotated copy's address.
    const int64_t k = iter.offset();
    const int64_t nb_run = k != 0 ? (n - k + bs - 1) / bs : -1;  // -1: every batch of the loaded plan
    dlr_ctx *ctx = kv_->ctx();
    if (kv_->train_shard != sh.get() || kv_->train_rot != k || kv_->train_batch != batch_size) {
        std::shared_ptr<Shard> load = k != 0 ? rotated_shard(*sh, k) : sh;
        int64_t nb = 0;
        kv_->train_shard = nullptr;  // nothing valid is resident if the load fails
        check(dlr_load_train(ctx, load->get(), batch_size, &nb), ctx, "dlr_load_train");
        kv_->train_shard = sh.get();
        kv_->train_rot = k;
        kv_->train_keep = load;
        kv_->train_src = sh;
        kv_->train_batch = batch_size;
        kv_->train_batches = nb;
    }
    const int64_t nb = nb_run < 0 ? kv_->train_batches : nb_run;
    const float lr = kv_->learning_rate();
    const int mode = kv_->mode();
    if (kv_->ps()) {  // worker half on this GPU, server half in ParamServer
        std::vector<float> grad((size_t)num_feature_dim_);
        for (int64_t b = 0; b < nb; ++b) {
            PullWeight_();
            check(dlr_worker_gradient(ctx, b, C_, grad.data(), num_feature_dim_), ctx, "dlr_worker_gradient");
            kv_->ps()->Push(rank_, grad);
        }
    } else {
        for (int64_t b = 0; b < nb; ++b) {
            // Every batch pulls before it computes (lr.cc:32); only the last
            // pull of the epoch is observable (GetWeight/SaveModel), so only
            // it is copied to the host.
            if (b == nb - 1) PullWeight_();
            check(dlr_train_step(ctx, b, lr, C_, mode), ctx, "dlr_train_step");
        }
        check(dlr_sync(ctx), ctx, "dlr_sync");
    }
    if (k == 0)
        iter.ConsumeEpoch();
    else
        iter.ConsumeRows(nb * bs);
}

void LR::Test(DataIter &iter, int num_iter) {
    if (!kv_) throw std::logic_error("LR::Test: SetKVWorker first");
    dlr_ctx *ctx = kv_->ctx();
    PullWeight_();  // lr.cc:48
    const std::shared_ptr<Shard> &sh = iter.shard();
    const int64_t n = sh->rows();
    int64_t correct = 0;
    double ll = 0;
    if (n > 0) {
        if (kv_->test_shard != sh.get()) {
            check(dlr_load_test(ctx, sh->get()), ctx, "dlr_load_test");
            kv_->test_shard = sh.get();
            kv_->test_keep = sh;
        }
        int64_t rows = 0;
        check(dlr_predict(ctx, &correct, &rows, &ll), ctx, "dlr_predict");
    }
    iter.ConsumeEpoch();  // NextBatch(-1) (lr.cc:49)
    last_correct_ = correct;
    last_total_ = n;
    last_logloss_ = ll;
    // lr.cc:50-55: acc is a float counter (it stops growing at 2^24).
    const float acc = correct >= (1 << 24) ? 16777216.0f : (float)correct;
    time_t rawtime;
    time(&rawtime);
    struct tm tmv;
    localtime_r(&rawtime, &tmv);
    std::cout << std::setw(2) << tmv.tm_hour << ':' << std::setw(2) << tmv.tm_min << ':' << std::setw(2)
              << tmv.tm_sec << " Iteration " << num_iter << ", accuracy: " << acc / (float)(size_t)n << std::endl;
}

bool LR::SaveModel(std::string &filename) {
    int64_t need = 0;
    dlr_format_model(weight_.data(), num_feature_dim_, nullptr, 0, &need);
    std::string text((size_t)need, '\0');
    dlr_format_model(weight_.data(), num_feature_dim_, &text[0], need, &need);
    std::ofstream fout(filename.c_str(), std::ios::binary);
    fout << text;
    fout.close();
    return true;  // lr.cc:81: the reference reports success unconditionally
}

std::string LR::DebugInfo() {
    int64_t need = 0;
    dlr_format_model(weight_.data(), num_feature_dim_, nullptr, 0, &need);
    std::string text((size_t)need, '\0');
    dlr_format_model(weight_.data(), num_feature_dim_, &text[0], need, &need);
    // drop the "D\n" header and the trailing "\n": lr.cc:84-90 is "w w w "
    const size_t nl = text.find('\n');
    std::string body = text.substr(nl + 1);
    if (!body.empty() && body.back() == '\n') body.pop_back();
    return body;
}

}  // namespace distlr
