// distlr/lr.h -- drop-in for the reference's include/lr.h.
//
// Same class and methods (lr.h:8-54).  The single intentional API change:
// the ps-lite handle ps::KVWorker<float>* becomes distlr::KVWorker*, a
// handle on one rank of the MI355X engine (GPU, rank/world, RCCL id) that
// also carries the server-side settings the reference reads in its
// KVStoreDistServer (SYNC_MODE, LEARNING_RATE: main.cc:26-27).  As in the
// reference, LR owns the handle it is given (lr.h:13-15 deletes it).
#ifndef DISTLR_AMD_LR_H_
#define DISTLR_AMD_LR_H_

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "distlr/data_iter.h"

struct dlr_ctx;

namespace distlr {

// In-process parameter server for the parameter-server topology: W worker
// threads that may share GPUs push their gradients, the server context
// merges them in rank order once all W arrived (main.cc:57-84) and every
// worker pulls the result.  Used when there are more workers than GPUs
// (e.g. local.sh's 2 workers on one GPU); one GPU per worker uses RCCL.
class ParamServer {
   public:
    ParamServer(int device, int num_workers, float learning_rate, bool sync_mode, int64_t num_feature_dim);
    ~ParamServer();
    ParamServer(const ParamServer &) = delete;
    ParamServer &operator=(const ParamServer &) = delete;

    // The first push initialises the weights (main.cc:50-56).
    void Init(const std::vector<float> &w);
    void Pull(std::vector<float> &w);
    // Blocks until the step of all W pushes has been applied.
    // Throws if the step failed; then every later Push throws too.
    void Push(int rank, const std::vector<float> &grad);
    // Releases the workers waiting in Push with an error (a worker that
    // cannot push any more, e.g. it threw, calls this so its peers stop).
    void Abort(const std::string &why);
    int num_workers() const { return num_workers_; }

   private:
    struct State;
    State *st_;
    int num_workers_;
};

// Replaces ps::KVWorker<float> + the server process.  world > 1 needs the
// same 128-byte unique id on every rank (dlr_get_unique_id on rank 0).
class KVWorker {
   public:
    KVWorker(int device, int rank, int world, const void *unique_id, float learning_rate, bool sync_mode,
             int64_t num_feature_dim);
    // Parameter-server topology: this worker's own context on `device`,
    // exchanging through `ps` (not owned).
    KVWorker(int device, int rank, ParamServer *ps, float learning_rate, bool sync_mode, int64_t num_feature_dim);
    // Loopback-group topology: the `world` ranks of one device linked
    // in-process (dlr_create_group) -- the same world > 1 engine step as
    // over RCCL when there are more workers than GPUs.  Drive each
    // returned worker from its own thread.
    static std::vector<KVWorker *> Group(int device, int world, float learning_rate, bool sync_mode,
                                         int64_t num_feature_dim);
    ParamServer *ps() const { return ps_; }
    // This worker failed and will not reach its next exchange: release its
    // peers (ParamServer::Abort for the parameter-server topology,
    // dlr_comm_abort for RCCL / loopback-group ranks).
    void Abort(const std::string &why);
    ~KVWorker();
    KVWorker(const KVWorker &) = delete;
    KVWorker &operator=(const KVWorker &) = delete;

    dlr_ctx *ctx() const { return ctx_; }
    int rank() const { return rank_; }
    int world() const { return world_; }
    float learning_rate() const { return learning_rate_; }
    int mode() const;  // DLR_MODE_* from sync_mode
    // Device residency cache: the shard currently resident for training
    // (the caller's shard, the row it starts from -- LR::Train loads a
    // partially consumed DataIter's shard rotated by that many rows -- and
    // the batch size) and for testing.  train_keep holds what was loaded,
    // train_src the caller's shard (so its address is not reused while cached).
    const Shard *train_shard = nullptr;
    int64_t train_rot = 0;
    int64_t train_batch = 0;
    int64_t train_batches = 0;
    const Shard *test_shard = nullptr;
    std::shared_ptr<Shard> train_keep, train_src, test_keep;

   private:
    KVWorker(dlr_ctx *ctx, int rank, int world, float learning_rate, bool sync_mode);  // adopts ctx
    dlr_ctx *ctx_ = nullptr;
    ParamServer *ps_ = nullptr;
    int rank_, world_;
    float learning_rate_;
    bool sync_mode_;
};

class LR {
   public:
    explicit LR(int num_feature_dim, float learning_rate = 0.001, float C_ = 1, int random_state = 0);

    virtual ~LR() { delete kv_; }

    // Takes ownership; pushes this LR's initial weights (main.cc:141-148).
    void SetKVWorker(KVWorker *kv);

    void SetRank(int rank);

    // lr.cc:28-45: one epoch over iter's remaining batches on the GPU
    // (consumes iter like NextBatch does).
    void Train(DataIter &iter, int num_iter, int batch_size);

    // lr.cc:47-63: pulls the latest weights, evaluates the whole of iter on
    // the GPU and prints "HH:MM:SS Iteration N, accuracy: A".
    void Test(DataIter &iter, int num_iter);

    // Last pulled weights (lr.cc:65-67).
    std::vector<float> GetWeight();

    KVWorker *GetKVWorker();

    // lr.cc:73-82: text model of the last pulled weights.
    bool SaveModel(std::string &filename);

    // lr.cc:84-90
    std::string DebugInfo();

    // Not in the reference: the last Test's results.
    int64_t last_correct() const { return last_correct_; }
    int64_t last_total() const { return last_total_; }
    double last_logloss() const { return last_logloss_; }

   private:
    void InitWeight_();
    void PullWeight_();

    int num_feature_dim_;
    float learning_rate_;
    float C_;
    int random_state_;
    int rank_ = 0;
    std::vector<float> weight_;
    KVWorker *kv_ = nullptr;
    int64_t last_correct_ = 0, last_total_ = 0;
    double last_logloss_ = 0;
};

}  // namespace distlr

#endif  // DISTLR_AMD_LR_H_
