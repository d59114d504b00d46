// distlr/data_iter.h -- drop-in for the reference's include/data_iter.h.
//
// Same surface (data_iter.h:16-59): DataIter(filename, num_feature_dim),
// NextBatch(batch_size = 100) with the reference's wrap-around batching,
// HasNext().  The file is parsed once into a CSR shard (dlr_dataset) that is
// shared by every DataIter of the same (file, size, mtime, D): main.cc
// constructs a new DataIter every epoch (main.cc:158-159), which here costs
// a cache lookup instead of a re-parse.  LR::Train/Test hand the shard to
// the GPU engine; NextBatch materialises Samples only for callers that ask.
#ifndef DISTLR_AMD_DATA_ITER_H_
#define DISTLR_AMD_DATA_ITER_H_

#include <memory>
#include <string>
#include <vector>

#include "distlr/sample.h"
#include "distlr/util.h"

struct dlr_dataset;

namespace distlr {

// Shared, immutable parsed shard.
class Shard {
   public:
    explicit Shard(dlr_dataset *ds) : ds_(ds) {}
    ~Shard();
    Shard(const Shard &) = delete;
    Shard &operator=(const Shard &) = delete;
    const dlr_dataset *get() const { return ds_; }
    int64_t rows() const;
    int64_t feature_dim() const;

   private:
    dlr_dataset *ds_;
};

class DataIter {
   public:
    // data_iter.h:16-35.  Throws std::runtime_error where the reference has
    // undefined behaviour (index outside [1, D], token without ':').  A
    // missing file gives an empty iterator, as in the reference.
    explicit DataIter(std::string filename, int num_feature_dim);

    virtual ~DataIter() = default;

    // data_iter.h:40-55.  batch_size < 0 means all samples.
    std::vector<Sample> NextBatch(int batch_size = 100);

    // data_iter.h:57-59
    bool HasNext() const { return !round_end_; }

    // Engine-side accessors (not in the reference).
    const std::shared_ptr<Shard> &shard() const { return shard_; }
    int offset() const { return offset_; }
    int num_feature_dim() const { return num_feature_dim_; }
    // What NextBatch would do for a whole epoch: moves to the end state.
    void ConsumeEpoch() {
        offset_ = 0;
        round_end_ = true;
    }
    // What NextBatch would do to the position for `rows` more rows
    // (data_iter.h:49-52: offset wraps to 0 and ends the round at the end).
    void ConsumeRows(int64_t rows);
    // Drops every cached shard (frees host memory).
    static void ClearCache();

   private:
    std::string filename_;
    int num_feature_dim_;
    int offset_;
    bool round_end_;
    std::shared_ptr<Shard> shard_;
};

}  // namespace distlr

#endif  // DISTLR_AMD_DATA_ITER_H_
