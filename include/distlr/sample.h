// distlr/sample.h -- drop-in for the reference's include/sample.h.
//
// Same public surface (sample.h:14-57).  Storage is sparse (ascending
// column, non-zero value) with the dense feature vector materialised on
// demand by GetFeature()/GetSample(), so a Sample of a 2^28-feature model
// costs its non-zeros, not 1 GiB.
#ifndef DISTLR_AMD_SAMPLE_H_
#define DISTLR_AMD_SAMPLE_H_

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace distlr {

class Sample {
   public:
    // sample.h:14-16: an all-zero sample of num_feature_dim features.
    explicit Sample(int num_feature_dim);

    // sample.h:18-20: from a dense feature vector and a label.
    explicit Sample(std::vector<float> &feature, int label);

    // Sparse constructor (not in the reference): ascending columns.
    Sample(int num_feature_dim, std::vector<int32_t> cols, std::vector<float> vals, int label);

    virtual ~Sample() {}

    void SetLabel(int label) { label_ = label; }

    void SetFeatures(const std::vector<float> &feature);

    std::pair<std::vector<float>, int> GetSample() { return std::make_pair(GetFeature(), label_); }

    std::vector<float> GetFeature();

    float GetFeature(int index);

    int GetLabel() const { return label_; }

    // sample.h:49-57: label, then " i:v" for every non-zero feature with a
    // 0-based index and std::to_string formatting.
    std::string DebugInfo();

    // Sparse accessors (not in the reference).
    int NumFeatureDim() const { return num_feature_dim_; }
    const std::vector<int32_t> &Columns() const { return cols_; }
    const std::vector<float> &Values() const { return vals_; }

   private:
    int num_feature_dim_;
    std::vector<int32_t> cols_;
    std::vector<float> vals_;
    int label_ = 0;
};

}  // namespace distlr

#endif  // DISTLR_AMD_SAMPLE_H_
