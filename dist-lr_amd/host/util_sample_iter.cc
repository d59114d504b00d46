// util_sample_iter.cc -- the drop-in util / Sample / DataIter surface
// (include/distlr/{util,sample,data_iter}.h) over the C-ABI.
#include <sys/stat.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "distlr/data_iter.h"
#include "distlr/sample.h"
#include "distlr/util.h"
#include "distlr_amd.h"

namespace distlr {

// ------------------------------------------------------------------ util

std::vector<std::string> Split(std::string line, char separator) {
    std::vector<char> buf(2 * (line.size() + 1) * (line.size() + 2) + 16);
    const int n = dlr_split(line.c_str(), separator, buf.data(), (int)buf.size());
    std::vector<std::string> out;
    const char *p = buf.data();
    for (int i = 0; i < n; ++i) {
        out.emplace_back(p);
        p += out.back().size() + 1;
    }
    return out;
}

int ToInt(const char *str) { return dlr_to_int(str); }
int ToInt(const std::string &str) { return dlr_to_int(str.c_str()); }
float ToFloat(const char *str) { return dlr_to_float(str); }
float ToFloat(const std::string &str) { return dlr_to_float(str.c_str()); }

// ------------------------------------------------------------------ Sample

Sample::Sample(int num_feature_dim) : num_feature_dim_(num_feature_dim) {}

Sample::Sample(std::vector<float> &feature, int label) : num_feature_dim_((int)feature.size()), label_(label) {
    SetFeatures(feature);
}

Sample::Sample(int num_feature_dim, std::vector<int32_t> cols, std::vector<float> vals, int label)
    : num_feature_dim_(num_feature_dim), cols_(std::move(cols)), vals_(std::move(vals)), label_(label) {}

void Sample::SetFeatures(const std::vector<float> &feature) {
    num_feature_dim_ = (int)feature.size();
    cols_.clear();
    vals_.clear();
    for (size_t j = 0; j < feature.size(); ++j)
        if (feature[j] != 0.0f) {
            cols_.push_back((int32_t)j);
            vals_.push_back(feature[j]);
        }
}

std::vector<float> Sample::GetFeature() {
    std::vector<float> x((size_t)std::max(num_feature_dim_, 0), 0.0f);
    for (size_t k = 0; k < cols_.size(); ++k) x[(size_t)cols_[k]] = vals_[k];
    return x;
}

float Sample::GetFeature(int index) {
    auto it = std::lower_bound(cols_.begin(), cols_.end(), index);
    return (it != cols_.end() && *it == index) ? vals_[(size_t)(it - cols_.begin())] : 0.0f;
}

std::string Sample::DebugInfo() {
    std::string str = std::to_string(label_);
    for (size_t k = 0; k < cols_.size(); ++k) str += " " + std::to_string(cols_[k]) + ":" + std::to_string(vals_[k]);
    return str;
}

// ------------------------------------------------------------------ DataIter

Shard::~Shard() { dlr_dataset_free(ds_); }

int64_t Shard::rows() const {
    int64_t n = 0;
    dlr_dataset_info(ds_, &n, nullptr, nullptr);
    return n;
}

int64_t Shard::feature_dim() const {
    int64_t d = 0;
    dlr_dataset_info(ds_, nullptr, nullptr, &d);
    return d;
}

namespace {
struct CacheKey {
    std::string file;
    int dim;
    long long size, mtime_ns;
    bool operator<(const CacheKey &o) const {
        return std::tie(file, dim, size, mtime_ns) < std::tie(o.file, o.dim, o.size, o.mtime_ns);
    }
};
std::mutex g_cache_mu;
std::map<CacheKey, std::shared_ptr<Shard>> g_cache;

std::shared_ptr<Shard> empty_shard(int D) {
    const int64_t rp[1] = {0};
    dlr_dataset *ds = nullptr;
    if (dlr_dataset_from_csr(0, std::max(D, 1), rp, nullptr, nullptr, nullptr, &ds) != DLR_OK)
        throw std::runtime_error(dlr_last_error(nullptr));
    return std::make_shared<Shard>(ds);
}
}  // namespace

DataIter::DataIter(std::string filename, int num_feature_dim)
    : filename_(filename), num_feature_dim_(num_feature_dim), offset_(0), round_end_(false) {
    struct stat st;
    if (stat(filename_.c_str(), &st) != 0) {  // reference: unopened file -> 0 samples
        shard_ = empty_shard(num_feature_dim);
        return;
    }
    const CacheKey key{filename_, num_feature_dim, (long long)st.st_size,
                       (long long)st.st_mtim.tv_sec * 1000000000ll + st.st_mtim.tv_nsec};
    {
        std::lock_guard<std::mutex> g(g_cache_mu);
        auto it = g_cache.find(key);
        if (it != g_cache.end()) {
            shard_ = it->second;
            return;
        }
    }
    dlr_dataset *ds = nullptr;
    // DISTLR_CSR_CACHE=1: reuse <file>.dlrcsr (dlr_dataset_save_binary) when
    // it is newer than the text and holds the same D; else parse and write it
    const char *cc = getenv("DISTLR_CSR_CACHE");
    const bool use_cache = cc && strcmp(cc, "1") == 0;
    const std::string cache = filename_ + ".dlrcsr";
    if (use_cache) {
        struct stat cs;
        if (stat(cache.c_str(), &cs) == 0 &&
            (cs.st_mtim.tv_sec > st.st_mtim.tv_sec ||
             (cs.st_mtim.tv_sec == st.st_mtim.tv_sec && cs.st_mtim.tv_nsec >= st.st_mtim.tv_nsec)) &&
            dlr_dataset_load_binary(cache.c_str(), &ds) == DLR_OK) {
            int64_t n = 0, nnz = 0, d = 0;
            dlr_dataset_info(ds, &n, &nnz, &d);
            if (d != num_feature_dim) {
                dlr_dataset_free(ds);
                ds = nullptr;
            }
        }
    }
    if (!ds) {
        const int rc = dlr_dataset_load_libsvm(filename_.c_str(), num_feature_dim, 0, &ds);
        if (rc == DLR_E_IO) {
            shard_ = empty_shard(num_feature_dim);
            return;
        }
        if (rc != DLR_OK) throw std::runtime_error(std::string("DataIter: ") + dlr_last_error(nullptr));
        if (use_cache) (void)dlr_dataset_save_binary(ds, cache.c_str());  // best effort (read-only dirs)
    }
    shard_ = std::make_shared<Shard>(ds);
    std::lock_guard<std::mutex> g(g_cache_mu);
    g_cache[key] = shard_;
}

void DataIter::ClearCache() {
    std::lock_guard<std::mutex> g(g_cache_mu);
    g_cache.clear();
}

void DataIter::ConsumeRows(int64_t rows) {
    const int64_t n = shard_->rows();
    if (n == 0 || rows <= 0) {
        if (n == 0) round_end_ = true;
        return;
    }
    const int64_t end = (int64_t)offset_ + rows;
    if (end >= n) round_end_ = true;
    offset_ = (int)(end % n);
}

std::vector<Sample> DataIter::NextBatch(int batch_size) {
    const int64_t n = shard_->rows();
    if (batch_size < 0) batch_size = (int)n;
    std::vector<Sample> batch;
    if (n == 0) {  // the reference indexes an empty vector here; end the round instead
        round_end_ = true;
        return batch;
    }
    const int64_t *rp;
    const int32_t *col;
    const float *val;
    const int32_t *lab;
    dlr_dataset_view(shard_->get(), &rp, &col, &val, &lab);
    batch.reserve((size_t)batch_size);
    for (int i = 0; i < batch_size; ++i) {
        const int64_t r = offset_;
        batch.emplace_back(num_feature_dim_, std::vector<int32_t>(col + rp[r], col + rp[r + 1]),
                           std::vector<float>(val + rp[r], val + rp[r + 1]), lab[r]);
        if (++offset_ == (int)n) {
            offset_ = 0;
            round_end_ = true;
        }
    }
    return batch;
}

}  // namespace distlr
