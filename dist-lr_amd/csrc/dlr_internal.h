// dlr_internal.h -- shared internals of libdistlr_amd (not part of the ABI).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "distlr_amd.h"

// Host CSR shard: what distlr::DataIter holds after parsing
// (include/data_iter.h:16-35), stored sparse instead of dense.
struct dlr_dataset {
    int64_t n_rows = 0;
    int64_t D = 0;
    std::vector<int64_t> row_ptr;  // n_rows + 1
    std::vector<int32_t> col;      // 0-based, ascending, distinct per row
    std::vector<float> val;        // non-zero values
    std::vector<int32_t> label;    // 0 / 1
};

// Dense shard: what distlr::DataIter itself holds (data_iter.h:28: every
// Sample is a D-float vector), row-major N x D fp32.
struct dlr_dense {
    int64_t n_rows = 0;
    int64_t D = 0;
    std::vector<float> X;        // n_rows * D
    std::vector<int32_t> label;  // 0 / 1
};

namespace dlr {

// Thread-local "last error" for calls that have no context (and mirror of
// the context's message for calls that do).
void set_error(const std::string &msg);
const char *thread_error();

int default_threads();

// Batch plan of one epoch (data_iter.h:40-59).
struct BatchSpan {
    int64_t first_row;  // row of the shard where the batch starts
    int64_t rows;       // B (every batch has exactly B rows)
    bool contiguous;    // rows [first_row, first_row + rows) with no wrap
};
std::vector<BatchSpan> plan_batches(int64_t n_rows, int64_t batch_size);

}  // namespace dlr
