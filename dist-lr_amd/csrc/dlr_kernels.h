// dlr_kernels.h -- launchers of the gfx950 kernels (dlr_kernels.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace dlr {

// One batch as CSR: rows [0, rows) with row_ptr[i] absolute offsets into
// col/val (row_ptr may point into the middle of the shard's array).
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
};

hipError_t launch_margin_residual(const DevBatch &bt, const float *w, float *resid, hipStream_t s);
int predict_grid(int64_t rows);
hipError_t launch_predict(const DevBatch &bt, const float *w, unsigned long long *correct, double *ll_part,
                          double *ll_out, hipStream_t s);
hipError_t launch_grad(const DevCsc &cs, int64_t D, const float *resid, float *w, float *gout, int64_t B, float lr,
                       float C, bool fused, hipStream_t s);
hipError_t launch_merge_update(const float *recv, int W, int64_t chunk, int64_t n, float *w_own, float lr, int mode,
                               hipStream_t s);

}  // namespace dlr
