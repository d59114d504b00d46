/*
 * lr_cpu_omp.c -- "BUILD CPU PATH, NOT REFERENCE": an efficient multi-core
 * CPU logistic-regression trainer, used ONLY as bench.py's second CPU
 * baseline.  Not the product (the product
 * has no CPU path) and not the parity oracle: its sums are reordered across
 * threads, so it is checked against the oracle with a tolerance only
 * (tests/test_cpu_baselines.py).
 *
 * Same step as the engine (lr.cc:28-45 + main.cc:70-72 for one worker):
 * residuals r_i = sigma(w.x_i) - y_i for the batch rows (b*B + i) mod N
 * (data_iter.h:40-55), G = X_b^T r, g_j = G_j/B + C w_j/B (lr.cc:40) for
 * every j, w_j -= lr g_j.  OpenMP over rows; the gradient goes to
 * per-thread column arrays reduced in parallel (or float atomics when
 * threads x D would exceed 2 GiB: huge-D configs).  Threads: OpenMP's
 * default (OMP_NUM_THREADS; 16 on the GPU box's CPU share).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static double now_s(void) { return omp_get_wtime(); }

int cpu_omp_threads(void) { return omp_get_max_threads(); }

/* steps sparse steps from batch `first_batch`; val NULL = unit values.
 * Returns seconds, or -1 on a bad argument / allocation failure. */
double cpu_omp_train_csr(const int64_t *row_ptr, const int32_t *col, const float *val, const int32_t *y,
                         int64_t N, int64_t D, int64_t B, float *w, float lr, float C, int64_t first_batch,
                         int64_t steps) {
    if (N <= 0 || D <= 0 || B == 0) return -1.0;
    if (B < 0) B = N;
    const int64_t nb = (N + B - 1) / B;
    const int T = omp_get_max_threads();
    const int priv = (double)T * (double)D * 4.0 <= 2147483648.0;
    float *resid = (float *)malloc(sizeof(float) * (size_t)B);
    float *G = (float *)malloc(sizeof(float) * (size_t)D * (size_t)(priv ? T : 1));
    if (!resid || !G) {
        free(resid);
        free(G);
        return -1.0;
    }
    const double t0 = now_s();
    for (int64_t s = 0; s < steps; ++s) {
        const int64_t off = (((first_batch + s) % nb) * B) % N;
#pragma omp parallel
        {
            const int t = omp_get_thread_num();
            float *Gt = G + (priv ? (size_t)t * (size_t)D : 0);
            if (priv) memset(Gt, 0, sizeof(float) * (size_t)D);
            else {
#pragma omp for schedule(static)
                for (int64_t j = 0; j < D; ++j) G[j] = 0.0f;
            }
#pragma omp for schedule(static)
            for (int64_t i = 0; i < B; ++i) {
                const int64_t r = (off + i) % N;
                float z = 0.0f;
                for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) z += w[col[k]] * (val ? val[k] : 1.0f);
                resid[i] = (float)(1.0 / (1.0 + exp(-(double)z))) - (float)y[r];
            }
            /* implicit barrier: w is read above, written below */
#pragma omp for schedule(static)
            for (int64_t i = 0; i < B; ++i) {
                const int64_t r = (off + i) % N;
                const float ri = resid[i];
                for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
                    const float c = ri * (val ? val[k] : 1.0f);
                    if (priv) {
                        Gt[col[k]] += c;
                    } else {
#pragma omp atomic
                        G[col[k]] += c;
                    }
                }
            }
#pragma omp for schedule(static)
            for (int64_t j = 0; j < D; ++j) {
                float g = G[j];
                if (priv)
                    for (int q = 1; q < T; ++q) g += G[(size_t)q * (size_t)D + (size_t)j];
                const float gj = g / (float)B + C * w[j] / (float)B;
                w[j] -= lr * gj;
            }
        }
    }
    const double el = now_s() - t0;
    free(resid);
    free(G);
    return el;
}

/* Dense rows X (N x D row-major). */
double cpu_omp_train_dense(const float *X, const int32_t *y, int64_t N, int64_t D, int64_t B, float *w, float lr,
                           float C, int64_t first_batch, int64_t steps) {
    if (N <= 0 || D <= 0 || B == 0) return -1.0;
    if (B < 0) B = N;
    const int64_t nb = (N + B - 1) / B;
    const int T = omp_get_max_threads();
    float *resid = (float *)malloc(sizeof(float) * (size_t)B);
    float *G = (float *)malloc(sizeof(float) * (size_t)D * (size_t)T);
    if (!resid || !G) {
        free(resid);
        free(G);
        return -1.0;
    }
    const double t0 = now_s();
    for (int64_t s = 0; s < steps; ++s) {
        const int64_t off = (((first_batch + s) % nb) * B) % N;
#pragma omp parallel
        {
            const int t = omp_get_thread_num();
            float *Gt = G + (size_t)t * (size_t)D;
            memset(Gt, 0, sizeof(float) * (size_t)D);
#pragma omp for schedule(static)
            for (int64_t i = 0; i < B; ++i) {
                const int64_t r = (off + i) % N;
                const float *x = X + (size_t)r * (size_t)D;
                float z = 0.0f;
                for (int64_t j = 0; j < D; ++j) z += w[j] * x[j];
                const float ri = (float)(1.0 / (1.0 + exp(-(double)z))) - (float)y[r];
                resid[i] = ri;
            }
#pragma omp for schedule(static)
            for (int64_t i = 0; i < B; ++i) {
                const float *x = X + (size_t)((off + i) % N) * (size_t)D;
                const float ri = resid[i];
                for (int64_t j = 0; j < D; ++j) Gt[j] += ri * x[j];
            }
#pragma omp for schedule(static)
            for (int64_t j = 0; j < D; ++j) {
                float g = 0.0f;
                for (int q = 0; q < T; ++q) g += G[(size_t)q * (size_t)D + (size_t)j];
                const float gj = g / (float)B + C * w[j] / (float)B;
                w[j] -= lr * gj;
            }
        }
    }
    const double el = now_s() - t0;
    free(resid);
    free(G);
    return el;
}
