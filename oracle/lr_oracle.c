/*
 * lr_oracle.c -- CPU restatement of future-xy/dist-lr's logistic-regression
 * path.  TEST INFRASTRUCTURE ONLY: this file is the checker, never the thing
 * measured or shipped.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it (as oracle/build/liblr_oracle.so).
 *
 * Pinning status (see DESIGN.md "Oracle"):
 *   - orc_to_int / orc_to_float / orc_split / orc_parse_*: PINNED against the
 *     reference itself -- oracle/_ref is compiled from
 *     /root/reference/src/util.cc + include/data_iter.h and its outputs are the
 *     golden fixtures under tests/golden/ (tests/golden/make_golden.py).
 *   - orc_init_weight: pinned by glibc's own srand/rand (the reference's
 *     dependency, lr.cc:92-98) and the known first value 1804289383.
 *   - orc_grad_* / orc_server_update / orc_predict_*: restatement of
 *     src/lr.cc and src/main.cc.  Those files include ps-lite's "ps/ps.h"
 *     (an un-vendored submodule, /root/reference/ps-lite is empty), so they
 *     are unbuildable here and this arithmetic is "parity unpinned" by
 *     reference execution: it follows the cited lines operation by operation.
 *
 * Floating-point contract: built with -O2 -ffp-contract=off (no FMA), x86-64
 * SSE (FLT_EVAL_METHOD 0), glibc exp -- the same arithmetic the reference
 * gets from g++ -O3 on x86-64 (no -mfma).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- parsing */

/* util.cc:20-36  ToInt: optional sign, then r = r*10 + (c-'0') with no
 * validation.  Signed overflow wraps (two's complement), as the -O3 build
 * does in practice. */
int orc_to_int(const char *str) {
    int flag = 1;
    uint32_t ret = 0;
    const char *p = str;
    if (*p == '-') {
        ++p;
        flag = -1;
    } else if (*p == '+') {
        ++p;
    }
    while (*p) {
        ret = ret * 10u + (uint32_t)(int)(*p - '0');
        ++p;
    }
    return (int)((uint32_t)flag * ret);
}

/* util.cc:42-63  ToFloat: digit accumulation in float; '.' resets base to
 * (float)0.1; base *= 0.1 is evaluated in double then stored as float; no
 * sign and no exponent handling. */
float orc_to_float(const char *str) {
    float integer = 0, decimal = 0;
    float base = 1;
    const char *p = str;
    while (*p) {
        if (*p == '.') {
            base = (float)0.1;
            ++p;
            continue;
        }
        if ((double)base >= 1.0) {
            integer = integer * 10.0f + (float)(*p - '0');
        } else {
            decimal = decimal + base * (float)(*p - '0');
            base = (float)((double)base * 0.1);
        }
        ++p;
    }
    return integer + decimal;
}

/* util.cc:6-18  Split: note substr(start, pos) uses the ABSOLUTE position of
 * the separator as the length (correct only for <= 2 fields).  Fields are
 * written NUL-separated into out; returns the field count or -1 if cap is
 * too small. */
int orc_split(const char *line, char sep, char *out, int cap) {
    size_t len = strlen(line);
    size_t start = 0;
    int n = 0, used = 0;
    for (;;) {
        const char *hit = (start <= len) ? memchr(line + start, sep, len - start) : NULL;
        size_t cnt;
        if (hit) {
            size_t pos = (size_t)(hit - line);
            cnt = pos;                       /* the reference's quirk */
            if (cnt > len - start) cnt = len - start;
            if (used + (int)cnt + 1 > cap) return -1;
            memcpy(out + used, line + start, cnt);
            used += (int)cnt;
            out[used++] = '\0';
            ++n;
            start = pos + 1;
        } else {
            cnt = len - start;
            if (used + (int)cnt + 1 > cap) return -1;
            memcpy(out + used, line + start, cnt);
            used += (int)cnt;
            out[used++] = '\0';
            ++n;
            return n;
        }
    }
}

static int is_ws(char c) {   /* isspace() in the "C" locale, as operator>> uses */
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

/* Reads the whole file; returns malloc'd buffer (NUL-terminated) or NULL. */
static char *slurp(const char *path, size_t *len_out) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)sz + 1);
    if (!buf) { fclose(f); return NULL; }
    size_t got = fread(buf, 1, (size_t)sz, f);
    fclose(f);
    buf[got] = '\0';
    *len_out = got;
    return buf;
}

/* data_iter.h:16-35  DataIter ctor, dense.  For each getline() line: first
 * token (operator>>, whitespace-delimited) is the label, label = ToInt==1;
 * a blank line keeps the PREVIOUS token in buf (operator>> leaves it
 * untouched on failure).  Remaining tokens: Split(':'), feature[ToInt-1] =
 * ToFloat (last duplicate wins).  X (n x D, row-major) and y may be NULL to
 * count lines only.  Returns the sample count, or a negative error:
 *   -1 cannot open, -2 token without ':' (reference: out-of-bounds read),
 *   -3 feature index outside [1, D] (reference: unchecked write),
 *   -4 more samples than cap.  Line numbers of errors go to *err_line. */
long orc_parse_dense(const char *path, int D, float *X, int *y, long cap, long *err_line) {
    size_t len;
    char *txt = slurp(path, &len);
    if (!txt) return -1;
    char buf[4096];
    buf[0] = '\0';
    char fields[8192];
    long n = 0;
    size_t p = 0;
    long line_no = 0;
    while (p < len) {                      /* std::getline: stop at EOF w/o chars */
        size_t e = p;
        while (e < len && txt[e] != '\n') ++e;
        ++line_no;
        /* tokenise txt[p, e) */
        size_t q = p;
        int first = 1;
        int label = 0;
        if (X && n < cap) memset(X + (size_t)n * D, 0, sizeof(float) * (size_t)D);
        for (;;) {
            while (q < e && is_ws(txt[q])) ++q;
            if (q >= e) {
                if (first) label = (orc_to_int(buf) == 1) ? 1 : 0;  /* blank line */
                break;
            }
            size_t t = q;
            while (t < e && !is_ws(txt[t])) ++t;
            size_t tl = t - q;
            if (tl >= sizeof(buf)) tl = sizeof(buf) - 1;
            memcpy(buf, txt + q, tl);
            buf[tl] = '\0';
            q = t;
            if (first) {
                label = (orc_to_int(buf) == 1) ? 1 : 0;
                first = 0;
                continue;
            }
            int nf = orc_split(buf, ':', fields, (int)sizeof(fields));
            if (nf < 2) { free(txt); if (err_line) *err_line = line_no; return -2; }
            const char *f0 = fields;
            const char *f1 = fields + strlen(fields) + 1;
            int idx = orc_to_int(f0) - 1;
            if (idx < 0 || idx >= D) { free(txt); if (err_line) *err_line = line_no; return -3; }
            if (X) {
                if (n >= cap) { free(txt); return -4; }
                X[(size_t)n * D + idx] = orc_to_float(f1);
            }
        }
        if (y) {
            if (n >= cap) { free(txt); return -4; }
            y[n] = label;
        }
        ++n;
        p = (e < len) ? e + 1 : e;
    }
    free(txt);
    return n;
}

/* Dense -> CSR (ascending column, non-zero values only).  The sparse port
 * below is bitwise equal to the dense loops because every skipped term is a
 * product with an exact 0 (w*0 and r*0 are +-0, which never change a
 * running fp32 sum that starts at +0). */
long orc_dense_to_csr(const float *X, long n, int D, int64_t *row_ptr, int32_t *col, float *val, long cap) {
    long k = 0;
    row_ptr[0] = 0;
    for (long i = 0; i < n; ++i) {
        for (int j = 0; j < D; ++j) {
            float v = X[(size_t)i * D + j];
            if (v != 0.0f) {
                if (k >= cap) return -1;
                col[k] = j;
                val[k] = v;
                ++k;
            }
        }
        row_ptr[i + 1] = k;
    }
    return k;
}

/* ---------------------------------------------------------------- batching */

/* data_iter.h:40-55  NextBatch(B): B<0 -> all samples; copies B samples
 * starting at offset, wrapping to row 0 (and ending the round) when the
 * offset reaches N.  Batch b of an epoch therefore holds rows
 * (b*B + i) mod N for i in [0, B).  Returns the batch count of an epoch
 * (ceil(N/B)); fills rows_out[B] for batch_idx if rows_out != NULL. */
long orc_batch_rows(long N, long B, long batch_idx, int64_t *rows_out) {
    if (N <= 0) return 0;
    if (B < 0) B = N;
    if (B == 0) return -1;                 /* reference loops forever */
    long nb = (N + B - 1) / B;
    if (rows_out) {
        long off = (batch_idx * B) % N;
        for (long i = 0; i < B; ++i) {
            rows_out[i] = off;
            if (++off == N) off = 0;
        }
    }
    return nb;
}

/* ---------------------------------------------------------------- model */

/* lr.cc:92-98  InitWeight_: srand(random_state); w_j = (float)rand() /
 * (float)RAND_MAX.  Uses glibc itself (the reference's dependency). */
void orc_init_weight(int random_state, float *w, long D) {
    srand((unsigned)random_state);
    for (long j = 0; j < D; ++j) w[j] = (float)rand() / (float)RAND_MAX;
}

/* lr.cc:108-114  Sigmoid_: z = sum_j w_j*x_j in fp32, j ascending, separate
 * multiply and add; sigma = 1./(1.+exp(-z)) in double (glibc exp), returned
 * as float. */
static float sigmoid_dense(const float *w, const float *x, int D) {
    float z = 0;
    for (int j = 0; j < D; ++j) z = z + w[j] * x[j];
    return (float)(1. / (1. + exp(-(double)z)));
}

static float margin_csr(const float *w, const int32_t *col, const float *val, int64_t a, int64_t b) {
    float z = 0;
    for (int64_t k = a; k < b; ++k) z = z + w[col[k]] * val[k];
    return z;
}

/* lr.cc:34-41  one batch of LR::Train, dense.  rows[B] indexes X.  The
 * reference recomputes Sigmoid_ for every (j, sample) pair; the value is a
 * pure function of (w, x) so computing it once per sample is bitwise equal.
 *   grad[j] = sum_{s in batch order} fl32((sigma_s - y_s) * x_sj)   (fp32)
 *   grad[j] = fl32(1.*grad[j]/B + (double)(fl32(C*w_j) / (float)B))  (lr.cc:40)
 * sig_scratch needs B floats. */
void orc_grad_dense(const float *X, const int *y, int D, const int64_t *rows, long B,
                    const float *w, float C, float *grad, float *sig_scratch) {
    for (long s = 0; s < B; ++s) {
        const float *x = X + (size_t)rows[s] * D;
        sig_scratch[s] = sigmoid_dense(w, x, D) - (float)y[rows[s]];
    }
    for (int j = 0; j < D; ++j) {
        float g = 0;
        for (long s = 0; s < B; ++s) {
            const float *x = X + (size_t)rows[s] * D;
            g = g + sig_scratch[s] * x[j];
        }
        double bs = (double)B;                               /* batch.size() */
        grad[j] = (float)(1. * (double)g / bs + (double)((C * w[j]) / (float)B));
    }
}

/* Sparse port of orc_grad_dense (bitwise equal, see orc_dense_to_csr).
 * Column sums are accumulated in batch-row order, so they equal the dense
 * j-outer / sample-inner loop exactly.  resid_scratch needs B floats. */
void orc_grad_csr(const int64_t *row_ptr, const int32_t *col, const float *val, const int *y,
                  long D, const int64_t *rows, long B, const float *w, float C,
                  float *grad, float *resid_scratch) {
    for (long j = 0; j < D; ++j) grad[j] = 0;
    for (long s = 0; s < B; ++s) {
        int64_t i = rows[s];
        float z = margin_csr(w, col, val, row_ptr[i], row_ptr[i + 1]);
        float sg = (float)(1. / (1. + exp(-(double)z)));
        float r = sg - (float)y[i];
        resid_scratch[s] = r;
        for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) grad[col[k]] = grad[col[k]] + r * val[k];
    }
    for (long j = 0; j < D; ++j)
        grad[j] = (float)(1. * (double)grad[j] / (double)B + (double)((C * w[j]) / (float)B));
}

/* main.cc:41-96  KVStoreDistServer::DataHandle, applied once all W pushes of
 * a step have arrived (pushes arrive in rank order).  grads[r] = rank r's
 * pushed gradient.  mode:
 *   0 "mean"  -- the intended sync merge: merged = ((0+g_0)+g_1)+... in fp32
 *               (main.cc:59-65), w -= fl32(fl32(lr*merged)/(float)W)
 *   1 "last"  -- what main.cc:71 actually does: uses the LAST push only,
 *               w -= fl32(fl32(lr*g_{W-1})/(float)W)
 *   2 "async" -- main.cc:79-84 per push, in rank order: w -= fl32(lr*g_r)
 * With W == 1 all three are identical. */
void orc_server_update(float *w, const float *const *grads, int W, long D, float lr, int mode) {
    for (long i = 0; i < D; ++i) {
        if (mode == 2) {
            for (int r = 0; r < W; ++r) w[i] = w[i] - lr * grads[r][i];
        } else if (mode == 1) {
            w[i] = w[i] - (lr * grads[W - 1][i]) / (float)W;
        } else {
            float merged = 0;
            for (int r = 0; r < W; ++r) merged = merged + grads[r][i];
            w[i] = w[i] - (lr * merged) / (float)W;
        }
    }
}

/* lr.cc:47-63, 100-106  Test: pred = (z > 0) with z the fp32 dense dot
 * product; counts matches.  Also our own logloss (not in the reference):
 * sum of softplus(-z) for y=1 / softplus(z) for y=0, in double. */
static double softplus(double t) { return t > 0 ? t + log1p(exp(-t)) : log1p(exp(t)); }

void orc_predict_dense(const float *X, const int *y, long N, int D, const float *w,
                       int64_t *correct, double *logloss) {
    int64_t c = 0;
    double ll = 0;
    for (long i = 0; i < N; ++i) {
        const float *x = X + (size_t)i * D;
        float z = 0;
        for (int j = 0; j < D; ++j) z = z + w[j] * x[j];
        int pred = z > 0;
        if (pred == y[i]) ++c;
        ll += y[i] ? softplus(-(double)z) : softplus((double)z);
    }
    *correct = c;
    *logloss = ll;
}

void orc_predict_csr(const int64_t *row_ptr, const int32_t *col, const float *val, const int *y,
                     long N, const float *w, int64_t *correct, double *logloss) {
    int64_t c = 0;
    double ll = 0;
    for (long i = 0; i < N; ++i) {
        float z = margin_csr(w, col, val, row_ptr[i], row_ptr[i + 1]);
        int pred = z > 0;
        if (pred == y[i]) ++c;
        ll += y[i] ? softplus(-(double)z) : softplus((double)z);
    }
    *correct = c;
    *logloss = ll;
}

/* lr.cc:50-61  acc is a float counter; printed value is acc / batch.size()
 * in float. */
float orc_accuracy(int64_t correct, long n) {
    float acc = 0;
    for (int64_t i = 0; i < correct; ++i) ++acc;
    return acc / (float)n;
}

/* lr.cc:73-82  SaveModel text: "D\n" then each weight with default ostream
 * formatting (%g, precision 6) followed by ' ', then "\n".  Returns bytes
 * written into out (or needed, if out is too small / NULL). */
long orc_format_model(const float *w, long D, char *out, long cap) {
    long used = 0;
    char tmp[64];
    int n = snprintf(tmp, sizeof tmp, "%ld\n", D);
    if (out && used + n <= cap) memcpy(out + used, tmp, (size_t)n);
    used += n;
    for (long j = 0; j < D; ++j) {
        n = snprintf(tmp, sizeof tmp, "%g ", (double)w[j]);
        if (out && used + n <= cap) memcpy(out + used, tmp, (size_t)n);
        used += n;
    }
    if (out && used + 1 <= cap) out[used] = '\n';
    used += 1;
    return used;
}
