// dlr_host.cpp -- host half of libdistlr_amd: the reference's parsing and
// batching semantics, the model helpers, and the synthetic data generator.
// Nothing here touches a GPU.
//
// Reference semantics followed (file:line in /root/reference):
//   ToInt   src/util.cc:20-36      ToFloat src/util.cc:42-63
//   Split   src/util.cc:6-18       DataIter ctor include/data_iter.h:16-35
//   NextBatch/HasNext include/data_iter.h:40-59
//   InitWeight_ src/lr.cc:92-98    SaveModel src/lr.cc:73-82
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "dlr_internal.h"

namespace dlr {

static thread_local std::string g_error;

void set_error(const std::string &msg) { g_error = msg; }
const char *thread_error() { return g_error.c_str(); }

int default_threads() {
    unsigned hc = std::thread::hardware_concurrency();
    if (hc == 0) hc = 4;
    return (int)std::min(16u, hc);
}

std::vector<BatchSpan> plan_batches(int64_t n_rows, int64_t batch_size) {
    std::vector<BatchSpan> plan;
    if (n_rows <= 0 || batch_size == 0) return plan;
    const int64_t B = batch_size < 0 ? n_rows : batch_size;
    const int64_t nb = (n_rows + B - 1) / B;
    plan.reserve((size_t)nb);
    for (int64_t b = 0; b < nb; ++b) {
        // NextBatch never resets the offset except at the wrap, so batch b
        // starts at (b*B) mod N; it is contiguous unless it reaches row N.
        const int64_t start = (b * B) % n_rows;
        plan.push_back({start, B, start + B <= n_rows});
    }
    return plan;
}

}  // namespace dlr

using dlr::set_error;

// ------------------------------------------------------------------ parsing

extern "C" int dlr_to_int(const char *str) {
    // Optional sign, then ret = ret*10 + (c - '0') for EVERY remaining char
    // (no validation).  Arithmetic wraps like the reference's -O3 build.
    const char *p = str;
    uint32_t sign = 1u;
    if (*p == '-') {
        sign = 0xffffffffu;
        ++p;
    } else if (*p == '+') {
        ++p;
    }
    uint32_t acc = 0;
    for (; *p; ++p) acc = acc * 10u + (uint32_t)(int)(*p - '0');
    return (int)(sign * acc);
}

extern "C" float dlr_to_float(const char *str) {
    // Integer digits accumulate as fl32(i*10 + d); after a '.', digits add
    // fl32(base*d) with base starting at (float)0.1 and stepping by
    // (float)((double)base * 0.1).  '-' and 'e' are just more "digits".
    float ipart = 0.0f, fpart = 0.0f, scale = 1.0f;
    for (const char *p = str; *p; ++p) {
        const char c = *p;
        if (c == '.') {
            scale = (float)0.1;
            continue;
        }
        const float d = (float)(int)(c - '0');
        if ((double)scale >= 1.0) {
            const float t = ipart * 10.0f;
            ipart = t + d;
        } else {
            const float t = scale * d;
            fpart = fpart + t;
            scale = (float)((double)scale * 0.1);
        }
    }
    return ipart + fpart;
}

// Field i of Split(s, sep): the reference takes substr(start, pos) where pos
// is the separator's absolute index, so field i (i < last) spans
// [start_i, start_i + min(pos_i, len - start_i)).
struct FieldRef {
    size_t begin, len;
};
static size_t split_fields(const char *s, size_t len, char sep, FieldRef *out, size_t max_out) {
    size_t n = 0, start = 0;
    for (;;) {
        const void *hit = start <= len ? memchr(s + start, sep, len - start) : nullptr;
        if (!hit) {
            if (n < max_out) out[n] = {start, len - start};
            return n + 1;
        }
        const size_t pos = (size_t)((const char *)hit - s);
        if (n < max_out) out[n] = {start, std::min(pos, len - start)};
        ++n;
        start = pos + 1;
    }
}

extern "C" int dlr_split(const char *line, char separator, char *out, int cap) {
    const size_t len = strlen(line);
    std::vector<FieldRef> f(len + 2);
    const size_t n = split_fields(line, len, separator, f.data(), f.size());
    size_t used = 0;
    for (size_t i = 0; i < n; ++i) {
        if (used + f[i].len + 1 > (size_t)cap) return DLR_E_ARG;
        memcpy(out + used, line + f[i].begin, f[i].len);
        used += f[i].len;
        out[used++] = '\0';
    }
    return (int)n;
}

// ------------------------------------------------------------------ datasets

static inline bool c_space(char c) {  // isspace() in the "C" locale (operator>>)
    return c == ' ' || (c >= '\t' && c <= '\r');
}

namespace {

// One thread's share of a libsvm file: [begin, end) on line boundaries.
struct ChunkOut {
    std::vector<int64_t> row_nnz;
    std::vector<int32_t> col;
    std::vector<float> val;
    std::vector<int32_t> label;
    std::vector<int64_t> unresolved;  // blank rows before the chunk's first token
    std::string last_token;           // last token extracted in the chunk
    bool has_token = false;
    std::string error;
    int64_t error_line = 0;  // 1-based within the chunk
};

void parse_chunk(const char *txt, size_t begin, size_t end, int64_t D, ChunkOut &o) {
    std::vector<std::pair<int32_t, float>> feats;
    std::string tok;
    tok.reserve(64);
    char tmp[128];
    size_t p = begin;
    int64_t line_no = 0;
    while (p < end) {
        size_t e = p;
        while (e < end && txt[e] != '\n') ++e;
        ++line_no;
        size_t q = p;
        bool first = true;
        int32_t label = 0;
        feats.clear();
        for (;;) {
            while (q < e && c_space(txt[q])) ++q;
            if (q >= e) break;
            size_t t = q;
            while (t < e && !c_space(txt[t])) ++t;
            // A token is a NUL-terminated string in the reference (c_str()),
            // so an embedded NUL ends it for ToInt/ToFloat/Split purposes.
            const char *ts = txt + q;
            size_t tl = t - q;
            const void *nul = memchr(ts, '\0', tl);
            size_t cl = nul ? (size_t)((const char *)nul - ts) : tl;
            o.last_token.assign(ts, tl);
            o.has_token = true;
            q = t;
            if (first) {
                first = false;
                const std::string s(ts, cl);
                label = dlr_to_int(s.c_str()) == 1 ? 1 : 0;
                continue;
            }
            FieldRef fr[2];
            const size_t nf = split_fields(ts, cl, ':', fr, 2);
            if (nf < 2) {
                o.error = "token without ':' (reference reads past Split's result)";
                o.error_line = line_no;
                return;
            }
            auto field = [&](const FieldRef &f) -> const char * {
                const size_t n = std::min(f.len, sizeof(tmp) - 1);
                memcpy(tmp, ts + f.begin, n);
                tmp[n] = '\0';
                return tmp;
            };
            const int idx = dlr_to_int(field(fr[0])) - 1;
            if (idx < 0 || (int64_t)idx >= D) {
                o.error = "feature index outside [1, num_feature_dim] (reference writes out of bounds)";
                o.error_line = line_no;
                return;
            }
            const float v = dlr_to_float(field(fr[1]));
            feats.emplace_back(idx, v);
        }
        if (first) {
            // Blank line: operator>> failed and left the previous token in
            // buf, which becomes the label (data_iter.h:26-27).
            if (o.has_token) {
                const std::string &s = o.last_token;
                const size_t cl = strnlen(s.data(), s.size());
                label = dlr_to_int(std::string(s.data(), cl).c_str()) == 1 ? 1 : 0;
            } else {
                o.unresolved.push_back((int64_t)o.label.size());
            }
        }
        // Dense semantics: feature[idx] = v in token order, so the LAST
        // occurrence of an index wins; zeros vanish.
        std::stable_sort(feats.begin(), feats.end(),
                         [](const std::pair<int32_t, float> &a, const std::pair<int32_t, float> &b) {
                             return a.first < b.first;
                         });
        int64_t kept = 0;
        for (size_t i = 0; i < feats.size(); ++i) {
            if (i + 1 < feats.size() && feats[i + 1].first == feats[i].first) continue;
            if (feats[i].second == 0.0f) continue;
            o.col.push_back(feats[i].first);
            o.val.push_back(feats[i].second);
            ++kept;
        }
        o.row_nnz.push_back(kept);
        o.label.push_back(label);
        p = (e < end) ? e + 1 : e;
    }
}

}  // namespace

extern "C" int dlr_dataset_load_libsvm(const char *path, int64_t num_feature_dim, int nthreads, dlr_dataset **out) {
    if (!path || !out || num_feature_dim <= 0) {
        set_error("dlr_dataset_load_libsvm: bad argument");
        return DLR_E_ARG;
    }
    *out = nullptr;
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        set_error(std::string("cannot open ") + path);
        return DLR_E_IO;
    }
    std::string txt((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const size_t len = txt.size();
    if (nthreads <= 0) nthreads = dlr::default_threads();
    int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nthreads, len / (1 << 20) + 1));
    std::vector<size_t> cuts(nt + 1, len);
    cuts[0] = 0;
    for (int i = 1; i < nt; ++i) {
        size_t c = std::max(cuts[i - 1], len * i / nt);
        while (c < len && txt[c - 1] != '\n') ++c;
        cuts[i] = c;
    }
    std::vector<ChunkOut> parts(nt);
    {
        std::vector<std::thread> th;
        for (int i = 0; i < nt; ++i)
            th.emplace_back([&, i] { parse_chunk(txt.data(), cuts[i], cuts[i + 1], num_feature_dim, parts[i]); });
        for (auto &t : th) t.join();
    }
    int64_t lines_before = 0;
    for (int i = 0; i < nt; ++i) {
        if (!parts[i].error.empty()) {
            set_error(std::string(path) + ":" + std::to_string(lines_before + parts[i].error_line) + ": " +
                      parts[i].error);
            return DLR_E_PARSE;
        }
        lines_before += (int64_t)parts[i].label.size();
    }
    // Resolve blank rows that precede a chunk's first token with the token
    // carried over from earlier chunks ("" before the first token: label 0).
    std::string carry;
    for (int i = 0; i < nt; ++i) {
        const int32_t lab = dlr_to_int(std::string(carry.c_str()).c_str()) == 1 ? 1 : 0;
        for (int64_t r : parts[i].unresolved) parts[i].label[(size_t)r] = lab;
        if (parts[i].has_token) carry = parts[i].last_token;
    }
    auto ds = std::make_unique<dlr_dataset>();
    ds->D = num_feature_dim;
    int64_t rows = 0, nnz = 0;
    for (auto &p : parts) {
        rows += (int64_t)p.label.size();
        nnz += (int64_t)p.col.size();
    }
    ds->n_rows = rows;
    ds->row_ptr.resize((size_t)rows + 1);
    ds->col.reserve((size_t)nnz);
    ds->val.reserve((size_t)nnz);
    ds->label.reserve((size_t)rows);
    int64_t r = 0, k = 0;
    ds->row_ptr[0] = 0;
    for (auto &p : parts) {
        for (int64_t c : p.row_nnz) {
            k += c;
            ds->row_ptr[(size_t)++r] = k;
        }
        ds->col.insert(ds->col.end(), p.col.begin(), p.col.end());
        ds->val.insert(ds->val.end(), p.val.begin(), p.val.end());
        ds->label.insert(ds->label.end(), p.label.begin(), p.label.end());
    }
    *out = ds.release();
    return DLR_OK;
}

extern "C" int dlr_dataset_from_csr(int64_t n_rows, int64_t num_feature_dim, const int64_t *row_ptr,
                                    const int32_t *col, const float *val, const int32_t *label,
                                    dlr_dataset **out) {
    if (!out || n_rows < 0 || num_feature_dim <= 0 || !row_ptr || (n_rows > 0 && !label)) {
        set_error("dlr_dataset_from_csr: bad argument");
        return DLR_E_ARG;
    }
    *out = nullptr;
    const int64_t nnz = row_ptr[n_rows] - row_ptr[0];
    if (row_ptr[0] != 0 || nnz < 0 || (nnz > 0 && (!col || !val))) {
        set_error("dlr_dataset_from_csr: row_ptr must start at 0 and be non-decreasing");
        return DLR_E_ARG;
    }
    for (int64_t i = 0; i < n_rows; ++i) {
        if (row_ptr[i + 1] < row_ptr[i]) {
            set_error("dlr_dataset_from_csr: row_ptr not non-decreasing");
            return DLR_E_ARG;
        }
        for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
            if (col[k] < 0 || col[k] >= num_feature_dim || (k > row_ptr[i] && col[k] <= col[k - 1])) {
                set_error("dlr_dataset_from_csr: columns must be ascending, distinct and in [0, D)");
                return DLR_E_ARG;
            }
        }
        if (label[i] != 0 && label[i] != 1) {
            set_error("dlr_dataset_from_csr: labels must be 0/1");
            return DLR_E_ARG;
        }
    }
    auto ds = std::make_unique<dlr_dataset>();
    ds->n_rows = n_rows;
    ds->D = num_feature_dim;
    ds->row_ptr.assign(row_ptr, row_ptr + n_rows + 1);
    if (nnz > 0) {
        ds->col.assign(col, col + nnz);
        ds->val.assign(val, val + nnz);
    }
    if (n_rows > 0) ds->label.assign(label, label + n_rows);
    *out = ds.release();
    return DLR_OK;
}

extern "C" int dlr_dataset_info(const dlr_dataset *ds, int64_t *n_rows, int64_t *nnz, int64_t *D) {
    if (!ds) return DLR_E_ARG;
    if (n_rows) *n_rows = ds->n_rows;
    if (nnz) *nnz = (int64_t)ds->col.size();
    if (D) *D = ds->D;
    return DLR_OK;
}

extern "C" int dlr_dataset_view(const dlr_dataset *ds, const int64_t **row_ptr, const int32_t **col,
                                const float **val, const int32_t **label) {
    if (!ds) return DLR_E_ARG;
    if (row_ptr) *row_ptr = ds->row_ptr.data();
    if (col) *col = ds->col.data();
    if (val) *val = ds->val.data();
    if (label) *label = ds->label.data();
    return DLR_OK;
}

extern "C" void dlr_dataset_free(dlr_dataset *ds) { delete ds; }

// ------------------------------------------------------------------ dense

extern "C" int dlr_dense_from_dataset(const dlr_dataset *ds, dlr_dense **out) {
    if (!ds || !out) {
        set_error("dlr_dense_from_dataset: bad argument");
        return DLR_E_ARG;
    }
    *out = nullptr;
    auto d = std::make_unique<dlr_dense>();
    d->n_rows = ds->n_rows;
    d->D = ds->D;
    try {
        d->X.assign((size_t)(ds->n_rows * ds->D), 0.0f);
    } catch (...) {
        set_error("dlr_dense_from_dataset: out of host memory");
        return DLR_E_NOMEM;
    }
    for (int64_t i = 0; i < ds->n_rows; ++i)
        for (int64_t k = ds->row_ptr[(size_t)i]; k < ds->row_ptr[(size_t)i + 1]; ++k)
            d->X[(size_t)(i * ds->D + ds->col[(size_t)k])] = ds->val[(size_t)k];
    d->label = ds->label;
    *out = d.release();
    return DLR_OK;
}

extern "C" int dlr_dense_from_array(int64_t n_rows, int64_t num_feature_dim, const float *X, const int32_t *label,
                                    dlr_dense **out) {
    if (!out || n_rows < 0 || num_feature_dim <= 0 || (n_rows > 0 && (!X || !label))) {
        set_error("dlr_dense_from_array: bad argument");
        return DLR_E_ARG;
    }
    *out = nullptr;
    for (int64_t i = 0; i < n_rows; ++i)
        if (label[i] != 0 && label[i] != 1) {
            set_error("dlr_dense_from_array: labels must be 0/1");
            return DLR_E_ARG;
        }
    auto d = std::make_unique<dlr_dense>();
    d->n_rows = n_rows;
    d->D = num_feature_dim;
    try {
        d->X.assign(X, X + n_rows * num_feature_dim);
        d->label.assign(label, label + n_rows);
    } catch (...) {
        set_error("dlr_dense_from_array: out of host memory");
        return DLR_E_NOMEM;
    }
    *out = d.release();
    return DLR_OK;
}

extern "C" int dlr_dense_info(const dlr_dense *ds, int64_t *n_rows, int64_t *D) {
    if (!ds) return DLR_E_ARG;
    if (n_rows) *n_rows = ds->n_rows;
    if (D) *D = ds->D;
    return DLR_OK;
}

extern "C" int dlr_dense_view(const dlr_dense *ds, const float **X, const int32_t **label) {
    if (!ds) return DLR_E_ARG;
    if (X) *X = ds->X.data();
    if (label) *label = ds->label.data();
    return DLR_OK;
}

extern "C" void dlr_dense_free(dlr_dense *ds) { delete ds; }

extern "C" int dlr_dataset_write_libsvm(const dlr_dataset *ds, const char *path, int value_mode) {
    if (!ds || !path) return DLR_E_ARG;
    FILE *f = fopen(path, "wb");
    if (!f) {
        set_error(std::string("cannot write ") + path);
        return DLR_E_IO;
    }
    std::vector<char> buf(1 << 20);
    setvbuf(f, buf.data(), _IOFBF, buf.size());
    for (int64_t i = 0; i < ds->n_rows; ++i) {
        fputs(ds->label[(size_t)i] ? "+1" : "-1", f);
        for (int64_t k = ds->row_ptr[(size_t)i]; k < ds->row_ptr[(size_t)i + 1]; ++k) {
            if (value_mode == 0)
                fprintf(f, " %d:1", ds->col[(size_t)k] + 1);
            else
                fprintf(f, " %d:%.4f", ds->col[(size_t)k] + 1, (double)ds->val[(size_t)k]);
        }
        fputc('\n', f);
    }
    const bool ok = fclose(f) == 0;
    return ok ? DLR_OK : DLR_E_IO;
}

// ------------------------------------------------------------ binary CSR cache
// A parsed shard saved as its four CSR arrays (SURVEY 8(f) ingest: C2's
// 500M-entry text parse is paid once).  Layout, little-endian:
//   "DLRCSR" 0 1 | n_rows D nnz (int64) | checksum (uint64) |
//   row_ptr[n_rows+1] (int64) | col[nnz] (int32) | val[nnz] (fp32) | label[n_rows] (int32)
// The checksum mixes every 8-byte word of the arrays; a load verifies it and
// the CSR invariants before handing the shard out.

namespace {

constexpr char kBinMagic[8] = {'D', 'L', 'R', 'C', 'S', 'R', 0, 1};

uint64_t mix_words(uint64_t h, const void *p, size_t bytes) {
    const unsigned char *b = static_cast<const unsigned char *>(p);
    size_t i = 0;
    for (; i + 8 <= bytes; i += 8) {
        uint64_t w;
        memcpy(&w, b + i, 8);
        h = (h ^ w) * 0x100000001B3ull;
        h ^= h >> 29;
    }
    uint64_t w = 0;
    memcpy(&w, b + i, bytes - i);
    return ((h ^ w ^ (uint64_t)bytes) * 0x100000001B3ull) ^ (h >> 31);
}

uint64_t csr_checksum(const dlr_dataset &d) {
    uint64_t h = 0xCBF29CE484222325ull;
    h = mix_words(h, d.row_ptr.data(), d.row_ptr.size() * 8);
    h = mix_words(h, d.col.data(), d.col.size() * 4);
    h = mix_words(h, d.val.data(), d.val.size() * 4);
    return mix_words(h, d.label.data(), d.label.size() * 4);
}

}  // namespace

extern "C" int dlr_dataset_save_binary(const dlr_dataset *ds, const char *path) {
    if (!ds || !path) {
        set_error("dlr_dataset_save_binary: bad argument");
        return DLR_E_ARG;
    }
    FILE *f = fopen(path, "wb");
    if (!f) {
        set_error(std::string("dlr_dataset_save_binary: cannot write ") + path);
        return DLR_E_IO;
    }
    const int64_t hdr[3] = {ds->n_rows, ds->D, (int64_t)ds->col.size()};
    const uint64_t sum = csr_checksum(*ds);
    bool ok = fwrite(kBinMagic, 1, 8, f) == 8 && fwrite(hdr, 8, 3, f) == 3 && fwrite(&sum, 8, 1, f) == 1;
    ok = ok && fwrite(ds->row_ptr.data(), 8, ds->row_ptr.size(), f) == ds->row_ptr.size();
    ok = ok && fwrite(ds->col.data(), 4, ds->col.size(), f) == ds->col.size();
    ok = ok && fwrite(ds->val.data(), 4, ds->val.size(), f) == ds->val.size();
    ok = ok && fwrite(ds->label.data(), 4, ds->label.size(), f) == ds->label.size();
    ok = (fclose(f) == 0) && ok;
    if (!ok) {
        set_error(std::string("dlr_dataset_save_binary: write failed: ") + path);
        return DLR_E_IO;
    }
    return DLR_OK;
}

extern "C" int dlr_dataset_load_binary(const char *path, dlr_dataset **out) {
    if (!path || !out) {
        set_error("dlr_dataset_load_binary: bad argument");
        return DLR_E_ARG;
    }
    *out = nullptr;
    FILE *f = fopen(path, "rb");
    if (!f) {
        set_error(std::string("dlr_dataset_load_binary: cannot open ") + path);
        return DLR_E_IO;
    }
    auto bad = [&](const std::string &why) {
        fclose(f);
        set_error("dlr_dataset_load_binary: " + std::string(path) + ": " + why);
        return DLR_E_PARSE;
    };
    char magic[8];
    int64_t hdr[3];
    uint64_t sum = 0;
    if (fread(magic, 1, 8, f) != 8 || memcmp(magic, kBinMagic, 8) != 0) return bad("not a DLRCSR v1 file");
    if (fread(hdr, 8, 3, f) != 3 || fread(&sum, 8, 1, f) != 1) return bad("truncated header");
    const int64_t n = hdr[0], D = hdr[1], nnz = hdr[2];
    if (n < 0 || D <= 0 || D > INT32_MAX || nnz < 0) return bad("bad header");
    if (fseeko(f, 0, SEEK_END) != 0) return bad("cannot size the file");
    const int64_t expect = 40 + 8 * (n + 1) + 8 * nnz + 4 * n;
    if ((int64_t)ftello(f) != expect) return bad("size does not match the header");
    fseeko(f, 40, SEEK_SET);
    auto ds = std::make_unique<dlr_dataset>();
    ds->n_rows = n;
    ds->D = D;
    try {
        ds->row_ptr.resize((size_t)n + 1);
        ds->col.resize((size_t)nnz);
        ds->val.resize((size_t)nnz);
        ds->label.resize((size_t)n);
    } catch (const std::bad_alloc &) {
        fclose(f);
        set_error("dlr_dataset_load_binary: out of host memory");
        return DLR_E_NOMEM;
    }
    bool ok = fread(ds->row_ptr.data(), 8, ds->row_ptr.size(), f) == ds->row_ptr.size();
    ok = ok && fread(ds->col.data(), 4, ds->col.size(), f) == ds->col.size();
    ok = ok && fread(ds->val.data(), 4, ds->val.size(), f) == ds->val.size();
    ok = ok && fread(ds->label.data(), 4, ds->label.size(), f) == ds->label.size();
    if (!ok) return bad("short read");
    fclose(f);
    if (csr_checksum(*ds) != sum) {
        set_error(std::string("dlr_dataset_load_binary: ") + path + ": checksum mismatch");
        return DLR_E_PARSE;
    }
    if (ds->row_ptr[0] != 0 || ds->row_ptr[(size_t)n] != nnz) {
        set_error(std::string("dlr_dataset_load_binary: ") + path + ": row offsets do not span the entries");
        return DLR_E_PARSE;
    }
    for (int64_t i = 0; i < n; ++i) {
        const int64_t a = ds->row_ptr[(size_t)i], b = ds->row_ptr[(size_t)i + 1];
        bool rowok = a <= b && (ds->label[(size_t)i] == 0 || ds->label[(size_t)i] == 1);
        for (int64_t k = a; rowok && k < b; ++k)
            rowok = ds->col[(size_t)k] >= 0 && ds->col[(size_t)k] < D && (k == a || ds->col[(size_t)k] > ds->col[(size_t)k - 1]);
        if (!rowok) {
            set_error(std::string("dlr_dataset_load_binary: ") + path + ": invalid row " + std::to_string(i));
            return DLR_E_PARSE;
        }
    }
    *out = ds.release();
    return DLR_OK;
}

// ------------------------------------------------------------------ batching

extern "C" int64_t dlr_num_batches(int64_t n_rows, int64_t batch_size) {
    if (batch_size == 0) return DLR_E_ARG;  // the reference would loop forever
    if (n_rows <= 0) return 0;              // reference: Train never terminates
    const int64_t B = batch_size < 0 ? n_rows : batch_size;
    return (n_rows + B - 1) / B;
}

extern "C" int dlr_batch_rows(int64_t n_rows, int64_t batch_size, int64_t batch, int64_t *rows_out) {
    const int64_t nb = dlr_num_batches(n_rows, batch_size);
    if (nb <= 0 || batch < 0 || batch >= nb || !rows_out) return DLR_E_ARG;
    const int64_t B = batch_size < 0 ? n_rows : batch_size;
    int64_t off = (batch * B) % n_rows;
    for (int64_t i = 0; i < B; ++i) {
        rows_out[i] = off;
        if (++off == n_rows) off = 0;
    }
    return DLR_OK;
}

// ------------------------------------------------------------------ model helpers

namespace {
// glibc rand() = random() with the default TYPE_3 state: a degree-31
// additive lagged-Fibonacci generator (taps 31/3) seeded by the 16807 LCG,
// 310 outputs discarded, outputs >> 1.
class GlibcRand {
   public:
    explicit GlibcRand(unsigned seed) {
        int32_t *s = st_;
        s[0] = (int32_t)(seed == 0 ? 1u : seed);
        long word = s[0];
        for (int i = 1; i < 31; ++i) {
            const long hi = word / 127773, lo = word % 127773;
            word = 16807 * lo - 2836 * hi;
            if (word < 0) word += 2147483647;
            s[i] = (int32_t)word;
        }
        f_ = 3;
        r_ = 0;
        for (int i = 0; i < 310; ++i) next();
    }
    int32_t next() {
        const uint32_t v = (uint32_t)st_[f_] + (uint32_t)st_[r_];
        st_[f_] = (int32_t)v;
        f_ = (f_ + 1) % 31;
        r_ = (r_ + 1) % 31;
        return (int32_t)(v >> 1);
    }

   private:
    int32_t st_[31];
    int f_, r_;
};
}  // namespace

extern "C" int dlr_init_weight(int random_state, float *w, int64_t D) {
    if (!w || D < 0) return DLR_E_ARG;
    GlibcRand g((unsigned)random_state);
    const float rmax = (float)2147483647;  // RAND_MAX as float
    for (int64_t j = 0; j < D; ++j) w[j] = (float)g.next() / rmax;
    return DLR_OK;
}

extern "C" int dlr_format_model(const float *w, int64_t D, char *out, int64_t cap, int64_t *needed) {
    if ((!w && D > 0) || D < 0) return DLR_E_ARG;
    // libstdc++ writes a float through "%.*g" with the stream precision (6).
    std::string s = std::to_string(D) + "\n";
    char tmp[64];
    for (int64_t j = 0; j < D; ++j) {
        const int n = snprintf(tmp, sizeof tmp, "%.*g ", 6, (double)w[j]);
        s.append(tmp, (size_t)n);
    }
    s.push_back('\n');
    if (needed) *needed = (int64_t)s.size();
    if (out && cap > 0) {
        const size_t n = std::min((size_t)cap, s.size());
        memcpy(out, s.data(), n);
        if (n < (size_t)cap) out[n] = '\0';
    }
    return DLR_OK;
}

extern "C" int dlr_key_range(int64_t D, int world, int rank, int64_t *begin, int64_t *end) {
    if (D < 0 || world <= 0 || rank < 0 || rank >= world || !begin || !end) return DLR_E_ARG;
    const int64_t chunk = (D + world - 1) / world;
    *begin = std::min(D, (int64_t)rank * chunk);
    *end = std::min(D, (int64_t)(rank + 1) * chunk);
    return DLR_OK;
}

// ------------------------------------------------------------------ generator

namespace {

inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() { return mix64(s += 0x632BE59BD9B4E019ull); }
    uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
    double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
    double gauss() {
        double u1 = unit(), u2 = unit();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

double normal_quantile(double p) {  // inverse of Phi by bisection on erfc
    double lo = -12, hi = 12;
    for (int i = 0; i < 200; ++i) {
        const double m = 0.5 * (lo + hi);
        if (0.5 * std::erfc(-m / std::sqrt(2.0)) < p)
            lo = m;
        else
            hi = m;
    }
    return 0.5 * (lo + hi);
}

// k distinct uniform columns of [0, D), ascending.
void draw_columns(Rng &g, int64_t D, int k, std::vector<int32_t> &cols) {
    cols.clear();
    if ((int64_t)k * 2 >= D) {  // selection sampling (Knuth S)
        int64_t need = k;
        for (int64_t j = 0; j < D && need > 0; ++j)
            if ((int64_t)g.below((uint64_t)(D - j)) < need) {
                cols.push_back((int32_t)j);
                --need;
            }
        return;
    }
    while ((int)cols.size() < k) {
        while ((int)cols.size() < k) cols.push_back((int32_t)g.below((uint64_t)D));
        std::sort(cols.begin(), cols.end());
        cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
    }
}

}  // namespace

// Planted model w*_j ~ N(0,1), one generator per column (so it is the same
// for every stream and thread count).
std::vector<float> planted_model(uint64_t seed, int64_t D, int nthreads) {
    std::vector<float> wstar((size_t)D);
    int nt = nthreads > 0 ? nthreads : dlr::default_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, D / 65536 + 1));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int64_t j = D * t / nt; j < D * (t + 1) / nt; ++j) {
                Rng g(mix64(seed * 0x9E3779B97F4A7C15ull ^ (uint64_t)j) ^ 0xA5A5A5A5ull);
                wstar[(size_t)j] = (float)g.gauss();
            }
        });
    for (auto &x : th) x.join();
    return wstar;
}

extern "C" int dlr_dataset_generate(const dlr_gen_spec *spec, dlr_dataset **out) {
    if (!spec || !out || spec->n_rows < 0 || spec->num_feature_dim <= 0 || spec->nnz_per_row < 0 ||
        spec->num_feature_dim > INT32_MAX) {
        set_error("dlr_dataset_generate: bad spec");
        return DLR_E_ARG;
    }
    *out = nullptr;
    const int64_t N = spec->n_rows, D = spec->num_feature_dim;
    const int k = (int)std::min<int64_t>(spec->nnz_per_row, D);
    auto ds = std::make_unique<dlr_dataset>();
    ds->n_rows = N;
    ds->D = D;
    try {
        ds->row_ptr.resize((size_t)N + 1);
        ds->col.resize((size_t)(N * k));
        ds->val.resize((size_t)(N * k));
        ds->label.resize((size_t)N);
    } catch (...) {
        set_error("dlr_dataset_generate: out of host memory");
        return DLR_E_NOMEM;
    }
    for (int64_t i = 0; i <= N; ++i) ds->row_ptr[(size_t)i] = i * k;
    // Planted model w* ~ N(0,1) per column (shared by every stream of a seed).
    std::vector<float> wstar = planted_model(spec->seed, D, spec->nthreads);
    // Four-decimal values q/10000, q in [1, 10000], as ToFloat of the text.
    std::vector<float> lut(10001);
    for (int q = 1; q <= 10000; ++q) {
        char t[16];
        if (q == 10000)
            snprintf(t, sizeof t, "1.0000");
        else
            snprintf(t, sizeof t, "0.%04d", q);
        lut[(size_t)q] = dlr_to_float(t);
    }
    const double thr = normal_quantile(1.0 - std::min(std::max(spec->positive_frac, 1e-6), 1.0 - 1e-6));
    const uint64_t stream_key = mix64(spec->seed ^ mix64(0x5EEDull + spec->stream));
    int nt = spec->nthreads > 0 ? spec->nthreads : dlr::default_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, N / 4096 + 1));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
        th.emplace_back([&, t] {
            std::vector<int32_t> cols;
            const int64_t r0 = N * t / nt, r1 = N * (t + 1) / nt;
            for (int64_t i = r0; i < r1; ++i) {
                Rng g(mix64(stream_key ^ (uint64_t)i * 0xD1342543DE82EF95ull));
                draw_columns(g, D, k, cols);
                double m = 0, nrm = 0;
                for (int e = 0; e < k; ++e) {
                    const float v = spec->value_mode == 0 ? 1.0f : lut[(size_t)(1 + g.below(10000))];
                    ds->col[(size_t)(i * k + e)] = cols[(size_t)e];
                    ds->val[(size_t)(i * k + e)] = v;
                    m += (double)wstar[(size_t)cols[(size_t)e]] * v;
                    nrm += (double)v * v;
                }
                bool pos = nrm > 0 ? (m / std::sqrt(nrm)) > thr : g.unit() < spec->positive_frac;
                if (g.unit() < spec->label_noise) pos = !pos;
                ds->label[(size_t)i] = pos ? 1 : 0;
            }
        });
    }
    for (auto &x : th) x.join();
    *out = ds.release();
    return DLR_OK;
}

// Criteo-shaped hashed rows (BASELINE.json configs[2]):
// each of `fields` categorical fields draws a value v ~ Zipf(s) over
// [1, cardinality] (inverse CDF); the feature is splitmix64(field, v) mod D;
// duplicates within a row collapse; columns ascending; value 1.  Labels come
// from a planted model as in dlr_dataset_generate.
extern "C" int dlr_dataset_generate_hashed(const dlr_hashed_spec *spec, dlr_dataset **out) {
    if (!spec || !out || spec->n_rows < 0 || spec->num_feature_dim <= 0 || spec->num_feature_dim > INT32_MAX ||
        spec->fields <= 0 || spec->fields > 1024 || spec->cardinality <= 0 || spec->zipf_s <= 0.0) {
        set_error("dlr_dataset_generate_hashed: bad spec");
        return DLR_E_ARG;
    }
    *out = nullptr;
    const int64_t N = spec->n_rows, D = spec->num_feature_dim;
    const int F = spec->fields;
    auto ds = std::make_unique<dlr_dataset>();
    ds->n_rows = N;
    ds->D = D;
    // Zipf(s) CDF over [1, cardinality]
    std::vector<double> cdf((size_t)spec->cardinality);
    double acc = 0.0;
    for (int64_t v = 1; v <= spec->cardinality; ++v) {
        acc += std::pow((double)v, -spec->zipf_s);
        cdf[(size_t)v - 1] = acc;
    }
    for (double &c : cdf) c /= acc;
    std::vector<float> wstar = planted_model(spec->seed, D, spec->nthreads);
    const double thr = normal_quantile(1.0 - std::min(std::max(spec->positive_frac, 1e-6), 1.0 - 1e-6));
    const uint64_t stream_key = mix64(spec->seed ^ mix64(0xC4173ull + spec->stream));
    int nt = spec->nthreads > 0 ? spec->nthreads : dlr::default_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, N / 4096 + 1));
    // rows are generated per thread block, then concatenated
    std::vector<std::vector<int32_t>> tcol((size_t)nt);
    std::vector<std::vector<int64_t>> tlen((size_t)nt);
    try {
        ds->label.resize((size_t)N);
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) {
            th.emplace_back([&, t] {
                const int64_t r0 = N * t / nt, r1 = N * (t + 1) / nt;
                std::vector<int32_t> &cc = tcol[(size_t)t];
                std::vector<int64_t> &ll = tlen[(size_t)t];
                cc.reserve((size_t)((r1 - r0) * F));
                ll.reserve((size_t)(r1 - r0));
                std::vector<int32_t> row;
                for (int64_t i = r0; i < r1; ++i) {
                    Rng g(mix64(stream_key ^ (uint64_t)i * 0xD1342543DE82EF95ull));
                    row.clear();
                    for (int f = 0; f < F; ++f) {
                        const double u = g.unit();
                        const int64_t v = 1 + (int64_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
                        const uint64_t h = mix64(((uint64_t)f << 40) ^ (uint64_t)v ^ 0x51ED2701ull);
                        row.push_back((int32_t)(h % (uint64_t)D));
                    }
                    std::sort(row.begin(), row.end());
                    row.erase(std::unique(row.begin(), row.end()), row.end());
                    double m = 0;
                    for (int32_t c : row) m += (double)wstar[(size_t)c];
                    bool pos = !row.empty() ? (m / std::sqrt((double)row.size())) > thr : g.unit() < spec->positive_frac;
                    if (g.unit() < spec->label_noise) pos = !pos;
                    ds->label[(size_t)i] = pos ? 1 : 0;
                    cc.insert(cc.end(), row.begin(), row.end());
                    ll.push_back((int64_t)row.size());
                }
            });
        }
        for (auto &x : th) x.join();
        int64_t total = 0;
        for (auto &v : tcol) total += (int64_t)v.size();
        ds->row_ptr.resize((size_t)N + 1);
        ds->col.resize((size_t)total);
        ds->val.assign((size_t)total, 1.0f);
        int64_t at = 0, i = 0;
        ds->row_ptr[0] = 0;
        for (int t = 0; t < nt; ++t) {
            std::copy(tcol[(size_t)t].begin(), tcol[(size_t)t].end(), ds->col.begin() + at);
            at += (int64_t)tcol[(size_t)t].size();
            std::vector<int32_t>().swap(tcol[(size_t)t]);
            for (int64_t len : tlen[(size_t)t]) {
                ds->row_ptr[(size_t)i + 1] = ds->row_ptr[(size_t)i] + len;
                ++i;
            }
        }
    } catch (...) {
        set_error("dlr_dataset_generate_hashed: out of host memory");
        return DLR_E_NOMEM;
    }
    *out = ds.release();
    return DLR_OK;
}

// Dense rows for C4 (4,096 features x 20M samples fp32): every feature a
// 4-decimal value in (0,1] held as ToFloat of its text; planted labels.
extern "C" int dlr_dense_generate(const dlr_dense_spec *spec, dlr_dense **out) {
    if (!spec || !out || spec->n_rows < 0 || spec->num_feature_dim <= 0) {
        set_error("dlr_dense_generate: bad spec");
        return DLR_E_ARG;
    }
    *out = nullptr;
    const int64_t N = spec->n_rows, D = spec->num_feature_dim;
    auto d = std::make_unique<dlr_dense>();
    d->n_rows = N;
    d->D = D;
    try {
        d->X.resize((size_t)(N * D));
        d->label.resize((size_t)N);
    } catch (...) {
        set_error("dlr_dense_generate: out of host memory");
        return DLR_E_NOMEM;
    }
    std::vector<float> wstar = planted_model(spec->seed, D, spec->nthreads);
    std::vector<float> lut(10001);
    for (int q = 1; q <= 10000; ++q) {
        char t[16];
        if (q == 10000)
            snprintf(t, sizeof t, "1.0000");
        else
            snprintf(t, sizeof t, "0.%04d", q);
        lut[(size_t)q] = dlr_to_float(t);
    }
    // centre the planted margin: E[x] = 0.50005 per feature
    const double thr = normal_quantile(1.0 - std::min(std::max(spec->positive_frac, 1e-6), 1.0 - 1e-6));
    const uint64_t stream_key = mix64(spec->seed ^ mix64(0xDE45Eull + spec->stream));
    int nt = spec->nthreads > 0 ? spec->nthreads : dlr::default_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, N / 256 + 1));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int64_t i = N * t / nt; i < N * (t + 1) / nt; ++i) {
                Rng g(mix64(stream_key ^ (uint64_t)i * 0xD1342543DE82EF95ull));
                float *x = d->X.data() + (size_t)(i * D);
                double m = 0;
                for (int64_t j = 0; j < D; ++j) {
                    const uint64_t q = 1 + g.below(10000);
                    x[j] = lut[(size_t)q];
                    m += (double)wstar[(size_t)j] * ((double)q * 1e-4 - 0.50005);
                }
                bool pos = (m / std::sqrt((double)D / 12.0)) > thr;
                if (g.unit() < spec->label_noise) pos = !pos;
                d->label[(size_t)i] = pos ? 1 : 0;
            }
        });
    for (auto &x : th) x.join();
    *out = d.release();
    return DLR_OK;
}

