// ref_loop.cc -- CPU BASELINE / TEST INFRASTRUCTURE ONLY (never the
// product).  Loaded by bench.py's cpu_baseline leg and by tests/.
//
// The reference's CPU path with its own COST STRUCTURE, restated: local.sh's
// topology (W worker threads + one in-process server) running
// RunWorker (src/main.cc:124-170) for every rank:
//   * every epoch re-parses the rank's libsvm part file into DENSE samples
//     (main.cc:158-159 -> data_iter.h:16-35: getline, istringstream tokens,
//     Split(':'), ToInt/ToFloat, a D-float vector per line);
//   * NextBatch copies B samples (data_iter.h:40-55);
//   * LR::Train (lr.cc:28-45): Pull (copy of the D weights), then for every
//     column j and every sample s: Sigmoid_(s.GetFeature()) -- the feature
//     vector copied by value twice (sample.h:37-39, lr.cc:108) and the
//     O(D) margin recomputed -- so O(B * D^2) per batch; then lr.cc:40's
//     normalisation and L2; Push (copy of D gradients) and wait for the
//     server (main.cc:57-84: sync waits for all W pushes);
//   * rank 0 tests every TEST_INTERVAL epochs on test/part-001 (lr.cc:47-63).
// Arithmetic is the oracle's (lr_oracle.c, same operation order): the
// result is bitwise the oracle's W-worker run (tests/test_ref_loop.py), so
// this baseline does the reference's work and gets the reference's bits.
// Server rule: the oracle's modes (0 mean, 1 last push, 2 async; pushes
// merged in rank order).
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int orc_to_int(const char *str);
float orc_to_float(const char *str);
int orc_split(const char *line, char sep, char *out, int cap);
void orc_init_weight(int random_state, float *w, long D);
void orc_server_update(float *w, const float *const *grads, int W, long D, float lr, int mode);
}

namespace {

struct DenseSample {
    std::vector<float> feature;  // D floats (sample.h: feature_)
    int label;
    std::vector<float> features_by_value() const { return feature; }  // sample.h:37-39 GetFeature()
};

// data_iter.h:16-35: one dense sample per line.
std::vector<DenseSample> parse_part(const std::string &path, int D) {
    std::vector<DenseSample> out;
    std::ifstream input(path.c_str());
    std::string line, tok;
    std::vector<char> fields(8192);
    while (std::getline(input, line)) {
        std::istringstream in(line);
        in >> tok;  // a blank line keeps the previous token (operator>> fails)
        DenseSample s;
        s.label = orc_to_int(tok.c_str()) == 1 ? 1 : 0;
        s.feature.assign((size_t)D, 0.0f);
        while (in >> tok) {
            if (orc_split(tok.c_str(), ':', fields.data(), (int)fields.size()) < 2) continue;
            const char *f0 = fields.data();
            const char *f1 = f0 + strlen(f0) + 1;
            const int idx = orc_to_int(f0) - 1;
            if (idx >= 0 && idx < D) s.feature[(size_t)idx] = orc_to_float(f1);
        }
        out.push_back(s);
    }
    return out;
}

struct Iter {  // data_iter.h:40-59
    std::vector<DenseSample> samples;
    size_t offset = 0;
    bool round_end = false;
    std::vector<DenseSample> next_batch(long B) {
        if (B < 0) B = (long)samples.size();
        std::vector<DenseSample> batch;
        for (long i = 0; i < B; ++i) {
            batch.push_back(samples[offset]);
            if (++offset == samples.size()) {
                offset = 0;
                round_end = true;
            }
        }
        return batch;
    }
};

// The in-process server (main.cc:41-96, the stand-in for ps-lite's KV
// server): pushes of a step are merged in rank order once all W arrived.
struct Server {
    std::mutex mu;
    std::condition_variable cv;
    int W, mode;
    float lr;
    std::vector<float> w;
    std::vector<std::vector<float>> pushes;
    int arrived = 0;
    uint64_t gen = 0;
    Server(int W_, int D, float lr_, int mode_) : W(W_), mode(mode_), lr(lr_), pushes((size_t)W_) {
        w.assign((size_t)D, 0.0f);
    }
    void pull(std::vector<float> &out) {
        std::lock_guard<std::mutex> g(mu);
        out = w;
    }
    void push(int rank, const std::vector<float> &grad) {
        std::unique_lock<std::mutex> lk(mu);
        pushes[(size_t)rank] = grad;
        const uint64_t my = gen;
        if (++arrived == W) {
            std::vector<const float *> gp((size_t)W);
            for (int r = 0; r < W; ++r) gp[(size_t)r] = pushes[(size_t)r].data();
            orc_server_update(w.data(), gp.data(), W, (long)w.size(), lr, mode);
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != my; });
        }
    }
};

// lr.cc:108-114, argument by value as in the reference.
float sigmoid_by_value(const std::vector<float> &w, std::vector<float> feature) {
    float z = 0;
    for (size_t j = 0; j < w.size(); ++j) z = z + w[j] * feature[j];
    return (float)(1. / (1. + std::exp(-(double)z)));
}

struct Job {
    std::string root;
    int W, D, num_iteration, batch, test_interval, mode;
    float lr, C = 1.0f;
    Server *server;
    std::vector<float> pulled0;  // rank 0's last pulled weights
    int64_t correct_last = -1, test_rows = 0;
    int64_t sample_steps = 0;
    std::mutex stat_mu;
};

void run_rank(Job *job, int rank) {
    const int D = job->D;
    std::vector<float> weight((size_t)D);
    int64_t steps = 0;
    for (int it = 0; it < job->num_iteration; ++it) {
        Iter iter;
        iter.samples = parse_part(job->root + "/train/part-00" + std::to_string(rank + 1), D);
        if (iter.samples.empty()) break;  // the reference would never terminate
        while (!iter.round_end) {  // lr.cc:28-45
            std::vector<DenseSample> batch = iter.next_batch(job->batch);
            job->server->pull(weight);
            std::vector<float> grad((size_t)D);
            for (int j = 0; j < D; ++j) {
                grad[(size_t)j] = 0;
                for (auto &s : batch)
                    grad[(size_t)j] = grad[(size_t)j] + (sigmoid_by_value(weight, s.features_by_value()) -
                                                         (float)s.label) * s.feature[(size_t)j];
                grad[(size_t)j] = (float)(1. * (double)grad[(size_t)j] / (double)batch.size() +
                                          (double)((job->C * weight[(size_t)j]) / (float)batch.size()));
            }
            job->server->push(rank, grad);
            steps += (int64_t)batch.size();
        }
        if (rank == 0 && (it + 1) % job->test_interval == 0) {  // lr.cc:47-63
            Iter test;
            test.samples = parse_part(job->root + "/test/part-001", D);
            job->server->pull(weight);
            std::vector<DenseSample> all = test.next_batch(-1);
            int64_t c = 0;
            for (auto &s : all) {
                std::vector<float> f = s.features_by_value();
                float z = 0;
                for (int j = 0; j < D; ++j) z = z + weight[(size_t)j] * f[(size_t)j];
                if ((int)(z > 0) == s.label) ++c;
            }
            std::lock_guard<std::mutex> g(job->stat_mu);
            job->correct_last = c;
            job->test_rows = (int64_t)all.size();
        }
    }
    std::lock_guard<std::mutex> g(job->stat_mu);
    job->sample_steps += steps;
    if (rank == 0) job->pulled0 = weight;
}

}  // namespace

extern "C" {

// Runs local.sh's job (W worker threads + server) on DATA_DIR `root`.
// Returns 0, or -1 on a bad argument.  w_out[D] receives the server's final
// weights; *sample_steps the samples consumed by all ranks' Train steps;
// *seconds the wall time; *correct / *test_rows rank 0's last Test.
int orc_ref_local_run(const char *root, int W, int D, int num_iteration, int batch_size, int test_interval,
                      float lr, int mode, float *w_out, int64_t *sample_steps, double *seconds, int64_t *correct,
                      int64_t *test_rows) {
    if (!root || W < 1 || D < 1 || num_iteration < 0 || batch_size == 0 || test_interval == 0) return -1;
    Server server(W, D, lr, mode);
    orc_init_weight(0, server.w.data(), D);  // rank 0's initial push (main.cc:141-148)
    Job job;
    job.root = root;
    job.W = W;
    job.D = D;
    job.num_iteration = num_iteration;
    job.batch = batch_size;
    job.test_interval = test_interval;
    job.mode = mode;
    job.lr = lr;
    job.server = &server;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int r = 0; r < W; ++r) th.emplace_back(run_rank, &job, r);
    for (auto &t : th) t.join();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (w_out) memcpy(w_out, server.w.data(), sizeof(float) * (size_t)D);
    if (sample_steps) *sample_steps = job.sample_steps;
    if (seconds) *seconds = el;
    if (correct) *correct = job.correct_last;
    if (test_rows) *test_rows = job.test_rows;
    return 0;
}

// One (j, sample) iteration of lr.cc:35-39 at dimension D, timed: the
// reference's per-sample cost at configurations it cannot run (D = 10^6+:
// a dense sample is D floats and the gradient O(B * D^2)).  Runs `iters`
// iterations over `n` dense samples with the real loop body (two by-value
// copies + the O(D) margin); returns seconds per iteration.
double orc_ref_inner_cost(int D, int n, int64_t iters) {
    if (D < 1 || n < 1 || iters < 1) return -1.0;
    std::vector<DenseSample> batch((size_t)n);
    for (int s = 0; s < n; ++s) {
        batch[(size_t)s].feature.assign((size_t)D, 0.0f);
        for (int k = 0; k < 50 && k < D; ++k) batch[(size_t)s].feature[(size_t)((k * 7919 + s) % D)] = 1.0f;
        batch[(size_t)s].label = s & 1;
    }
    std::vector<float> weight((size_t)D);
    orc_init_weight(0, weight.data(), D);
    volatile float sink = 0;
    float g = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int64_t i = 0; i < iters; ++i) {
        const DenseSample &s = batch[(size_t)(i % n)];
        const int j = (int)(i % D);
        g = g + (sigmoid_by_value(weight, s.features_by_value()) - (float)s.label) * s.feature[(size_t)j];
    }
    sink = g;
    (void)sink;
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / (double)iters;
}

}  // extern "C"
