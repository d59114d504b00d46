// main.cc -- `distlr`, the drop-in for the reference's bin/distlr
// (src/main.cc:124-181) on MI355X.
//
// Same configuration (environment variables, examples/local.sh:12-19):
//   DATA_DIR, NUM_FEATURE_DIM, NUM_ITERATION, BATCH_SIZE, TEST_INTERVAL,
//   SYNC_MODE ("1" = sync), LEARNING_RATE (parsed with ToFloat, main.cc:27)
// and the worker count DMLC_NUM_WORKER (local.sh:24).  Same files:
// DATA_DIR/train/part-00{r+1}, DATA_DIR/test/part-001,
// DATA_DIR/models/part-00{r+1}.  Same output lines.
//
// Topology: one process, one thread per worker (rank).  With at least as
// many GPUs as workers each rank owns a GPU and gradients are exchanged
// over RCCL (all-to-all of key ranges + rank-ordered merge + all-gather).
// With more workers than GPUs (e.g. local.sh's 2 workers on one GPU) and a
// single GPU, the ranks share it as a loopback group (dlr_create_group:
// the same engine step, the collectives become device-to-device copies);
// with several GPUs but more workers than GPUs, the workers share GPUs and
// exchange through the in-process ParamServer.
// Optional: DISTLR_GPUS (GPUs to use), DISTLR_TOPOLOGY=rccl|group|ps,
// DISTLR_SYNC_MERGE=last (main.cc:71 as written instead of the mean),
// DISTLR_TIMING=1 (each rank reports its epoch loop's wall time on stderr).
// Missing variables are reported (the reference dereferences NULL).
//
// Roles (DMLC_ROLE, examples/local.sh:30-49; main.cc:172-181 dispatches
// on it through ps::IsServer / ps::IsWorker): local.sh starts one
// scheduler, S servers and W workers of this binary.  Here the scheduler
// process runs the whole W-rank job (the ranks are threads of it, so it is
// also where the collectives and the server update happen); a server
// process prints its mode line (main.cc:30) and exits; a worker process
// exits at once.  So local.sh's launch pattern produces exactly one
// training run, one set of accuracy lines and one set of model files.
// Without DMLC_ROLE the binary runs the job standalone.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "distlr/data_iter.h"
#include "distlr/lr.h"
#include "distlr/util.h"
#include "distlr_amd.h"

namespace {

std::mutex g_out;

const char *need_env(const char *name) {
    const char *v = getenv(name);
    if (!v) {
        std::cerr << "distlr: environment variable " << name << " is not set" << std::endl;
        exit(2);
    }
    return v;
}

struct Config {
    std::string root;
    int num_feature_dim, num_iteration, batch_size, test_interval, workers;
    bool sync_mode;
    float learning_rate;
};

// main.cc:124-170 for one rank.
// The LR (which owns kv, lr.h:13-15) lives in `owner`, a slot of main's:
// every rank's KVWorker stays alive until all threads have joined, so a
// failing rank can release every peer through `all` whatever state they are in.
void run_worker(const Config &cfg, int rank, distlr::KVWorker *kv, std::vector<distlr::KVWorker *> *all,
                std::unique_ptr<distlr::LR> *owner_slot, std::vector<int> *failed) {
    std::unique_ptr<distlr::LR> &owner = *owner_slot;
    try {
        {
            std::lock_guard<std::mutex> g(g_out);
            std::cout << 0 << "I got a rank " << rank << std::endl;  // main.cc:134 (customer id 0)
        }
        owner.reset(new distlr::LR(cfg.num_feature_dim));
        distlr::LR &lr = *owner;
        lr.SetKVWorker(kv);
        lr.SetRank(rank);
        {
            std::lock_guard<std::mutex> g(g_out);
            std::cout << 0 << "I'm going to push " << rank << std::endl;  // main.cc:140
            std::cout << 0 << "I'm here " << rank << std::endl;           // main.cc:149
            std::cout << "Worker[" << rank << "]: start working..." << std::endl;
        }
        const auto t_loop = std::chrono::steady_clock::now();
        for (int i = 0; i < cfg.num_iteration; ++i) {
            std::string train_filename = cfg.root + "/train/part-00" + std::to_string(rank + 1);
            distlr::DataIter iter(train_filename, cfg.num_feature_dim);
            lr.Train(iter, i, cfg.batch_size);
            if (rank == 0 && (i + 1) % cfg.test_interval == 0) {
                std::string test_filename = cfg.root + "/test/part-001";
                distlr::DataIter test_iter(test_filename, cfg.num_feature_dim);
                std::lock_guard<std::mutex> g(g_out);
                lr.Test(test_iter, i + 1);
            }
        }
        if (getenv("DISTLR_TIMING")) {  // not in the reference: the epoch loop's wall time (bench.py c1e2e)
            const double sec =
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t_loop).count();
            std::lock_guard<std::mutex> g(g_out);
            std::cerr << "distlr: rank " << rank << " epoch loop " << sec << " s" << std::endl;
        }
        std::string modelfile = cfg.root + "/models/part-00" + std::to_string(rank + 1);
        lr.SaveModel(modelfile);
    } catch (const std::exception &e) {
        // release its peers: every rank's transport (the ranks are threads
        // of this process, so the failing thread can flag their RCCL
        // communicators too -- each rank's own thread then aborts its
        // communicator at its next wait, which returns its stuck collectives)
        const std::string why = std::string("worker ") + std::to_string(rank) + " failed: " + e.what();
        for (distlr::KVWorker *p : *all)
            if (p) p->Abort(why);
        std::lock_guard<std::mutex> g(g_out);
        std::cerr << "distlr: worker " << rank << ": " << e.what() << std::endl;
        (*failed)[(size_t)rank] = 1;
    }
}

}  // namespace

int main(int argc, char **argv) {
    (void)argc;
    (void)argv;  // like the reference, configuration comes from the environment
    Config cfg;
    cfg.root = need_env("DATA_DIR");
    cfg.num_feature_dim = distlr::ToInt(need_env("NUM_FEATURE_DIM"));
    cfg.num_iteration = distlr::ToInt(need_env("NUM_ITERATION"));
    cfg.batch_size = distlr::ToInt(need_env("BATCH_SIZE"));
    cfg.test_interval = distlr::ToInt(need_env("TEST_INTERVAL"));
    cfg.sync_mode = !strcmp(need_env("SYNC_MODE"), "1");
    cfg.learning_rate = distlr::ToFloat(need_env("LEARNING_RATE"));
    const char *nw = getenv("DMLC_NUM_WORKER");
    cfg.workers = nw ? distlr::ToInt(nw) : 1;
    if (cfg.workers < 1 || cfg.num_feature_dim < 1 || cfg.test_interval == 0) {
        std::cerr << "distlr: bad configuration" << std::endl;
        return 2;
    }
    const char *role_env = getenv("DMLC_ROLE");
    const std::string role = role_env ? role_env : "";
    if (!role.empty() && role != "scheduler" && role != "server" && role != "worker") {
        std::cerr << "distlr: unknown DMLC_ROLE '" << role << "'" << std::endl;
        return 2;
    }
    if (role == "worker") {
        std::cerr << "distlr: DMLC_ROLE=worker: the worker ranks run as threads of the scheduler process"
                  << std::endl;
        return 0;
    }
    // main.cc:30, printed by each server (KVStoreDistServer's constructor)
    if (role.empty() || role == "server")
        std::cout << "Server mode: " << (cfg.sync_mode ? "sync" : "async") << std::endl;
    if (role == "server") return 0;

    int ngpu = 0;
    if (hipGetDeviceCount(&ngpu) != hipSuccess || ngpu < 1) {
        std::cerr << "distlr: no GPU visible" << std::endl;
        return 3;
    }
    if (const char *g = getenv("DISTLR_GPUS")) ngpu = std::max(1, std::min(ngpu, atoi(g)));
    std::string topo = getenv("DISTLR_TOPOLOGY") ? getenv("DISTLR_TOPOLOGY") : "";
    if (topo.empty()) topo = cfg.workers <= ngpu ? "rccl" : ngpu == 1 ? "group" : "ps";
    if (topo != "rccl" && topo != "group" && topo != "ps") {
        std::cerr << "distlr: DISTLR_TOPOLOGY must be rccl, group or ps" << std::endl;
        return 2;
    }
    if (topo == "rccl" && cfg.workers > ngpu) {
        std::cerr << "distlr: DISTLR_TOPOLOGY=rccl needs one GPU per worker" << std::endl;
        return 2;
    }
    if (topo == "group" && cfg.workers > 16) {
        std::cerr << "distlr: DISTLR_TOPOLOGY=group supports at most 16 workers" << std::endl;
        return 2;
    }

    std::vector<int> failed((size_t)cfg.workers, 0);
    std::vector<std::unique_ptr<distlr::LR>> models((size_t)cfg.workers);  // destroyed after every thread joined
    std::vector<std::thread> th;
    std::unique_ptr<distlr::ParamServer> ps;
    std::vector<distlr::KVWorker *> kvs((size_t)cfg.workers, nullptr);
    try {
        if (topo == "group") {
            std::vector<distlr::KVWorker *> g =
                distlr::KVWorker::Group(0, cfg.workers, cfg.learning_rate, cfg.sync_mode, cfg.num_feature_dim);
            for (int r = 0; r < cfg.workers; ++r) kvs[(size_t)r] = g[(size_t)r];
        } else if (topo == "rccl") {
            char uid[DLR_UNIQUE_ID_BYTES] = {0};
            if (cfg.workers > 1 && dlr_get_unique_id(uid) != DLR_OK) {
                std::cerr << "distlr: " << dlr_last_error(nullptr) << std::endl;
                return 4;
            }
            // Communicator creation is collective: create every rank's
            // context concurrently (this is the barrier of main.cc:150).
            std::vector<std::thread> init;
            std::vector<std::string> err((size_t)cfg.workers);
            for (int r = 0; r < cfg.workers; ++r)
                init.emplace_back([&, r] {
                    try {
                        kvs[(size_t)r] = new distlr::KVWorker(r, r, cfg.workers, uid, cfg.learning_rate,
                                                              cfg.sync_mode, cfg.num_feature_dim);
                    } catch (const std::exception &e) {
                        err[(size_t)r] = e.what();
                    }
                });
            for (auto &t : init) t.join();
            for (auto &e : err)
                if (!e.empty()) throw std::runtime_error(e);
        } else {
            ps.reset(new distlr::ParamServer(0, cfg.workers, cfg.learning_rate, cfg.sync_mode,
                                             cfg.num_feature_dim));
            for (int r = 0; r < cfg.workers; ++r)
                kvs[(size_t)r] = new distlr::KVWorker(r % ngpu, r, ps.get(), cfg.learning_rate, cfg.sync_mode,
                                                      cfg.num_feature_dim);
        }
    } catch (const std::exception &e) {
        std::cerr << "distlr: " << e.what() << std::endl;
        return 4;
    }
    for (int r = 0; r < cfg.workers; ++r)
        th.emplace_back(run_worker, std::cref(cfg), r, kvs[(size_t)r], &kvs, &models[(size_t)r], &failed);
    for (auto &t : th) t.join();
    for (int f : failed)
        if (f) return 1;
    return 0;
}
