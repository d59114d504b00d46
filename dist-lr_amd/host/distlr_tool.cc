// distlr_tool.cc -- host-only checks of the C++ drop-in surface
// (distlr::Split/ToInt/ToFloat, DataIter, Sample).  Prints the same text
// formats as oracle/ref_driver (the reference's own code), so tests can
// compare this surface with the reference-built goldens without a GPU.
//   distlr_tool kat <strings-file>
//   distlr_tool parse <libsvm-file> <D>
//   distlr_tool batches <libsvm-file> <D> <B>
//   distlr_tool debuginfo <libsvm-file> <D>   (Sample::DebugInfo per sample)
//   distlr_tool lrdebug <D> [random_state]      (LR::DebugInfo of a new LR: its
//                                               initial weights, lr.cc:84-90)
//   distlr_tool partial <libsvm-file> <D> <B> <k> <lr>   (GPU: NextBatch(k), then
//       LR::Train on what is left of the round, lr.cc:29-30; prints the
//       iterator's state and the last pulled weights as hex bits)
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "distlr/data_iter.h"
#include "distlr/lr.h"
#include "distlr/sample.h"
#include "distlr/util.h"

static uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

static uint64_t fnv(const std::vector<float> &v) {
    uint64_t h = 1469598103934665603ull;
    for (float f : v) {
        const uint32_t u = bits(f);
        for (int k = 0; k < 4; ++k) {
            h ^= (u >> (8 * k)) & 0xffu;
            h *= 1099511628211ull;
        }
    }
    return h;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const std::string mode = argv[1];
    try {
        if (mode == "kat") {
            std::ifstream in(argv[2]);
            std::string s;
            while (std::getline(in, s)) {
                const std::vector<std::string> f = distlr::Split(s, ':');
                std::printf("%d %08x %zu", distlr::ToInt(s), bits(distlr::ToFloat(s)), f.size());
                for (auto &x : f) {
                    std::printf("\t");
                    for (unsigned char ch : x) std::printf("%02x", ch);
                }
                std::printf("\n");
            }
            return 0;
        }
        if (mode == "lrdebug") {  // host only: no KVWorker, no GPU
            distlr::LR lr(std::atoi(argv[2]), 0.001f, 1.0f, argc > 3 ? std::atoi(argv[3]) : 0);
            std::printf("%s", lr.DebugInfo().c_str());
            return 0;
        }
        if (argc < 4) return 2;
        const int D = std::atoi(argv[3]);
        distlr::DataIter it(argv[2], D);
        if (mode == "parse") {
            std::vector<distlr::Sample> all = it.NextBatch(-1);
            std::printf("n %zu\n", all.size());
            for (auto &s : all) {
                std::vector<float> x = s.GetFeature();
                int nnz = 0;
                for (float v : x) nnz += (v != 0.0f);
                std::printf("%d %d", s.GetLabel(), nnz);
                for (int j = 0; j < D; ++j)
                    if (x[(size_t)j] != 0.0f) std::printf(" %d:%08x", j, bits(x[(size_t)j]));
                std::printf("\n");
            }
            return 0;
        }
        if (mode == "batches" && argc >= 5) {
            const int B = std::atoi(argv[4]);
            int b = 0;
            while (it.HasNext()) {
                std::vector<distlr::Sample> batch = it.NextBatch(B);
                std::printf("batch %d %zu\n", b++, batch.size());
                for (auto &s : batch)
                    std::printf("%d %016llx\n", s.GetLabel(), (unsigned long long)fnv(s.GetFeature()));
            }
            return 0;
        }
        if (mode == "partial" && argc >= 7) {  // GPU: one rank, KVWorker on device 0
            const int B = std::atoi(argv[4]), k = std::atoi(argv[5]);
            const float lr = (float)std::atof(argv[6]);
            if (k > 0) (void)it.NextBatch(k);
            std::printf("before %d %d\n", it.offset(), it.HasNext() ? 1 : 0);
            distlr::LR model(D);
            model.SetKVWorker(new distlr::KVWorker(0, 0, 1, nullptr, lr, true, D));
            model.Train(it, 0, B);
            std::printf("after %d %d\n", it.offset(), it.HasNext() ? 1 : 0);
            for (float v : model.GetWeight()) std::printf("%08x\n", bits(v));
            return 0;
        }
        if (mode == "debuginfo") {
            for (auto &s : it.NextBatch(-1)) std::printf("%s\n", s.DebugInfo().c_str());
            return 0;
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "distlr_tool: %s\n", e.what());
        return 1;
    }
    return 2;
}
