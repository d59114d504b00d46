// ref_driver.cc -- TEST INFRASTRUCTURE.  A command-line harness around the
// reference's OWN parsing code, compiled where it lies:
//   /root/reference/src/util.cc            (Split / ToInt / ToFloat)
//   /root/reference/include/data_iter.h    (DataIter, header-only)
//   /root/reference/include/sample.h       (Sample, header-only)
// These need nothing outside the reference (no ps-lite), so the build is the
// reference's code as written.  src/lr.cc and src/main.cc include ps-lite's
// "ps/ps.h", which this image lacks; they are NOT built (unbuildable here).
//
// Output is consumed by tests/golden/make_golden.py, which writes the golden
// fixtures.  Built into oracle/_ref/ by oracle/Makefile; never shipped.
//
// Usage:
//   ref_driver kat <strings-file>            one line per input string:
//        ToInt  ToFloat-bits(hex)  nfields  <TAB>hex(field0)<TAB>hex(field1)...
//   ref_driver parse <libsvm-file> <D>       one line per sample:
//        label  nnz  idx:bits ...           (0-based idx, hex float bits)
//   ref_driver batches <libsvm-file> <D> <B> one line per NextBatch() call
//        until HasNext() is false: "batch <b> <size>" then per sample the
//        label and an FNV-1a hash of its dense feature bits.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "data_iter.h"
#include "sample.h"
#include "util.h"

static uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

static uint64_t fnv(const std::vector<float> &v) {
    uint64_t h = 1469598103934665603ull;
    for (float f : v) {
        uint32_t u = bits(f);
        for (int k = 0; k < 4; ++k) {
            h ^= (u >> (8 * k)) & 0xffu;
            h *= 1099511628211ull;
        }
    }
    return h;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s kat|parse|batches ...\n", argv[0]);
        return 2;
    }
    std::string mode = argv[1];
    if (mode == "kat") {
        std::ifstream in(argv[2]);
        std::string s;
        while (std::getline(in, s)) {
            int iv = distlr::ToInt(s);
            float fv = distlr::ToFloat(s);
            std::vector<std::string> f = distlr::Split(s, ':');
            std::printf("%d %08x %zu", iv, bits(fv), f.size());
            for (auto &x : f) {  // fields hex-encoded so tabs/spaces survive
                std::printf("\t");
                for (unsigned char ch : x) std::printf("%02x", ch);
            }
            std::printf("\n");
        }
        return 0;
    }
    if (mode == "parse" && argc >= 4) {
        int D = std::atoi(argv[3]);
        distlr::DataIter it(argv[2], D);
        std::vector<distlr::Sample> all = it.NextBatch(-1);
        // NextBatch(-1) on an empty file returns nothing; report the count.
        std::printf("n %zu\n", all.size());
        for (auto &s : all) {
            std::vector<float> x = s.GetFeature();
            int nnz = 0;
            for (float v : x) nnz += (v != 0.0f);
            std::printf("%d %d", s.GetLabel(), nnz);
            for (int j = 0; j < D; ++j)
                if (x[j] != 0.0f) std::printf(" %d:%08x", j, bits(x[j]));
            std::printf("\n");
        }
        return 0;
    }
    if (mode == "batches" && argc >= 5) {
        int D = std::atoi(argv[3]);
        int B = std::atoi(argv[4]);
        distlr::DataIter it(argv[2], D);
        int b = 0;
        while (it.HasNext()) {
            std::vector<distlr::Sample> batch = it.NextBatch(B);
            std::printf("batch %d %zu\n", b++, batch.size());
            for (auto &s : batch) std::printf("%d %016llx\n", s.GetLabel(), (unsigned long long)fnv(s.GetFeature()));
        }
        return 0;
    }
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}
