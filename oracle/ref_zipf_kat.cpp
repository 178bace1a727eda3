// TEST INFRASTRUCTURE: prints known answers of the reference's own FastRandom and
// ZipfDistribution (benchmark/benchmark_common.h:10-98), compiled from the reference checkout
// into oracle/_ref/ (never committed, never linked into the product) to pin the harness's
// stream generator (tests/golden/make_zipf_kat.py -> tests/golden/zipf_kat.json).
// The reference seeds ZipfDistribution's generator with rand(); the driver replaces that
// generator by FastRandom(seed) after construction, so the draws are reproducible.
//   ref_zipf_kat fast SEED COUNT          -> FastRandom(SEED).next() x COUNT
//   ref_zipf_kat zipf N THETA SEED COUNT  -> zeta values (hex bits) + GetNextNumber() x COUNT
//   ref_zipf_kat ops SEED COUNT RATIO     -> RunMixed's per-op draws (ycsb_mixed.cpp:26, 37, 43):
//                                            NextUniform() < RATIO, then next_char() for an update
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "benchmark_common.h"

using mvstore::benchmark::FastRandom;
using mvstore::benchmark::ZipfDistribution;

static unsigned long long bits(double d) {
    unsigned long long u;
    std::memcpy(&u, &d, 8);
    return u;
}

int main(int argc, char **argv) {
    if (argc >= 4 && !std::strcmp(argv[1], "fast")) {
        FastRandom r(std::strtoull(argv[2], nullptr, 0));
        const unsigned long long count = std::strtoull(argv[3], nullptr, 0);
        std::printf("{\"next\": [");
        for (unsigned long long i = 0; i < count; ++i) std::printf("%s%lu", i ? ", " : "", r.next());
        std::printf("]}\n");
        return 0;
    }
    if (argc >= 6 && !std::strcmp(argv[1], "zipf")) {
        const uint64_t n = std::strtoull(argv[2], nullptr, 0);
        const double theta = std::strtod(argv[3], nullptr);
        ZipfDistribution z(n, theta);
        z.rand_generator = FastRandom(std::strtoull(argv[4], nullptr, 0));
        const unsigned long long count = std::strtoull(argv[5], nullptr, 0);
        std::printf("{\"zeta_n_bits\": \"%016llx\", \"zeta_2_bits\": \"%016llx\", \"draws\": [", bits(z.denom),
                    bits(z.zeta_2_theta));
        for (unsigned long long i = 0; i < count; ++i)
            std::printf("%s%llu", i ? ", " : "", (unsigned long long)z.GetNextNumber());
        std::printf("]}\n");
        return 0;
    }
    if (argc >= 5 && !std::strcmp(argv[1], "ops")) {
        FastRandom rng(std::strtoull(argv[2], nullptr, 0));
        const unsigned long long count = std::strtoull(argv[3], nullptr, 0);
        const double ratio = std::strtod(argv[4], nullptr);
        std::printf("{\"ops\": [");
        for (unsigned long long i = 0; i < count; ++i) {
            auto rng_val = rng.NextUniform();
            int v = -1;  // read
            if (rng_val < ratio) {
                char chr = rng.next_char();
                v = (unsigned char)chr;
            }
            std::printf("%s%d", i ? ", " : "", v);
        }
        std::printf("]}\n");
        return 0;
    }
    std::fprintf(stderr, "usage: ref_zipf_kat fast SEED COUNT | zipf N THETA SEED COUNT | ops SEED COUNT RATIO\n");
    return 2;
}
