// ycsb_gen.cpp -- the YCSB driver's key generators (benchmark/benchmark_common.h:12-105),
// restated for the harness with explicit seeds (the reference seeds with rand() after
// srand(time(0)), ycsb_workload.cpp:520, so its streams are not reproducible).
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "../../include/stage_hip.h"

namespace {

constexpr uint64_t kMask48 = (1ull << 48) - 1;
constexpr uint64_t kMul = 0x5DEECE66Dull;
constexpr uint64_t kAdd = 0xBull;

struct FastRandom {  // Java LCG, benchmark_common.h:12-64
    uint64_t seed;
    explicit FastRandom(uint64_t s) : seed((s ^ kMul) & kMask48) {}
    uint64_t next(unsigned bits) {
        seed = (seed * kMul + kAdd) & kMask48;
        return seed >> (48 - bits);
    }
    uint64_t next64() { return (next(32) << 32) + next(32); }
    double uniform() { return (double)((next(26) << 27) + next(27)) / (double)(1ull << 53); }
    // advance by k LCG steps (affine map composed by squaring)
    void jump(uint64_t k) {
        uint64_t a = kMul, c = kAdd, A = 1, C = 0;
        while (k) {
            if (k & 1) {
                A = (A * a) & kMask48;
                C = (C * a + c) & kMask48;
            }
            c = (c * a + c) & kMask48;
            a = (a * a) & kMask48;
            k >>= 1;
        }
        seed = (seed * A + C) & kMask48;
    }
};

// ZipfDistribution::zeta (benchmark_common.h:80-84); sequential as the reference up to
// 2^25 terms, fixed 64-way chunking above (deterministic, not bit-identical to a serial sum)
double zeta(uint64_t n, double theta) {
    if (n <= (1ull << 25)) {
        double sum = 0;
        for (uint64_t i = 1; i <= n; i++) sum += std::pow(1.0 / (double)i, theta);
        return sum;
    }
    const int chunks = 64;
    std::vector<double> part(chunks, 0.0);
    std::vector<std::thread> th;
    for (int c = 0; c < chunks; ++c)
        th.emplace_back([&, c] {
            uint64_t b = 1 + n * (uint64_t)c / chunks, e = n * (uint64_t)(c + 1) / chunks;
            double s = 0;
            for (uint64_t i = b; i <= e; i++) s += std::pow(1.0 / (double)i, theta);
            part[c] = s;
        });
    for (auto &x : th) x.join();
    double sum = 0;
    for (double v : part) sum += v;
    return sum;
}

}  // namespace

extern "C" int stage_fastrandom_next(uint64_t seed, uint64_t count, uint64_t *out) {
    if (!out && count) return STAGE_E_ARG;
    FastRandom r(seed);
    for (uint64_t i = 0; i < count; ++i) out[i] = r.next64();
    return STAGE_OK;
}

// ZipfDistribution(n, theta).GetNextNumber() (benchmark_common.h:67-98): draws in [1, n]
extern "C" int stage_zipf_draws(uint64_t n, double theta, uint64_t seed, uint64_t count, uint64_t *out,
                                int nthreads) {
    if (n < 2 || !(theta > 0.0) || theta >= 1.0 || (!out && count)) return STAGE_E_ARG;
    const double zeta2 = zeta(2, theta);
    const double zetan = zeta(n, theta);
    const double alpha = 1.0 / (1.0 - theta);
    const double eta = (1.0 - std::pow(2.0 / (double)n, 1.0 - theta)) / (1.0 - zeta2 / zetan);
    const double half_pow = 1.0 + std::pow(0.5, theta);
    if (nthreads < 1) nthreads = 1;
    if (count < 4096) nthreads = 1;
    std::vector<std::thread> th;
    for (int k = 0; k < nthreads; ++k)
        th.emplace_back([=] {
            const uint64_t b = count * (uint64_t)k / nthreads, e = count * (uint64_t)(k + 1) / nthreads;
            FastRandom r(seed);
            r.jump(2 * b);  // every draw consumes two LCG steps (NextUniform)
            for (uint64_t i = b; i < e; ++i) {
                const double u = r.uniform();
                const double uz = u * zetan;
                uint64_t v;
                if (uz < 1) v = 1;
                else if (uz < half_pow) v = 2;
                else v = 1 + (uint64_t)((double)n * std::pow(eta * u - eta + 1, alpha));
                out[i] = v;
            }
        });
    for (auto &x : th) x.join();
    return STAGE_OK;
}
