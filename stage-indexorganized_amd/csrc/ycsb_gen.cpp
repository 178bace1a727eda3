// ycsb_gen.cpp -- the YCSB driver's key generators (benchmark/benchmark_common.h:12-105),
// restated for the harness with explicit seeds (the reference seeds with rand() after
// srand(time(0)), ycsb_workload.cpp:520, so its streams are not reproducible).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
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

// ZipfDistribution::zeta (benchmark_common.h:80-84), bit-identical to the reference's serial
// sum for every n: the pow() terms of a block are computed by worker threads, the block is then
// added in the reference's order (i = 1, 2, ...) on this thread.  Cached per (n, theta): the
// drivers draw many streams over one key range.
double zeta_serial(uint64_t n, double theta) {
    constexpr uint64_t kBlock = 1ull << 20;
    if (n <= kBlock) {
        double sum = 0;
        for (uint64_t i = 1; i <= n; i++) sum += std::pow(1.0 / (double)i, theta);
        return sum;
    }
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<double> buf[2] = {std::vector<double>(kBlock), std::vector<double>(kBlock)};
    auto fill = [&](std::vector<double> &dst, uint64_t b, uint64_t e) {  // terms b..e-1 (1-based)
        std::vector<std::thread> th;
        for (unsigned k = 0; k < nt; ++k)
            th.emplace_back([&, k] {
                const uint64_t lo = b + (e - b) * k / nt, hi = b + (e - b) * (k + 1) / nt;
                for (uint64_t i = lo; i < hi; ++i) dst[i - b] = std::pow(1.0 / (double)i, theta);
            });
        for (auto &x : th) x.join();
    };
    double sum = 0;
    uint64_t b = 1;
    fill(buf[0], 1, std::min(n + 1, 1 + kBlock));
    for (int cur = 0; b <= n; cur ^= 1) {
        const uint64_t e = std::min(n + 1, b + kBlock);
        const uint64_t nb = e, ne = std::min(n + 1, nb + kBlock);
        std::thread next;  // the next block's terms while this block is summed
        if (nb <= n) next = std::thread([&, nb, ne, cur] { fill(buf[cur ^ 1], nb, ne); });
        const double *t = buf[cur].data();
        for (uint64_t i = 0; i < e - b; ++i) sum += t[i];
        if (next.joinable()) next.join();
        b = e;
    }
    return sum;
}

double zeta(uint64_t n, double theta) {
    static std::mutex mu;
    static std::map<std::pair<uint64_t, uint64_t>, double> cache;
    uint64_t tb;
    std::memcpy(&tb, &theta, 8);
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({n, tb});
    if (it != cache.end()) return it->second;
    const double z = zeta_serial(n, theta);
    cache.emplace(std::make_pair(n, tb), z);
    return z;
}

}  // namespace

extern "C" int stage_fastrandom_next(uint64_t seed, uint64_t count, uint64_t *out) {
    if (!out && count) return STAGE_E_ARG;
    FastRandom r(seed);
    for (uint64_t i = 0; i < count; ++i) out[i] = r.next64();
    return STAGE_OK;
}

// RunMixed's per-op draws from its FastRandom (ycsb_mixed.cpp:26, 37, 43): rng.NextUniform() <
// update_ratio makes op i an update, whose 100-B delta is memset to rng.next_char() (next(8) %
// 256, benchmark_common.h:29) drawn right after; a read consumes only the uniform.
extern "C" int stage_ycsb_ops(uint64_t seed, uint64_t count, double update_ratio, uint8_t *is_update,
                              uint8_t *chr) {
    if (count && (!is_update || !chr)) return STAGE_E_ARG;
    FastRandom r(seed);
    for (uint64_t i = 0; i < count; ++i) {
        const bool upd = r.uniform() < update_ratio;
        is_update[i] = upd;
        chr[i] = upd ? (uint8_t)(r.next(8) % 256) : 0;
    }
    return STAGE_OK;
}

extern "C" int stage_zipf_zeta(uint64_t n, double theta, double *out) {
    if (!out) return STAGE_E_ARG;
    *out = zeta(n, theta);
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
