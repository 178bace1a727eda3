// reader_drive.cpp -- host-side driver for the two host-memory forms of the boundary, written
// against include/stage_hip.h only (what a reference driver would link):
//
//   mode "reader": T worker threads each run read-only transactions of `ops` BTree::Read
//     calls (RunMixed, ycsb_mixed.cpp:25-110, u = 0) through stage_reader_read -- the
//     single-key adapter that coalesces the threads' calls into device batches, or, with
//     resident_waves > 0, the resident reader (stage_reader_create_resident: that many
//     device-resident waves polling a 4096-slot request ring); per-read latency percentiles;
//   mode "host":   the same keys through stage_probe_host in batches of `batch` (pinned
//     buffers), i.e. a driver that already batches.
//
// Prints one JSON line.  Usage:
//   reader_drive <rows> <seconds> <threads> <max_batch> <max_wait_us> <batch> [theta] [resident_waves]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/stage_hip.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        int rc_ = (x);                                                                          \
        if (rc_) {                                                                              \
            std::fprintf(stderr, "%s failed: rc=%d %s\n", #x, rc_, stage_last_error());       \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

using clk = std::chrono::steady_clock;

int main(int argc, char **argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s rows seconds threads max_batch max_wait_us batch [theta]\n", argv[0]);
        return 2;
    }
    const uint64_t rows = std::strtoull(argv[1], nullptr, 10);
    const double seconds = std::atof(argv[2]);
    const int threads = std::atoi(argv[3]);
    const uint32_t max_batch = (uint32_t)std::atoi(argv[4]);
    const uint32_t max_wait = (uint32_t)std::atoi(argv[5]);
    const uint64_t batch = std::strtoull(argv[6], nullptr, 10);
    const double theta = argc > 7 ? std::atof(argv[7]) : 0.9;
    const uint32_t resident_waves = argc > 8 ? (uint32_t)std::atoi(argv[8]) : 0;

    stage_params p{16 * 1024, 32 * 1024, 64 * 1024, 1000, 8, 0};
    stage_table *t = nullptr;
    CK(stage_table_create(&p, &t));
    uint64_t loaded = 0;
    auto t0 = clk::now();
    CK(stage_load_ycsb(t, 0, rows, 8, 0, &loaded));
    CK(stage_sync(t));
    const double t_setup = std::chrono::duration<double>(clk::now() - t0).count();
    const uint32_t stride = stage_record_stride(t);

    // key streams: Zipf(theta) over [1, rows-1] (ycsb_workload.cpp:193), one per thread
    const uint64_t per_thread = 1 << 20;
    std::vector<std::vector<uint64_t>> keys(threads, std::vector<uint64_t>(per_thread));
    for (int i = 0; i < threads; ++i) CK(stage_zipf_draws(rows - 1, theta, 0x5EED + i, per_thread, keys[i].data(), 8));

    // ---- mode reader
    stage_reader *r = nullptr;
    if (resident_waves) CK(stage_reader_create_resident(t, 4096, resident_waves, 5000, &r));
    else CK(stage_reader_create(t, max_batch, max_wait, &r));
    std::atomic<bool> go{false}, stop{false};
    std::atomic<uint64_t> bad{0};
    std::vector<uint64_t> done(threads, 0);
    std::vector<std::vector<float>> lat(threads);  // per-read latency samples (us)
    std::vector<std::thread> th;
    for (int i = 0; i < threads; ++i)
        th.emplace_back([&, i] {
            std::vector<uint8_t> rec(1008);
            stage_probe_out o;
            lat[i].reserve(1 << 20);
            while (!go.load()) std::this_thread::yield();
            uint64_t n = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                const uint64_t k = keys[i][n % per_thread];
                const auto a = clk::now();
                if (stage_reader_read(r, k, 8, 0xFFFFFFFEu, &o, rec.data())) {
                    bad++;
                    break;
                }
                if (lat[i].size() < (1u << 20))
                    lat[i].push_back(std::chrono::duration<float, std::micro>(clk::now() - a).count());
                if (o.status != STAGE_ST_LATEST || rec[8] != (uint8_t)k || std::memcmp(rec.data(), &k, 8)) bad++;
                ++n;
            }
            done[i] = n;
        });
    t0 = clk::now();
    go = true;
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (auto &x : th) x.join();
    const double t_reader = std::chrono::duration<double>(clk::now() - t0).count();
    uint64_t reads = 0;
    for (auto d : done) reads += d;
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : (double)all[(size_t)(p * (all.size() - 1))]; };
    uint64_t st[3];
    CK(stage_reader_stats(r, st));
    CK(stage_reader_destroy(r));

    // ---- mode host (pinned buffers, batches of `batch`)
    uint64_t *hk = nullptr;
    stage_probe_out *ho = nullptr;
    uint8_t *hr = nullptr;
    CK(stage_host_alloc(batch * 8, (void **)&hk));
    CK(stage_host_alloc(batch * sizeof(stage_probe_out), (void **)&ho));
    CK(stage_host_alloc(batch * stride, (void **)&hr));
    for (uint64_t i = 0; i < batch; ++i) hk[i] = keys[i % threads][(i / threads) % per_thread];
    CK(stage_probe_host(t, hk, nullptr, nullptr, batch, ho, hr));  // warm
    uint64_t host_ops = 0;
    t0 = clk::now();
    double t_host = 0;
    while (t_host < seconds) {
        CK(stage_probe_host(t, hk, nullptr, nullptr, batch, ho, hr));
        host_ops += batch;
        t_host = std::chrono::duration<double>(clk::now() - t0).count();
    }
    uint64_t host_bad = 0;
    for (uint64_t i = 0; i < batch; ++i)
        if (ho[i].status != STAGE_ST_LATEST || std::memcmp(hr + i * stride, &hk[i], 8)) ++host_bad;
    stage_host_free(hk);
    stage_host_free(ho);
    stage_host_free(hr);
    CK(stage_table_destroy(t));

    std::printf(
        "{\"rows\": %llu, \"theta\": %.2f, \"setup_s\": %.1f, \"reader\": {\"kind\": \"%s\", \"waves\": %u, "
        "\"threads\": %d, \"max_batch\": %u, "
        "\"max_wait_us\": %u, \"reads\": %llu, \"seconds\": %.2f, \"reads_per_s\": %.1f, \"batches\": %llu, "
        "\"avg_batch\": %.1f, \"full_batches\": %llu, \"lat_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f}, "
        "\"bad\": %llu}, \"probe_host\": {\"batch\": %llu, "
        "\"lookups\": %llu, \"seconds\": %.2f, \"lookups_per_s\": %.1f, \"bytes_back_per_lookup\": %u, "
        "\"bad\": %llu}}\n",
        (unsigned long long)rows, theta, t_setup, resident_waves ? "resident" : "coalescing", resident_waves, threads,
        max_batch, max_wait, (unsigned long long)reads, t_reader, reads / t_reader, (unsigned long long)st[0],
        st[0] ? (double)st[1] / st[0] : 0.0, (unsigned long long)st[2], pct(0.5), pct(0.9), pct(0.99),
        (unsigned long long)bad.load(), (unsigned long long)batch, (unsigned long long)host_ops, t_host,
        host_ops / t_host, (unsigned)(32 + stride), (unsigned long long)host_bad);
    return bad.load() || host_bad ? 1 : 0;
}
