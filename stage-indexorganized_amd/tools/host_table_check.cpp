// host_table_check.cpp -- host-code sanitizer driver for the host table (csrc/host_table.cpp):
// a randomized single-writer workload (inserts with leaf splits, updates, commits, finalizes,
// deletes, aborted updates and inserts, batched epochs, leaf-image export/import, location
// resolution) over three geometries (variable-length keys in 4 KiB leaves, 8-byte keys in
// 64 KiB leaves, 32-byte keys), checked against a std::map model of which keys are present.
// Built with -fsanitize=address,undefined by `make -C csrc check_host` (CPU only, no HIP).
//   host_table_check [ops=200000] [seed=1]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "../csrc/host_table.hpp"

using stage::HostTable;

static int fails = 0;
#define CHECK(c, ...)                                    \
    do {                                                 \
        if (!(c)) {                                      \
            if (fails++ < 20) {                          \
                std::fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
                std::fprintf(stderr, __VA_ARGS__);       \
                std::fprintf(stderr, "\n");              \
            }                                            \
        }                                                \
    } while (0)

struct Geo {
    const char *name;
    stage_params p;
    uint32_t klen;  // 0 = variable 1..8
};

static std::string make_key(std::mt19937_64 &rng, const Geo &g, uint64_t space) {
    const uint64_t v = rng() % space;
    const uint32_t len = g.klen ? g.klen : 1 + (uint32_t)(v % 8);
    std::string k(len, '\0');
    for (uint32_t i = 0; i < len; ++i) k[i] = (char)((v >> (8 * (i % 8))) ^ (i * 0x3B));
    return k;
}

static void run(const Geo &g, uint64_t ops, uint64_t seed) {
    HostTable t(g.p);
    std::mt19937_64 rng(seed);
    std::map<std::string, int> model;  // key -> 1 present (committed), 2 in-flight update
    std::vector<uint8_t> payload(g.p.payload_size);
    uint32_t tid = 10;
    const uint64_t space = ops / 2 + 16;
    for (uint64_t i = 0; i < ops; ++i) {
        const std::string k = make_key(rng, g, space);
        const auto *kb = reinterpret_cast<const uint8_t *>(k.data());
        const uint32_t kl = (uint32_t)k.size();
        const int op = (int)(rng() % 100);
        auto it = model.find(k);
        if (op < 45) {
            for (auto &b : payload) b = (uint8_t)rng();
            const int rc = t.insert(kb, kl, payload.data(), 0, 0, ++tid);
            if (it == model.end()) {
                CHECK(rc == STAGE_RC_OK, "%s insert rc=%d", g.name, rc);
                if (rc == STAGE_RC_OK) model[k] = 1;
            } else {
                CHECK(rc != STAGE_RC_OK, "%s insert of a present key rc=%d", g.name, rc);
            }
        } else if (op < 70) {
            uint8_t d[4] = {(uint8_t)i, 1, 2, 3};
            const int rc = t.update(kb, kl, 0, d, 4, ++tid);
            if (it == model.end()) {
                CHECK(rc != STAGE_RC_OK, "%s update of an absent key rc=%d", g.name, rc);
            } else if (rc == STAGE_RC_OK) {
                const int c = (int)(rng() % 3);
                if (c == 0) CHECK(t.commit_update(kb, kl, ++tid, tid) == STAGE_RC_OK, "%s commit", g.name);
                else if (c == 1) CHECK(t.abort_update(kb, kl) == STAGE_RC_OK, "%s abort_update", g.name);
                else CHECK(t.finalize_update(kb, kl, ++tid) == STAGE_RC_OK, "%s finalize", g.name);
            }
        } else if (op < 82) {
            const int rc = t.remove(kb, kl, ++tid);
            // RC_INVALID: deleted, and the leaf is below merge_threshold (merge not restated)
            if (it != model.end() && (rc == STAGE_RC_OK || rc == STAGE_RC_INVALID)) model.erase(it);
            if (it == model.end()) CHECK(rc != STAGE_RC_OK, "%s remove of an absent key rc=%d", g.name, rc);
        } else if (op < 84) {
            // insert then abort it (the aborted insert is its leaf's last slot right after insert)
            if (it == model.end()) {
                for (auto &b : payload) b = (uint8_t)rng();
                if (t.insert(kb, kl, payload.data(), 0, 0, ++tid) == STAGE_RC_OK) {
                    const int rc = t.abort_insert(kb, kl);
                    if (rc != STAGE_RC_OK) model[k] = 1;  // not its leaf's last slot: still present
                }
            }
        } else if (op < 86 && g.klen == 8 && !std::getenv("NO_BATCH")) {
            // a batched epoch over present keys, some twice
            std::vector<uint64_t> keys;
            for (auto &kv : model) {
                if (keys.size() >= 64) break;
                if (rng() % 4 == 0) {
                    uint64_t w = 0;
                    std::memcpy(&w, kv.first.data(), 8);
                    keys.push_back(w);
                    if (rng() % 3 == 0) keys.push_back(w);
                }
            }
            const uint64_t n = keys.size();
            std::vector<uint8_t> deltas(n * 8, 7), rcs(n);
            std::vector<uint32_t> wid(n), cid(n);
            for (uint64_t j = 0; j < n; ++j) wid[j] = ++tid, cid[j] = ++tid;
            t.update_batch(reinterpret_cast<const uint8_t *>(keys.data()), 8, n, 8, 0, deltas.data(), 8, wid.data(),
                           cid.data(), nullptr, rcs.data());
        } else if (op < 88) {
            uint32_t leaf, slot;
            CHECK((t.find(kb, kl, &leaf, &slot) >= 0) == (it != model.end()), "%s find", g.name);
        }
        if (std::getenv("TRACE")) {  // the touched key agrees with the model after every op
            uint32_t leaf, slot;
            const bool f = t.find(kb, kl, &leaf, &slot) >= 0, m = model.count(k) != 0;
            if (f != m) {
                std::fprintf(stderr, "op %llu kind %d: found %d model %d\n", (unsigned long long)i, op, f, m);
                return;
            }
        }
    }
    // every model key is found, locations resolve onto the key's slot
    for (auto &kv : model) {
        uint32_t leaf, slot;
        CHECK(t.find(reinterpret_cast<const uint8_t *>(kv.first.data()), (uint32_t)kv.first.size(), &leaf, &slot) >=
                  0,
              "%s final find", g.name);
    }
    const uint64_t nloc = t.export_locations(0, nullptr, nullptr, nullptr);
    std::vector<uint64_t> h(nloc);
    std::vector<uint32_t> lf(nloc), lf2(nloc);
    std::vector<uint16_t> sl(nloc), sl2(nloc);
    t.export_locations(nloc, h.data(), lf.data(), sl.data());
    t.resolve_locations(h.data(), nloc, lf2.data(), sl2.data());
    for (uint64_t i = 0; i < nloc; ++i) CHECK(lf[i] == lf2[i] && sl[i] == sl2[i], "%s location %llu", g.name,
                                              (unsigned long long)i);
    // leaf-image round trip into a fresh table
    uint64_t st[8] = {0};
    t.stats(st);
    const uint64_t nl = st[2];
    std::vector<uint8_t> blocks(nl * g.p.leaf_node_size);
    std::vector<uint64_t> seps(nl * t.key_words());  // key_words() u64 words per separator
    std::vector<uint16_t> seplen(nl);
    const int64_t got = t.export_leaf_images(nl, blocks.data(), seps.data(), seplen.data());
    CHECK(got == (int64_t)nl, "%s export %lld of %llu", g.name, (long long)got, (unsigned long long)nl);
    if (g.klen <= 8) {
        HostTable u(g.p);
        const uint64_t nrec = u.import_leaf_images(blocks.data(), nl, g.p.leaf_node_size, seps.data(), seplen.data());
        CHECK(nrec >= model.size(), "%s import %llu records < %zu", g.name, (unsigned long long)nrec, model.size());
        for (auto &kv : model) {
            uint32_t leaf, slot;
            CHECK(u.find(reinterpret_cast<const uint8_t *>(kv.first.data()), (uint32_t)kv.first.size(), &leaf,
                         &slot) >= 0,
                  "%s imported find", g.name);
        }
    }
    std::printf("%s: %llu ops, %zu keys, %llu leaves, %llu locations\n", g.name, (unsigned long long)ops,
                model.size(), (unsigned long long)nl, (unsigned long long)nloc);
}

int main(int argc, char **argv) {
    const uint64_t ops = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 200000;
    const uint64_t seed = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1;
    const Geo geos[] = {
        {"varlen-4k", {3072, 1024, 4096, 8, 0, 0}, 0},
        {"u64-64k", {16 * 1024, 32 * 1024, 64 * 1024, 1000, 8, 0}, 8},
        {"key32", {16 * 1024, 32 * 1024, 64 * 1024, 60, 32, 0}, 32},
    };
    for (const Geo &g : geos) run(g, ops, seed);
    std::printf(fails ? "host_table_check: %d failures\n" : "host_table_check: ok\n", fails);
    return fails ? 1 : 0;
}
