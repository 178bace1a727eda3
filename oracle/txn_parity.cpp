// txn_parity.cpp -- TEST INFRASTRUCTURE ONLY: the kept transaction manager (ssn_txn.hpp, a
// restatement of src/concurrency/transaction_manager.cpp) driven by device probe results through
// the reference-side adapter (include/stage_btree_adapter.hpp) over the C-ABI, against the same
// manager driven by the oracle (stage_oracle.c).  Both runs follow one seeded schedule of
// concurrent YCSB-style transactions (reads and 100-B column updates of a hot key set, commits
// split into commit id and the rest, explicit aborts, bursts of committed inserts that split the
// leaves holding hot records between a transaction's reads and its commit); every step's facts
// and outcome and, at the end, every transaction, overwrite-copy header (stamps, readers, count)
// and RecordLocation cell must be equal.
//
//   txn_parity oracle|device|both SEED [ROWS] [TXNS]
//       oracle / device: one run, its trace on stdout; both: the two runs compared -- prints
//       "MATCH" and the coverage summary (exit 0) or the first differing line (exit 1)
//   txn_parity sched oracle|device|both < SCHEDULES
//       the reference's TransactionScheduler tests (testing_transaction_util.h:142-440) whose ops
//       are point reads, point updates, commits and aborts, run through the same manager: one
//       "txn" line per transaction (txn_result and the read results) per schedule, for the test
//       to hold against the reference's own assertions (tests/golden/make_scenarios.py); both =
//       the two stores' traces must also be equal.  Input, one directive a line:
//         schedule NAME | table new N | table same | tick N
//         op TXN read KEY FU | op TXN update KEY VALUE FU | op TXN commit | op TXN abort | end
#include <algorithm>
#include <cstdio>
#include <iostream>
#include <map>
#include <memory>
#include <stdexcept>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../include/stage_btree_adapter.hpp"
#include "../include/stage_hip.h"
#include "ssn_txn.hpp"
#include "stage_oracle.h"

namespace {

constexpr uint32_t kPayload = 1000, kDelta = 100, kKey = 8;

// ParameterSet (b_tree.h:23-40): YCSB's (ycsb.cpp:72) and CreateTable's (testing_transaction_util.cpp:31)
struct Geometry {
    uint32_t split, merge, leaf, payload;
};
constexpr Geometry kYcsb{16 * 1024, 0, 64 * 1024, kPayload};
// CreateTable's 64 KiB leaves of 8-B payloads hold 1637 records, above the device layout's 1024
// slots: both backends run 32 KiB leaves (as tests/scenarios.py geometry()); the schedules hold
// 10-11 rows, so no leaf splits in either geometry
constexpr Geometry kTestTable{32 * 1024, 16 * 1024, 32 * 1024, 8};

inline uint64_t word_at(const uint8_t *p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

#define CK(x)                                                                             \
    do {                                                                                  \
        int rc_ = (x);                                                                    \
        if (rc_) {                                                                        \
            std::fprintf(stderr, "%s failed: rc=%d %s\n", #x, rc_, stage_last_error()); \
            std::exit(3);                                                                 \
        }                                                                                 \
    } while (0)

// ---- the oracle as the manager's store
struct OracleStore {
    orc_tree *t = nullptr;
    std::vector<uint8_t> rec;
    explicit OracleStore(uint64_t rows) : OracleStore(kYcsb) { orc_load_ycsb(t, 0, rows, kKey, 0); }
    explicit OracleStore(const Geometry &g) : rec(8 + g.payload) {
        t = orc_tree_new(g.leaf, g.split, g.payload);
        if (g.merge) orc_tree_set_merge_threshold(t, g.merge);
    }
    // TestingTransactionUtil::CreateTable: keys 0..n-1, value 0, one committed transaction
    void create_table(uint32_t n, uint32_t cid) {
        std::vector<uint8_t> pay(rec.size() - 8, 0);
        for (uint64_t k = 0; k < n; ++k) orc_insert(t, (const uint8_t *)&k, kKey, pay.data(), cid);
    }
    ~OracleStore() { orc_tree_free(t); }
    ssn::ReadFacts read(uint64_t key, uint32_t rid, bool fu) {
        orc_read_out o;
        if (fu) {  // the manager takes no record facts from a for-update read
            orc_read_fu(t, (const uint8_t *)&key, kKey, rid, 1, &o, rec.data());
            return ssn::ReadFacts{o.status, o.cstamp, 0, 0, 0, word_at(rec.data() + 8)};
        }
        uint64_t m;
        uint32_t loc, nx;
        orc_read_ident(t, (const uint8_t *)&key, kKey, rid, &o, rec.data(), &m, &loc, &nx);
        return ssn::ReadFacts{o.status, o.cstamp, m, loc, nx, word_at(rec.data() + 8)};
    }
    bool header(uint32_t id, ssn::Hdr &h) {
        uint32_t st[7];
        if (orc_copy_state(t, id, st) != 0) return false;
        h.cstamp = st[0], h.pstamp = st[1], h.rstamp = st[2], h.sstamp = st[3];
        h.count = (uint16_t)st[5], h.waiting = (uint8_t)st[6];
        h.readers.resize(st[4]);
        if (st[4]) orc_copy_readers(t, id, h.readers.data(), st[4]);
        return true;
    }
    void add_reader(uint32_t id, uint32_t rid) { orc_copy_add_reader(t, id, rid); }
    int wr_count(uint32_t id, int d) { return orc_copy_wr_count(t, id, d) > 0 ? 1 : 0; }
    void update_ps(uint32_t id, uint32_t ps) { orc_copy_update_ps(t, id, ps); }
    void location(uint32_t loc, uint64_t &meta, uint32_t &next) { orc_location_meta(t, loc, &meta, &next); }
    int update(uint64_t key, const std::vector<uint8_t> &d, bool fu, uint32_t writer, ssn::RecordMeta &upt) {
        if (fu) return orc_update_owned(t, (const uint8_t *)&key, kKey, 0, d.data(), (uint32_t)d.size(), writer);
        const int rc = orc_update(t, (const uint8_t *)&key, kKey, 0, d.data(), (uint32_t)d.size(), writer);
        if (rc == 1) {
            uint32_t loc, nx;
            orc_record_meta(t, (const uint8_t *)&key, kKey, &upt.meta, &loc, &nx);
            upt.loc_ptr = loc, upt.next_ptr = nx;
        }
        return rc;
    }
    int commit_update(uint64_t key, uint32_t cid, uint32_t ss) {
        return orc_commit_update(t, (const uint8_t *)&key, kKey, cid, ss);
    }
    int abort_update(uint64_t key) { return orc_abort_update(t, (const uint8_t *)&key, kKey); }
    void insert_burst(const std::vector<uint64_t> &keys) {
        std::vector<uint8_t> pay(kPayload);
        for (uint64_t k : keys) {
            orc_fill_payload(k, 0, pay.data(), kPayload);
            orc_insert(t, (const uint8_t *)&k, kKey, pay.data(), 0);
        }
    }
    // (leaf index in key order, slot) of a location, 0xFFFFFFFF when dropped
    uint64_t where(uint32_t loc) {
        uint64_t h = loc;
        uint32_t leaf;
        uint16_t slot;
        orc_resolve_locations(t, &h, 1, &leaf, &slot);
        return (uint64_t)leaf << 16 | slot;
    }
    uint64_t locations() { return orc_location_count(t); }
};

// ---- the device path as the manager's store: probes on the GPU, the Record framed by the
// adapter, the location deref and the pool through the adapter's LocationTable / OverwritePool
struct DeviceStore {
    stage_table *t = nullptr;
    stage_adapter::LocationTable *locs = nullptr;
    stage_adapter::OverwritePool *pool = nullptr;
    void *dk = nullptr, *dr = nullptr, *dout = nullptr, *did = nullptr, *drow = nullptr, *dfu = nullptr;
    uint32_t stride = 0;
    std::vector<uint8_t> row;
    explicit DeviceStore(uint64_t rows) : DeviceStore(kYcsb) {
        uint64_t n = 0;
        CK(stage_load_ycsb(t, 0, rows, kKey, 0, &n));
        ready();
    }
    explicit DeviceStore(const Geometry &g) {
        stage_params p{g.split, g.merge ? g.merge : 32 * 1024, g.leaf, g.payload, kKey, 0};
        CK(stage_table_create(&p, &t));
    }
    void create_table(uint32_t n, uint32_t cid) {
        std::vector<uint8_t> pay(stage_record_stride(t), 0);
        for (uint64_t k = 0; k < n; ++k) {
            uint8_t rc;
            CK(stage_insert(t, k, kKey, pay.data(), 0, 0, cid, &rc));
        }
        ready();
    }
    void ready() {  // after the load: location cells, the first publish, the adapter's views
        CK(stage_location_cells(t));
        CK(stage_sync(t));
        locs = new stage_adapter::LocationTable(t);
        pool = new stage_adapter::OverwritePool(t);
        stride = stage_record_stride(t);
        row.resize(stride);
        CK(stage_dev_alloc(8, &dk));
        CK(stage_dev_alloc(4, &dr));
        CK(stage_dev_alloc(32, &dout));
        CK(stage_dev_alloc(8, &did));
        CK(stage_dev_alloc(stride, &drow));
        CK(stage_dev_alloc(1, &dfu));
    }
    ~DeviceStore() {
        for (void *p : {dk, dr, dout, did, drow, dfu})
            if (p) stage_dev_free(p);
        delete pool;
        delete locs;
        stage_table_destroy(t);
    }
    ssn::ReadFacts read(uint64_t key, uint32_t rid, bool fu) {
        const uint8_t f = fu ? 1 : 0;
        CK(stage_memcpy_h2d(dk, &key, 8, nullptr));
        CK(stage_memcpy_h2d(dr, &rid, 4, nullptr));
        CK(stage_memcpy_h2d(dfu, &f, 1, nullptr));
        CK(stage_probe_batch_ex(t, (const uint64_t *)dk, nullptr, (const uint32_t *)dr, nullptr, (const uint8_t *)dfu, 1,
                                (stage_probe_out *)dout, (uint8_t *)drow, nullptr));
        if (!fu) CK(stage_probe_identify(t, (const stage_probe_out *)dout, 1, (stage_probe_ident *)did, nullptr));
        CK(stage_device_sync());  // the probe ran on the table's stream, the copies use the null stream
        stage_probe_out o;
        stage_probe_ident id;
        CK(stage_memcpy_d2h(&o, dout, 32, nullptr));
        CK(stage_memcpy_d2h(row.data(), drow, stride, nullptr));
        last = o;
        const uint64_t value = word_at(row.data() + 8);
        if (fu) return ssn::ReadFacts{o.status, o.cstamp, 0, 0, 0, value};
        CK(stage_memcpy_d2h(&id, did, 8, nullptr));
        if (o.status == STAGE_ST_NOT_FOUND) return ssn::ReadFacts{o.status, o.cstamp, 0, 0, 0, value};
        // the RecordMeta BTree::Read hands the executor, framed by the adapter; its loc_ptr is
        // the facade's RecordLocation, mapped back to the handle for the manager's rw-set key
        stage_adapter::RecordLocation *rl = locs->get(id.loc);
        const stage_adapter::RecordMeta rm =
            stage_adapter::record_meta(o, id, reinterpret_cast<uint64_t>(rl), kPayload);
        const uint32_t loc = (uint32_t)stage_adapter::LocationTable::handle_of(
            reinterpret_cast<const stage_adapter::RecordLocation *>(rm.meta_data.loc_ptr));
        return ssn::ReadFacts{o.status, rm.cstamp, rm.meta_data.meta, loc, (uint32_t)rm.meta_data.next_ptr, value};
    }
    bool header(uint32_t id, ssn::Hdr &h) {
        stage_adapter::OverwriteHeader oh;
        if (!pool->GetOversionHeader(STAGE_NEXT_COPY | id, oh)) return false;
        h.cstamp = oh.cstamp, h.pstamp = oh.pstamp, h.rstamp = oh.rstamp, h.sstamp = oh.sstamp;
        h.count = oh.count, h.waiting = oh.waiting;
        h.readers = oh.readers;
        return true;
    }
    void add_reader(uint32_t id, uint32_t rid) { pool->AddReader(STAGE_NEXT_COPY | id, rid); }
    int wr_count(uint32_t id, int d) {
        if (d > 0) return pool->IncreaseWRCount(STAGE_NEXT_COPY | id) ? 1 : 0;
        pool->DecreaseWRCount(STAGE_NEXT_COPY | id);
        return 1;
    }
    void update_ps(uint32_t id, uint32_t ps) { pool->UpdatePs(STAGE_NEXT_COPY | id, ps); }
    // `reinterpret_cast<RecordMetadata *>(loc->record_meta_ptr)`, as the manager dereferences it
    void location(uint32_t loc, uint64_t &meta, uint32_t &next) {
        const stage_adapter::RecordMetadata *m = stage_adapter::LocationTable::record_meta(locs->get(loc));
        meta = m->meta;
        next = (uint32_t)m->next_ptr;
    }
    int update(uint64_t key, const std::vector<uint8_t> &d, bool fu, uint32_t writer, ssn::RecordMeta &upt) {
        uint8_t rc = 0;
        if (fu) {
            CK(stage_update_key_owned(t, (const uint8_t *)&key, kKey, 0, d.data(), (uint32_t)d.size(), writer, &rc));
            CK(stage_sync(t));
            return rc;
        }
        CK(stage_update_key(t, (const uint8_t *)&key, kKey, 0, d.data(), (uint32_t)d.size(), writer, &rc));
        if (rc == STAGE_RC_OK) {
            stage_probe_ident id;
            uint8_t r2;
            CK(stage_record_meta_key(t, (const uint8_t *)&key, kKey, &upt.meta, &id, &r2));
            upt.loc_ptr = id.loc, upt.next_ptr = id.next;
        }
        CK(stage_sync(t));
        return rc;
    }
    int commit_update(uint64_t key, uint32_t cid, uint32_t ss) {
        uint8_t rc = 0;
        CK(stage_commit_update_key(t, (const uint8_t *)&key, kKey, cid, ss, &rc));
        CK(stage_sync(t));
        return rc;
    }
    int abort_update(uint64_t key) {
        uint8_t rc = 0;
        CK(stage_abort_update_key(t, (const uint8_t *)&key, kKey, &rc));
        CK(stage_sync(t));
        return rc;
    }
    void insert_burst(const std::vector<uint64_t> &keys) {
        for (uint64_t k : keys) {
            uint8_t rc;
            CK(stage_insert(t, k, kKey, nullptr, k, 0, 0, &rc));
        }
        CK(stage_sync(t));
    }
    uint64_t where(uint32_t loc) {
        uint64_t h = loc;
        uint32_t leaf;
        uint16_t slot;
        CK(stage_resolve_locations(t, &h, 1, &leaf, &slot));
        return (uint64_t)leaf << 16 | slot;
    }
    stage_probe_out last{};
};

uint64_t g_locations = 0;  // the oracle's location count: both runs dump the same handles
template <class Store>
uint64_t st_locations(Store &) {
    return g_locations;
}

struct Run {
    std::string trace;
    ssn::Stats stats;
    uint64_t moved = 0;  // READ entries whose record a split moved between the read and the commit
    uint64_t copy_reader_commits = 0;  // writers committed over a copy that had registered readers
};

template <class Store>
Run run(Store &st, uint32_t seed, uint64_t rows, uint32_t ntx) {
    ssn::Manager<Store> m(st);
    std::mt19937_64 rng(seed);
    auto uni = [&](uint64_t n) { return (uint64_t)(rng() % n); };
    auto chance = [&](double p) { return (double)(rng() % 1000000) < p * 1e6; };
    const uint64_t hot = 48;
    struct Live {
        ssn::Txn *t;
        int ops_left;
        bool committing;
        std::vector<std::pair<uint32_t, uint64_t>> reads;  // (location, where at read time)
    };
    std::vector<Live> live;
    uint32_t started = 0;
    uint64_t fresh = rows + 4096, moved = 0, copy_reader_commits = 0;
    std::set<uint32_t> seen_copies;
    for (uint64_t step = 0; started < ntx || !live.empty(); ++step) {
        if (step > 200000) {
            std::fprintf(stderr, "schedule did not finish\n");
            std::exit(4);
        }
        // a burst of committed inserts beside a hot key: its leaf (and neighbours) split
        if (step % 37 == 36) {
            const uint64_t h = uni(hot);
            std::vector<uint64_t> keys;
            for (int i = 0; i < 48; ++i) keys.push_back((fresh++ << 8) | h);  // same low byte as the hot key
            st.insert_burst(keys);
            m.log += "insert_burst around key " + std::to_string(h) + "\n";
            continue;
        }
        if (started < ntx && live.size() < 5 && (live.empty() || chance(0.3))) {
            live.push_back(Live{m.begin(), 1 + (int)uni(5), false, {}});
            ++started;
            continue;
        }
        const size_t k = uni(live.size());
        Live &L = live[k];
        bool done = false;
        if (L.committing) {
            if (m.would_block(L.t)) {
                bool any = false;  // someone else must be able to move
                for (const Live &o : live) any |= !o.committing || !m.would_block(o.t);
                if (!any) {
                    std::fprintf(stderr, "deadlock in the schedule\n");
                    std::exit(4);
                }
                continue;
            }
            uint64_t mv = 0;
            for (auto &r : L.reads) mv += st.where(r.first) != r.second;
            for (const ssn::Entry &e : L.t->rw) {
                ssn::Hdr h;
                uint64_t meta;
                uint32_t nx;
                st.location(e.rm.loc_ptr, meta, nx);
                if (e.type == ssn::RW::UPDATE && (nx & ssn::kKindMask) == ssn::kCopy && st.header(nx & ssn::kIndexMask, h) &&
                    !h.readers.empty())
                    ++copy_reader_commits;
            }
            m.log += "moved_since_read=" + std::to_string(mv) + "\n";
            moved += mv;
            m.finish_commit(L.t);
            done = true;
        } else if (L.ops_left > 0) {
            // hot keys, the rest of the table, now and then a key that is not there
            const uint64_t key = chance(0.75) ? uni(hot) : uni(rows + rows / 16);
            bool ok;
            if (chance(0.35)) {
                ok = m.update(L.t, key, std::vector<uint8_t>(kDelta, (uint8_t)uni(256)));
            } else {
                ok = m.read(L.t, key, false);
                if (ok && !L.t->rw.empty()) {
                    const uint32_t loc = L.t->rw.back().rm.loc_ptr;
                    if (loc) L.reads.emplace_back(loc, st.where(loc));
                }
            }
            --L.ops_left;
            if (!ok) {  // the executor failed: RunMixed aborts (ycsb_mixed.cpp:62-68, 94-99)
                m.abort(L.t);
                done = true;
            }
        } else if (chance(0.04)) {
            m.abort(L.t);
            done = true;
        } else {
            m.begin_commit(L.t);
            L.committing = true;
        }
        if (done) live.erase(live.begin() + (long)k);
    }
    // the final state: transactions, overwrite-copy headers, location cells
    std::ostringstream os;
    for (const auto &t : m.txns())
        os << "txn " << t->id << " rid=" << t->read_id << " cid=" << t->commit_id << " pred=" << t->pred
           << " succ=" << t->succ << " result=" << (int)t->result << " aborted=" << t->aborted
           << " finished=" << t->finished << "\n";
    for (uint32_t id = 0;; ++id) {
        ssn::Hdr h;
        if (!st.header(id, h)) break;
        os << "copy " << id << " cstamp=" << h.cstamp << " pstamp=" << h.pstamp << " rstamp=" << h.rstamp
           << " sstamp=" << h.sstamp << " count=" << h.count << " waiting=" << (int)h.waiting << " readers=";
        for (uint32_t r : h.readers) os << r << ",";
        os << "\n";
    }
    for (uint32_t loc = 1; loc <= st_locations(st); ++loc) {
        uint64_t meta;
        uint32_t nx;
        st.location(loc, meta, nx);
        os << "loc " << loc << " meta=" << std::hex << meta << " next=" << nx << std::dec << "\n";
    }
    Run r;
    r.trace = m.log + os.str();
    r.stats = m.stats;
    r.moved = moved;
    r.copy_reader_commits = copy_reader_commits;
    return r;
}

void summary(const Run &r) {
    const ssn::Stats &s = r.stats;
    std::printf(
        "{\"reads\": %llu, \"reads_via_copy\": %llu, \"perform_read_fail\": %llu, \"updates_ok\": %llu, "
        "\"updates_failed\": %llu, \"commits\": %llu, \"commit_failures\": %llu, \"aborts\": %llu, "
        "\"min_sstamp_writers\": %llu, \"min_sstamp_inflight\": %llu, \"max_pstamp_readers\": %llu, "
        "\"max_pstamp_headers\": %llu, \"moved_between_read_and_commit\": %llu, \"copy_reader_commits\": %llu, "
        "\"trace_lines\": %llu}\n",
        (unsigned long long)s.reads, (unsigned long long)s.reads_via_copy, (unsigned long long)s.perform_read_fail,
        (unsigned long long)s.updates_ok, (unsigned long long)s.updates_failed, (unsigned long long)s.commits,
        (unsigned long long)s.commit_failures, (unsigned long long)s.aborts, (unsigned long long)s.min_sstamp_writers,
        (unsigned long long)s.min_sstamp_inflight, (unsigned long long)s.max_pstamp_readers,
        (unsigned long long)s.max_pstamp_headers, (unsigned long long)r.moved, (unsigned long long)r.copy_reader_commits,
        (unsigned long long)std::count(r.trace.begin(), r.trace.end(), '\n'));
}

// ---- the reference's TransactionScheduler tests (testing_transaction_util.h:142-440)
struct SOp {
    int txn;         // -1: a directive
    std::string op;  // read / update / commit / abort; table-new / table-same / tick
    uint64_t key = 0, value = 0;
    bool fu = false;
};
struct Sched {
    std::string name;
    std::vector<SOp> ops;
};

std::vector<Sched> parse_schedules(std::istream &in) {
    std::vector<Sched> out;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string w;
        if (!(ls >> w) || w[0] == '#') continue;
        if (w == "schedule") {
            out.emplace_back();
            ls >> out.back().name;
            continue;
        }
        if (out.empty()) throw std::runtime_error("directive before 'schedule': " + line);
        SOp o;
        o.txn = -1;
        if (w == "table") {
            std::string kind;
            ls >> kind;
            o.op = "table-" + kind;
            if (kind == "new") ls >> o.key;
        } else if (w == "tick") {
            o.op = "tick";
            ls >> o.key;
        } else if (w == "op") {
            int fu = 0;
            ls >> o.txn >> o.op;
            if (o.op == "read") ls >> o.key >> fu;
            else if (o.op == "update") ls >> o.key >> o.value >> fu;
            else if (o.op != "commit" && o.op != "abort") throw std::runtime_error("unknown op: " + line);
            o.fu = fu != 0;
        } else if (w == "end") {
            continue;
        } else {
            throw std::runtime_error("unknown directive: " + line);
        }
        out.back().ops.push_back(o);
    }
    return out;
}

// Runs every schedule in order; "table same" keeps the previous schedule's table and manager
// (the reference's tests that run several TransactionSchedulers over one table and one
// SSNTransactionManager).  The reference's driver runs one op at a time and waits for it; a
// commit that would spin in FindMinSstamp / FindMaxPstamp on a transaction of the same schedule
// is parked here and finished as soon as the state it waits for is reached (after the op that
// reaches it), which is the outcome the tests' assertions describe.
template <class Store>
std::string run_schedules(const std::vector<Sched> &ss, std::string &trace) {
    std::unique_ptr<Store> st;
    std::unique_ptr<ssn::Manager<Store>> m;
    std::ostringstream out;
    std::string all;  // every manager's trace
    for (const Sched &s : ss) {
        struct TS {
            ssn::Txn *t = nullptr;
            const char *result = "FAILURE";  // TransactionSchedule's initial txn_result (:150)
            std::vector<int64_t> results;
            bool parked = false;
        };
        std::map<int, TS> ts;
        std::vector<int> parked;
        auto finish = [&](int i) {
            ts[i].result = m->finish_commit(ts[i].t) == ssn::Result::SUCCESS ? "SUCCESS" : "FAILURE";
            ts[i].parked = false;
        };
        auto resume = [&] {
            for (bool moved = true; moved;) {
                moved = false;
                for (size_t k = 0; k < parked.size(); ++k)
                    if (!m->would_block(ts[parked[k]].t)) {
                        finish(parked[k]);
                        parked.erase(parked.begin() + (long)k);
                        moved = true;
                        break;
                    }
            }
        };
        for (const SOp &o : s.ops) {
            if (o.txn < 0) {
                if (o.op == "table-new") {
                    if (m) all += m->log;
                    m.reset();
                    st.reset(new Store(kTestTable));
                    st->create_table((uint32_t)o.key, 2);  // CreateTable's transaction: read id 1, commit id 2
                    m.reset(new ssn::Manager<Store>(*st, 3));
                } else if (o.op == "table-same") {
                    if (!m) throw std::runtime_error("table same without a table");
                } else if (o.op == "tick") {
                    m->tick((uint32_t)o.key);
                }
                continue;
            }
            TS &x = ts[o.txn];
            if (!x.t) x.t = m->begin();                         // cur_seq == 0 (:213-219)
            if (std::strcmp(x.result, "ABORTED") == 0) continue;  // (:221-224)
            if (o.op == "read") {
                int64_t v = -1;
                const bool ok = m->read(x.t, o.key, o.fu, &v);
                x.results.push_back(ok ? v : -2);  // -2: the executor failed (result unset)
            } else if (o.op == "update") {
                std::vector<uint8_t> d(8);
                std::memcpy(d.data(), &o.value, 8);
                m->update(x.t, o.key, d, o.fu);
            } else if (o.op == "abort") {
                m->abort_explicit(x.t);
                x.result = "ABORTED";
            } else {  // commit
                m->begin_commit(x.t);
                if (m->would_block(x.t)) {
                    x.parked = true;
                    parked.push_back(o.txn);
                    m->log += "parked T" + std::to_string(x.t->id) + "\n";
                } else {
                    finish(o.txn);
                }
            }
            // a failed executor: AbortTransaction, txn_result ABORTED (:302-308)
            if ((o.op == "read" || o.op == "update") && x.t->result == ssn::Result::FAILURE) {
                m->abort(x.t);
                x.result = "ABORTED";
            }
            resume();
        }
        if (m) m->log += "end of " + s.name + "\n";
        out << "schedule " << s.name << "\n";
        for (auto &kv : ts) {
            out << "txn " << kv.first << " result=" << (kv.second.parked ? "BLOCKED" : kv.second.result) << " results=";
            for (size_t i = 0; i < kv.second.results.size(); ++i) out << (i ? "," : "") << kv.second.results[i];
            out << "\n";
        }
    }
    trace = all + (m ? m->log : std::string());
    return out.str();
}

int sched_main(const std::string &mode) {
    const std::vector<Sched> ss = parse_schedules(std::cin);
    std::string ta, tb;
    const std::string a = run_schedules<OracleStore>(ss, ta);
    if (mode == "oracle" || mode == "oracle-trace") {
        std::fputs(a.c_str(), stdout);
        if (mode == "oracle-trace") std::fputs(ta.c_str(), stdout);
        return 0;
    }
    const std::string b = run_schedules<DeviceStore>(ss, tb);
    if (mode == "device") {
        std::fputs(b.c_str(), stdout);
        return 0;
    }
    if (a == b && ta == tb) {
        std::printf("MATCH\n");
        std::fputs(a.c_str(), stdout);
        return 0;
    }
    std::printf("MISMATCH\n--- oracle\n%s%s--- device\n%s%s", a.c_str(), ta.c_str(), b.c_str(), tb.c_str());
    return 1;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc >= 3 && std::string(argv[1]) == "sched") return sched_main(argv[2]);
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s oracle|device|both SEED [ROWS] [TXNS]\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    const uint32_t seed = (uint32_t)std::strtoul(argv[2], nullptr, 0);
    const uint64_t rows = argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 3000;
    const uint32_t ntx = argc > 4 ? (uint32_t)std::strtoul(argv[4], nullptr, 0) : 300;
    Run a, b;
    {
        OracleStore o(rows);
        // the dump covers the oracle's locations after the schedule: run it once to learn them
        g_locations = 0;
        a = run(o, seed, rows, ntx);
        g_locations = o.locations();
    }
    {
        OracleStore o(rows);  // rerun with the location dump sized
        a = run(o, seed, rows, ntx);
    }
    if (mode == "oracle") {
        std::fputs(a.trace.c_str(), stdout);
        summary(a);
        return 0;
    }
    {
        DeviceStore d(rows);
        b = run(d, seed, rows, ntx);
    }
    if (mode == "device") {
        std::fputs(b.trace.c_str(), stdout);
        summary(b);
        return 0;
    }
    if (a.trace == b.trace) {
        std::printf("MATCH\n");
        summary(a);
        return 0;
    }
    std::istringstream x(a.trace), y(b.trace);
    std::string lx, ly;
    for (uint64_t line = 1;; ++line) {
        const bool gx = (bool)std::getline(x, lx), gy = (bool)std::getline(y, ly);
        if (!gx && !gy) break;
        if (lx != ly || gx != gy) {
            std::printf("MISMATCH at line %llu\n  oracle: %s\n  device: %s\n", (unsigned long long)line,
                        gx ? lx.c_str() : "<end>", gy ? ly.c_str() : "<end>");
            break;
        }
    }
    summary(a);
    summary(b);
    return 1;
}
