// ssn_txn.hpp -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A restatement of the reference's Index-SSN transaction manager -- the subsystem the north star
// KEEPS on the host -- over an abstract record store, so that the facts the device path hands
// across the C-ABI can drive it and be compared with the same manager driven by the oracle:
//
//   BeginTransaction          src/concurrency/transaction_manager.cpp:280-309
//   PerformRead               :362-410   (RecordRead: transaction_context.cpp:88-99)
//   PerformUpdate             :435-491   (RecordUpdate: transaction_context.cpp:115-141)
//   FindMaxPstamp             :29-102    (the readers of the copy each UPDATE entry overwrote)
//   FindMinSstamp             :113-221   (the writers that overwrote each READ entry)
//   CommitTransaction         :535-815   (UPDATE entry :610-676, READ entry :749-764)
//   AbortTransaction          :825-1046  (UPDATE entry :850-924, READ entry :986-1000)
//   TransactionContext        include/execute/txn_context.h:83-164 (SetSuccessor = min,
//                             SetPredecessor = max, CheckExclusion = successor > predecessor)
//   BTree::Read's AddReader   src/vstore/b_tree.cpp:2087-2110 (a read served by the copy)
//   IndexScanExecutor         include/execute/executor.h:374-454 (point lookup)
//   PointUpdateExecutor       include/execute/executor.h:206-322
//
// What the manager reads from the store is exactly what the reference reads through a Record and
// the EphemeralPool: the Record's RecordMetadata {meta, next_ptr, loc_ptr} and cstamp, the
// location's CURRENT RecordMetadata (`GetLocationPtr()->record_meta_ptr`), the overwrite-copy
// header named by a next_ptr (stamps, readers, count, waiting) and its mutators.  next_ptr /
// loc_ptr are the C-ABI's handles (stage_hip.h STAGE_NEXT_*, location handles).
//
// The reference runs transactions on threads and spins where one waits for another
// (FindMaxPstamp :58-68, FindMinSstamp :165-175, :186-196).  Here the schedule is sequential:
// a commit is split into begin_commit (the commit id: tid_counter.fetch_add, SetCommitting) and
// finish_commit (the rest), and would_block() reports -- without side effects -- whether
// finish_commit would reach one of those spins with its condition false, so the scheduler runs
// something else first.  Ids start at 1 (the reference's tid_counter starts at INVALID_CID = 0,
// whose first transaction would share the id AbortTransaction files aborted contexts under).
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace ssn {

constexpr uint32_t kMaxCid = 0xFFFFFFFFu, kInvalidCid = 0;
constexpr uint32_t kKindMask = 0xC0000000u, kCopy = 0x40000000u, kIndexMask = 0x3FFFFFFFu;
constexpr uint64_t kControl = 1ull << 63, kVisible = 1ull << 62;
enum : uint8_t { ST_NOT_FOUND = 0, ST_LATEST = 1, ST_COPY = 2, ST_OLD = 3, ST_FAIL = 4, ST_CHAIN_MISS = 5 };

inline uint32_t cstamp_of(uint64_t meta) { return (uint32_t)meta; }
inline bool inserting(uint64_t meta) { return (meta & kVisible) && (meta & kControl); }

// BTree::Read + the IndexScanExecutor point-lookup outcome of one key, with the Record's
// RecordMetadata (meta word, next_ptr handle, loc_ptr handle) and cstamp
struct ReadFacts {
    uint8_t status;
    uint32_t cstamp;
    uint64_t meta;
    uint32_t loc, next;
    uint64_t value = 0;  // the tuple's first payload word (TestTuple::value, testing_transaction_util.h:82-92)
};

// EphemeralPool::OverwriteVersionHeader (ephemeral_pool.h:26-150)
struct Hdr {
    uint32_t cstamp, pstamp, rstamp, sstamp;
    uint16_t count;
    uint8_t waiting;
    std::vector<uint32_t> readers;
};

enum class RW : uint8_t { READ, UPDATE };
enum class Result : uint8_t { INVALID, SUCCESS, FAILURE, ABORTED };

struct RecordMeta {  // the rw-set key: hash on meta, equality on loc_ptr (txn_context.h:16-24,
    uint64_t meta;   // record_meta.h:248-251): an entry is found only when both agree
    uint32_t next_ptr, loc_ptr;
};

struct Entry {
    RecordMeta rm;
    RW type;
    uint64_t key;
};

struct Txn {
    uint32_t id = 0;  // creation order (for reports)
    uint32_t read_id = 0, commit_id = kInvalidCid;
    uint32_t pred = kInvalidCid, succ = kMaxCid;
    bool aborted = false, finished = false, committing = false;
    Result result = Result::INVALID;
    std::vector<Entry> rw;
    void set_succ(uint32_t s) { succ = s < succ ? s : succ; }
    void set_pred(uint32_t p) { pred = p > pred ? p : pred; }
    bool check() const { return succ > pred; }  // CheckExclusion
};

// Store (duck-typed):
//   ReadFacts read(uint64_t key, uint32_t read_id, bool for_update)
//                                                                -- no side effects on the pool
//   bool header(uint32_t copy_id, Hdr &out)                     -- GetOversionHeader by copy id
//   void add_reader(uint32_t copy_id, uint32_t read_id)          -- AddReader
//   int  wr_count(uint32_t copy_id, int delta)                   -- 1 ok, 0 refused (waiting)
//   void update_ps(uint32_t copy_id, uint32_t pstamp)            -- UpdatePs
//   void location(uint32_t loc, uint64_t &meta, uint32_t &next)  -- *record_meta_ptr now
//   int  update(uint64_t key, const std::vector<uint8_t> &delta, bool for_update, uint32_t writer,
//               RecordMeta &meta_upt)                            -- BTree::Update (ReturnCode)
//   int  commit_update(uint64_t key, uint32_t cid, uint32_t sstamp), abort_update(uint64_t key)
// what the run exercised (for coverage assertions; equal between stores when the traces are)
struct Stats {
    uint64_t reads = 0, reads_via_copy = 0, perform_read_fail = 0, updates_ok = 0, updates_failed = 0;
    uint64_t commits = 0, commit_failures = 0, aborts = 0;
    uint64_t min_sstamp_writers = 0;   // FindMinSstamp took a committed overwriter's successor
    uint64_t min_sstamp_inflight = 0;  // ... or an in-flight overwriter's (through the live copy)
    uint64_t max_pstamp_readers = 0;   // FindMaxPstamp took a finished reader's predecessor
    uint64_t max_pstamp_headers = 0;   // FindMaxPstamp read an overwritten copy's pstamp
};

template <class Store>
class Manager {
public:
    Stats stats;
    explicit Manager(Store &s, uint32_t first_tid = 1) : st_(s), counter_(first_tid) {}

    std::string log;  // one line per step: the trace two stores must agree on

    Txn *begin() {  // BeginTransaction
        txns_.emplace_back(new Txn);
        Txn *t = txns_.back().get();
        t->id = (uint32_t)txns_.size() - 1;
        t->read_id = counter_++;
        active_.emplace(t->read_id, t);
        emit("begin T%u read_id=%u", t->id, t->read_id);
        return t;
    }

    // IndexScanExecutor point lookup (executor.h:374-454) through BTree::Read; false = the
    // executor failed (the caller aborts the transaction).  *value: the tuple's value, -1 when
    // the executor produced none (ExecuteRead, testing_transaction_util.cpp:111-119).
    // is_for_update: BTree::Read's own-record branch (b_tree.cpp:2087 -- no copy, no AddReader)
    // and no PerformRead (executor.h:388)
    bool read(Txn *t, uint64_t key, bool for_update = false, int64_t *value = nullptr) {
        const ReadFacts f = st_.read(key, t->read_id, for_update);
        // BTree::Read served from the overwrite copy tracks the reader (b_tree.cpp:2087-2105)
        const bool via_copy =
            !for_update && inserting(f.meta) && (f.next & kKindMask) == kCopy && f.status != ST_NOT_FOUND;
        if (via_copy) st_.add_reader(f.next & kIndexMask, t->read_id);
        bool ok = true;
        int pr = -1;
        if (f.status == ST_LATEST || f.status == ST_COPY) {  // txn_id >= the record's cstamp
            if (!for_update) {
                pr = perform_read(t, RecordMeta{f.meta, f.next, f.loc}, f.cstamp) ? 1 : 0;
                ok = pr == 1;
            }
        } else if (f.status == ST_FAIL) {
            ok = false;
        }
        const bool tuple = f.status == ST_LATEST || f.status == ST_COPY || f.status == ST_OLD;
        if (value) *value = tuple ? (int64_t)f.value : -1;
        if (!ok) t->result = Result::FAILURE;
        stats.reads++;
        stats.reads_via_copy += via_copy;
        stats.perform_read_fail += pr == 0;
        emit("read T%u key=%llu fu=%d st=%u cstamp=%u meta=%016llx loc=%u next=%08x value=%llu via_copy=%d "
             "perform_read=%d ok=%d",
             t->id, (unsigned long long)key, (int)for_update, f.status, f.cstamp, (unsigned long long)f.meta, f.loc,
             f.next, (unsigned long long)(tuple ? f.value : 0), (int)via_copy, pr, (int)ok);
        return ok;
    }

    // PointUpdateExecutor (executor.h:206-322): BTree::Update, then PerformUpdate; a failure is
    // retried until retry_count > 5 -- the retries meet the transaction's own in-flight update
    // (Dirty), so a failed PerformUpdate ends the executor with FAILURE all the same.
    // is_for_update: the writer's own record, patched in place, no PerformUpdate (:246-256)
    bool update(Txn *t, uint64_t key, const std::vector<uint8_t> &delta, bool for_update = false) {
        RecordMeta upt{0, 0, 0};  // BTree::Update's meta_upt_ (b_tree.cpp:2153)
        const int rc = st_.update(key, delta, for_update, t->read_id, upt);
        bool ok = true;
        int pu = -1;
        if (rc == 1) {  // Ok
            if (!for_update) {
                pu = perform_update(t, upt, key) ? 1 : 0;
                ok = pu == 1;
            }
        } else if (rc != 7 && rc != 3) {  // not NotNeededUpdate / NotFound
            ok = false;
        }
        t->result = ok ? Result::SUCCESS : Result::FAILURE;
        (rc == 1 && ok ? stats.updates_ok : stats.updates_failed) += (rc == 1 || !ok);
        emit("update T%u key=%llu byte=%u len=%u fu=%d rc=%d perform_update=%d ok=%d", t->id, (unsigned long long)key,
             delta.empty() ? 0u : delta[0], (unsigned)delta.size(), (int)for_update, rc, pu, (int)ok);
        return ok;
    }

    // TXN_OP_ABORT (testing_transaction_util.h:271-279): the aborting transaction takes a counter
    // value as its commit id (GetNextCurrentTidCounter) before AbortTransaction
    void abort_explicit(Txn *t) {
        t->commit_id = counter_++;
        emit("abort_id T%u cid=%u", t->id, t->commit_id);
        abort(t);
    }

    // transactions outside the schedule that took counter values (begin / commit ids)
    void tick(uint32_t n) { counter_ += n; }

    void begin_commit(Txn *t) {  // CommitTransaction up to SetCommitting (:550-564)
        t->commit_id = counter_++;
        t->committing = true;
        emit("commit_id T%u cid=%u", t->id, t->commit_id);
    }

    // finish_commit would spin in FindMinSstamp / FindMaxPstamp on a transaction that has not
    // reached the state it waits for
    bool would_block(const Txn *t) { return scan(const_cast<Txn *>(t), true) < 0; }

    Result finish_commit(Txn *t) {  // CommitTransaction :566-814
        const uint32_t tc = t->commit_id;
        const bool mn = find_min_sstamp(t), mx = find_max_pstamp(t);
        if (!(mn && mx)) {
            t->aborted = true;  // SetAbort; the driver does not call AbortTransaction (ycsb_mixed.cpp:143-147)
            t->result = Result::FAILURE;
            stats.commit_failures++;
            emit("commit T%u FAILURE pred=%u succ=%u", t->id, t->pred, t->succ);
            return Result::FAILURE;
        }
        const uint32_t t_sstamp = t->succ;
        t->finished = true;  // SetFinish
        for (const Entry &e : t->rw) {
            if (e.type == RW::UPDATE) {  // :610-676
                const int rc = st_.commit_update(e.key, tc, t_sstamp);
                emit("  commit_update key=%llu rc=%d", (unsigned long long)e.key, rc);
            } else {  // READ :749-764: the snapshot's next_ptr
                Hdr h;
                if (header(e.rm.next_ptr, h)) {
                    const uint32_t id = e.rm.next_ptr & kIndexMask;
                    st_.update_ps(id, h.pstamp > tc ? h.pstamp : tc);
                    st_.wr_count(id, -1);
                }
            }
        }
        t->result = Result::SUCCESS;
        t->set_succ(t_sstamp);
        active_.emplace(tc, t);
        stats.commits++;
        emit("commit T%u SUCCESS cid=%u pred=%u succ=%u", t->id, tc, t->pred, t->succ);
        return Result::SUCCESS;
    }

    void abort(Txn *t) {  // AbortTransaction :825-1046
        t->aborted = true;
        t->result = Result::ABORTED;
        active_.emplace(t->commit_id, t);
        for (const Entry &e : t->rw) {
            if (e.type == RW::UPDATE) {
                const int rc = st_.abort_update(e.key);
                emit("  abort_update key=%llu rc=%d", (unsigned long long)e.key, rc);
            } else {
                Hdr h;
                if (header(e.rm.next_ptr, h)) st_.wr_count(e.rm.next_ptr & kIndexMask, -1);
            }
        }
        stats.aborts++;
        emit("abort T%u", t->id);
    }

    const std::vector<std::unique_ptr<Txn>> &txns() const { return txns_; }

private:
    template <class... A>
    void emit(const char *fmt, A... a) {
        char buf[512];
        std::snprintf(buf, sizeof buf, fmt, a...);
        log += buf;
        log += '\n';
    }

    Txn *find(uint32_t tid) {  // active_tids.Find
        auto it = active_.find(tid);
        return it == active_.end() ? nullptr : it->second;
    }

    bool header(uint32_t next_ptr, Hdr &h) {  // EphemeralPool::GetOversionHeader(next_ptr)
        if (next_ptr == 0 || (next_ptr & kKindMask) != kCopy) return false;
        return st_.header(next_ptr & kIndexMask, h);
    }

    Entry *rw_find(Txn *t, const RecordMeta &rm) {
        for (Entry &e : t->rw)
            if (e.rm.meta == rm.meta && e.rm.loc_ptr == rm.loc_ptr) return &e;
        return nullptr;
    }

    bool perform_read(Txn *t, const RecordMeta &rm, uint32_t cstamp) {  // :362-410
        if (rw_find(t, rm)) return true;  // RecordRead returns false: nothing more
        t->rw.push_back(Entry{rm, RW::READ, 0});
        t->set_pred(cstamp);
        Hdr h;
        if (header(rm.next_ptr, h)) {
            if (!st_.wr_count(rm.next_ptr & kIndexMask, +1)) return false;  // IncreaseWRCount refused
            if (h.sstamp != kMaxCid) t->set_succ(h.sstamp);
        }
        if (!t->check()) {
            t->aborted = true;  // SetAbort
            return false;
        }
        return true;
    }

    bool perform_update(Txn *t, const RecordMeta &rm, uint64_t key) {  // :435-491
        if (!inserting(rm.meta)) return false;
        Hdr h;
        if (!header(rm.next_ptr, h)) return false;
        bool fresh = false;
        if (Entry *e = rw_find(t, rm)) {  // RecordUpdate: READ -> UPDATE returns false
            if (e->type == RW::READ) e->type = RW::UPDATE, e->key = key;
        } else {
            t->rw.push_back(Entry{rm, RW::UPDATE, key});
            fresh = true;
        }
        if (fresh) {
            t->set_pred(h.pstamp);
            if (!t->check()) {
                t->aborted = true;
                return false;
            }
        }
        return true;
    }

    bool find_min_sstamp(Txn *t) { return scan(t, false) > 0 ? true : false; }

    // FindMinSstamp (dry = only report a spin: -1) -- returns 1 / 0 for result_ true / false
    int scan(Txn *t, bool dry) {
        const uint32_t tc = t->commit_id;
        bool res = true;
        if (!dry) t->set_succ(tc);
        for (const Entry &e : t->rw) {
            if (e.type != RW::READ) continue;
            uint64_t cur;
            uint32_t cur_next;
            st_.location(e.rm.loc_ptr, cur, cur_next);
            const uint32_t meta_c = cstamp_of(e.rm.meta), curr_c = cstamp_of(cur);
            if (curr_c != meta_c && curr_c < tc) {  // overwritten and committed before us
                if (curr_c == kInvalidCid) continue;
                Txn *u = find(curr_c);
                if (!u || u->aborted) continue;
                if (!dry) {
                    t->set_succ(u->succ);
                    stats.min_sstamp_writers++;
                    if (!t->check()) res = false;
                }
            } else {  // being overwritten now?
                Hdr h;
                if (!header(cur_next, h)) continue;
                Txn *u = find(h.cstamp);
                if (!u || u->commit_id == tc || u->aborted) continue;
                if (u->commit_id == kInvalidCid) {  // spins until the writer has a commit id
                    if (dry) return -1;
                    continue;
                }
                if (u->commit_id < tc) {
                    if (!u->finished && !u->aborted) {  // spins until it finished or aborted
                        if (dry) return -1;
                        continue;
                    }
                    if (u->finished && !dry) {
                        t->set_succ(u->succ);
                        stats.min_sstamp_inflight++;
                        if (!t->check()) res = false;
                    }
                }
            }
        }
        if (dry) {  // FindMaxPstamp's spin: a reader of an overwritten copy without a commit id
            for (const Entry &e : t->rw) {
                if (e.type != RW::UPDATE) continue;
                uint64_t m;
                uint32_t nx;
                st_.location(e.rm.loc_ptr, m, nx);
                Hdr h;
                if (!header(nx, h)) continue;
                for (uint32_t rd : h.readers) {
                    Txn *r = find(rd);
                    if (!r || r->commit_id == tc || r->aborted) continue;
                    if (r->commit_id == kInvalidCid) return -1;
                }
            }
        }
        return res ? 1 : 0;
    }

    bool find_max_pstamp(Txn *t) {  // :29-102
        const uint32_t tc = t->commit_id;
        bool res = true;
        for (const Entry &e : t->rw) {
            if (e.type != RW::UPDATE) continue;
            uint64_t m;
            uint32_t nx;
            st_.location(e.rm.loc_ptr, m, nx);
            Hdr h;
            if (!header(nx, h)) continue;
            for (uint32_t rd : h.readers) {
                Txn *r = find(rd);
                if (!r || r->commit_id == tc || r->aborted) continue;
                if (r->commit_id < tc && r->finished) {
                    t->set_pred(r->pred);
                    stats.max_pstamp_readers++;
                    if (!t->check()) res = false;
                }
            }
            stats.max_pstamp_headers++;
            t->set_pred(h.pstamp);
            if (!t->check()) res = false;
        }
        return res;
    }

    Store &st_;
    uint32_t counter_;
    std::multimap<uint32_t, Txn *> active_;  // active_tids: Insert never replaces (the first wins)
    std::vector<std::unique_ptr<Txn>> txns_;
};

}  // namespace ssn
