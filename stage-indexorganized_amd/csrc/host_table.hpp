// host_table.hpp -- the host side of one index-organized table.
//
// Keeps the reference's leaf layout (which records live in which leaf, in which slot, the
// sorted/unsorted split, the RecordMetadata words) exactly as the reference's single-loader
// write path would produce it, but in structure-of-arrays form with no payload bytes:
// payloads live in the device record heap and are produced there from their sources.
// Inner-node traversal is replaced on the host by a bucketed separator router (same leaf for
// every key as BTree::TraverseToLeaf) and on the device by an implicit separator tree.
//
// Keys: 1..8 bytes (fixed width or variable, YCSB / BTreeTest) or a fixed width of 9..32
// bytes (TPC-C composite keys of int64 fields, tpcc_record.h).  A key is held as up to four
// order words (stage_core.hpp order_key per 8-byte chunk) plus its length; the unsigned order
// of (words, len) is the reference's KeyCompare order.
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "chunked.hpp"
#include "huge_alloc.hpp"
#include "stage_core.hpp"
#include "../../include/stage_hip.h"

namespace stage {

struct Key {
    uint64_t w[kMaxKeyWords];
    uint32_t len;
};
inline bool key_lt(const Key &a, const Key &b) {
    for (int i = 0; i < kMaxKeyWords; ++i)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i];
    return a.len < b.len;
}
inline bool key_eq(const Key &a, const Key &b) {
    for (int i = 0; i < kMaxKeyWords; ++i)
        if (a.w[i] != b.w[i]) return false;
    return a.len == b.len;
}
inline bool key_le(const Key &a, const Key &b) { return !key_lt(b, a); }
constexpr uint32_t kInfLen = 0xFFFF;
inline Key key_inf() {
    Key k;
    for (int i = 0; i < kMaxKeyWords; ++i) k.w[i] = ~0ull;
    k.len = kInfLen;
    return k;
}
inline Key key_zero() { return Key{{0, 0, 0, 0}, 0}; }
inline bool key_is_inf(const Key &k) { return k.len == kInfLen; }
// key bytes (len <= 32) -> order words; uns: unsigned byte order (tables of 16..32-byte keys)
Key make_key(const uint8_t *bytes, uint32_t len, bool uns);
// order words -> key bytes (len bytes written)
void key_to_bytes(const Key &k, uint8_t *out, bool uns);

// Source of one record-heap image: generated from a rowid, or explicit bytes in the arena.
struct ImageDesc {
    uint64_t key_le;  // key bytes (little-endian, zero above key_len) -- keys of <= 8 bytes
    uint64_t arg;     // rowid (generated) or arena byte offset (explicit)
    uint32_t kind;    // 0 = generated, 1 = arena payload (key in key_le), 2 = arena row [key pad][payload],
                      // 3 = written by the device write path, bytes only in the device heap until
                      //     materialize_device_rows() pulls them into the arena
    uint32_t mode;    // payload generator mode (generated images)
};

// The RecordMetadata each RecordLocation points at (record_location.h:13-42: record_meta_ptr),
// kept current by the host write path: 24-B cells {meta, next_ptr, loc_ptr} in the reference's
// RecordMetadata layout (record_meta.h:30-60) at stable addresses, so a transaction manager can
// dereference a location at commit without a call or a lock (tm.cpp:37, 123, 605), as the
// reference reads the live slot.  next_ptr = the slot's next handle (stage_hip.h STAGE_NEXT_*),
// loc_ptr = the handle; a dropped location reads meta 0.  Cells live in 2^20-entry chunks
// behind a fixed directory: chunks are allocated by the writer before any handle in them is
// published, readers only load.
class LocCells {
public:
    static constexpr uint32_t kChunkBits = 20, kDir = 4096;  // 2^32 handles
    struct Cell {
        std::atomic<uint64_t> meta, next, loc;
    };
    static_assert(sizeof(Cell) == 24, "a cell is a RecordMetadata");
    // read by stage_location_cell and the adoption thread beside the writer that enables it
    bool on() const { return on_.load(std::memory_order_acquire); }
    void enable() { on_.store(true, std::memory_order_release); }
    void ensure(uint64_t handle);  // the chunk holding `handle` exists (writer)
    void set(uint64_t handle, uint64_t meta, uint32_t next) {
        Cell &c = at(handle);
        c.next.store(next, std::memory_order_relaxed);
        c.loc.store(handle, std::memory_order_relaxed);
        c.meta.store(meta, std::memory_order_release);
    }
    const Cell *find(uint64_t handle) const {
        if (handle == 0 || (handle >> kChunkBits) >= kDir) return nullptr;
        const Cell *c = dir_[handle >> kChunkBits].load(std::memory_order_acquire);
        return c ? c + (handle & ((1u << kChunkBits) - 1)) : nullptr;
    }
    ~LocCells();

private:
    Cell &at(uint64_t handle) { return dir_[handle >> kChunkBits].load(std::memory_order_relaxed)[handle & ((1u << kChunkBits) - 1)]; }
    std::atomic<bool> on_{false};
    std::atomic<Cell *> dir_[kDir] = {};
};

// The transaction side of an overwrite copy: EphemeralPool::OverwriteVersionHeader's cstamp
// (writer id), pstamp, rstamp, sstamp, readers, dependency count and waiting flag
// (ephemeral_pool.h:26-150).  The device keeps {rstamp, sstamp, next, image} per copy for reads
// (CopyHdr); this is what the kept SSNTransactionManager reads and updates (AddReader,
// b_tree.cpp:2105; IncreaseWRCount / DecreaseWRCount / UpdatePs, ephemeral_pool.cpp:69-205).
// The pool never frees a header (no GC, as the reference with its cleaner off): an aborted
// update's header stays, waiting.  Reader threads and the writer reach it concurrently: one mutex.
struct CopySsn {
    uint32_t cstamp, pstamp, rstamp, sstamp;
    uint16_t count;
    uint8_t waiting, pad;
};
class CopySsnTable {
public:
    std::mutex mu;
    std::vector<CopySsn, HugeAllocNoInit<CopySsn>> e;                  // by copy id (an epoch appends ~10^6)
    std::unordered_map<uint32_t, std::vector<uint32_t>> readers;  // copy id -> AddReader ids
    // EphemeralPool::Allocate (ephemeral_pool.cpp:17-44): cstamp = pstamp = writer, sstamp MAX
    void created(uint64_t id, uint32_t writer, uint32_t rstamp);
    // CommitTransaction UPDATE entry: SetSstamp(t_sstamp), SetWaiting(true) (tm.cpp:618-619)
    void committed(uint64_t id, uint32_t sstamp);
    // AbortTransaction UPDATE entry: UpdateSs(MAX_CID), SetWaiting(true) (tm.cpp:872-875)
    void aborted(uint64_t id);
};

class HostTable {
public:
    explicit HostTable(const stage_params &p);

    const stage_params &params() const { return p_; }
    uint32_t cap() const { return cap_; }
    uint32_t stride() const { return stride_; }
    uint32_t hstride() const { return stride_; }
    uint32_t key_words() const { return kw_; }      // order words stored per slot
    uint32_t key_pad() const { return kpad_; }      // bytes of the key part of a row
    bool key_unsigned() const { return uns_; }        // KeyCompare's memcmp branch (>= 16 bytes)
    Key key_of(const uint8_t *bytes, uint32_t len) const { return make_key(bytes, len, uns_); }

    // write path, reference ReturnCode values; keys as bytes (len <= 32)
    // inflight: an uncommitted transaction's insert -- the record stays PrepareForInsert
    // (control + visible, cstamp = commit_id = the writer's read id) until commit_insert
    int insert(const uint8_t *key, uint32_t len, const uint8_t *payload, uint64_t gen_rowid, int mode,
               uint32_t commit_id, bool inflight = false);
    int commit_insert(const uint8_t *key, uint32_t len, uint32_t commit_id);
    int update(const uint8_t *key, uint32_t len, uint32_t payload_off, const uint8_t *delta, uint32_t delta_len,
               uint32_t writer_id);
    int commit_update(const uint8_t *key, uint32_t len, uint32_t commit_id, uint32_t sstamp);
    int finalize_update(const uint8_t *key, uint32_t len, uint32_t commit_id);
    int remove(const uint8_t *key, uint32_t len, uint32_t commit_id);
    // the writer's own record (is_for_update = true): LeafNode::Update patches in place, no copy
    // (b_tree.cpp:1101-1104); LeafNode::Delete clears the meta word, no copy reachable
    // (:1210-1220)
    int update_owned(const uint8_t *key, uint32_t len, uint32_t payload_off, const uint8_t *delta, uint32_t delta_len,
                     uint32_t writer_id);
    int remove_owned(const uint8_t *key, uint32_t len);
    int abort_update(const uint8_t *key, uint32_t len);
    int abort_insert(const uint8_t *key, uint32_t len);
    // the same for keys of <= 8 bytes passed little-endian in a u64
    int insert(uint64_t key_le, uint32_t len, const uint8_t *payload, uint64_t gen_rowid, int mode,
               uint32_t commit_id) {
        return len > 8 ? STAGE_RC_INVALID : insert(le(key_le), len, payload, gen_rowid, mode, commit_id);
    }
    int update(uint64_t key_le, uint32_t len, uint32_t payload_off, const uint8_t *delta, uint32_t delta_len,
               uint32_t writer_id) {
        return len > 8 ? STAGE_RC_NOT_FOUND : update(le(key_le), len, payload_off, delta, delta_len, writer_id);
    }
    int commit_update(uint64_t key_le, uint32_t len, uint32_t commit_id, uint32_t sstamp) {
        return len > 8 ? STAGE_RC_NOT_FOUND : commit_update(le(key_le), len, commit_id, sstamp);
    }
    int finalize_update(uint64_t key_le, uint32_t len, uint32_t commit_id) {
        return len > 8 ? STAGE_RC_NOT_FOUND : finalize_update(le(key_le), len, commit_id);
    }
    int remove(uint64_t key_le, uint32_t len, uint32_t commit_id) {
        return len > 8 ? STAGE_RC_NOT_FOUND : remove(le(key_le), len, commit_id);
    }

    uint64_t load_ycsb(uint64_t begin, uint64_t end, uint32_t key_size, int mode);
    uint64_t load_keys(const uint64_t *keys, uint64_t n, uint32_t key_size, int mode);
    // explicit rows: key i = keys + i*key_stride (key_size bytes), payload i = payloads + i*payload_stride
    uint64_t load_rows(const uint8_t *keys, uint32_t key_stride, uint32_t key_size, const uint8_t *payloads,
                       uint32_t payload_stride, uint64_t n, uint32_t commit_id, uint8_t *rc_out);

    // host traversal (TraverseToLeaf equivalent) -> host leaf id
    uint32_t route(const Key &k, bool le_child) const;
    // key -> (leaf, slot) of its first visible record; -1 if absent
    int find(const uint8_t *key, uint32_t len, uint32_t *leaf, uint32_t *slot) const;

    void stats(uint64_t *out) const;
    // leaves in key order
    void key_order(std::vector<uint32_t> &order) const;
    int64_t export_leaves(uint32_t cap, uint64_t max_leaves, uint32_t *rc, uint32_t *sc, uint64_t *meta,
                          uint64_t *keyw) const;
    // leaf-level snapshot in the reference's 64 KiB block format (see host_table.cpp)
    int64_t export_leaf_images(uint64_t max_leaves, uint8_t *blocks, uint64_t *sep_key_le, uint16_t *sep_len) const;
    uint64_t import_leaf_images(const uint8_t *blocks, uint64_t n, uint32_t block_size, const uint64_t *sep_key_le,
                                const uint16_t *sep_len);

    // slot key (order words) of host slot index i = leaf*cap + slot
    Key slot_key(size_t i) const {
        Key k = key_zero();
        for (uint32_t w = 0; w < kw_; ++w) k.w[w] = okey_[i * kw_ + w];
        k.len = meta_keylen(meta_[i]);
        return k;
    }
    // record-heap image payload bytes
    void image_payload(uint32_t img, uint8_t *dst) const;

    // storage (read by the device-image builder)
    struct Leaf {
        uint32_t count = 0, sorted = 0, block = 0, deleted = 0;
        int32_t prev = -1, next = -1;   // key-order neighbours
        Key sep = key_inf();            // inclusive upper bound of the leaf's key range
        bool live = false;
    };
    std::vector<Leaf> leaves_;
    std::vector<uint64_t, HugeAlloc<uint64_t>> okey_;   // [(leaf*cap + slot)*kw + word]
    std::vector<uint64_t, HugeAlloc<uint64_t>> meta_;   // [leaf*cap + slot]
    std::vector<uint32_t, HugeAlloc<uint32_t>> next_;
    std::vector<uint32_t, HugeAlloc<uint32_t>> image_;
    int32_t head_ = 0;
    uint32_t nleaves_live_ = 0;

    // RecordLocation indirection (record_location.h:13-42; BTree::RecordIndirectLocation,
    // b_tree.cpp:2034-2050): one location per Insert attempt, numbered in allocation order as
    // the reference's indirection offsets are; a record's location follows it through splits
    // (LeafNode::CopyFrom, b_tree.cpp:1520-1527).  Handle = location id + 1.
    static constexpr uint64_t kNoPos = ~0ull;
    std::vector<uint32_t, HugeAlloc<uint32_t>> loc_;   // [leaf*cap + slot] -> handle (0 = none)
    std::vector<uint64_t> locpos_;   // location id -> host leaf << 16 | slot, kNoPos = dropped
    uint64_t export_locations(uint64_t max, uint64_t *handles, uint32_t *leaf, uint16_t *slot) const;
    void resolve_locations(const uint64_t *handles, uint64_t n, uint32_t *leaf, uint16_t *slot) const;

    // location cells (stage_location_cell): off until enable_cells(); then every write keeps them
    LocCells cells_;
    void enable_cells();
    // the transaction side of the overwrite copies (stage_copy_*)
    CopySsnTable ssn_;

    ChunkedVector<ImageDesc, (1u << 20)> images_;
    ChunkedArena arena_;
    std::vector<CopyHdr, HugeAllocNoInit<CopyHdr>> copies_;
    std::vector<uint8_t, HugeAlloc<uint8_t>> copy_live_;
    std::vector<VersionHdr, HugeAllocNoInit<VersionHdr>> versions_;
    uint64_t images_synced_ = 0;     // images already present on the device
    uint64_t arena_synced_ = 0;
    bool layout_dirty_ = true;       // any host write since the last publish
    bool structure_dirty_ = true;    // a split (or the first load) changed the leaf set/order
    std::vector<uint64_t> dirty_slots_;  // leaf*cap + slot written since the last publish
    uint64_t copies_synced_ = 0, versions_synced_ = 0;  // headers already on the device
    uint64_t copies_dirty_from_ = ~0ull;                 // lowest synced copy header rewritten since

    // batched write path (one call per YCSB-B epoch): update + optional commit per key;
    // keys: key_stride bytes apart (8 for u64 keys of <= 8 bytes)
    uint64_t update_batch(const uint8_t *keys, uint32_t key_stride, uint64_t n, uint32_t len, uint32_t payload_off,
                          const uint8_t *deltas, uint32_t delta_len, const uint32_t *writer_ids,
                          const uint32_t *commit_ids, const uint32_t *sstamps, uint8_t *rc_out);

    // ---- device write path (write_path.hip): the device applied an update epoch in place;
    // the host adopts its bookkeeping (new copy / version headers, the final slot words of the
    // touched records, `nimages` new heap rows of kind 3) without touching payload bytes.
    struct SlotWords {
        uint64_t idx;   // host slot index leaf*cap + slot
        uint64_t meta;
        uint32_t next, image;
    };
    // slots with idx == ~0 are skipped
    // writers[k] = the writer id of copy k (its OverwriteVersionHeader cstamp)
    void adopt_device_epoch(const CopyHdr *copies, const uint32_t *writers, uint64_t nc, const VersionHdr *versions,
                            uint64_t nv, uint64_t nimages, const SlotWords *slots, uint64_t nslots);
    // room for `add` more copy / version headers with no reallocation inside adopt_device_epoch
    // (a reallocation there moves every earlier header -- ~30 ms at 4M -- on the adoption thread,
    // which the next epochs' calls wait for); called while no adoption is running
    void reserve_adoption(uint64_t add);
    // fn(begin, end) over [0, n) on up to 16 threads (one below 65536 items)
    static void parallel_chunks(uint64_t n, const std::function<void(uint64_t, uint64_t)> &fn);
    bool has_device_rows() const { return !device_rows_.empty(); }
    // pull the bytes of device-written rows into the arena (host-side writes and the leaf-image
    // export read payloads); fetch(first, count, dst) copies heap rows [first, first+count)
    void materialize_device_rows(const std::function<void(uint64_t, uint64_t, uint8_t *)> &fetch);
    std::vector<std::pair<uint64_t, uint64_t>> device_rows_;  // (first image, count) of kind 3

private:
    struct RouteEntry {
        Key sep;
        uint32_t leaf;
    };
    static uint32_t bucket_of(const Key &k) { return (uint32_t)(k.w[0] >> 48); }
    static bool entry_lt_key(const RouteEntry &e, const Key &k) { return key_lt(e.sep, k); }
    static const uint8_t *le(const uint64_t &key_le) { return reinterpret_cast<const uint8_t *>(&key_le); }

    // slot i's words changed: its location's cell follows
    void cell(size_t i) {
        if (cells_.on() && loc_[i]) cells_.set(loc_[i], meta_[i], next_[i]);
    }
    void cell_drop(uint32_t handle) {
        if (cells_.on() && handle) cells_.set(handle, 0, 0);
    }
    void touch(uint32_t leaf, uint32_t slot) {
        layout_dirty_ = true;
        if (!structure_dirty_) dirty_slots_.push_back((uint64_t)leaf * cap_ + slot);
    }
    uint32_t alloc_leaf();
    int64_t search(uint32_t leaf, const Key &k) const;  // SearchRecordMeta (check_concurrency)
    uint32_t used_space(const Leaf &l) const { return 40u + l.block + l.count * 24u; }
    bool split(uint32_t leaf);
    void route_split(uint32_t p, uint32_t r, const Key &lo, const Key &s, const Key &hi);
    uint32_t new_image(const uint8_t *key, uint32_t len, const uint8_t *payload, uint64_t gen_rowid, int mode);
    bool key_ok(uint32_t len) const;
    void set_slot_key(size_t i, const Key &k) {
        for (uint32_t w = 0; w < kw_; ++w) okey_[i * kw_ + w] = k.w[w];
    }
    void clear_slot_key(size_t i) {
        for (uint32_t w = 0; w < kw_; ++w) okey_[i * kw_ + w] = 0;
    }

    stage_params p_;
    uint32_t cap_ = 64;
    uint32_t kw_ = 1;      // order words per slot
    uint32_t kpad_ = 8;    // key bytes in a row (padded to 8)
    bool uns_ = false;     // unsigned byte order
    uint32_t stride_ = 1008;
    uint32_t max_records_ = 63;
    std::vector<std::vector<RouteEntry>> buckets_;
    std::vector<uint32_t> free_leaves_;
};

// payload generator (data only; same definition as the test oracle's)
void gen_payload(uint64_t rowid, int mode, uint8_t *dst, uint32_t payload_size);

}  // namespace stage
