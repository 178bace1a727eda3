// stage_btree_adapter.hpp -- the reference-side framing of a stage_probe_out, header-only C++17
// over stage_hip.h.  What a reference BTree facade needs to hand the unchanged executors the
// objects they consume:
//
//   read_return_code()    LeafNode::Read's ReturnCode (b_tree.cpp:1042-1051): Ok / NotFound
//   make_record()         the heap Record BTree::Read returns (b_tree.cpp:2066-2129):
//                         Record::New for the latest image, Record::Neww for an in-flight
//                         update's overwrite copy; byte framing of b_tree.h:400-448 =
//                         [RecordMeta 48 B][cstamp 4 B][key padded to 8][payload]
//   point_lookup()        IndexScanExecutor::Execute's point-lookup outcome (executor.h:374-454):
//                         ResultType, whether PerformRead runs (and its three facts), whether a
//                         tuple is produced and from where
//   ycsb_tuple_int()      the executor's `T` bytes for the YCSB driver's YCSBTupleInt (1004 B):
//                         latest / copy = memcpy(sizeof(T)) from Record::GetData() =
//                         [key 4][pad 4][payload 0..995]; retired = memcpy from the TupleHeader
//                         slot = [key 4][payload 0..999] (executor.h:396-401, 424)
//
// and what the kept SSNTransactionManager dereferences through such a Record
// (transaction_manager.cpp:29-221, 362-410, 535-1046):
//
//   LocationTable         RecordMetadata::loc_ptr -> RecordLocation -> record_meta_ptr: one
//                         RecordLocation per location handle (record_location.h:13-42) whose
//                         record_meta_ptr is the library's live cell (stage_location_cell), so
//                         `*reinterpret_cast<RecordMetadata *>(loc->record_meta_ptr)` is the
//                         record's current RecordMetadata wherever splits moved it (tm.cpp:37,
//                         123, 605)
//   OverwritePool         the EphemeralPool methods the manager calls on a next_ptr
//                         (GetOversionHeader, IncreaseWRCount, DecreaseWRCount, UpdatePs) and
//                         the AddReader BTree::Read does (b_tree.cpp:2104-2105), over stage_copy_*
//   read_via_copy()       whether BTree::Read served the read from the overwrite copy (then it
//                         registers the reader: b_tree.cpp:2087-2105)
//
// next_ptr is the library's next handle (stage_hip.h STAGE_NEXT_*: the overwrite copy while an
// update is in flight -- the EphemeralPool key --, the newest TupleHeader after a commit);
// loc_ptr is whatever the facade uses for RecordLocation * (LocationTable::get(handle)).
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "stage_hip.h"

namespace stage_adapter {

// RecordMetadata (record_meta.h:30-204): 24 B
struct RecordMetadata {
    uint64_t meta;
    uint64_t next_ptr;
    uint64_t loc_ptr;
};
static_assert(sizeof(RecordMetadata) == 24, "RecordMetadata is 24 B in the reference");

// RecordMeta (record_meta.h:223-298): 48 B with the compiler's padding
struct RecordMeta {
    RecordMetadata meta_data;
    uint32_t total_size;
    uint64_t next_tuple_ptr;
    uint32_t cstamp;
};
static_assert(sizeof(RecordMeta) == 48, "RecordMeta is 48 B in the reference (SURVEY App. B)");

// ResultType values the executors set (include/common/constants.h:112-121)
enum class ResultType : int { INVALID = 0, SUCCESS = 1, FAILURE = 2, ABORTED = 3 };

constexpr uint64_t kControl = 1ull << 63;
constexpr uint64_t kVisible = 1ull << 62;

inline uint64_t meta_word(const stage_probe_out &o) { return ((uint64_t)o.meta_hi << 32) | o.rec_cstamp; }
inline uint32_t key_length(uint64_t meta) { return (uint32_t)((meta >> 48) & 0x2FFF); }
inline uint32_t padded_key_length(uint64_t meta) { return (key_length(meta) + 7u) / 8u * 8u; }
inline bool is_inserting(uint64_t meta) { return (meta & kVisible) && (meta & kControl); }
inline bool is_copy_handle(uint64_t next_ptr) {
    return next_ptr != 0 && (next_ptr & STAGE_NEXT_KIND_MASK) == STAGE_NEXT_COPY && next_ptr <= 0xFFFFFFFFull;
}
inline uint32_t copy_id(uint64_t next_ptr) { return (uint32_t)(next_ptr & STAGE_NEXT_INDEX_MASK); }

// the probe was answered as BTree::Read(..., is_for_update = true) (stage_probe_batch_ex,
// stage_reader_read_ex)
inline bool for_update(const stage_probe_out &o) { return (o.flags & STAGE_FLAG_FOR_UPDATE) != 0; }

// BTree::Read served the read from the overwrite copy (record in flight, copy header found,
// not for update): Record::Neww + AddReader(commit_id) (b_tree.cpp:2087-2105)
inline bool read_via_copy(const stage_probe_out &o, const stage_probe_ident &id) {
    return !for_update(o) && o.status != STAGE_ST_NOT_FOUND && is_inserting(meta_word(o)) && is_copy_handle(id.next);
}

// RecordLocation (record_location.h:13-42)
struct RecordLocation {
    uint64_t node_header_ptr;
    uint64_t record_meta_ptr;
};

// One RecordLocation per location handle at a stable address; record_meta_ptr = the library's
// cell for the handle (stage_location_cells must be on).  The facade puts get(handle) into
// RecordMetadata::loc_ptr; handle_of() maps it back.  Thread-safe.
class LocationTable {
public:
    explicit LocationTable(stage_table *t) : t_(t) {}
    RecordLocation *get(uint64_t handle) {
        if (handle == 0) return nullptr;
        std::lock_guard<std::mutex> g(mu_);
        const uint64_t c = (handle - 1) >> kBits, i = (handle - 1) & ((1u << kBits) - 1);
        if (chunks_.size() <= c) chunks_.resize(c + 1);
        if (!chunks_[c]) chunks_[c].reset(new RecordLocation[1u << kBits]());
        RecordLocation &l = chunks_[c][i];
        if (!l.record_meta_ptr) {
            const void *cell = nullptr;
            if (stage_location_cell(t_, handle, &cell) != STAGE_OK) throw std::runtime_error(stage_last_error());
            l.record_meta_ptr = reinterpret_cast<uint64_t>(cell);
        }
        return &l;
    }
    // the RecordMetadata the location points at now (the manager's `meta_location` deref)
    static const RecordMetadata *record_meta(const RecordLocation *l) {
        return reinterpret_cast<const RecordMetadata *>(l->record_meta_ptr);
    }
    static uint64_t handle_of(const RecordLocation *l) { return l ? record_meta(l)->loc_ptr : 0; }

private:
    static constexpr uint32_t kBits = 16;
    stage_table *t_;
    std::mutex mu_;
    std::vector<std::unique_ptr<RecordLocation[]>> chunks_;
};

// EphemeralPool::OverwriteVersionHeader as the manager reads it (ephemeral_pool.h:26-150)
struct OverwriteHeader {
    uint32_t cstamp, pstamp, rstamp, sstamp;
    uint16_t count;
    bool waiting;
    std::vector<uint32_t> readers;
    int GetReadersNum() const { return (int)readers.size(); }
    uint32_t GetReaders(int i) const { return i < (int)readers.size() ? readers[i] : 0u; }
};

// The EphemeralPool calls of the kept manager, keyed by next_ptr as the reference keys them by
// copy location (ephemeral_pool.cpp:69-205); a next_ptr that is not a copy handle has no header.
class OverwritePool {
public:
    explicit OverwritePool(stage_table *t) : t_(t) {}
    bool GetOversionHeader(uint64_t next_ptr, OverwriteHeader &h) const {
        if (!is_copy_handle(next_ptr)) return false;
        const uint32_t id = copy_id(next_ptr);
        stage_copy_state s;
        if (stage_copy_get(t_, &id, 1, &s) != STAGE_OK) return false;
        h.cstamp = s.cstamp, h.pstamp = s.pstamp, h.rstamp = s.rstamp, h.sstamp = s.sstamp;
        h.count = s.count, h.waiting = s.waiting != 0;
        h.readers.resize(s.readers);
        uint32_t k = 0;
        if (s.readers && stage_copy_readers(t_, id, h.readers.data(), s.readers, &k) != STAGE_OK) return false;
        h.readers.resize(k < s.readers ? k : s.readers);
        return true;
    }
    void AddReader(uint64_t next_ptr, uint32_t read_id) {  // OverwriteVersionHeader::AddReader
        if (is_copy_handle(next_ptr)) check(stage_copy_add_reader(t_, copy_id(next_ptr), read_id));
    }
    bool IncreaseWRCount(uint64_t next_ptr) {
        int ok = 0;
        if (!is_copy_handle(next_ptr) || stage_copy_wr_count(t_, copy_id(next_ptr), +1, &ok) != STAGE_OK) return false;
        return ok != 0;
    }
    void DecreaseWRCount(uint64_t next_ptr) {
        int ok = 0;
        if (is_copy_handle(next_ptr)) check(stage_copy_wr_count(t_, copy_id(next_ptr), -1, &ok));
    }
    bool UpdatePs(uint64_t next_ptr, uint32_t pstamp) {
        return is_copy_handle(next_ptr) && stage_copy_update_ps(t_, copy_id(next_ptr), pstamp) == STAGE_OK;
    }

private:
    static void check(int rc) {
        if (rc != STAGE_OK) throw std::runtime_error(stage_last_error());
    }
    stage_table *t_;
};

// LeafNode::Read -> SearchRecordMeta hit or RecordMetadata{0}
inline int read_return_code(const stage_probe_out &o) {
    return o.status == STAGE_ST_NOT_FOUND ? STAGE_RC_NOT_FOUND : STAGE_RC_OK;
}

// Does BTree::Read return a Record?  Latest image (Record::New) or copy (Record::Neww); an OLD /
// FAIL / CHAIN_MISS outcome also came from a Record of the latest image (its cstamp is above the
// reader), which the executor deletes after walking the chain -- it is not materialised here.
inline bool has_record(const stage_probe_out &o) {
    return o.status == STAGE_ST_LATEST || o.status == STAGE_ST_COPY;
}

// The RecordMeta BTree::Read builds (RecordMeta(*meta), b_tree.cpp:2083): the hit slot's
// RecordMetadata -- meta word, next_ptr = its next handle, loc_ptr = the facade's RecordLocation
// for its location handle (LocationTable::get(id.loc), or any stable value the facade maps back)
inline RecordMeta record_meta(const stage_probe_out &o, const stage_probe_ident &id, uint64_t loc_ptr,
                              uint32_t payload_size) {
    RecordMeta rm{};
    rm.meta_data.meta = meta_word(o);
    rm.meta_data.next_ptr = id.next;
    rm.meta_data.loc_ptr = loc_ptr;
    rm.total_size = padded_key_length(rm.meta_data.meta) + payload_size;  // SetTotalSize, b_tree.cpp:2084
    rm.next_tuple_ptr = 0;  // TupleHeader / copy-next handles stay device-side
    rm.cstamp = o.cstamp;   // latest: reader id; copy: the copy's rstamp
    return rm;
}

// The Record bytes (b_tree.h:400-448): RecordMeta, then tuple_data_ = [cstamp][key][payload].
// `row` = the probe's tuple row [key padded to 8][payload] (canonical: the pad bytes, which
// Record::Neww leaves uninitialised, are zero).  Empty when has_record() is false.
inline std::vector<uint8_t> make_record(const stage_probe_out &o, const stage_probe_ident &id, uint64_t loc_ptr,
                                        const uint8_t *row, uint32_t payload_size) {
    std::vector<uint8_t> out;
    if (!has_record(o)) return out;
    const uint64_t meta = meta_word(o);
    const uint32_t kp = padded_key_length(meta);
    RecordMeta rm = record_meta(o, id, loc_ptr, payload_size);
    out.resize(sizeof(RecordMeta) + 4 + kp + payload_size);
    std::memcpy(out.data(), &rm, sizeof rm);
    std::memcpy(out.data() + sizeof rm, &o.cstamp, 4);  // Record::SetCstamp
    const uint32_t row_key = kp > 8 ? kp : 8;  // the row's key region: the key padded to 8
    std::memcpy(out.data() + sizeof rm + 4, row, kp);
    std::memcpy(out.data() + sizeof rm + 4 + kp, row + row_key, payload_size);
    return out;
}

struct PointLookup {
    ResultType result;     // what Execute() leaves in the transaction (FAILURE => returns false)
    bool perform_read;     // PerformRead(txn, record->meta, cstamp) is called (not for update)
    bool tuple;            // ycsb_tuple is produced
    bool retired;          // ... from a TupleHeader slot (retired framing)
    uint32_t cstamp;       // PerformRead facts (transaction_manager.cpp:362-410)
    bool copy_present;
    uint32_t copy_sstamp;
};

// IndexScanExecutor point lookup (executor.h:374-454); a for-update probe (STAGE_FLAG_FOR_UPDATE)
// is the executor built with is_for_update: no PerformRead on the latest branch (:388)
inline PointLookup point_lookup(const stage_probe_out &o) {
    PointLookup p{ResultType::SUCCESS, false, false, false, o.cstamp,
                  (o.flags & STAGE_FLAG_COPY_PRESENT) != 0, o.copy_sstamp};
    switch (o.status) {
        case STAGE_ST_LATEST:
        case STAGE_ST_COPY: p.perform_read = !for_update(o); p.tuple = true; break;  // txn_id >= cstamp
        case STAGE_ST_OLD: p.tuple = true; p.retired = true; break;       // begin <= txn_id <= end
        case STAGE_ST_FAIL_INVALID_TS: p.result = ResultType::FAILURE; break;  // begin/end INVALID
        default: break;  // NOT_FOUND: Read -> nullptr; CHAIN_MISS: walked off the chain
    }
    return p;
}

// YCSBTupleInt {uint32_t key; char cols[10][100]} (ycsb_configuration.h): 1004 B
constexpr uint32_t kYcsbTupleInt = 1004;
inline bool ycsb_tuple_int(const stage_probe_out &o, const uint8_t *row, uint8_t *t /* 1004 B */) {
    const PointLookup p = point_lookup(o);
    if (!p.tuple) return false;
    if (!p.retired) {
        std::memcpy(t, row, kYcsbTupleInt);  // GetData() = [key padded to 8][payload]
    } else {
        std::memcpy(t, row, 4);               // slot = [key(key_len = 4)][payload]
        std::memcpy(t + 4, row + 8, kYcsbTupleInt - 4);
    }
    return true;
}

}  // namespace stage_adapter
