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
// Pointers the reference keeps in these objects (RecordMetadata::next_ptr / loc_ptr,
// RecordMeta::next_tuple_ptr) are process-local addresses there; here they are stable opaque
// handles: loc_ptr = record_handle() (the rw-set identity, RecordMeta::operator== compares
// loc_ptr only, record_meta.h:248-251), next_ptr = a non-zero copy handle exactly when an
// overwrite header exists (what PerformRead's GetOversionHeader(next_ptr) tests), else 0.
#pragma once
#include <cstdint>
#include <cstring>
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
// stable identity of the hit record (leaf, slot) -- never 0
inline uint64_t record_handle(const stage_probe_out &o) { return ((uint64_t)o.leaf << 16 | o.slot) + 1; }

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

// The Record bytes (b_tree.h:400-448): RecordMeta, then tuple_data_ = [cstamp][key][payload].
// `row` = the probe's tuple row [key padded to 8][payload] (canonical: the pad bytes, which
// Record::Neww leaves uninitialised, are zero).  Empty when has_record() is false.
inline std::vector<uint8_t> make_record(const stage_probe_out &o, const uint8_t *row, uint32_t payload_size) {
    std::vector<uint8_t> out;
    if (!has_record(o)) return out;
    const uint64_t meta = meta_word(o);
    const uint32_t kp = padded_key_length(meta);
    RecordMeta rm{};
    rm.meta_data.meta = meta;
    rm.meta_data.next_ptr = (o.flags & STAGE_FLAG_COPY_PRESENT) ? (record_handle(o) | (1ull << 63)) : 0;
    rm.meta_data.loc_ptr = record_handle(o);
    rm.total_size = kp + payload_size;  // SetTotalSize(padded key + payload), b_tree.cpp:2079
    rm.next_tuple_ptr = 0;              // TupleHeader / copy-next handles stay device-side
    rm.cstamp = o.cstamp;               // latest: reader id; copy: the copy's rstamp
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
    bool perform_read;     // PerformRead(txn, record->meta, cstamp) is called (not for_update)
    bool tuple;            // ycsb_tuple is produced
    bool retired;          // ... from a TupleHeader slot (retired framing)
    uint32_t cstamp;       // PerformRead facts (transaction_manager.cpp:362-410)
    bool copy_present;
    uint32_t copy_sstamp;
};

// IndexScanExecutor point lookup (executor.h:374-454) for a reader that is not for_update
inline PointLookup point_lookup(const stage_probe_out &o) {
    PointLookup p{ResultType::SUCCESS, false, false, false, o.cstamp,
                  (o.flags & STAGE_FLAG_COPY_PRESENT) != 0, o.copy_sstamp};
    switch (o.status) {
        case STAGE_ST_LATEST:
        case STAGE_ST_COPY: p.perform_read = true; p.tuple = true; break;  // txn_id >= cstamp
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
