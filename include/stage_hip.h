/*
 * stage_hip.h -- C-ABI of the MI355X-native index-organized probe/scan path.
 *
 * This is the drop-in boundary for the hot path of sheepTnT/Stage-IndexOrganized
 * (reference @ 2024-12-18).  Every entry point below names the reference interface it
 * replaces (file:line inside the reference checkout).  All types are plain C: fixed-width
 * integers and pointers; no C++ exceptions cross this boundary.  Device pointers are
 * HIP device allocations (stage_dev_alloc or any hipMalloc'd buffer of the same
 * process); `stream` is a hipStream_t passed as void* (NULL = the table's own stream).
 *
 * Return value of every int function: STAGE_OK (0) or a negative STAGE_E_* code;
 * stage_last_error() gives the message for the calling thread.
 */
#ifndef STAGE_HIP_H_
#define STAGE_HIP_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define STAGE_OK 0
#define STAGE_E_ARG (-1)
#define STAGE_E_HIP (-2)
#define STAGE_E_NOMEM (-3)
#define STAGE_E_STATE (-4)
#define STAGE_E_UNSUPPORTED (-5)
#define STAGE_E_RCCL (-6)

/* ReturnCode (include/vstore/b_tree.h:42-54), reported by the host write path */
#define STAGE_RC_INVALID 0
#define STAGE_RC_OK 1
#define STAGE_RC_KEY_EXISTS 2
#define STAGE_RC_NOT_FOUND 3
#define STAGE_RC_NODE_FROZEN 4
#define STAGE_RC_CAS_FAIL 5
#define STAGE_RC_NOT_ENOUGH_SPACE 6
#define STAGE_RC_NOT_NEEDED_UPDATE 7
#define STAGE_RC_RETRY_FAILURE 8
#define STAGE_RC_DIRTY 9

/* per-probe status (canonical outcome of BTree::Read b_tree.cpp:2066-2129 followed by the
 * point-lookup branch of IndexScanExecutor::Execute, executor.h:374-454) */
#define STAGE_ST_NOT_FOUND 0      /* Read returned nullptr                                */
#define STAGE_ST_LATEST 1         /* txn_id >= meta cstamp, tuple from the leaf            */
#define STAGE_ST_COPY 2           /* in-flight update: tuple from the overwrite copy       */
#define STAGE_ST_OLD 3            /* retired version from the TupleHeader chain            */
#define STAGE_ST_FAIL_INVALID_TS 4/* chain hit begin/end == INVALID_CID -> ResultType::FAILURE */
#define STAGE_ST_CHAIN_MISS 5     /* no version visible to txn_id (tuple stays null)       */

#define STAGE_FLAG_COPY_PRESENT 1u /* PerformRead would find an overwrite header (tm.cpp:379-399) */
#define STAGE_FLAG_FOR_UPDATE 2u   /* answered as BTree::Read(..., is_for_update = true): the
                                      executor skips PerformRead (executor.h:388) and Read did not
                                      AddReader (b_tree.cpp:2087, 2114-2120)                  */

typedef struct stage_table stage_table; /* one index-organized table: BTree + device image */

/* ParameterSet (b_tree.h:23-40) plus the key column width of the Catalog */
typedef struct stage_params {
    uint32_t split_threshold; /* inner-node split threshold (YCSB: 16 KiB, ycsb.cpp:72)   */
    uint32_t merge_threshold; /* (YCSB: 32 KiB)                                          */
    uint32_t leaf_node_size;  /* leaf block == leaf split threshold (YCSB: 64 KiB)       */
    uint32_t payload_size;    /* bytes after the 8-byte padded key (YCSB: 1000)          */
    uint32_t key_width;       /* 1..32 = every key has this many bytes; 0 = variable 1..8 */
    int32_t device;           /* HIP device ordinal for the device image                  */
} stage_params;

/* one probe result (32 B) */
typedef struct stage_probe_out {
    uint8_t status;       /* STAGE_ST_*                                                    */
    uint8_t flags;        /* STAGE_FLAG_*                                                  */
    uint16_t hops;        /* TupleHeader hops walked                                       */
    uint32_t leaf;        /* leaf index in key order                                       */
    uint16_t slot;        /* record slot inside the leaf (0xFFFF if none)                  */
    uint16_t key_len;     /* key length of the hit record                                  */
    uint32_t cstamp;      /* Record cstamp handed to PerformRead: latest -> read id,
                             copy -> overwrite rstamp, old -> TupleHeader begin            */
    uint32_t rec_cstamp;  /* meta.GetTxnCommitId() of the hit slot (executor.h:383)        */
    uint32_t copy_sstamp; /* overwrite header sstamp, 0xFFFFFFFF when none                 */
    uint32_t image;       /* record-heap row that supplied the tuple (0xFFFFFFFF if none)  */
    uint32_t meta_hi;     /* upper half of the hit slot's RecordMetadata word (control, visible,
                             key length, offset; record_meta.h:66-70): meta = meta_hi << 32 |
                             rec_cstamp.  STAGE_REPLY_OWNER status records carry the owner-local
                             row index here instead (stage_probe_sharded_ex)               */
} stage_probe_out;

/* lean probe result (16 B, opt-in for stage_probe_batch via stage_set_output_layout): what the
 * IndexScanExecutor point branch and PerformRead consume -- the outcome, the PerformRead facts
 * and the record cstamp; no leaf / slot / image / meta word. */
typedef struct stage_probe_out16 {
    uint8_t status;
    uint8_t flags;
    uint16_t hops;
    uint32_t cstamp;
    uint32_t copy_sstamp;
    uint32_t rec_cstamp;
} stage_probe_out16;

const char *stage_last_error(void);
const char *stage_version(void);

/* ---- table lifecycle ------------------------------------------------------------------
 * replaces: BTree::BTree (b_tree.h:793-803), ParameterSet (b_tree.h:23-40) */
int stage_table_create(const stage_params *params, stage_table **out);
int stage_table_destroy(stage_table *t);

/* ---- host write path (kept on host per the north star) ---------------------------------
 * stage_insert      = BTree::Insert + BTree::FinalizeInsert (b_tree.cpp:1849-2020, 2238-2251)
 *                     payload == NULL inserts the generated payload of `gen_rowid`.
 * stage_load_ycsb   = LoadYCSBRows (benchmark/ycsb/ycsb_loader.cpp:93-171), one loader,
 *                     rows [begin,end) with key = rowid (key_size 4 or 8 bytes), payload
 *                     mode 0 = memset(rowid) as the reference, 1 = per-word pattern.
 * stage_load_keys   = the same for an explicit key order (keys are rowids).
 * stage_update      = BTree::Update / LeafNode::Update (b_tree.cpp:2132-2160, 1061-1163)
 * stage_commit_update = CommitTransaction UPDATE entry (transaction_manager.cpp:610-676)
 * stage_finalize_update = BTree::FinalizeUpdate (b_tree.cpp:2252-2268)
 * stage_delete      = BTree::Delete + FinalizeDelete (b_tree.cpp:2184-2237, 2275-2310); the
 *                     record is deleted either way, and STAGE_RC_INVALID (instead of OK) says
 *                     the leaf fell below merge_threshold, where the reference would merge it
 *                     with a sibling (CheckMerge, not restated: the leaf stays as it is)
 * rc_out receives the reference ReturnCode (STAGE_RC_*). */
int stage_insert(stage_table *t, uint64_t key, uint16_t key_size, const uint8_t *payload,
                 uint64_t gen_rowid, int payload_mode, uint32_t commit_id, uint8_t *rc_out);
int stage_load_ycsb(stage_table *t, uint64_t begin_rowid, uint64_t end_rowid, uint32_t key_size,
                    int payload_mode, uint64_t *inserted);
int stage_load_keys(stage_table *t, const uint64_t *keys, uint64_t n, uint32_t key_size,
                    int payload_mode, uint64_t *inserted);
int stage_update(stage_table *t, uint64_t key, uint16_t key_size, uint32_t payload_off,
                 const uint8_t *delta, uint32_t delta_len, uint32_t writer_id, uint8_t *rc_out);
int stage_commit_update(stage_table *t, uint64_t key, uint16_t key_size, uint32_t commit_id,
                        uint32_t sstamp, uint8_t *rc_out);
int stage_finalize_update(stage_table *t, uint64_t key, uint16_t key_size, uint32_t commit_id,
                          uint8_t *rc_out);
int stage_delete(stage_table *t, uint64_t key, uint16_t key_size, uint32_t commit_id,
                 uint8_t *rc_out);
/* batched write path of one transaction epoch (the YCSB-B writers, ycsb.cpp:200-260): for
 * key i (key_size bytes at keys + i*key_stride; u64 keys of <= 8 bytes: key_stride 8),
 * stage_update(key i, payload_off, deltas + i*delta_len, writer_ids[i]) and, when it
 * succeeded and commit_ids[i] != 0, stage_commit_update(key i, commit_ids[i], sstamps[i]
 * (or commit_ids[i] when sstamps is NULL)).  rc_out[i] (optional) = the last ReturnCode;
 * *n_ok (optional) = keys whose update (and commit) returned STAGE_RC_OK. */
int stage_update_batch(stage_table *t, const void *keys, uint32_t key_stride, uint64_t n,
                       uint16_t key_size, uint32_t payload_off, const uint8_t *deltas,
                       uint32_t delta_len, const uint32_t *writer_ids, const uint32_t *commit_ids,
                       const uint32_t *sstamps, uint8_t *rc_out, uint64_t *n_ok);
/* the same epoch applied by the device to the published image (in-place
 * column update + overwrite copy + retire-at-commit, b_tree.cpp:1061-1163,
 * transaction_manager.cpp:610-676), no re-publish: keys / lens as stage_probe_batch, deltas
 * (n x delta_len), ids and d_rc (n ReturnCodes) in device memory; the table must be synced.
 * Same return codes and resulting reads as stage_update_batch + stage_sync.  Returns after the
 * host has adopted the epoch's bookkeeping (copy / version headers, slot words); the new
 * payload bytes stay in HBM and are fetched only when a host path needs them. */
int stage_update_batch_device(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens, uint64_t n,
                              uint32_t payload_off, const uint8_t *d_deltas, uint32_t delta_len,
                              const uint32_t *d_writer_ids, const uint32_t *d_commit_ids,
                              const uint32_t *d_sstamps, uint8_t *d_rc, uint64_t *n_ok, void *stream);
/* waits for the host table's adoption of the last stage_update_batch_device epoch (it runs on a
 * background thread; every host-table entry point waits for it anyway) and reports its error */
int stage_settle(stage_table *t);
/* write-overlap mode of stage_update_batch_device (default 0): an epoch's kernels up to the
 * publish of its slot words run on the table's own stream as soon as the previous epoch has
 * published, beside whatever the caller enqueued on `stream` after that (e.g. the previous
 * epoch's read probes); only the publish waits for `stream`.  Results are the same.  Contract:
 * the epoch's inputs (keys, deltas, ids) are complete when the call is made -- not produced by
 * work still pending on `stream` -- and stay unmodified until the work enqueued on `stream`
 * behind the call has run (stream order, as for every device entry point).  A deferred-publish
 * mode 2 was measured and retired. */
int stage_set_write_overlap(stage_table *t, int on);

/* byte-key forms, for every key width a table takes: 1..8 bytes (key_width 1..8 or 0 =
 * variable) or a fixed width of 9..32 bytes (TPC-C composite keys, tpcc_record.h: int64
 * fields, e.g. OrderLineKey = 32 bytes).  Same ReturnCodes as the u64 forms above.
 * stage_load_rows inserts n rows in order (key i at keys + i*key_stride, payload i at
 * payloads + i*payload_stride), rc_out[i] optional.
 * Device key buffers (stage_probe_batch, stage_scan_batch, stage_resolve_batch,
 * stage_traverse_batch) hold stage_key_words(t) u64 words per key: the key bytes
 * little-endian, zero padded (1 word for keys of <= 8 bytes, 2 for 9..16, 4 for 17..32). */
int stage_insert_key(stage_table *t, const uint8_t *key, uint16_t key_size, const uint8_t *payload,
                     uint32_t commit_id, uint8_t *rc_out);
/* an uncommitted transaction's insert (InsertExecutor, executor.h:26-85 -> BTree::Insert, which
 * leaves the record PrepareForInsert: control + visible, cstamp = writer_id, b_tree.cpp:860-864;
 * other transactions' reads of it return nothing, b_tree.cpp:2087-2095), and the
 * CommitTransaction INSERT entry that publishes it (FinalizeForInsert(t_cstamp),
 * transaction_manager.cpp:677-695).  stage_abort_insert_key aborts it. */
int stage_insert_key_inflight(stage_table *t, const uint8_t *key, uint16_t key_size, const uint8_t *payload,
                              uint32_t writer_id, uint8_t *rc_out);
int stage_commit_insert_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t commit_id,
                            uint8_t *rc_out);
int stage_load_rows(stage_table *t, const uint8_t *keys, uint32_t key_stride, uint16_t key_size,
                    const uint8_t *payloads, uint32_t payload_stride, uint64_t n, uint32_t commit_id,
                    uint8_t *rc_out, uint64_t *inserted);
int stage_update_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t payload_off,
                     const uint8_t *delta, uint32_t delta_len, uint32_t writer_id, uint8_t *rc_out);
int stage_commit_update_key(stage_table *t, const uint8_t *key, uint16_t key_size,
                            uint32_t commit_id, uint32_t sstamp, uint8_t *rc_out);
int stage_delete_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t commit_id,
                     uint8_t *rc_out);
/* AbortTransaction (transaction_manager.cpp:825-1045) for one key of the table:
 * stage_abort_update_key = the UPDATE entry (:846-921): the old image back from the overwrite
 *   copy, control bit cleared, next := the chain the update found, the copy released;
 * stage_abort_insert_key = the INSERT entry (:949-979): FinalizeForDelete + FailForInsert on
 *   the leaf's last slot (an insert not in its leaf's last slot: STAGE_RC_INVALID). */
int stage_abort_update_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint8_t *rc_out);
/* the writer's own record, is_for_update = true (PointUpdateExecutor / PointDeleteExecutor built
 * with is_for_update, executor.h:194-340, 101-193; TestingTransactionUtil's Update(.., true) /
 * Delete(.., true)): stage_update_key_owned = LeafNode::Update's in-place branch (b_tree.cpp:
 * 1101-1104: no Dirty refusal of an in-flight record, no overwrite copy, no version; NotFound /
 * NotNeededUpdate as stage_update_key); stage_delete_key_owned = LeafNode::Delete's is_for_update
 * branch (:1210-1220: the meta word cleared, nothing for a commit to finalize; STAGE_RC_INVALID
 * where stage_delete_key's merge rule applies).  Publish with stage_sync as any host write. */
int stage_update_key_owned(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t payload_off,
                           const uint8_t *delta, uint32_t delta_len, uint32_t writer_id, uint8_t *rc_out);
int stage_delete_key_owned(stage_table *t, const uint8_t *key, uint16_t key_size, uint8_t *rc_out);
int stage_abort_insert_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint8_t *rc_out);
uint32_t stage_key_words(stage_table *t);

/* publish the host layout to HBM (leaf key columns, slot words, visibility masks, the
 * separator search tree, record heap, overwrite copies and retired versions). */
int stage_sync(stage_table *t);
/* what the last stage_sync did: info[0] = 1 if it patched in place (no split since the
 * previous publish), info[1] = leaves re-headed, info[2] = slots patched; *seconds = wall time */
int stage_sync_info(stage_table *t, double *seconds, uint64_t *info);

/* stats[0]=height(host equivalent: 1 + ceil(log_fanout)) stats[1]=0 stats[2]=leaves
 * stats[3]=records stats[4]=sorted slots stats[5]=unsorted slots stats[6]=max records/leaf
 * stats[7]=retired versions */
int stage_stats(stage_table *t, uint64_t *stats);
uint32_t stage_record_stride(stage_table *t); /* bytes between output/heap rows */
uint32_t stage_leaf_capacity(stage_table *t); /* slots per leaf on the device (64/128) */

/* host traversal -> leaf index in key order (BTree::TraverseToLeaf, b_tree.cpp:1804-1846) */
int stage_traverse_batch(stage_table *t, const uint64_t *keys, const uint16_t *lens, uint64_t n,
                         int le_child, uint32_t *leaf_out);
/* export the leaf layout (key order) for layout parity against a reference tree:
 * rc/sc = record_count/sorted_count, meta words and the first 8 key bytes per slot (cap
 * slots); returns the number of leaves, STAGE_E_ARG if max_leaves < stage_stats[2] */
int64_t stage_export_leaves(stage_table *t, uint32_t cap, uint64_t max_leaves, uint32_t *rc,
                            uint32_t *sc, uint64_t *meta, uint64_t *keyw);

/* ---- leaf-level snapshot in the reference's block format -----------
 * A block is one LeafNode of leaf_node_size bytes exactly as the reference lays it out
 * (b_tree.h:571-740: BaseNode{is_leaf, NodeHeader{size, sorted_count, next_record_slot,
 * StatusWord}} b_tree.h:109-113 / version_store.h:158-231, RecordMetadata{meta, next_ptr,
 * loc_ptr} record_meta.h:30-60 per slot, records [key][pad to 8][payload] growing down).
 * Canonical form: next_ptr (a process pointer: TupleHeader / copy buffer) is 0, loc_ptr is the
 * record's RecordLocation handle (see below; 0 = none), unreferenced record bytes are 0.
 * sep_keys[i]/sep_lens[i] = leaf i's upper bound, the inner-node key that routes to it
 * (GetChildIndex, b_tree.cpp:664-702), len 0xFFFF = +inf for the last leaf.
 * stage_export_leaf_images returns the number of leaves (STAGE_E_ARG if max_leaves is below
 *   stage_stats[2]); blocks holds max_leaves * leaf_node_size bytes; seps may be NULL (both).
 * stage_import_leaf_images loads such a snapshot into an EMPTY table (a quiesced leaf level:
 *   no control bits; version chains are not part of the format).  sep_keys NULL -> each
 *   leaf's largest visible key.  *n_records = visible records imported. */
int64_t stage_export_leaf_images(stage_table *t, uint64_t max_leaves, uint8_t *blocks,
                                 uint64_t *sep_keys, uint16_t *sep_lens);
int stage_import_leaf_images(stage_table *t, const uint8_t *blocks, uint64_t n_leaves,
                             uint32_t block_size, const uint64_t *sep_keys,
                             const uint16_t *sep_lens, uint64_t *n_records);
/* RecordLocation indirection (record_location.h:13-42): the stable name of a record across leaf
 * splits.  The reference allocates one location per Insert attempt
 * (BTree::RecordIndirectLocation, b_tree.cpp:1865-1866, 2034-2050) and LeafNode::CopyFrom
 * repoints it at the record's new slot on every split (b_tree.cpp:1520-1527); handle = the
 * location's allocation index + 1, exported as the RecordMetadata loc_ptr of the leaf images
 * and kept by the import.  A record dropped by a split (deleted / invisible) or an aborted
 * insert loses its location.  leaf = leaf index in key order (= stage_probe_out.leaf).
 * stage_export_locations: every live location (handle order); returns the count (only the
 *   first `max` written).
 * stage_resolve_locations: where each handle's record is now; leaf 0xFFFFFFFF, slot 0xFFFF = none. */
int64_t stage_export_locations(stage_table *t, uint64_t max, uint64_t *handles, uint32_t *leaf,
                               uint16_t *slot);
int stage_resolve_locations(stage_table *t, const uint64_t *handles, uint64_t n, uint32_t *leaf,
                            uint16_t *slot);

/* ---- what the kept transaction manager reads through a Record -----------------------------
 * The reference's Record carries RecordMetadata{meta, next_ptr, loc_ptr} (record_meta.h:30-60)
 * and SSNTransactionManager dereferences two of them (transaction_manager.cpp:29-221, 362-410,
 * 535-815): loc_ptr -> RecordLocation -> record_meta_ptr, the record's CURRENT RecordMetadata
 * wherever splits moved it (FindMaxPstamp :37, FindMinSstamp :123, commit :605), and next_ptr ->
 * EphemeralPool::GetOversionHeader, the in-flight update's overwrite-copy header with its
 * readers (PerformRead :379-399, FindMinSstamp :148-215, FindMaxPstamp :41-97, post-commit
 * READ :753-762).  Here both are stable handles:
 *   location handle  = the RecordLocation's allocation index + 1 (stage_export_locations);
 *   next handle      = 0, STAGE_NEXT_COPY | copy id (the overwrite copy, EphemeralPool's
 *                      location) or STAGE_NEXT_VERSION | version id (the newest TupleHeader).
 * stage_probe_identify: for probe results d_out[0..n) (32-B records of stage_probe_batch on the same
 *   published image, same stream), the hit record's {location handle, next handle} -- the
 *   loc_ptr / next_ptr of the RecordMetadata BTree::Read put in the Record (0/0 for NOT_FOUND).
 *   stage_reader_read_ident is stage_reader_read with the same two handles.
 * stage_location_cells turns on the cells: from then on every host write keeps, per location,
 *   the RecordMetadata it points at as 24 B {meta, next_ptr = next handle, loc_ptr = handle} at a
 *   stable address -- what RecordLocation::record_meta_ptr points at, readable without a call or
 *   a lock from any thread (a dropped location reads meta 0).  stage_location_cell gives the cell
 *   of one handle (valid for the table's lifetime).
 * stage_copy_*: the transaction side of overwrite copy `copy_id` (EphemeralPool::
 *   OverwriteVersionHeader, ephemeral_pool.h:26-150): its stamps, AddReader (BTree::Read for a
 *   read served from the copy, b_tree.cpp:2104-2105), the reader list FindMaxPstamp walks,
 *   IncreaseWRCount (+1, refused -- *ok = 0 -- once the header is waiting) / DecreaseWRCount (-1)
 *   (ephemeral_pool.cpp:69-103) and UpdatePs (:194-205).  The writer's commit (stage_commit_update*)
 *   sets sstamp and waiting (tm.cpp:618-619), its abort waiting with sstamp MAX (:872-875); the
 *   pool never frees a header (no GC).  Thread-safe among themselves and against the writer. */
#define STAGE_NEXT_KIND_MASK 0xC0000000u
#define STAGE_NEXT_COPY 0x40000000u
#define STAGE_NEXT_VERSION 0x80000000u
#define STAGE_NEXT_INDEX_MASK 0x3FFFFFFFu
typedef struct stage_probe_ident {
    uint32_t loc;   /* RecordLocation handle of the hit record (0 = none)                     */
    uint32_t next;  /* the hit slot's next handle (STAGE_NEXT_*), as BTree::Read saw it        */
} stage_probe_ident;
typedef struct stage_copy_state {
    uint32_t cstamp;   /* the writer's id (OverwriteVersionHeader::cstamp)                      */
    uint32_t pstamp;   /* version access stamp: the writer's id until UpdatePs                  */
    uint32_t rstamp;   /* the overwritten version's cstamp                                      */
    uint32_t sstamp;   /* 0xFFFFFFFF until the writer commits                                   */
    uint32_t readers;  /* GetReadersNum                                                         */
    uint16_t count;    /* read dependency count (IncreaseWRCount - DecreaseWRCount)              */
    uint8_t waiting;   /* the writer committed or aborted                                       */
    uint8_t pad;
} stage_copy_state;
int stage_probe_identify(stage_table *t, const stage_probe_out *d_out, uint64_t n, stage_probe_ident *d_ident,
                      void *stream);
/* the host layout's RecordMetadata of the key's record now (SearchRecordMeta on the host leaf):
 * what BTree::Update hands back in meta_upt_ for PerformUpdate (b_tree.cpp:2144-2155) -- meta word
 * and {location handle, next handle}; *rc_out = STAGE_RC_NOT_FOUND when the key has no record */
int stage_record_meta_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint64_t *meta,
                          stage_probe_ident *ident, uint8_t *rc_out);
int stage_location_cells(stage_table *t);
int stage_location_cell(stage_table *t, uint64_t handle, const void **cell);
int stage_copy_get(stage_table *t, const uint32_t *copy_ids, uint64_t n, stage_copy_state *out);
int stage_copy_readers(stage_table *t, uint32_t copy_id, uint32_t *read_ids, uint32_t max, uint32_t *count);
int stage_copy_add_reader(stage_table *t, uint32_t copy_id, uint32_t read_id);
int stage_copy_wr_count(stage_table *t, uint32_t copy_id, int delta, int *ok);
int stage_copy_update_ps(stage_table *t, uint32_t copy_id, uint32_t pstamp);

/* ---- device batch path (the replaced hot path) ------------------------------------------
 * stage_probe_batch  replaces LeafNode::Read/SearchRecordMeta (b_tree.cpp:1042-1051, 18-122),
 *   Record::New/Neww (b_tree.h:407-448), BTree::Read (b_tree.cpp:2066-2129) and the
 *   visibility walk of IndexScanExecutor (executor.h:374-454), batched.
 *   d_keys: stage_key_words(t) u64 words per key, key bytes little-endian (one word for
 *   keys of <= 8 bytes); d_lens NULL -> table key_width;
 *   d_read_ids NULL -> 0xFFFFFFFE; d_leaf_ids NULL -> device traversal of the separator
 *   mirror, else host-traversed leaf indices (stage_traverse_batch).
 *   d_records: n rows of stage_record_stride() bytes = [key padded to 8][payload]; NULL to
 *   skip the tuple copy.
 * stage_scan_batch replaces BTree::RangeScanBySize + Iterator::GetNext + TableScanExecutor
 *   (b_tree.h:830-953, b_tree.cpp:1261-1315, executor.h:611-642): for each start key up to
 *   scan_size tuples in KeyCompare order into d_records[i*scan_size + j], count in d_counts.
 * stage_resolve_batch: device traversal only (le_child as TraverseToLeaf).
 * stage_set_output_layout: stage_probe_batch's output layout (default 0, 32): row_stride 0 =
 *   stage_record_stride's default (the row rounded to 128 B above 128 B), else any multiple of
 *   16 of at least key pad + payload (e.g. 1008 for YCSB rows: no pad bytes written);
 *   status_bytes 32 = stage_probe_out, 16 = stage_probe_out16 records in d_out (fixed-width
 *   keys of <= 8 bytes in 64-slot leaves).  Both apply to stage_probe_host too (its `out`
 *   then holds n packed stage_probe_out16 records); every other entry point keeps 32-B
 *   records. */
int stage_set_output_layout(stage_table *t, uint32_t row_stride, uint32_t status_bytes);
int stage_probe_batch(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens,
                      const uint32_t *d_read_ids, const uint32_t *d_leaf_ids, uint64_t n,
                      stage_probe_out *d_out, uint8_t *d_records, void *stream);
/* stage_probe_batch with BTree::Read's is_for_update per probe (b_tree.h:812-813; the
 *   IndexScanExecutor point lookup of a transaction reading its own record, executor.h:376-388;
 *   e.g. the TPC-C drivers' executors built with is_for_update, tpcc_delivery.cpp:104).
 *   d_for_update[i] != 0: the record is read from the leaf even while an update is in flight
 *   (b_tree.cpp:2087 takes the overwrite copy only when !is_for_update; :2114-2120 Record::New,
 *   cstamp = the reader's id, no AddReader), i.e. the writer sees its own patched image; the
 *   executor rule is then the same (read id >= the record's cstamp -> LATEST, else the chain)
 *   with PerformRead skipped, which STAGE_FLAG_FOR_UPDATE in the status record says.  An
 *   uncommitted insert is found by its own writer (the ordinary rule returns nothing for it).
 *   d_for_update NULL = stage_probe_batch.  32-B status records only (STAGE_E_UNSUPPORTED with
 *   stage_set_output_layout(.., 16)). */
int stage_probe_batch_ex(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens,
                         const uint32_t *d_read_ids, const uint32_t *d_leaf_ids, const uint8_t *d_for_update,
                         uint64_t n, stage_probe_out *d_out, uint8_t *d_records, void *stream);
int stage_scan_batch(stage_table *t, const uint64_t *d_start_keys, const uint16_t *d_lens,
                     uint64_t n, uint32_t scan_size, uint32_t *d_counts, uint8_t *d_records,
                     void *stream);
int stage_resolve_batch(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens, uint64_t n,
                        int le_child, uint32_t *d_leaf, void *stream);
/* IndexScanExecutor::Execute range branch (executor.h:456-530): the scan of stage_scan_batch
 * with per-record visibility for d_read_ids[i] (NULL -> 0xFFFFFFFE).  For iterator record j
 * of scan i: d_row_status[i*scan_size + j] = STAGE_ST_LATEST (the leaf record, read_id >= its
 * commit id), STAGE_ST_OLD (the TupleHeader version with begin <= read_id <= end) or
 * STAGE_ST_NOT_FOUND (nothing produced; row zeroed); d_counts[i] = records consumed. */
int stage_index_scan_batch(stage_table *t, const uint64_t *d_start_keys, const uint16_t *d_lens,
                           const uint32_t *d_read_ids, uint64_t n, uint32_t scan_size,
                           uint32_t *d_counts, uint8_t *d_records, uint8_t *d_row_status,
                           void *stream);
/* The IndexScanExecutor range branch of stage_index_scan_batch consumed only up to its first
 * produced tuple (LATEST or OLD) whose key begins with the start key's first `prefix_words`
 * 8-byte fields (0..key_words) -- the predicate TPC-C stock-level puts on its ORDER_LINE scans
 * (tpcc_stock_level.cpp:104-135 keeps ol_i_ids[0]).  Fixed-width keys of 9..32 bytes (or 8),
 * scan_size 1..63.  d_image[i] = the tuple's record-heap row (0xFFFFFFFF if none),
 * d_status[i] = STAGE_ST_LATEST / STAGE_ST_OLD / STAGE_ST_NOT_FOUND. */
int stage_index_scan_first_batch(stage_table *t, const uint64_t *d_start_keys, const uint32_t *d_read_ids,
                                 uint64_t n, uint32_t scan_size, uint32_t prefix_words, uint32_t *d_image,
                                 uint8_t *d_status, void *stream);

/* ---- host-buffer forms (keys and results in host memory) --------------------------------
 * stage_probe_host: stage_probe_batch for host buffers; the batch is cut into chunks that
 *   rotate over three streams so H2D, probe and D2H overlap.  Pass pinned buffers
 *   (stage_host_alloc) for full PCIe rate; pageable buffers work but copy through HIP's staging.
 *   Calls on one table are serialised.
 * stage_reader_*: the single-key adapter for BTree::Read callers (b_tree.cpp:2066-2129 as used
 *   by IndexScanExecutor::Execute, executor.h:374-454, from every worker thread).  Thread-safe:
 *   concurrent stage_reader_read calls are coalesced into one device batch of up to max_batch
 *   keys, shipped when full or when its oldest request has waited max_wait_us; each call
 *   blocks until its own result (stage_probe_out + [key padded to 8][payload] in `record`,
 *   either may be NULL) is filled.  stats[0] = batches, [1] = reads, [2] = full batches.
 *   Writers must not stage_sync while readers are running (the host is the single writer and
 *   publishes between epochs, as for every other device entry point).
 * stage_reader_create_resident: the same adapter without a launch per batch: `waves` one-wave
 *   workgroups stay resident on the device and poll a ring of `ring_slots` requests (a multiple
 *   of 64 * waves; consecutive tickets go to different waves) in pinned host memory; a caller takes a ticket, writes its request into the slot,
 *   publishes it and spins until the device publishes the results in the slot.  Each device
 *   instance ends after `life_us` (a keeper thread queues the next one behind it, so no wave
 *   outlives a bounded lifetime).  stage_reader_read / _stats / _destroy take either kind;
 *   for the resident kind stats[0] = device instances launched, [1] = reads, [2] = 0.  Keys of
 *   <= 8 bytes; a table that needs stage_sync ends the reader (reads fail with STAGE_E_STATE). */
typedef struct stage_reader stage_reader;
int stage_host_alloc(uint64_t bytes, void **ptr);
int stage_host_free(void *ptr);
int stage_probe_host(stage_table *t, const uint64_t *keys, const uint16_t *lens,
                     const uint32_t *read_ids, uint64_t n, stage_probe_out *out, uint8_t *records);
int stage_reader_create(stage_table *t, uint32_t max_batch, uint32_t max_wait_us,
                        stage_reader **out);
int stage_reader_create_resident(stage_table *t, uint32_t ring_slots, uint32_t waves, uint32_t life_us,
                                 stage_reader **out);
int stage_reader_read(stage_reader *r, uint64_t key, uint16_t key_size, uint32_t read_id,
                      stage_probe_out *out, uint8_t *record);
int stage_reader_read_ident(stage_reader *r, uint64_t key, uint16_t key_size, uint32_t read_id,
                            stage_probe_out *out, uint8_t *record, stage_probe_ident *ident);
/* stage_reader_read_ident with BTree::Read's is_for_update (see stage_probe_batch_ex); either
 * reader kind */
int stage_reader_read_ex(stage_reader *r, uint64_t key, uint16_t key_size, uint32_t read_id, int is_for_update,
                         stage_probe_out *out, uint8_t *record, stage_probe_ident *ident);
int stage_reader_stats(stage_reader *r, uint64_t *stats);
int stage_reader_destroy(stage_reader *r);

/* launch shape of stage_probe_batch: probes in flight per wave (1, 2, 4 or 8) and the grid
 * cap in 256-thread blocks (0 = default).  A tuning knob, not a semantic one. */
int stage_set_probe_tuning(stage_table *t, int group, int max_blocks);

/* cache policy of stage_probe_batch's output stores (rows + status records), 8-probe launch
 * shape: STAGE_STORE_TEMPORAL, STAGE_STORE_NONTEMPORAL (default) or STAGE_STORE_WRITE_THROUGH
 * (the output lines leave the GPU's L2 at once, which keeps hot rows and index lines cached).
 * A tuning knob, not a semantic one. */
#define STAGE_STORE_TEMPORAL 0
#define STAGE_STORE_NONTEMPORAL 1
#define STAGE_STORE_WRITE_THROUGH 2
int stage_set_probe_store(stage_table *t, int policy);

/* MurmurHash64A (misc/murmur/MurmurHash2.cpp:99-147) over n keys of key_len bytes laid out
 * key_stride bytes apart; d_out[i] = hash.  Used as the multi-GPU shard router. */
int stage_murmur64a_batch(const void *d_keys, uint32_t key_len, uint32_t key_stride, uint64_t seed,
                          uint64_t n, uint64_t *d_out, void *stream);

/* ---- TPC-C stock-level through the path (tpcc_stock_level.cpp:37-180), batched -----------
 * district: DistrictKey{int64 D_W_ID, int64 D_ID} (16 B) table whose payload starts with
 * D_NEXT_O_ID (int32); order_line: OrderLineKey{W, D, O, NUMBER} (32 B), payload starts with
 * OL_I_ID (int32); stock: StockKey{W, I} (16 B), payload starts with S_QUANTITY (int32)
 * (tpcc_record.h GetData layouts).  Transaction i = (d_w_ids[i], d_d_ids[i],
 * d_thresholds[i], read id d_read_ids[i] or 0xFFFFFFFE): DISTRICT point lookup; for the 20
 * orders below D_NEXT_O_ID an ORDER_LINE range scan of 10 records from {w, d, o, 5} with
 * IndexScanExecutor visibility, keeping OL_I_IDs of (w, d, o); a STOCK point lookup of each
 * scan's first item; d_result[i] = number of distinct S_I_IDs with S_QUANTITY < threshold,
 * or -1 when the transaction aborts (FAILURE / missing district).  All device-resident: three
 * batched probe/scan launches and four small glue kernels, no host round trip. */
int stage_tpcc_stock_level(stage_table *district, stage_table *order_line, stage_table *stock,
                           const int64_t *d_w_ids, const int64_t *d_d_ids, const int32_t *d_thresholds,
                           const uint32_t *d_read_ids, uint64_t n, int32_t *d_result, void *stream);

/* ---- CH-benCHmark Q2 -------------------------------------------------
 * RunQuery2 (benchmark/tpcc/tpcc_new_order.cpp:608-982) at read id `read_id` over REGION /
 * NATION / SUPPLIER / ITEM (8-byte keys; payloads R_NAME.., N_REGIONKEY.., SU_NATIONKEY..,
 * I_IM_ID I_NAME I_PRICE I_DATA, tpcc_record.h:160-200, 773-880) and STOCK ({S_W_ID, S_I_ID},
 * 16 bytes; payload S_QUANTITY S_YTD S_ORDER_CNT S_REMOTE_CNT .., :417-500).  The region named
 * regions[target_region] (tpcc_record.h:931), its nations, their suppliers (every SUPPLIER
 * record); per supplier the STOCK lookups of its supp_stock_map entries (tpcc_workload.cpp:
 * 398-404, given as host CSR offsets map_off[10001] + device keys d_map_keys, two words {w, i}
 * per entry in push order), the ITEM lookup of the last stock's S_I_ID, the I_DATA ('b') and
 * S_QUANTITY < 10 tests.  out[k]: one record per visited supplier (nation order, then supplier
 * key order; *n_out of them, at most max_out copied); *aborted = 1 where the reference aborts
 * (a FAILURE read, or a STOCK / ITEM lookup without a tuple).  commit_id != 0 and not aborted:
 * the marked updates (S_QUANTITY..S_REMOTE_CNT = q + 50, ytd, order_cnt, remote_cnt) are
 * applied through stage_update_batch_device (writer read_id, commit commit_id), update_rc =
 * their return codes. */
typedef struct stage_q2_rec {
    int64_t supp_key, s_w_id, s_i_id;  /* supplier; the stock its loop kept (the last one read) */
    int32_t s_quantity, s_ytd, s_order_cnt, s_remote_cnt;
    uint8_t item_has_b, update, update_rc, pad[5];
} stage_q2_rec;
int stage_ch_query2(stage_table *region, stage_table *nation, stage_table *supplier, stage_table *item,
                    stage_table *stock, const uint32_t *map_off, const uint64_t *d_map_keys, int32_t target_region,
                    uint32_t read_id, uint32_t commit_id, stage_q2_rec *out, uint64_t max_out, uint64_t *n_out,
                    int32_t *aborted, void *stream);

/* nq read-only Q2 transactions at read_ids[0..nq) in one pass (the scans once, every
 * query's STOCK / ITEM lookups in the same launches): out[q * max_per_query + k],
 * aborted[q]; *n_out = records per query (the visited suppliers do not depend on the read
 * id: the scans are TableScanExecutor ones, without visibility).  No updates are applied.
 * Each STOCK / ITEM key is probed once and its hit slot's visibility evaluated at every read
 * id.  `out` in page-locked memory (stage_host_alloc) with max_per_query >= *n_out: the
 * records are copied into it straight from the device (both entry points). */
int stage_ch_query2_batch(stage_table *region, stage_table *nation, stage_table *supplier, stage_table *item,
                          stage_table *stock, const uint32_t *map_off, const uint64_t *d_map_keys,
                          int32_t target_region, const uint32_t *read_ids, uint32_t nq, stage_q2_rec *out,
                          uint64_t max_per_query, uint64_t *n_out, int32_t *aborted, void *stream);
/* the same batch without waiting for it: enqueued on `stream` into slot 0 or 1 (two batches
 * may be in flight, the host enqueueing one while the device runs the other); `out` must be
 * page-locked (stage_host_alloc) and stay untouched until stage_ch_query2_wait(slot) returns
 * *n_out and aborted[nq].  STAGE_E_STATE: the slot still holds a batch not waited for.
 * The two slots (and a synchronous batch) share the tables' device scratch: a batch enqueued on
 * another stream than a batch still in flight first waits for it on the device
 * (hipStreamWaitEvent), so batches on different streams are correct but do not overlap; on one
 * stream they overlap the host's staging of the next batch with the device's run of the last.
 * The records are finished into the slot's own device buffer and reach `out` by a copy on a
 * side stream, beside the next batch's kernels; records past *n_out in a query's row of `out`
 * are unspecified (the copy takes the previous batch's count per query, the wait the rest). */
int stage_ch_query2_batch_async(stage_table *region, stage_table *nation, stage_table *supplier,
                                stage_table *item, stage_table *stock, const uint32_t *map_off,
                                const uint64_t *d_map_keys, int32_t target_region, const uint32_t *read_ids,
                                uint32_t nq, stage_q2_rec *out, uint64_t max_per_query, int slot, void *stream);
int stage_ch_query2_wait(stage_table *stock, int slot, uint64_t *n_out, int32_t *aborted);
/* self-check of the multi-table operations' device scratch plans, no device work: op 0 = CH-Q2
 * (users: the batch buffers, the REGION scan rows, the NATION scan rows, the stock-update
 * staging; roles 0..4 = region, nation, supplier, item, stock), op 1 = TPC-C stock-level (its
 * batch buffers, role 0 = district).  roles NULL: the library's own plan; else n roles, one per
 * user (e.g. a past layout).  STAGE_OK when no two users share one table's per-call scratch,
 * STAGE_E_ARG naming them otherwise.  Every CH-Q2 call runs the same check on the tables it is
 * given and refuses one table passed for two roles whose scratch users would collide. */
int stage_scratch_plan_check(int op, const int32_t *roles, int n);

/* ---- multi-GPU: hash-sharded probe front-end over RCCL (one process per GPU) ------------
 * stage_comm_unique_id fills 128 bytes on rank 0 (broadcast them out of band);
 * stage_comm_init joins the communicator; stage_probe_sharded routes each key to rank
 * MurmurHash64A(key, key_width, 0) % world, probes it there and returns the results in the
 * caller's order (all-to-all-v out, local probe, all-to-all-v back). */
int stage_comm_unique_id(uint8_t *id128);
/* the sharded batch's requests are exchanged in `chunks` pieces whose result transfers overlap
 * the next piece's probe (0 = STAGE_SHARD_CHUNKS env, or 4 -- 1 at world 1); set before
 * stage_comm_init, same value on every rank */
int stage_set_shard_chunks(stage_table *t, int chunks);
int stage_comm_init(stage_table *t, const uint8_t *id128, int rank, int world);
int stage_comm_destroy(stage_table *t);
int stage_probe_sharded(stage_table *t, const uint64_t *d_keys, const uint32_t *d_read_ids,
                        uint64_t n, stage_probe_out *d_out, uint8_t *d_records, void *stream);
/* reply modes: STAGE_REPLY_ROWS = status records and tuple rows come back to the caller (what
 * stage_probe_sharded does); STAGE_REPLY_OWNER = the owner materialises the tuple rows in its
 * own HBM result buffer and only the 32-B status records come back, each carrying the row's
 * owner-local index in `meta_hi` (owner rank = MurmurHash64A(key, 8, 0) % world); the owner
 * reads its buffer with stage_sharded_owner_rows (valid until its next sharded probe). */
#define STAGE_REPLY_ROWS 0
#define STAGE_REPLY_OWNER 1
/* STAGE_REPLY_PEER: what STAGE_REPLY_ROWS returns (status records and rows at the caller's
 * positions), but only the 32-B status records travel over RCCL: each owner keeps the rows of the
 * remote requests it probed in one of two row buffers of its own (by call parity) and the caller's
 * fan-out reads each row there -- over xGMI, through the owner's buffers opened by IPC handle
 * (hipIpcGetMemHandle / hipIpcOpenMemHandle, handles exchanged over the communicator when a buffer
 * grows).  No RCCL receive buffer is written and read back for the rows.  Every rank knows every
 * rank's send counts (an allgather instead of the count all-to-all), hence where each owner put
 * each row.  d_records required; at world 1 the same as STAGE_REPLY_ROWS. */
#define STAGE_REPLY_PEER 2
/* STAGE_REPLY_DIRECT: what STAGE_REPLY_ROWS returns, with each owner probing a remote request
 * straight into its caller's d_out / d_records -- status record and row at the request's first
 * caller position, carried in the request record -- through the caller's buffers opened by IPC
 * handle (each rank's (allocation handle, offset) pairs travel with the send counts every call;
 * a mapping is reopened when its allocation changes).  Over RCCL only the keys go out and a 16-B
 * token per chunk and peer comes back, after the owner's system-scope release; the caller then
 * acquires and copies its coalesced requests' duplicates from their first positions.  The rows
 * cross xGMI once and land once.  Tables of the YCSB geometry (8-byte keys, 64-slot leaves, rows
 * <= 1024 B); d_records required; d_out and d_records must be IPC-exportable device memory
 * (hipMalloc); at world 1 the same as STAGE_REPLY_ROWS. */
#define STAGE_REPLY_DIRECT 3
int stage_probe_sharded_ex(stage_table *t, const uint64_t *d_keys, const uint32_t *d_read_ids,
                           uint64_t n, stage_probe_out *d_out, uint8_t *d_records, int reply_mode,
                           void *stream);
/* loopback != 0: the buffer of stage_probe_sharded_loopback's shard state */
int stage_sharded_owner_rows(stage_table *t, int loopback, uint8_t **d_rows, uint64_t *n_rows);
/* request coalescing (default on; STAGE_SHARD_DEDUPE=0 or on = 0 turns it off, -1 = the env
 * default): requests with equal (key, read id) anywhere in the batch are routed and probed once
 * (runs of more than 64 callers are cut into requests of at most 64) and the result is copied to
 * every caller position -- results are identical, the key and tuple traffic over xGMI shrinks by
 * the batch's duplicate share (55 % of a 16M-key Zipf-0.9 batch over 100M rows).  Owner-reply
 * rows are then one per request. */
int stage_set_shard_dedupe(stage_table *t, int on);
/* coalescing sorts the batch's keys on their low `bits` bits (0 or 64 = all; default 64).  Any
 * value gives the same results -- keys equal in those bits but different above them still form
 * separate requests -- a caller whose keys are < 2^bits only saves radix passes.  bits <= 32
 * (batches without read ids): the sort moves 32-bit key words and positions instead of 64-bit
 * keys; a batch holding a key above 2^32 is still answered exactly (its keys are gathered back
 * by position). */
int stage_set_shard_key_bits(stage_table *t, int bits);
/* the RCCL the process runs: ncclGetVersion (e.g. 22707 = 2.27.7), the RCCL header version
 * libstage_hip was built against, and the file that provided ncclGetVersion.  stage_comm_init
 * fails (STAGE_E_HIP; stage_last_error names both versions and the file) when the runtime
 * major.minor differs from the headers, unless STAGE_RCCL_ALLOW_MISMATCH=1. */
int stage_rccl_info(int *runtime_version, int *header_version, char *path, uint64_t path_len);
/* the last sharded probe on this rank: caller keys, requests routed after coalescing, and of
 * those the ones owned by other ranks (loopback != 0: the loopback shard state) */
int stage_sharded_stats(stage_table *t, int loopback, uint64_t *n_keys, uint64_t *n_routed, uint64_t *n_remote);
/* the same and more: v[0..nv) = {caller keys, requests routed, of those remote, requests this
 * rank probed as owner (its own + the ones other ranks routed to it)} */
int stage_sharded_stats_ex(stage_table *t, int loopback, uint64_t *v, int nv);
/* control plane over the table's communicator, for callers without another one (the bench's
 * barrier, max-over-ranks timing and per-rank reports): in-place allreduce of n doubles (op 0
 * sum, 1 max, 2 min) and allgather (out[r * n + i] = rank r's in[i]); both wait for completion */
int stage_comm_allreduce_f64(stage_table *t, double *values, uint64_t n, int op);
int stage_comm_allgather_f64(stage_table *t, const double *in, uint64_t n, double *out);

/* single-process rehearsal of stage_probe_sharded: `world` shard tables on ONE device play the
 * ranks; the routing, count exchange, offsets, local probes and un-permutation are the same
 * code, with device-to-device copies where the RCCL path has ncclSend/ncclRecv.  Arrays are
 * indexed by rank (d_read_ids may be NULL; d_records all NULL or none).  For testing the
 * multi-GPU data path on one GPU. */
int stage_probe_sharded_loopback(stage_table *const *shards, int world, const uint64_t *const *d_keys,
                                 const uint32_t *const *d_read_ids, const uint64_t *n,
                                 stage_probe_out *const *d_out, uint8_t *const *d_records,
                                 int reply_mode, void *stream);

/* ---- plumbing for callers without their own HIP binding (ctypes) ----------------------- */
int stage_set_device(int device);
int stage_device_count(int *count);
int stage_dev_alloc(uint64_t bytes, void **ptr);
int stage_dev_free(void *ptr);
int stage_dev_memset(void *ptr, int value, uint64_t bytes, void *stream);
int stage_memcpy_h2d(void *dst, const void *src, uint64_t bytes, void *stream);
int stage_memcpy_d2h(void *dst, const void *src, uint64_t bytes, void *stream);
int stage_stream_create(void **stream);
int stage_stream_destroy(void *stream);
int stage_stream_sync(void *stream);
int stage_device_sync(void);
/* event pair timing on `stream`: returns the elapsed milliseconds between two records */
int stage_event_create(void **ev);
int stage_event_destroy(void *ev);
int stage_event_record(void *ev, void *stream);
int stage_event_elapsed(void *ev_start, void *ev_stop, float *ms);

/* ---- YCSB harness generators (benchmark/benchmark_common.h:12-105) -----------------------
 * FastRandom(seed) stream and ZipfDistribution(n, theta).GetNextNumber() draws in [1, n], the
 * generator seeded FastRandom(seed) (the reference seeds it with rand()); stage_zipf_zeta =
 * ZipfDistribution::zeta (benchmark_common.h:80-84), bit-identical to its serial sum. */
int stage_fastrandom_next(uint64_t seed, uint64_t count, uint64_t *out);
int stage_zipf_draws(uint64_t n, double theta, uint64_t seed, uint64_t count, uint64_t *out,
                     int nthreads);
int stage_zipf_zeta(uint64_t n, double theta, double *out);
/* RunMixed's operation stream (benchmark/ycsb/ycsb_mixed.cpp:26-44) from FastRandom(seed): op i
 * is an update when NextUniform() < update_ratio (is_update[i] = 1) and then draws its delta
 * byte chr[i] = next_char() (the 100-B column patch memset to it); a read draws nothing more
 * (chr[i] = 0). */
int stage_ycsb_ops(uint64_t seed, uint64_t count, double update_ratio, uint8_t *is_update, uint8_t *chr);

#ifdef __cplusplus
}
#endif
#endif
