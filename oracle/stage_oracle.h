/*
 * stage_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker, never product code).
 *
 * Plain-C restatement of the reference's index-organized hot path
 * (sheepTnT/Stage-IndexOrganized @ 2024-12-18):
 *   - signed-byte key order            include/vstore/b_tree.h:99-134
 *   - 64-bit RecordMetadata word       include/vstore/record_meta.h:30-204
 *   - BzTree leaf image / insert/split src/vstore/b_tree.cpp:809-947, 1558-1690, 1849-2020
 *   - inner nodes + GetChildIndex      src/vstore/b_tree.cpp:363-702
 *   - leaf probe SearchRecordMeta      src/vstore/b_tree.cpp:18-122, 1042-1051
 *   - BTree::Read (+copy path)         src/vstore/b_tree.cpp:2066-2129
 *   - point-lookup visibility          include/execute/executor.h:374-454
 *   - RangeScanBySize + Iterator       src/vstore/b_tree.cpp:1261-1315, b_tree.h:883-953,
 *                                      executor.h:611-642 (TableScanExecutor)
 *   - update/commit (version chain)    b_tree.cpp:1061-1163, transaction_manager.cpp:610-676
 *   - MurmurHash64A                    misc/murmur/MurmurHash2.cpp:99-147
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline.
 */
#ifndef STAGE_ORACLE_H_
#define STAGE_ORACLE_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ReturnCode values, b_tree.h:42-54 */
enum { ORC_RET_INVALID = 0, ORC_RET_OK = 1, ORC_RET_KEY_EXISTS = 2, ORC_RET_NOT_FOUND = 3,
       ORC_RET_NODE_FROZEN = 4, ORC_RET_CAS_FAIL = 5, ORC_RET_NOT_ENOUGH_SPACE = 6,
       ORC_RET_NOT_NEEDED_UPDATE = 7, ORC_RET_RETRY_FAILURE = 8, ORC_RET_DIRTY = 9 };

/* canonical per-probe outcome of BTree::Read + IndexScanExecutor */
enum { ORC_ST_NOT_FOUND = 0, ORC_ST_LATEST = 1, ORC_ST_COPY = 2, ORC_ST_OLD = 3,
       ORC_ST_FAIL_INVALID_TS = 4, ORC_ST_CHAIN_MISS = 5 };

typedef struct orc_read_out {
    uint8_t status;        /* ORC_ST_* */
    uint8_t copy_present;  /* PerformRead found an overwrite header for meta.next_ptr */
    uint16_t hops;         /* TupleHeader hops walked */
    uint32_t cstamp;       /* Record cstamp: latest -> reader id, copy -> rstamp, old -> begin */
    uint32_t rec_cstamp;   /* meta.GetTxnCommitId() of the hit slot */
    uint32_t copy_sstamp;  /* overwrite header sstamp (MAX_CID if none) */
} orc_read_out;

typedef struct orc_tree orc_tree;

/* ParameterSet(split_threshold, merge_threshold, leaf_node_size, payload_size), b_tree.h:23-40 */
orc_tree *orc_tree_new(uint32_t leaf_node_size, uint32_t split_threshold, uint32_t payload_size);
void orc_tree_set_merge_threshold(orc_tree *t, uint32_t merge_threshold);
void orc_tree_free(orc_tree *t);

/* BTree::Insert + BTree::FinalizeInsert (loader semantics, ycsb_loader.cpp:152-171) */
int orc_insert(orc_tree *t, const uint8_t *key, uint32_t key_size, const uint8_t *payload,
               uint32_t commit_id);
/* an uncommitted transaction's insert (PrepareForInsert, cstamp = writer id) and its commit */
int orc_insert_inflight(orc_tree *t, const uint8_t *key, uint32_t key_size, const uint8_t *payload,
                        uint32_t writer_id);
int orc_commit_insert(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id);
/* LoadYCSBRows (ycsb_loader.cpp:93-171) single loader, rows [begin,end), key = rowid as
 * key_size (4 or 8) little-endian bytes.  payload_mode 0 = reference memset(rowid),
 * 1 = "strong" per-word pattern (stage_payload_word).  Returns rows inserted. */
uint64_t orc_load_ycsb(orc_tree *t, uint64_t begin, uint64_t end, uint32_t key_size,
                       int payload_mode);
/* insert keys[i] (key_size-byte little-endian) in the given order, payload from rowid=keys[i] */
uint64_t orc_load_keys(orc_tree *t, const uint64_t *keys, uint64_t n, uint32_t key_size,
                       int payload_mode);

/* point lookup: rec receives [key padded to 8][payload] (8 + payload_size bytes), zeroed
 * when no tuple is produced. */
int orc_read(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t read_id,
             orc_read_out *out, uint8_t *rec);
/* orc_read with BTree::Read's is_for_update (b_tree.cpp:2087, 2114-2120): an in-flight record is
 * read from the leaf (the writer's own image), never from its overwrite copy */
int orc_read_fu(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t read_id, int for_update,
                orc_read_out *out, uint8_t *rec);
/* the writer's own record (is_for_update = true): LeafNode::Update's in-place branch
 * (b_tree.cpp:1101-1104) and LeafNode::Delete's meta := 0 branch (:1210-1220) */
int orc_update_owned(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t payload_off, const uint8_t *delta,
                     uint32_t delta_len, uint32_t writer_id);
int orc_delete_owned(orc_tree *t, const uint8_t *key, uint32_t key_size);
/* batch of little-endian u64 keys of key_size bytes; rec may be NULL (only outs). */
int orc_read_batch(orc_tree *t, const uint64_t *keys, uint32_t key_size, const uint32_t *read_ids,
                   uint64_t n, orc_read_out *outs, uint8_t *recs, int nthreads);
/* timing helper for the CPU baseline: same work as orc_read_batch, records written to a
 * per-thread scratch row (the reference hands every Record to the caller and frees it).
 * Returns a checksum of the records so nothing is optimised away. */
uint64_t orc_read_batch_timed(orc_tree *t, const uint64_t *keys, uint32_t key_size,
                              const uint32_t *read_ids, uint64_t n, int nthreads,
                              double *seconds);

/* CPU baseline full-txn mode: n_txns read-only RunMixed transactions of ops_per_txn reads
 * (keys[x*ops_per_txn + op]) through the IndexScanExecutor point-lookup branch and the
 * Index-SSN read side (PerformRead, CommitTransaction); tid_counter starts at first_tid.
 * results[0] = commits, results[1] = aborts, results[2] = checksum. */
void orc_ycsb_txn_timed(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint32_t ops_per_txn, uint64_t n_txns,
                        int nthreads, uint32_t first_tid, double *seconds, uint64_t *results);
/* LoadYCSBRows built by nthreads threads: the same leaves as orc_load_ycsb, inner levels
 * rebuilt bottom-up (same routing); for the CPU baseline's large tables */
uint64_t orc_load_ycsb_parallel(orc_tree *t, uint64_t begin, uint64_t end, uint32_t key_size, int payload_mode,
                                int nthreads);
/* a load of distinct keys skips LeafNode::Insert's CheckUnique (same leaves, faster build) */
void orc_tree_set_bulk(orc_tree *t, int bulk);

/* TableScanExecutor (scan_sz >= 0) over RangeScanBySize/Iterator.  recs receives up to
 * scan_size rows of [key padded 8][payload]; returns the number of records produced. */
uint32_t orc_scan(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t scan_size,
                  uint8_t *recs);
uint64_t orc_scan_batch(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n,
                        uint32_t scan_size, uint32_t *counts, uint8_t *recs, int nthreads);
/* CPU baseline for scans: TableScanExecutor copies every record into its result vector
 * (executor.h:637); rows go to a per-thread scratch buffer.  Returns records produced. */
uint64_t orc_scan_batch_timed(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n,
                              uint32_t scan_size, int nthreads, double *seconds);

/* host-side traversal result (BTree::TraverseToLeaf): leaf index in key order */
int64_t orc_traverse_leaf_index(orc_tree *t, const uint8_t *key, uint32_t key_size, int le_child);

/* write path used to construct visibility scenarios (single writer):
 *   orc_update        = BTree::Update / LeafNode::Update (b_tree.cpp:1061-1163): in-place column
 *                       patch of payload[payload_off, +delta_len), old image into a copy buffer.
 *   orc_commit_update = CommitTransaction UPDATE branch (transaction_manager.cpp:610-676):
 *                       TupleHeader{begin=rstamp, end=sstamp}, meta cstamp := commit_id,
 *                       next := TupleHeader.
 *   orc_finalize_update = BTree::FinalizeUpdate (b_tree.cpp:2252-2268, test style).
 *   orc_delete          = BTree::Delete + FinalizeDelete (no merge). */
int orc_update(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t payload_off,
               const uint8_t *delta, uint32_t delta_len, uint32_t writer_id);
int orc_commit_update(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id,
                      uint32_t sstamp);
uint64_t orc_update_batch(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n, uint32_t payload_off,
                          const uint8_t *deltas, uint32_t delta_len, const uint32_t *wid, const uint32_t *cid,
                          uint8_t *rc);
/* the same epoch with nthreads concurrent writers, each key's ops on one writer in batch order
 * (rc and every record's final state equal orc_update_batch's); seconds = wall time of the writers */
uint64_t orc_update_batch_mt(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n, uint32_t payload_off,
                             const uint8_t *deltas, uint32_t delta_len, const uint32_t *wid, const uint32_t *cid,
                             uint8_t *rc, int nthreads, double *seconds);
/* AbortTransaction UPDATE / INSERT entries (transaction_manager.cpp:846-921, 949-979) */
int orc_abort_update(orc_tree *t, const uint8_t *key, uint32_t key_size);
int orc_abort_insert(orc_tree *t, const uint8_t *key, uint32_t key_size);
int orc_finalize_update(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id);
int orc_delete(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id);

/* stats[0]=height stats[1]=inner nodes stats[2]=leaves stats[3]=records stats[4]=sorted slots
 * stats[5]=unsorted slots stats[6]=max records/leaf stats[7]=retired versions */
void orc_stats(orc_tree *t, uint64_t *stats);
/* leaves in key order: rc[i]=record_count, sc[i]=sorted_count; slot arrays (cap per leaf):
 * meta[i*cap+s], key bytes as little-endian u64 keyw[i*cap+s]; returns number of leaves,
 * or -(needed) when max_leaves is too small. */
/* leaves in key order as reference-format blocks of leaf_node_size bytes (pointers zeroed,
 * dead record bytes zeroed) + each leaf's upper separator (len 0xFFFF = +inf) */
int64_t orc_export_leaf_images(orc_tree *t, uint64_t max_leaves, uint8_t *blocks, uint64_t *sep_key,
                               uint16_t *sep_len);
/* the same with kwords u64 words of separator key bytes per leaf (keys above 8 bytes) */
int64_t orc_export_leaf_images_k(orc_tree *t, uint64_t max_leaves, uint8_t *blocks, uint64_t *sep_key,
                                 uint32_t kwords, uint16_t *sep_len);
/* IndexScanExecutor range branch (executor.h:456-530): the iterator records of a scan of
 * scan_size with per-record visibility for read_id; status[j] = 1 latest, 3 old version,
 * 0 nothing (row zeroed).  Returns the number of iterator records consumed. */
uint32_t orc_index_scan(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t scan_size, uint32_t read_id,
                        uint8_t *recs, uint8_t *status);
/* bulk insert of explicit rows (key i at keys + i*key_stride, payload i at payloads + i*payload_stride) */
uint64_t orc_load_rows(orc_tree *t, const uint8_t *keys, uint32_t key_stride, uint32_t key_size,
                       const uint8_t *payloads, uint32_t payload_stride, uint64_t n);
/* TPC-C stock-level (tpcc_stock_level.cpp:37-180): distinct items below threshold, -1 = abort */
int32_t orc_stock_level(orc_tree *dist, orc_tree *ol, orc_tree *stock, int64_t w, int64_t d, int32_t threshold,
                        uint32_t read_id);
void orc_stock_level_batch(orc_tree *dist, orc_tree *ol, orc_tree *stock, const int64_t *w, const int64_t *d,
                           const int32_t *thr, const uint32_t *rid, uint64_t n, int32_t *res, int nthreads,
                           double *seconds);
/* canonical tuple rows [key padded to key_pad][payload]; default 8 (keys of <= 8 bytes) */
void orc_tree_set_key_pad(orc_tree *t, uint32_t key_pad);
/* batch forms over byte keys (key i at keys + i*key_stride) */
int orc_read_batch_k(orc_tree *t, const uint8_t *keys, uint32_t key_stride, uint32_t key_size,
                     const uint32_t *read_ids, uint64_t n, orc_read_out *outs, uint8_t *recs, int nthreads);
uint64_t orc_scan_batch_k(orc_tree *t, const uint8_t *keys, uint32_t key_stride, uint32_t key_size, uint64_t n,
                          uint32_t scan_size, uint32_t *counts, uint8_t *recs, int nthreads);
int64_t orc_export_leaves(orc_tree *t, uint32_t cap, uint64_t max_leaves, uint32_t *rc,
                          uint32_t *sc, uint64_t *meta, uint64_t *keyw);

/* RecordLocation handles (allocation index + 1) -> (leaf index in key order, slot);
 * 0xFFFFFFFF / 0xFFFF = the location dangles */
void orc_resolve_locations(orc_tree *t, const uint64_t *handles, uint64_t n, uint32_t *leaf, uint16_t *slot);
uint64_t orc_location_count(orc_tree *t);

/* transaction-manager facts (see stage_oracle.c "transaction-manager facts"): the hit slot's meta
 * word, RecordLocation handle and next handle (0 / 0x40000000 | copy id / 0x80000000 | version
 * id); a location's current meta word + next handle; overwrite-copy state st[7] = {cstamp,
 * pstamp, rstamp, sstamp, readers, count, waiting}, its readers, AddReader, WR count (+1 / -1;
 * returns 0 when IncreaseWRCount is refused), UpdatePs */
int orc_read_ident(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t read_id, orc_read_out *out,
                   uint8_t *rec, uint64_t *meta, uint32_t *loc, uint32_t *next);
int orc_location_meta(orc_tree *t, uint64_t handle, uint64_t *meta, uint32_t *next);
int orc_record_meta(orc_tree *t, const uint8_t *key, uint32_t key_size, uint64_t *meta, uint32_t *loc, uint32_t *next);
int orc_copy_state(orc_tree *t, uint32_t copy_id, uint32_t *st);
uint32_t orc_copy_readers(orc_tree *t, uint32_t copy_id, uint32_t *out, uint32_t max);
int orc_copy_add_reader(orc_tree *t, uint32_t copy_id, uint32_t read_id);
int orc_copy_wr_count(orc_tree *t, uint32_t copy_id, int delta);
int orc_copy_update_ps(orc_tree *t, uint32_t copy_id, uint32_t pstamp);

/* KeyCompare (b_tree.h:116-134) */
int orc_key_compare(const uint8_t *k1, uint32_t s1, const uint8_t *k2, uint32_t s2);
/* MurmurHash64A (misc/murmur/MurmurHash2.cpp:99-147) */
uint64_t orc_murmur64a(const void *key, int len, uint64_t seed);
void orc_murmur64a_batch(const uint64_t *keys, uint64_t n, int len, uint64_t seed, uint64_t *out);
/* payload generator shared by both sides' loaders (data, not algorithm) */
uint64_t orc_payload_word(uint64_t rowid, uint32_t j);
void orc_fill_payload(uint64_t rowid, int mode, uint8_t *dst, uint32_t payload_size);

#ifdef __cplusplus
}
#endif

/* CH-benCHmark Q2 (RunQuery2, benchmark/tpcc/tpcc_new_order.cpp:608-982): see stage_oracle.c */
typedef struct {
    int64_t supp_key, s_w_id, s_i_id;
    int32_t s_quantity, s_ytd, s_order_cnt, s_remote_cnt;
    uint8_t item_has_b, update, pad[6];
} orc_q2_rec;
int64_t orc_ch_query2(orc_tree *region, orc_tree *nation, orc_tree *supplier, orc_tree *item, orc_tree *stock,
                      const uint32_t *map_off, const int32_t *map_w, const int32_t *map_i, int target_region,
                      uint32_t read_id, orc_q2_rec *out, uint64_t max_out, int *aborted);
uint64_t orc_ch_query2_timed(orc_tree *region, orc_tree *nation, orc_tree *supplier, orc_tree *item, orc_tree *stock,
                             const uint32_t *map_off, const int32_t *map_w, const int32_t *map_i, int target_region,
                             uint32_t read_id, uint64_t count, int nthreads, double *seconds);
#endif
