// kernel_api.hpp -- launchers of the gfx950 kernels (kernels.hip), called by the host side.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "stage_core.hpp"

namespace stage {

// same bytes as stage_probe_out (include/stage_hip.h)
struct alignas(16) stage_probe_out_dev {
    uint32_t w[8];
};

// device copy of ImageDesc (host_table.hpp)
struct alignas(8) ImageDescDev {
    uint64_t key_le;
    uint64_t arg;
    uint32_t kind;
    uint32_t mode;
};

struct ProbeTuning {
    int group = 8;         // probes per wave in flight (swept: 8 > 4 > 2 > 1 at 100M rows)
    int max_blocks = 0;    // 0 = default grid cap (16384 blocks of 256 threads)
    int store = 1;         // output stores: 0 temporal, 1 nontemporal, 2 write-through (sc1)
    int status_bytes = 32; // status record: 32 (stage_probe_out) or 16 (stage_probe_out16)
};

hipError_t launch_resolve(const DevTable &t, const uint64_t *keys, const uint16_t *lens, uint64_t n, int le_child,
                          uint32_t *out, hipStream_t s);
// d_n (optional, the split-probe tables only -- wide keys or leaves above 128 slots): the batch's
// size lives on the device (written by an earlier kernel of the stream); n is its upper bound and
// sizes the grid, shape_n (0 = n) the expected size that picks the launch shape
hipError_t launch_probe(const DevTable &t, const uint64_t *keys, const uint16_t *lens, const uint32_t *rids,
                        const uint32_t *leaf_in, uint64_t n, stage_probe_out_dev *out, uint8_t *recs, hipStream_t s,
                        const ProbeTuning &tune, const uint64_t *d_n = nullptr, uint64_t shape_n = 0);
// launch_probe with no read id (status records only) that also evaluates each hit at the read
// ids mrids[0..mnq) and sets missed[q] when a probe produces no tuple at read id q (the miss pass
// of launch_revisit_segments, folded in).  The lane-probe tables only (probe_missed_supported:
// wide fixed-width keys or 8-byte keys in leaves above 128 slots, leaves of at most 256 slots);
// otherwise hipErrorInvalidValue and nothing is launched.
bool probe_missed_supported(const DevTable &t);
hipError_t launch_probe_missed(const DevTable &t, const uint64_t *keys, uint64_t n, stage_probe_out_dev *out,
                               hipStream_t s, const ProbeTuning &tune, const uint64_t *d_n, uint64_t shape_n,
                               const uint32_t *mrids, uint32_t mnq, int32_t *missed);
// fan-out probe (sharded front-end, dist.hip): probe i's status record and row are stored at
// every caller position flist[k], k in [fan[i].lo, fan[i].hi) (flist null: k itself; fan null:
// the one position flist[i]).  Tables of the YCSB geometry only (fixed-width 8-byte keys, 64-slot
// leaves, rows <= 1024 B).
struct alignas(8) FanRange {
    uint32_t lo, hi;
};
// dest (device memory, optional): the probes fall in dest->nseg consecutive segments (segment g
// ends at probe dest->end[g], launch-relative), each with its own output buffers out[g] / recs[g]
// in place of out / recs -- one launch for the requests of several callers (STAGE_REPLY_DIRECT)
constexpr int kFanDests = 64;
struct FanDest {
    uint32_t nseg;
    uint32_t end[kFanDests];
    stage_probe_out_dev *out[kFanDests];
    uint8_t *recs[kFanDests];
};
bool probe_fanout_supported(const DevTable &t);
hipError_t launch_probe_fanout(const DevTable &t, const uint64_t *keys, const uint32_t *rids, uint64_t n,
                               const FanRange *fan, const uint32_t *flist, stage_probe_out_dev *out, uint8_t *recs,
                               hipStream_t s, const ProbeTuning &tune, const FanDest *dest = nullptr);
struct ScanTuning {
    int max_blocks = 0;  // 0 = default grid cap (16384 blocks of 256 threads)
};

// row_status != nullptr: IndexScanExecutor range semantics (per-record visibility for
// rids[i]); row_status[i*scan_size + j] = ST_LATEST / ST_OLD / ST_NOT_FOUND (row zeroed)
hipError_t launch_scan(const DevTable &t, const uint64_t *keys, const uint16_t *lens, uint64_t n, uint32_t scan_size,
                       uint32_t *counts, uint8_t *recs, hipStream_t s, const ScanTuning &tune,
                       const uint32_t *rids = nullptr, uint8_t *row_status = nullptr);
// two single scans (no read id) of two tables in one launch, the same records as launch_scan of
// each (n = 1): 8-byte keys, leaves of the same size above 128 slots, 1..63 records each
// (scan_pair_supported; otherwise hipErrorInvalidValue and nothing is launched)
hipError_t launch_scan_pair(const DevTable &t0, const uint64_t *k0, uint32_t sz0, uint32_t *c0, uint8_t *r0,
                            const DevTable &t1, const uint64_t *k1, uint32_t sz1, uint32_t *c1, uint8_t *r1,
                            hipStream_t s);
bool scan_pair_supported(const DevTable &t0, uint32_t sz0, const DevTable &t1, uint32_t sz1);
// IndexScanExecutor range scan (fixed-width tables) kept only up to its first produced tuple
// whose key starts with the start key's first `words` order words: img_out[i] = its heap row
// (0xFFFFFFFF if none), st_out[i] = ST_LATEST / ST_OLD / ST_NOT_FOUND
hipError_t launch_scan_first(const DevTable &t, const uint64_t *keys, uint64_t n, uint32_t scan_size,
                             const uint32_t *rids, uint32_t words, uint32_t *img_out, uint8_t *st_out, hipStream_t s,
                             const ScanTuning &tune);
// request ring of the resident reader (all arrays in pinned, device-mapped host memory except
// pos, which is device memory of `waves` words initialised to 0)
// one request: {key bytes (LE), read id, tag}, tag = (ticket + 1) << 4 | key length, written by
// the caller last (release); 16-B aligned, so one device load sees the tag with its key
struct alignas(16) ReaderReq {
    uint64_t key;
    uint32_t rid;
    uint32_t tag;
};
struct ReaderRing {
    const ReaderReq *req;      // [slots]
    uint32_t *done;            // [slots] ticket + 1 once its results are in place (device)
    stage_probe_out_dev *out;  // [slots]
    uint8_t *rows;             // [slots * stride]
    const uint32_t *stop;      // non-zero: instances end at their next poll
    uint64_t *pos;             // [waves] next own ticket index k of each wave, kept across instances
    uint32_t slots;            // multiple of 64 * waves
    uint32_t waves;
    uint64_t life_ticks;       // lifetime of one instance in real-time counter ticks
    uint32_t *ident;           // [slots * 2] {location handle, next handle} of each read (stage_probe_ident)
};
hipError_t launch_resident_reader(const DevTable &t, const ReaderRing &g, hipStream_t s);
// the probes of one key set at several read ids: base[0..n) holds probe results (any read id) of
// n keys; out[q * n + i] = the result of key i at rids[q], q < nq -- the hit slot is the same for
// every read id (SearchRecordMeta does not depend on it), only the visibility walk is redone;
// perm (may be null): base[i] is key perm[i]'s result, written to out[q * n + perm[i]]
// d_n (optional): the key count on the device (n its upper bound); out is then [nq][*d_n]
hipError_t launch_revisit(const DevTable &t, const stage_probe_out_dev *base, uint64_t n, const uint32_t *rids,
                          uint32_t nq, const uint32_t *perm, stage_probe_out_dev *out, hipStream_t s,
                          const uint64_t *d_n = nullptr);
// launch_revisit folded, for n probes cut into segments (segment k = base[seg_off[k], + seg_cnt[k])):
// missed[q] |= 1 when any probe yields no record (LATEST / COPY / OLD) at rids[q], and
// last[q * nseg + k] = segment k's last probe at rids[q] (left as it is for an empty segment) --
// the n * nq results themselves are never stored
hipError_t launch_revisit_segments(const DevTable &t, const stage_probe_out_dev *base, uint64_t n,
                                   const uint64_t *seg_off, const uint32_t *seg_cnt, uint32_t nseg,
                                   const uint32_t *rids, uint32_t nq, stage_probe_out_dev *last, int32_t *missed,
                                   hipStream_t s, const uint64_t *d_n = nullptr, const uint64_t *d_nseg = nullptr);
// stage_probe_batch_ex: after launch_probe of the same batch, re-answer the probes with fu[i] != 0
// as BTree::Read(..., is_for_update = true) (status record and, if recs, the row); 32-B records
hipError_t launch_for_update(const DevTable &t, const uint8_t *fu, const uint32_t *rids, uint64_t n,
                             stage_probe_out_dev *out, uint8_t *recs, hipStream_t s);
// stage_probe_ident: {location handle, next handle} of each probe's hit slot (two u32 per probe)
hipError_t launch_ident(const DevTable &t, const stage_probe_out_dev *out, uint64_t n, uint32_t *ident, hipStream_t s);
hipError_t launch_murmur(const void *keys, uint32_t key_len, uint32_t key_stride, uint64_t seed, uint64_t n,
                         uint64_t *out, hipStream_t s);
hipError_t launch_fill(uint8_t *heap, uint32_t stride, uint32_t payload_size, uint32_t row_bytes,
                       const ImageDescDev *descs, const uint8_t *arena, uint64_t first, uint64_t count,
                       uint64_t ident_rowid0, uint32_t ident_key_width, int ident_mode, hipStream_t s);
hipError_t launch_patch(uint8_t *head, uint64_t *okey, SlotInfo *slot, uint32_t head_bytes, uint32_t cap, uint32_t kw,
                        const uint32_t *head_leaf, const void *head_src, uint64_t nhead, const uint64_t *slot_idx,
                        const SlotInfo *slot_src, const uint64_t *words, uint64_t nslot, hipStream_t s);

}  // namespace stage
