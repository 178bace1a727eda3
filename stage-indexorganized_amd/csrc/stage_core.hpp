// stage_core.hpp -- definitions shared by the host table builder and the gfx950 kernels.
//
// Device image of one index-organized table (DESIGN.md "Data layout in HBM"):
//   head[L]         cap+cap/8 B rounded to 128: 1-byte key fingerprint per slot, then the
//                   visible-slot masks -- the only per-leaf bytes a point probe reads
//   okey[L*KW*cap]  u64  order key columns, one plane of cap words per key word (range scans
//                   read them whole, 512 B/leaf for keys of <= 8 bytes)
//   slot[L*cap]     32 B {okey word 0, meta word, next handle, image id, location handle}
//                   (probe: candidates)
//   tree            u64  implicit 16-ary separator tree (KW words per entry), all levels
//   heap[I*hstride] u8   record images [key padded to 8][payload] (current, copies,
//                   versions); rows 128-B aligned when larger than 128 B
//   chdr[C]         16 B overwrite-copy headers   (EphemeralPool::OverwriteVersionHeader)
//   vhdr[V]         16 B retired-version headers  (TupleHeader)
#pragma once
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#define STAGE_HD __host__ __device__ __forceinline__
#else
#define STAGE_HD inline
#endif

namespace stage {

// RecordMetadata word, bit-identical to the reference (record_meta.h:66-70) so a device
// leaf can be compared word-for-word with a reference leaf.
constexpr uint64_t kMetaControl = 1ull << 63;
constexpr uint64_t kMetaVisible = 1ull << 62;
constexpr uint64_t kMetaKeyLen = 0x2FFFull << 48;
constexpr uint64_t kMetaOffset = 0xFFFFull << 32;
constexpr uint64_t kMetaTxn = 0xFFFFFFFFull;
constexpr uint32_t kMaxCid = 0xFFFFFFFFu;
constexpr uint32_t kInvalidCid = 0u;

STAGE_HD uint32_t meta_keylen(uint64_t m) { return (uint32_t)((m & kMetaKeyLen) >> 48); }
STAGE_HD uint32_t meta_offset(uint64_t m) { return (uint32_t)((m & kMetaOffset) >> 32); }
STAGE_HD bool meta_visible(uint64_t m) { return (m & kMetaVisible) != 0; }
STAGE_HD bool meta_inserting(uint64_t m) { return (m & kMetaVisible) && (m & kMetaControl); }
STAGE_HD uint32_t meta_cstamp(uint64_t m) { return (uint32_t)(m & kMetaTxn); }
STAGE_HD uint32_t pad8(uint32_t n) { return (n + 7u) & ~7u; }

// 32-bit next handle: kind in bits 30-31, index below.  The reference stores a raw pointer
// (copy-buffer location while an update is in flight, TupleHeader* after commit).
constexpr uint32_t kNextKindMask = 3u << 30;
constexpr uint32_t kNextCopy = 1u << 30;
constexpr uint32_t kNextVersion = 2u << 30;
constexpr uint32_t kNextIndexMask = (1u << 30) - 1;

// Order key: the reference orders keys by signed-byte lexicographic compare of the first
// min(len) bytes, then by length (BaseNode::KeyCompare, b_tree.h:99-134).  For keys of at
// most 8 bytes that order is the unsigned order of (okey, len) where okey holds byte i ^ 0x80
// at big-endian position i and zero below the key.
STAGE_HD uint64_t bswap64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bswap64(x);
#else
    return __builtin_bswap64(x);
#endif
}
STAGE_HD uint64_t order_key(uint64_t le_bytes, uint32_t len) {
    const uint64_t mask = len >= 8 ? ~0ull : ((1ull << (8u * len)) - 1ull);
    return bswap64((le_bytes & mask) ^ (0x8080808080808080ull & mask));
}
STAGE_HD uint64_t key_bytes_from_order(uint64_t okey, uint32_t len) {
    const uint64_t mask = len >= 8 ? ~0ull : ((1ull << (8u * len)) - 1ull);
    return (bswap64(okey) ^ 0x8080808080808080ull) & mask;
}

// Keys longer than 8 bytes (fixed width 9..32, TPC-C): one order word per 8-byte chunk,
// compared word by word, then by length.  KeyCompare (b_tree.h:114-134, and Sorter's copy at
// b_tree.h:527-545) uses the signed-byte my_memcmp only when min(size1, size2) < 16 and libc
// memcmp -- UNSIGNED bytes -- from 16 bytes up, so tables whose keys are 16..32 bytes order
// by unsigned bytes (no 0x80 flip).
constexpr int kMaxKeyWords = 4;
constexpr uint32_t kMaxKeyBytes = 32;
// order words per key of a table: 1 (<= 8 bytes), 2 (9..16), 4 (17..32; 24-byte keys carry a
// zero fourth word, which every key of the table shares)
STAGE_HD uint32_t table_key_words(uint32_t key_width) { return key_width <= 8 ? 1u : (key_width <= 16 ? 2u : 4u); }
// order word j of a key of `len` bytes whose little-endian chunk j is `le_word`
STAGE_HD bool key_order_unsigned(uint32_t key_width) { return key_width >= 16; }
STAGE_HD uint64_t order_word(uint64_t le_word, uint32_t len, uint32_t j, bool uns) {
    if (8u * j >= len) return 0;
    const uint32_t rem = len - 8u * j;
    const uint32_t nb = rem > 8u ? 8u : rem;
    if (!uns) return order_key(le_word, nb);
    const uint64_t mask = nb >= 8 ? ~0ull : ((1ull << (8u * nb)) - 1ull);
    return bswap64(le_word & mask);
}
STAGE_HD uint32_t key_fp_words(const uint64_t *w, uint32_t kw) {
    uint64_t h = w[0];
    for (uint32_t j = 1; j < kw; ++j) h = (h ^ (h >> 29)) * 0xBF58476D1CE4E5B9ull + w[j];
    const uint32_t fp = (uint32_t)((h * 0x9E3779B97F4A7C15ull) >> 56);
    return fp ? fp : 1u;  // 0 marks a slot that is empty or invisible in the leaf head
}

// per-slot word, read by the fingerprint candidates of a probe
struct alignas(32) SlotInfo {
    uint64_t okey;  // order key (confirms a fingerprint match)
    uint64_t meta;  // reference RecordMetadata.meta
    uint32_t next;  // tagged next handle
    uint32_t image; // record-heap row of the current image
    uint32_t loc;   // RecordLocation handle of the record (host loc_; read only by stage_probe_ident)
    uint32_t pad;
};

// leaf head: [fp: cap bytes, 0 = empty or invisible slot][visible masks: cap/8 bytes][group max keys: cap/64 x KW words],
// 128-B multiple.  A group's max key (over its live slots) lets a range scan skip slot groups
// that hold nothing >= its start key.
STAGE_HD uint32_t head_gmax_offset(uint32_t cap) { return cap + cap / 8; }
// leaf info word after the group maxima: record count (bits 0-15) | mp (bits 16-31), the length
// of the longest slot prefix whose keys increase strictly (>= the sorted region)
STAGE_HD uint32_t head_info_offset(uint32_t cap, uint32_t kw) { return head_gmax_offset(cap) + (cap / 64) * kw * 8u; }
STAGE_HD uint32_t leaf_head_bytes(uint32_t cap, uint32_t kw) {
    return (head_info_offset(cap, kw) + 8u + 127u) & ~127u;
}

struct alignas(16) CopyHdr {  // EphemeralPool::OverwriteVersionHeader (ephemeral_pool.h:26-150)
    uint32_t rstamp;          // old cstamp (lower bound of the copy's visibility)
    uint32_t sstamp;          // successor stamp (MAX_CID until the writer commits)
    uint32_t next;            // TupleHeader chain at update time (tagged)
    uint32_t image;           // record-heap row of the old image
};

struct alignas(16) VersionHdr { // TupleHeader (version_store.h:28-155)
    uint32_t begin_id;
    uint32_t comm_id;
    uint32_t next;              // tagged (kNextVersion | idx) or 0
    uint32_t image;
};

// probe statuses (mirror of include/stage_hip.h)
enum : uint8_t { ST_NOT_FOUND = 0, ST_LATEST = 1, ST_COPY = 2, ST_OLD = 3, ST_FAIL_INVALID_TS = 4,
                 ST_CHAIN_MISS = 5 };

constexpr int kTreeFanout = 16;        // keys per inner separator-tree node (one 128-B line)
constexpr int kLeafFanout = 8;         // keys per bottom-level node (one 64-B sector for 8-B keys)
STAGE_HD int tree_fanout(int level) { return level ? kTreeFanout : kLeafFanout; }
constexpr int kMaxTreeLevels = 16;

// Everything a kernel needs to read one table (passed by value).
struct DevTable {
    const uint8_t *head;        // [L * head_bytes]: fp[cap] then vis[cap/64]
    const uint64_t *okey;       // [(leaf*KW + word)*cap + slot]
    const SlotInfo *slot;
    const uint64_t *tree;       // all levels, level 0 (leaf separators) first; [entry*KW + word]
    const uint8_t *tree_len;    // variable-length tables only: key length per tree entry
    const uint8_t *heap;
    const CopyHdr *chdr;
    const VersionHdr *vhdr;
    uint64_t level_off[kMaxTreeLevels]; // entry offset of each level inside `tree`
    uint32_t levels;            // number of levels (top = levels-1 has one node)
    uint32_t nleaves;
    uint32_t nseps;             // nleaves - 1
    uint32_t cap;               // slots per leaf (64 or 128)
    uint32_t stride;            // output row bytes (multiple of 16, >= 8 + payload)
    uint32_t hstride;           // heap row bytes (stride, rounded to 128 when above 128)
    uint32_t head_bytes;        // bytes per leaf head
    uint32_t payload_size;
    uint32_t key_width;         // 0 = variable
    uint32_t key_words;         // KW: order words per key (1 for keys of <= 8 bytes)
};

}  // namespace stage
