// visibility.hpp -- device-side version visibility of one hit slot, shared by the probe / scan
// kernels (kernels.hip) and the kernels that re-evaluate a probe's hit at other read ids inside
// their own pass (chq2.hip: CH-Q2's per-supplier reduce and its finishing kernel).
#pragma once

#include <hip/hip_runtime.h>

#include "stage_core.hpp"

namespace stage {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct ProbeRes {
    uint32_t status, flags, hops, slot, meta_hi, cstamp, rec_cstamp, copy_sstamp, image;  // meta_hi: meta >> 32
};

// BTree::Read + IndexScanExecutor visibility for one wave-uniform probe whose slot word
// (meta, next, image) is already known.  FU: BTree::Read(..., is_for_update = true), the
// writer's read of its own record: an in-flight record is read from the leaf, not from the
// overwrite copy (b_tree.cpp:2087 takes the copy branch only when !is_for_update; the else
// branch :2114-2120 is Record::New of the leaf image with cstamp = the reader's id and no
// AddReader), and the executor skips PerformRead (executor.h:388) -- flag bit 2 says so.
template <bool FU = false>
__device__ __forceinline__ void visibility(const DevTable &t, int slot, uint64_t m, uint32_t next, uint32_t image,
                                           uint32_t rid, ProbeRes &r) {
    r.flags = FU ? 2u : 0u;
    r.hops = 0;
    r.copy_sstamp = kMaxCid;
    r.image = 0xFFFFFFFFu;
    r.cstamp = 0;
    r.rec_cstamp = 0;
    r.meta_hi = 0;
    r.slot = 0xFFFF;
    if (slot < 0) {
        r.status = ST_NOT_FOUND;
        return;
    }
    r.slot = (uint32_t)slot;
    r.rec_cstamp = meta_cstamp(m);
    r.meta_hi = (uint32_t)(m >> 32);
    CopyHdr c = {0, kMaxCid, 0, 0};
    const bool has_copy = (next & kNextKindMask) == kNextCopy;
    if (has_copy) {  // PerformRead: GetOversionHeader(meta.next_ptr) != nullptr
        c = t.chdr[next & kNextIndexMask];
        r.flags |= 1u;
        r.copy_sstamp = c.sstamp;
    }
    uint32_t img, chain;
    bool from_copy = false;
    if (!FU && meta_inserting(m)) {
        if (!has_copy) {  // copy location 0 / header gone: Read returns nullptr
            r.status = ST_NOT_FOUND;
            return;
        }
        img = c.image;
        r.cstamp = c.rstamp;
        chain = c.next;
        from_copy = true;
    } else {
        img = image;
        r.cstamp = rid;
        chain = next;
    }
    if (rid >= r.rec_cstamp) {
        r.status = from_copy ? ST_COPY : ST_LATEST;
        r.image = img;
        return;
    }
    // older snapshot: TupleHeader chain (executor.h:407-449)
    if ((chain & kNextKindMask) != kNextVersion) {
        r.status = ST_CHAIN_MISS;
        return;
    }
    for (uint32_t guard = 0; guard < (1u << 24); ++guard) {
        const VersionHdr v = t.vhdr[chain & kNextIndexMask];
        r.hops++;
        if (v.begin_id == kInvalidCid || v.comm_id == kInvalidCid) {
            r.status = ST_FAIL_INVALID_TS;
            return;
        }
        if (rid >= v.begin_id && rid <= v.comm_id) {
            r.status = ST_OLD;
            r.cstamp = v.begin_id;
            r.image = v.image;
            return;
        }
        if ((v.next & kNextKindMask) != kNextVersion) break;
        chain = v.next;
    }
    r.status = ST_CHAIN_MISS;
}

__device__ __forceinline__ void pack_out(uint32_t leaf, const ProbeRes &r, u32x4 &a, u32x4 &b) {
    a.x = (r.status & 0xFF) | ((r.flags & 0xFF) << 8) | ((r.hops > 0xFFFF ? 0xFFFF : r.hops) << 16);
    a.y = leaf;
    a.z = (r.slot & 0xFFFF) | (meta_keylen((uint64_t)r.meta_hi << 32) << 16);
    a.w = r.cstamp;
    b.x = r.rec_cstamp;
    b.y = r.copy_sstamp;
    b.z = r.image;
    b.w = r.meta_hi;
}

// a probe's status record (a, b: its two 16-B halves) re-evaluated at read id rid: the hit
// slot's word from the same published image, visibility() again.  A NOT_FOUND result (no
// visible slot, or an in-flight insert without a copy) holds for every read id and stays as it is.
__device__ __forceinline__ void revisit_one(const DevTable &t, uint32_t rid, u32x4 &a, u32x4 &b) {
    const uint32_t slot = a.z & 0xFFFF, leaf = a.y;
    if ((a.x & 0xFF) != ST_NOT_FOUND && slot < t.cap && leaf < t.nleaves) {
        const SlotInfo si = t.slot[(uint64_t)leaf * t.cap + slot];
        ProbeRes r;
        visibility(t, (int)slot, si.meta, si.next, si.image, rid, r);
        pack_out(leaf, r, a, b);
    }
}

}  // namespace stage
