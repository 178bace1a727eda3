// kernels.hip -- gfx950 (CDNA4, wave64) kernels of the index-organized read path.
//
// Integer/pointer work only (no MFMA).  Mapping:
//   * leaf resolve: lane-per-probe descent of the implicit separator tree (16-entry 128-B
//     inner nodes, 8-entry 64-B bottom nodes), replaces InternalNode::GetChildIndex
//     (b_tree.cpp:664-702) / BTree::TraverseToLeaf (b_tree.cpp:1804-1846).
//   * leaf probe: wave-per-probe.  64 lanes read the leaf head's fingerprints (1 byte per
//     slot, 0 = empty/invisible: one 64-B sector); ballot gives the fingerprint candidates, the
//     candidate lanes read their 32-B slot words and a second ballot confirms the order key:
//     first visible slot holding the key in slot order == BaseNode::SearchRecordMeta
//     (b_tree.cpp:18-122).
//   * visibility: wave-uniform scalar walk (BTree::Read copy path b_tree.cpp:2087-2123,
//     IndexScanExecutor executor.h:383-450); latest-version fast path inline.
//   * tuple copy: 63 lanes x 16 B = the 1008-B [key|payload] row (Record::New b_tree.h:407-428),
//     read from a 128-B aligned heap row, written with nontemporal stores.
//   * range scan: ballot + mbcnt prefix counts give RangeScanBySize's slot-order truncation
//     (b_tree.cpp:1276-1302), an in-wave rank sort replaces std::sort, continuation as
//     Iterator::GetNext (b_tree.h:899-941).
#include <hip/hip_runtime.h>

#include "kernel_api.hpp"
#include "stage_core.hpp"
#include "visibility.hpp"

namespace stage {

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l);
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// popcount of mask bits below this lane
__device__ __forceinline__ uint32_t count_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ bool kv_lt(uint64_t ao, uint32_t al, uint64_t bo, uint32_t bl) {
    return ao < bo || (ao == bo && al < bl);
}
__device__ __forceinline__ uint64_t head_vis(const DevTable &t, uint32_t leaf, int s) {
    return *reinterpret_cast<const uint64_t *>(t.head + (uint64_t)leaf * t.head_bytes + t.cap + 8 * s);
}

// branch-free lexicographic a < b (for several compares in flight in one lane)
template <int KW>
__device__ __forceinline__ bool kw_lt_flat(const uint64_t *a, const uint64_t *b) {
    bool lt = false, eq = true;
#pragma unroll
    for (int j = 0; j < KW; ++j) {
        lt = lt | (eq & (a[j] < b[j]));
        eq = eq & (a[j] == b[j]);
    }
    return lt;
}

// multi-word order keys (fixed-width keys of 9..32 bytes): lexicographic word order.  Written
// as selects from the last word to the first rather than early returns: per-lane early exits
// become exec-mask branches and lane-mask logic on the CU's one scalar pipe, which the
// first-tuple scans saturate; selects stay on the SIMD's vector pipe
template <int KW>
__device__ __forceinline__ bool kw_lt(const uint64_t *a, const uint64_t *b) {
    uint32_t r = 0;
#pragma unroll
    for (int j = KW - 1; j >= 0; --j) r = a[j] < b[j] ? 1u : (a[j] != b[j] ? 0u : r);
    return r != 0;
}

// chunk c (16 B) of heap row img; zeros past the heap row (an output stride above the heap
// stride, stage_set_output_layout: the rest of the output row is zero, not the next heap row)
__device__ __forceinline__ u32x4 heap_chunk(const DevTable &t, uint32_t img, uint32_t c) {
    return c < (t.hstride >> 4) ? reinterpret_cast<const u32x4 *>(t.heap + (uint64_t)img * t.hstride)[c]
                                : u32x4{0, 0, 0, 0};
}

// separators of one node (F entries) below x.  KW = 1: the node is F x 8 B (F/2 16-B loads
// per lane); KW > 1: F entries of KW words each, compared lexicographically.
template <bool VARLEN, int KW, int F>
__device__ __forceinline__ uint32_t node_count_below(const DevTable &t, uint64_t off, const uint64_t *x, uint32_t xl) {
    uint32_t cnt = 0;
    if (KW > 1) {
        const uint64_t *e = t.tree + off * KW;
#pragma unroll
        for (int k = 0; k < F; ++k) {
            uint64_t w[KW];
#pragma unroll
            for (int j = 0; j < KW; ++j) w[j] = e[k * KW + j];
            cnt += kw_lt<KW>(w, x) ? 1u : 0u;
        }
        return cnt;
    }
    const u32x4 *e = reinterpret_cast<const u32x4 *>(t.tree + off);
    u32x4 q[F / 2];
#pragma unroll
    for (int k = 0; k < F / 2; ++k) q[k] = e[k];
    if (VARLEN) {
        const uint64_t *lp = reinterpret_cast<const uint64_t *>(t.tree_len + off);
        uint64_t lw[F / 8];
#pragma unroll
        for (int k = 0; k < F / 8; ++k) lw[k] = lp[k];
#pragma unroll
        for (int k = 0; k < F / 2; ++k) {
            const uint64_t l = lw[k / 4];
            const int sh = 16 * (k & 3);
            const uint64_t v0 = ((uint64_t)q[k].y << 32) | q[k].x, v1 = ((uint64_t)q[k].w << 32) | q[k].z;
            cnt += kv_lt(v0, (uint32_t)((l >> sh) & 0xFF), x[0], xl) ? 1u : 0u;
            cnt += kv_lt(v1, (uint32_t)((l >> (sh + 8)) & 0xFF), x[0], xl) ? 1u : 0u;
        }
    } else {
#pragma unroll
        for (int k = 0; k < F / 2; ++k) {
            cnt += ((((uint64_t)q[k].y << 32) | q[k].x) < x[0]) ? 1u : 0u;
            cnt += ((((uint64_t)q[k].w << 32) | q[k].z) < x[0]) ? 1u : 0u;
        }
    }
    return cnt;
}

// lower_bound over the separators: number of separators < x, i.e. the leaf whose range
// (sep[i-1], sep[i]] holds x (le_child semantics).  Upper-bound callers pass succ(x).
// Inner levels are 16-entry nodes (one 128-B line for 8-B keys), the bottom level 8-entry
// nodes (one 64-B sector): the bottom node is the one the probe usually fetches from beyond L2.
template <bool VARLEN, int KW>
__device__ __forceinline__ uint32_t tree_lower_bound(const DevTable &t, const uint64_t *x, uint32_t xl) {
    static_assert(kTreeFanout == 16 && kLeafFanout == 8, "node loads sized for 16 / 8 entries");
    uint32_t node = 0;
    for (int lvl = (int)t.levels - 1; lvl > 0; --lvl)
        node = node * kTreeFanout +
               node_count_below<VARLEN, KW, kTreeFanout>(t, t.level_off[lvl] + (uint64_t)node * kTreeFanout, x, xl);
    node = node * kLeafFanout + node_count_below<VARLEN, KW, kLeafFanout>(t, t.level_off[0] + (uint64_t)node * kLeafFanout,
                                                                          x, xl);
    return node < t.nseps ? node : t.nseps;
}

template <bool VARLEN, int KW>
__device__ __forceinline__ uint32_t resolve_leaf(const DevTable &t, const uint64_t *okey, uint32_t len, bool le_child) {
    if (le_child) return tree_lower_bound<VARLEN, KW>(t, okey, len);
    if (VARLEN) return tree_lower_bound<VARLEN, KW>(t, okey, len + 1);  // (okey, len+1) = succ
    // fixed width: succ = the key plus one in its last word, with carry
    uint64_t s[KW];
    bool carry = true;
#pragma unroll
    for (int j = KW - 1; j >= 0; --j) {
        s[j] = okey[j] + (carry ? 1ull : 0ull);
        carry = carry && okey[j] == ~0ull;
    }
    if (carry) return t.nseps;
    return tree_lower_bound<VARLEN, KW>(t, s, len);
}

// Wave-cooperative descent for a wave-uniform key (range scans): per level, lane e < fanout loads
// separator e of the node and one ballot counts the separators below the key -- one load
// round per level instead of every lane reading the whole node.
template <bool VARLEN, int KW>
__device__ __forceinline__ uint32_t tree_lower_bound_uniform(const DevTable &t, const uint64_t *x, uint32_t xl,
                                                             uint32_t lane) {
    uint32_t node = 0;
    for (int lvl = (int)t.levels - 1; lvl >= 0; --lvl) {
        const uint32_t f = (uint32_t)tree_fanout(lvl);
        const uint64_t off = t.level_off[lvl] + (uint64_t)node * f;
        bool lt = false;
        if (lane < f) {
            uint64_t e[KW];
#pragma unroll
            for (int j = 0; j < KW; ++j) e[j] = t.tree[(off + lane) * KW + j];
            if (KW == 1) lt = VARLEN ? kv_lt(e[0], t.tree_len[off + lane], x[0], xl) : e[0] < x[0];
            else lt = kw_lt<KW>(e, x);
        }
        node = node * f + (uint32_t)__builtin_popcountll(ballot(lt));
    }
    return node < t.nseps ? node : t.nseps;
}

template <bool VARLEN, int KW>
__device__ __forceinline__ uint32_t resolve_leaf_uniform(const DevTable &t, const uint64_t *okey, uint32_t len,
                                                         bool le_child, uint32_t lane) {
    if (le_child) return tree_lower_bound_uniform<VARLEN, KW>(t, okey, len, lane);
    if (VARLEN) return tree_lower_bound_uniform<VARLEN, KW>(t, okey, len + 1, lane);
    uint64_t s[KW];
    bool carry = true;
#pragma unroll
    for (int j = KW - 1; j >= 0; --j) {
        s[j] = okey[j] + (carry ? 1ull : 0ull);
        carry = carry && okey[j] == ~0ull;
    }
    if (carry) return t.nseps;
    return tree_lower_bound_uniform<VARLEN, KW>(t, s, len, lane);
}

// Iterator continuation (le_child = false from the last popped key x) when x came from
// `leaf`: every key of a leaf lies in its separator range (sep[leaf-1], sep[leaf]], so the
// separators <= x are those left of `leaf` plus sep[leaf] itself when it equals x -- the
// upper-bound descent collapses to one load of sep[leaf] (+inf padding past the last leaf).
template <bool VARLEN, int KW>
__device__ __forceinline__ uint32_t next_leaf_after(const DevTable &t, uint32_t leaf, const uint64_t *x, uint32_t xl) {
    if (leaf >= t.nseps) return t.nseps;
    const uint64_t e = t.level_off[0] + leaf;
    uint64_t sep[KW];
#pragma unroll
    for (int w = 0; w < KW; ++w) sep[w] = t.tree[e * KW + w];
    bool x_lt_sep;
    if (KW == 1) x_lt_sep = VARLEN ? kv_lt(x[0], xl, sep[0], t.tree_len[e]) : x[0] < sep[0];
    else x_lt_sep = kw_lt<KW>(x, sep);
    return x_lt_sep ? leaf : leaf + 1;
}

// order words of a key passed as KW little-endian u64 words (fixed width) or one word
template <int KW>
__device__ __forceinline__ void load_okey(const uint64_t *keys, uint64_t i, bool valid, uint32_t len, uint64_t *okw) {
#pragma unroll
    for (int j = 0; j < KW; ++j) {
        const uint64_t le = valid ? keys[i * KW + j] : 0ull;
        okw[j] = KW == 1 ? order_key(le, len) : order_word(le, len, (uint32_t)j, key_order_unsigned(len));
    }
}

template <int KW>
__global__ __launch_bounds__(256) void resolve_kernel(DevTable t, const uint64_t *__restrict__ keys,
                                                      const uint16_t *__restrict__ lens, uint64_t n, int le_child,
                                                      uint32_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t len = t.key_width ? t.key_width : (lens ? lens[i] : 8u);
    uint64_t ok[KW];
    load_okey<KW>(keys, i, true, len, ok);
    out[i] = t.key_width ? resolve_leaf<false, KW>(t, ok, len, le_child != 0)
                         : resolve_leaf<true, 1>(t, ok, len, le_child != 0);
}

// ----------------------------------------------------------------------------------------
// point probe

// 16-B output store at base + off (base wave-uniform).  POL 0: temporal; 1: nontemporal (the
// line is still kept in the XCD's L2); 2: write-through (sc1 buffer store: the line leaves L2,
// so the output stream does not evict cached rows, heads and separator nodes --
// MI355X_MICROARCH.md, store flavours).  Measured (scripts/ab_store.py, 100M rows): 1 is
// fastest (6.35 ms), 0 +1.7 %, 2 +2.6 %; nontemporal heap-row loads on top of 1 +5 %.
template <int POL>
__device__ __forceinline__ void st16(u32x4 v, uint8_t *base, uint32_t off) {
    if constexpr (POL == 2) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)off, 0, 16);
    } else {
        // plain pointer arithmetic (u32x4 *) + chunk: the (base, off) form above, used for the
        // flat stores too, raised probe_kernel<.., 8> from 95 to 154 VGPRs (3 waves/SIMD
        // instead of 5) and cost 9 % of the launch time
        u32x4 *p = reinterpret_cast<u32x4 *>(base) + (off >> 4);
        if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
        else *p = v;
    }
}

// CH: probes per wave chunk (64; 16 for small batches of the one-probe-in-flight instances, so
// that a wave's chunk is not a chain of 64 dependent probes while most of the chip idles).
// ST: status record bytes -- 32 (stage_probe_out) or 16 (stage_probe_out16, opt-in: status |
// flags | hops, cstamp, copy_sstamp, rec_cstamp -- what IndexScanExecutor and PerformRead use)
// FAN: fan-out probes (the sharded front-end's coalesced requests, dist.hip): probe i's status
// record and row go to every caller position flist[k], k in [fan[i].lo, fan[i].hi) (flist null:
// the positions k themselves; fan null: {i, i + 1}, probe i's one position flist[i]) instead of
// position i -- the row leaves registers once per caller and no second pass copies it (rows of
// at most 1024 B, recs required).
template <bool VARLEN, int SPL, int G, int POL = 1, int KW = 1, int CH = 64, int ST = 32, bool FAN = false,
          bool DEST = false>
__global__ __launch_bounds__(256) void probe_kernel(DevTable t, const uint64_t *__restrict__ keys,
                                                    const uint16_t *__restrict__ lens,
                                                    const uint32_t *__restrict__ rids,
                                                    const uint32_t *__restrict__ leaf_in, uint64_t n,
                                                    stage_probe_out_dev *__restrict__ out,
                                                    uint8_t *__restrict__ recs, const FanRange *__restrict__ fan,
                                                    const uint32_t *__restrict__ flist,
                                                    const FanDest *__restrict__ dest = nullptr) {
    const uint32_t lane = lane_id();
    // FAN with per-segment destinations: the segment table in LDS (every thread reaches this
    // barrier: nothing returns before it)
    __shared__ uint32_t s_dend[DEST ? kFanDests : 1];
    __shared__ stage_probe_out_dev *s_dout[DEST ? kFanDests : 1];
    __shared__ uint8_t *s_drec[DEST ? kFanDests : 1];
    uint32_t nseg = 0;
    if constexpr (DEST) {
        nseg = dest->nseg;
        for (uint32_t g = threadIdx.x; g < nseg; g += blockDim.x)
            s_dend[g] = dest->end[g], s_dout[g] = dest->out[g], s_drec[g] = dest->recs[g];
        __syncthreads();
    }
    // threadIdx.x / 64 made provably wave-uniform: the chunk base and the output row addresses
    // live in SGPRs (probe_kernel<.., 8>: 78 VGPRs, 6 waves/SIMD, instead of 95 and 5)
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + uni32(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t out_chunks = t.stride >> 4;
    for (uint64_t base = wave * CH; base < n; base += nwaves * CH) {
        const uint64_t i = base + lane;
        const bool valid = lane < (uint32_t)CH && i < n;
        u32x4 my_a = u32x4{0, 0, 0, 0}, my_b = u32x4{0, 0, 0, 0};  // this lane's probe result
        const uint32_t len = t.key_width ? t.key_width : (lens && valid ? (uint32_t)lens[i] : 8u);
        const uint32_t rid = rids ? (valid ? rids[i] : 0u) : 0xFFFFFFFEu;
        FanRange my_fan = FanRange{0u, 0u};
        if (FAN && valid) my_fan = fan ? fan[i] : FanRange{(uint32_t)i, (uint32_t)i + 1u};
        uint64_t my_o = 0, my_r = 0;  // DEST: this lane's probe's segment's buffers
        if constexpr (DEST) {
            uint32_t sg = 0;
            for (uint32_t g = 0; g + 1 < nseg; ++g) sg += i >= s_dend[g] ? 1u : 0u;
            my_o = (uint64_t)s_dout[sg];
            my_r = (uint64_t)s_drec[sg];
        }
        uint64_t ok[KW];
        load_okey<KW>(keys, i, valid, len, ok);
        uint32_t leaf = 0;
        if (valid) leaf = leaf_in ? leaf_in[i] : resolve_leaf<VARLEN, KW>(t, ok, len, true);
        if (leaf > t.nseps) leaf = t.nseps;  // host-supplied ids are clamped to the table
        const int cnt = (int)((n - base) < CH ? (n - base) : CH);
        // one probe in flight (G = 1: the wide-key and large-leaf instances): the next probe's
        // fingerprint bytes load while this one runs, so a probe exposes one dependent round
        // trip (its candidates' slot words) instead of two
        constexpr bool PFH = G == 1;
        uint32_t nfp[SPL];
        if (PFH) {
            const uint8_t *h = t.head + (uint64_t)rl32(leaf, 0) * t.head_bytes;
#pragma unroll
            for (int s = 0; s < SPL; ++s) nfp[s] = h[s * 64 + lane];
        }
        for (int j0 = 0; j0 < cnt; j0 += G) {
            uint32_t lf[G], rd[G], xl[G];
            uint64_t x[G][KW];
            uint32_t fpb[G][SPL];
            // phase 1: leaf heads of G probes -- the fingerprint bytes only: an empty or
            // invisible slot holds fingerprint 0, which no key has (key_fp_words), so the
            // visible masks behind them are not read
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int j = j0 + g < cnt ? j0 + g : cnt - 1;
                lf[g] = rl32(leaf, j);
                rd[g] = rl32(rid, j);
#pragma unroll
                for (int w = 0; w < KW; ++w) x[g][w] = rl64(ok[w], j);
                xl[g] = VARLEN ? rl32(len, j) : t.key_width;
                if (PFH) {
#pragma unroll
                    for (int s = 0; s < SPL; ++s) fpb[g][s] = nfp[s];
                    if (j0 + 1 < cnt) {
                        const uint8_t *h = t.head + (uint64_t)rl32(leaf, j0 + 1) * t.head_bytes;
#pragma unroll
                        for (int s = 0; s < SPL; ++s) nfp[s] = h[s * 64 + lane];
                    }
                } else {
                    const uint8_t *h = t.head + (uint64_t)lf[g] * t.head_bytes;
#pragma unroll
                    for (int s = 0; s < SPL; ++s) fpb[g][s] = h[s * 64 + lane];
                }
            }
            // phase 2: fingerprint candidates read their slot words
            uint64_t wok[G][SPL], wmeta[G][SPL];
            uint32_t wnext[G][SPL], wimg[G][SPL];
            bool cand[G][SPL];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const uint32_t fx = key_fp_words(x[g], KW);
#pragma unroll
                for (int s = 0; s < SPL; ++s) {
                    cand[g][s] = fpb[g][s] == fx;
                    wok[g][s] = 0;
                    wmeta[g][s] = 0;
                    wnext[g][s] = 0;
                    wimg[g][s] = 0;
                    if (cand[g][s]) {
                        const u32x4 *w = reinterpret_cast<const u32x4 *>(t.slot + (uint64_t)lf[g] * t.cap + s * 64 + lane);
                        const u32x4 w0 = w[0], w1 = w[1];
                        // the other key words load with the slot word (one round trip) in leaves
                        // of up to 4 slot groups; larger leaves load them after the order-key
                        // match (fewer registers in flight)
                        constexpr bool COK = SPL <= 4;
                        uint64_t kw[KW > 1 ? KW : 1];
#pragma unroll
                        for (int w = 1; w < KW; ++w)
                            kw[w] = COK ? t.okey[((uint64_t)lf[g] * KW + w) * t.cap + s * 64 + lane] : 0ull;
                        wok[g][s] = ((uint64_t)w0.y << 32) | w0.x;
                        wmeta[g][s] = ((uint64_t)w0.w << 32) | w0.z;
                        wnext[g][s] = w1.x;
                        wimg[g][s] = w1.y;
                        if (KW > 1 && wok[g][s] == x[g][0]) {  // confirm the other key words
                            bool eq = true;
#pragma unroll
                            for (int w = 1; w < KW; ++w)
                                eq = eq && (COK ? kw[w] : t.okey[((uint64_t)lf[g] * KW + w) * t.cap + s * 64 + lane]) ==
                                               x[g][w];
                            if (!eq) wok[g][s] = ~x[g][0];
                        }
                    }
                }
            }
            // phase 3: confirm (order key, key length), first hit in slot order, visibility
            ProbeRes r[G];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                int slot = -1;
                uint64_t m = 0;
                uint32_t nx = 0, im = 0;
#pragma unroll
                for (int s = SPL - 1; s >= 0; --s) {
                    const bool hitl = cand[g][s] && wok[g][s] == x[g][0] && (!VARLEN || meta_keylen(wmeta[g][s]) == xl[g]);
                    const uint64_t hit = ballot(hitl);
                    if (hit) {
                        const int b = __builtin_ctzll(hit);
                        slot = s * 64 + b;
                        m = rl64(wmeta[g][s], b);
                        nx = rl32(wnext[g][s], b);
                        im = rl32(wimg[g][s], b);
                    }
                }
                const bool fast = slot >= 0 && !meta_inserting(m) && rd[g] >= meta_cstamp(m) &&
                                  (nx & kNextKindMask) != kNextCopy;
                if (fast) {
                    r[g].status = ST_LATEST;
                    r[g].flags = 0;
                    r[g].hops = 0;
                    r[g].slot = (uint32_t)slot;
                    r[g].meta_hi = (uint32_t)(m >> 32);
                    r[g].cstamp = rd[g];
                    r[g].rec_cstamp = meta_cstamp(m);
                    r[g].copy_sstamp = kMaxCid;
                    r[g].image = im;
                } else {
                    visibility(t, slot, m, nx, im, rd[g], r[g]);
                }
            }
            // phase 4 (FAN): G rows in flight, each stored at its caller positions with its
            // status record (lanes 0-1); up to 64 positions are loaded at once, one per lane
            if constexpr (FAN) {
                // the G rows and the first 64 caller positions of each request, all in flight
                // together (a request has at most kFanCap = 64 callers; longer runs loop)
                u32x4 v[G];
                uint32_t mine0[G];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    v[g] = u32x4{0, 0, 0, 0};
                    if (lane < out_chunks && r[g].image != 0xFFFFFFFFu)
                        v[g] = heap_chunk(t, r[g].image, lane);
                    const int j = j0 + g;
                    const uint32_t lo = rl32(my_fan.lo, j & 63), hi = rl32(my_fan.hi, j & 63);
                    const uint32_t kk = lo + lane;
                    mine0[g] = j < cnt && kk < hi ? (flist ? flist[kk] : kk) : 0u;
                }
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int j = j0 + g;
                    if (j >= cnt) break;
                    u32x4 a, b;
                    pack_out(lf[g], r[g], a, b);
                    const u32x4 half = lane == 0 ? a : b;
                    const uint32_t lo = rl32(my_fan.lo, j), hi = rl32(my_fan.hi, j);
                    stage_probe_out_dev *o_j = out;
                    uint8_t *r_j = recs;
                    if constexpr (DEST) {  // probe j's segment's buffers (wave-uniform: scalar registers)
                        o_j = reinterpret_cast<stage_probe_out_dev *>(rl64(my_o, j));
                        r_j = reinterpret_cast<uint8_t *>(rl64(my_r, j));
                    }
                    for (uint32_t k0 = lo; k0 < hi; k0 += 64) {
                        const uint32_t kk = k0 + lane;
                        const uint32_t mine = k0 == lo ? mine0[g] : kk < hi ? (flist ? flist[kk] : kk) : 0u;
                        const uint32_t kn = hi - k0 < 64u ? hi - k0 : 64u;
                        for (uint32_t k = 0; k < kn; ++k) {
                            const uint64_t pos = rl32(mine, (int)k);
                            if (lane < out_chunks) st16<POL>(v[g], r_j + pos * (uint64_t)t.stride, lane * 16u);
                            if (lane < 2) st16<POL>(half, reinterpret_cast<uint8_t *>(o_j + pos), lane * 16u);
                        }
                    }
                }
                continue;
            }
            // phase 4: tuple rows (G rows in flight), then nontemporal stores
            if (recs) {
                for (uint32_t c0 = 0; c0 < out_chunks; c0 += 64) {
                    const uint32_t c = c0 + lane;
                    u32x4 v[G];
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        v[g] = u32x4{0, 0, 0, 0};
                        if (c < out_chunks && r[g].image != 0xFFFFFFFFu)
                            v[g] = heap_chunk(t, r[g].image, c);
                    }
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        const int j = j0 + g;
                        if (j < cnt && c < out_chunks)
                            st16<POL>(v[g], recs + (base + j) * (uint64_t)t.stride, c * 16u);
                    }
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                u32x4 a, b;
                pack_out(lf[g], r[g], a, b);
                if (lane == (uint32_t)(j0 + g)) {
                    my_a = a;
                    my_b = b;
                }
            }
        }
        // one coalesced 2-KiB (1-KiB) store of the chunk's 64 results
        if constexpr (FAN) {
        } else if constexpr (ST == 16) {
            if (valid)
                st16<POL>(u32x4{my_a.x, my_a.w, my_b.y, my_b.x}, reinterpret_cast<uint8_t *>(out) + base * 16u,
                          lane * 16u);
        } else {
            if (valid) {
                uint8_t *ob = reinterpret_cast<uint8_t *>(out + base);
                st16<POL>(my_a, ob, lane * 32u);
                st16<POL>(my_b, ob, lane * 32u + 16u);
            }
        }
    }
}

// ----------------------------------------------------------------------------------------
// resident single-key reader: one-wave workgroups poll a request ring in pinned host memory
// (the stage_reader_* adapter of BTree::Read callers, b_tree.cpp:2066-2129, without a launch
// per request).  Ticket q belongs to wave w = q % W as its k-th ticket, k = q / W, and lives in
// slot w * P + k % P of the ring (P = slots / W, a multiple of 64): concurrent callers land on
// different waves, and a wave's tickets are contiguous in the ring.  A caller writes its 16-B
// request record -- key, read id, then the tag (q + 1) << 4 | key length with release -- so a
// wave's poll is one 16-B load per lane over PCIe that brings the key along with the tag; the
// wave takes the published prefix of its
// current 64-ticket block, probes it (lane j = the block's j-th ticket throughout), writes the
// status record and the row into the slot and publishes done[slot] = q + 1 (system-scope
// release).  Every instance ends after life_ticks of the
// 100 MHz real-time counter or when *stop is set, saving its position in pos[w] for the next
// instance queued behind it on the same stream -- no wave outlives its instance's lifetime.

// one wave-uniform probe (request j of the wave's lanes) with one probe in flight
template <bool VARLEN, int SPL, bool FU = false>
__device__ __forceinline__ void ring_probe_one(const DevTable &t, uint32_t lane, int j, uint32_t leaf_l, uint64_t ok_l,
                                               uint32_t len_l, uint32_t rid_l, uint8_t *row, uint32_t out_chunks,
                                               u32x4 &a, u32x4 &b, uint32_t &id_loc, uint32_t &id_next) {
    const uint32_t lf = rl32(leaf_l, j);
    const uint64_t x = rl64(ok_l, j);
    const uint32_t xl = VARLEN ? rl32(len_l, j) : t.key_width;
    const uint32_t rd = rl32(rid_l, j);
    const uint8_t *h = t.head + (uint64_t)lf * t.head_bytes;
    const uint32_t fx = key_fp_words(&x, 1);
    int slot = -1;
    uint64_t m = 0;
    uint32_t nx = 0, im = 0, lc = 0;
#pragma unroll
    for (int s = SPL - 1; s >= 0; --s) {  // first hit in slot order (SearchRecordMeta)
        const bool cand = h[s * 64 + lane] == fx;
        uint64_t wok = 0, wmeta = 0;
        uint32_t wnext = 0, wimg = 0, wloc = 0;
        if (cand) {
            const u32x4 *w = reinterpret_cast<const u32x4 *>(t.slot + (uint64_t)lf * t.cap + s * 64 + lane);
            const u32x4 w0 = w[0], w1 = w[1];
            wok = ((uint64_t)w0.y << 32) | w0.x;
            wmeta = ((uint64_t)w0.w << 32) | w0.z;
            wnext = w1.x;
            wimg = w1.y;
            wloc = w1.z;
        }
        const uint64_t hit = ballot(cand && wok == x && (!VARLEN || meta_keylen(wmeta) == xl));
        if (hit) {
            const int bl = __builtin_ctzll(hit);
            slot = s * 64 + bl;
            m = rl64(wmeta, bl);
            nx = rl32(wnext, bl);
            im = rl32(wimg, bl);
            lc = rl32(wloc, bl);
        }
    }
    ProbeRes r;
    visibility<FU>(t, slot, m, nx, im, rd, r);
    id_loc = r.status == ST_NOT_FOUND ? 0u : lc;
    id_next = r.status == ST_NOT_FOUND ? 0u : nx;
    for (uint32_t c0 = 0; c0 < out_chunks; c0 += 64) {
        const uint32_t c = c0 + lane;
        if (c < out_chunks) {
            u32x4 v = u32x4{0, 0, 0, 0};
            if (r.image != 0xFFFFFFFFu) v = heap_chunk(t, r.image, c);
            reinterpret_cast<u32x4 *>(row)[c] = v;
        }
    }
    pack_out(lf, r, a, b);
}

template <bool VARLEN, int SPL>
__global__ __launch_bounds__(64) void resident_reader_kernel(DevTable t, ReaderRing g) {
    const uint32_t lane = lane_id();
    const uint32_t w = blockIdx.x;
    const uint32_t out_chunks = t.stride >> 4;
    const uint32_t per = g.slots / g.waves;
    uint64_t pos = g.pos[w];  // this wave's next k
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (__hip_atomic_load(g.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > g.life_ticks) break;
        const uint64_t blk = pos & ~63ull;
        const uint32_t d = (uint32_t)(pos & 63u);
        const uint32_t s0 = w * per + (uint32_t)(blk % per);
        const uint32_t want = (uint32_t)((blk + lane) * g.waves + w + 1u);
        u32x4 rq = u32x4{0, 0, 0, 0};
        // the whole record in one load (volatile: system-coherent, past the caches); the tag is
        // written after the key and read id, in the same 16-B line, so seeing it brings them
        if (lane >= d) rq = *reinterpret_cast<const volatile u32x4 *>(g.req + s0 + lane);
        const bool ready = lane >= d && (rq.w >> 4) == (want & 0x0FFFFFFFu);
        const uint64_t m = ballot(ready) >> d;
        const uint32_t k = ~m ? (uint32_t)__builtin_ctzll(~m) : 64u;  // published prefix from d
        if (k == 0) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        const bool mine = lane >= d && lane < d + k;
        // tag low nibble: key length - 1 (bits 0-2), is_for_update (bit 3)
        const uint32_t len = t.key_width ? t.key_width : (mine ? (rq.w & 7u) + 1u : 8u);
        const uint32_t rid = mine ? rq.z : 0u;
        const bool fu = mine && (rq.w & 8u) != 0;
        const uint64_t ok = order_key(mine ? ((uint64_t)rq.y << 32 | rq.x) : 0ull, len);
        uint32_t leaf = mine ? resolve_leaf<VARLEN, 1>(t, &ok, len, true) : 0u;
        u32x4 my_a = u32x4{0, 0, 0, 0}, my_b = u32x4{0, 0, 0, 0};
        uint32_t my_loc = 0, my_next = 0;
        for (uint32_t j = d; j < d + k; ++j) {
            u32x4 a, b;
            uint32_t il, in;
            if (rl32(fu ? 1u : 0u, (int)j))
                ring_probe_one<VARLEN, SPL, true>(t, lane, (int)j, leaf, ok, len, rid,
                                                  g.rows + (uint64_t)(s0 + j) * t.stride, out_chunks, a, b, il, in);
            else
                ring_probe_one<VARLEN, SPL>(t, lane, (int)j, leaf, ok, len, rid, g.rows + (uint64_t)(s0 + j) * t.stride,
                                            out_chunks, a, b, il, in);
            if (lane == j) {
                my_a = a;
                my_b = b;
                my_loc = il;
                my_next = in;
            }
        }
        if (mine) {
            u32x4 *o = reinterpret_cast<u32x4 *>(g.out + s0 + lane);
            o[0] = my_a;
            o[1] = my_b;
            g.ident[2 * (uint64_t)(s0 + lane)] = my_loc;
            g.ident[2 * (uint64_t)(s0 + lane) + 1] = my_next;
            // status record and row before the flag, system-wide
            __hip_atomic_store(g.done + s0 + lane, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        pos += k;
    }
    if (lane == 0) g.pos[w] = pos;
}

// ----------------------------------------------------------------------------------------
// range scan (TableScanExecutor over Iterator), one wave per scan

template <int R>
__device__ __forceinline__ void copy_rows(const DevTable &t, const uint32_t *img, const uint32_t *dst, int n,
                                          uint8_t *recs, uint32_t lane) {
    const uint32_t chunks = t.stride >> 4;
    for (uint32_t c0 = 0; c0 < chunks; c0 += 64) {
        const uint32_t c = c0 + lane;
        u32x4 v[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            v[k] = u32x4{0, 0, 0, 0};
            if (k < n && c < chunks && img[k] != 0xFFFFFFFFu)
                v[k] = heap_chunk(t, img[k], c);
        }
#pragma unroll
        for (int k = 0; k < R; ++k)
            if (k < n && c < chunks)
                __builtin_nontemporal_store(v[k], reinterpret_cast<u32x4 *>(recs + (uint64_t)dst[k] * t.stride) + c);
    }
}

// position of the k-th (from 0) set bit of m (m has more than k bits set), per lane
__device__ __forceinline__ uint32_t kth_set_bit(uint64_t m, uint32_t k) {
    uint32_t pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint32_t c = (uint32_t)__builtin_popcountll(m & ((1ull << w) - 1));
        if (k >= c) {
            k -= c;
            m >>= w;
            pos += (uint32_t)w;
        }
    }
    return pos;
}

// Rows of at most 32 16-B chunks (512 B): the emitting lanes' rows (lane b of em: heap row
// img, output position dst) copied with the whole wave spread over (row, chunk) pairs -- U
// loads in flight per lane cover 64 * U / chunks rows per round trip (16 rows of 256 B), where
// copy_rows moves R rows per round trip whatever their size.  Same bytes as copy_rows.
template <int U>
__device__ __forceinline__ void copy_rows_flat(const DevTable &t, uint64_t em, uint32_t img, uint32_t dst,
                                               uint8_t *recs, uint32_t lane) {
    const uint32_t chunks = t.stride >> 4;
    const uint32_t rpr = (uint32_t)(U * 64) / chunks, nrows = (uint32_t)__builtin_popcountll(em);
    uint32_t rk[U], ck[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t f = (uint32_t)u * 64u + lane;
        rk[u] = f / chunks;
        ck[u] = f - rk[u] * chunks;
    }
    for (uint32_t r0 = 0; r0 < nrows; r0 += rpr) {
        u32x4 v[U];
        uint32_t d[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = r0 + rk[u];
            ok[u] = rk[u] < rpr && k < nrows;
            const int src = ok[u] ? (int)kth_set_bit(em, k) : 0;
            const uint32_t im = (uint32_t)__shfl((int)img, src);
            d[u] = (uint32_t)__shfl((int)dst, src);
            v[u] = u32x4{0, 0, 0, 0};
            if (ok[u] && im != 0xFFFFFFFFu) v[u] = heap_chunk(t, im, ck[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4 *>(recs + (uint64_t)d[u] * t.stride) + ck[u]);
    }
}

template <bool VARLEN, int KW>
__device__ __forceinline__ bool key_less(const uint64_t *a, uint32_t al, const uint64_t *b, uint32_t bl) {
    if (KW == 1) return kv_lt(a[0], al, b[0], bl);
    return kw_lt<KW>(a, b);  // fixed width: equal lengths
}

// IndexScanExecutor range branch (executor.h:456-530) for one iterator record: the leaf
// image when rid >= its commit id, else the TupleHeader version with begin <= rid <= end
// (nothing when begin/end is INVALID_CID, the chain ends, or next is an overwrite copy).
__device__ __forceinline__ uint32_t scan_visible(const DevTable &t, const SlotInfo &si, uint32_t rid, uint8_t &st) {
    if (rid >= meta_cstamp(si.meta)) {
        st = ST_LATEST;
        return si.image;
    }
    st = ST_NOT_FOUND;
    uint32_t chain = si.next;
    for (uint32_t guard = 0; guard < (1u << 24) && (chain & kNextKindMask) == kNextVersion; ++guard) {
        const VersionHdr v = t.vhdr[chain & kNextIndexMask];
        if (v.begin_id == kInvalidCid || v.comm_id == kInvalidCid) break;
        if (rid >= v.begin_id && rid <= v.comm_id) {
            st = ST_OLD;
            return v.image;
        }
        chain = v.next;
    }
    return 0xFFFFFFFFu;
}

template <bool VARLEN, int SPL, int R, int KW, bool VIS = false>
__device__ void scan_one(const DevTable &t, const uint64_t *x0, uint32_t xl, uint32_t leaf, uint32_t scan_size,
                         uint8_t *recs, uint32_t *count_out, uint32_t lane, uint32_t rid = 0,
                         uint8_t *row_status = nullptr) {
    uint32_t remaining = scan_size, produced = 0;
    bool cont = false;
    uint64_t x[KW];
#pragma unroll
    for (int w = 0; w < KW; ++w) x[w] = x0[w];
    for (uint32_t guard = 0; guard < scan_size + 2 && remaining > 0; ++guard) {
        const uint64_t base = (uint64_t)leaf * t.cap;
        // the leaf's monotone slot prefix (info word), loaded beside the key columns
        const uint32_t mp =
            *reinterpret_cast<const uint32_t *>(t.head + (uint64_t)leaf * t.head_bytes + head_info_offset(t.cap, KW)) >> 16;
        uint64_t col[SPL][KW];
        uint32_t kl[SPL];
        uint64_t q[SPL];
#pragma unroll
        for (int s = 0; s < SPL; ++s)
#pragma unroll
            for (int w = 0; w < KW; ++w) col[s][w] = t.okey[((uint64_t)leaf * KW + w) * t.cap + s * 64 + lane];
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            const uint64_t vm = head_vis(t, leaf, s);
            const bool vis = (vm >> lane) & 1;
            kl[s] = t.key_width;
            if (VARLEN) kl[s] = vis ? meta_keylen(t.slot[base + s * 64 + lane].meta) : 0u;
            // RangeScanBySize keeps visible records with KeyCompare(start, key) <= 0
            q[s] = ballot(vis && !key_less<VARLEN, KW>(col[s], kl[s], x, xl));
        }
        // slot-order truncation: records are collected until more than to_scan are held
        const uint32_t to_scan = remaining;
        uint32_t before = 0, m = 0;
        bool keep[SPL];
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            const uint32_t rank = before + count_below(q[s]);
            keep[s] = ((q[s] >> lane) & 1) && rank <= to_scan;
            before += (uint32_t)__builtin_popcountll(q[s]);
        }
        uint64_t km[SPL];
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            km[s] = ballot(keep[s]);
            m += (uint32_t)__builtin_popcountll(km[s]);
        }
        if (m == 0) break;
        // key rank among the kept records (std::sort by KeyCompare; keys are unique).  When
        // every kept record lies in the leaf's monotone slot prefix [0, mp) (info word), keys
        // increase with the slot, so a record's rank is its slot-order position: no compare loop
        uint32_t kr[SPL];
        uint32_t top = 0;  // one past the highest kept slot
#pragma unroll
        for (int s = 0; s < SPL; ++s)
            if (km[s]) top = (uint32_t)s * 64u + 64u - (uint32_t)__builtin_clzll(km[s]);
        const bool mono = top <= mp;
        {
            uint32_t pre = 0;
#pragma unroll
            for (int s = 0; s < SPL; ++s) {
                kr[s] = mono ? pre + count_below(km[s]) : 0u;
                pre += (uint32_t)__builtin_popcountll(km[s]);
            }
        }
#pragma unroll
        for (int s2 = 0; s2 < SPL; ++s2) {
            uint64_t mm = mono ? 0ull : km[s2];
            while (mm) {
                const int b = __builtin_ctzll(mm);
                mm &= mm - 1;
                uint64_t ko[KW];
#pragma unroll
                for (int w = 0; w < KW; ++w) ko[w] = rl64(col[s2][w], b);
                const uint32_t kll = rl32(kl[s2], b);
#pragma unroll
                for (int s = 0; s < SPL; ++s) kr[s] += key_less<VARLEN, KW>(ko, kll, col[s], kl[s]) ? 1u : 0u;
            }
        }
        // continuation: if the new batch starts with the last key, the iterator stops
        if (cont) {
            bool dup = false;
#pragma unroll
            for (int s = 0; s < SPL; ++s) {
                bool eq = kl[s] == xl;
#pragma unroll
                for (int w = 0; w < KW; ++w) eq = eq && col[s][w] == x[w];
                dup |= keep[s] && kr[s] == 0 && eq;
            }
            if (ballot(dup)) break;
        }
        const uint32_t e = m < remaining ? m : remaining;
        // emit the e smallest kept records at produced + rank, R rows in flight
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            const bool emit = keep[s] && kr[s] < e;
            uint32_t img = 0;
            if (emit) {
                if (VIS) {
                    uint8_t st;
                    img = scan_visible(t, t.slot[base + s * 64 + lane], rid, st);
                    row_status[produced + kr[s]] = st;
                } else {
                    img = t.slot[base + s * 64 + lane].image;
                }
            }
            uint64_t em = ballot(emit);
            if (em && t.stride <= 512) {  // small rows: several per load instruction
                copy_rows_flat<4>(t, em, img, produced + kr[s], recs, lane);
                em = 0;
            }
            while (em) {
                uint32_t imr[R], dr[R];
                int nk = 0;
                for (; nk < R && em; ++nk) {
                    const int b = __builtin_ctzll(em);
                    em &= em - 1;
                    imr[nk] = rl32(img, b);
                    dr[nk] = produced + rl32(kr[s], b);
                }
                copy_rows<R>(t, imr, dr, nk, recs, lane);
            }
        }
        produced += e;
        remaining -= e;
        if (e < m) break;
        // last record popped: continue from its key with le_child = false (next_leaf_after)
        uint32_t lastl = 0;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            const uint64_t lm = ballot(keep[s] && kr[s] == m - 1);
            if (lm) {
                const int b = __builtin_ctzll(lm);
#pragma unroll
                for (int w = 0; w < KW; ++w) x[w] = rl64(col[s][w], b);
                lastl = rl32(kl[s], b);
            }
        }
        xl = lastl;
        leaf = uni32(next_leaf_after<VARLEN, KW>(t, leaf, x, xl));
        cont = true;
    }
    if (lane == 0) *count_out = produced;
}

// Range scan for leaves of many slot groups (wide-key tables, up to 1024 slots) and scans of
// at most 63 records: RangeScanBySize's collection (first to_scan+1 qualifying records in slot
// order) walks only the slot groups whose max key (leaf head) reaches the start key and stops
// as soon as to_scan+1 records are held; the kept records (<= 64) go to a per-wave LDS list,
// one lane per record ranks them (std::sort) and they are handed to the sink in key order.
//
// Sinks: emit() sees, per lane, whether the lane emits a record on this leaf visit (`on`), its
// slot, its rank `kr` among this visit's records (`produced` records came before) and its key
// words; it returns true to end the scan early.
template <bool VIS>
struct RowSink {  // rows (and, for VIS, per-record statuses) as scan_one writes them
    uint8_t *recs;
    uint8_t *row_status;
    uint32_t rid;
    template <int KW>
    __device__ __forceinline__ bool emit(const DevTable &t, uint64_t base, bool on, uint32_t mslot, uint32_t kr,
                                         uint32_t produced, const uint64_t *, uint32_t lane) {
        uint32_t img = 0;
        if (on) {
            if (VIS) {
                uint8_t st;
                img = scan_visible(t, t.slot[base + mslot], rid, st);
                row_status[produced + kr] = st;
            } else {
                img = t.slot[base + mslot].image;
            }
        }
        uint64_t em = ballot(on);
        if (em && t.stride <= 512) {  // small rows: several per load instruction
            copy_rows_flat<4>(t, em, img, produced + kr, recs, lane);
            em = 0;
        }
        while (em) {
            uint32_t imr[4], dr[4];
            int nk = 0;
            for (; nk < 4 && em; ++nk) {
                const int b = __builtin_ctzll(em);
                em &= em - 1;
                imr[nk] = rl32(img, b);
                dr[nk] = produced + rl32(kr, b);
            }
            copy_rows<4>(t, imr, dr, nk, recs, lane);
        }
        return false;
    }
};

// IndexScanExecutor range branch consumed up to its first produced tuple (LATEST or OLD) whose
// key begins with the start key's first `words` order words -- a predicate over the scan that
// keeps only that tuple (TPC-C stock-level, tpcc_stock_level.cpp:104-135, takes ol_i_ids[0]).
// Result (wave-uniform): the tuple's heap row and status, or 0xFFFFFFFF / NOT_FOUND.
template <int KW>
struct FirstPrefixSink {
    uint64_t pre[KW];
    uint32_t words;
    uint32_t rid;
    uint32_t img;
    uint32_t st;
    template <int KW2>
    __device__ __forceinline__ bool emit(const DevTable &t, uint64_t base, bool on, uint32_t mslot, uint32_t kr,
                                         uint32_t, const uint64_t *mk, uint32_t) {
        uint8_t s = ST_NOT_FOUND;
        uint32_t im = 0xFFFFFFFFu;
        bool pass = false;
        if (on) {
            im = scan_visible(t, t.slot[base + mslot], rid, s);
            pass = s == ST_LATEST || s == ST_OLD;
#pragma unroll
            for (int w = 0; w < KW; ++w)
                if ((uint32_t)w < words) pass = pass && mk[w] == pre[w];
        }
        uint64_t pm = ballot(pass);
        if (!pm) return false;
        uint32_t best = 0xFFFFFFFFu;
        int bl = 0;
        while (pm) {  // the passing record of lowest rank
            const int b = __builtin_ctzll(pm);
            pm &= pm - 1;
            const uint32_t k = rl32(kr, b);
            if (k < best) {
                best = k;
                bl = b;
            }
        }
        img = rl32(im, bl);
        st = rl32((uint32_t)s, bl);
        return true;
    }
};

template <bool VARLEN, int SPL, int KW, class Sink>
__device__ uint32_t scan_one_compact(const DevTable &t, const uint64_t *x0, uint32_t xl, uint32_t leaf,
                                     uint32_t scan_size, uint32_t lane, Sink &sink, uint64_t *lk, uint32_t *ll,
                                     uint32_t *ls) {
    uint32_t remaining = scan_size, produced = 0;
    bool cont = false;
    uint64_t x[KW];
#pragma unroll
    for (int w = 0; w < KW; ++w) x[w] = x0[w];
    for (uint32_t guard = 0; guard < scan_size + 2 && remaining > 0; ++guard) {
        const uint64_t base = (uint64_t)leaf * t.cap;
        const uint8_t *hd = t.head + (uint64_t)leaf * t.head_bytes;
        const uint32_t mp = *reinterpret_cast<const uint32_t *>(hd + head_info_offset(t.cap, KW)) >> 16;  // info word
        // slot groups that can hold a key >= x (lane g tests group g's max key)
        bool act = false;
        if (lane < (uint32_t)SPL) {
            const uint64_t *gm = reinterpret_cast<const uint64_t *>(hd + head_gmax_offset(t.cap)) + lane * KW;
            uint64_t g[KW];
#pragma unroll
            for (int w = 0; w < KW; ++w) g[w] = gm[w];
            act = !kw_lt<KW>(g, x);
        }
        uint64_t active = ballot(act);
        const uint32_t to_scan = remaining;
        uint32_t kept = 0;
        while (active) {
            const int s = __builtin_ctzll(active);
            active &= active - 1;
            const uint64_t vm = head_vis(t, leaf, s);
            if (!vm) continue;
            const bool vis = (vm >> lane) & 1;
            uint64_t col[KW];
#pragma unroll
            for (int w = 0; w < KW; ++w) col[w] = t.okey[((uint64_t)leaf * KW + w) * t.cap + s * 64 + lane];
            uint32_t kl = t.key_width;
            if (VARLEN) kl = vis ? meta_keylen(t.slot[base + s * 64 + lane].meta) : 0u;
            const uint64_t q = ballot(vis && !key_less<VARLEN, KW>(col, kl, x, xl));
            if (!q) continue;
            const uint32_t rank = kept + count_below(q);
            const bool take = ((q >> lane) & 1) && rank <= to_scan;
            if (take) {
#pragma unroll
                for (int w = 0; w < KW; ++w) lk[rank * KW + w] = col[w];
                ll[rank] = kl;
                ls[rank] = (uint32_t)(s * 64) + lane;
            }
            kept += (uint32_t)__builtin_popcountll(ballot(take));
            if (kept > to_scan) break;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t m = kept;
        if (m == 0) break;
        // lane k < m holds kept record k; its rank among the kept records = position after sort
        const bool mine = lane < m;
        uint64_t mk[KW];
        uint32_t ml = 0, mslot = 0;
#pragma unroll
        for (int w = 0; w < KW; ++w) mk[w] = mine ? lk[lane * KW + w] : 0ull;
        if (mine) {
            ml = ll[lane];
            mslot = ls[lane];
        }
        // the list is in slot order; when its last (highest) slot lies in the leaf's monotone slot
        // prefix [0, mp) (info word), keys increase with the slot and the list order is the rank
        const bool mono = ls[m - 1] < mp;
        uint32_t kr = mono ? lane : 0u;
        for (uint32_t j = 0; j < (mono ? 0u : m); ++j) {
            uint64_t kj[KW];
#pragma unroll
            for (int w = 0; w < KW; ++w) kj[w] = lk[j * KW + w];
            kr += (mine && key_less<VARLEN, KW>(kj, ll[j], mk, ml)) ? 1u : 0u;
        }
        __builtin_amdgcn_wave_barrier();  // the LDS list is rewritten on the next leaf
        if (cont) {
            bool eq = ml == xl;
#pragma unroll
            for (int w = 0; w < KW; ++w) eq = eq && mk[w] == x[w];
            if (ballot(mine && kr == 0 && eq)) break;
        }
        const uint32_t e = m < remaining ? m : remaining;
        if (sink.template emit<KW>(t, base, mine && kr < e, mslot, kr, produced, mk, lane)) {
            produced += e;
            break;
        }
        produced += e;
        remaining -= e;
        if (e < m) break;
        // last record popped: continue from its key with le_child = false (next_leaf_after)
        const uint64_t lm = ballot(mine && kr == m - 1);
        const int b = __builtin_ctzll(lm);
#pragma unroll
        for (int w = 0; w < KW; ++w) x[w] = rl64(mk[w], b);
        xl = rl32(ml, b);
        leaf = uni32(next_leaf_after<VARLEN, KW>(t, leaf, x, xl));
        cont = true;
    }
    return produced;
}

// one scan of scan_compact (a wave; the LDS buffers are the wave's)
template <bool VARLEN, int SPL, int KW, bool VIS>
__device__ __forceinline__ void scan_compact_one(const DevTable &t, const uint64_t *keys, const uint16_t *lens, uint64_t i,
                                                 uint32_t scan_size, uint32_t *counts, uint8_t *recs,
                                                 const uint32_t *rids, uint8_t *row_status, uint32_t lane,
                                                 uint64_t *s_keys, uint32_t *s_len, uint32_t *s_slot) {
    const uint32_t len = t.key_width ? t.key_width : (lens ? (uint32_t)lens[i] : 8u);
    uint64_t ok[KW];
    load_okey<KW>(keys, i, true, len, ok);
    const uint32_t leaf = uni32(resolve_leaf_uniform<VARLEN, KW>(t, ok, len, true, lane));
    RowSink<VIS> sink{recs + i * (uint64_t)scan_size * t.stride, VIS ? row_status + i * (uint64_t)scan_size : nullptr,
                      VIS ? (rids ? rids[i] : 0xFFFFFFFEu) : 0u};
    const uint32_t produced =
        scan_one_compact<VARLEN, SPL, KW>(t, ok, len, leaf, scan_size, lane, sink, s_keys, s_len, s_slot);
    if (lane == 0) counts[i] = produced;
}

template <bool VARLEN, int SPL, int KW, bool VIS>
__global__ __launch_bounds__(256) void scan_kernel_compact(DevTable t, const uint64_t *__restrict__ keys,
                                                           const uint16_t *__restrict__ lens, uint64_t n,
                                                           uint32_t scan_size, uint32_t *__restrict__ counts,
                                                           uint8_t *__restrict__ recs,
                                                           const uint32_t *__restrict__ rids,
                                                           uint8_t *__restrict__ row_status) {
    __shared__ uint64_t s_keys[4][64 * KW];
    __shared__ uint32_t s_len[4][64], s_slot[4][64];
    const uint32_t lane = lane_id(), wv = uni32(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t i = wave; i < n; i += nwaves)
        scan_compact_one<VARLEN, SPL, KW, VIS>(t, keys, lens, i, scan_size, counts, recs, rids, row_status, lane,
                                               s_keys[wv], s_len[wv], s_slot[wv]);
}

// two single scans of two tables (the same leaf size, 8-byte keys, at most 63 records each) in
// one launch: block 0 scans t0 from k0[0], block 1 t1 from k1[0] -- CH-Q2's REGION and NATION
// scans, whose latency chains then overlap instead of running back to back
template <int SPL>
__global__ __launch_bounds__(64) void scan_pair_compact_kernel(DevTable t0, DevTable t1, const uint64_t *__restrict__ k0,
                                                             const uint64_t *__restrict__ k1, uint32_t sz0, uint32_t sz1,
                                                             uint32_t *__restrict__ c0, uint32_t *__restrict__ c1,
                                                             uint8_t *__restrict__ r0, uint8_t *__restrict__ r1) {
    __shared__ uint64_t s_keys[64];
    __shared__ uint32_t s_len[64], s_slot[64];
    const uint32_t lane = lane_id();
    if (blockIdx.x == 0)
        scan_compact_one<false, SPL, 1, false>(t0, k0, nullptr, 0, sz0, c0, r0, nullptr, nullptr, lane, s_keys, s_len,
                                               s_slot);
    else
        scan_compact_one<false, SPL, 1, false>(t1, k1, nullptr, 0, sz1, c1, r1, nullptr, nullptr, lane, s_keys, s_len,
                                               s_slot);
}

// The IndexScanExecutor range scan of `scan_size` records from key i (a wave per scan, the
// start-leaf descents of kFirstChunk scans done lane-parallel first), kept
// only up to its first produced tuple with the start key's first `words` order words
// (FirstPrefixSink); img_out[i] / st_out[i] = that tuple's heap row and status.
constexpr int kFirstChunk = 16;
constexpr uint8_t kFirstUndecided = 0xFE;  // scan_first_split_kernel -> scan_first_rest_kernel
// Point probes of the one-probe-in-flight instances (fixed-width keys of 9..32 bytes, or
// 8-byte keys in leaves above 128 slots) in two stages per chunk of CH probes -- the results of
// probe_kernel<false, SPL, 1, .., KW, CH>:
//  A (wave per probe, in turn): the leaf head's fingerprint bytes (the next 4 probes' in flight
//    while this one runs -- the next one only for leaves above 256 slots, whose larger heads
//    would cost occupancy), one ballot per slot group, and the candidate slots in slot order
//    written to LDS (at most kProbeCand; a probe with more is resolved by a lane-serial walk of
//    its leaf head in stage B);
//  B (lane per probe, all CH together): each candidate's slot word and remaining key words in
//    slot order until the first confirmed one (SearchRecordMeta's first hit), then
//    visibility() -- per lane, so the CH probes' dependent loads are in flight together instead
//    of one probe's at a time.
//  Rows (if requested) are then copied wave-wide, probe by probe, as probe_kernel's phase 4.
constexpr int kProbeCand = 8;
template <int SPL, int KW, int CH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void probe_split_kernel(DevTable t, const uint64_t *__restrict__ keys,
                                                          const uint32_t *__restrict__ rids,
                                                          const uint32_t *__restrict__ leaf_in, uint64_t n,
                                                          stage_probe_out_dev *__restrict__ out,
                                                          uint8_t *__restrict__ recs,
                                                          const uint64_t *__restrict__ dn) {
    __shared__ uint16_t s_cand[4][64][kProbeCand];
    if (dn) n = *dn < n ? *dn : n;  // the batch's size as a previous kernel left it (launched for n at most)
    const uint32_t lane = lane_id(), wv = uni32(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t out_chunks = t.stride >> 4;
    const uint32_t len = t.key_width;
    for (uint64_t base = wave * CH; base < n; base += nwaves * CH) {
        const uint64_t i = base + lane;
        const bool valid = lane < (uint32_t)CH && i < n;
        const uint32_t rid = rids ? (valid ? rids[i] : 0u) : 0xFFFFFFFEu;
        uint64_t ok[KW];
        load_okey<KW>(keys, i, valid, len, ok);
        uint32_t leaf = 0;
        if (valid) leaf = leaf_in ? leaf_in[i] : resolve_leaf<false, KW>(t, ok, len, true);
        if (leaf > t.nseps) leaf = t.nseps;  // host-supplied ids are clamped to the table
        const uint32_t fx_mine = key_fp_words(ok, KW);
        const int cnt = (int)((n - base) < CH ? (n - base) : CH);
        // ---- stage A: the heads of the next PD probes in flight while one is examined (a ring of
        // PD register sets, indexed statically by unrolling PD probes per pass)
        constexpr int PD = SPL <= 4 ? 4 : 1;
        uint32_t pf[PD][SPL];
#pragma unroll
        for (int d = 0; d < PD; ++d) {
            if (d < cnt) {
                const uint8_t *h = t.head + (uint64_t)rl32(leaf, d) * t.head_bytes;
#pragma unroll
                for (int s = 0; s < SPL; ++s) pf[d][s] = h[s * 64 + lane];
            }
        }
        uint32_t my_nc = 0;
        for (int j0 = 0; j0 < cnt; j0 += PD) {
#pragma unroll
            for (int u = 0; u < PD; ++u) {
                const int j = j0 + u;
                if (j >= cnt) break;
                uint32_t fpb[SPL];
#pragma unroll
                for (int s = 0; s < SPL; ++s) fpb[s] = pf[u][s];
                if (j + PD < cnt) {
                    const uint8_t *h = t.head + (uint64_t)rl32(leaf, j + PD) * t.head_bytes;
#pragma unroll
                    for (int s = 0; s < SPL; ++s) pf[u][s] = h[s * 64 + lane];
                }
                const uint32_t fx = rl32(fx_mine, j);
                uint32_t nc = 0;
#pragma unroll
                for (int s = 0; s < SPL; ++s) {
                    const bool c = fpb[s] == fx;
                    const uint64_t cm = ballot(c);
                    const uint32_t r = nc + count_below(cm);
                    if (c && r < (uint32_t)kProbeCand) s_cand[wv][j][r] = (uint16_t)(s * 64 + lane);
                    nc += (uint32_t)__builtin_popcountll(cm);
                }
                if (lane == (uint32_t)j) my_nc = nc;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- stage B: lane = probe
        int slot = -1;
        uint64_t m = 0;
        uint32_t nx = 0, im = 0;
        if (valid) {
            const uint64_t lb = (uint64_t)leaf * t.cap;
            auto confirm = [&](uint32_t sl) {
                const u32x4 *w = reinterpret_cast<const u32x4 *>(t.slot + lb + sl);
                const u32x4 w0 = w[0], w1 = w[1];
                bool eq = (((uint64_t)w0.y << 32) | w0.x) == ok[0];
#pragma unroll
                for (int k = 1; k < KW; ++k) eq = eq && t.okey[((uint64_t)leaf * KW + k) * t.cap + sl] == ok[k];
                if (eq) {
                    slot = (int)sl;
                    m = ((uint64_t)w0.w << 32) | w0.z;
                    nx = w1.x;
                    im = w1.y;
                }
                return eq;
            };
            if (my_nc <= (uint32_t)kProbeCand) {
                for (uint32_t c = 0; c < my_nc; ++c)
                    if (confirm(s_cand[wv][lane][c])) break;
            } else {  // more candidates than the list holds: walk the head in slot order
                const uint8_t *h = t.head + (uint64_t)leaf * t.head_bytes;
                for (uint32_t sl = 0; sl < t.cap; ++sl)
                    if (h[sl] == fx_mine && confirm(sl)) break;
            }
        }
        ProbeRes r;
        visibility(t, slot, m, nx, im, rid, r);
        // rows: wave-wide, probe by probe
        if (recs) {
            for (int j = 0; j < cnt; ++j) {
                const uint32_t img = rl32(r.image, j);
                for (uint32_t c0 = 0; c0 < out_chunks; c0 += 64) {
                    const uint32_t c = c0 + lane;
                    if (c >= out_chunks) continue;
                    u32x4 v = u32x4{0, 0, 0, 0};
                    if (img != 0xFFFFFFFFu) v = heap_chunk(t, img, c);
                    st16<1>(v, recs + (base + j) * (uint64_t)t.stride, c * 16u);
                }
            }
        }
        if (valid) {
            u32x4 a, b;
            pack_out(leaf, r, a, b);
            uint8_t *ob = reinterpret_cast<uint8_t *>(out + base);
            st16<1>(a, ob, lane * 32u);
            st16<1>(b, ob, lane * 32u + 16u);
        }
        __builtin_amdgcn_wave_barrier();  // s_cand is rewritten by the next chunk
    }
}

// Wave-cooperative lower bound of the wave's 64 fixed-width keys (one per lane, le_child), for
// the one-probe-in-flight tables whose separators are 2-4 words: per level a team of f lanes
// (the node's fanout, 16 inner / 8 bottom) reads one key's node, one entry per lane -- 64 / f
// keys per load instruction, each team's f entries contiguous -- instead of every lane reading
// its own whole node (a lane's 16 loads of 16 B touch 64 different nodes per instruction: 4x the
// cache lines for the texture addresser, CH-Q2's STOCK probe ran it 58-79 % busy, r05/lanepmc).
// A team's ballot bits count its key's separators below the key; the keys and their nodes pass
// through LDS (s_x: 64 keys, s_node: their nodes at this level).  All 64 lanes take part.
template <int KW>
__device__ __forceinline__ uint32_t coop_lower_bound(const DevTable &t, const uint64_t *ok, uint32_t lane,
                                                     uint64_t *s_x, uint32_t *s_node) {
#pragma unroll
    for (int j = 0; j < KW; ++j) s_x[lane * KW + j] = ok[j];
    uint32_t node = 0;
    for (int lvl = (int)t.levels - 1; lvl >= 0; --lvl) {
        const uint32_t f = lvl > 0 ? (uint32_t)kTreeFanout : (uint32_t)kLeafFanout;
        const uint32_t sh = lvl > 0 ? 4u : 3u, kpr = 64u >> sh;  // keys per round: 4 / 8
        const uint32_t rounds = 64u / kpr;                        // 16 / 8
        s_node[lane] = node;
        __builtin_amdgcn_wave_barrier();
        const uint64_t lbase = t.level_off[lvl];
        const uint32_t e = lane & (f - 1), kq = lane >> sh;  // entry of the node, key in the round
        const uint32_t my_round = lane / kpr, my_team = lane % kpr;
        uint64_t ball = 0;
        // rounds in batches of 8 whose loads are in flight together (8 x KW x 8 B per lane)
        constexpr int kBatch = 8;
#pragma unroll
        for (int r0 = 0; r0 < 16; r0 += kBatch) {
            if ((uint32_t)r0 >= rounds) break;  // wave-uniform: the bottom level has 8 rounds
            uint64_t w[kBatch][KW];
#pragma unroll
            for (int r = 0; r < kBatch; ++r) {
                const uint32_t kk = (uint32_t)(r0 + r) * kpr + kq;
                const uint64_t ent = lbase + (uint64_t)s_node[kk] * f + e;
#pragma unroll
                for (int j = 0; j < KW; ++j) w[r][j] = t.tree[ent * KW + j];
            }
#pragma unroll
            for (int r = 0; r < kBatch; ++r) {
                const uint32_t kk = (uint32_t)(r0 + r) * kpr + kq;
                uint64_t x[KW];
#pragma unroll
                for (int j = 0; j < KW; ++j) x[j] = s_x[kk * KW + j];
                const uint64_t b = __builtin_amdgcn_ballot_w64(kw_lt<KW>(w[r], x));
                ball = (uint32_t)(r0 + r) == my_round ? b : ball;
            }
        }
        const uint32_t cnt = (uint32_t)__builtin_popcountll((ball >> (my_team * f)) & ((1ull << f) - 1));
        node = node * f + cnt;
        __builtin_amdgcn_wave_barrier();  // s_node is rewritten by the next level
    }
    return node < t.nseps ? node : t.nseps;
}

// Point probes of the same instances as probe_split_kernel with a lane per probe throughout
// (the default for leaves of up to 256 slots): each lane descends, loads its leaf head's
// fingerprint bytes itself (SPL x 4 16-B loads, all in flight), finds its candidate slots in slot
// order with byte-wise compares in registers, and confirms the first three candidates in up to
// three rounds of loads that every lane of the wave issues together -- 64 probes' dependent
// loads in flight per wave at every step instead of 4-16 (SearchRecordMeta's first hit; a probe
// with more than three candidates falls back to a walk of the rest).  Then visibility() and the
// rows, wave-wide, as probe_split_kernel.
// MISS (launch_probe_missed): the hit is also evaluated at every read id mrids[0..mnq) and a
// probe that produces no tuple at read id q sets missed[q] -- launch_revisit_segments' miss pass
// folded into the probe, whose slot word is already in registers.
template <int SPL, int KW, bool MISS = false>
__global__ __launch_bounds__(256) void probe_lane_kernel(DevTable t, const uint64_t *__restrict__ keys,
                                                         const uint32_t *__restrict__ rids,
                                                         const uint32_t *__restrict__ leaf_in, uint64_t n,
                                                         stage_probe_out_dev *__restrict__ out,
                                                         uint8_t *__restrict__ recs, const uint64_t *__restrict__ dn,
                                                         const uint32_t *__restrict__ mrids = nullptr,
                                                         uint32_t mnq = 0, int32_t *__restrict__ missed = nullptr) {
    static_assert(SPL <= 4, "head of at most 256 slots in registers");
    __shared__ uint64_t s_x[4][64 * KW];
    __shared__ uint32_t s_node[4][64];
    if (dn) n = *dn < n ? *dn : n;
    const uint32_t lane = lane_id(), wv = uni32(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t out_chunks = t.stride >> 4;
    const uint32_t len = t.key_width;
    for (uint64_t base = wave * 64; base < n; base += nwaves * 64) {
        const uint64_t i = base + lane;
        const bool valid = i < n;
        const uint32_t rid = rids ? (valid ? rids[i] : 0u) : 0xFFFFFFFEu;
        uint64_t ok[KW];
        load_okey<KW>(keys, i, valid, len, ok);
        uint32_t leaf = 0;
        if (leaf_in) leaf = valid ? leaf_in[i] : 0u;
        else leaf = coop_lower_bound<KW>(t, ok, lane, s_x[wv], s_node[wv]);  // every lane takes part
        if (!valid) leaf = 0;
        if (leaf > t.nseps) leaf = t.nseps;
        const uint32_t rep = (key_fp_words(ok, KW) & 0xFFu) * 0x01010101u;
        // the head: fingerprint byte j = slot j
        u32x4 hv[SPL * 4];
        const u32x4 *hp = reinterpret_cast<const u32x4 *>(t.head + (uint64_t)leaf * t.head_bytes);
#pragma unroll
        for (int q = 0; q < SPL * 4; ++q) hv[q] = valid ? hp[q] : u32x4{0, 0, 0, 0};
        // candidates in slot order: the first three kept, the count of all
        uint32_t c0 = 0, c1 = 0, c2 = 0, nc = 0;
#pragma unroll
        for (int q = 0; q < SPL * 4; ++q) {
            const uint32_t wq[4] = {hv[q].x, hv[q].y, hv[q].z, hv[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t w = wq[e] ^ rep;
                uint32_t zm = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;  // bytes equal to the fingerprint
                while (zm) {
                    const uint32_t sl = (uint32_t)(q * 16 + e * 4) + ((uint32_t)__builtin_ctz(zm) >> 3);
                    c0 = nc == 0 ? sl : c0;
                    c1 = nc == 1 ? sl : c1;
                    c2 = nc == 2 ? sl : c2;
                    ++nc;
                    zm &= zm - 1;
                }
            }
        }
        if (!valid) nc = 0;
        int slot = -1;
        uint64_t m = 0;
        uint32_t nx = 0, im = 0;
        const uint64_t lb = (uint64_t)leaf * t.cap;
        auto confirm = [&](uint32_t sl) {
            const u32x4 *w = reinterpret_cast<const u32x4 *>(t.slot + lb + sl);
            const u32x4 w0 = w[0], w1 = w[1];
            bool eq = (((uint64_t)w0.y << 32) | w0.x) == ok[0];
#pragma unroll
            for (int k = 1; k < KW; ++k) eq = eq && t.okey[((uint64_t)leaf * KW + k) * t.cap + sl] == ok[k];
            if (eq) {
                slot = (int)sl;
                m = ((uint64_t)w0.w << 32) | w0.z;
                nx = w1.x;
                im = w1.y;
            }
            return eq;
        };
        // rounds: every lane still looking confirms its next candidate, the loads together
        if (nc > 0) confirm(c0);
        if (slot < 0 && nc > 1) confirm(c1);
        if (slot < 0 && nc > 2) confirm(c2);
        if (slot < 0 && nc > 3) {  // rare: walk the rest of the head in slot order
            const uint8_t *h = t.head + (uint64_t)leaf * t.head_bytes;
            const uint8_t fx = (uint8_t)rep;
            for (uint32_t sl = c2 + 1; sl < t.cap; ++sl)
                if (h[sl] == fx && confirm(sl)) break;
        }
        ProbeRes r;
        visibility(t, slot, m, nx, im, rid, r);
        if (MISS && valid)
            for (uint32_t q = 0; q < mnq; ++q) {
                ProbeRes rq;
                visibility(t, slot, m, nx, im, mrids[q], rq);
                if (rq.status != ST_LATEST && rq.status != ST_COPY && rq.status != ST_OLD) atomicOr(missed + q, 1);
            }
        if (recs) {  // rows: wave-wide, probe by probe
            const int cnt = (int)((n - base) < 64 ? (n - base) : 64);
            for (int j = 0; j < cnt; ++j) {
                const uint32_t img = rl32(r.image, j);
                for (uint32_t cc0 = 0; cc0 < out_chunks; cc0 += 64) {
                    const uint32_t c = cc0 + lane;
                    if (c >= out_chunks) continue;
                    u32x4 v = u32x4{0, 0, 0, 0};
                    if (img != 0xFFFFFFFFu) v = heap_chunk(t, img, c);
                    st16<1>(v, recs + (base + j) * (uint64_t)t.stride, c * 16u);
                }
            }
        }
        if (valid) {
            u32x4 a, b;
            pack_out(leaf, r, a, b);
            uint8_t *ob = reinterpret_cast<uint8_t *>(out + base);
            st16<1>(a, ob, lane * 32u);
            st16<1>(b, ob, lane * 32u + 16u);
        }
    }
}

// Chunk-cooperative lower bound of kFirstChunk fixed-width start keys: lane L works for scan
// L/4 and compares a quarter of each node (4 of the 16 inner entries, 2 of the 8 bottom ones);
// two xor-shuffles sum the quarter counts.  Same result as tree_lower_bound (le_child = true),
// one round trip per level for all 16 scans, a quarter of the per-lane loads and compares.
template <int KW>
__device__ __forceinline__ uint32_t chunk_lower_bound(const DevTable &t, const uint64_t *x, uint32_t part) {
    static_assert(kTreeFanout == 16 && kLeafFanout == 8, "quarters sized for 16 / 8 entries");
    uint32_t node = 0;
    for (int lvl = (int)t.levels - 1; lvl >= 0; --lvl) {
        const bool inner = lvl > 0;
        const uint32_t f = inner ? (uint32_t)kTreeFanout : (uint32_t)kLeafFanout;
        const uint32_t per = f / 4;
        const uint64_t *e = t.tree + (t.level_off[lvl] + (uint64_t)node * f + part * per) * KW;
        uint64_t w0[KW], w1[KW], w2[KW], w3[KW];
#pragma unroll
        for (int j = 0; j < KW; ++j) {
            w0[j] = e[j];
            w1[j] = e[KW + j];
            w2[j] = inner ? e[2 * KW + j] : ~0ull;
            w3[j] = inner ? e[3 * KW + j] : ~0ull;
        }
        int c = (kw_lt<KW>(w0, x) ? 1 : 0) + (kw_lt<KW>(w1, x) ? 1 : 0);
        if (inner) c += (kw_lt<KW>(w2, x) ? 1 : 0) + (kw_lt<KW>(w3, x) ? 1 : 0);
        c += __shfl_xor(c, 1);
        c += __shfl_xor(c, 2);
        node = node * f + (uint32_t)c;
    }
    return node < t.nseps ? node : t.nseps;
}

// The first-tuple scans split in two stages per chunk of 16 (same results as scan_first_kernel):
//  A (wave per scan, in turn): the start leaf's first visit -- active groups (all 16 scans' in
//    one round trip), the first group prefetched while the previous scan runs, the kept records
//    ranked (slot order when increasing), and the first e = min(m, scan_size) of them in rank
//    order written to LDS as candidates: the slot of a record carrying the start key's prefix,
//    or a hole;
//  B (lane per scan, all 16 together): the candidates' slot words and visibility in rank order,
//    the first LATEST / OLD one is the result -- one round trip for the 16 scans instead of one
//    per scan;
//  a scan whose first visit decides nothing (no candidate passed, the visit held m <= e records
//    and the scan has records left) is re-run by the general loop (scan_one_compact +
//    FirstPrefixSink), which continues across leaves.
template <int SPL, int KW, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void scan_first_split_kernel(
    DevTable t, const uint64_t *__restrict__ keys, uint64_t n, uint32_t scan_size, const uint32_t *__restrict__ rids,
    uint32_t words, uint32_t *__restrict__ img_out, uint8_t *__restrict__ st_out) {
    __shared__ uint64_t s_keys[4][64 * KW];
    __shared__ uint32_t s_slot[4][64];
    __shared__ uint16_t s_cand[4][kFirstChunk][64];
    const uint32_t lane = lane_id(), wv = uni32(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t len = t.key_width;
    uint64_t *lk = s_keys[wv];
    uint32_t *ls = s_slot[wv];
    constexpr uint16_t kHole = 0xFFFF;
    for (uint64_t c0 = wave * kFirstChunk; c0 < n; c0 += nwaves * kFirstChunk) {
        const uint64_t i = c0 + (lane >> 2);  // the scan this lane descends for
        const bool valid = i < n;
        uint64_t ok[KW];
        load_okey<KW>(keys, i, valid, len, ok);
        const uint32_t leafv = chunk_lower_bound<KW>(t, ok, lane & 3);
        const uint32_t ridv = valid && rids ? rids[i] : 0xFFFFFFFEu;
        const int cnt = (int)((n - c0) < (uint64_t)kFirstChunk ? (n - c0) : (uint64_t)kFirstChunk);
        // active slot groups of every start leaf (lane L tests groups L%4, L%4+4, ... of scan L/4)
        uint32_t actv = 0;
        {
            const uint64_t *gm = reinterpret_cast<const uint64_t *>(t.head + (uint64_t)leafv * t.head_bytes +
                                                                    head_gmax_offset(t.cap));
#pragma unroll
            for (int g = 0; g < SPL; g += 4) {
                const uint32_t gg = (uint32_t)g + (lane & 3);
                if (gg < (uint32_t)SPL) {
                    uint64_t e[KW];
#pragma unroll
                    for (int w = 0; w < KW; ++w) e[w] = gm[gg * KW + w];
                    actv |= kw_lt<KW>(e, ok) ? 0u : (1u << gg);
                }
            }
            actv |= (uint32_t)__shfl_xor((int)actv, 1);
            actv |= (uint32_t)__shfl_xor((int)actv, 2);
        }
        // the start leaf's monotone prefix length mp (info word, beside the group maxima): slots
        // [0, mp) hold strictly increasing keys
        const uint32_t mpv = *reinterpret_cast<const uint32_t *>(t.head + (uint64_t)leafv * t.head_bytes +
                                                                 head_info_offset(t.cap, KW)) >> 16;
        uint64_t pf_vm, pf_col[KW];
        int pf_s = -1;
        uint32_t pf_leaf = 0xFFFFFFFFu;
        // the next scan's first active group; the scans of a chunk are mostly one transaction's
        // consecutive orders in one leaf, so that group is often the one already held in the
        // pf registers (data of a kernel's lifetime never changes): then nothing is loaded and
        // the scan starts without a round trip
        auto prefetch = [&](int jn) {
            const uint32_t an = rl32(actv, 4 * jn), ln = rl32(leafv, 4 * jn);
            const int s = an ? __builtin_ctz(an) : 0;
            if (ln == pf_leaf && s == pf_s) return;
            pf_s = s;
            pf_leaf = ln;
            pf_vm = head_vis(t, ln, pf_s);
#pragma unroll
            for (int w = 0; w < KW; ++w) pf_col[w] = t.okey[((uint64_t)ln * KW + w) * t.cap + pf_s * 64 + lane];
        };
        prefetch(0);
        uint32_t my_info = 0;  // lane j: scan j's candidate count e | 0x100 if an undecided visit continues
        // ---- stage A
        for (int j = 0; j < cnt; ++j) {
            const int src = 4 * j;
            uint64_t x[KW];
#pragma unroll
            for (int w = 0; w < KW; ++w) x[w] = rl64(ok[w], src);
            const uint32_t leaf = rl32(leafv, src);
            const uint32_t mp = rl32(mpv, src);
            uint64_t active = ballot(lane < (uint32_t)SPL && ((rl32(actv, src) >> lane) & 1));
            bool pending = true, mono = false;
            uint32_t kept = 0;
            while (active) {
                const int s = __builtin_ctzll(active);
                active &= active - 1;
                uint64_t vm, col[KW];
                const bool from_pf = pending && s == pf_s;
                // a later group may be the one just prefetched for the next scan (in flight
                // since this scan's first group was consumed)
                if (from_pf || (leaf == pf_leaf && s == pf_s)) {
                    vm = pf_vm;
#pragma unroll
                    for (int w = 0; w < KW; ++w) col[w] = pf_col[w];
                } else {
                    vm = head_vis(t, leaf, s);
#pragma unroll
                    for (int w = 0; w < KW; ++w) col[w] = t.okey[((uint64_t)leaf * KW + w) * t.cap + s * 64 + lane];
                }
                const bool vis = (vm >> lane) & 1;
                const uint64_t q = ballot(vis && !kw_lt<KW>(col, x));
                const uint32_t rank = kept + count_below(q);
                // fast path: nothing kept yet, the group lies in the monotone prefix and holds
                // more than scan_size qualifying records -- the kept scan_size + 1 records are
                // its first ones, already in key order (unique keys), so their ranks are their
                // slot order and the first e = scan_size are the candidates; no LDS list
                if (kept == 0 && (uint32_t)s * 64u + 64u <= mp && (uint32_t)__builtin_popcountll(q) > scan_size) {
                    if (((q >> lane) & 1) && rank < scan_size) {
                        bool pfx = true;
#pragma unroll
                        for (int w = 0; w < KW; ++w)
                            if ((uint32_t)w < words) pfx = pfx && col[w] == x[w];
                        s_cand[wv][j][rank] = pfx ? (uint16_t)(s * 64 + (int)lane) : kHole;
                    }
                    if (from_pf) {
                        pending = false;
                        if (j + 1 < cnt) prefetch(j + 1);
                    }
                    mono = true;
                    break;
                }
                const bool take = ((q >> lane) & 1) && rank <= scan_size;
                if (take) {
#pragma unroll
                    for (int w = 0; w < KW; ++w) lk[rank * KW + w] = col[w];
                    ls[rank] = (uint32_t)(s * 64) + lane;
                }
                if (from_pf) {
                    pending = false;
                    if (j + 1 < cnt) prefetch(j + 1);
                }
                kept += (uint32_t)__builtin_popcountll(ballot(take));
                if (kept > scan_size) break;
            }
            if (pending && j + 1 < cnt) prefetch(j + 1);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t m = kept;
            uint32_t info = 0;
            if (mono) {
                info = scan_size;
            } else if (m > 0) {
                const bool mine = lane < m;
                uint64_t mk[KW];
                uint32_t mslot = 0;
#pragma unroll
                for (int w = 0; w < KW; ++w) mk[w] = mine ? lk[lane * KW + w] : 0ull;
                bool ord = true;
                if (mine) {
                    mslot = ls[lane];
                    if (lane > 0) {
                        uint64_t pk[KW];
#pragma unroll
                        for (int w = 0; w < KW; ++w) pk[w] = lk[(lane - 1) * KW + w];
                        ord = kw_lt<KW>(pk, mk);
                    }
                }
                uint32_t kr = lane;
                bool dup = false;
                if (ballot(!ord)) {
                    kr = 0;
                    for (uint32_t jj = 0; jj < m; ++jj) {
                        uint64_t kj[KW];
                        bool eq = jj != lane;
#pragma unroll
                        for (int w = 0; w < KW; ++w) {
                            kj[w] = lk[jj * KW + w];
                            eq = eq && kj[w] == mk[w];
                        }
                        kr += (mine && kw_lt<KW>(kj, mk)) ? 1u : 0u;
                        dup = dup || (mine && eq);
                    }
                }
                const uint32_t e = m < scan_size ? m : scan_size;
                if (ballot(dup)) {
                    info = 0x200u;  // equal keys share a rank: the general loop decides
                } else {
                    if (lane < e) s_cand[wv][j][lane] = kHole;
                    if (mine && kr < e) {
                        bool pfx = true;
#pragma unroll
                        for (int w = 0; w < KW; ++w)
                            if ((uint32_t)w < words) pfx = pfx && mk[w] == x[w];
                        if (pfx) s_cand[wv][j][kr] = (uint16_t)mslot;
                    }
                    info = e | (e == m && scan_size > e ? 0x100u : 0u);
                }
            }
            __builtin_amdgcn_wave_barrier();  // the LDS list is rewritten by the next scan
            if (lane == (uint32_t)j) my_info = info;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- stage B: lane j resolves scan j's candidates in rank order
        const uint32_t my_leaf = (uint32_t)__shfl((int)leafv, (int)(4 * (lane & 15)));
        const uint32_t my_rid = (uint32_t)__shfl((int)ridv, (int)(4 * (lane & 15)));
        uint32_t my_img = 0xFFFFFFFFu, my_st = ST_NOT_FOUND;
        bool found = false;
        if (lane < (uint32_t)cnt) {
            const uint32_t e = my_info & 0xFF;
            const uint64_t base = (uint64_t)my_leaf * t.cap;
            for (uint32_t c = 0; c < e; ++c) {
                const uint16_t sl = s_cand[wv][lane][c];
                if (sl == kHole) continue;
                uint8_t sv;
                const uint32_t im = scan_visible(t, t.slot[base + sl], my_rid, sv);
                if (sv == ST_LATEST || sv == ST_OLD) {
                    my_img = im;
                    my_st = sv;
                    found = true;
                    break;
                }
            }
        }
        // ---- undecided scans: marked for scan_first_rest_kernel
        if (lane < (uint32_t)cnt && ((!found && (my_info & 0x100u)) || (my_info & 0x200u))) my_st = kFirstUndecided;
        if (lane < (uint32_t)cnt) {
            img_out[c0 + lane] = my_img;
            st_out[c0 + lane] = (uint8_t)my_st;
        }
        __builtin_amdgcn_wave_barrier();  // s_cand is rewritten by the next chunk
    }
}

// The scans scan_first_split_kernel left undecided (st_out == kFirstUndecided): the general loop
// (scan_one_compact + FirstPrefixSink) from the start key, a wave per scan; 64 statuses are
// read per wave and step, so a batch without undecided scans costs one pass over st_out.
template <int SPL, int KW>
__global__ __launch_bounds__(256) void scan_first_rest_kernel(DevTable t, const uint64_t *__restrict__ keys,
                                                              uint64_t n, uint32_t scan_size,
                                                              const uint32_t *__restrict__ rids, uint32_t words,
                                                              uint32_t *__restrict__ img_out,
                                                              uint8_t *__restrict__ st_out) {
    __shared__ uint64_t s_keys[4][64 * KW];
    __shared__ uint32_t s_len[4][64], s_slot[4][64];
    const uint32_t lane = lane_id(), wv = uni32(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t len = t.key_width;
    for (uint64_t c0 = wave * 64; c0 < n; c0 += nwaves * 64) {
        const uint64_t i = c0 + lane;
        uint64_t und = ballot(i < n && st_out[i] == kFirstUndecided);
        while (und) {
            const int b = __builtin_ctzll(und);
            und &= und - 1;
            const uint64_t k = c0 + (uint64_t)b;
            uint64_t x[KW];
            load_okey<KW>(keys, k, true, len, x);
            FirstPrefixSink<KW> sink;
#pragma unroll
            for (int w = 0; w < KW; ++w) sink.pre[w] = x[w];
            sink.words = words;
            sink.rid = rids ? rids[k] : 0xFFFFFFFEu;
            sink.img = 0xFFFFFFFFu;
            sink.st = ST_NOT_FOUND;
            const uint32_t leaf = uni32(resolve_leaf_uniform<false, KW>(t, x, len, true, lane));
            scan_one_compact<false, SPL, KW>(t, x, len, leaf, scan_size, lane, sink, s_keys[wv], s_len[wv],
                                             s_slot[wv]);
            if (lane == 0) {
                img_out[k] = sink.img;
                st_out[k] = (uint8_t)sink.st;
            }
        }
    }
}

// One wave per scan (grid-stride over scans): the start key's descent is wave-uniform, and a
// wide grid keeps many scans -- and their R rows in flight each -- resident per CU.
template <bool VARLEN, int SPL, int R, int KW = 1, bool VIS = false>
__global__ __launch_bounds__(256) void scan_kernel(DevTable t, const uint64_t *__restrict__ keys,
                                                   const uint16_t *__restrict__ lens, uint64_t n, uint32_t scan_size,
                                                   uint32_t *__restrict__ counts, uint8_t *__restrict__ recs,
                                                   const uint32_t *__restrict__ rids = nullptr,
                                                   uint8_t *__restrict__ row_status = nullptr) {
    const uint32_t lane = lane_id();
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + uni32(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t i = wave; i < n; i += nwaves) {
        const uint32_t len = t.key_width ? t.key_width : (lens ? (uint32_t)lens[i] : 8u);
        uint64_t ok[KW];
        load_okey<KW>(keys, i, true, len, ok);
        const uint32_t leaf = uni32(resolve_leaf_uniform<VARLEN, KW>(t, ok, len, true, lane));
        scan_one<VARLEN, SPL, R, KW, VIS>(t, ok, len, leaf, scan_size, recs + i * (uint64_t)scan_size * t.stride,
                                          counts + i, lane, VIS ? (rids ? rids[i] : 0xFFFFFFFEu) : 0u,
                                          VIS ? row_status + i * (uint64_t)scan_size : nullptr);
    }
}

// ----------------------------------------------------------------------------------------
// MurmurHash64A (misc/murmur/MurmurHash2.cpp:99-147), lane per key

__device__ __forceinline__ uint64_t murmur64a_dev(const uint8_t *p, uint32_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = seed ^ ((uint64_t)len * m);
    const uint32_t nb = len / 8;
    for (uint32_t i = 0; i < nb; ++i) {
        uint64_t k = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) k |= (uint64_t)p[8 * i + b] << (8 * b);
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
    }
    const uint8_t *d2 = p + 8 * nb;
    const uint32_t rem = len & 7;
    if (rem) {
        for (int b = (int)rem - 1; b >= 0; --b) h ^= (uint64_t)d2[b] << (8 * b);
        h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}

__global__ __launch_bounds__(256) void murmur_kernel(const uint8_t *__restrict__ keys, uint32_t key_len,
                                                     uint32_t key_stride, uint64_t seed, uint64_t n,
                                                     uint64_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *p = keys + i * key_stride;
    if (key_len == 8 && (key_stride & 7) == 0) {  // the router's case: one aligned word
        const uint64_t m = 0xc6a4a7935bd1e995ull;
        uint64_t h = seed ^ (8ull * m);
        uint64_t k = *reinterpret_cast<const uint64_t *>(p);
        k *= m;
        k ^= k >> 47;
        k *= m;
        h ^= k;
        h *= m;
        h ^= h >> 47;
        h *= m;
        h ^= h >> 47;
        out[i] = h;
    } else {
        out[i] = murmur64a_dev(p, key_len, seed);
    }
}

// ----------------------------------------------------------------------------------------
// record-heap fill: row = [key padded to 8][payload][zero pad to stride]

__device__ __forceinline__ uint64_t splitmix64_dev(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t payload_word(const ImageDescDev &d, const uint8_t *arena, uint32_t j,
                                                 uint32_t payload_size) {
    const uint32_t off = j * 8;
    if (off >= payload_size) return 0;
    const uint32_t nb = payload_size - off < 8 ? payload_size - off : 8;
    uint64_t w;
    if (d.kind == 1) {
        w = 0;
        const uint8_t *s = arena + d.arg + off;
        for (uint32_t b = 0; b < nb; ++b) w |= (uint64_t)s[b] << (8 * b);
        return w;
    }
    if (d.mode == 0) w = 0x0101010101010101ull * (d.arg & 0xFF);
    else w = splitmix64_dev((d.arg << 8) ^ j);
    if (nb < 8) w &= (1ull << (8 * nb)) - 1;
    return w;
}

// 8 bytes of an arena row (kind 2 images: [key padded][payload] copied whole), zero past `limit`
__device__ __forceinline__ uint64_t arena_word(const uint8_t *arena, uint64_t base, uint32_t off, uint32_t limit) {
    if (off >= limit) return 0;
    const uint32_t nb = limit - off < 8 ? limit - off : 8;
    uint64_t w = 0;
    const uint8_t *s = arena + base + off;
    for (uint32_t b = 0; b < nb; ++b) w |= (uint64_t)s[b] << (8 * b);
    return w;
}

__global__ __launch_bounds__(256) void fill_kernel(uint8_t *__restrict__ heap, uint32_t stride, uint32_t payload_size,
                                                   uint32_t row_bytes, const ImageDescDev *__restrict__ descs,
                                                   const uint8_t *__restrict__ arena, uint64_t first, uint64_t count,
                                                   uint64_t ident_rowid0, uint32_t ident_key_width, int ident_mode) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t chunks = stride >> 4;
    for (uint64_t r = wave; r < count; r += nwaves) {
        ImageDescDev d;
        if (descs) {
            d = descs[r];
        } else {  // identity run: image = rowid = key (LoadYCSBRows)
            d.arg = ident_rowid0 + r;
            d.key_le = ident_key_width >= 8 ? d.arg : (d.arg & ((1ull << (8 * ident_key_width)) - 1));
            d.kind = 0;
            d.mode = (uint32_t)ident_mode;
        }
        u32x4 *row = reinterpret_cast<u32x4 *>(heap + (first + r) * stride);
        if (d.kind == 2) {
            for (uint32_t c = lane; c < chunks; c += 64) {
                const uint64_t w0 = arena_word(arena, d.arg, 16 * c, row_bytes);
                const uint64_t w1 = arena_word(arena, d.arg, 16 * c + 8, row_bytes);
                row[c] = u32x4{(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
            }
            continue;
        }
        for (uint32_t c = lane; c < chunks; c += 64) {
            uint64_t w0 = c == 0 ? d.key_le : payload_word(d, arena, 2 * c - 1, payload_size);
            uint64_t w1 = payload_word(d, arena, 2 * c, payload_size);
            row[c] = u32x4{(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
        }
    }
}

// Incremental publish: rewrite the heads of dirty leaves (16-B chunks) and the dirty slot
// words + key-plane entries in place.  One thread per chunk / slot, grid-stride.
__global__ __launch_bounds__(256) void patch_kernel(uint8_t *__restrict__ head, uint64_t *__restrict__ okey,
                                                    SlotInfo *__restrict__ slot, uint32_t head_bytes, uint32_t cap,
                                                    uint32_t kw, const uint32_t *__restrict__ head_leaf,
                                                    const u32x4 *__restrict__ head_src, uint64_t nhead,
                                                    const uint64_t *__restrict__ slot_idx,
                                                    const SlotInfo *__restrict__ slot_src,
                                                    const uint64_t *__restrict__ words, uint64_t nslot) {
    const uint32_t cpl = head_bytes >> 4;
    const uint64_t nchunk = nhead * cpl;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nchunk + nslot; i += stride) {
        if (i < nchunk) {
            const uint64_t l = i / cpl, c = i % cpl;
            reinterpret_cast<u32x4 *>(head + (uint64_t)head_leaf[l] * head_bytes)[c] = head_src[i];
        } else {
            const uint64_t k = i - nchunk, d = slot_idx[k];
            slot[d] = slot_src[k];
            const uint64_t leaf = d / cap, sl = d % cap;
            for (uint32_t j = 0; j < kw; ++j) okey[(leaf * kw + j) * cap + sl] = words[k * kw + j];
        }
    }
}

// ----------------------------------------------------------------------------------------
// launchers

static int grid_for(uint64_t waves_needed, int waves_per_block, int max_blocks) {
    uint64_t b = (waves_needed + waves_per_block - 1) / waves_per_block;
    if (b < 1) b = 1;
    if (b > (uint64_t)max_blocks) b = (uint64_t)max_blocks;
    return (int)b;
}

hipError_t launch_resolve(const DevTable &t, const uint64_t *keys, const uint16_t *lens, uint64_t n, int le_child,
                          uint32_t *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned b = (unsigned)((n + 255) / 256);
    if (t.key_words == 4) resolve_kernel<4><<<b, 256, 0, s>>>(t, keys, lens, n, le_child, out);
    else if (t.key_words == 2) resolve_kernel<2><<<b, 256, 0, s>>>(t, keys, lens, n, le_child, out);
    else resolve_kernel<1><<<b, 256, 0, s>>>(t, keys, lens, n, le_child, out);
    return hipGetLastError();
}

constexpr uint64_t kSmallBelow = 16384;  // 64-probe chunks: about the waves the chip holds at once

hipError_t launch_probe(const DevTable &t, const uint64_t *keys, const uint16_t *lens, const uint32_t *rids,
                        const uint32_t *leaf_in, uint64_t n, stage_probe_out_dev *out, uint8_t *recs, hipStream_t s,
                        const ProbeTuning &tune, const uint64_t *d_n, uint64_t shape_n) {
    if (n == 0) return hipSuccess;
    if (d_n) {  // device-sized batches: the wide-key / large-leaf kernels only
        if (!(t.key_words > 1 || (t.key_width != 0 && t.cap > 128))) return hipErrorInvalidValue;
    }
    const uint64_t chunks = (n + 63) / 64;
    const int blocks = grid_for(chunks, 4, tune.max_blocks > 0 ? tune.max_blocks : 16384);
    const bool var = t.key_width == 0;
    // wide fixed-width keys, and 8-byte keys in leaves above 128 slots (small rows): leaves of
    // up to 1024 slots -- probe_lane_kernel for leaves of up to 256 slots, probe_split_kernel
    // above (in 16-probe wave chunks when 64-probe ones cannot fill the chip).  Retired (DESIGN
    // §4): probe_kernel's one-probe-in-flight form and the split kernel for every leaf size.
    if (t.key_words > 1 || (!var && t.cap > 128)) {
        // launch shape from the expected size (a device-sized batch's hint), the grid from n
        const uint64_t sn = d_n && shape_n ? std::min(shape_n, n) : n;
        const bool small = (sn + 63) / 64 < (uint64_t)kSmallBelow;  // fewer 64-probe chunks than the chip holds waves
        // tiny batches (fewer 16-probe chunks than a quarter of that, e.g. CH-Q2's ~2.5 K item
        // lookups): 4-probe wave chunks, a quarter of the serial probes per wave
        const bool tiny = (sn + 15) / 16 < (uint64_t)kSmallBelow / 4;
        const int mb = tune.max_blocks > 0 ? tune.max_blocks : 16384;
        const int wblocks = tiny ? grid_for((sn + 3) / 4, 4, mb) : small ? grid_for((sn + 15) / 16, 4, mb) : blocks;
        // the lane kernel strides over the batch: its grid from the expected size too
        const int lblocks = grid_for((sn + 63) / 64, 4, tune.max_blocks > 0 ? tune.max_blocks : 16384);
#define STAGE_PROBE_W(S, KW)                                                                                  \
    if (S <= 4)                                                                                               \
        probe_lane_kernel<(S <= 4 ? S : 4), KW><<<lblocks, 256, 0, s>>>(t, keys, rids, leaf_in, n, out, recs, d_n); \
    else if (tiny)                                                                                            \
        probe_split_kernel<S, KW, 4><<<wblocks, 256, 0, s>>>(t, keys, rids, leaf_in, n, out, recs, d_n);       \
    else if (small)                                                                                           \
        probe_split_kernel<S, KW, 16><<<wblocks, 256, 0, s>>>(t, keys, rids, leaf_in, n, out, recs, d_n);      \
    else                                                                                                      \
        probe_split_kernel<S, KW, 64><<<blocks, 256, 0, s>>>(t, keys, rids, leaf_in, n, out, recs, d_n)
#define STAGE_PROBE_WK(KW)                      \
    switch (t.cap / 64) {                       \
        case 1: STAGE_PROBE_W(1, KW); break;    \
        case 2: STAGE_PROBE_W(2, KW); break;    \
        case 4: STAGE_PROBE_W(4, KW); break;    \
        case 8: STAGE_PROBE_W(8, KW); break;    \
        default: STAGE_PROBE_W(16, KW); break;  \
    }
        if (t.key_words == 1) {
            STAGE_PROBE_WK(1)
        } else if (t.key_words == 2) {
            STAGE_PROBE_WK(2)
        } else {
            STAGE_PROBE_WK(4)
        }
#undef STAGE_PROBE_WK
#undef STAGE_PROBE_W
        return hipGetLastError();
    }
#define STAGE_PROBE(V, S, G) \
    probe_kernel<V, S, G><<<blocks, 256, 0, s>>>(t, keys, lens, rids, leaf_in, n, out, recs, nullptr, nullptr)
    if (tune.status_bytes == 16) {  // opt-in lean status records: the YCSB geometry only
        if (var || t.cap != 64 || tune.group != 8 || tune.store != 1) return hipErrorInvalidValue;
        probe_kernel<false, 1, 8, 1, 1, 64, 16><<<blocks, 256, 0, s>>>(t, keys, lens, rids, leaf_in, n, out, recs,
                                                                       nullptr, nullptr);
        return hipGetLastError();
    }
    if (t.cap == 64) {
        if (var) STAGE_PROBE(true, 1, 4);
        else if (tune.group == 1) STAGE_PROBE(false, 1, 1);
        else if (tune.group == 2) STAGE_PROBE(false, 1, 2);
        else if (tune.group == 4) STAGE_PROBE(false, 1, 4);
        else if (tune.store == 0)
            probe_kernel<false, 1, 8, 0><<<blocks, 256, 0, s>>>(t, keys, lens, rids, leaf_in, n, out, recs, nullptr,
                                                                 nullptr);
        else if (tune.store == 2)
            probe_kernel<false, 1, 8, 2><<<blocks, 256, 0, s>>>(t, keys, lens, rids, leaf_in, n, out, recs, nullptr,
                                                                 nullptr);
        else STAGE_PROBE(false, 1, 8);
    } else {
        if (var) STAGE_PROBE(true, 2, 4);
        else STAGE_PROBE(false, 2, 4);
    }
#undef STAGE_PROBE
    return hipGetLastError();
}

hipError_t launch_probe_missed(const DevTable &t, const uint64_t *keys, uint64_t n, stage_probe_out_dev *out,
                               hipStream_t s, const ProbeTuning &tune, const uint64_t *d_n, uint64_t shape_n,
                               const uint32_t *mrids, uint32_t mnq, int32_t *missed) {
    if (!probe_missed_supported(t)) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    const uint64_t sn = d_n && shape_n ? std::min(shape_n, n) : n;
    const int blocks = grid_for((sn + 63) / 64, 4, tune.max_blocks > 0 ? tune.max_blocks : 16384);
#define STAGE_PROBE_M(S, KW)                                                                                    \
    probe_lane_kernel<S, KW, true><<<blocks, 256, 0, s>>>(t, keys, nullptr, nullptr, n, out, nullptr, d_n, mrids, \
                                                          mnq, missed)
#define STAGE_PROBE_MK(KW)                   \
    switch (t.cap / 64) {                    \
        case 1: STAGE_PROBE_M(1, KW); break; \
        case 2: STAGE_PROBE_M(2, KW); break; \
        default: STAGE_PROBE_M(4, KW); break; \
    }
    if (t.key_words == 1) {
        STAGE_PROBE_MK(1)
    } else if (t.key_words == 2) {
        STAGE_PROBE_MK(2)
    } else {
        STAGE_PROBE_MK(4)
    }
#undef STAGE_PROBE_MK
#undef STAGE_PROBE_M
    return hipGetLastError();
}

bool probe_missed_supported(const DevTable &t) {
    // the lane kernel's instances: wide fixed-width keys, or 8-byte keys in leaves above 128
    // slots, in leaves of up to 256 slots
    const bool wide = t.key_words > 1 || (t.key_width != 0 && t.cap > 128);
    return wide && t.key_width != 0 && t.cap <= 256 && (t.cap == 64 || t.cap == 128 || t.cap == 256);
}

hipError_t launch_probe_fanout(const DevTable &t, const uint64_t *keys, const uint32_t *rids, uint64_t n,
                               const FanRange *fan, const uint32_t *flist, stage_probe_out_dev *out, uint8_t *recs,
                               hipStream_t s, const ProbeTuning &tune, const FanDest *dest) {
    if (!probe_fanout_supported(t)) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    if ((!recs && !dest) || (!fan && !flist)) return hipErrorInvalidValue;
    const int blocks = grid_for((n + 63) / 64, 4, tune.max_blocks > 0 ? tune.max_blocks : 16384);
    if (dest)
        probe_kernel<false, 1, 4, 1, 1, 64, 32, true, true><<<blocks, 256, 0, s>>>(t, keys, nullptr, rids, nullptr, n,
                                                                                   out, recs, fan, flist, dest);
    else
        probe_kernel<false, 1, 8, 1, 1, 64, 32, true><<<blocks, 256, 0, s>>>(t, keys, nullptr, rids, nullptr, n, out,
                                                                             recs, fan, flist);
    return hipGetLastError();
}

bool probe_fanout_supported(const DevTable &t) {
    return t.key_width != 0 && t.key_words == 1 && t.cap == 64 && t.stride <= 1024;
}

// launch_revisit: thread per (key i, read id q), revisit_one (visibility.hpp)
__global__ __launch_bounds__(256) void revisit_kernel(DevTable t, const stage_probe_out_dev *__restrict__ base,
                                                      uint64_t n, const uint32_t *__restrict__ rids, uint32_t nq,
                                                      const uint32_t *__restrict__ perm,
                                                      stage_probe_out_dev *__restrict__ out,
                                                      const uint64_t *__restrict__ dn) {
    if (dn) n = *dn < n ? *dn : n;  // out[q * n + i] with the device count n
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * nq) return;
    const uint64_t i = g % n, q = g / n;
    const u32x4 *bp = reinterpret_cast<const u32x4 *>(base + i);
    u32x4 a = bp[0], b = bp[1];
    revisit_one(t, rids[q], a, b);
    u32x4 *op = reinterpret_cast<u32x4 *>(out + q * n + (perm ? perm[i] : i));
    op[0] = a;
    op[1] = b;
}

// launch_revisit_segments, the misses: thread per (probe i, kRevisitQ read ids) -- the probe's
// status record and slot word are loaded once and the visibility walk redone per read id; nothing
// is stored but a miss (rare: the transaction aborts)
constexpr uint32_t kRevisitQ = 16;
__global__ __launch_bounds__(256) void revisit_missed_kernel(DevTable t, const stage_probe_out_dev *__restrict__ base,
                                                             uint64_t n, const uint32_t *__restrict__ rids, uint32_t nq,
                                                             int32_t *__restrict__ missed, const uint64_t *__restrict__ dn) {
    if (dn) n = *dn < n ? *dn : n;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * ((nq + kRevisitQ - 1) / kRevisitQ)) return;
    const uint64_t i = g % n;
    const uint32_t q0 = (uint32_t)(g / n) * kRevisitQ, q1 = q0 + kRevisitQ < nq ? q0 + kRevisitQ : nq;
    const u32x4 *bp = reinterpret_cast<const u32x4 *>(base + i);
    const u32x4 a0 = bp[0];
    const uint32_t slot = a0.z & 0xFFFF, leaf = a0.y;
    const bool redo = (a0.x & 0xFF) != ST_NOT_FOUND && slot < t.cap && leaf < t.nleaves;
    SlotInfo si = {};
    if (redo) si = t.slot[(uint64_t)leaf * t.cap + slot];
    for (uint32_t q = q0; q < q1; ++q) {
        uint32_t st = a0.x & 0xFF;
        if (redo) {
            ProbeRes r;
            visibility(t, (int)slot, si.meta, si.next, si.image, rids[q], r);
            st = r.status;
        }
        if (st != ST_LATEST && st != ST_COPY && st != ST_OLD) atomicOr(missed + q, 1);
    }
}

// launch_revisit_segments, the last probes: thread per (read id q, segment k)
__global__ __launch_bounds__(256) void revisit_last_kernel(DevTable t, const stage_probe_out_dev *__restrict__ base,
                                                           const uint64_t *__restrict__ seg_off,
                                                           const uint32_t *__restrict__ seg_cnt, uint32_t nseg,
                                                           const uint32_t *__restrict__ rids, uint32_t nq,
                                                           stage_probe_out_dev *__restrict__ last,
                                                           const uint64_t *__restrict__ dseg) {
    if (dseg) nseg = *dseg < nseg ? (uint32_t)*dseg : nseg;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint64_t)nseg * nq) return;
    const uint32_t k = (uint32_t)(g % nseg), q = (uint32_t)(g / nseg);
    const uint32_t c = seg_cnt[k];
    if (c == 0) return;
    const u32x4 *bp = reinterpret_cast<const u32x4 *>(base + seg_off[k] + c - 1);
    u32x4 a = bp[0], b = bp[1];
    revisit_one(t, rids[q], a, b);
    u32x4 *op = reinterpret_cast<u32x4 *>(last + g);
    op[0] = a;
    op[1] = b;
}

hipError_t launch_revisit_segments(const DevTable &t, const stage_probe_out_dev *base, uint64_t n,
                                   const uint64_t *seg_off, const uint32_t *seg_cnt, uint32_t nseg,
                                   const uint32_t *rids, uint32_t nq, stage_probe_out_dev *last, int32_t *missed,
                                   hipStream_t s, const uint64_t *d_n, const uint64_t *d_nseg) {
    if (nq == 0) return hipSuccess;
    const uint64_t tm = n * ((nq + kRevisitQ - 1) / kRevisitQ), tl = (uint64_t)nseg * nq;
    if (tm) revisit_missed_kernel<<<(unsigned)((tm + 255) / 256), 256, 0, s>>>(t, base, n, rids, nq, missed, d_n);
    if (tl)
        revisit_last_kernel<<<(unsigned)((tl + 255) / 256), 256, 0, s>>>(t, base, seg_off, seg_cnt, nseg, rids, nq, last,
                                                                         d_nseg);
    return hipGetLastError();
}

hipError_t launch_revisit(const DevTable &t, const stage_probe_out_dev *base, uint64_t n, const uint32_t *rids,
                          uint32_t nq, const uint32_t *perm, stage_probe_out_dev *out, hipStream_t s,
                          const uint64_t *d_n) {
    if (n == 0 || nq == 0) return hipSuccess;
    revisit_kernel<<<(unsigned)((n * nq + 255) / 256), 256, 0, s>>>(t, base, n, rids, nq, perm, out, d_n);
    return hipGetLastError();
}

// stage_probe_ident: a probe's hit slot (leaf, slot in its status record) -> the slot word's
// location handle and next handle, from the same published image.  A thread per probe.
__global__ __launch_bounds__(256) void ident_kernel(DevTable t, const stage_probe_out_dev *__restrict__ out, uint64_t n,
                                                    uint32_t *__restrict__ ident) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32x4 a = reinterpret_cast<const u32x4 *>(out + i)[0];
    const uint32_t status = a.x & 0xFF, leaf = a.y, slot = a.z & 0xFFFF;
    uint32_t loc = 0, next = 0;
    if (status != ST_NOT_FOUND && slot < t.cap && leaf < t.nleaves) {
        const u32x4 w1 = reinterpret_cast<const u32x4 *>(t.slot + (uint64_t)leaf * t.cap + slot)[1];
        next = w1.x;
        loc = w1.z;
    }
    reinterpret_cast<uint2 *>(ident)[i] = make_uint2(loc, next);
}

// stage_probe_batch_ex's is_for_update probes: a second pass over the flagged probes of a batch
// the ordinary probe has answered (so the probe kernels stay as they are).  The hit slot is in
// each status record -- also for an in-flight record the ordinary rule left NOT_FOUND (an
// uncommitted insert without a copy) -- and its slot word gives the for-update outcome
// (visibility<true>); the status record is rewritten and the row re-copied from the leaf image.
// A wave takes 64 probes and walks its flagged ones wave-uniformly (lanes 0-1 store the record,
// every lane a 16-B chunk of the row).
__global__ __launch_bounds__(256) void for_update_kernel(DevTable t, const uint8_t *__restrict__ fu,
                                                         const uint32_t *__restrict__ rids, uint64_t n,
                                                         stage_probe_out_dev *__restrict__ out, uint8_t *__restrict__ recs) {
    const uint32_t lane = lane_id();
    const uint64_t base = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + uni32(threadIdx.x >> 6)) * 64;
    const uint64_t i = base + lane;
    uint64_t todo = ballot(i < n && fu[i] != 0);
    const uint32_t chunks = t.stride >> 4;
    while (todo) {
        const int j = __builtin_ctzll(todo);
        todo &= todo - 1;
        const uint64_t p = base + (uint64_t)j;
        const u32x4 *op = reinterpret_cast<const u32x4 *>(out + p);
        u32x4 a = op[0], b = op[1];
        const uint32_t rid = rids ? rids[p] : 0xFFFFFFFEu;
        const uint32_t slot = a.z & 0xFFFF, leaf = a.y;
        uint32_t image = 0xFFFFFFFFu;
        if (slot < t.cap && leaf < t.nleaves) {
            const SlotInfo si = t.slot[(uint64_t)leaf * t.cap + slot];
            ProbeRes r;
            visibility<true>(t, (int)slot, si.meta, si.next, si.image, rid, r);
            pack_out(leaf, r, a, b);
            image = r.image;
        } else {
            a.x |= 2u << 8;  // no record: NOT_FOUND stays, flagged for update
        }
        if (lane < 2) reinterpret_cast<u32x4 *>(out + p)[lane] = lane == 0 ? a : b;
        if (recs) {
            for (uint32_t c = lane; c < chunks; c += 64) {
                u32x4 v = u32x4{0, 0, 0, 0};
                if (image != 0xFFFFFFFFu) v = heap_chunk(t, image, c);
                reinterpret_cast<u32x4 *>(recs + p * (uint64_t)t.stride)[c] = v;
            }
        }
    }
}

hipError_t launch_for_update(const DevTable &t, const uint8_t *fu, const uint32_t *rids, uint64_t n,
                             stage_probe_out_dev *out, uint8_t *recs, hipStream_t s) {
    if (n == 0) return hipSuccess;
    for_update_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(t, fu, rids, n, out, recs);
    return hipGetLastError();
}

hipError_t launch_ident(const DevTable &t, const stage_probe_out_dev *out, uint64_t n, uint32_t *ident, hipStream_t s) {
    if (n == 0) return hipSuccess;
    ident_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(t, out, n, ident);
    return hipGetLastError();
}

hipError_t launch_resident_reader(const DevTable &t, const ReaderRing &g, hipStream_t s) {
    if (t.key_words != 1 || g.waves == 0 || g.slots % (64 * g.waves)) return hipErrorInvalidValue;
    const dim3 grid(g.waves), block(64);
    if (t.key_width == 0) {
        if (t.cap == 64) resident_reader_kernel<true, 1><<<grid, block, 0, s>>>(t, g);
        else if (t.cap == 128) resident_reader_kernel<true, 2><<<grid, block, 0, s>>>(t, g);
        else return hipErrorInvalidValue;
    } else {
        switch (t.cap / 64) {
            case 1: resident_reader_kernel<false, 1><<<grid, block, 0, s>>>(t, g); break;
            case 2: resident_reader_kernel<false, 2><<<grid, block, 0, s>>>(t, g); break;
            case 4: resident_reader_kernel<false, 4><<<grid, block, 0, s>>>(t, g); break;
            case 8: resident_reader_kernel<false, 8><<<grid, block, 0, s>>>(t, g); break;
            case 16: resident_reader_kernel<false, 16><<<grid, block, 0, s>>>(t, g); break;
            default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}

template <int KW, bool VIS, int R = 4>
static void launch_scan_w(const DevTable &t, const uint64_t *keys, uint64_t n, uint32_t scan_size, uint32_t *counts,
                          uint8_t *recs, const uint32_t *rids, uint8_t *st, hipStream_t s, int blocks) {
    if (scan_size <= 63) {  // at most 64 kept records per leaf visit: group-skipping LDS form
#define STAGE_SCAN_C(S)                                                                                        \
    scan_kernel_compact<false, S, KW, VIS><<<blocks, 256, 0, s>>>(t, keys, nullptr, n, scan_size, counts, recs, \
                                                                  rids, st)
        switch (t.cap / 64) {
            case 1: STAGE_SCAN_C(1); break;
            case 2: STAGE_SCAN_C(2); break;
            case 4: STAGE_SCAN_C(4); break;
            case 8: STAGE_SCAN_C(8); break;
            default: STAGE_SCAN_C(16);
        }
#undef STAGE_SCAN_C
        return;
    }
#define STAGE_SCAN_W(S) \
    scan_kernel<false, S, R, KW, VIS><<<blocks, 256, 0, s>>>(t, keys, nullptr, n, scan_size, counts, recs, rids, st)
    switch (t.cap / 64) {
        case 1: STAGE_SCAN_W(1); break;
        case 2: STAGE_SCAN_W(2); break;
        case 4: STAGE_SCAN_W(4); break;
        case 8: STAGE_SCAN_W(8); break;
        default: STAGE_SCAN_W(16);
    }
#undef STAGE_SCAN_W
}

template <int R, bool VIS>
static void launch_scan_r(const DevTable &t, const uint64_t *keys, const uint16_t *lens, uint64_t n,
                          uint32_t scan_size, uint32_t *counts, uint8_t *recs, const uint32_t *rids, uint8_t *st,
                          hipStream_t s, int blocks) {
    const bool var = t.key_width == 0;
    if (t.key_words == 2) return launch_scan_w<2, VIS>(t, keys, n, scan_size, counts, recs, rids, st, s, blocks);
    if (t.key_words == 4) return launch_scan_w<4, VIS>(t, keys, n, scan_size, counts, recs, rids, st, s, blocks);
    if (!var && t.cap > 128) return launch_scan_w<1, VIS, R>(t, keys, n, scan_size, counts, recs, rids, st, s, blocks);
#define STAGE_SCAN(V, S) \
    scan_kernel<V, S, R, 1, VIS><<<blocks, 256, 0, s>>>(t, keys, lens, n, scan_size, counts, recs, rids, st)
    if (t.cap == 64) {
        if (var) STAGE_SCAN(true, 1);
        else STAGE_SCAN(false, 1);
    } else {
        if (var) STAGE_SCAN(true, 2);
        else STAGE_SCAN(false, 2);
    }
#undef STAGE_SCAN
}

hipError_t launch_scan(const DevTable &t, const uint64_t *keys, const uint16_t *lens, uint64_t n, uint32_t scan_size,
                       uint32_t *counts, uint8_t *recs, hipStream_t s, const ScanTuning &tune, const uint32_t *rids,
                       uint8_t *row_status) {
    if (n == 0) return hipSuccess;
    const int blocks = grid_for(n, 4, tune.max_blocks > 0 ? tune.max_blocks : 16384);
    if (row_status) {  // IndexScanExecutor range branch: per-record visibility
        launch_scan_r<4, true>(t, keys, lens, n, scan_size, counts, recs, rids, row_status, s, blocks);
    } else {  // 4 rows in flight per wave (2 and 8 measured no faster)
        launch_scan_r<4, false>(t, keys, lens, n, scan_size, counts, recs, nullptr, nullptr, s, blocks);
    }
    return hipGetLastError();
}

hipError_t launch_scan_pair(const DevTable &t0, const uint64_t *k0, uint32_t sz0, uint32_t *c0, uint8_t *r0,
                            const DevTable &t1, const uint64_t *k1, uint32_t sz1, uint32_t *c1, uint8_t *r1,
                            hipStream_t s) {
    if (!scan_pair_supported(t0, sz0, t1, sz1)) return hipErrorInvalidValue;
#define STAGE_SCAN_P(S) scan_pair_compact_kernel<S><<<2, 64, 0, s>>>(t0, t1, k0, k1, sz0, sz1, c0, c1, r0, r1)
    switch (t0.cap / 64) {
        case 1: STAGE_SCAN_P(1); break;
        case 2: STAGE_SCAN_P(2); break;
        case 4: STAGE_SCAN_P(4); break;
        case 8: STAGE_SCAN_P(8); break;
        default: STAGE_SCAN_P(16);
    }
#undef STAGE_SCAN_P
    return hipGetLastError();
}

bool scan_pair_supported(const DevTable &t0, uint32_t sz0, const DevTable &t1, uint32_t sz1) {
    auto one = [](const DevTable &t, uint32_t sz) {
        return t.key_width == 8 && t.key_words == 1 && t.cap > 128 && sz >= 1 && sz <= 63;
    };
    return one(t0, sz0) && one(t1, sz1) && t0.cap == t1.cap;
}

hipError_t launch_scan_first(const DevTable &t, const uint64_t *keys, uint64_t n, uint32_t scan_size,
                             const uint32_t *rids, uint32_t words, uint32_t *img_out, uint8_t *st_out, hipStream_t s,
                             const ScanTuning &tune) {
    if (n == 0) return hipSuccess;
    if (t.key_width == 0 || scan_size == 0 || scan_size > 63) return hipErrorInvalidValue;
    const int blocks = grid_for((n + kFirstChunk - 1) / kFirstChunk, 4, tune.max_blocks > 0 ? tune.max_blocks : 16384);
    // scan_first_split_kernel decides the scans whose start leaf's first visit does, then
    // scan_first_rest_kernel runs the general loop for the rest.  Retired variants (measured
    // no faster): a single-scan kernel, NS scans in lockstep, the prefetching
    // "fast" kernel, the lane-parallel "mono" kernel, segmented stage A, a point-probe first
    // pass, the split kernel at 6 / 7 waves per SIMD.
#define STAGE_FIRST(S, KW)                                                                                  \
    scan_first_split_kernel<S, KW, 8><<<blocks, 256, 0, s>>>(t, keys, n, scan_size, rids, words, img_out,    \
                                                             st_out);                                       \
    scan_first_rest_kernel<S, KW><<<grid_for((n + 63) / 64, 4, 4096), 256, 0, s>>>(t, keys, n, scan_size, rids, \
                                                                                words, img_out, st_out)
#define STAGE_FIRST_K(KW)                      \
    switch (t.cap / 64) {                      \
        case 1: STAGE_FIRST(1, KW); break;     \
        case 2: STAGE_FIRST(2, KW); break;     \
        case 4: STAGE_FIRST(4, KW); break;     \
        case 8: STAGE_FIRST(8, KW); break;     \
        default: STAGE_FIRST(16, KW);          \
    }
    if (t.key_words == 4) {
        STAGE_FIRST_K(4)
    } else if (t.key_words == 2) {
        STAGE_FIRST_K(2)
    } else {
        STAGE_FIRST_K(1)
    }
#undef STAGE_FIRST_K
#undef STAGE_FIRST
    return hipGetLastError();
}

hipError_t launch_murmur(const void *keys, uint32_t key_len, uint32_t key_stride, uint64_t seed, uint64_t n,
                         uint64_t *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    murmur_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>((const uint8_t *)keys, key_len, key_stride, seed, n, out);
    return hipGetLastError();
}

hipError_t launch_fill(uint8_t *heap, uint32_t stride, uint32_t payload_size, uint32_t row_bytes,
                       const ImageDescDev *descs, const uint8_t *arena, uint64_t first, uint64_t count,
                       uint64_t ident_rowid0, uint32_t ident_key_width, int ident_mode, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const int blocks = grid_for(count, 4, 8192);
    fill_kernel<<<blocks, 256, 0, s>>>(heap, stride, payload_size, row_bytes, descs, arena, first, count, ident_rowid0,
                                       ident_key_width, ident_mode);
    return hipGetLastError();
}

hipError_t launch_patch(uint8_t *head, uint64_t *okey, SlotInfo *slot, uint32_t head_bytes, uint32_t cap, uint32_t kw,
                        const uint32_t *head_leaf, const void *head_src, uint64_t nhead, const uint64_t *slot_idx,
                        const SlotInfo *slot_src, const uint64_t *words, uint64_t nslot, hipStream_t s) {
    const uint64_t work = nhead * (head_bytes >> 4) + nslot;
    if (work == 0) return hipSuccess;
    uint64_t blocks = (work + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    patch_kernel<<<(unsigned)blocks, 256, 0, s>>>(head, okey, slot, head_bytes, cap, kw, head_leaf,
                                                  (const u32x4 *)head_src, nhead, slot_idx, slot_src, words, nslot);
    return hipGetLastError();
}

}  // namespace stage
