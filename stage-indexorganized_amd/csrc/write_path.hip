// write_path.hip -- the YCSB-B write path on the device.
//
// stage_update_batch_device applies an epoch of column updates, each optionally committed,
// with the host path's semantics (HostTable::update / commit_update = LeafNode::Update,
// b_tree.cpp:1061-1163, and the CommitTransaction UPDATE entry, transaction_manager.cpp:610-676),
// directly on the HBM image:
//   1. locate   probe_kernel without rows: each key's leaf and first visible slot
//               (SearchRecordMeta);
//   2. group    radix sort of (slot location, op index): a slot's ops stay in batch order;
//   3. decide   every op's return code.  An op's outcome depends only on the slot state left
//               by the previous successful op of its group (in-flight flag, cstamp, the
//               patched column); failures leave the state unchanged.  Each op is first
//               evaluated as if its predecessor succeeded, which is exact for the group's
//               leading run of successes; a group with a failure is finished by one wave that
//               evaluates the next 64 ops against the last success and jumps to the first that
//               succeeds;
//   4. number   exclusive scan of successes and commits: overwrite-copy, image and version
//               indices in (slot, batch) order;
//   5. write    per success (one wave) the overwrite-copy header, the retired-version header
//               when committed, and the new heap row: the record's row at epoch start with the
//               column window patched (all ops of a call patch the same window, so the k-th
//               successive image is the epoch-start row with the k-th delta);
//   6. publish  the last success of each group rewrites the slot word (meta, next, image).
// The host then adopts the bookkeeping (HostTable::adopt_device_epoch): the new copy / version
// headers and the touched slot words come back over PCIe; payload bytes stay in HBM until a
// host-side path needs them (stage_capi::ensure_host_rows).
#include <hip/hip_runtime.h>

#include <atomic>
#include <string>

#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "handle.hpp"

using namespace stage_capi;

namespace stage {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct WpArgs {
    const uint64_t *loc;     // sorted slot locations (device leaf * cap + slot); `none` = key absent
    const uint32_t *op;      // sorted op indices
    const uint32_t *gs;      // sorted position -> its group's first position
    const uint8_t *deltas;
    const uint32_t *writer;
    const uint32_t *cid;     // nullptr: no op commits
    const uint32_t *sst;     // nullptr: sstamp = commit id
    uint64_t n, none;
    uint32_t delta_len, win_off;  // window = row bytes [win_off, win_off + delta_len)
    uint32_t bad_range;
};

__device__ __forceinline__ uint32_t commit_of(const WpArgs &a, uint32_t o) { return a.cid ? a.cid[o] : 0u; }

// reference ReturnCode of op at sorted position q given the slot state after sorted position
// `last` (-1: the state at epoch start)
__device__ uint8_t wp_eval(const WpArgs &a, const DevTable &t, uint64_t q, int64_t last, const SlotInfo &base) {
    const uint32_t o = a.op[q];
    bool inserting;
    uint32_t cst;
    const uint8_t *win;
    if (last < 0) {
        inserting = meta_inserting(base.meta);
        cst = meta_cstamp(base.meta);
        win = t.heap + (uint64_t)base.image * t.hstride + a.win_off;
    } else {
        const uint32_t lo = a.op[last];
        cst = commit_of(a, lo);
        inserting = cst == 0;  // an uncommitted update leaves the record in flight
        win = a.deltas + (uint64_t)lo * a.delta_len;
    }
    if (inserting) return STAGE_RC_DIRTY;
    if (a.bad_range) return STAGE_RC_INVALID;
    const uint8_t *d = a.deltas + (uint64_t)o * a.delta_len;
    // no early exit: the loads of a whole window are independent and issue back to back
    uint32_t diff = 0;
    if ((((uintptr_t)d | (uintptr_t)win | a.delta_len) & 3u) == 0) {
        const uint32_t *dw = reinterpret_cast<const uint32_t *>(d), *ww = reinterpret_cast<const uint32_t *>(win);
#pragma unroll 8
        for (uint32_t b = 0; b < a.delta_len / 4; ++b) diff |= dw[b] ^ ww[b];
    } else {
#pragma unroll 8
        for (uint32_t b = 0; b < a.delta_len; ++b) diff |= (uint32_t)(d[b] ^ win[b]);
    }
    if (diff == 0 || cst > a.writer[o]) return STAGE_RC_NOT_NEEDED_UPDATE;
    return STAGE_RC_OK;
}

__global__ void wp_keys(const stage_probe_out_dev *__restrict__ pout, uint64_t n, uint32_t cap, uint64_t none,
                        uint64_t *__restrict__ loc, uint32_t *__restrict__ op) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = pout[i].w[2] & 0xFFFF;
    loc[i] = slot == 0xFFFF ? none : (uint64_t)pout[i].w[1] * cap + slot;
    op[i] = (uint32_t)i;
}

__global__ void wp_heads(const uint64_t *__restrict__ loc, uint64_t n, uint32_t *__restrict__ head) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    head[q] = (q == 0 || loc[q] != loc[q - 1]) ? (uint32_t)q : 0u;
}

// step 3a: every op evaluated against its predecessor-as-success
__global__ void wp_speculate(WpArgs a, DevTable t, uint8_t *__restrict__ rcs, uint8_t *__restrict__ succ,
                             int32_t *__restrict__ prev, uint32_t *__restrict__ first_fail) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    if (a.loc[q] == a.none) {
        rcs[q] = STAGE_RC_NOT_FOUND;
        succ[q] = 0;
        prev[q] = -1;
        return;
    }
    const uint32_t g = a.gs[q];
    const int64_t last = q > g ? (int64_t)q - 1 : -1;
    const SlotInfo base = t.slot[a.loc[q]];
    const uint8_t r = wp_eval(a, t, q, last, base);
    rcs[q] = r;
    succ[q] = r == STAGE_RC_OK;
    prev[q] = (int32_t)last;
    if (r != STAGE_RC_OK) atomicMin(&first_fail[g], (uint32_t)q);
}

// step 3b: groups with a failure, one wave each, from the first failure on.  A pass
// evaluates the next kFinishChunks x 64 ops of the group against the last success (their
// loads independent), takes the first success in batch order and restarts behind it: a hot
// key's long run of NotNeededUpdate / DIRTY ops goes 512 ops per pass.
constexpr int kFinishChunks = 8;
constexpr uint32_t kBigGroup = 2048;  // ops from the first failure on: a workgroup finishes it (wp_finish_big)
__global__ __launch_bounds__(256) void wp_finish_groups(WpArgs a, DevTable t, uint8_t *__restrict__ rcs,
                                                        uint8_t *__restrict__ succ, int32_t *__restrict__ prev,
                                                        const uint32_t *__restrict__ first_fail,
                                                        const uint32_t *__restrict__ gend) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t base_q = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64;
    const uint64_t mine = base_q + lane;
    const bool start = mine < a.n && a.loc[mine] != a.none && a.gs[mine] == mine && first_fail[mine] != 0xFFFFFFFFu &&
                       gend[mine] - first_fail[mine] < kBigGroup;
    uint64_t groups = __builtin_amdgcn_ballot_w64(start);
    while (groups) {
        const uint64_t g = base_q + __builtin_ctzll(groups);
        groups &= groups - 1;
        const uint64_t l = a.loc[g];
        const SlotInfo base = t.slot[l];
        const uint64_t f = first_fail[g];
        int64_t last = f > g ? (int64_t)f - 1 : -1;  // [g, f) all succeeded
        uint64_t pos = f;
        while (pos < a.n) {
            bool in[kFinishChunks];
            uint8_t r[kFinishChunks];
#pragma unroll
            for (int k = 0; k < kFinishChunks; ++k) {
                const uint64_t q = pos + 64 * k + lane;
                in[k] = q < a.n && a.loc[q] == l;
                r[k] = in[k] ? wp_eval(a, t, q, last, base) : (uint8_t)0xFF;
            }
            int kf = -1;
            uint32_t first = 0;
            bool whole = true;  // every chunk lies inside the group
#pragma unroll
            for (int k = 0; k < kFinishChunks; ++k) {
                const uint64_t okm = __builtin_amdgcn_ballot_w64(in[k] && r[k] == STAGE_RC_OK);
                if (kf < 0 && okm) {
                    kf = k;
                    first = (uint32_t)__builtin_ctzll(okm);
                }
                whole = whole && __builtin_amdgcn_ballot_w64(in[k]) == ~0ull;
            }
#pragma unroll
            for (int k = 0; k < kFinishChunks; ++k) {
                const uint64_t q = pos + 64 * k + lane;
                const bool upto = kf < 0 || k < kf || (k == kf && lane <= first);
                if (in[k] && upto) {
                    rcs[q] = r[k];
                    succ[q] = k == kf && lane == first;
                    prev[q] = (int32_t)last;
                }
            }
            if (kf >= 0) {
                last = (int64_t)(pos + 64 * (uint64_t)kf + first);
                pos = (uint64_t)last + 1;
                continue;
            }
            if (!whole) break;  // the group ends inside this pass
            pos += 64 * kFinishChunks;
        }
    }
}

// group extents: gend[g] = one past the last sorted position of the group starting at g
__global__ void wp_group_ends(WpArgs a, uint32_t *__restrict__ gend) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    if (q + 1 == a.n || a.loc[q + 1] != a.loc[q]) gend[a.gs[q]] = (uint32_t)(q + 1);
}

// failing groups with at least kBigGroup ops from their first failure on (a hot key's run of
// NotNeededUpdate / DIRTY ops) -> list
__global__ void wp_big_groups(WpArgs a, const uint32_t *__restrict__ first_fail, const uint32_t *__restrict__ gend,
                              uint32_t *__restrict__ list, uint32_t *__restrict__ count) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n || a.loc[q] == a.none || a.gs[q] != q || first_fail[q] == 0xFFFFFFFFu) return;
    if (gend[q] - first_fail[q] >= kBigGroup) list[atomicAdd(count, 1u)] = (uint32_t)q;
}

// step 3b for big groups: one 1024-thread workgroup per group, 16 waves x kFinishChunks x 64 =
// 8192 ops evaluated against the last success per pass, the first success in batch order
// found across the waves through LDS
__global__ __launch_bounds__(1024) void wp_finish_big(WpArgs a, DevTable t, uint8_t *__restrict__ rcs,
                                                      uint8_t *__restrict__ succ, int32_t *__restrict__ prev,
                                                      const uint32_t *__restrict__ first_fail,
                                                      const uint32_t *__restrict__ gend,
                                                      const uint32_t *__restrict__ list,
                                                      const uint32_t *__restrict__ count) {
    __shared__ uint64_t s_first[16];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr uint64_t kPass = 16ull * kFinishChunks * 64;
    const uint32_t nbig = *count;
    for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) {
        const uint64_t g = list[i];
        const uint64_t l = a.loc[g], end = gend[g];
        const SlotInfo base = t.slot[l];
        const uint64_t f = first_fail[g];
        int64_t last = f > g ? (int64_t)f - 1 : -1;  // [g, f) all succeeded
        uint64_t pos = f;
        while (pos < end) {
            uint8_t r[kFinishChunks];
            uint64_t mine_first = ~0ull;
#pragma unroll
            for (int k = 0; k < kFinishChunks; ++k) {
                const uint64_t q = pos + (uint64_t)wv * (kFinishChunks * 64) + 64 * k + lane;
                r[k] = q < end ? wp_eval(a, t, q, last, base) : (uint8_t)0xFF;
                if (r[k] == STAGE_RC_OK && q < mine_first) mine_first = q;
            }
            // the wave's first success, then the block's
            uint64_t wf = mine_first;
            for (int o = 32; o > 0; o >>= 1) {
                const uint64_t x = __shfl_xor(wf, o, 64);
                wf = x < wf ? x : wf;
            }
            __syncthreads();  // the previous pass's readers of s_first are done
            if (lane == 0) s_first[wv] = wf;
            __syncthreads();
            uint64_t bf = ~0ull;
#pragma unroll
            for (int w = 0; w < 16; ++w) bf = s_first[w] < bf ? s_first[w] : bf;
#pragma unroll
            for (int k = 0; k < kFinishChunks; ++k) {
                const uint64_t q = pos + (uint64_t)wv * (kFinishChunks * 64) + 64 * k + lane;
                if (q < end && q <= bf) {
                    rcs[q] = r[k];
                    succ[q] = q == bf;
                    prev[q] = (int32_t)last;
                }
            }
            if (bf != ~0ull) {
                last = (int64_t)bf;
                pos = bf + 1;
            } else {
                pos += kPass;
            }
        }
    }
}

// step 4 input: successes in the low word, committed successes in the high word
__global__ void wp_flags(WpArgs a, const uint8_t *__restrict__ succ, uint64_t *__restrict__ flags) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    const uint64_t s = succ[q] ? 1ull : 0ull;
    flags[q] = s | ((s && commit_of(a, a.op[q]) != 0) ? (1ull << 32) : 0ull);
}

__global__ void wp_totals(const uint64_t *__restrict__ ranks, const uint64_t *__restrict__ flags, uint64_t n,
                          uint64_t *__restrict__ tot) {
    const uint64_t v = ranks[n - 1] + flags[n - 1];
    tot[0] = v & 0xFFFFFFFFull;
    tot[1] = v >> 32;
}

// step 5: one wave per sorted position; successes write their headers and their new row
__global__ __launch_bounds__(256) void wp_write(WpArgs a, DevTable t, uint8_t *__restrict__ heap,
                                                CopyHdr *__restrict__ chdr, VersionHdr *__restrict__ vhdr,
                                                const uint8_t *__restrict__ succ, const int32_t *__restrict__ prev,
                                                const uint64_t *__restrict__ ranks, uint32_t *__restrict__ last_succ,
                                                uint64_t cbase, uint64_t vbase, uint64_t ibase) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t q = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); q < a.n; q += nwaves) {
        if (!succ[q]) continue;
        const uint32_t o = a.op[q];
        const SlotInfo base = t.slot[a.loc[q]];
        const uint64_t rk = ranks[q];
        const uint64_t irank = rk & 0xFFFFFFFFull, vrank = rk >> 32;
        const uint32_t cid = commit_of(a, o);
        const uint64_t img = ibase + irank;
        if (lane == 0) {
            const int32_t p = prev[q];
            CopyHdr c;
            if (p < 0) {  // first success of the group: the epoch-start record
                c.rstamp = meta_cstamp(base.meta);
                c.next = base.next;
                c.image = base.image;
            } else {      // the previous success, committed (an in-flight one makes this op DIRTY)
                const uint64_t pr = ranks[p];
                c.rstamp = commit_of(a, a.op[p]);
                c.next = kNextVersion | (uint32_t)(vbase + (pr >> 32));
                c.image = (uint32_t)(ibase + (pr & 0xFFFFFFFFull));
            }
            c.sstamp = cid ? (a.sst ? a.sst[o] : cid) : kMaxCid;
            chdr[cbase + irank] = c;
            if (cid) vhdr[vbase + vrank] = VersionHdr{c.rstamp, c.sstamp, c.next, c.image};
            atomicMax(&last_succ[a.gs[q]], (uint32_t)q + 1u);
        }
        // new row: epoch-start row with the window patched (CopyPayload)
        const uint8_t *src = t.heap + (uint64_t)base.image * t.hstride;
        uint8_t *dst = heap + img * t.hstride;
        const uint8_t *d = a.deltas + (uint64_t)o * a.delta_len;
        const uint32_t w0 = a.win_off, w1 = a.win_off + a.delta_len;
        for (uint32_t c = lane; c < t.hstride / 16; c += 64) {
            u32x4 v = reinterpret_cast<const u32x4 *>(src)[c];
            const uint32_t b0 = c * 16;
            if (b0 + 16 > w0 && b0 < w1) {
                union {
                    u32x4 v;
                    uint8_t b[16];
                } u;
                u.v = v;
                for (uint32_t j = 0; j < 16; ++j)
                    if (b0 + j >= w0 && b0 + j < w1) u.b[j] = d[b0 + j - w0];
                v = u.v;
            }
            reinterpret_cast<u32x4 *>(dst)[c] = v;
        }
    }
}

struct FinRec {
    uint64_t loc, meta;
    uint32_t next, image;
};

// step 6: the last success of each group publishes the slot word; every op gets its code
__global__ void wp_publish(WpArgs a, SlotInfo *__restrict__ slot, const uint8_t *__restrict__ rcs,
                           const uint8_t *__restrict__ succ, const int32_t *__restrict__ prev,
                           const uint64_t *__restrict__ ranks, const uint32_t *__restrict__ last_succ,
                           uint64_t cbase, uint64_t vbase, uint64_t ibase, FinRec *__restrict__ fin,
                           uint8_t *__restrict__ rc_out) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    const uint32_t o = a.op[q];
    rc_out[o] = rcs[q];
    if (!succ[q] || last_succ[a.gs[q]] != q + 1) return;
    const uint64_t l = a.loc[q];
    const uint64_t m0 = slot[l].meta;
    const uint32_t cid = commit_of(a, o);
    const uint64_t rk = ranks[q];
    auto committed_meta = [&](uint32_t c) { return ((m0 | kMetaVisible) & ~kMetaTxn & ~kMetaControl) | c; };
    uint64_t meta;
    uint32_t next;
    if (cid) {  // PrepareForUpdate then FinalizeForUpdate(t_cstamp)
        meta = committed_meta(cid);
        next = kNextVersion | (uint32_t)(vbase + (rk >> 32));
    } else {    // still in flight
        const int32_t p = prev[q];
        const uint64_t mb = p < 0 ? m0 : committed_meta(commit_of(a, a.op[p]));
        meta = mb | kMetaControl | kMetaVisible;
        next = kNextCopy | (uint32_t)(cbase + (rk & 0xFFFFFFFFull));
    }
    const uint32_t image = (uint32_t)(ibase + (rk & 0xFFFFFFFFull));
    slot[l].meta = meta;
    slot[l].next = next;
    slot[l].image = image;
    fin[rk & 0xFFFFFFFFull] = FinRec{l, meta, next, image};  // at the success rank: the first ns entries
}

unsigned blocks_for(uint64_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

}  // namespace
}  // namespace stage

namespace stage_capi {
void ensure_host_rows(stage_table *t) {
    if (!host(t).has_device_rows()) return;
    using namespace stage;
    hip_check(hipSetDevice(t->dev.device), "hipSetDevice");
    const uint64_t stride = host(t).hstride();
    host(t).materialize_device_rows([&](uint64_t first, uint64_t count, uint8_t *dst) {
        hip_check(hipMemcpy(dst, (const uint8_t *)t->dev.heap.p + first * stride, count * stride,
                            hipMemcpyDeviceToHost),
                  "device row fetch");
    });
}
}  // namespace stage_capi

extern "C" int stage_update_batch_device(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens, uint64_t n,
                                         uint32_t payload_off, const uint8_t *d_deltas, uint32_t delta_len,
                                         const uint32_t *d_writer_ids, const uint32_t *d_commit_ids,
                                         const uint32_t *d_sstamps, uint8_t *d_rc, uint64_t *n_ok, void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (n && (!d_keys || !d_writer_ids || !d_rc || (!d_deltas && delta_len)))
        return fail(STAGE_E_ARG, "null device buffer");
    if (n >= (1ull << 31)) return fail(STAGE_E_ARG, "batch too large");
    if (n_ok) *n_ok = 0;
    if (n == 0) return STAGE_OK;
    return guarded([&] {
        using namespace stage;
        HostTable &h = host(t);
        DeviceImage &dv = t->dev;
        hip_check(hipSetDevice(dv.device), "hipSetDevice");
        hipStream_t s = pick(t, stream);
        // STAGE_WP_TRACE=1: per-phase host wall times on stderr
        static const bool trace = std::getenv("STAGE_WP_TRACE") != nullptr;
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        auto ms = [&](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
        // room for one copy, image and version per op
        reserve_device_rows(h, dv, n, n, n, s);
        const double t_reserve = ms(t0);
        const DevTable &view = dv.view;
        const uint64_t cbase = h.copies_.size(), vbase = h.versions_.size(), ibase = h.images_.size();
        const uint64_t none = (uint64_t)view.nleaves * view.cap;
        int end_bit = 1;
        while (end_bit < 64 && (none >> end_bit)) ++end_bit;

        // scratch
        size_t cub_sort = 0, cub_scan = 0, cub_sum = 0;
        hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, cub_sort, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                                     (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, 0, end_bit, s),
                  "sort size");
        hip_check(hipcub::DeviceScan::InclusiveScan(nullptr, cub_scan, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                    hipcub::Max(), (int)n, s),
                  "scan size");
        hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, cub_sum, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)n,
                                                   s),
                  "sum size");
        const size_t cub_bytes = std::max(cub_sort, std::max(cub_scan, cub_sum));
        auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
        uint64_t off = 0;
        auto take = [&](uint64_t bytes) {
            const uint64_t o = off;
            off += al(bytes);
            return o;
        };
        const uint64_t o_pout = take(n * 32), o_loc0 = take(n * 8), o_loc = take(n * 8), o_op0 = take(n * 4),
                       o_op = take(n * 4), o_head = take(n * 4), o_gs = take(n * 4), o_rcs = take(n), o_succ = take(n),
                       o_prev = take(n * 4), o_ff = take(n * 4), o_ls = take(n * 4), o_gend = take(n * 4), o_big = take(n * 4), o_flags = take(n * 8),
                       o_ranks = take(n * 8), o_cub = take(cub_bytes);
        uint8_t *buf = scratch_bytes(dv, off);
        auto *pout = (stage_probe_out_dev *)(buf + o_pout);
        auto *loc0 = (uint64_t *)(buf + o_loc0);
        auto *loc = (uint64_t *)(buf + o_loc);
        auto *op0 = (uint32_t *)(buf + o_op0);
        auto *op = (uint32_t *)(buf + o_op);
        auto *head = (uint32_t *)(buf + o_head);
        auto *gs = (uint32_t *)(buf + o_gs);
        auto *rcs = buf + o_rcs;
        auto *succ = buf + o_succ;
        auto *prev = (int32_t *)(buf + o_prev);
        auto *ff = (uint32_t *)(buf + o_ff);
        auto *ls = (uint32_t *)(buf + o_ls);
        auto *gend = (uint32_t *)(buf + o_gend);
        auto *big = (uint32_t *)(buf + o_big);
        auto *flags = (uint64_t *)(buf + o_flags);
        auto *ranks = (uint64_t *)(buf + o_ranks);
        // slot words + totals: read back after this call returns (background adoption)
        uint8_t *wo = wp_out_bytes(dv, al(n * sizeof(FinRec)) + 256);
        auto *fin = (FinRec *)wo;
        auto *tot = (uint64_t *)(wo + al(n * sizeof(FinRec)));
        void *cub = buf + o_cub;
        size_t cb = cub_bytes;

        // 1. locate
        hip_check(launch_probe(view, d_keys, d_lens, nullptr, nullptr, n, pout, nullptr, s, t->tune), "locate");
        wp_keys<<<blocks_for(n, 256), 256, 0, s>>>(pout, n, view.cap, none, loc0, op0);
        // 2. group
        hip_check(hipcub::DeviceRadixSort::SortPairs(cub, cb, loc0, loc, op0, op, (int)n, 0, end_bit, s), "sort");
        wp_heads<<<blocks_for(n, 256), 256, 0, s>>>(loc, n, head);
        cb = cub_bytes;
        hip_check(hipcub::DeviceScan::InclusiveScan(cub, cb, head, gs, hipcub::Max(), (int)n, s), "group starts");
        // 3. decide
        WpArgs a{loc, op, gs, d_deltas, d_writer_ids, d_commit_ids, d_sstamps, n, none, delta_len,
                 h.key_pad() + payload_off, (uint64_t)payload_off + delta_len > h.params().payload_size ? 1u : 0u};
        hip_check(hipMemsetAsync(ff, 0xFF, n * 4, s), "memset");
        hip_check(hipMemsetAsync(ls, 0, n * 4, s), "memset");
        hip_check(hipMemsetAsync(fin, 0xFF, n * sizeof(FinRec), s), "memset");
        wp_speculate<<<blocks_for(n, 256), 256, 0, s>>>(a, view, rcs, succ, prev, ff);
        wp_group_ends<<<blocks_for(n, 256), 256, 0, s>>>(a, gend);
        hip_check(hipMemsetAsync(tot + 1, 0, 4, s), "memset");  // big-group count (tot is rewritten in step 4)
        wp_big_groups<<<blocks_for(n, 256), 256, 0, s>>>(a, ff, gend, big, (uint32_t *)(tot + 1));
        wp_finish_groups<<<blocks_for(n, 256), 256, 0, s>>>(a, view, rcs, succ, prev, ff, gend);
        wp_finish_big<<<256, 1024, 0, s>>>(a, view, rcs, succ, prev, ff, gend, big, (uint32_t *)(tot + 1));
        // 4. number
        wp_flags<<<blocks_for(n, 256), 256, 0, s>>>(a, succ, flags);
        cb = cub_bytes;
        hip_check(hipcub::DeviceScan::ExclusiveSum(cub, cb, flags, ranks, (int)n, s), "ranks");
        wp_totals<<<1, 1, 0, s>>>(ranks, flags, n, tot);
        // 5. write, 6. publish
        const int wblocks = (int)std::min<uint64_t>(blocks_for(n, 4), 16384);
        wp_write<<<wblocks, 256, 0, s>>>(a, view, (uint8_t *)dv.heap.p, (CopyHdr *)dv.chdr.p, (VersionHdr *)dv.vhdr.p,
                                         succ, prev, ranks, ls, cbase, vbase, ibase);
        wp_publish<<<blocks_for(n, 256), 256, 0, s>>>(a, (SlotInfo *)dv.slot.p, rcs, succ, prev, ranks, ls, cbase,
                                                      vbase, ibase, fin, d_rc);
        hip_check(hipGetLastError(), "write-path kernels");

        // the host adopts the epoch.  The headers and slot words come back on a stream of their
        // own into pinned staging (full PCIe rate) and the host adopts them on a background
        // thread (stage_table::adopt) while the caller's stream goes on (the next probe overlaps
        // the copies); the next call that needs the host table waits for it (host() / settle).
        const double t_enqueue = ms(t0);
        if (!dv.adopt_stream) hip_check(hipStreamCreateWithFlags(&dv.adopt_stream, hipStreamNonBlocking), "adopt stream");
        if (!dv.adopt_ev) hip_check(hipEventCreateWithFlags(&dv.adopt_ev, hipEventDisableTiming), "adopt event");
        hip_check(hipEventRecord(dv.adopt_ev, s), "adopt event");
        // staging: [totals 64 B][copy headers][version headers][slot words], sized for the worst
        // case (one copy and one version per op); every part starts on a 16-B boundary (the
        // headers are 16-B aligned types: a misaligned source faults in the vectorised copy)
        const uint64_t bf = n * sizeof(FinRec), bmax = 2 * n * sizeof(CopyHdr);
        static_assert(sizeof(CopyHdr) == sizeof(VersionHdr) && sizeof(CopyHdr) % 16 == 0, "header sizes");
        uint8_t *pin = pinned_bytes(dv, 64 + bmax + bf);
        auto *totals = reinterpret_cast<uint64_t *>(pin);
        auto *fr = reinterpret_cast<FinRec *>(pin + 64 + bmax);
        uint64_t ns = 0;
        if (n_ok) {  // the caller wants the count now: wait for the kernels
            hip_check(hipMemcpyAsync(totals, tot, 16, hipMemcpyDeviceToHost, s), "totals");
            hip_check(hipStreamSynchronize(s), "write path");
            ns = totals[0];
        }
        const double t_kernels = ms(t0);
        // FinRec and HostTable::SlotWords share a layout: device slot locations become host slot
        // indices in place (ops that published nothing keep ~0 and are skipped by the adoption)
        static_assert(sizeof(FinRec) == sizeof(HostTable::SlotWords) &&
                          offsetof(FinRec, meta) == offsetof(HostTable::SlotWords, meta) &&
                          offsetof(FinRec, next) == offsetof(HostTable::SlotWords, next) &&
                          offsetof(FinRec, image) == offsetof(HostTable::SlotWords, image),
                      "FinRec / SlotWords layout");
        t->start_adoption([t, &h, &dv, cap = view.cap, n, cbase, vbase, pin, totals, fr, tot, fin, t0, t_kernels,
                           t_enqueue, t_reserve]() mutable {
            try {
                hip_check(hipSetDevice(dv.device), "hipSetDevice");
                hipStream_t a = dv.adopt_stream;
                hip_check(hipStreamWaitEvent(a, dv.adopt_ev, 0), "adopt wait");
                hip_check(hipMemcpyAsync(totals, tot, 16, hipMemcpyDeviceToHost, a), "totals");
                hip_check(hipStreamSynchronize(a), "adopt totals");
                const uint64_t ns = totals[0], nv = totals[1];
                if (ns > n) throw std::runtime_error("write path: more successes than ops");
                // slot words sit at the success ranks (the last success of each key; the other
                // entries stay ~0): ns records instead of n
                if (ns) hip_check(hipMemcpyAsync(fr, fin, ns * sizeof(FinRec), hipMemcpyDeviceToHost, a), "slot words");
                auto *copies = reinterpret_cast<CopyHdr *>(pin + 64);
                auto *versions = reinterpret_cast<VersionHdr *>(pin + 64 + ns * sizeof(CopyHdr));
                if (ns)
                    hip_check(hipMemcpyAsync(copies, (CopyHdr *)dv.chdr.p + cbase, ns * sizeof(CopyHdr),
                                             hipMemcpyDeviceToHost, a),
                              "copy headers");
                if (nv)
                    hip_check(hipMemcpyAsync(versions, (VersionHdr *)dv.vhdr.p + vbase, nv * sizeof(VersionHdr),
                                             hipMemcpyDeviceToHost, a),
                              "version headers");
                hip_check(hipStreamSynchronize(a), "adopt headers");
                const double t_d2h = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
                const std::vector<uint32_t> &d2h = dv.dev_to_host;
                std::atomic<uint64_t> bad{0};
                HostTable::parallel_chunks(ns, [&](uint64_t b, uint64_t e) {
                    for (uint64_t k = b; k < e; ++k) {
                        if (fr[k].loc == ~0ull) continue;
                        if (fr[k].loc / cap >= d2h.size()) {
                            bad.fetch_add(1);
                            fr[k].loc = ~0ull;
                            continue;
                        }
                        fr[k].loc = (uint64_t)d2h[fr[k].loc / cap] * cap + fr[k].loc % cap;
                    }
                });
                if (bad.load())
                    throw std::runtime_error("write path: " + std::to_string(bad.load()) +
                                             " slot words outside the table (ns " + std::to_string(ns) + ")");
                h.adopt_device_epoch(copies, ns, versions, nv, ns, reinterpret_cast<const HostTable::SlotWords *>(fr), ns);
                if (trace)
                    std::fprintf(stderr,
                                 "[wp] n=%llu ok=%llu reserve %.2f enqueue %.2f kernels %.2f d2h %.2f adopted %.2f ms "
                                 "(background)\n",
                                 (unsigned long long)n, (unsigned long long)ns, t_reserve, t_enqueue, t_kernels, t_d2h,
                                 std::chrono::duration<double, std::milli>(clk::now() - t0).count());
            } catch (...) {
                t->adopt_err = std::current_exception();
            }
        });
        if (n_ok) *n_ok = ns;
        return STAGE_OK;
    });
}
