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
//               patched column); failures leave the state unchanged.  The column comparison
//               (new value == current value: NotNeededUpdate) is prepared once per op by
//               wp_classify: runs of equal deltas in sorted order share a class number, and
//               every delta (and each group's epoch-start window) has a 64-bit content
//               fingerprint -- same class: equal; different fingerprints: different; only a
//               fingerprint match across classes compares the bytes.  Each op is first
//               evaluated as if its predecessor succeeded, which is exact for the group's
//               leading run of successes; a group with a failure is finished by one wave that
//               evaluates the next 64 ops against the last success and jumps to the first that
//               succeeds;
//   4. number   exclusive scan of successes and commits: overwrite-copy, image and version
//               indices in (slot, batch) order;
//   5. write    per success the overwrite-copy header and the retired-version header when
//               committed (one thread per op, wp_headers), then the new heap row (a 16-lane
//               team per success, wp_write): the record's row at epoch start with the column
//               window patched (all ops of a call patch the same window, so the k-th
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
#include "radix_sort.hpp"

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

// per sorted position q (wp_classify): cls = number of breaks up to q, where a break is a group
// head or a delta unequal to its predecessor's (so cls[q] == cls[p], p < q in one group, means
// equal deltas); fp = the delta's content fingerprint; for group heads, eqw = the delta equals
// the epoch-start window, wfp = the window's fingerprint
struct WpCls {
    const uint32_t *cls;
    const uint64_t *fp, *wfp;
    const uint8_t *eqw;
};

__device__ __forceinline__ bool bytes_equal(const uint8_t *d, const uint8_t *w, uint32_t len) {
    uint32_t diff = 0;
    if ((((uintptr_t)d | (uintptr_t)w | len) & 3u) == 0) {
        const uint32_t *dw = reinterpret_cast<const uint32_t *>(d), *ww = reinterpret_cast<const uint32_t *>(w);
#pragma unroll 8
        for (uint32_t b = 0; b < len / 4; ++b) diff |= dw[b] ^ ww[b];
    } else {
#pragma unroll 8
        for (uint32_t b = 0; b < len; ++b) diff |= (uint32_t)(d[b] ^ w[b]);
    }
    return diff == 0;
}

// reference ReturnCode of op at sorted position q (group head g) given the slot state after
// sorted position `last` (-1: the state at epoch start, base)
__device__ uint8_t wp_eval(const WpArgs &a, const WpCls &k, const DevTable &t, uint64_t q, uint64_t g, int64_t last,
                           const SlotInfo &base) {
    const uint32_t o = a.op[q];
    bool inserting;
    uint32_t cst;
    if (last < 0) {
        inserting = meta_inserting(base.meta);
        cst = meta_cstamp(base.meta);
    } else {
        cst = commit_of(a, a.op[last]);
        inserting = cst == 0;  // an uncommitted update leaves the record in flight
    }
    if (inserting) return STAGE_RC_DIRTY;
    if (a.bad_range) return STAGE_RC_INVALID;
    const uint8_t *d = a.deltas + (uint64_t)o * a.delta_len;
    bool eq;
    if (last >= 0) {
        if (k.cls[q] == k.cls[last]) eq = true;
        else if (k.fp[q] != k.fp[last]) eq = false;
        else eq = bytes_equal(d, a.deltas + (uint64_t)a.op[last] * a.delta_len, a.delta_len);
    } else {
        if (k.cls[q] == k.cls[g]) eq = k.eqw[g] != 0;
        else if (k.fp[q] != k.wfp[g]) eq = false;
        else eq = bytes_equal(d, t.heap + (uint64_t)base.image * t.hstride + a.win_off, a.delta_len);
    }
    if (eq || cst > a.writer[o]) return STAGE_RC_NOT_NEEDED_UPDATE;
    return STAGE_RC_OK;
}

// bytes [4k, 4k + 4) of p (those below len; the rest read as 0)
__device__ __forceinline__ uint32_t ld_word(const uint8_t *p, uint32_t k, uint32_t len, bool aligned) {
    if (aligned && 4 * k + 4 <= len) return reinterpret_cast<const uint32_t *>(p)[k];
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; ++j)
        if (4 * k + j < len) v |= (uint32_t)p[4 * k + j] << (8 * j);
    return v;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h;
}
__device__ __forceinline__ uint64_t word_fp(uint32_t w, uint32_t k) {
    return fmix64(((uint64_t)k << 32 | w) ^ 0x9e3779b97f4a7c15ull);
}

// step 3 preparation, in op order before the sort (so it runs beside the read probe rather
// than after it): a team of kTeam lanes per op reads its delta and, for a found key, its slot's
// epoch-start window with word loads, 4 per lane in flight together -> the delta's fingerprint,
// the window's, and whether the two are equal.  The sort's input and the epoch's
// position-indexed state (first failures none, last-success marks 0, FinRecs all ones -- 24 B
// each -- and the big-group count 0) are written on the way, so no fills follow on the stream.
constexpr uint32_t kTeam = 8;
__global__ __launch_bounds__(256) void wp_keys(const stage_probe_out_dev *__restrict__ pout, uint64_t n, uint64_t none,
                                               DevTable t, const uint8_t *__restrict__ deltas, uint32_t delta_len,
                                               uint32_t win_off, uint32_t bad_range, uint64_t *__restrict__ loc,
                                               uint32_t *__restrict__ op,
                                               uint64_t *__restrict__ fp_op, uint64_t *__restrict__ wfp_op,
                                               uint8_t *__restrict__ eqw_op, uint32_t *__restrict__ first_fail,
                                               uint32_t *__restrict__ last_succ, uint64_t *__restrict__ fin_words,
                                               uint32_t *__restrict__ big_count) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, tl = lane & (kTeam - 1);
    const uint64_t i = gid / kTeam;
    if (gid == 0) *big_count = 0;
    const bool valid = i < n;
    uint64_t l = none;
    if (valid) {
        const uint32_t slot = pout[i].w[2] & 0xFFFF;
        l = slot == 0xFFFF ? none : (uint64_t)pout[i].w[1] * t.cap + slot;
    }
    const bool found = valid && l != none;
    const uint8_t *d = valid ? deltas + i * delta_len : nullptr;
    // (a window past the payload: every op is INVALID, wp_eval never compares with it)
    const uint8_t *w = found && !bad_range ? t.heap + (uint64_t)t.slot[l].image * t.hstride + win_off : nullptr;
    const bool al = found && ((((uintptr_t)d | (uintptr_t)w) & 3u) == 0);
    uint64_t h = 0, hw = 0;
    bool ne = false;
    const uint32_t words = found ? (delta_len + 3) / 4 : 0u;
    for (uint32_t k0 = 0; k0 < words; k0 += 4 * kTeam) {
        uint32_t x[4], y[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * kTeam + tl;
            x[u] = k < words ? ld_word(d, k, delta_len, al) : 0u;
            y[u] = k < words && w ? ld_word(w, k, delta_len, al) : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * kTeam + tl;
            if (k < words) {
                h ^= word_fp(x[u], k);
                hw ^= word_fp(y[u], k);
                ne |= x[u] != y[u];
            }
        }
    }
    const uint64_t nem = __builtin_amdgcn_ballot_w64(ne);
    const bool team_ne = ((nem >> (lane & ~(kTeam - 1))) & ((1ull << kTeam) - 1)) != 0;
#pragma unroll
    for (int o = kTeam / 2; o > 0; o >>= 1) {
        h ^= __shfl_xor(h, o, 64);
        hw ^= __shfl_xor(hw, o, 64);
    }
    if (tl == 0 && valid) {
        loc[i] = l;
        op[i] = (uint32_t)i;
        fp_op[i] = h;
        if (found) {
            wfp_op[i] = hw;
            eqw_op[i] = team_ne ? 0 : 1;
        }
        first_fail[i] = 0xFFFFFFFFu;
        last_succ[i] = 0;
        fin_words[3 * i] = ~0ull;
        fin_words[3 * i + 1] = ~0ull;
        fin_words[3 * i + 2] = ~0ull;
    }
}

// step 3 preparation after the sort, a thread per sorted position: the op's fingerprints
// gathered; a break where the group starts or the delta differs from its predecessor's (a
// fingerprint mismatch, or equal fingerprints and unequal bytes)
__global__ __launch_bounds__(256) void wp_classify(WpArgs a, const uint64_t *__restrict__ fp_op, const uint64_t *__restrict__ wfp_op,
                            const uint8_t *__restrict__ eqw_op, uint32_t *__restrict__ brk, uint64_t *__restrict__ fp,
                            uint64_t *__restrict__ wfp, uint8_t *__restrict__ eqw) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    const bool live = a.loc[q] != a.none;
    const bool head = live && a.gs[q] == q;
    const uint32_t o = a.op[q];
    const uint64_t h = live ? fp_op[o] : 0ull;
    uint32_t b = 1;
    if (live && !head) {
        const uint32_t po = a.op[q - 1];
        b = h != fp_op[po] ? 1u
                           : (bytes_equal(a.deltas + (uint64_t)o * a.delta_len, a.deltas + (uint64_t)po * a.delta_len,
                                          a.delta_len)
                                  ? 0u
                                  : 1u);
    }
    brk[q] = b;
    fp[q] = h;
    if (head) {
        wfp[q] = wfp_op[o];
        eqw[q] = eqw_op[o];
    }
}

// lanes [from, lane) of a wave
__device__ __forceinline__ uint64_t lanes_between(uint32_t from, uint32_t lane) {
    const uint64_t below = lane ? ~0ull >> (64 - lane) : 0ull;
    const uint64_t skip = from ? ~0ull >> (64 - from) : 0ull;
    return below & ~skip;
}

__global__ __launch_bounds__(256) void wp_heads(const uint64_t *__restrict__ loc, uint64_t n, uint32_t *__restrict__ head) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    head[q] = (q == 0 || loc[q] != loc[q - 1]) ? (uint32_t)q : 0u;
}

// step 3a: every op evaluated against its predecessor-as-success; on the way the group extents
// (gend[g] = one past the group's last position) and the first position of every delta class
// (cfirst; cls = inclusive sum of wp_classify's breaks, cfirst[last class + 1] = n, so the run
// after a group's last run starts at or past the group's end)
__global__ __launch_bounds__(256) void wp_speculate(WpArgs a, WpCls k, DevTable t, uint8_t *__restrict__ rcs, uint8_t *__restrict__ succ,
                             int32_t *__restrict__ prev, uint32_t *__restrict__ first_fail, uint32_t *__restrict__ gend,
                             const uint32_t *__restrict__ brk, uint32_t *__restrict__ cfirst) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // blockDim: a multiple of 64
    if (q >= a.n) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lq = a.loc[q];
    const bool found = lq != a.none;
    const uint32_t g = a.gs[q];
    const uint32_t cq = k.cls[q];
    if (q + 1 == a.n || a.loc[q + 1] != lq) gend[g] = (uint32_t)(q + 1);
    if (brk[q]) cfirst[cq] = (uint32_t)q;
    if (q + 1 == a.n) cfirst[cq + 1] = (uint32_t)a.n;
    const int64_t last = q > g ? (int64_t)q - 1 : -1;
    uint8_t r = STAGE_RC_NOT_FOUND;
    if (found) {
        SlotInfo base{};
        if (last < 0) base = t.slot[a.loc[q]];  // the epoch-start state matters to the head only
        r = wp_eval(a, k, t, q, g, last, base);
    }
    rcs[q] = r;
    succ[q] = r == STAGE_RC_OK;
    prev[q] = found ? (int32_t)last : -1;
    // a group's first failure: only the first failing lane of the group in this wave competes
    // (a hot key's run of failures would otherwise serialise on one address)
    const bool fail = found && r != STAGE_RC_OK;
    const uint64_t fm = __builtin_amdgcn_ballot_w64(fail);
    const uint64_t wbase = q - lane;
    const uint32_t glane = g > wbase ? (uint32_t)(g - wbase) : 0u;
    if (fail && !(fm & lanes_between(glane, lane))) atomicMin(&first_fail[g], (uint32_t)q);
}

// step 3b: groups with a failure, one wave each, from the first failure on.  A pass
// evaluates the next kFinishChunks x 64 ops of the group against the last success (their
// loads independent), takes the first success in batch order and restarts behind it: a hot
// key's long run of NotNeededUpdate / DIRTY ops goes 512 ops per pass.
constexpr int kFinishChunks = 8;
constexpr uint32_t kJumpFrom = 128;  // ops from the first failure on: pointer jumping (wp_jump_*; 128 from the r05 sweep)
// Groups with at least big_from ops from their first failure on go to `list` instead (one
// atomic per big group; their finishing kernels follow).
// (<= 80 VGPRs, amdgpu_waves_per_eu(6): a retired read-probe wave's registers fit one of its
// waves, so it runs beside C3's probe -- at 91 VGPRs it waited for the probe's last dispatch)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void wp_finish_groups(WpArgs a, WpCls kc, DevTable t, uint8_t *__restrict__ rcs,
                                                        uint8_t *__restrict__ succ, int32_t *__restrict__ prev,
                                                        const uint32_t *__restrict__ first_fail,
                                                        const uint32_t *__restrict__ gend, uint32_t big_from,
                                                        uint32_t *__restrict__ list, uint32_t *__restrict__ count,
                                                        uint8_t *__restrict__ junr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t base_q = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64;
    const uint64_t mine = base_q + lane;
    const bool failing = mine < a.n && a.loc[mine] != a.none && a.gs[mine] == mine && first_fail[mine] != 0xFFFFFFFFu;
    const bool start = failing && gend[mine] - first_fail[mine] < big_from;
    if (failing && !start) {
        list[atomicAdd(count, 1u)] = (uint32_t)mine;
        if (junr) junr[mine] = 0;  // wp_jump_links: no unresolved candidate yet
    }
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
                r[k] = in[k] ? wp_eval(a, kc, t, q, g, last, base) : (uint8_t)0xFF;
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
                // ops after a success hold their speculative outcome (evaluated against their
                // predecessor as a success: exact now) up to the next speculative failure,
                // which is exact too; re-evaluation resumes behind it
                const uint64_t bq = pos + 64 * (uint64_t)kf + first;
                uint64_t nf = ~0ull;
                for (uint64_t s0 = bq + 1; s0 < a.n && nf == ~0ull; s0 += 64 * kFinishChunks) {
                    bool more = true;
#pragma unroll
                    for (int k = 0; k < kFinishChunks; ++k) {
                        const uint64_t q = s0 + 64 * k + lane;
                        const bool ing = q < a.n && a.loc[q] == l;
                        const uint64_t fm = __builtin_amdgcn_ballot_w64(ing && !succ[q]);
                        if (nf == ~0ull && fm) nf = s0 + 64 * k + (uint64_t)__builtin_ctzll(fm);
                        more = more && __builtin_amdgcn_ballot_w64(ing) == ~0ull;
                    }
                    if (!more) break;  // the group ends inside this stretch
                }
                if (nf == ~0ull) break;  // no failure left: the rest of the group stands
                last = (int64_t)nf - 1;
                pos = nf + 1;
                continue;
            }
            if (!whole) break;  // the group ends inside this pass
            pos += 64 * kFinishChunks;
        }
    }
}

// The big-group kernels' workgroups (wp_jump_chain, finish_big_walk inside it): 256 threads, so
// that they are dispatched beside C3's read probe, whose 256-thread workgroups fill every CU --
// a larger workgroup needs several retired probe workgroups on one CU at once and waits for the
// probe's last dispatch (round 6; 1024 threads before).
constexpr uint32_t kJumpThreads = 256, kJumpWaves = kJumpThreads / 64;

// step 3b for big groups, the walk (round 4; now the fallback of the pointer jumping when a
// candidate's writer is older than the commit): one workgroup per group, kJumpWaves waves x
// kFinishChunks x 64 ops evaluated against the last success per pass, the first success in batch
// order found across the waves through LDS.  Serial in the group's failures: ~700 passes for a
// Zipf-0.99 hot key on RunMixed's stream.
__device__ void finish_big_walk(const WpArgs &a, const WpCls &kc, const DevTable &t, uint8_t *__restrict__ rcs,
                                uint8_t *__restrict__ succ, int32_t *__restrict__ prev, uint64_t g, uint64_t end,
                                uint64_t f, const SlotInfo &base, uint64_t *s_first) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr uint64_t kPass = (uint64_t)kJumpWaves * kFinishChunks * 64;
    int64_t last = f > g ? (int64_t)f - 1 : -1;  // [g, f) all succeeded
    uint64_t pos = f;
    while (pos < end) {
        // a pass: up to kFinishChunks slices of kJumpThreads ops (one 64-op chunk per wave), evaluated
        // against the last success slice by slice until one holds a success -- behind a
        // single failure the next op usually succeeds, so most passes take one slice
        uint64_t bf = ~0ull, done = pos;
        for (int k = 0; k < kFinishChunks && bf == ~0ull && done < end; ++k) {
            const uint64_t q = done + (uint64_t)wv * 64 + lane;
            const uint8_t r = q < end ? wp_eval(a, kc, t, q, g, last, base) : (uint8_t)0xFF;
            uint64_t wf = r == STAGE_RC_OK ? q : ~0ull;  // the wave's first success, then the block's
            for (int o = 32; o > 0; o >>= 1) {
                const uint64_t x = __shfl_xor(wf, o, 64);
                wf = x < wf ? x : wf;
            }
            __syncthreads();  // the previous slice's readers of s_first are done
            if (lane == 0) s_first[wv] = wf;
            __syncthreads();
#pragma unroll
            for (uint32_t w = 0; w < kJumpWaves; ++w) bf = s_first[w] < bf ? s_first[w] : bf;
            if (q < end && q <= bf) {
                rcs[q] = r;
                succ[q] = q == bf;
                prev[q] = (int32_t)last;
            }
            done += kJumpThreads;
        }
        if (bf != ~0ull) {
            // as wp_finish_groups: the speculative outcomes behind a success stand up to
            // and including the next speculative failure
            uint64_t nf = ~0ull;
            for (uint64_t s0 = bf + 1; s0 < end && nf == ~0ull; s0 += kPass) {
                uint64_t mf = ~0ull;
#pragma unroll
                for (int k = 0; k < kFinishChunks; ++k) {
                    const uint64_t q = s0 + (uint64_t)wv * (kFinishChunks * 64) + 64 * k + lane;
                    if (q < end && !succ[q] && q < mf) mf = q;
                }
                for (int o = 32; o > 0; o >>= 1) {
                    const uint64_t x = __shfl_xor(mf, o, 64);
                    mf = x < mf ? x : mf;
                }
                __syncthreads();
                if (lane == 0) s_first[wv] = mf;
                __syncthreads();
#pragma unroll
                for (uint32_t w = 0; w < kJumpWaves; ++w) nf = s_first[w] < nf ? s_first[w] : nf;
            }
            if (nf == ~0ull) break;
            last = (int64_t)nf - 1;
            pos = nf + 1;
        } else {
            pos = done;
        }
    }
}

// step 3b for big groups by pointer jumping (round 5).  An op's outcome depends only on the
// last success before it (wp_eval), so the group's successes are the chain s0, nxt(s0),
// nxt(nxt(s0)), ... where nxt(p) = the first later op of the group that succeeds if p is the
// last success: none after an uncommitted success (the record stays in flight: DIRTY), else
// the first op whose delta differs from p's -- the start of the next run of equal deltas
// (wp_classify's class numbers; cfirst[c] = the first position of class c) when p+1 repeats
// p's delta, else p+1 -- provided its writer is not older than p's commit id.  When that
// writer is older (NotNeededUpdate by cstamp) the candidate fails and the chain is not known
// locally: the group is finished by finish_big_walk instead (never on RunMixed's stream, whose
// writer ids grow with the batch).  Per group:
//   A. per 64-op chunk (a wave), nxt of every op, then exit(p) (the first chain node at or past
//      the chunk's end) and mask(p) (the chain's nodes inside the chunk) by 6 doubling steps
//      over the wave's lanes (shuffles, no memory);
//   B. one wave follows the chain chunk to chunk: entry(c) = the chain's first node in chunk c,
//      carry(c) = the last success before it -- one dependent load per chunk that holds a success;
//   C. per chunk, successes = mask(entry); every op's return code against the last success
//      before it (wp_eval) and its prev.
// Scratch (position-indexed, disjoint between groups): jx (exit), jm (mask), ci (entry | carry).
constexpr uint32_t kNone = 0xFFFFFFFFu;
// The phases run over every big group at once where they are per op: A and C a wave per absolute
// 64-position chunk (wp_jump_links, wp_jump_codes), and the per-group workgroup keeps the start
// search and the chain walk B (wp_jump_chain).  (Round 5 first ran A and C inside the group's
// workgroup, a 64-op chunk per wave and pass: a Zipf-0.99 hot key (~44 K ops) took ~43 dependent
// passes per wave in each -- retired)  A chunk may hold the end of one group and the
// start of the next: the chain's per-chunk record is keyed by max(chunk start, group head),
// distinct for the two.  Phase A starts at the chain's earliest possible node (f - 1 when the head
// succeeded, else the head), so an unresolved candidate before the actual start (the head-failed
// case) only sends the group to the walk, which is exact either way.
__device__ __forceinline__ bool jump_member(const WpArgs &a, const uint32_t *__restrict__ first_fail,
                                            const uint32_t *__restrict__ gend, uint32_t big_from, uint64_t p,
                                            uint64_t &g, uint64_t &f, uint64_t &end) {
    if (p >= a.n || a.loc[p] == a.none) return false;
    g = a.gs[p];
    const uint32_t ff = first_fail[g];
    if (ff == 0xFFFFFFFFu || gend[g] - ff < big_from) return false;
    f = ff;
    end = gend[g];
    return true;
}

__global__ __launch_bounds__(256) void wp_jump_links(WpArgs a, WpCls kc, const uint32_t *__restrict__ first_fail,
                                                     const uint32_t *__restrict__ gend, uint32_t big_from,
                                                     const uint32_t *__restrict__ cfirst, uint32_t *__restrict__ jx,
                                                     uint64_t *__restrict__ jm, uint8_t *__restrict__ junr) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // blockDim: a multiple of 64
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t cb = p - lane;
    uint64_t g = 0, f = 0, end = 0;
    bool in = jump_member(a, first_fail, gend, big_from, p, g, f, end);
    in = in && p >= (f > g ? f - 1 : g);
    if (!__builtin_amdgcn_ballot_w64(in)) return;  // wave-uniform
    uint32_t J = kNone;
    uint64_t M = 0;
    if (in) {
        M = 1ull << lane;
        const uint32_t cp = commit_of(a, a.op[p]);
        if (cp != 0) {  // an uncommitted success leaves every later op DIRTY
            const uint32_t cl = kc.cls[p];
            const uint64_t cand = (p + 1 < end && kc.cls[p + 1] == cl) ? cfirst[cl + 1] : p + 1;
            if (cand < end) {
                if (a.writer[a.op[cand]] >= cp) J = (uint32_t)cand;
                else junr[g] = 1;  // (benign race: every writer stores 1)
            }
        }
    }
    const uint32_t cend = (uint32_t)(cb + 64);
#pragma unroll
    for (int r = 0; r < 6; ++r) {  // doubling inside the chunk: J = f^(2^r)(p), M = its path
        const bool hop = J < cend;
        const int src = hop ? (int)(J - (uint32_t)cb) : (int)lane;
        const uint32_t Jn = (uint32_t)__shfl((int)J, src, 64);
        const uint64_t Mn = __shfl(M, src, 64);
        if (hop) {
            J = Jn;
            M |= Mn;
        }
    }
    if (in) {
        jx[p] = J;
        jm[p] = M;
    }
}

__global__ __launch_bounds__(kJumpThreads) __attribute__((amdgpu_waves_per_eu(6))) void wp_jump_chain(WpArgs a, WpCls kc, DevTable t, uint8_t *__restrict__ rcs,
                                                      uint8_t *__restrict__ succ, int32_t *__restrict__ prev,
                                                      const uint32_t *__restrict__ first_fail,
                                                      const uint32_t *__restrict__ gend,
                                                      const uint32_t *__restrict__ list,
                                                      const uint32_t *__restrict__ count,
                                                      const uint32_t *__restrict__ jx, const uint64_t *__restrict__ jm,
                                                      uint64_t *__restrict__ ci, uint32_t *__restrict__ gst,
                                                      const uint8_t *__restrict__ junr) {
    constexpr uint32_t kSpanChunks = 16, kSpan = kSpanChunks * 64;  // 1024 positions, 12 KB a buffer
    __shared__ uint32_t s_jx[2][kSpan];
    __shared__ uint64_t s_jm[2][kSpan];
    __shared__ uint64_t s_first[kJumpWaves];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t nbig = *count;
    for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) {
        const uint64_t g = list[i];
        const uint64_t l = a.loc[g], end = gend[g];
        const SlotInfo base = t.slot[l];
        const uint64_t f = first_fail[g];
        uint64_t start;
        if (f > g) {
            start = f - 1;
        } else {  // the head failed: the first op that succeeds against the epoch-start state
            start = ~0ull;
            for (uint64_t done = g; done < end && start == ~0ull; done += kJumpThreads) {
                const uint64_t q = done + (uint64_t)wv * 64 + lane;
                const uint8_t r = q < end ? wp_eval(a, kc, t, q, g, -1, base) : (uint8_t)0xFF;
                uint64_t wf = r == STAGE_RC_OK ? q : ~0ull;
                for (int o = 32; o > 0; o >>= 1) {
                    const uint64_t x = __shfl_xor(wf, o, 64);
                    wf = x < wf ? x : wf;
                }
                __syncthreads();
                if (lane == 0) s_first[wv] = wf;
                __syncthreads();
                uint64_t bf = ~0ull;
#pragma unroll
                for (uint32_t w = 0; w < kJumpWaves; ++w) bf = s_first[w] < bf ? s_first[w] : bf;
                if (q < end && q <= bf) {
                    rcs[q] = r;
                    succ[q] = q == bf;
                    prev[q] = -1;
                }
                start = bf;
            }
        }
        if (threadIdx.x == 0) gst[g] = start == ~0ull ? kNone : (uint32_t)start;
        if (start == ~0ull) continue;  // nothing succeeds: every op was evaluated above
        if (junr[g]) {  // a candidate's writer is older than the commit: walk the group instead
            finish_big_walk(a, kc, t, rcs, succ, prev, g, end, f, base, s_first);
            __syncthreads();
            continue;
        }
        // B. the chain, chunk to chunk, over absolute chunks, the
        // exits and masks staged through LDS a span of kSpanChunks chunks at a time: waves 1..
        // fill the next span while wave 0 walks this one (from registers, kPre chunks per LDS
        // batch, by readlane)
        const uint64_t c_lo = start & ~63ull, nch = (end - c_lo + 63) / 64;
        const uint64_t nspan = (nch + kSpanChunks - 1) / kSpanChunks;
        auto fill = [&](uint64_t sp, int buf, uint32_t t0, uint32_t nt) {
            const uint64_t pbase = c_lo + sp * kSpan;
            for (uint32_t j0 = t0; j0 < kSpan; j0 += 8 * nt) {  // one round trip for 512+ threads
                uint32_t x[8];
                uint64_t m[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t j = j0 + u * nt;
                    const uint64_t p = pbase + j;
                    const bool ok = j < kSpan && p >= start && p < end;
                    x[u] = ok ? jx[p] : kNone;
                    m[u] = ok ? jm[p] : 0ull;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t j = j0 + u * nt;
                    if (j < kSpan) {
                        s_jx[buf][j] = x[u];
                        s_jm[buf][j] = m[u];
                    }
                }
            }
        };
        fill(0, 0, threadIdx.x, blockDim.x);
        __syncthreads();
        // the walk's state is wave-uniform and kept in scalar registers (32-bit positions, values
        // taken by readlane), so each chunk step is a few scalar instructions and no exec-mask
        // branches; lane kk collects chunk kk's record and the span's records are stored at once
        // (start comes through LDS in the head-failed case: readfirstlane tells the compiler it is
        // uniform, so the walk stays on the scalar unit)
        uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)start);
        int32_t carry = __builtin_amdgcn_readfirstlane(f > g ? (start > g ? (int32_t)(start - 1) : -1) : -1);
        for (uint64_t sp = 0; sp < nspan; ++sp) {
            const int buf = (int)(sp & 1);
            if (wv != 0) {
                if (sp + 1 < nspan) fill(sp + 1, buf ^ 1, threadIdx.x - 64, blockDim.x - 64);
            } else {
                constexpr int kPre = 16;
                const uint64_t ch0 = sp * kSpanChunks;
                const uint32_t nin = (uint32_t)(nch - ch0 < kSpanChunks ? nch - ch0 : kSpanChunks);
                const uint32_t cs = (uint32_t)(c_lo + 64 * ch0);  // the span's first chunk start
                int rec_lo = 0, rec_hi = 0;  // lane kk: chunk kk's record
                for (uint32_t k0 = 0; k0 < nin; k0 += kPre) {
                    uint32_t xr[kPre], ml[kPre], mh[kPre];
#pragma unroll
                    for (int k = 0; k < kPre; ++k) {
                        const uint32_t j = (k0 + k) * 64 + lane;
                        xr[k] = s_jx[buf][j];
                        const uint64_t m = s_jm[buf][j];
                        ml[k] = (uint32_t)m;
                        mh[k] = (uint32_t)(m >> 32);
                    }
#pragma unroll
                    for (int k = 0; k < kPre; ++k) {
                        const uint32_t kk = k0 + k, cb = cs + 64 * kk;
                        e = (uint32_t)__builtin_amdgcn_readfirstlane((int)e);  // scalar compares below
                        carry = __builtin_amdgcn_readfirstlane(carry);
                        uint32_t entry = kNone;
                        int32_t next_carry = carry;
                        if (kk < nin && e != kNone && e - cb < 64u) {
                            const int el = (int)(e - cb);
                            const uint64_t m = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mh[k], el) << 32) |
                                               (uint32_t)__builtin_amdgcn_readlane((int)ml[k], el);
                            next_carry = (int32_t)(cb + 63 - (uint32_t)__builtin_clzll(m));
                            entry = e;
                            e = (uint32_t)__builtin_amdgcn_readlane((int)xr[k], el);
                        }
                        rec_lo = lane == kk ? (int)entry : rec_lo;
                        rec_hi = lane == kk ? carry : rec_hi;
                        carry = next_carry;
                    }
                }
                if (lane < nin) {
                    const uint64_t cb = (uint64_t)cs + 64ull * lane;
                    ci[cb > g ? cb : g] = (uint64_t)(uint32_t)rec_lo | ((uint64_t)(uint32_t)rec_hi << 32);
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(256) void wp_jump_codes(WpArgs a, WpCls kc, DevTable t, uint8_t *__restrict__ rcs,
                                                     uint8_t *__restrict__ succ, int32_t *__restrict__ prev,
                                                     const uint32_t *__restrict__ first_fail,
                                                     const uint32_t *__restrict__ gend, uint32_t big_from,
                                                     const uint32_t *__restrict__ gst, const uint8_t *__restrict__ junr,
                                                     const uint64_t *__restrict__ jm, const uint64_t *__restrict__ ci) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = (uint32_t)(p & 63);
    const uint64_t cb = p - lane;
    uint64_t g = 0, f = 0, end = 0;
    if (!jump_member(a, first_fail, gend, big_from, p, g, f, end) || junr[g]) return;
    const uint32_t st = gst[g];
    if (st == kNone || p < st) return;
    const uint64_t info = ci[cb > g ? cb : g];
    const uint32_t entry = (uint32_t)info;
    const int32_t carry = (int32_t)(uint32_t)(info >> 32);
    const uint64_t M = entry != kNone ? jm[entry] : 0ull;
    const bool s = (M >> lane) & 1ull;
    const uint64_t below = M & (lane ? ~0ull >> (64 - lane) : 0ull);
    const int64_t ps = below ? (int64_t)(cb + 63 - __builtin_clzll(below)) : (int64_t)carry;
    succ[p] = s;
    prev[p] = (int32_t)ps;
    if (s) {
        rcs[p] = (uint8_t)STAGE_RC_OK;
    } else {
        SlotInfo base{};
        if (ps < 0) base = t.slot[a.loc[g]];  // the epoch-start state matters only against no success
        rcs[p] = wp_eval(a, kc, t, p, g, ps, base);
    }
}

// step 4 input: successes in the low word, committed successes in the high word
__global__ __launch_bounds__(256) void wp_flags(WpArgs a, const uint8_t *__restrict__ succ, uint64_t *__restrict__ flags) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    const uint64_t s = succ[q] ? 1ull : 0ull;
    flags[q] = s | ((s && commit_of(a, a.op[q]) != 0) ? (1ull << 32) : 0ull);
}

// tot = {successes, committed successes, this epoch's copy / version / image bases}; the
// device's append counters (bases) move past this epoch's entries
__global__ __launch_bounds__(256) void wp_totals(const uint64_t *__restrict__ ranks, const uint64_t *__restrict__ flags, uint64_t n,
                          uint64_t *__restrict__ tot, uint64_t *__restrict__ bases) {
    const uint64_t v = ranks[n - 1] + flags[n - 1];
    const uint64_t ns = v & 0xFFFFFFFFull, nv = v >> 32;
    tot[0] = ns;
    tot[1] = nv;
    tot[2] = bases[0];
    tot[3] = bases[1];
    tot[4] = bases[2];
    bases[0] += ns;
    bases[1] += nv;
    bases[2] += ns;
}

__global__ __launch_bounds__(256) void wp_set_bases(uint64_t *__restrict__ bases, uint64_t c, uint64_t v, uint64_t i) {
    bases[0] = c;
    bases[1] = v;
    bases[2] = i;
}

// what wp_write needs per success, at its success rank: the epoch-start image to copy and the op
struct WRec {
    uint32_t image, op;
};

// step 5a, one thread per sorted position: a success writes its overwrite-copy header, the
// retired-version header when committed, and its WRec; the last success of each group is
// marked (last_succ; one atomic per group per wave)
__global__ __launch_bounds__(256) void wp_headers(WpArgs a, DevTable t, const uint8_t *__restrict__ succ, const int32_t *__restrict__ prev,
                           const uint64_t *__restrict__ ranks, CopyHdr *__restrict__ chdr, VersionHdr *__restrict__ vhdr,
                           uint32_t *__restrict__ last_succ, WRec *__restrict__ wrec, const uint64_t *__restrict__ tot,
                           uint32_t *__restrict__ cwriter) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // blockDim: a multiple of 64
    if (q >= a.n) return;
    const uint64_t cbase = tot[2], vbase = tot[3], ibase = tot[4];
    const uint32_t lane = threadIdx.x & 63;
    const bool ok = succ[q] != 0;
    const uint32_t g = a.gs[q];
    if (ok) {
        const uint32_t o = a.op[q];
        const SlotInfo base = t.slot[a.loc[q]];
        const uint64_t rk = ranks[q];
        const uint64_t irank = rk & 0xFFFFFFFFull, vrank = rk >> 32;
        const uint32_t cid = commit_of(a, o);
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
        wrec[irank] = WRec{base.image, o};
        cwriter[irank] = a.writer[o];  // the copy's OverwriteVersionHeader cstamp (the host's SSN state)
    }
    // the group's last success in this wave (no later lane of the group -- the lanes up to the
    // next group head -- succeeded) competes for last_succ
    const uint64_t sm = __builtin_amdgcn_ballot_w64(ok);
    const uint64_t hm = __builtin_amdgcn_ballot_w64(g == q);
    const uint64_t after = lane == 63 ? 0ull : ~0ull << (lane + 1);
    const uint64_t nh = hm & after;
    const uint64_t mine_after = after & (nh ? (nh & (~nh + 1)) - 1 : ~0ull);
    if (ok && !(sm & mine_after)) atomicMax(&last_succ[g], (uint32_t)q + 1u);
}

// step 5b: the new rows, a team of 16 lanes per success (4 per wave, 4 chunks of 16 B per lane
// in flight): the epoch-start row with the column window patched (CopyPayload)
constexpr uint32_t kRowTeam = 16;
__global__ __launch_bounds__(256) void wp_write(WpArgs a, DevTable t, uint8_t *__restrict__ heap,
                                                const WRec *__restrict__ wrec, const uint64_t *__restrict__ tot) {
    const uint64_t ibase = tot[4];
    const uint32_t tl = threadIdx.x & (kRowTeam - 1);
    const uint64_t nteams = (uint64_t)gridDim.x * (blockDim.x / kRowTeam);
    const uint64_t ns = tot[0];
    const uint32_t chunks = t.hstride / 16;
    const uint32_t w0 = a.win_off, w1 = a.win_off + a.delta_len;
    for (uint64_t si = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kRowTeam; si < ns; si += nteams) {
        const WRec w = wrec[si];
        const u32x4 *src = reinterpret_cast<const u32x4 *>(t.heap + (uint64_t)w.image * t.hstride);
        u32x4 *dst = reinterpret_cast<u32x4 *>(heap + (ibase + si) * t.hstride);
        const uint8_t *d = a.deltas + (uint64_t)w.op * a.delta_len;
        for (uint32_t c0 = 0; c0 < chunks; c0 += 4 * kRowTeam) {
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t c = c0 + u * kRowTeam + tl;
                v[u] = c < chunks ? src[c] : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t c = c0 + u * kRowTeam + tl;
                if (c >= chunks) continue;
                const uint32_t b0 = c * 16;
                if (b0 + 16 > w0 && b0 < w1) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        uint32_t x = v[u][k];
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const uint32_t pos = b0 + 4 * k + j;
                            if (pos >= w0 && pos < w1)
                                x = (x & ~(0xFFu << (8 * j))) | ((uint32_t)d[pos - w0] << (8 * j));
                        }
                        v[u][k] = x;
                    }
                }
                dst[c] = v[u];
            }
        }
    }
}

struct FinRec {
    uint64_t loc, meta;
    uint32_t next, image;
};
static_assert(sizeof(FinRec) == 24, "wp_keys initialises a FinRec as three 8-byte words");

// step 6: the last success of each group publishes the slot word; every op gets its code
__global__ void wp_publish(WpArgs a, SlotInfo *__restrict__ slot, const uint8_t *__restrict__ rcs,
                           const uint8_t *__restrict__ succ, const int32_t *__restrict__ prev,
                           const uint64_t *__restrict__ ranks, const uint32_t *__restrict__ last_succ,
                           const uint64_t *__restrict__ tot, FinRec *__restrict__ fin, uint8_t *__restrict__ rc_out) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    const uint64_t cbase = tot[2], vbase = tot[3], ibase = tot[4];
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

// the epoch's results for the host, written by the GPU straight into pinned host memory as soon
// as the write path is done (on the adoption stream, beside the next probe): totals, the new
// copy and version headers, the slot words -- the staging layout of stage_update_batch_device
__global__ __launch_bounds__(256) void wp_export(const uint64_t *__restrict__ tot, const FinRec *__restrict__ fin,
                                                 const CopyHdr *__restrict__ chdr, const VersionHdr *__restrict__ vhdr,
                                                 const uint32_t *__restrict__ cwriter, uint8_t *__restrict__ pin,
                                                 uint64_t fin_off, uint64_t wr_off) {
    const uint64_t ns = tot[0], nv = tot[1];
    const uint64_t *c = reinterpret_cast<const uint64_t *>(chdr + tot[2]);
    const uint64_t *v = reinterpret_cast<const uint64_t *>(vhdr + tot[3]);
    const uint64_t *f = reinterpret_cast<const uint64_t *>(fin);
    uint64_t *oc = reinterpret_cast<uint64_t *>(pin + 64), *ov = oc + ns * 2;
    uint64_t *of = reinterpret_cast<uint64_t *>(pin + fin_off);
    static_assert(sizeof(CopyHdr) == 16 && sizeof(VersionHdr) == 16 && sizeof(FinRec) == 24, "export words");
    const uint64_t w1 = ns * 2, w2 = w1 + nv * 2, total = w2 + ns * 3;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = gid; i < total; i += stride) {
        if (i < w1) oc[i] = c[i];
        else if (i < w2) ov[i - w1] = v[i - w1];
        else of[i - w2] = f[i - w2];
    }
    uint32_t *ow = reinterpret_cast<uint32_t *>(pin + wr_off);
    for (uint64_t i = gid; i < ns; i += stride) ow[i] = cwriter[i];
    if (gid < 5) reinterpret_cast<uint64_t *>(pin)[gid] = tot[gid];
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
        // the host table is NOT settled here: the previous epoch may still be adopted in the
        // background (stage_table::start_adoption) -- this call reads only the table's fixed
        // geometry and the device image
        HostTable &h = *t->host;
        DeviceImage &dv = t->dev;
        hip_check(hipSetDevice(dv.device), "hipSetDevice");
        hipStream_t s = pick(t, stream);
        // STAGE_WP_TRACE=1: per-phase host wall times on stderr
        static const bool trace = std::getenv("STAGE_WP_TRACE") != nullptr;
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        static const auto g0 = t0;  // trace: the first call's start
        auto ms = [&](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
        // epoch e uses output buffers e % kWpDepth: epoch e - kWpDepth's adoption must be done with them
        const uint64_t epoch = ++t->wp_started;
        const int par = (int)(epoch % kWpDepth);
        // an epoch that fails before its adoption starts still counts as adopted -- with a
        // sticky error (the device may hold part of it): later calls neither hang nor go on
        // -- unless nothing of it reached the device yet (an allocation or stream / event creation
        // failed): then the epoch is rolled back and the table stays usable
        struct EpochGuard {
            stage_table *t;
            uint64_t epoch;
            bool enqueued = false, started = false;
            ~EpochGuard() {
                if (started) return;
                if (!enqueued) {
                    --t->wp_started;
                    return;
                }
                t->start_adoption(epoch, [] { throw std::runtime_error("a device write-path epoch failed"); });
            }
        } guard{t, epoch};
        if (epoch > (uint64_t)kWpDepth) t->wait_adopted(epoch - kWpDepth);
        if (t->adopt_failed.load(std::memory_order_acquire)) t->settle();  // rethrows the adoption's error
        // pending: epochs (adopted, e) are still being adopted, so the device's append counters
        // are ahead of the host table; otherwise (no epoch in flight) they are set from the
        // host's counts.  wp_adopted is read before adopted_sz (stored after it): the bound below
        // can only come out high
        const uint64_t adopted = t->wp_adopted.load(std::memory_order_acquire);
        bool pending = adopted + 1 < epoch;
        if (!dv.wp_bases.p) {
            hip_check(hipMalloc(&dv.wp_bases.p, 64), "wp bases");
            dv.wp_bases.cap = 64;
        }
        // room for one copy, image and version per op beyond the device's counters -- at most the
        // host's counts after the last adopted epoch plus the ops of the one still pending.
        // Growing moves the header arrays, which a pending adoption may be reading: settle
        // first then, and leave room for the next pipelined epoch too
        uint64_t *ub = dv.wp_ub;
        if (!pending) {  // no adoption running: the host's counts are the device's
            h.reserve_adoption(16 * n);  // the next 16 epochs of this size adopt without reallocating
            ub[0] = h.copies_.size(), ub[1] = h.versions_.size(), ub[2] = h.images_.size();
            for (int k = 0; k < 3; ++k) t->adopted_sz[k].store(ub[k], std::memory_order_relaxed);
        } else {
            uint64_t inflight = 0;  // the ops of epochs adopted + 1 .. e - 1 (at most kWpDepth - 1 of them)
            for (uint64_t j = adopted + 1; j < epoch; ++j) inflight += t->wp_epoch_n[j % kWpDepth];
            for (int k = 0; k < 3; ++k) ub[k] = t->adopted_sz[k].load(std::memory_order_acquire) + inflight;
        }
        const bool fits = dv.heap_rows >= ub[2] + n && dv.chdr.cap >= (ub[0] + n) * sizeof(CopyHdr) &&
                          dv.vhdr.cap >= (ub[1] + n) * sizeof(VersionHdr) && dv.chdr.p && dv.vhdr.p && dv.heap.p;
        if (!fits) {  // room for the next 8 epochs of this size: a growth drains the pipeline
            t->settle();
            pending = false;
            reserve_device_rows(h, dv, 8 * n, 8 * n, 8 * n, s);
        }
        const double t_reserve = ms(t0);
        if (t->wp_overlap && !dv.wp_stream) {
            // the overlapped write kernels on a high-priority stream, so their workgroups are
            // dispatched as the probe's retire instead of after all of them (C3 +1.5-2.5 %)
            int lo = 0, hi = 0;
            hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priorities");
            hip_check(hipStreamCreateWithPriority(&dv.wp_stream, hipStreamNonBlocking, hi), "write stream");
        }
        for (hipEvent_t *e : {&dv.wp_pub_ev, &dv.wp_pre_ev})
            if (!*e) hip_check(hipEventCreateWithFlags(e, hipEventDisableTiming), "write event");
        if (!dv.adopt_stream) {  // high priority: the export gets its CUs beside the next probe
            int lo = 0, hi = 0;
            hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priorities");
            hip_check(hipStreamCreateWithPriority(&dv.adopt_stream, hipStreamNonBlocking, hi), "adopt stream");
        }
        for (int k = 0; k < kWpDepth; ++k)
            for (hipEvent_t *e : {&dv.adopt_ev[k], &dv.export_ev[k]})
                if (!*e) hip_check(hipEventCreateWithFlags(e, hipEventDisableTiming), "adopt event");
        const DevTable &view = dv.view;
        const uint64_t none = (uint64_t)view.nleaves * view.cap;
        int end_bit = 1;
        while (end_bit < 64 && (none >> end_bit)) ++end_bit;

        // scratch
        size_t cub_sort = 0, cub_scan = 0, cub_sum = 0;
        hip_check(sort_pairs(nullptr, cub_sort, (const uint64_t *)nullptr, (uint64_t *)nullptr, (const uint32_t *)nullptr,
                             (uint32_t *)nullptr, n, 0, end_bit, s),
                  "sort size");
        hip_check(hipcub::DeviceScan::InclusiveScan(nullptr, cub_scan, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                    hipcub::Max(), (int)n, s),
                  "scan size");
        hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, cub_sum, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)n,
                                                   s),
                  "sum size");
        size_t cub_cls = 0;
        hip_check(hipcub::DeviceScan::InclusiveSum(nullptr, cub_cls, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, s),
                  "class scan size");
        const size_t cub_bytes = std::max(std::max(cub_sort, cub_cls), std::max(cub_scan, cub_sum));
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
                       o_ranks = take(n * 8), o_brk = take(n * 4), o_cls = take(n * 4),
                       o_fp = take(n * 8), o_wfp = take(n * 8), o_eqw = take(n), o_wrec = take(n * sizeof(WRec)),
                       o_cfirst = take((n + 2) * 4), o_jx = take(n * 4), o_jm = take(n * 8), o_ci = take(n * 8),
                       o_gst = take(n * 4), o_junr = take(n), o_fpo = take(n * 8), o_wfpo = take(n * 8),
                       o_eqwo = take(n),
                       o_cub = take(cub_bytes);
        // the write path's own scratch: an overlapped epoch runs beside the caller's later work,
        // which may use the table's shared scratch (stock-level, CH-Q2, scans)
        uint8_t *buf = wp_scratch_bytes(dv, off);
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
        auto *brk = (uint32_t *)(buf + o_brk);
        auto *cls = (uint32_t *)(buf + o_cls);
        auto *fpd = (uint64_t *)(buf + o_fp);
        auto *wfp = (uint64_t *)(buf + o_wfp);
        auto *eqw = buf + o_eqw;
        auto *wrec = (WRec *)(buf + o_wrec);
        auto *cfirst = (uint32_t *)(buf + o_cfirst);
        auto *jx = (uint32_t *)(buf + o_jx);
        auto *jm = (uint64_t *)(buf + o_jm);
        auto *ci = (uint64_t *)(buf + o_ci);
        auto *gst = (uint32_t *)(buf + o_gst);
        auto *junr = buf + o_junr;
        auto *fp_op = (uint64_t *)(buf + o_fpo), *wfp_op = (uint64_t *)(buf + o_wfpo);
        auto *eqw_op = buf + o_eqwo;
        // slot words + totals: read back after this call returns (background adoption)
        // every epoch's buffers are sized together when no adoption is reading another one: a
        // first use inside a run of epochs would allocate (and drain the device) in the middle of it
        const uint64_t wo_bytes = al(n * sizeof(FinRec)) + 256 + al(n * 4);
        uint8_t *wo = wp_out_bytes(dv, wo_bytes, par);
        for (int k = 0; k < kWpDepth && !pending; ++k) wp_out_bytes(dv, wo_bytes, k);
        auto *fin = (FinRec *)wo;
        auto *tot = (uint64_t *)(wo + al(n * sizeof(FinRec)));
        auto *cwriter = (uint32_t *)(wo + al(n * sizeof(FinRec)) + 256);  // writer id per new copy
        void *cub = buf + o_cub;
        size_t cb = cub_bytes;
        // pinned staging of the adoption: [totals 64 B][copy headers][version headers][slot
        // words], sized for the worst case (one copy and one version per op); every part starts
        // on a 16-B boundary (the headers are 16-B aligned types: a misaligned source faults in
        // the vectorised copy)
        // [.. slot words][writer id per copy]
        const uint64_t bf = n * sizeof(FinRec), bmax = 2 * n * sizeof(CopyHdr), bw = n * 4;
        static_assert(sizeof(CopyHdr) == sizeof(VersionHdr) && sizeof(CopyHdr) % 16 == 0, "header sizes");
        uint8_t *pin = pinned_bytes(dv, 64 + bmax + bf + bw, par);
        for (int k = 0; k < kWpDepth && !pending; ++k) pinned_bytes(dv, 64 + bmax + bf + bw, k);
        // write-overlap mode: the kernels up to the publish go on the table's write stream ks,
        // which waits for the previous epoch's publish only (or, when the device image changed
        // otherwise since, for all of s) -- not for the caller's work enqueued after it, such as
        // the previous epoch's read probes.  They read the slot words that publish left and
        // write only scratch, this epoch's output parity and the appended header / row ranges
        // no published slot word reaches yet; the publish joins s behind them.
        // Either mode: the epoch starts after the previous epoch's publish (wp_pub_ev, recorded
        // after every publish), so a caller that alternates streams between epochs stays ordered
        // on the device append counters and slot words the previous epoch left.
        hipStream_t ks = s;
        if (t->wp_overlap) {
            if (!dv.wp_pub_valid) hip_check(hipEventRecord(dv.wp_pub_ev, s), "write event");
            hip_check(hipStreamWaitEvent(dv.wp_stream, dv.wp_pub_ev, 0), "write wait");
            ks = dv.wp_stream;
        } else if (dv.wp_pub_valid) {
            hip_check(hipStreamWaitEvent(s, dv.wp_pub_ev, 0), "previous publish");
        }
        // from here on the epoch reaches the device: a failure is sticky (see EpochGuard)
        guard.enqueued = true;
        if (!pending)
            wp_set_bases<<<1, 1, 0, ks>>>((uint64_t *)dv.wp_bases.p, h.copies_.size(), h.versions_.size(),
                                          h.images_.size());
        t->wp_epoch_n[par] = n;

        // 1. locate
        hip_check(launch_probe(view, d_keys, d_lens, nullptr, nullptr, n, pout, nullptr, ks, t->tune), "locate");
        wp_keys<<<blocks_for(n * kTeam, 256), 256, 0, ks>>>(pout, n, none, view, d_deltas, delta_len,
                                                            facts(t).key_pad() + payload_off,
                                                            (uint64_t)payload_off + delta_len > facts(t).params().payload_size,
                                                            loc0, op0, fp_op, wfp_op,
                                                            eqw_op, ff, ls, (uint64_t *)fin, (uint32_t *)(tot + 1));
        // 2. group
        hip_check(sort_pairs(cub, cb, (const uint64_t *)loc0, loc, (const uint32_t *)op0, op, n, 0, end_bit, ks), "sort");
        wp_heads<<<blocks_for(n, 256), 256, 0, ks>>>(loc, n, head);
        cb = cub_bytes;
        hip_check(hipcub::DeviceScan::InclusiveScan(cub, cb, head, gs, hipcub::Max(), (int)n, ks), "group starts");
        // 3. decide
        WpArgs a{loc, op, gs, d_deltas, d_writer_ids, d_commit_ids, d_sstamps, n, none, delta_len,
                 facts(t).key_pad() + payload_off,
                 (uint64_t)payload_off + delta_len > facts(t).params().payload_size ? 1u : 0u};
        wp_classify<<<blocks_for(n, 256), 256, 0, ks>>>(a, fp_op, wfp_op, eqw_op, brk, fpd, wfp, eqw);
        cb = cub_bytes;
        hip_check(hipcub::DeviceScan::InclusiveSum(cub, cb, brk, cls, (int)n, ks), "delta classes");
        const WpCls kc{cls, fpd, wfp, eqw};
        wp_speculate<<<blocks_for(n, 256), 256, 0, ks>>>(a, kc, view, rcs, succ, prev, ff, gend, brk, cfirst);
        // big failing groups (at least kJumpFrom ops from their first failure on) by pointer
        // jumping, smaller ones a wave each (wp_finish_groups)
        // (the big-group count, tot[1]'s low word, was zeroed by wp_keys; tot is rewritten in step 4)
        wp_finish_groups<<<blocks_for(n, 256), 256, 0, ks>>>(a, kc, view, rcs, succ, prev, ff, gend, kJumpFrom, big,
                                                             (uint32_t *)(tot + 1), junr);
        wp_jump_links<<<blocks_for(n, 256), 256, 0, ks>>>(a, kc, ff, gend, kJumpFrom, cfirst, jx, jm, junr);
        wp_jump_chain<<<1024, kJumpThreads, 0, ks>>>(a, kc, view, rcs, succ, prev, ff, gend, big, (uint32_t *)(tot + 1), jx, jm, ci,
                                            gst, junr);
        wp_jump_codes<<<blocks_for(n, 256), 256, 0, ks>>>(a, kc, view, rcs, succ, prev, ff, gend, kJumpFrom, gst, junr, jm,
                                                          ci);
        // 4. number
        wp_flags<<<blocks_for(n, 256), 256, 0, ks>>>(a, succ, flags);
        cb = cub_bytes;
        hip_check(hipcub::DeviceScan::ExclusiveSum(cub, cb, flags, ranks, (int)n, ks), "ranks");
        wp_totals<<<1, 1, 0, ks>>>(ranks, flags, n, tot, (uint64_t *)dv.wp_bases.p);
        wp_headers<<<blocks_for(n, 256), 256, 0, ks>>>(a, view, succ, prev, ranks, (CopyHdr *)dv.chdr.p,
                                                      (VersionHdr *)dv.vhdr.p, ls, wrec, tot, cwriter);
        // 5. write, 6. publish
        const int wblocks = (int)std::min<uint64_t>(blocks_for(n, 256 / kRowTeam), 32768);
        wp_write<<<wblocks, 256, 0, ks>>>(a, view, (uint8_t *)dv.heap.p, wrec, tot);
        if (ks != s) hip_check(hipEventRecord(dv.wp_pre_ev, ks), "write event");
        // the publish and everything after it (the slot words, the export to the host, the host
        // table's adoption)
        auto finish = [=, &h, &dv](hipStream_t s, bool want_n) -> uint64_t {
            if (ks != s) hip_check(hipStreamWaitEvent(s, dv.wp_pre_ev, 0), "publish wait");
            wp_publish<<<blocks_for(n, 256), 256, 0, s>>>(a, (SlotInfo *)dv.slot.p, rcs, succ, prev, ranks, ls, tot, fin,
                                                          d_rc);
            hip_check(hipGetLastError(), "write-path kernels");
            hip_check(hipEventRecord(dv.wp_pub_ev, s), "write event");  // the next epoch starts after it
            dv.wp_pub_valid = true;

            // the host adopts the epoch.  The headers and slot words come back on a stream of their
            // own into pinned staging (full PCIe rate) and the host adopts them on a background
            // thread (stage_table::start_adoption) while the caller's stream goes on (the next probe
            // -- and the next epoch's write path -- overlap the copies); the next call that needs the
            // host table waits for it (host() / settle).
            const double t_enqueue = ms(t0);
            const double t_events = ms(t0);
            hip_check(hipEventRecord(dv.adopt_ev[par], s), "adopt event");
            auto *totals = reinterpret_cast<uint64_t *>(pin);
            auto *fr = reinterpret_cast<FinRec *>(pin + 64 + bmax);
            auto *writers = reinterpret_cast<const uint32_t *>(pin + 64 + bmax + bf);
            const double t_pinned = ms(t0);
            void *pin_dev = nullptr;
            hip_check(hipHostGetDevicePointer(&pin_dev, pin, 0), "pinned device pointer");
            hip_check(hipStreamWaitEvent(dv.adopt_stream, dv.adopt_ev[par], 0), "export wait");
            constexpr int kExportBlocks = 32;  // beside the next probe: 32 was the best of the r05 sweep
            wp_export<<<kExportBlocks, 256, 0, dv.adopt_stream>>>(tot, fin, (const CopyHdr *)dv.chdr.p, (const VersionHdr *)dv.vhdr.p,
                                                        cwriter, (uint8_t *)pin_dev, 64 + bmax, 64 + bmax + bf);
            hip_check(hipGetLastError(), "export");
            hip_check(hipEventRecord(dv.export_ev[par], dv.adopt_stream), "export event");
            uint64_t ns = 0;
            if (want_n) {  // the caller wants the count now: wait for the kernels
                uint64_t tv[2] = {0, 0};
                hip_check(hipMemcpyAsync(tv, tot, 16, hipMemcpyDeviceToHost, s), "totals");
                hip_check(hipStreamSynchronize(s), "write path");
                ns = tv[0];
            }
            const double t_kernels = ms(t0);
            // FinRec and HostTable::SlotWords share a layout: device slot locations become host slot
            // indices in place (ops that published nothing keep ~0 and are skipped by the adoption)
            static_assert(sizeof(FinRec) == sizeof(HostTable::SlotWords) &&
                              offsetof(FinRec, meta) == offsetof(HostTable::SlotWords, meta) &&
                              offsetof(FinRec, next) == offsetof(HostTable::SlotWords, next) &&
                              offsetof(FinRec, image) == offsetof(HostTable::SlotWords, image),
                          "FinRec / SlotWords layout");
            t->start_adoption(epoch, [t, &h, &dv, par, epoch, cap = view.cap, n, pin, totals, fr, writers, t0, t_kernels, t_enqueue,
                               t_reserve, t_events, t_pinned]() {
                const double t_join = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
                hip_check(hipSetDevice(dv.device), "hipSetDevice");
                hip_check(hipEventSynchronize(dv.export_ev[par]), "adopt export");
                const uint64_t ns = totals[0], nv = totals[1], cbase = totals[2], vbase = totals[3];
                if (ns > n) throw std::runtime_error("write path: more successes than ops");
                // the epochs are adopted in order: the host's counts are this epoch's bases
                if (h.copies_.size() != cbase || h.versions_.size() != vbase || h.images_.size() != totals[4])
                    throw std::runtime_error("write path: device append counters disagree with the host table");
                auto *copies = reinterpret_cast<CopyHdr *>(pin + 64);
                auto *versions = reinterpret_cast<VersionHdr *>(pin + 64 + ns * sizeof(CopyHdr));
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
                h.adopt_device_epoch(copies, writers, ns, versions, nv, ns, reinterpret_cast<const HostTable::SlotWords *>(fr), ns);
                t->adopted_sz[0].store(h.copies_.size(), std::memory_order_release);
                t->adopted_sz[1].store(h.versions_.size(), std::memory_order_release);
                t->adopted_sz[2].store(h.images_.size(), std::memory_order_release);
                if (trace)
                    std::fprintf(stderr,
                                 "[wp] epoch %llu at %.2f ms: n=%llu ok=%llu reserve %.2f enqueue %.2f events %.2f pinned %.2f kernels %.2f "
                                 "previous adopted %.2f exported %.2f adopted %.2f ms (background)\n",
                                 (unsigned long long)epoch,
                                 std::chrono::duration<double, std::milli>(t0 - g0).count(), (unsigned long long)n,
                                 (unsigned long long)ns, t_reserve, t_enqueue, t_events, t_pinned, t_kernels, t_join, t_d2h,
                                 std::chrono::duration<double, std::milli>(clk::now() - t0).count());
            });
            return ns;
        };
        const uint64_t ns = finish(s, n_ok != nullptr);
        guard.started = true;
        if (n_ok) *n_ok = ns;
        return STAGE_OK;
    });
}
