// chq2.hip -- CH-benCHmark Q2 (RunQuery2, benchmark/tpcc/tpcc_new_order.cpp:608-982) through the
// index-organized read path.
//
// Reference transaction at one read id:
//   1. REGION TableScan of 6 from key 0, NATION TableScan of 65 from key 0 (:650-761);
//   2. for the region named regions[target] (tpcc_record.h:931) and each of its nations, the
//      SUPPLIER table scan (scan_sz -1: every record, :779-797) filtered on SU_NATIONKEY;
//   3. per supplier: the STOCK point lookups {w, i} of its supp_stock_map entries
//      (tpcc_workload.cpp:398-404) -- a FAILURE read or a lookup with no tuple aborts; the
//      "minimum" keeps the LAST stock read because min_qty is never updated (:812-859);
//   4. the ITEM point lookup of that stock's S_I_ID (:862-887); I_DATA containing 'b' skips
//      the supplier (:890-892); otherwise S_QUANTITY < 10 updates S_QUANTITY..S_REMOTE_CNT to
//      (q + 50, ytd, order_cnt, remote_cnt) (:893-950), committed with the transaction.
//
// Here REGION / NATION run as device scans and SUPPLIER as a one-lane-per-slot leaf dump; one
// workgroup (q2_select) filters them -- the region named regions[target], its nations, their
// suppliers in visiting order -- and lays out each visited supplier's supp_stock_map segment; the
// hot part -- every visited supplier's stock lookups (W * I / 10^4 each, ~2600 suppliers for
// EUROPE) and the item lookups -- is one gather kernel, one probe launch over all stock keys,
// their visibility folded at every read id of the batch (aborts and each supplier's last
// stock), one item probe launch and one finishing kernel that writes the records straight into
// the caller's page-locked `out`.  The counts stay on the device (the kernels read them there),
// so a batch has ONE host synchronisation, at its end (round 5; before, the host filtered the
// scans between two synchronisations).  Updates go through the device write path when a commit
// id is given.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "handle.hpp"

using namespace stage_capi;

namespace stage {
namespace {

constexpr int kRegionScan = 6, kNationScan = 65;  // scan_sz of :653 and :734
constexpr uint32_t kIDataOff = 4 + 32 + 8;         // I_DATA in Item's payload (I_IM_ID, I_NAME, I_PRICE)
static const char *const kRegions[] = {"AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"};

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ bool produced(uint32_t st) { return st == ST_LATEST || st == ST_COPY || st == ST_OLD; }

__device__ __forceinline__ int32_t ld_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

__global__ void q2_set_u64(uint64_t *p, uint64_t v) { *p = v; }

// blocks copy the visited suppliers' map entries (2 words each) to their segments; counts[0] =
// the number of visited suppliers (q2_select); nothing is written past m_cap keys (the host
// rejects counts above it after the batch)
__global__ void q2_gather(const uint64_t *__restrict__ map_keys, const uint64_t *__restrict__ src,
                          const uint64_t *__restrict__ dst, const uint32_t *__restrict__ cnt,
                          const uint64_t *__restrict__ counts, uint64_t m_cap, uint64_t *__restrict__ keys) {
    const uint64_t n = counts[0];
    for (uint64_t s = blockIdx.x; s < n; s += gridDim.x)
        for (uint32_t e = threadIdx.x; e < cnt[s] && dst[s] + e < m_cap; e += blockDim.x) {
            keys[2 * (dst[s] + e)] = map_keys[2 * (src[s] + e)];
            keys[2 * (dst[s] + e) + 1] = map_keys[2 * (src[s] + e) + 1];
        }
}

// RunQuery2's selection (tpcc_new_order.cpp:650-797) in one workgroup, from the REGION / NATION
// scan rows and the SUPPLIER slot dump:
//   visits   = for each REGION row named the target (scan order), each NATION row of that region
//              (scan order); a nation is visited at most once (it has one region key, region
//              keys are unique), so at most kNationScan visits, found through an LDS hash;
//   sel      = every SUPPLIER record of each visited nation, visit by visit, in ScanLeafNode
//              (slot dump) order: a stable counting sort by visit.  The slots go through LDS in
//              windows of kSelWin; in each, every lane finds its slots' visits (independent
//              loads), then wave w ranks the window's w-th 1024 slots per visit (one ballot per
//              distinct visit of a 64-slot chunk, LDS only) -- the visit and rank of every slot go
//              to global scratch; one prefix over (visit, window, wave) gives each group's start,
//              and a parallel pass places every selected supplier at start + rank;
//   segments = src / cnt of each selected supplier's supp_stock_map entries (map_off, keys
//              below 10000), dst = their exclusive prefix sum;
//   counts   = {suppliers, stock keys}.
// No loop of this kernel waits on a global load per iteration: the loads are issued side by side.
constexpr int kVisits = kNationScan, kVisitHash = 256;
constexpr uint32_t kSelWin = 16384, kSelMaxWin = 8;  // slots per LDS window, windows per call
__global__ __launch_bounds__(1024) void q2_select(const uint8_t *__restrict__ regs, uint32_t rs,
                                                  const uint8_t *__restrict__ nats, uint32_t ns, uint64_t name0,
                                                  uint64_t name1, const uint64_t *__restrict__ pairs, uint64_t nslots,
                                                  const uint32_t *__restrict__ map_off, int8_t *__restrict__ g_vis,
                                                  uint16_t *__restrict__ g_rank, uint64_t *__restrict__ sel,
                                                  uint64_t *__restrict__ src, uint32_t *__restrict__ cnt,
                                                  uint64_t *__restrict__ dst, uint64_t *__restrict__ counts) {
    __shared__ uint8_t s_rmatch[kRegionScan];
    __shared__ uint8_t s_flag[kRegionScan * kNationScan];
    __shared__ uint32_t s_nvisit;
    __shared__ int64_t s_hkey[kVisitHash];
    __shared__ int32_t s_hval[kVisitHash];
    __shared__ int8_t s_vis[kSelWin];
    __shared__ uint32_t s_grp[kSelMaxWin * 16][kVisits];  // per (window, wave): counts, then starts
    __shared__ uint32_t s_vstart[kVisits];
    __shared__ uint64_t s_wsum[16];
    __shared__ uint64_t s_n;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t nreg = *reinterpret_cast<const uint32_t *>(regs - 8);
    const uint32_t nnat = *reinterpret_cast<const uint32_t *>(nats - 8);
    const uint32_t nwin = (uint32_t)((nslots + kSelWin - 1) / kSelWin);  // <= kSelMaxWin (host check)
    // 1. the visits
    if (tid < kRegionScan && tid < nreg) {  // R_NAME (55 bytes, NUL-terminated) == regions[target]
        const uint8_t *name = regs + (uint64_t)tid * rs + 8;
        bool eq = true;
        for (int i = 0; i < 55; ++i) {
            const uint8_t c = name[i];
            const uint8_t want = i < 8 ? (uint8_t)(name0 >> (8 * i)) : i < 16 ? (uint8_t)(name1 >> (8 * (i - 8))) : 0;
            if (c != want) {
                eq = false;
                break;
            }
            if (c == 0) break;
        }
        s_rmatch[tid] = eq;
    }
    for (uint32_t i = tid; i < kVisitHash; i += blockDim.x) s_hkey[i] = INT64_MIN, s_hval[i] = -1;
    for (uint32_t i = tid; i < kSelMaxWin * 16 * kVisits; i += blockDim.x) (&s_grp[0][0])[i] = 0;
    __syncthreads();
    if (tid < nreg * nnat && tid < kRegionScan * kNationScan) {
        const uint32_t r = tid / nnat, a = tid % nnat;
        const uint8_t *rr = regs + (uint64_t)r * rs, *nr = nats + (uint64_t)a * ns;
        s_flag[tid] = s_rmatch[r] && *reinterpret_cast<const int64_t *>(nr + 8) == *reinterpret_cast<const int64_t *>(rr);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t nv = 0;
        for (uint32_t f = 0; f < nreg * nnat && f < kRegionScan * kNationScan; ++f)
            if (s_flag[f] && nv < (uint32_t)kVisits) {
                const int64_t nk = *reinterpret_cast<const int64_t *>(nats + (uint64_t)(f % nnat) * ns);
                uint32_t h = (uint32_t)(((uint64_t)nk * 0x9E3779B97F4A7C15ull) >> 56);
                while (s_hkey[h] != INT64_MIN && s_hkey[h] != nk) h = (h + 1) & (kVisitHash - 1);
                if (s_hkey[h] == nk) continue;  // (cannot happen: one region per nation)
                s_hkey[h] = nk;
                s_hval[h] = (int32_t)nv++;
            }
        s_nvisit = nv;
    }
    __syncthreads();
    const uint32_t nv = s_nvisit;
    auto visit_of = [&](uint64_t key, uint64_t nat) -> int {
        if (key == ~0ull || nv == 0) return -1;
        uint32_t h = (uint32_t)((nat * 0x9E3779B97F4A7C15ull) >> 56);
        while (s_hkey[h] != INT64_MIN) {
            if (s_hkey[h] == (int64_t)nat) return s_hval[h];
            h = (h + 1) & (kVisitHash - 1);
        }
        return -1;
    };
    // 2. per window: visits of its slots (A), per-wave counts and ranks (B)
    for (uint32_t win = 0; win < nwin; ++win) {
        const uint64_t w0 = (uint64_t)win * kSelWin;
#pragma unroll 4
        for (uint32_t j = tid; j < kSelWin; j += 1024) {
            const uint64_t i = w0 + j;
            int v = -1;
            if (i < nslots) v = visit_of(pairs[2 * i], pairs[2 * i + 1]);
            s_vis[j] = (int8_t)v;
        }
        __syncthreads();
        uint32_t *gc = s_grp[win * 16 + wv];
        for (uint32_t c0 = wv * 1024; c0 < (wv + 1) * 1024; c0 += 64) {
            const uint32_t j = c0 + lane;
            const int v = s_vis[j];
            uint32_t rank = 0;
            uint64_t todo = ballot(v >= 0);
            while (todo) {
                const int vl = (int)rl32((uint32_t)v, (int)__builtin_ctzll(todo));
                const uint64_t mm = ballot(v == vl);
                const uint32_t before = gc[vl];
                if (v == vl) rank = before + (uint32_t)__builtin_popcountll(mm & ((1ull << lane) - 1));
                if (lane == 0) gc[vl] = before + (uint32_t)__builtin_popcountll(mm);
                todo &= ~mm;
            }
            const uint64_t i = w0 + j;
            if (i < nslots) {
                g_vis[i] = (int8_t)v;
                g_rank[i] = (uint16_t)rank;
            }
        }
        __syncthreads();
    }
    // 3. group starts, visit-major, then window, then wave (slot order within a visit)
    const uint32_t ngrp = nwin * 16;
    if (tid < nv) {
        uint32_t t = 0;
        for (uint32_t g = 0; g < ngrp; ++g) t += s_grp[g][tid];
        s_vstart[tid] = t;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t pos = 0;
        for (uint32_t v = 0; v < nv; ++v) {
            const uint32_t t = s_vstart[v];
            s_vstart[v] = pos;
            pos += t;
        }
        counts[0] = pos;
        s_n = pos;
    }
    __syncthreads();
    if (tid < nv) {
        uint32_t pos = s_vstart[tid];
        for (uint32_t g = 0; g < ngrp; ++g) {
            const uint32_t c = s_grp[g][tid];
            s_grp[g][tid] = pos;
            pos += c;
        }
    }
    __syncthreads();
    // 4. placement and map segments, every slot independent
#pragma unroll 4
    for (uint64_t i = tid; i < nslots; i += 1024) {
        const int v = g_vis[i];
        if (v < 0) continue;
        const uint32_t pos = s_grp[(uint32_t)(i / kSelWin) * 16 + (uint32_t)((i % kSelWin) >> 10)][v] + g_rank[i];
        const uint64_t sk = pairs[2 * i];
        uint64_t s0 = 0, c = 0;
        if (sk < 10000) {
            s0 = map_off[sk];
            c = map_off[sk + 1] > map_off[sk] ? map_off[sk + 1] - map_off[sk] : 0;
        }
        sel[pos] = sk;
        src[pos] = s0;
        cnt[pos] = (uint32_t)c;
    }
    __syncthreads();
    // 5. dst = exclusive prefix of cnt in selection order
    const uint64_t n = s_n;
    uint64_t carry = 0;
    for (uint64_t b = 0; b < n; b += blockDim.x) {
        const uint64_t i = b + tid;
        const uint64_t c = i < n ? cnt[i] : 0;
        uint64_t x = c;  // inclusive scan in the wave, then across the 16 waves
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) s_wsum[wv] = x;
        __syncthreads();
        uint64_t before = carry;
        for (uint32_t w = 0; w < wv; ++w) before += s_wsum[w];
        if (i < n) dst[i] = before + x - c;
        uint64_t total = 0;
        for (uint32_t w = 0; w < 16; ++w) total += s_wsum[w];
        carry += total;
        __syncthreads();
    }
    if (tid == 0) counts[1] = carry;
}

// thread per (query q, supplier s): the abort for a stock lookup that produced no tuple is already
// in abort_flag (launch_revisit_segments); the last entry's stock row, at q's read id, gives
// (w, i, quantity, ytd, order_cnt, remote_cnt) and the item key
__global__ void q2_reduce(const stage_probe_out_dev *__restrict__ slast, const uint64_t *__restrict__ skeys,
                          const uint64_t *__restrict__ dst, const uint32_t *__restrict__ cnt,
                          const uint64_t *__restrict__ supp, const uint8_t *__restrict__ sheap, uint32_t shstride,
                          uint32_t skpad, const uint64_t *__restrict__ counts, uint32_t nq,
                          stage_q2_rec *__restrict__ out, uint64_t *__restrict__ ikeys) {
    const uint32_t n = (uint32_t)counts[0];
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;  // q * n + s
    if (g >= n * nq) return;
    const uint32_t s = g % n;
    const uint64_t kb = dst[s];
    const uint32_t c = cnt[s];
    stage_q2_rec r;
    memset(&r, 0, sizeof(r));
    r.supp_key = (int64_t)supp[s];
    if (c) {  // stock_0 / stock_1 of the last lookup (a supplier without stocks keeps zeros)
        const uint64_t klast = kb + c - 1;
        r.s_w_id = (int64_t)skeys[2 * klast];
        r.s_i_id = (int64_t)skeys[2 * klast + 1];
        if (produced(slast[g].w[0] & 0xFF)) {
            const uint8_t *row = sheap + (uint64_t)slast[g].w[6] * shstride + skpad;
            r.s_quantity = ld_i32(row);
            r.s_ytd = ld_i32(row + 4);
            r.s_order_cnt = ld_i32(row + 8);
            r.s_remote_cnt = ld_i32(row + 12);
        }
    }
    out[g] = r;
    ikeys[g] = (uint64_t)r.s_i_id;
}

// item outcome: no tuple aborts; I_DATA up to its first NUL containing 'b' skips; else a
// quantity below 10 marks the update
// ... and each record straight into the caller's page-locked records (host_out, row pitch
// max_out; null: the records stay in `out` on the device)
__global__ void q2_finish(const stage_probe_out_dev *__restrict__ iout, const uint8_t *__restrict__ iheap,
                          uint32_t ihstride, uint32_t ikpad, const uint64_t *__restrict__ counts, uint32_t nq,
                          stage_q2_rec *__restrict__ out, int32_t *__restrict__ abort_flag,
                          stage_q2_rec *__restrict__ host_out, uint64_t max_out) {
    const uint32_t n = (uint32_t)counts[0];
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;  // q * n + supplier
    if (s >= n * nq) return;
    const uint32_t st = iout[s].w[0] & 0xFF;
    stage_q2_rec r = out[s];
    if (!produced(st)) {
        atomicOr(abort_flag + s / n, 1);
    } else {
        // I_DATA's 64 bytes in 16 word loads issued together (4-B aligned), scanned in registers
        const uint32_t *d = reinterpret_cast<const uint32_t *>(iheap + (uint64_t)iout[s].w[6] * ihstride + ikpad +
                                                               kIDataOff);
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = d[k];
        uint8_t has_b = 0;
        bool end = false;
#pragma unroll
        for (int c = 0; c < 64; ++c) {
            const uint8_t ch = (uint8_t)(w[c >> 2] >> (8 * (c & 3)));
            end |= ch == 0;
            has_b |= !end && ch == 'b';
        }
        r.item_has_b = has_b;
        r.update = !has_b && r.s_quantity < 10;
        out[s] = r;
    }
    if (host_out && s % n < max_out) host_out[(uint64_t)(s / n) * max_out + s % n] = r;
}

// SUPPLIER scan with scan_sz -1 (TableScanExecutor::ScanLeafNode, executor.h:580-612): every
// slot of every leaf in leaf order, slots in slot order, raw records without a visibility
// test -- one lane per slot; pairs[i] = {SU_SUPPKEY, SU_NATIONKEY} of slot i, or ~0 for a slot
// holding no record
__global__ void q2_dump_leaves(DevTable t, uint32_t kpad, uint64_t *__restrict__ pairs) {
    const uint64_t n = (uint64_t)t.nleaves * t.cap;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const SlotInfo si = t.slot[i];
        uint64_t k = ~0ull, nat = ~0ull;
        if (si.meta != 0) {
            const uint8_t *row = t.heap + (uint64_t)si.image * t.hstride;
            k = *reinterpret_cast<const uint64_t *>(row);
            nat = *reinterpret_cast<const uint64_t *>(row + kpad);
        }
        pairs[2 * i] = k;
        pairs[2 * i + 1] = nat;
    }
}

// TableScanExecutor rows of one scan from `start` (device scan) into the table's scratch: the
// returned pointer is the first row, the row count (u32) 8 bytes before it
const uint8_t *scan_rows(stage_table *t, uint64_t start, uint32_t scan_size, hipStream_t s) {
    const DevTable &v = t->dev.view;
    const uint64_t rows = (uint64_t)scan_size * v.stride;
    uint8_t *buf = scratch_bytes(t->dev, 64 + rows);
    auto *key = (uint64_t *)buf;
    auto *cnt = (uint32_t *)(buf + 56);  // 8 bytes before the rows
    q2_set_u64<<<1, 1, 0, s>>>(key, start);  // no host buffer outlives the call
    hip_check(launch_scan(v, key, nullptr, 1, scan_size, cnt, buf + 64, s, t->scan_tune), "scan");
    return buf + 64;
}

}  // namespace
}  // namespace stage

// nq transactions at read ids rq[0..nq): out[q * max_out + k], aborted[q]; commit only for nq == 1
static int q2_run(stage_table *region, stage_table *nation, stage_table *supplier, stage_table *item,
                  stage_table *stock, const uint32_t *map_off, const uint64_t *d_map_keys, int32_t target_region,
                  const uint32_t *rq, uint32_t nq, uint32_t commit_id, stage_q2_rec *out, uint64_t max_out,
                  uint64_t *n_out, int32_t *aborted, void *stream) {
    for (stage_table *t : {region, nation, supplier, item, stock}) {
        int rc = need_synced(t);
        if (rc) return rc;
    }
    if (!map_off || !d_map_keys || !n_out || !aborted || (max_out && !out))
        return fail(STAGE_E_ARG, "null argument");
    if (target_region < 0 || target_region > 4) return fail(STAGE_E_ARG, "target_region must be 0..4");
    for (stage_table *t : {region, nation, supplier, item})
        if (facts(t).params().key_width != 8) return fail(STAGE_E_ARG, "REGION/NATION/SUPPLIER/ITEM keys are 8 bytes");
    if (facts(stock).params().key_width != 16) return fail(STAGE_E_ARG, "STOCK keys are {w, i}: 16 bytes");
    if (facts(region).params().payload_size < 55 || facts(nation).params().payload_size < 8 ||
        facts(supplier).params().payload_size < 8 || facts(item).params().payload_size < stage::kIDataOff + 64 ||
        facts(stock).params().payload_size < 16)
        return fail(STAGE_E_ARG, "payloads too short for the Q2 columns");
    for (stage_table *t : {region, nation, supplier, item})
        if (t->dev.device != stock->dev.device) return fail(STAGE_E_ARG, "tables on different devices");
    return guarded([&] {
        using namespace stage;
        hip_check(hipSetDevice(stock->dev.device), "hipSetDevice");
        hipStream_t s = pick(stock, stream);
        // STAGE_Q2_TRACE=1: host wall time of each phase on stderr
        static const bool trace = std::getenv("STAGE_Q2_TRACE") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        auto lap = [&](const char *what) {
            if (trace)
                std::fprintf(stderr, "[q2] %s %.1f us\n", what,
                             std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        };
        *n_out = 0;
        for (uint32_t q = 0; q < nq; ++q) aborted[q] = 0;
        const DevTable &pv = supplier->dev.view, &sv = stock->dev.view, &iv = item->dev.view;
        const uint64_t nslots = (uint64_t)pv.nleaves * pv.cap;
        if (nslots > (uint64_t)kSelWin * kSelMaxWin)
            return fail(STAGE_E_UNSUPPORTED, "SUPPLIER has more slots than q2_select's windows hold (131072)");
        // upper bounds (buffer sizes, grids): every SUPPLIER slot visited, every map entry looked up
        constexpr uint32_t kMapKeys = 10000;
        uint64_t m_max = 0;
        for (uint32_t k = 0; k < kMapKeys; ++k) m_max += map_off[k + 1] > map_off[k] ? map_off[k + 1] - map_off[k] : 0;
        const uint64_t n_max = std::max<uint64_t>(nslots, 1);
        // launch shapes from the previous call's counts (the visited set depends on the data only)
        const uint64_t n_hint = stock->q2_hint[0] ? std::min(stock->q2_hint[0], n_max) : n_max;
        const uint64_t m_hint = stock->q2_hint[1] ? std::min(stock->q2_hint[1], std::max<uint64_t>(m_max, 1)) : m_max;
        // pinned call staging mirrored at the head of the device scratch: [map_off][read ids]
        // [aborted] go down in one copy; [counts][aborted] come back in one copy
        auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
        const uint64_t q_map = 0, q_rq = q_map + al((kMapKeys + 1) * 4ull), q_cn = q_rq + al(nq * 4ull),
                       q_ab = q_cn + 16, q_end = q_ab + al(nq * 4ull);
        uint8_t *pq = pinned_bytes(stock->dev, q_end, 2);
        std::memcpy(pq + q_map, map_off, (kMapKeys + 1) * 4ull);
        std::memcpy(pq + q_rq, rq, nq * 4ull);
        std::memset(pq + q_cn, 0, 16 + nq * 4ull);
        uint64_t off = 0;
        auto take = [&](uint64_t bytes) {
            const uint64_t o = off;
            off += al(bytes);
            return o;
        };
        const uint64_t o_mir = take(q_end), o_pairs = take(n_max * 16), o_sel = take(n_max * 8),
                       o_src = take(n_max * 8), o_cnt = take(n_max * 4), o_dst = take(n_max * 8),
                       o_keys = take(std::max<uint64_t>(m_max, 1) * 16), o_sbase = take(std::max<uint64_t>(m_max, 1) * 32),
                       o_slast = take(n_max * 32 * nq), o_ik = take(n_max * 8 * nq), o_iout = take(n_max * 32 * nq),
                       o_ibase = take(n_max * 32), o_rec = take(n_max * nq * sizeof(stage_q2_rec)),
                       o_vis = take(n_max), o_rank = take(n_max * 2);
        // the SUPPLIER table's scratch: REGION's and NATION's hold their scan rows (scan_rows)
        uint8_t *buf = scratch_bytes(supplier->dev, off), *mir = buf + o_mir;
        auto *d_map = (const uint32_t *)(mir + q_map);
        auto *d_rq = (const uint32_t *)(mir + q_rq);
        auto *d_counts = (uint64_t *)(mir + q_cn);
        auto *d_ab = (int32_t *)(mir + q_ab);
        auto *d_pairs = (uint64_t *)(buf + o_pairs), *d_sel = (uint64_t *)(buf + o_sel);
        auto *d_src = (uint64_t *)(buf + o_src), *d_dst = (uint64_t *)(buf + o_dst);
        auto *d_cnt = (uint32_t *)(buf + o_cnt);
        auto *d_keys = (uint64_t *)(buf + o_keys), *d_ik = (uint64_t *)(buf + o_ik);
        auto *d_iout = (stage_probe_out_dev *)(buf + o_iout), *d_slast = (stage_probe_out_dev *)(buf + o_slast);
        auto *d_sbase = (stage_probe_out_dev *)(buf + o_sbase), *d_ibase = (stage_probe_out_dev *)(buf + o_ibase);
        auto *d_rec = (stage_q2_rec *)(buf + o_rec);
        hip_check(hipMemcpyAsync(mir, pq, q_end, hipMemcpyHostToDevice, s), "h2d");
        // 1. REGION / NATION scans on their tables' own streams beside the SUPPLIER dump on s
        // (forked from and joined back into s): three short dependent chains side by side
        hipEvent_t *ev = stock->dev.call_ev;
        for (int k = 0; k < 3; ++k)
            if (!ev[k]) hip_check(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), "call event");
        hipStream_t rs_s = region->dev.stream ? region->dev.stream : s, ns_s = nation->dev.stream ? nation->dev.stream : s;
        hip_check(hipEventRecord(ev[0], s), "fork");
        hip_check(hipStreamWaitEvent(rs_s, ev[0], 0), "fork");
        hip_check(hipStreamWaitEvent(ns_s, ev[0], 0), "fork");
        const uint8_t *regs = scan_rows(region, 0, kRegionScan, rs_s);
        const uint8_t *nats = scan_rows(nation, 0, kNationScan, ns_s);
        hip_check(hipEventRecord(ev[1], rs_s), "join");
        hip_check(hipEventRecord(ev[2], ns_s), "join");
        q2_dump_leaves<<<(unsigned)std::min<uint64_t>((nslots + 255) / 256, 4096), 256, 0, s>>>(
            pv, facts(supplier).key_pad(), d_pairs);
        hip_check(hipGetLastError(), "dump leaves");
        hip_check(hipStreamWaitEvent(s, ev[1], 0), "join");
        hip_check(hipStreamWaitEvent(s, ev[2], 0), "join");
        // 2. the selection and the map segments, on the device
        char tname[16] = {0};
        std::strncpy(tname, kRegions[target_region], 15);
        uint64_t name0, name1;
        std::memcpy(&name0, tname, 8);
        std::memcpy(&name1, tname + 8, 8);
        q2_select<<<1, 1024, 0, s>>>(regs, region->dev.view.stride, nats, nation->dev.view.stride, name0, name1, d_pairs,
                                     nslots, d_map, (int8_t *)(buf + o_vis), (uint16_t *)(buf + o_rank), d_sel, d_src,
                                     d_cnt, d_dst, d_counts);
        hip_check(hipGetLastError(), "select");
        lap("selection enqueued");
        // 3. every visited supplier's STOCK keys, one probe of them all (the counts on the device)
        q2_gather<<<(unsigned)std::max<uint64_t>(std::min<uint64_t>(n_hint, 4096), 1), 256, 0, s>>>(
            d_map_keys, d_src, d_dst, d_cnt, d_counts, m_max, d_keys);
        // every query of the batch looks up the same STOCK keys (the visited suppliers and their
        // supp_stock_map do not depend on the read id): each key is probed once, with no read id
        // (the hit slot does not depend on it), and its visibility evaluated at every query's read
        // id inside the per-supplier fold (launch_revisit_segments: the aborts and each
        // supplier's last stock, per query)
        if (m_max)
            hip_check(launch_probe(sv, d_keys, nullptr, nullptr, nullptr, m_max, d_sbase, nullptr, s, stock->tune,
                                   d_counts + 1, m_hint),
                      "stock probe");
        if (m_max)
            hip_check(launch_revisit_segments(sv, d_sbase, m_max, d_dst, d_cnt, (uint32_t)n_max, d_rq, nq, d_slast, d_ab, s,
                                              d_counts + 1, d_counts),
                      "stock read ids");
        q2_reduce<<<(unsigned)((n_max * nq + 255) / 256), 256, 0, s>>>(d_slast, d_keys, d_dst, d_cnt, d_sel, sv.heap,
                                                                       sv.hstride, facts(stock).key_pad(), d_counts,
                                                                       nq, d_rec, d_ik);
        // 4. item lookups of the last stocks (the same keys in every query: probed once, as above),
        // the I_DATA filter, the records into `out`
        hip_check(launch_probe(iv, d_ik, nullptr, nullptr, nullptr, n_max, d_ibase, nullptr, s, item->tune, d_counts,
                               n_hint),
                  "item probe");
        hip_check(launch_revisit(iv, d_ibase, n_max, d_rq, nq, nullptr, d_iout, s, d_counts), "item read ids");
        // `out` in page-locked memory (stage_host_alloc, stage.pinned_empty): the finishing kernel
        // writes the records into it directly; otherwise they are copied once the count is known
        stage_q2_rec *host_out = nullptr;
        static const bool copy_out = [] {
            const char *e = std::getenv("STAGE_Q2_OUT");  // "copy": records copied after the batch (A/B)
            return e && std::strcmp(e, "copy") == 0;
        }();
        if (out && max_out && !copy_out) {  // page-locked memory has a device view; pageable memory has none
            void *dp = nullptr;
            if (hipHostGetDevicePointer(&dp, out, 0) == hipSuccess && dp) host_out = (stage_q2_rec *)dp;
            (void)hipGetLastError();  // a pageable pointer is not an error here
        }
        if (trace) std::fprintf(stderr, "[q2] out %s\n", host_out ? "page-locked: written by q2_finish" : "pageable: copied");
        q2_finish<<<(unsigned)((n_max * nq + 255) / 256), 256, 0, s>>>(d_iout, iv.heap, iv.hstride, facts(item).key_pad(),
                                                                       d_counts, nq, d_rec, d_ab, host_out, max_out);
        hip_check(hipGetLastError(), "q2 kernels");
        hip_check(hipMemcpyAsync(pq + q_cn, d_counts, 16 + nq * 4ull, hipMemcpyDeviceToHost, s), "d2h");
        lap("enqueued");
        hip_check(hipStreamSynchronize(s), "q2 sync");  // the batch's one synchronisation
        lap("results back");
        uint64_t cn[2];
        std::memcpy(cn, pq + q_cn, 16);
        std::memcpy(aborted, pq + q_ab, 4ull * nq);
        const uint64_t n = cn[0];
        if (n > n_max || cn[1] > m_max) throw std::runtime_error("q2: device counts out of range");
        stock->q2_hint[0] = n;
        stock->q2_hint[1] = cn[1];
        *n_out = n;
        if (n == 0) {
            for (uint32_t q = 0; q < nq; ++q) aborted[q] = 0;
            return STAGE_OK;
        }
        std::vector<stage_q2_rec> recs_buf;
        const stage_q2_rec *recs = host_out ? out : nullptr;
        if (!host_out) {  // a pageable (or no) `out`: the records come back now
            recs_buf.resize(n * nq);
            hip_check(hipMemcpy(recs_buf.data(), d_rec, n * nq * sizeof(stage_q2_rec), hipMemcpyDeviceToHost), "d2h");
            recs = recs_buf.data();
        }
        auto rec = [&](uint32_t q, uint64_t k) -> stage_q2_rec & {
            return host_out ? out[(uint64_t)q * max_out + k] : recs_buf[(uint64_t)q * n + k];
        };
        const uint32_t read_id = rq[0];
        // 5. the transaction's stock updates, through the device write path
        if (nq == 1 && commit_id && !*aborted) {
            std::vector<uint64_t> uk;
            std::vector<int32_t> ud;
            std::vector<uint32_t> ui;
            for (uint32_t k = 0; k < n && (!host_out || k < max_out); ++k)
                if (rec(0, k).update) {
                    uk.push_back((uint64_t)rec(0, k).s_w_id);
                    uk.push_back((uint64_t)rec(0, k).s_i_id);
                    ud.insert(ud.end(), {rec(0, k).s_quantity + 50, rec(0, k).s_ytd, rec(0, k).s_order_cnt,
                                         rec(0, k).s_remote_cnt});
                    ui.push_back(k);
                }
            const uint64_t nu = ui.size();
            if (nu) {
                uint64_t o2 = 0;
                auto take2 = [&](uint64_t bytes) {
                    const uint64_t o = o2;
                    o2 += al(bytes);
                    return o;
                };
                const uint64_t u_k = take2(nu * 16), u_d = take2(nu * 16), u_w = take2(nu * 4), u_c = take2(nu * 4),
                               u_rc = take2(nu);
                uint8_t *ub = scratch_bytes(item->dev, o2);
                std::vector<uint32_t> wid(nu, read_id), cid(nu, commit_id);
                hip_check(hipMemcpyAsync(ub + u_k, uk.data(), nu * 16, hipMemcpyHostToDevice, s), "h2d");
                hip_check(hipMemcpyAsync(ub + u_d, ud.data(), nu * 16, hipMemcpyHostToDevice, s), "h2d");
                hip_check(hipMemcpyAsync(ub + u_w, wid.data(), nu * 4, hipMemcpyHostToDevice, s), "h2d");
                hip_check(hipMemcpyAsync(ub + u_c, cid.data(), nu * 4, hipMemcpyHostToDevice, s), "h2d");
                uint64_t ok = 0;
                const int rc = stage_update_batch_device(stock, (const uint64_t *)(ub + u_k), nullptr, nu, 0,
                                                         ub + u_d, 16, (const uint32_t *)(ub + u_w),
                                                         (const uint32_t *)(ub + u_c), nullptr, ub + u_rc, &ok, s);
                if (rc) return rc;
                std::vector<uint8_t> rcs(nu);
                hip_check(hipMemcpyAsync(rcs.data(), ub + u_rc, nu, hipMemcpyDeviceToHost, s), "d2h");
                hip_check(hipStreamSynchronize(s), "update sync");
                for (uint64_t j = 0; j < nu; ++j) rec(0, ui[j]).update_rc = rcs[j];
            }
        }
        if (!host_out && out)
            for (uint32_t q = 0; q < nq; ++q)
                std::memcpy(out + (uint64_t)q * max_out, recs + (uint64_t)q * n,
                            std::min<uint64_t>(n, max_out) * sizeof(stage_q2_rec));
        lap("out copied");
        return STAGE_OK;
    });
}

extern "C" int stage_ch_query2(stage_table *region, stage_table *nation, stage_table *supplier, stage_table *item,
                               stage_table *stock, const uint32_t *map_off, const uint64_t *d_map_keys,
                               int32_t target_region, uint32_t read_id, uint32_t commit_id, stage_q2_rec *out,
                               uint64_t max_out, uint64_t *n_out, int32_t *aborted, void *stream) {
    return q2_run(region, nation, supplier, item, stock, map_off, d_map_keys, target_region, &read_id, 1, commit_id,
                  out, max_out, n_out, aborted, stream);
}

extern "C" int stage_ch_query2_batch(stage_table *region, stage_table *nation, stage_table *supplier,
                                     stage_table *item, stage_table *stock, const uint32_t *map_off,
                                     const uint64_t *d_map_keys, int32_t target_region, const uint32_t *read_ids,
                                     uint32_t nq, stage_q2_rec *out, uint64_t max_per_query, uint64_t *n_out,
                                     int32_t *aborted, void *stream) {
    if (nq == 0) return STAGE_OK;
    if (!read_ids || nq > 4096) return fail(STAGE_E_ARG, "read_ids: 1..4096 queries");
    return q2_run(region, nation, supplier, item, stock, map_off, d_map_keys, target_region, read_ids, nq, 0, out,
                  max_per_query, n_out, aborted, stream);
}
