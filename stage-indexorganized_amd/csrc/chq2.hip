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
// Here REGION / NATION run as device scans; four short kernels (q2_sel_*) read the SUPPLIER leaves
// slot by slot and select -- the region named regions[target], its nations, their suppliers in
// visiting order -- and lay out each visited supplier's supp_stock_map segment; the
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
#include "visibility.hpp"

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

// blocks copy the visited suppliers' map entries (2 words each) to their segments; counts[0] =
// the number of visited suppliers (q2_sel_start); nothing is written past m_cap keys (the host
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

// RunQuery2's selection (tpcc_new_order.cpp:650-797) on the device, from the REGION / NATION scan
// rows and the SUPPLIER leaves (TableScanExecutor::ScanLeafNode with scan_sz -1, executor.h:
// 580-612: every slot of every leaf in leaf order, slots in slot order, raw records):
//   visits   = for each REGION row named the target (scan order), each NATION row of that region
//              (scan order); a nation is visited at most once (one region key per nation, region
//              keys unique), so at most kNationScan visits;
//   sel      = every SUPPLIER record of each visited nation, visit by visit, in slot order: a
//              stable counting sort by visit over 64-slot chunks --
//                q2_sel_count  (a wave per chunk) the visits, each slot's visit, its rank and its
//                              map entries' offset among its chunk's slots of that visit, the
//                              chunk's supplier and entry counts per visit (stored
//                              visit-major: a visit's chunks side by side);
//                q2_sel_start  (one block) each (visit, chunk)'s supplier and entry starts:
//                              visit, then chunk order;
//                q2_sel_place  (a lane per slot) sel[start + rank], the supplier's map segment
//                              (src, cnt) and its first STOCK key (dst = entry start + offset);
//   counts   = {suppliers, stock keys}.
// Every block derives the visits itself from the (L2-resident) scan rows, so no launch is spent
// on them; no loop waits on one global load per iteration.
constexpr int kVisits = kNationScan;
constexpr uint32_t kDirect = 1024;  // nation keys below this: a direct LDS map, the rest searched

struct VisitMap {  // nation key -> visit (LDS)
    int8_t dir[kDirect];
    int64_t big_key[kVisits];
    int32_t big_val[kVisits];
    uint32_t nbig, nv;
};

// the visit map of the target region, built by every block (blockDim.x >= 64)
__device__ void build_visits(VisitMap &vm, const uint8_t *regs, uint32_t rs, const uint8_t *nats, uint32_t ns,
                             uint64_t name0, uint64_t name1, uint64_t mask0, uint64_t mask1, uint8_t *s_rmatch,
                             uint8_t *s_flag) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t nreg = min(*reinterpret_cast<const uint32_t *>(regs - 8), (uint32_t)kRegionScan);
    const uint32_t nnat = min(*reinterpret_cast<const uint32_t *>(nats - 8), (uint32_t)kNationScan);
    for (uint32_t i = tid; i < kDirect; i += blockDim.x) vm.dir[i] = -1;
    if (tid == 0) vm.nbig = 0;
    // R_NAME == regions[target]: the bytes up to and including the target's NUL (< 16)
    if (tid < nreg) {
        const uint64_t *nm = reinterpret_cast<const uint64_t *>(regs + (uint64_t)tid * rs + 8);
        s_rmatch[tid] = ((nm[0] ^ name0) & mask0) == 0 && ((nm[1] ^ name1) & mask1) == 0;
    }
    __syncthreads();
    const uint32_t nf = nreg * nnat;  // flag f = (region row f / nnat, nation row f % nnat), visit order
    for (uint32_t f = tid; f < nf; f += blockDim.x) {
        const uint32_t r = f / nnat, a = f % nnat;
        s_flag[f] = s_rmatch[r] && *reinterpret_cast<const int64_t *>(nats + (uint64_t)a * ns + 8) ==
                                       *reinterpret_cast<const int64_t *>(regs + (uint64_t)r * rs);
    }
    __syncthreads();
    if (tid < 64) {  // wave 0 numbers the flagged (region, nation) pairs in order
        uint32_t base = 0;
        for (uint32_t f0 = 0; f0 < nf; f0 += 64) {
            const uint32_t f = f0 + lane;
            const bool fl = f < nf && s_flag[f];
            const uint64_t b = ballot(fl);
            if (fl) {
                const uint32_t idx = base + (uint32_t)__builtin_popcountll(b & ((1ull << lane) - 1));
                const int64_t nk = *reinterpret_cast<const int64_t *>(nats + (uint64_t)(f % nnat) * ns);
                if (idx < (uint32_t)kVisits) {
                    if (nk >= 0 && nk < (int64_t)kDirect) {
                        vm.dir[nk] = (int8_t)idx;
                    } else {
                        const uint32_t k = atomicAdd(&vm.nbig, 1u);
                        vm.big_key[k] = nk;
                        vm.big_val[k] = (int32_t)idx;
                    }
                }
            }
            base += (uint32_t)__builtin_popcountll(b);
        }
        if (lane == 0) vm.nv = min(base, (uint32_t)kVisits);
    }
    __syncthreads();
}

__device__ __forceinline__ int visit_of(const VisitMap &vm, uint64_t nat) {
    if ((int64_t)nat >= 0 && (int64_t)nat < (int64_t)kDirect) return vm.dir[nat];
    for (uint32_t k = 0; k < vm.nbig; ++k)
        if (vm.big_key[k] == (int64_t)nat) return vm.big_val[k];
    return -1;
}

// a wave per 64-slot chunk of the SUPPLIER leaves (blocks of 4 waves)
__global__ __launch_bounds__(256) void q2_sel_count(const uint8_t *__restrict__ regs, uint32_t rs,
                                                    const uint8_t *__restrict__ nats, uint32_t ns, uint64_t name0,
                                                    uint64_t name1, uint64_t mask0, uint64_t mask1, DevTable t,
                                                    uint32_t kpad, uint64_t nchunks, const uint32_t *__restrict__ map_off,
                                                    int8_t *__restrict__ g_vis, uint8_t *__restrict__ g_rank,
                                                    uint32_t *__restrict__ g_koff, uint64_t *__restrict__ g_key,
                                                    uint32_t *__restrict__ ccnt, uint32_t *__restrict__ kcnt,
                                                    uint32_t *__restrict__ g_nv) {
    __shared__ VisitMap vm;
    __shared__ uint8_t s_rmatch[kRegionScan];
    __shared__ uint8_t s_flag[kRegionScan * kNationScan];
    __shared__ uint32_t s_cnt[4][kVisits], s_kcnt[4][kVisits];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t c = (uint64_t)blockIdx.x * 4 + wv;
    // the slot's record first -- slot word, key, nation key, map segment: none of it depends on
    // the visits, so these dependent loads overlap build_visits' own (the scan rows)
    const uint64_t i = c * 64 + lane;
    uint64_t key = ~0ull, nat = 0;
    uint32_t ma = 0, mb = 0;
    if (c < nchunks) {
        const SlotInfo si = t.slot[i];
        if (si.meta != 0) {
            const uint8_t *row = t.heap + (uint64_t)si.image * t.hstride;
            key = *reinterpret_cast<const uint64_t *>(row);
            nat = *reinterpret_cast<const uint64_t *>(row + kpad);
        }
        if (key < 10000) ma = map_off[key], mb = map_off[key + 1];
    }
    build_visits(vm, regs, rs, nats, ns, name0, name1, mask0, mask1, s_rmatch, s_flag);
    if (blockIdx.x == 0 && threadIdx.x == 0) *g_nv = vm.nv;
    if (c >= nchunks) return;
    for (uint32_t v = lane; v < (uint32_t)kVisits; v += 64) s_cnt[wv][v] = 0, s_kcnt[wv][v] = 0;
    const int v = key == ~0ull ? -1 : visit_of(vm, nat);
    // the supplier's supp_stock_map entries (keys below 10000)
    const uint32_t mc = v >= 0 && key < 10000 && mb > ma ? mb - ma : 0;
    // per visit present in the chunk: each slot's rank and its entries' offset among the
    // chunk's slots of that visit, the visit's supplier and entry counts
    uint32_t rank = 0, koff = 0;
    uint64_t todo = ballot(v >= 0);
    while (todo) {
        const int vl = (int)rl32((uint32_t)v, (int)__builtin_ctzll(todo));
        const bool in = v == vl;
        const uint64_t mm = ballot(in);
        const uint32_t x = in ? mc : 0u;
        uint32_t y = x;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t z = __shfl_up(y, o, 64);
            if (lane >= (uint32_t)o) y += z;
        }
        if (in) {
            rank = (uint32_t)__builtin_popcountll(mm & ((1ull << lane) - 1));
            koff = y - x;
        }
        const uint32_t ktot = rl32(y, 63);
        if (lane == 0) {
            s_cnt[wv][vl] = (uint32_t)__builtin_popcountll(mm);
            s_kcnt[wv][vl] = ktot;
        }
        todo &= ~mm;
    }
    g_vis[i] = (int8_t)v;
    g_rank[i] = (uint8_t)rank;
    g_koff[i] = koff;
    g_key[i] = key;
    for (uint32_t w = lane; w < vm.nv; w += 64) {  // visit-major: q2_sel_start reads a visit's chunks coalesced
        ccnt[(uint64_t)w * nchunks + c] = s_cnt[wv][w];
        kcnt[(uint64_t)w * nchunks + c] = s_kcnt[wv][w];
    }
}

// one block, after q2_sel_count: the (visit, chunk) supplier counts ccnt and entry counts kcnt
// (visit-major) -> their starts, in place (visit, then chunk order); counts = {suppliers, stock
// keys}.  A wave per visit; lane l takes chunks l, l + 64, ... so each load and store of the
// wave is 64 consecutive words; 16 chunks per lane in flight at once.  (Round 6: a lane per
// contiguous run of chunks in the chunk-major layout made every load touch 64 lines -- ~10 K
// line requests through the block's one CU, ~13 µs of the chain.)
constexpr uint32_t kSelBatch = 16;
__device__ __forceinline__ void load_batch(const uint32_t *__restrict__ ccnt, const uint32_t *__restrict__ kcnt,
                                           uint64_t row, uint64_t nchunks, uint64_t c0, uint32_t lane,
                                           uint32_t (&x0)[kSelBatch], uint32_t (&x1)[kSelBatch]) {
#pragma unroll
    for (uint32_t k = 0; k < kSelBatch; ++k) {  // unconditional loads (an index past the end re-reads chunk 0)
        const uint64_t c = c0 + k * 64 + lane;
        const uint64_t at = row + (c < nchunks ? c : 0);
        x0[k] = ccnt[at];
        x1[k] = kcnt[at];
    }
#pragma unroll
    for (uint32_t k = 0; k < kSelBatch; ++k) {
        const bool in = c0 + k * 64 + lane < nchunks;
        x0[k] = in ? x0[k] : 0u;
        x1[k] = in ? x1[k] : 0u;
    }
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t y, uint32_t lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t z = __shfl_up(y, o, 64);
        if (lane >= (uint32_t)o) y += z;
    }
    return y;
}

__global__ __launch_bounds__(1024) void q2_sel_start(uint32_t *__restrict__ ccnt, uint32_t *__restrict__ kcnt,
                                                     uint64_t nchunks, const uint32_t *__restrict__ g_nv,
                                                     uint64_t *__restrict__ counts) {
    __shared__ uint32_t s_tot[2][kVisits];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    const uint32_t nv = *g_nv;
    for (uint32_t v = wv; v < nv; v += nw) {  // the visit's totals
        uint32_t t0 = 0, t1 = 0;
        for (uint64_t c0 = 0; c0 < nchunks; c0 += 64 * kSelBatch) {
            uint32_t x0[kSelBatch], x1[kSelBatch];
            load_batch(ccnt, kcnt, (uint64_t)v * nchunks, nchunks, c0, lane, x0, x1);
#pragma unroll
            for (uint32_t k = 0; k < kSelBatch; ++k) t0 += x0[k], t1 += x1[k];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t0 += __shfl_xor(t0, o, 64), t1 += __shfl_xor(t1, o, 64);
        if (lane == 0) s_tot[0][v] = t0, s_tot[1][v] = t1;
    }
    __syncthreads();
    if (tid < 2) {
        uint32_t pos = 0;
        for (uint32_t v = 0; v < nv; ++v) {
            const uint32_t t = s_tot[tid][v];
            s_tot[tid][v] = pos;
            pos += t;
        }
        counts[tid] = pos;
    }
    __syncthreads();
    for (uint32_t v = wv; v < nv; v += nw) {  // exclusive scan over the chunks, in place
        uint32_t p0 = s_tot[0][v], p1 = s_tot[1][v];  // the start of the next 64 chunks
        const uint64_t row = (uint64_t)v * nchunks;
        for (uint64_t c0 = 0; c0 < nchunks; c0 += 64 * kSelBatch) {
            uint32_t x0[kSelBatch], x1[kSelBatch];
            load_batch(ccnt, kcnt, row, nchunks, c0, lane, x0, x1);
#pragma unroll
            for (uint32_t k = 0; k < kSelBatch; ++k) {
                const uint64_t c = c0 + k * 64 + lane;
                const uint32_t y0 = wave_incl_scan(x0[k], lane), y1 = wave_incl_scan(x1[k], lane);
                if (c < nchunks) ccnt[row + c] = p0 + y0 - x0[k], kcnt[row + c] = p1 + y1 - x1[k];
                p0 += rl32(y0, 63);
                p1 += rl32(y1, 63);
            }
        }
    }
}

// a lane per slot: each selected supplier at its place, with its supp_stock_map segment (src,
// cnt) and the segment's offset among all looked-up STOCK keys (dst)
__global__ void q2_sel_place(const uint32_t *__restrict__ ccnt, const uint32_t *__restrict__ kcnt, uint64_t nslots,
                             const int8_t *__restrict__ g_vis, const uint8_t *__restrict__ g_rank,
                             const uint32_t *__restrict__ g_koff, const uint64_t *__restrict__ g_key,
                             const uint32_t *__restrict__ map_off, uint64_t *__restrict__ sel,
                             uint64_t *__restrict__ src, uint32_t *__restrict__ cnt, uint64_t *__restrict__ dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nslots) return;
    const int v = g_vis[i];
    if (v < 0) return;
    const uint64_t g = (uint64_t)v * (nslots >> 6) + (i >> 6);  // visit-major (q2_sel_start)
    const uint32_t pos = ccnt[g] + g_rank[i];
    const uint64_t sk = g_key[i];
    uint64_t s0 = 0, c = 0;
    if (sk < 10000) {
        const uint32_t a = map_off[sk], b = map_off[sk + 1];
        s0 = a;
        c = b > a ? b - a : 0;
    }
    sel[pos] = sk;
    src[pos] = s0;
    cnt[pos] = (uint32_t)c;
    dst[pos] = (uint64_t)kcnt[g] + g_koff[i];
}

// q2_sel_start + q2_sel_place + q2_gather in one launch, for SUPPLIER tables of at most
// kPlaceChunks 64-slot chunks.  A block of 16 waves per 4 chunks (sel_count's chunks of a block):
//   1. per visit, a wave sums the (visit, chunk) counts of every chunk and of the chunks before
//      the block's first (coalesced loads, L2-resident: ~26 KB per block at 256 chunks and 13
//      visits) -- one load round when the visits fit the 16 waves -- and keeps the block's own
//      chunks' counts in LDS; the visit totals are scanned in LDS (block 0 writes counts);
//   2. a thread per slot of the 4 chunks places its supplier as q2_sel_place and lists it;
//   3. the block's listed suppliers' map segments are copied as q2_gather, a wave per supplier,
//      each segment's loads issued together (up to 256 entries of 16 B per round).
// Removes two launches and the one-block scan from the chain (round 6).
constexpr uint64_t kPlaceChunks = 1024;
__global__ __launch_bounds__(1024) void q2_place(const uint32_t *__restrict__ ccnt, const uint32_t *__restrict__ kcnt,
                                                 uint64_t nchunks, const uint32_t *__restrict__ g_nv,
                                                 const int8_t *__restrict__ g_vis, const uint8_t *__restrict__ g_rank,
                                                 const uint32_t *__restrict__ g_koff, const uint64_t *__restrict__ g_key,
                                                 const uint32_t *__restrict__ map_off, const uint64_t *__restrict__ map_keys,
                                                 uint64_t m_cap, uint64_t *__restrict__ sel, uint64_t *__restrict__ src,
                                                 uint32_t *__restrict__ cnt, uint64_t *__restrict__ dst,
                                                 uint64_t *__restrict__ counts, uint64_t *__restrict__ keys) {
    __shared__ uint32_t s_base[2][kVisits];  // visit start + the counts of chunks before the block's first
    __shared__ uint32_t s_tot[2][kVisits];
    __shared__ uint32_t s_loc[2][4][kVisits];  // the block's own chunks' counts
    __shared__ uint64_t s_a[256], s_d[256];    // listed suppliers: map segment start, first STOCK key
    __shared__ uint32_t s_m[256], s_n;         // ... entry count; list length
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    const uint64_t c_first = (uint64_t)blockIdx.x * 4;
    // the slot's selection (threads 0..255: the block's 4 chunks) first, its map segment next:
    // independent of the counts, so these loads overlap the count pass below
    const bool slot_thread = tid < 256 && c_first + (tid >> 6) < nchunks;
    const uint64_t i = (c_first + (tid >> 6)) * 64 + lane;
    int v_i = -1;
    uint32_t rank_i = 0, koff_i = 0, lo_i = 0, hi_i = 0;
    uint64_t key_i = ~0ull;
    if (slot_thread) {
        v_i = g_vis[i];
        rank_i = g_rank[i];
        koff_i = g_koff[i];
        key_i = g_key[i];
        if (key_i < 10000) lo_i = map_off[key_i], hi_i = map_off[key_i + 1];
    }
    const uint32_t nv = *g_nv;
    if (tid == 0) s_n = 0;
    for (uint32_t j = tid; j < 2 * 4 * kVisits; j += blockDim.x)  // chunks past the table's end
        if (c_first + (j / kVisits) % 4 >= nchunks) (&s_loc[0][0][0])[j] = 0;
    for (uint32_t v = wv; v < nv; v += nw) {
        uint32_t t0 = 0, t1 = 0, p0 = 0, p1 = 0;
        for (uint64_t c0 = 0; c0 < nchunks; c0 += 64 * kSelBatch) {
            uint32_t x0[kSelBatch], x1[kSelBatch];
            load_batch(ccnt, kcnt, (uint64_t)v * nchunks, nchunks, c0, lane, x0, x1);
#pragma unroll
            for (uint32_t k = 0; k < kSelBatch; ++k) {
                const uint64_t c = c0 + k * 64 + lane;
                t0 += x0[k], t1 += x1[k];
                if (c < c_first) p0 += x0[k], p1 += x1[k];
                if (c >= c_first && c < c_first + 4 && c < nchunks)
                    s_loc[0][c - c_first][v] = x0[k], s_loc[1][c - c_first][v] = x1[k];
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            t0 += __shfl_xor(t0, o, 64), t1 += __shfl_xor(t1, o, 64);
            p0 += __shfl_xor(p0, o, 64), p1 += __shfl_xor(p1, o, 64);
        }
        if (lane == 0) s_tot[0][v] = t0, s_tot[1][v] = t1, s_base[0][v] = p0, s_base[1][v] = p1;
    }
    __syncthreads();
    if (tid < 2) {
        uint32_t pos = 0;
        for (uint32_t v = 0; v < nv; ++v) {
            s_base[tid][v] += pos;
            pos += s_tot[tid][v];
        }
        if (blockIdx.x == 0) counts[tid] = pos;
    }
    __syncthreads();
    if (slot_thread && v_i >= 0) {
        const uint32_t j = tid >> 6, v = (uint32_t)v_i;  // the block's chunk, the slot's visit
        uint32_t pos = s_base[0][v] + rank_i, kpos = s_base[1][v] + koff_i;
        for (uint32_t jj = 0; jj < j; ++jj) pos += s_loc[0][jj][v], kpos += s_loc[1][jj][v];
        const uint32_t m = key_i < 10000 && hi_i > lo_i ? hi_i - lo_i : 0;
        sel[pos] = key_i;
        src[pos] = lo_i;
        cnt[pos] = m;
        dst[pos] = kpos;
        if (m) {
            const uint32_t k = atomicAdd(&s_n, 1u);
            s_a[k] = lo_i;
            s_d[k] = kpos;
            s_m[k] = m;
        }
    }
    __syncthreads();
    const uint32_t nl = s_n;
    for (uint32_t k = wv; k < nl; k += nw) {  // a wave per listed supplier
        const uint64_t a = s_a[k], d = s_d[k];
        const uint32_t m = s_m[k];
        for (uint32_t e0 = 0; e0 < m; e0 += 256) {
            u32x4 x[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t e = e0 + r * 64 + lane;
                if (e < m && d + e < m_cap) x[r] = reinterpret_cast<const u32x4 *>(map_keys)[a + e];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t e = e0 + r * 64 + lane;
                if (e < m && d + e < m_cap) reinterpret_cast<u32x4 *>(keys)[d + e] = x[r];
            }
        }
    }
}

// thread per (query q, supplier s): the abort for a stock lookup that produced no tuple is already
// in abort_flag (launch_revisit_segments); the last entry's stock probe, its hit re-evaluated at
// q's read id here (revisit_one), gives (w, i, quantity, ytd, order_cnt, remote_cnt) and the item key
__global__ void q2_reduce(DevTable st, const stage_probe_out_dev *__restrict__ sbase, const uint32_t *__restrict__ rids,
                          const uint64_t *__restrict__ skeys, const uint64_t *__restrict__ dst,
                          const uint32_t *__restrict__ cnt, const uint64_t *__restrict__ supp, uint32_t skpad,
                          const uint64_t *__restrict__ counts, uint32_t nq, stage_q2_rec *__restrict__ out,
                          uint64_t *__restrict__ ikeys) {
    const uint32_t n = (uint32_t)counts[0];
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;  // q * n + s
    if (g >= n * nq) return;
    const uint32_t s = g % n, q = g / n;
    const uint64_t kb = dst[s];
    const uint32_t c = cnt[s];
    stage_q2_rec r;
    memset(&r, 0, sizeof(r));
    r.supp_key = (int64_t)supp[s];
    if (c) {  // stock_0 / stock_1 of the last lookup (a supplier without stocks keeps zeros)
        const uint64_t klast = kb + c - 1;
        r.s_w_id = (int64_t)skeys[2 * klast];
        r.s_i_id = (int64_t)skeys[2 * klast + 1];
        const u32x4 *bp = reinterpret_cast<const u32x4 *>(sbase + klast);
        u32x4 a = bp[0], b = bp[1];
        revisit_one(st, rids[q], a, b);
        if (produced(a.x & 0xFF)) {
            const uint8_t *row = st.heap + (uint64_t)b.z * st.hstride + skpad;
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
// ... and each record into the caller's page-locked records (host_out, row pitch max_out; null:
// the records stay in `out` on the device).  The host writes cross PCIe: a block's 256 records
// (48 B each) are staged in LDS and leave as 16-B chunks, consecutive lanes on consecutive
// chunks (a wave's store is 1 KB of one run of records), not as 48-B-strided lane stores.
// slot_out (split emit, host_out null): the records into the batch slot's own device buffer, row
// pitch slot_pitch (query q's supplier k at q * slot_pitch + k), for the side stream's copy to
// the caller.
static_assert(sizeof(stage_q2_rec) == 48, "three 16-B chunks per record");
__global__ __launch_bounds__(256) void q2_finish(DevTable it, const stage_probe_out_dev *__restrict__ ibase,
                                                 const uint32_t *__restrict__ rids, uint32_t ikpad,
                                                 const uint64_t *__restrict__ counts,
                                                 uint32_t nq, stage_q2_rec *__restrict__ out, int32_t *__restrict__ abort_flag,
                                                 stage_q2_rec *__restrict__ host_out, uint64_t max_out,
                                                 stage_q2_rec *__restrict__ slot_out, uint64_t slot_pitch) {
    __shared__ u32x4 s_rec[256 * 3];
    const uint32_t n = (uint32_t)counts[0];
    const uint64_t total = (uint64_t)n * nq;
    const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x;
    const uint64_t s = g0 + threadIdx.x;  // q * n + supplier
    if (g0 >= total) return;  // block-uniform
    if (s < total) {
        // the supplier's item probe, its hit re-evaluated at the query's read id (revisit_one)
        const u32x4 *bp = reinterpret_cast<const u32x4 *>(ibase + s % n);
        u32x4 ia = bp[0], ib = bp[1];
        revisit_one(it, rids[s / n], ia, ib);
        const uint32_t st = ia.x & 0xFF;
        stage_q2_rec r = out[s];
        if (!produced(st)) {
            atomicOr(abort_flag + s / n, 1);
        } else {
            // I_DATA's 64 bytes in 16 word loads issued together (4-B aligned), scanned in registers
            const uint32_t *d =
                reinterpret_cast<const uint32_t *>(it.heap + (uint64_t)ib.z * it.hstride + ikpad + kIDataOff);
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
        u32x4 rv[3];
        memcpy(rv, &r, sizeof(r));
#pragma unroll
        for (int k = 0; k < 3; ++k) s_rec[threadIdx.x * 3 + k] = rv[k];
        if (slot_out) {
            u32x4 *so = reinterpret_cast<u32x4 *>(slot_out + (s / n) * slot_pitch + s % n);
#pragma unroll
            for (int k = 0; k < 3; ++k) so[k] = rv[k];
        }
    }
    if (!host_out) return;  // uniform
    __syncthreads();
    const uint64_t nrec = total - g0 < 256 ? total - g0 : 256;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t c = k * 256 + threadIdx.x;  // chunk c: record c / 3, part c % 3
        const uint64_t rec = g0 + c / 3;
        if (c / 3 < nrec && rec % n < max_out)
            reinterpret_cast<u32x4 *>(host_out + (rec / n) * max_out + rec % n)[c % 3] = s_rec[c];
    }
}

// TableScanExecutor rows of one scan from `start` (device scan) into the table's scratch: the
// returned pointer is the first row, the row count (u32) 8 bytes before it
// (d_start: the start key, in device memory written before s reaches the scan)
uint8_t *scan_rows_buf(stage_table *t, uint32_t scan_size) {
    return scratch_bytes(t->dev, 64 + (uint64_t)scan_size * t->dev.view.stride) + 64;
}
// ... and both CH-Q2 dimension scans (REGION, NATION) from the same start key: one launch when
// launch_scan_pair takes them, else one each
void scan_dims(stage_table *a, uint32_t sa, stage_table *b, uint32_t sb, const uint64_t *d_start, hipStream_t s,
               const uint8_t **ra, const uint8_t **rb) {
    uint8_t *pa = scan_rows_buf(a, sa), *pb = scan_rows_buf(b, sb);
    auto cnt = [](uint8_t *rows) { return (uint32_t *)(rows - 8); };  // 8 bytes before the rows
    const DevTable &va = a->dev.view, &vb = b->dev.view;
    if (scan_pair_supported(va, sa, vb, sb)) {
        hip_check(launch_scan_pair(va, d_start, sa, cnt(pa), pa, vb, d_start, sb, cnt(pb), pb, s), "scan pair");
    } else {
        hip_check(launch_scan(va, d_start, nullptr, 1, sa, cnt(pa), pa, s, a->scan_tune), "scan");
        hip_check(launch_scan(vb, d_start, nullptr, 1, sb, cnt(pb), pb, s, b->scan_tune), "scan");
    }
    *ra = pa;
    *rb = pb;
}

}  // namespace
}  // namespace stage

// CH-Q2's users of the tables' per-call scratch, by table role (check_scratch_uses)
enum { kRoleRegion, kRoleNation, kRoleSupplier, kRoleItem, kRoleStock };
static const stage::ScratchUse kQ2Scratch[] = {{kRoleSupplier, "the CH-Q2 batch buffers"},
                                               {kRoleRegion, "the REGION scan rows"},
                                               {kRoleNation, "the NATION scan rows"},
                                               {kRoleItem, "the stock-update staging"}};
constexpr int kQ2ScratchUses = (int)(sizeof(kQ2Scratch) / sizeof(kQ2Scratch[0]));

// nq transactions at read ids rq[0..nq): out[q * max_out + k], aborted[q]; commit only for nq == 1
static int q2_run(stage_table *region, stage_table *nation, stage_table *supplier, stage_table *item,
                  stage_table *stock, const uint32_t *map_off, const uint64_t *d_map_keys, int32_t target_region,
                  const uint32_t *rq, uint32_t nq, uint32_t commit_id, stage_q2_rec *out, uint64_t max_out,
                  uint64_t *n_out, int32_t *aborted, void *stream, int slot = 0, bool async = false) {
    for (stage_table *t : {region, nation, supplier, item, stock})
        if (!t) return fail(STAGE_E_ARG, "null table");
    {
        const void *roles[] = {region, nation, supplier, item, stock};
        int rc = guarded([&] {
            stage::check_scratch_uses(kQ2Scratch, kQ2ScratchUses, roles);
            return STAGE_OK;
        });
        if (rc) return rc;
    }
    for (stage_table *t : {region, nation, supplier, item, stock}) {
        int rc = need_synced(t);
        if (rc) return rc;
    }
    if (!map_off || !d_map_keys || (!async && (!n_out || !aborted)) || (max_out && !out))
        return fail(STAGE_E_ARG, "null argument");
    if (slot < 0 || slot > 1) return fail(STAGE_E_ARG, "slot must be 0 or 1");
    if (stock->q2p[slot].active) return fail(STAGE_E_STATE, "CH-Q2 slot still in flight: stage_ch_query2_wait first");
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
        if (!async) {
            *n_out = 0;
            for (uint32_t q = 0; q < nq; ++q) aborted[q] = 0;
        }
        const DevTable &pv = supplier->dev.view, &sv = stock->dev.view, &iv = item->dev.view;
        const uint64_t nslots = (uint64_t)pv.nleaves * pv.cap;
        if (pv.cap % 64) return fail(STAGE_E_UNSUPPORTED, "SUPPLIER leaves of a multiple of 64 slots");
        const uint64_t nchunks = nslots / 64;
        // upper bounds (buffer sizes, grids): every SUPPLIER slot visited, every map entry looked up
        constexpr uint32_t kMapKeys = 10000;
        uint64_t m_max = 0;
        for (uint32_t k = 0; k < kMapKeys; ++k) m_max += map_off[k + 1] > map_off[k] ? map_off[k + 1] - map_off[k] : 0;
        const uint64_t n_max = std::max<uint64_t>(nslots, 1);
        // launch shapes from the previous call's counts (the visited set depends on the data only)
        const uint64_t n_hint = stock->q2_hint[0] ? std::min(stock->q2_hint[0], n_max) : n_max;
        const uint64_t m_hint = stock->q2_hint[1] ? std::min(stock->q2_hint[1], std::max<uint64_t>(m_max, 1)) : m_max;
        // q2_place up to kPlaceChunks SUPPLIER chunks (STAGE_Q2_PLACE_CHUNKS: another limit, for
        // the tests of the three-kernel form larger tables take)
        const char *pe = std::getenv("STAGE_Q2_PLACE_CHUNKS");
        const bool fused_place = nchunks <= (pe ? std::strtoull(pe, nullptr, 10) : kPlaceChunks);
        // pinned call staging mirrored at the head of the device scratch: [map_off][read ids]
        // [aborted] go down in one copy; [counts][aborted] come back in one copy
        auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
        const uint64_t q_map = 0, q_rq = q_map + al((kMapKeys + 1) * 4ull), q_cn = q_rq + al(nq * 4ull),
                       q_ab = q_cn + 16, q_zero = q_ab + al(nq * 4ull), q_end = q_zero + 16;
        uint8_t *pq = pinned_bytes(stock->dev, q_end, kQ2Pinned + slot);
        std::memcpy(pq + q_map, map_off, (kMapKeys + 1) * 4ull);
        std::memcpy(pq + q_rq, rq, nq * 4ull);
        std::memset(pq + q_cn, 0, 16 + nq * 4ull);
        std::memset(pq + q_zero, 0, 16);  // the REGION / NATION scans' start key: 0 (:653, :734)
        lap("staged");
        uint64_t off = 0;
        auto take = [&](uint64_t bytes) {
            const uint64_t o = off;
            off += al(bytes);
            return o;
        };
        const uint64_t o_mir = take(q_end), o_pairs = take(n_max * 16), o_sel = take(n_max * 8),
                       o_src = take(n_max * 8), o_cnt = take(n_max * 4), o_dst = take(n_max * 8),
                       o_keys = take(std::max<uint64_t>(m_max, 1) * 16), o_sbase = take(std::max<uint64_t>(m_max, 1) * 32),
                       o_ik = take(n_max * 8 * nq),
                       o_ibase = take(n_max * 32), o_rec = take(n_max * nq * sizeof(stage_q2_rec)),
                       o_vis = take(n_max), o_rank = take(n_max), o_koff = take(n_max * 4),
                       o_ccnt = take(std::max<uint64_t>(nchunks, 1) * kVisits * 4),
                       o_kcnt = take(std::max<uint64_t>(nchunks, 1) * kVisits * 4), o_nv = take(4);
        // NATION's scan (scan_sz 65) is past the compact scan kernel's 63 records; a table of fewer
        // slots than that returns the same records for every scan size of at least its slot count
        // (the scan ends at the table's end), so such a table is scanned with that size instead
        uint32_t nat_scan = kNationScan;
        if (nation->dev.view.nleaves <= 4) {
            uint64_t slots = 0;
            for (const auto &L : host(nation).leaves_)
                if (L.live) slots += L.count;
            if (slots < (uint64_t)kNationScan) nat_scan = (uint32_t)std::max<uint64_t>(slots, 1);
        }
        // a batch still in flight uses these scratch buffers: growing one (a reallocation) waits
        // for it first
        const uint64_t reg_rows = 64 + (uint64_t)kRegionScan * region->dev.view.stride,
                       nat_rows = 64 + (uint64_t)kNationScan * nation->dev.view.stride;
        if ((stock->q2p[0].active || stock->q2p[1].active) &&
            (supplier->dev.scratch.cap < off || region->dev.scratch.cap < reg_rows || nation->dev.scratch.cap < nat_rows))
            hip_check(hipDeviceSynchronize(), "q2 drain");
        // the SUPPLIER table's scratch: REGION's and NATION's hold their scan rows (scan_dims)
        uint8_t *buf = scratch_bytes(supplier->dev, off), *mir = buf + o_mir;
        auto *d_map = (const uint32_t *)(mir + q_map);
        auto *d_rq = (const uint32_t *)(mir + q_rq);
        auto *d_counts = (uint64_t *)(mir + q_cn);
        auto *d_ab = (int32_t *)(mir + q_ab);
        auto *d_sel = (uint64_t *)(buf + o_sel);
        auto *d_src = (uint64_t *)(buf + o_src), *d_dst = (uint64_t *)(buf + o_dst);
        auto *d_cnt = (uint32_t *)(buf + o_cnt);
        auto *d_keys = (uint64_t *)(buf + o_keys), *d_ik = (uint64_t *)(buf + o_ik);
        auto *d_sbase = (stage_probe_out_dev *)(buf + o_sbase), *d_ibase = (stage_probe_out_dev *)(buf + o_ibase);
        auto *d_rec = (stage_q2_rec *)(buf + o_rec);
        char tname[16] = {0};
        std::strncpy(tname, kRegions[target_region], 15);
        uint64_t name0, name1, mask0 = 0, mask1 = 0;
        std::memcpy(&name0, tname, 8);
        std::memcpy(&name1, tname + 8, 8);
        for (size_t b = 0; b <= std::strlen(tname); ++b)  // the name and its NUL
            (b < 8 ? mask0 : mask1) |= 0xFFull << (8 * (b % 8));
        auto *g_key = (uint64_t *)(buf + o_pairs);
        auto *g_vis = (int8_t *)(buf + o_vis);
        auto *g_rank = (uint8_t *)(buf + o_rank);
        auto *ccnt = (uint32_t *)(buf + o_ccnt), *kcnt = (uint32_t *)(buf + o_kcnt);
        auto *g_koff = (uint32_t *)(buf + o_koff);
        auto *g_nv = (uint32_t *)(buf + o_nv);
        // `out` in page-locked memory (stage_host_alloc, stage.pinned_empty): the finishing kernel
        // writes the records into it directly; otherwise they are copied once the count is known
        stage_q2_rec *host_out = nullptr;
        if (out && max_out) {  // page-locked memory has a device view; pageable memory has none
            void *dp = nullptr;
            if (hipHostGetDevicePointer(&dp, out, 0) == hipSuccess && dp) host_out = (stage_q2_rec *)dp;
            (void)hipGetLastError();  // a pageable pointer is not an error here
        }
        if (trace) std::fprintf(stderr, "[q2] out %s\n", host_out ? "page-locked: written by q2_finish" : "pageable: copied");
        if (async && out && max_out && !host_out)
            return fail(STAGE_E_ARG, "stage_ch_query2_batch_async needs a page-locked out (stage_host_alloc)");
        // an async batch's records leave from the side stream (Q2Pending::split): finished into
        // the slot's own device buffer, row pitch n_max
        Q2Pending &P = stock->q2p[slot];
        const bool split = async && host_out;
        stage_q2_rec *slot_out = nullptr;
        if (split) {
            const uint64_t need = n_max * nq * sizeof(stage_q2_rec);
            if (P.dcap < need) {  // the slot is idle (checked above): its old buffer is unused
                if (P.dbuf) hip_check(hipFree(P.dbuf), "q2 slot buffer");
                P.dbuf = nullptr;
                P.dcap = 0;
                hip_check(hipMalloc(&P.dbuf, need), "q2 slot buffer");
                P.dcap = need;
            }
            if (!stock->q2_side) hip_check(hipStreamCreateWithFlags(&stock->q2_side, hipStreamNonBlocking), "q2 side stream");
            if (!P.fin) hip_check(hipEventCreateWithFlags(&P.fin, hipEventDisableTiming), "q2 event");
            slot_out = (stage_q2_rec *)P.dbuf;
        }
        lap("buffers");
        // the scan rows' scratch sized before any capture (scan_dims asks for the same size again)
        (void)scratch_bytes(region->dev, reg_rows);
        (void)scratch_bytes(nation->dev, nat_rows);
        // work a caller left on the REGION / NATION tables' own streams (a call without a stream
        // runs there) is finished first: the whole batch then goes on s.  (Round 5 forked the two
        // scans onto those streams and joined them back: the cross-stream waits cost ~20 µs of
        // the ~35 µs the scans took, against ~10 µs for the two scans back to back on s.)
        for (stage_table *d : {region, nation})
            if (d->dev.stream && d->dev.stream != s) hip_check(hipStreamSynchronize(d->dev.stream), "dimension stream");
        // both slots share the SUPPLIER scratch and the REGION / NATION scan rows: a batch still in
        // flight on another stream is waited for on the device before this one is enqueued (on its
        // own stream, stream order already keeps them apart)
        for (const Q2Pending &o : stock->q2p)  // (a split batch's kernels: its copy reads only its slot buffer)
            if (o.active && o.stream != s) hip_check(hipStreamWaitEvent(s, o.split ? o.fin : o.ev, 0), "q2 other slot");
        // everything up to the batch's one synchronisation, enqueued on s
        auto enqueue = [&] {
            hip_check(hipMemcpyAsync(mir, pq, q_end, hipMemcpyHostToDevice, s), "h2d");
            // 1. the REGION / NATION scans
            const auto *d_zero = (const uint64_t *)(mir + q_zero);
            const uint8_t *regs = nullptr, *nats = nullptr;
            scan_dims(region, kRegionScan, nation, nat_scan, d_zero, s, &regs, &nats);
            // 2. the selection and the map segments, on the device (four kernels, no host wait)
            if (nchunks) {
                q2_sel_count<<<(unsigned)((nchunks + 3) / 4), 256, 0, s>>>(
                    regs, region->dev.view.stride, nats, nation->dev.view.stride, name0, name1, mask0, mask1, pv,
                    facts(supplier).key_pad(), nchunks, d_map, g_vis, g_rank, g_koff, g_key, ccnt, kcnt, g_nv);
                if (fused_place) {  // starts, places and the STOCK keys in one launch
                    q2_place<<<(unsigned)((nchunks + 3) / 4), 1024, 0, s>>>(ccnt, kcnt, nchunks, g_nv, g_vis, g_rank,
                                                                          g_koff, g_key, d_map, d_map_keys, m_max,
                                                                          d_sel, d_src, d_cnt, d_dst, d_counts, d_keys);
                } else {
                    q2_sel_start<<<1, 1024, 0, s>>>(ccnt, kcnt, nchunks, g_nv, d_counts);
                    q2_sel_place<<<(unsigned)((nslots + 255) / 256), 256, 0, s>>>(ccnt, kcnt, nslots, g_vis, g_rank,
                                                                                   g_koff, g_key, d_map, d_sel, d_src,
                                                                                   d_cnt, d_dst);
                }
            }
            hip_check(hipGetLastError(), "select");
            // 3. every visited supplier's STOCK keys, one probe of them all (the counts on the device)
            if (!fused_place)
                q2_gather<<<(unsigned)std::max<uint64_t>(std::min<uint64_t>(n_hint, 4096), 1), 256, 0, s>>>(
                    d_map_keys, d_src, d_dst, d_cnt, d_counts, m_max, d_keys);

            // every query of the batch looks up the same STOCK keys (the visited suppliers and their
            // supp_stock_map do not depend on the read id): each key is probed once, with no read id
            // (the hit slot does not depend on it), and its visibility evaluated at every query's read
            // id inside the per-supplier fold (launch_revisit_segments: the aborts and each
            // supplier's last stock, per query)
            // (the misses at every read id folded into the probe where its kernel takes them;
            // q2_reduce re-evaluates each supplier's last lookup)
            if (m_max && probe_missed_supported(sv)) {
                hip_check(launch_probe_missed(sv, d_keys, m_max, d_sbase, s, stock->tune, d_counts + 1, m_hint, d_rq, nq,
                                              d_ab),
                          "stock probe");
            } else if (m_max) {
                hip_check(launch_probe(sv, d_keys, nullptr, nullptr, nullptr, m_max, d_sbase, nullptr, s, stock->tune,
                                       d_counts + 1, m_hint),
                          "stock probe");
                hip_check(launch_revisit_segments(sv, d_sbase, m_max, nullptr, nullptr, 0, d_rq, nq, nullptr, d_ab, s,
                                                  d_counts + 1, nullptr),
                          "stock read ids");
            }
            q2_reduce<<<(unsigned)((n_max * nq + 255) / 256), 256, 0, s>>>(sv, d_sbase, d_rq, d_keys, d_dst, d_cnt, d_sel,
                                                                           facts(stock).key_pad(), d_counts, nq, d_rec,
                                                                           d_ik);
            // 4. item lookups of the last stocks (the same keys in every query: probed once, as above),
            // the I_DATA filter, the records into `out`
            hip_check(launch_probe(iv, d_ik, nullptr, nullptr, nullptr, n_max, d_ibase, nullptr, s, item->tune, d_counts,
                                   n_hint),
                      "item probe");
            q2_finish<<<(unsigned)((n_max * nq + 255) / 256), 256, 0, s>>>(iv, d_ibase, d_rq, facts(item).key_pad(),
                                                                           d_counts, nq, d_rec, d_ab,
                                                                           split ? nullptr : host_out, max_out,
                                                                           slot_out, n_max);
            hip_check(hipGetLastError(), "q2 kernels");
            hip_check(hipMemcpyAsync(pq + q_cn, d_counts, 16 + nq * 4ull, hipMemcpyDeviceToHost, s), "d2h");
        };
        // A hipGraph of the enqueue: captured on the second call with the same arguments (every
        // kernel argument, buffer, stream and launch shape is in the key), replayed while they
        // stay the same -- one launch instead of ~20 (STAGE_Q2_GRAPH=0: always enqueue)
        static const bool graphs = [] {
            const char *e = std::getenv("STAGE_Q2_GRAPH");
            return !(e && std::strcmp(e, "0") == 0);
        }();
        std::string key;
        auto put = [&key](const void *p, size_t n) { key.append((const char *)p, n); };
        auto putv = [&](auto v) { put(&v, sizeof v); };
        for (stage_table *t : {region, nation, supplier, item, stock}) {
            put(&t->dev.view, sizeof t->dev.view);
            putv(t->dev.stream);
            putv(t->dev.scratch.p);
        }
        put(&stock->tune, sizeof stock->tune);
        put(&item->tune, sizeof item->tune);
        put(&region->scan_tune, sizeof region->scan_tune);
        put(&nation->scan_tune, sizeof nation->scan_tune);
        for (uint64_t v : {(uint64_t)(uintptr_t)d_map_keys, (uint64_t)target_region, (uint64_t)nq, max_out,
                           (uint64_t)(uintptr_t)host_out, (uint64_t)(uintptr_t)pq, (uint64_t)(uintptr_t)buf, q_end,
                           n_max, m_max, n_hint, m_hint, (uint64_t)(uintptr_t)s, (uint64_t)nat_scan,
                           (uint64_t)(uintptr_t)slot_out, (uint64_t)fused_place})
            putv(v);
        lap("key");
        Q2Graph &G = stock->q2g[slot];
        bool launched = false;
        if (graphs && !G.failed) {
            if (G.exec && G.key == key) {
                hip_check(hipGraphLaunch(G.exec, s), "q2 graph launch");
                launched = true;
            } else if (G.last_key == key) {  // the same call twice: capture it
                if (G.exec) (void)hipGraphExecDestroy(G.exec);
                G.exec = nullptr;
                G.key.clear();
                hipGraph_t g = nullptr;
                hip_check(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), "q2 capture");
                try {
                    enqueue();
                } catch (...) {
                    (void)hipStreamEndCapture(s, &g);
                    if (g) (void)hipGraphDestroy(g);
                    (void)hipGetLastError();
                    throw;
                }
                hipError_t e = hipStreamEndCapture(s, &g);
                if (!e) e = hipGraphInstantiate(&G.exec, g, nullptr, nullptr, 0);
                if (g) (void)hipGraphDestroy(g);
                if (e) {  // no graph for this call shape: enqueue as before from now on
                    (void)hipGetLastError();
                    G.exec = nullptr;
                    G.failed = true;
                    if (trace) std::fprintf(stderr, "[q2] graph capture failed: %s\n", hipGetErrorString(e));
                } else {
                    G.key = key;
                    hip_check(hipGraphLaunch(G.exec, s), "q2 graph launch");
                    launched = true;
                }
            }
            G.last_key = key;
        }
        if (!launched) enqueue();
        lap("enqueued");
        if (async) {  // the results are read by stage_ch_query2_wait
            if (!P.ev) hip_check(hipEventCreateWithFlags(&P.ev, hipEventDisableTiming), "q2 event");
            P.split = split;
            if (split) {  // the records cross PCIe from the side stream while s goes on
                hip_check(hipEventRecord(P.fin, s), "q2 event");
                hip_check(hipStreamWaitEvent(stock->q2_side, P.fin, 0), "q2 side wait");
                // a 2-D copy (the DMA engine) of the expected count's columns -- the last call's
                // count; wait() copies any more.  (A kernel writing the records over PCIe from the
                // side stream slowed the next batch's kernels beside it ~4x, 0.153 ms a batch
                // against 0.127 with the copy, r06q2emit.)
                P.cols = std::min(n_hint, max_out);
                if (P.cols)
                    hip_check(hipMemcpy2DAsync(out, max_out * sizeof(stage_q2_rec), slot_out, n_max * sizeof(stage_q2_rec),
                                               P.cols * sizeof(stage_q2_rec), nq, hipMemcpyDeviceToHost, stock->q2_side),
                              "q2 records copy");
                P.out = out;
                P.max_out = max_out;
                P.slot_out = slot_out;
                hip_check(hipEventRecord(P.ev, stock->q2_side), "q2 event");
            } else {
                hip_check(hipEventRecord(P.ev, s), "q2 event");
            }
            P.pq = pq;
            P.q_cn = q_cn;
            P.q_ab = q_ab;
            P.nq = nq;
            P.stream = s;
            P.n_max = n_max;
            P.m_max = m_max;
            P.active = true;
            return STAGE_OK;
        }
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

extern "C" int stage_ch_query2_batch_async(stage_table *region, stage_table *nation, stage_table *supplier,
                                           stage_table *item, stage_table *stock, const uint32_t *map_off,
                                           const uint64_t *d_map_keys, int32_t target_region, const uint32_t *read_ids,
                                           uint32_t nq, stage_q2_rec *out, uint64_t max_per_query, int slot,
                                           void *stream) {
    if (nq == 0 || !read_ids || nq > 4096) return fail(STAGE_E_ARG, "read_ids: 1..4096 queries");
    if (!out || !max_per_query) return fail(STAGE_E_ARG, "an out array is required");
    return q2_run(region, nation, supplier, item, stock, map_off, d_map_keys, target_region, read_ids, nq, 0, out,
                  max_per_query, nullptr, nullptr, stream, slot, true);
}

extern "C" int stage_ch_query2_wait(stage_table *stock, int slot, uint64_t *n_out, int32_t *aborted) {
    if (!stock || slot < 0 || slot > 1 || !n_out || !aborted) return fail(STAGE_E_ARG, "bad arguments");
    Q2Pending &P = stock->q2p[slot];
    if (!P.active) return fail(STAGE_E_STATE, "no CH-Q2 batch in flight in this slot");
    return guarded([&] {
        P.active = false;
        stage::hip_check(hipEventSynchronize(P.ev), "q2 wait");
        uint64_t cn[2];
        std::memcpy(cn, P.pq + P.q_cn, 16);
        std::memcpy(aborted, P.pq + P.q_ab, 4ull * P.nq);
        if (cn[0] > P.n_max || cn[1] > P.m_max) throw std::runtime_error("q2: device counts out of range");
        const uint64_t want = std::min<uint64_t>(cn[0], P.max_out);
        if (P.split && want > P.cols)  // more records than the copy expected
            stage::hip_check(hipMemcpy2D(P.out + P.cols, P.max_out * sizeof(stage_q2_rec), P.slot_out + P.cols,
                                         P.n_max * sizeof(stage_q2_rec), (want - P.cols) * sizeof(stage_q2_rec), P.nq,
                                         hipMemcpyDeviceToHost),
                             "q2 records rest");
        stock->q2_hint[0] = cn[0];
        stock->q2_hint[1] = cn[1];
        *n_out = cn[0];
        if (cn[0] == 0)
            for (uint32_t q = 0; q < P.nq; ++q) aborted[q] = 0;
        return STAGE_OK;
    });
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

// the multi-table operations' scratch plans (stage_hip.h)
static const stage::ScratchUse kStockLevelScratch[] = {{0, "the stock-level batch buffers (DISTRICT)"}};

extern "C" int stage_scratch_plan_check(int op, const int32_t *roles, int n) {
    const stage::ScratchUse *plan;
    int np;
    if (op == 0) plan = kQ2Scratch, np = kQ2ScratchUses;
    else if (op == 1) plan = kStockLevelScratch, np = 1;
    else return fail(STAGE_E_ARG, "op: 0 = CH-Q2, 1 = stock-level");
    if (roles && n != np) return fail(STAGE_E_ARG, "roles: one per scratch user of the plan");
    return guarded([&] {
        std::vector<stage::ScratchUse> u(plan, plan + np);
        if (roles)
            for (int i = 0; i < np; ++i) u[i].role = roles[i];
        stage::check_scratch_uses(u.data(), np);
        return STAGE_OK;
    });
}
