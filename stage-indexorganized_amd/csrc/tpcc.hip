// tpcc.hip -- TPC-C stock-level through the index-organized path, batched and device-resident.
//
// The reference transaction (benchmark/tpcc/tpcc_stock_level.cpp:37-180), per (w_id, d_id,
// threshold, read id):
//   1. DISTRICT point lookup {w, d} (IndexScanExecutor point branch) -> D_NEXT_O_ID;
//      a FAILURE result or a missing district ends the transaction (aborted);
//   2. for o in [D_NEXT_O_ID - 20, D_NEXT_O_ID): ORDER_LINE range scan of 10 records from
//      {w, d, o, 5} (IndexScanExecutor range branch, per-record visibility); the predicate keeps
//      OL_I_ID of records whose (OL_W_ID, OL_D_ID, OL_O_ID) == (w, d, o) (it never stops the
//      scan: executor.h:479-482 ignores end_scan);
//   3. if that produced any item: STOCK point lookup {w, ol_i_ids[0]} (the first item only,
//      tpcc_stock_level.cpp:140-175); FAILURE aborts, not found skips; S_QUANTITY < threshold
//      inserts S_I_ID into the distinct set;
//   result = |distinct set| (the reference only logs it), or -1 when the transaction aborted.
//
// Here each step is one batched launch over all transactions (probe_kernel / the scan kernel in
// its IndexScanExecutor form) and three small glue kernels build the next step's keys on the
// device, so the whole batch runs without a host round trip.  Column positions: D_NEXT_O_ID,
// OL_I_ID and S_QUANTITY are the first 4 bytes of their payloads (tpcc_record.h GetData).
#include <hip/hip_runtime.h>

#include <stdexcept>

#include "handle.hpp"

using namespace stage_capi;

namespace stage {
namespace {

constexpr int kOrdersPerTxn = 20;   // min_o_id = max_o_id - 20
constexpr int kLinesPerScan = 10;   // scan_sz
constexpr int64_t kFirstLine = 5;   // OrderLineKey start {w, d, o, 5}

__global__ void sl_district_keys(const int64_t *__restrict__ w, const int64_t *__restrict__ d, uint64_t n,
                                 uint64_t *__restrict__ keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[2 * i] = (uint64_t)w[i];
    keys[2 * i + 1] = (uint64_t)d[i];
}

__device__ __forceinline__ int32_t ld_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}
__device__ __forceinline__ int64_t ld_i64(const uint8_t *p) {
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) v |= (uint64_t)p[b] << (8 * b);
    return (int64_t)v;
}

__device__ __forceinline__ bool produced_tuple(uint32_t st) {
    return st == ST_LATEST || st == ST_COPY || st == ST_OLD;
}

__global__ void sl_spread_rids(const uint32_t *__restrict__ rids, uint64_t ns, uint32_t *__restrict__ out) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s < ns) out[s] = rids ? rids[s / kOrdersPerTxn] : 0xFFFFFFFEu;
}

// step 1 -> 2: abort flags and the 20 order-line start keys of each transaction
__global__ void sl_order_keys(const int64_t *__restrict__ w, const int64_t *__restrict__ d, uint64_t n,
                              const stage_probe_out_dev *__restrict__ dout, const uint8_t *__restrict__ dheap,
                              uint32_t dhstride, uint32_t dkpad, int32_t *__restrict__ result,
                              uint64_t *__restrict__ okeys) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t st = dout[t].w[0] & 0xFF;
    int32_t next = 0;
    if (!produced_tuple(st)) {
        result[t] = -1;  // FAILURE -> abort; no district -> districts.size() != 1 -> return false
    } else {
        result[t] = 0;
        next = ld_i32(dheap + (uint64_t)dout[t].w[6] * dhstride + dkpad);  // D_NEXT_O_ID of the tuple read
    }
    for (int k = 0; k < kOrdersPerTxn; ++k) {
        uint64_t *key = okeys + (t * kOrdersPerTxn + k) * 4;
        key[0] = (uint64_t)w[t];
        key[1] = (uint64_t)d[t];
        key[2] = (uint64_t)(int64_t)(next - kOrdersPerTxn + k);
        key[3] = (uint64_t)kFirstLine;
    }
}

// step 2 -> 3: OL_I_ID of each scan's first predicate-passing tuple -> stock key {w, i}
__global__ void sl_stock_keys(const int64_t *__restrict__ w, uint64_t n, const int32_t *__restrict__ result,
                              const uint32_t *__restrict__ oimg, const uint8_t *__restrict__ ost,
                              const uint8_t *__restrict__ oheap, uint32_t ohstride, uint32_t okpad,
                              uint64_t *__restrict__ skeys, uint8_t *__restrict__ has_item) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n * kOrdersPerTxn) return;
    const uint64_t t = s / kOrdersPerTxn;
    const bool found = result[t] >= 0 && produced_tuple(ost[s]);
    const int32_t item = found ? ld_i32(oheap + (uint64_t)oimg[s] * ohstride + okpad) : 0;  // OL_I_ID
    has_item[s] = found ? 1 : 0;
    skeys[2 * s] = (uint64_t)w[t];
    skeys[2 * s + 1] = (uint64_t)(int64_t)item;
}

// step 3 -> result: one wave per transaction, lane k holds scan k's stock outcome
__global__ __launch_bounds__(64) void sl_count(uint64_t n, const int32_t *__restrict__ threshold,
                                               const uint8_t *__restrict__ has_item,
                                               const stage_probe_out_dev *__restrict__ sout,
                                               const uint8_t *__restrict__ sheap, uint32_t shstride, uint32_t skpad,
                                               int32_t *__restrict__ result) {
    const uint64_t t = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    if (t >= n) return;
    const bool aborted_before = result[t] < 0;
    bool fail = false, below = false;
    int64_t sid = 0;
    if (lane < (uint32_t)kOrdersPerTxn && !aborted_before) {
        const uint64_t s = t * kOrdersPerTxn + lane;
        if (has_item[s]) {
            const uint32_t st = sout[s].w[0] & 0xFF;
            if (st == ST_FAIL_INVALID_TS) {
                fail = true;
            } else if (produced_tuple(st)) {
                const uint8_t *row = sheap + (uint64_t)sout[s].w[6] * shstride;  // the tuple read
                below = ld_i32(row + skpad) < threshold[t];  // S_QUANTITY < threshold
                sid = (int64_t)(int32_t)ld_i64(row + 8);     // distinct_items.insert(int(S_I_ID))
            }
        }
    }
    // distinct S_I_IDs among the lanes below the threshold
    __shared__ int64_t ids[64];
    __shared__ int flags[64];
    ids[lane] = sid;
    flags[lane] = below ? 1 : 0;
    __syncthreads();
    bool first = below;
    if (below)
        for (uint32_t k = 0; k < lane; ++k)
            if (flags[k] && ids[k] == sid) first = false;
    const uint64_t fails = __builtin_amdgcn_ballot_w64(fail);
    const uint64_t firsts = __builtin_amdgcn_ballot_w64(first);
    if (lane == 0 && !aborted_before) result[t] = fails ? -1 : (int32_t)__builtin_popcountll(firsts);
}

}  // namespace
}  // namespace stage

extern "C" int stage_tpcc_stock_level(stage_table *district, stage_table *order_line, stage_table *stock,
                                      const int64_t *d_w_ids, const int64_t *d_d_ids, const int32_t *d_thresholds,
                                      const uint32_t *d_read_ids, uint64_t n, int32_t *d_result, void *stream) {
    for (stage_table *t : {district, order_line, stock}) {
        int rc = need_synced(t);
        if (rc) return rc;
    }
    if (facts(district).params().key_width != 16 || facts(stock).params().key_width != 16 ||
        facts(order_line).params().key_width != 32)
        return fail(STAGE_E_ARG, "expected DistrictKey (16 B), OrderLineKey (32 B), StockKey (16 B) tables");
    if (facts(district).params().payload_size < 4 || facts(order_line).params().payload_size < 4 ||
        facts(stock).params().payload_size < 4)
        return fail(STAGE_E_ARG, "payloads must hold the 4-byte first column");
    if (district->dev.device != order_line->dev.device || district->dev.device != stock->dev.device)
        return fail(STAGE_E_ARG, "tables on different devices");
    if (n && (!d_w_ids || !d_d_ids || !d_thresholds || !d_result)) return fail(STAGE_E_ARG, "null device buffer");
    if (n == 0) return STAGE_OK;
    return guarded([&] {
        using namespace stage;
        hip_check(hipSetDevice(district->dev.device), "hipSetDevice");
        hipStream_t s = pick(district, stream);
        const uint64_t ns = n * kOrdersPerTxn;
        const DevTable &dt = district->dev.view, &ot = order_line->dev.view, &st = stock->dev.view;
        // scratch (the district table's; stream-ordered reuse); tuples are read from the record
        // heaps in place
        const uint64_t o_dkeys = 0, o_dout = o_dkeys + n * 16, o_okeys = o_dout + n * 32, o_oimg = o_okeys + ns * 32,
                       o_ost = o_oimg + ns * 4, o_has = o_ost + ns, o_skeys = (o_has + ns + 15) & ~15ull,
                       o_sout = o_skeys + ns * 16, o_rids = o_sout + ns * 32, total = o_rids + ns * 4;
        uint8_t *buf = scratch_bytes(district->dev, total);
        auto *dkeys = (uint64_t *)(buf + o_dkeys);
        auto *dout = (stage_probe_out_dev *)(buf + o_dout);
        auto *okeys = (uint64_t *)(buf + o_okeys);
        auto *oimg = (uint32_t *)(buf + o_oimg);
        auto *ost = buf + o_ost;
        auto *skeys = (uint64_t *)(buf + o_skeys);
        auto *has = buf + o_has;
        auto *sout = (stage_probe_out_dev *)(buf + o_sout);
        auto *orids = (uint32_t *)(buf + o_rids);
        const unsigned b256 = (unsigned)((n + 255) / 256), bs256 = (unsigned)((ns + 255) / 256);
        // 1. DISTRICT point lookups (status + heap row; no row copies)
        sl_district_keys<<<b256, 256, 0, s>>>(d_w_ids, d_d_ids, n, dkeys);
        hip_check(launch_probe(dt, dkeys, nullptr, d_read_ids, nullptr, n, dout, nullptr, s, district->tune),
                  "district probe");
        // 2. ORDER_LINE range scans of 10 (IndexScanExecutor range branch), all transactions at
        //    once, each kept up to its first produced tuple of order (w, d, o)
        sl_order_keys<<<b256, 256, 0, s>>>(d_w_ids, d_d_ids, n, dout, dt.heap, dt.hstride,
                                           facts(district).key_pad(), d_result, okeys);
        sl_spread_rids<<<bs256, 256, 0, s>>>(d_read_ids, ns, orids);
        hip_check(launch_scan_first(ot, okeys, ns, kLinesPerScan, orids, 3, oimg, ost, s, order_line->scan_tune),
                  "order-line scans");
        // 3. STOCK point lookups of each scan's first item, then the distinct count
        sl_stock_keys<<<bs256, 256, 0, s>>>(d_w_ids, n, d_result, oimg, ost, ot.heap, ot.hstride,
                                            facts(order_line).key_pad(), skeys, has);
        hip_check(launch_probe(st, skeys, nullptr, orids, nullptr, ns, sout, nullptr, s, stock->tune),
                  "stock probe");
        sl_count<<<(unsigned)n, 64, 0, s>>>(n, d_thresholds, has, sout, st.heap, st.hstride, facts(stock).key_pad(),
                                            d_result);
        hip_check(hipGetLastError(), "stock-level kernels");
        return STAGE_OK;
    });
}
