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
// Here REGION / NATION run as device scans and SUPPLIER as a one-lane-per-slot leaf dump; the
// host filters their rows (a few hundred KB); the hot part -- every visited supplier's stock lookups (W * I / 10^4 each, ~2600
// suppliers for EUROPE) and the item lookups -- is one gather kernel, one probe_kernel launch
// over all stock keys, their visibility folded at every read id of the batch (aborts and each
// supplier's last stock), one item probe launch and one finishing kernel.  Updates go through the device write path when
// a commit id is given.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "handle.hpp"
#include "radix_sort.hpp"

using namespace stage_capi;

namespace stage {
namespace {

constexpr int kRegionScan = 6, kNationScan = 65;  // scan_sz of :653 and :734
constexpr uint32_t kIDataOff = 4 + 32 + 8;         // I_DATA in Item's payload (I_IM_ID, I_NAME, I_PRICE)
static const char *const kRegions[] = {"AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"};

__device__ __forceinline__ bool produced(uint32_t st) { return st == ST_LATEST || st == ST_COPY || st == ST_OLD; }

__device__ __forceinline__ int32_t ld_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

__global__ void q2_set_u64(uint64_t *p, uint64_t v) { *p = v; }

// block s copies supplier s's map entries (2 words each) to its segment
__global__ void q2_gather(const uint64_t *__restrict__ map_keys, const uint64_t *__restrict__ src,
                          const uint64_t *__restrict__ dst, const uint32_t *__restrict__ cnt,
                          uint64_t *__restrict__ keys) {
    const uint32_t s = blockIdx.x;
    for (uint32_t e = threadIdx.x; e < cnt[s]; e += blockDim.x) {
        keys[2 * (dst[s] + e)] = map_keys[2 * (src[s] + e)];
        keys[2 * (dst[s] + e) + 1] = map_keys[2 * (src[s] + e) + 1];
    }
}

__global__ void q2_iota(uint32_t *__restrict__ v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// the stock keys in leaf order: out[j] = keys[perm[j]] (2 words each)
__global__ void q2_permute_keys(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ perm, uint64_t m,
                                uint64_t *__restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t p = perm[j];
    out[2 * j] = keys[2 * p];
    out[2 * j + 1] = keys[2 * p + 1];
}

// the leaf-ordered probe results back in key order: out[perm[j]] = in[j]
__global__ void q2_unpermute(const stage_probe_out_dev *__restrict__ in, const uint32_t *__restrict__ perm, uint64_t m,
                             stage_probe_out_dev *__restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) out[perm[j]] = in[j];
}

// thread per (query q, supplier s): the abort for a stock lookup that produced no tuple is already
// in abort_flag (launch_revisit_segments); the last entry's stock row, at q's read id, gives
// (w, i, quantity, ytd, order_cnt, remote_cnt) and the item key
__global__ void q2_reduce(const stage_probe_out_dev *__restrict__ slast, const uint64_t *__restrict__ skeys,
                          const uint64_t *__restrict__ dst, const uint32_t *__restrict__ cnt,
                          const uint64_t *__restrict__ supp, const uint8_t *__restrict__ sheap, uint32_t shstride,
                          uint32_t skpad, uint32_t n, uint32_t nq, stage_q2_rec *__restrict__ out,
                          uint64_t *__restrict__ ikeys) {
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
__global__ void q2_finish(const stage_probe_out_dev *__restrict__ iout, const uint8_t *__restrict__ iheap,
                          uint32_t ihstride, uint32_t ikpad, uint32_t n, uint32_t nq, stage_q2_rec *__restrict__ out,
                          int32_t *__restrict__ abort_flag) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;  // q * n + supplier
    if (s >= n * nq) return;
    const uint32_t st = iout[s].w[0] & 0xFF;
    if (!produced(st)) {
        atomicOr(abort_flag + s / n, 1);
        return;
    }
    const uint8_t *d = iheap + (uint64_t)iout[s].w[6] * ihstride + ikpad + kIDataOff;
    uint8_t has_b = 0;
    for (int c = 0; c < 64 && d[c]; ++c) has_b |= d[c] == 'b';
    out[s].item_has_b = has_b;
    out[s].update = !has_b && out[s].s_quantity < 10;
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

int64_t rd64(const uint8_t *p) {
    int64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

// TableScanExecutor rows of one scan from `start` (device scan): area[0..4) = the row count and
// area + 8 the rows, one asynchronous copy to the pinned host area (the caller synchronises the
// stream before reading)
void scan_rows(stage_table *t, uint64_t start, uint32_t scan_size, uint8_t *area, hipStream_t s) {
    const DevTable &v = t->dev.view;
    const uint64_t rows = (uint64_t)scan_size * v.stride;
    uint8_t *buf = scratch_bytes(t->dev, 64 + rows);
    auto *key = (uint64_t *)buf;
    auto *cnt = (uint32_t *)(buf + 56);  // 8 bytes before the rows
    q2_set_u64<<<1, 1, 0, s>>>(key, start);  // no host buffer outlives the call
    hip_check(launch_scan(v, key, nullptr, 1, scan_size, cnt, buf + 64, s, t->scan_tune), "scan");
    hip_check(hipMemcpyAsync(area, cnt, 8 + rows, hipMemcpyDeviceToHost, s), "d2h");
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
        // 1. REGION / NATION scans, SUPPLIER scan of every record, filtered on the host
        const uint32_t rs = region->dev.view.stride, ns = nation->dev.view.stride;
        // SUPPLIER: every record, ScanLeafNode order
        const DevTable &pv = supplier->dev.view;
        const uint64_t nslots = (uint64_t)pv.nleaves * pv.cap;
        // the host copies go through the stock table's pinned call staging (pageable copies
        // are staged by the runtime and wait for each other): [REGION count, rows][NATION
        // count, rows][SUPPLIER (key, nation) pairs]
        auto alp = [](uint64_t x) { return (x + 255) & ~255ull; };
        const uint64_t p_regs = 0, p_nats = p_regs + alp(8 + (uint64_t)kRegionScan * rs),
                       p_pairs = p_nats + alp(8 + (uint64_t)kNationScan * ns), p_end = p_pairs + nslots * 16;
        uint8_t *pin = pinned_bytes(stock->dev, p_end, 2);
        // the REGION and NATION scans on their tables' own streams beside the SUPPLIER dump on
        // s (forked from and joined back into s): three short dependent chains side by side
        hipEvent_t *ev = stock->dev.call_ev;
        for (int k = 0; k < 3; ++k)
            if (!ev[k]) hip_check(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), "call event");
        hipStream_t rs_s = region->dev.stream ? region->dev.stream : s, ns_s = nation->dev.stream ? nation->dev.stream : s;
        hip_check(hipEventRecord(ev[0], s), "fork");
        hip_check(hipStreamWaitEvent(rs_s, ev[0], 0), "fork");
        hip_check(hipStreamWaitEvent(ns_s, ev[0], 0), "fork");
        scan_rows(region, 0, kRegionScan, pin + p_regs, rs_s);
        scan_rows(nation, 0, kNationScan, pin + p_nats, ns_s);
        hip_check(hipEventRecord(ev[1], rs_s), "join");
        hip_check(hipEventRecord(ev[2], ns_s), "join");
        uint8_t *pbuf = scratch_bytes(supplier->dev, nslots * 16);
        q2_dump_leaves<<<(unsigned)std::min<uint64_t>((nslots + 255) / 256, 4096), 256, 0, s>>>(
            pv, facts(supplier).key_pad(), (uint64_t *)pbuf);
        hip_check(hipGetLastError(), "dump leaves");
        hip_check(hipMemcpyAsync(pin + p_pairs, pbuf, nslots * 16, hipMemcpyDeviceToHost, s), "d2h");
        hip_check(hipStreamWaitEvent(s, ev[1], 0), "join");
        hip_check(hipStreamWaitEvent(s, ev[2], 0), "join");
        const uint8_t *regs_p = pin + p_regs + 8, *nats_p = pin + p_nats + 8;
        const uint64_t *pairs = (const uint64_t *)(pin + p_pairs);
        lap("scans enqueued");
        hip_check(hipStreamSynchronize(s), "scan sync");  // the three scans complete together
        lap("scans done");
        uint32_t nreg, nnat;
        std::memcpy(&nreg, pin + p_regs, 4);
        std::memcpy(&nnat, pin + p_nats, 4);
        // the visiting order of :770-797: for each region named regions[target] (scan order),
        // for each of its nations (scan order), every SUPPLIER slot of that nation in
        // ScanLeafNode order -- one pass over the slots into per-visit buckets
        std::vector<int64_t> visit;  // nation key of each (region, nation) visit, in order
        for (uint32_t r = 0; r < nreg; ++r) {
            const uint8_t *rr = regs_p + (uint64_t)r * rs;
            char name[56];
            std::memcpy(name, rr + 8, 55);
            name[55] = 0;
            if (std::string(name) != kRegions[target_region]) continue;
            for (uint32_t a = 0; a < nnat; ++a) {
                const uint8_t *nr = nats_p + (uint64_t)a * ns;
                if (rd64(nr + 8) == rd64(rr)) visit.push_back(rd64(nr));
            }
        }
        // visit index of each nation key: a direct table when the visited keys are small and
        // distinct (always, for the loader's nations 0..61), else the per-slot search over visits
        constexpr int64_t kDirect = 4096;
        std::vector<int32_t> vidx(kDirect, -1);
        bool direct = true;
        for (size_t j = 0; j < visit.size() && direct; ++j) {
            if (visit[j] < 0 || visit[j] >= kDirect || vidx[visit[j]] >= 0) direct = false;
            else vidx[visit[j]] = (int32_t)j;
        }
        std::vector<uint64_t> sel;  // visited suppliers in visiting order
        if (direct) {  // counting pass, then each slot placed at its visit's next position
            std::vector<uint32_t> pos(visit.size() + 1, 0);
            for (uint64_t k = 0; k < nslots; ++k) {
                const int64_t nat = (int64_t)pairs[2 * k + 1];
                if (pairs[2 * k] != ~0ull && nat >= 0 && nat < kDirect && vidx[nat] >= 0) ++pos[vidx[nat] + 1];
            }
            for (size_t j = 0; j < visit.size(); ++j) pos[j + 1] += pos[j];
            sel.resize(pos[visit.size()]);
            for (uint64_t k = 0; k < nslots; ++k) {
                const int64_t nat = (int64_t)pairs[2 * k + 1];
                if (pairs[2 * k] != ~0ull && nat >= 0 && nat < kDirect && vidx[nat] >= 0)
                    sel[pos[vidx[nat]]++] = pairs[2 * k];
            }
        } else {
            std::vector<std::vector<uint64_t>> bucket(visit.size());
            for (uint64_t k = 0; k < nslots; ++k) {
                if (pairs[2 * k] == ~0ull) continue;
                const int64_t nat = (int64_t)pairs[2 * k + 1];
                for (size_t j = 0; j < visit.size(); ++j)
                    if (visit[j] == nat) bucket[j].push_back(pairs[2 * k]);
            }
            for (const auto &b : bucket) sel.insert(sel.end(), b.begin(), b.end());
        }
        const uint32_t n = (uint32_t)sel.size();
        lap("suppliers selected");
        *n_out = n;
        if (n == 0) return STAGE_OK;
        // 2. stock keys of every visited supplier, one probe launch.  Pinned call staging again
        // (the scans' contents are no longer needed: a growth may move it), mirrored by the head
        // of the device scratch so that one copy goes down and one comes back:
        // [src][dst][cnt][sel][read ids] down, [aborted] (zeroed) down and up, [records] up
        const uint64_t q_src = 0, q_dst = q_src + alp(n * 8ull), q_cnt = q_dst + alp(n * 8ull),
                       q_sel = q_cnt + alp(n * 4ull), q_rq = q_sel + alp(n * 8ull), q_ab = q_rq + alp(nq * 4ull),
                       q_rec = q_ab + alp(nq * 4ull), q_end = q_rec + alp((uint64_t)n * nq * sizeof(stage_q2_rec));
        uint8_t *pq = pinned_bytes(stock->dev, q_end, 2);
        uint64_t *src = (uint64_t *)(pq + q_src), *dst = (uint64_t *)(pq + q_dst);
        uint32_t *cnt = (uint32_t *)(pq + q_cnt);
        std::memcpy(pq + q_sel, sel.data(), n * 8ull);
        std::memcpy(pq + q_rq, rq, nq * 4ull);
        std::memset(pq + q_ab, 0, nq * 4ull);
        uint64_t m = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const uint64_t sk = sel[k];
            src[k] = sk < 10000 ? map_off[sk] : 0;
            cnt[k] = sk < 10000 ? map_off[sk + 1] - map_off[sk] : 0;
            dst[k] = m;
            m += cnt[k];
        }
        // STAGE_Q2_SORT=1: the STOCK keys probed in leaf order (their descents first, a radix sort of
        // (leaf, position), the probe from the known leaves, results written back in place by the
        // per-read-id revisit) -- neighbouring probes share leaf heads and bottom nodes in L2
        const char *qs = std::getenv("STAGE_Q2_SORT");
        const bool sorted = m > 1 && qs && qs[0] == '1';
        const DevTable &sv0 = stock->dev.view;
        int lbits = 1;
        while (lbits < 32 && (1ull << lbits) <= sv0.nleaves) ++lbits;
        size_t cub_bytes = 0;
        if (sorted)
            hip_check(sort_pairs(nullptr, cub_bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                 (const uint32_t *)nullptr, (uint32_t *)nullptr, m, 0, lbits, s),
                      "sort size");
        auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
        uint64_t off = 0;
        auto take = [&](uint64_t bytes) {
            const uint64_t o = off;
            off += al(bytes);
            return o;
        };
        const uint64_t o_mir = take(q_end), o_keys = take(std::max<uint64_t>(m, 1) * 16),
                       o_sbase = take(std::max<uint64_t>(m, 1) * 32),
                       o_leaf = take(sorted ? m * 4 : 0), o_sleaf = take(sorted ? m * 4 : 0),
                       o_iota = take(sorted ? m * 4 : 0), o_perm = take(sorted ? m * 4 : 0),
                       o_skeys = take(sorted ? m * 16 : 0), o_cub = take(sorted ? cub_bytes : 0),
                       o_sout = take(sorted ? m * 32 : 0), o_slast = take(n * 32ull * nq),
                       o_ik = take(n * 8 * nq), o_iout = take(n * 32 * nq), o_ibase = take(n * 32);
        uint8_t *buf = scratch_bytes(nation->dev, off), *mir = buf + o_mir;
        auto *d_src = (uint64_t *)(mir + q_src), *d_dst = (uint64_t *)(mir + q_dst), *d_sup = (uint64_t *)(mir + q_sel);
        auto *d_cnt = (uint32_t *)(mir + q_cnt), *d_rq = (uint32_t *)(mir + q_rq);
        auto *d_keys = (uint64_t *)(buf + o_keys), *d_ik = (uint64_t *)(buf + o_ik);
        auto *d_sout = (stage_probe_out_dev *)(buf + o_sout), *d_iout = (stage_probe_out_dev *)(buf + o_iout);
        auto *d_slast = (stage_probe_out_dev *)(buf + o_slast);
        auto *d_sbase = (stage_probe_out_dev *)(buf + o_sbase), *d_ibase = (stage_probe_out_dev *)(buf + o_ibase);
        auto *d_rec = (stage_q2_rec *)(mir + q_rec);
        auto *d_ab = (int32_t *)(mir + q_ab);
        hip_check(hipMemcpyAsync(mir, pq, q_rec, hipMemcpyHostToDevice, s), "h2d");
        q2_gather<<<n, 256, 0, s>>>(d_map_keys, d_src, d_dst, d_cnt, d_keys);
        const DevTable &sv = stock->dev.view, &iv = item->dev.view;
        // every query of the batch looks up the same STOCK keys (the visited suppliers and their
        // supp_stock_map do not depend on the read id): each key is probed once, with no read id
        // (the hit slot does not depend on it), and its visibility evaluated at every query's read
        // id inside the per-supplier fold (launch_revisit_segments: the aborts and each
        // supplier's last stock, per query)
        const stage_probe_out_dev *d_stock = d_sbase;
        if (sorted) {
            auto *d_leaf = (uint32_t *)(buf + o_leaf), *d_sleaf = (uint32_t *)(buf + o_sleaf);
            auto *d_iota = (uint32_t *)(buf + o_iota), *d_perm = (uint32_t *)(buf + o_perm);
            auto *d_skeys = (uint64_t *)(buf + o_skeys);
            const unsigned mb = (unsigned)((m + 255) / 256);
            hip_check(launch_resolve(sv, d_keys, nullptr, m, 1, d_leaf, s), "stock descents");
            q2_iota<<<mb, 256, 0, s>>>(d_iota, m);
            size_t cb = cub_bytes;
            hip_check(sort_pairs(buf + o_cub, cb, (const uint32_t *)d_leaf, d_sleaf, (const uint32_t *)d_iota, d_perm, m, 0,
                                 lbits, s),
                      "stock leaf sort");
            q2_permute_keys<<<mb, 256, 0, s>>>(d_keys, d_perm, m, d_skeys);
            hip_check(launch_probe(sv, d_skeys, nullptr, nullptr, d_sleaf, m, d_sbase, nullptr, s, stock->tune),
                      "stock probe");
            q2_unpermute<<<mb, 256, 0, s>>>(d_sbase, d_perm, m, d_sout);
            d_stock = d_sout;
        } else if (m) {
            hip_check(launch_probe(sv, d_keys, nullptr, nullptr, nullptr, m, d_sbase, nullptr, s, stock->tune),
                      "stock probe");
        }
        if (m)
            hip_check(launch_revisit_segments(sv, d_stock, m, d_dst, d_cnt, n, d_rq, nq, d_slast, d_ab, s),
                      "stock read ids");
        q2_reduce<<<(n * nq + 255) / 256, 256, 0, s>>>(d_slast, d_keys, d_dst, d_cnt, d_sup, sv.heap, sv.hstride,
                                                       facts(stock).key_pad(), n, nq, d_rec, d_ik);
        // 3. item lookups of the last stocks (the same keys in every query: probed once, as above),
        // filter
        hip_check(launch_probe(iv, d_ik, nullptr, nullptr, nullptr, n, d_ibase, nullptr, s, item->tune), "item probe");
        hip_check(launch_revisit(iv, d_ibase, n, d_rq, nq, nullptr, d_iout, s), "item read ids");
        q2_finish<<<(n * nq + 255) / 256, 256, 0, s>>>(d_iout, iv.heap, iv.hstride, facts(item).key_pad(), n, nq,
                                                       d_rec, d_ab);
        hip_check(hipGetLastError(), "q2 kernels");
        // `out` in page-locked memory (stage_host_alloc, stage.pinned_empty) with room for every
        // record: the records go straight there (one 2-D copy) instead of through the call
        // staging and a host memcpy
        bool to_out = false;
        if (out && n <= max_out) {
            hipPointerAttribute_t pa;
            to_out = hipPointerGetAttributes(&pa, out) == hipSuccess && pa.type == hipMemoryTypeHost;
            (void)hipGetLastError();  // a pageable pointer is not an error here
        }
        stage_q2_rec *recs = to_out ? out : (stage_q2_rec *)(pq + q_rec);
        if (to_out) {
            hip_check(hipMemcpyAsync(pq + q_ab, d_ab, 4ull * nq, hipMemcpyDeviceToHost, s), "d2h");
            hip_check(hipMemcpy2DAsync(out, max_out * sizeof(stage_q2_rec), d_rec, n * sizeof(stage_q2_rec),
                                       n * sizeof(stage_q2_rec), nq, hipMemcpyDeviceToHost, s),
                      "d2h");
        } else {
            hip_check(hipMemcpyAsync(pq + q_ab, d_ab, (q_rec - q_ab) + (uint64_t)n * nq * sizeof(stage_q2_rec),
                                     hipMemcpyDeviceToHost, s),
                      "d2h");  // [aborted][records]
        }
        lap("probes enqueued");
        hip_check(hipStreamSynchronize(s), "q2 sync");
        lap("results back");
        std::memcpy(aborted, pq + q_ab, 4ull * nq);
        const uint32_t read_id = rq[0];
        // 4. the transaction's stock updates, through the device write path
        if (nq == 1 && commit_id && !*aborted) {
            std::vector<uint64_t> uk;
            std::vector<int32_t> ud;
            std::vector<uint32_t> ui;
            for (uint32_t k = 0; k < n; ++k)
                if (recs[k].update) {
                    uk.push_back((uint64_t)recs[k].s_w_id);
                    uk.push_back((uint64_t)recs[k].s_i_id);
                    ud.insert(ud.end(), {recs[k].s_quantity + 50, recs[k].s_ytd, recs[k].s_order_cnt,
                                         recs[k].s_remote_cnt});
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
                for (uint64_t j = 0; j < nu; ++j) recs[ui[j]].update_rc = rcs[j];
            }
        }
        if (!to_out)
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
