// dist.hip -- multi-GPU YCSB-C front-end: route every key to shard
// MurmurHash64A(key, 8, 0) % world (misc/murmur/MurmurHash2.cpp:99-147 as the router),
// exchange keys with one RCCL all-to-all-v (grouped ncclSend/ncclRecv over xGMI), probe the
// local shard, return results with the reverse all-to-all-v and scatter them back into the
// caller's order.  The reference has no distributed layer; this is the
// build's own exchange step for the 8-GPU config.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/stage_hip.h"
#include "dist.hpp"

namespace stage {

namespace {

void chk(hipError_t e, const char *what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void nchk(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

struct alignas(16) SendRec {
    uint64_t key;
    uint32_t rid;
    uint32_t pad;
};

__device__ __forceinline__ uint64_t mm64a_8(uint64_t k) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 0 ^ (8ull * m);
    k *= m;
    k ^= k >> 47;
    k *= m;
    h ^= k;
    h *= m;
    h ^= h >> 47;
    h *= m;
    h ^= h >> 47;
    return h;
}

// Routing without global atomics: per-block LDS histograms (blk[d*NB + b]), one exclusive
// scan over them (dest-major, so offsets come out grouped by destination rank), then a
// scatter that claims positions with LDS atomics inside each block's range.
constexpr int kRouteBlocks = 1024;
constexpr int kMaxWorld = 64;

__global__ __launch_bounds__(256) void route_hist(const uint64_t *__restrict__ keys, uint64_t n, int world,
                                                  uint8_t *__restrict__ dest, uint32_t *__restrict__ blk) {
    __shared__ uint32_t h[kMaxWorld];
    if (threadIdx.x < (unsigned)world) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        const uint32_t d = (uint32_t)(mm64a_8(keys[i]) % (uint64_t)world);
        dest[i] = (uint8_t)d;
        atomicAdd(&h[d], 1u);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)world) blk[threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of m = world*NB counters in one 1024-thread block; counts[d] = per-rank totals
__global__ __launch_bounds__(1024) void route_scan(const uint32_t *__restrict__ blk, uint32_t m, int world, int nb,
                                                   uint32_t *__restrict__ offs, uint32_t *__restrict__ counts) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (m + 1023) / 1024;
    const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < m ? b0 + per : m;
    uint32_t s = 0;
    for (uint32_t i = b0; i < b1; ++i) s += blk[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0u;
    for (uint32_t i = b0; i < b1; ++i) {
        offs[i] = run;
        run += blk[i];
    }
    if (threadIdx.x == 1023) offs[m] = part[1023];
    __syncthreads();
    if (threadIdx.x < (unsigned)world) {
        const uint32_t lo = offs[threadIdx.x * nb];
        const uint32_t hi = (int)threadIdx.x + 1 < world ? offs[(threadIdx.x + 1) * nb] : part[1023];
        counts[threadIdx.x] = hi - lo;
    }
}

__global__ __launch_bounds__(256) void route_scatter(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ rids,
                                                     uint64_t n, int world, const uint8_t *__restrict__ dest,
                                                     const uint32_t *__restrict__ offs, SendRec *__restrict__ send,
                                                     uint32_t *__restrict__ perm) {
    __shared__ uint32_t cur[kMaxWorld];
    if (threadIdx.x < (unsigned)world) cur[threadIdx.x] = offs[threadIdx.x * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        const uint32_t pos = atomicAdd(&cur[dest[i]], 1u);
        send[pos] = SendRec{keys[i], rids ? rids[i] : 0xFFFFFFFEu, 0};
        perm[pos] = (uint32_t)i;
    }
}

__global__ void unpack_keys(const SendRec *__restrict__ recv, uint64_t n, uint64_t *__restrict__ keys,
                            uint32_t *__restrict__ rids) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = recv[i].key;
    rids[i] = recv[i].rid;
}

// back in the caller's order: out[perm[p]] = bout[p], row copy by one wave per probe
__global__ void unpermute(const stage_probe_out_dev *__restrict__ bout, const uint8_t *__restrict__ brec,
                          const uint32_t *__restrict__ perm, uint64_t n, uint32_t stride,
                          stage_probe_out_dev *__restrict__ out, uint8_t *__restrict__ recs) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t p = w; p < n; p += nw) {
        const uint32_t dst = perm[p];
        if (lane < 2) reinterpret_cast<uint4 *>(out + dst)[lane] = reinterpret_cast<const uint4 *>(bout + p)[lane];
        if (recs) {
            const uint4 *s = reinterpret_cast<const uint4 *>(brec + p * (uint64_t)stride);
            uint4 *d = reinterpret_cast<uint4 *>(recs + (uint64_t)dst * stride);
            for (uint32_t c = lane; c < (stride >> 4); c += 64) d[c] = s[c];
        }
    }
}

void grow(void *&p, uint64_t bytes) {
    if (p) chk(hipFree(p), "hipFree");
    p = nullptr;
    chk(hipMalloc(&p, bytes ? bytes : 16), "hipMalloc");
}

}  // namespace

ShardComm::~ShardComm() {
    if (comm) ncclCommDestroy((ncclComm_t)comm);
    for (void *p : {dest, cursor, perm, send, recv, rout, rrec, bout, brec, cnt, lkeys, lrids})
        if (p) (void)hipFree(p);
}

int shard_unique_id(uint8_t *id128) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    nchk(ncclGetUniqueId(&id), "ncclGetUniqueId");
    std::memcpy(id128, &id, 128);
    return STAGE_OK;
}

int shard_init(ShardComm &c, const uint8_t *id128, int rank, int world) {
    ncclUniqueId id;
    std::memcpy(&id, id128, 128);
    ncclComm_t comm;
    nchk(ncclCommInitRank(&comm, world, id, rank), "ncclCommInitRank");
    c.comm = comm;
    c.rank = rank;
    c.world = world;
    if (world > kMaxWorld) throw std::invalid_argument("world size above 64");
    grow(c.cnt, 4 * sizeof(uint32_t) * (uint64_t)world);
    grow(c.cursor, (2ull * world * kRouteBlocks + 16) * sizeof(uint32_t));
    return STAGE_OK;
}

// ---- the phases of one sharded probe (shared by the RCCL path and the loopback rehearsal)

// route the caller's keys: send buffer grouped by destination, perm = caller index of each
// send slot; returns the per-destination counts (host)
static std::vector<uint32_t> phase_route(ShardComm &c, const uint64_t *d_keys, const uint32_t *d_rids, uint64_t n,
                                         uint32_t stride, hipStream_t s) {
    const int W = c.world;
    if (n > 0xFFFFFFFFull) throw std::invalid_argument("batch too large");
    if (n > c.cap_local || stride != c.rec_stride) {
        const uint64_t cap = n + n / 8 + 1024;
        grow(c.dest, cap);
        grow(c.perm, cap * 4);
        grow(c.send, cap * sizeof(SendRec));
        grow(c.bout, cap * sizeof(stage_probe_out_dev));
        grow(c.brec, cap * stride);
        c.cap_local = cap;
        c.rec_stride = stride;
        c.cap_remote = 0;  // remote buffers follow the stride too
    }
    uint32_t *counts = (uint32_t *)c.cnt;  // [0,W) send counts, [2W,3W) recv counts
    uint32_t *blk = (uint32_t *)c.cursor, *offs = blk + (uint64_t)W * kRouteBlocks;
    if (n) {
        route_hist<<<kRouteBlocks, 256, 0, s>>>(d_keys, n, W, (uint8_t *)c.dest, blk);
        route_scan<<<1, 1024, 0, s>>>(blk, (uint32_t)(W * kRouteBlocks), W, kRouteBlocks, offs, counts);
        route_scatter<<<kRouteBlocks, 256, 0, s>>>(d_keys, d_rids, n, W, (const uint8_t *)c.dest, offs,
                                                   (SendRec *)c.send, (uint32_t *)c.perm);
    } else {
        chk(hipMemsetAsync(counts, 0, W * sizeof(uint32_t), s), "memset");
    }
    std::vector<uint32_t> sc(W);
    chk(hipMemcpyAsync(sc.data(), counts, W * 4, hipMemcpyDeviceToHost, s), "counts d2h");
    chk(hipStreamSynchronize(s), "sync");
    return sc;
}

static void ensure_remote(ShardComm &c, uint64_t m, uint32_t stride) {
    if (m <= c.cap_remote) return;
    const uint64_t cap = m + m / 8 + 1024;
    grow(c.recv, cap * sizeof(SendRec));
    grow(c.rout, cap * sizeof(stage_probe_out_dev));
    grow(c.rrec, cap * stride);
    grow(c.lkeys, cap * 8);
    grow(c.lrids, cap * 4);
    c.cap_remote = cap;
}

// probe the m keys this shard received (recv buffer) into rout / rrec
static void phase_probe(ShardComm &c, const DevTable &t, const ProbeTuning &tune, uint64_t m, bool rows,
                        hipStream_t s) {
    if (!m) return;
    uint64_t *lk = (uint64_t *)c.lkeys;
    uint32_t *lr = (uint32_t *)c.lrids;
    unpack_keys<<<(unsigned)((m + 255) / 256), 256, 0, s>>>((const SendRec *)c.recv, m, lk, lr);
    chk(launch_probe(t, lk, nullptr, lr, nullptr, m, (stage_probe_out_dev *)c.rout, rows ? (uint8_t *)c.rrec : nullptr,
                     s, tune),
        "probe");
}

static void phase_unpermute(ShardComm &c, uint64_t n, uint32_t stride, stage_probe_out_dev *d_out, uint8_t *d_recs,
                            hipStream_t s) {
    if (n)
        unpermute<<<(unsigned)std::min<uint64_t>((n + 3) / 4, 8192), 256, 0, s>>>(
            (const stage_probe_out_dev *)c.bout, (const uint8_t *)c.brec, (const uint32_t *)c.perm, n, stride, d_out,
            d_recs);
    chk(hipGetLastError(), "unpermute");
}

static std::vector<uint64_t> prefix(const std::vector<uint32_t> &v) {
    std::vector<uint64_t> o(v.size() + 1, 0);
    for (size_t r = 0; r < v.size(); ++r) o[r + 1] = o[r] + v[r];
    return o;
}

int shard_probe(ShardComm &c, const DevTable &t, const ProbeTuning &tune, const uint64_t *d_keys,
                const uint32_t *d_rids, uint64_t n, stage_probe_out_dev *d_out, uint8_t *d_recs, hipStream_t s) {
    if (!c.comm) throw std::invalid_argument("not an RCCL communicator");
    const int W = c.world;
    const uint32_t stride = t.stride;
    const std::vector<uint32_t> sc = phase_route(c, d_keys, d_rids, n, stride, s);
    const std::vector<uint64_t> soff = prefix(sc);
    // exchange the per-destination counts
    uint32_t *counts = (uint32_t *)c.cnt;
    ncclComm_t comm = (ncclComm_t)c.comm;
    nchk(ncclAllToAll(counts, counts + 2 * W, 1, ncclUint32, comm, s), "ncclAllToAll counts");
    std::vector<uint32_t> rc(W);
    chk(hipMemcpyAsync(rc.data(), counts + 2 * W, W * 4, hipMemcpyDeviceToHost, s), "recv counts d2h");
    chk(hipStreamSynchronize(s), "sync");
    const std::vector<uint64_t> roff = prefix(rc);
    const uint64_t m = roff[W];
    ensure_remote(c, m, stride);
    // keys out: all-to-all-v as grouped point-to-point transfers
    nchk(ncclGroupStart(), "group");
    for (int r = 0; r < W; ++r) {
        if (sc[r]) nchk(ncclSend((const uint8_t *)c.send + soff[r] * sizeof(SendRec), (uint64_t)sc[r] * sizeof(SendRec),
                                 ncclUint8, r, comm, s), "send keys");
        if (rc[r]) nchk(ncclRecv((uint8_t *)c.recv + roff[r] * sizeof(SendRec), (uint64_t)rc[r] * sizeof(SendRec), ncclUint8,
                                 r, comm, s), "recv keys");
    }
    nchk(ncclGroupEnd(), "group end");
    phase_probe(c, t, tune, m, d_recs != nullptr, s);
    // results back
    const uint64_t ob = sizeof(stage_probe_out_dev);
    nchk(ncclGroupStart(), "group");
    for (int r = 0; r < W; ++r) {
        if (rc[r]) {
            nchk(ncclSend((const uint8_t *)c.rout + roff[r] * ob, (uint64_t)rc[r] * ob, ncclUint8, r, comm, s), "send out");
            if (d_recs)
                nchk(ncclSend((const uint8_t *)c.rrec + roff[r] * stride, (uint64_t)rc[r] * stride, ncclUint8, r, comm, s),
                     "send rows");
        }
        if (sc[r]) {
            nchk(ncclRecv((uint8_t *)c.bout + soff[r] * ob, (uint64_t)sc[r] * ob, ncclUint8, r, comm, s), "recv out");
            if (d_recs)
                nchk(ncclRecv((uint8_t *)c.brec + soff[r] * stride, (uint64_t)sc[r] * stride, ncclUint8, r, comm, s),
                     "recv rows");
        }
    }
    nchk(ncclGroupEnd(), "group end");
    phase_unpermute(c, n, stride, d_out, d_recs, s);
    return STAGE_OK;
}

int shard_init_loopback(ShardComm &c, int rank, int world) {
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
    c.comm = nullptr;
    c.rank = rank;
    c.world = world;
    grow(c.cnt, 4 * sizeof(uint32_t) * (uint64_t)world);
    grow(c.cursor, (2ull * world * kRouteBlocks + 16) * sizeof(uint32_t));
    return STAGE_OK;
}

// The same phases for W shards held by one process on one device, with device-to-device
// copies where shard_probe has RCCL transfers (same offsets, same order).  Every shard's
// stride must be equal.
int shard_probe_loopback(const std::vector<ShardComm *> &cs, const std::vector<const DevTable *> &ts,
                         const ProbeTuning &tune, const std::vector<const uint64_t *> &keys,
                         const std::vector<const uint32_t *> &rids, const std::vector<uint64_t> &n,
                         const std::vector<stage_probe_out_dev *> &outs, const std::vector<uint8_t *> &recs,
                         hipStream_t s) {
    const int W = (int)cs.size();
    const uint32_t stride = ts[0]->stride;
    for (int r = 0; r < W; ++r)
        if (ts[r]->stride != stride || cs[r]->world != W || cs[r]->rank != r)
            throw std::invalid_argument("loopback shards disagree on stride / rank / world");
    const bool rows = recs[0] != nullptr;
    std::vector<std::vector<uint32_t>> sc(W), rc(W, std::vector<uint32_t>(W));
    std::vector<std::vector<uint64_t>> soff(W), roff(W);
    for (int r = 0; r < W; ++r) {
        sc[r] = phase_route(*cs[r], keys[r], rids[r], n[r], stride, s);
        soff[r] = prefix(sc[r]);
    }
    for (int r = 0; r < W; ++r)
        for (int q = 0; q < W; ++q) rc[r][q] = sc[q][r];  // what the count all-to-all delivers
    for (int r = 0; r < W; ++r) {
        roff[r] = prefix(rc[r]);
        ensure_remote(*cs[r], roff[r][W], stride);
    }
    for (int r = 0; r < W; ++r)  // keys: q's send segment for r -> r's receive segment from q
        for (int q = 0; q < W; ++q)
            if (sc[q][r])
                chk(hipMemcpyAsync((uint8_t *)cs[r]->recv + roff[r][q] * sizeof(SendRec),
                                   (const uint8_t *)cs[q]->send + soff[q][r] * sizeof(SendRec),
                                   (uint64_t)sc[q][r] * sizeof(SendRec), hipMemcpyDeviceToDevice, s),
                    "loopback keys");
    for (int r = 0; r < W; ++r) phase_probe(*cs[r], *ts[r], tune, roff[r][W], rows, s);
    const uint64_t ob = sizeof(stage_probe_out_dev);
    for (int q = 0; q < W; ++q)  // results: owner q's segment for origin r -> r's slots of q
        for (int r = 0; r < W; ++r)
            if (rc[q][r]) {
                chk(hipMemcpyAsync((uint8_t *)cs[r]->bout + soff[r][q] * ob, (const uint8_t *)cs[q]->rout + roff[q][r] * ob,
                                   (uint64_t)rc[q][r] * ob, hipMemcpyDeviceToDevice, s),
                    "loopback out");
                if (rows)
                    chk(hipMemcpyAsync((uint8_t *)cs[r]->brec + soff[r][q] * stride,
                                       (const uint8_t *)cs[q]->rrec + roff[q][r] * stride, (uint64_t)rc[q][r] * stride,
                                       hipMemcpyDeviceToDevice, s),
                        "loopback rows");
            }
    for (int r = 0; r < W; ++r) phase_unpermute(*cs[r], n[r], stride, outs[r], recs[r], s);
    return STAGE_OK;
}

}  // namespace stage
