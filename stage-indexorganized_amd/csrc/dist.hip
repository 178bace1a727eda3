// dist.hip -- multi-GPU YCSB-C front-end: route every key to shard
// MurmurHash64A(key, 8, 0) % world (misc/murmur/MurmurHash2.cpp:99-147 as the router),
// exchange keys with one RCCL all-to-all-v (grouped ncclSend/ncclRecv over xGMI), probe the
// local shard, return results with the reverse all-to-all-v and scatter them back into the
// caller's order.  The reference has no distributed layer; this is the
// build's own exchange step for the 8-GPU config.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
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
constexpr int kDefaultChunks = 4;  // sharded batches are exchanged in this many overlapped chunks

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
                                                     uint32_t *__restrict__ perm, uint32_t idx_base,
                                                     uint32_t *__restrict__ upos) {
    __shared__ uint32_t cur[kMaxWorld];
    if (threadIdx.x < (unsigned)world) cur[threadIdx.x] = offs[threadIdx.x * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        const uint32_t pos = atomicAdd(&cur[dest[i]], 1u);
        send[pos] = SendRec{keys[i], rids ? rids[i] : 0xFFFFFFFEu, 0};
        perm[pos] = idx_base + (uint32_t)i;
        // coalesced requests: where request i was sent (send / perm start at the chunk base)
        if (upos) upos[idx_base + i] = idx_base + pos;
    }
}

// ---- request coalescing of one chunk [b, b + len): the chunk's keys are radix-sorted with
// their chunk positions; a sorted entry starts a request when its key or read id differs from
// its predecessor's; requests are numbered by an inclusive scan and packed at [b, b + nu).
__global__ void dd_iota_kernel(uint32_t *__restrict__ v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

__global__ void dd_heads(const uint64_t *__restrict__ skeys, const uint32_t *__restrict__ sidx,
                         const uint32_t *__restrict__ rids, uint64_t n, uint32_t *__restrict__ flag) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    bool head = j == 0 || skeys[j] != skeys[j - 1];
    if (!head && rids) head = rids[sidx[j]] != rids[sidx[j - 1]];
    flag[j] = head ? 1u : 0u;
}

// uidx[b + p] = b + request number of the caller position p; the request's key / read id packed
// at b + its number; nu[chunk] = the chunk's request count
__global__ void dd_pack(const uint64_t *__restrict__ skeys, const uint32_t *__restrict__ sidx,
                        const uint32_t *__restrict__ rids, const uint32_t *__restrict__ flag,
                        const uint32_t *__restrict__ useq, uint64_t n, uint32_t b, uint32_t *__restrict__ uidx,
                        uint64_t *__restrict__ ukeys, uint32_t *__restrict__ urids, uint32_t *__restrict__ nu,
                        int chunk) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t u = useq[j] - 1u, p = sidx[j];
    uidx[b + p] = b + u;
    if (flag[j]) {
        ukeys[b + u] = skeys[j];
        if (rids) urids[b + u] = rids[p];
    }
    if (j == n - 1) nu[chunk] = useq[j];
}

__global__ void unpack_keys(const SendRec *__restrict__ recv, uint64_t n, uint64_t *__restrict__ keys,
                            uint32_t *__restrict__ rids) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = recv[i].key;
    rids[i] = recv[i].rid;
}

// back in the caller's order: out[perm[p]] = bout[p] for p in [p0, p1), one wave per probe.
// Positions [q0, q1) are this rank's own keys: they never left the device, so they are read
// straight from the local probe's output (qout / qrec) instead of a received copy.
template <int R>
__global__ __launch_bounds__(256) void unpermute(const stage_probe_out_dev *__restrict__ bout, const uint8_t *__restrict__ brec,
                          const uint32_t *__restrict__ perm, uint64_t p0, uint64_t p1, uint32_t stride,
                          stage_probe_out_dev *__restrict__ out, uint8_t *__restrict__ recs, uint64_t q0, uint64_t q1,
                          const stage_probe_out_dev *__restrict__ qout, const uint8_t *__restrict__ qrec) {
    // R positions per wave pass, their rows in flight together (as expand)
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t chunks = stride >> 4;
    for (uint64_t pb = p0 + w * R; pb < p1; pb += nw * R) {
        const uint4 *sr[R];
        const uint4 *so[R];
        uint64_t dst[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint64_t p = pb + r < p1 ? pb + r : p1 - 1;
            dst[r] = perm[p];
            const bool own = p >= q0 && p < q1;
            so[r] = reinterpret_cast<const uint4 *>(own ? qout + (p - q0) : bout + p);
            sr[r] = reinterpret_cast<const uint4 *>(own ? qrec + (p - q0) * (uint64_t)stride : brec + p * (uint64_t)stride);
        }
        if (lane < 2 * R) {
            const int r = lane >> 1;
            const uint4 *src = so[0];
            uint64_t d = dst[0];
#pragma unroll
            for (int k = 1; k < R; ++k)
                if (r == k) src = so[k], d = dst[k];
            if (pb + r < p1) reinterpret_cast<uint4 *>(out + d)[lane & 1] = src[lane & 1];
        }
        if (recs) {
            for (uint32_t c0 = 0; c0 < chunks; c0 += 64) {
                const uint32_t c = c0 + lane;
                uint4 v[R];
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = c < chunks ? sr[r][c] : uint4{0, 0, 0, 0};
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (c < chunks && pb + r < p1) reinterpret_cast<uint4 *>(recs + dst[r] * stride)[c] = v[r];
            }
        }
    }
}

// coalesced requests back in the caller's order: caller position o takes the result of its
// request, sent from position p = upos[uidx[o]] (own requests read in place, as unpermute).
// A wave copies R caller positions per pass with their R source rows in flight together.
template <int R>
__global__ __launch_bounds__(256) void expand(const stage_probe_out_dev *__restrict__ bout, const uint8_t *__restrict__ brec,
                       const uint32_t *__restrict__ uidx, const uint32_t *__restrict__ upos, uint64_t o0, uint64_t o1,
                       uint32_t stride, stage_probe_out_dev *__restrict__ out, uint8_t *__restrict__ recs, uint64_t q0,
                       uint64_t q1, const stage_probe_out_dev *__restrict__ qout, const uint8_t *__restrict__ qrec) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t chunks = stride >> 4;
    for (uint64_t ob = o0 + w * R; ob < o1; ob += nw * R) {
        const uint4 *sr[R];
        const uint4 *so[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint64_t o = ob + r < o1 ? ob + r : o1 - 1;
            const uint64_t p = upos[uidx[o]];
            const bool own = p >= q0 && p < q1;
            so[r] = reinterpret_cast<const uint4 *>(own ? qout + (p - q0) : bout + p);
            sr[r] = reinterpret_cast<const uint4 *>(own ? qrec + (p - q0) * (uint64_t)stride : brec + p * (uint64_t)stride);
        }
        // status records: lanes 2r, 2r+1 copy position r's two halves
        if (lane < 2 * R) {
            const int r = lane >> 1;
            const uint4 *src = so[0];
#pragma unroll
            for (int k = 1; k < R; ++k)
                if (r == k) src = so[k];
            if (ob + r < o1) reinterpret_cast<uint4 *>(out + ob + r)[lane & 1] = src[lane & 1];
        }
        if (recs) {
            for (uint32_t c0 = 0; c0 < chunks; c0 += 64) {
                const uint32_t c = c0 + lane;
                uint4 v[R];
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = c < chunks ? sr[r][c] : uint4{0, 0, 0, 0};
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (c < chunks && ob + r < o1) reinterpret_cast<uint4 *>(recs + (ob + r) * stride)[c] = v[r];
            }
        }
    }
}

// reply mode "owner": the row stays in the owner's result buffer; the status record carries
// its owner-local index in the meta_hi word (stage_hip.h: STAGE_REPLY_OWNER)
__global__ void tag_rows(stage_probe_out_dev *__restrict__ out, uint64_t m, uint32_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i].w[7] = base + (uint32_t)i;
}

void grow(void *&p, uint64_t bytes) {
    if (p) chk(hipFree(p), "hipFree");
    p = nullptr;
    chk(hipMalloc(&p, bytes ? bytes : 16), "hipMalloc");
}

}  // namespace

ShardComm::~ShardComm() {
    if (cs) (void)hipStreamSynchronize(cs), (void)hipStreamDestroy(cs);
    if (us) (void)hipStreamSynchronize(us), (void)hipStreamDestroy(us);
    for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    if (comm) ncclCommDestroy((ncclComm_t)comm);
    for (void *p : {dest, cursor, perm, send, recv, rout, rrec, bout, brec, cnt, lkeys, lrids, dd_skeys, dd_iota,
                    dd_sidx, dd_flag, dd_useq, uidx, ukeys, urids, upos, dd_cub, dd_nu})
        if (p) (void)hipFree(p);
}

bool shard_default_dedupe() {
    const char *e = std::getenv("STAGE_SHARD_DEDUPE");
    return !(e && e[0] == '0');
}

int shard_unique_id(uint8_t *id128) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    nchk(ncclGetUniqueId(&id), "ncclGetUniqueId");
    std::memcpy(id128, &id, 128);
    return STAGE_OK;
}

static void init_common(ShardComm &c, int rank, int world, int chunks) {
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
    if (chunks < 1 || chunks > 64) throw std::invalid_argument("chunks must be 1..64");
    c.rank = rank;
    c.world = world;
    c.chunks = chunks;
    c.dedupe = shard_default_dedupe();
    grow(c.cnt, 4ull * sizeof(uint32_t) * (uint64_t)world * chunks);
    grow(c.cursor, (2ull * world * kRouteBlocks + 16) * sizeof(uint32_t));
    chk(hipStreamCreateWithFlags(&c.cs, hipStreamNonBlocking), "comm stream");
    chk(hipStreamCreateWithFlags(&c.us, hipStreamNonBlocking), "unpermute stream");
    c.evs.resize(3 * chunks + 2);
    for (auto &e : c.evs) chk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
}

static int env_chunks() {
    const char *e = std::getenv("STAGE_SHARD_CHUNKS");
    return e ? std::max(1, std::min(64, std::atoi(e))) : kDefaultChunks;
}

int shard_default_chunks() { return env_chunks(); }

int shard_init(ShardComm &c, const uint8_t *id128, int rank, int world, int chunks) {
    init_common(c, rank, world, chunks > 0 ? chunks : env_chunks());
    ncclUniqueId id;
    std::memcpy(&id, id128, 128);
    ncclComm_t comm;
    nchk(ncclCommInitRank(&comm, world, id, rank), "ncclCommInitRank");
    c.comm = comm;
    return STAGE_OK;
}

int shard_init_loopback(ShardComm &c, int rank, int world, int chunks) {
    init_common(c, rank, world, chunks > 0 ? chunks : env_chunks());
    c.comm = nullptr;
    return STAGE_OK;
}

// ---- the plan of one sharded probe, shared by the RCCL path and the loopback rehearsal.
// The caller's batch is cut into C chunks (C is the same on every rank, fixed at init, so the
// ranks issue matching transfers).  Chunk i's keys are routed into send/perm positions
// [cb_i, cb_{i+1}), grouped by destination; what arrives lands in recv positions
// [rb_i, rb_{i+1}), grouped by source.  All offsets are absolute.
struct Plan {
    int W = 1, C = 1;
    std::vector<uint64_t> cb, rb;           // chunk bases (send side / receive side), C+1
    std::vector<uint32_t> sc, rc;           // [i*W + r] counts sent to / received from r
    std::vector<uint64_t> soff, roff;       // [i*(W+1) + r] absolute segment starts
    bool dedupe = false;                    // chunk i routes its coalesced requests [cb_i, cb_i + nu_i)
    uint64_t m() const { return rb[C]; }
};

// route every chunk (caller stream), return the send counts [C][W] (host, synchronised)
static void plan_route(ShardComm &c, Plan &P, const uint64_t *d_keys, const uint32_t *d_rids, uint64_t n,
                       uint32_t stride, hipStream_t s) {
    const int W = c.world, C = c.chunks;
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
    P.W = W;
    P.C = C;
    P.cb.resize(C + 1);
    for (int i = 0; i <= C; ++i) P.cb[i] = n * (uint64_t)i / (uint64_t)C;
    P.dedupe = c.dedupe && n > 0 && n < (1ull << 31);
    // what is routed: the caller's keys, or each chunk's coalesced requests packed at its base
    const uint64_t *rkeys = d_keys;
    const uint32_t *rrids = d_rids;
    std::vector<uint64_t> rlen(C);
    for (int i = 0; i < C; ++i) rlen[i] = P.cb[i + 1] - P.cb[i];
    if (P.dedupe) {
        if (c.dd_cap < c.cap_local) {
            const uint64_t cap = c.cap_local;
            grow(c.dd_skeys, cap * 8);
            grow(c.dd_iota, cap * 4);
            grow(c.dd_sidx, cap * 4);
            grow(c.dd_flag, cap * 4);
            grow(c.dd_useq, cap * 4);
            grow(c.uidx, cap * 4);
            grow(c.ukeys, cap * 8);
            grow(c.urids, cap * 4);
            grow(c.upos, cap * 4);
            grow(c.dd_nu, 64 * 4);
            size_t sb = 0, cb = 0;
            chk(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                                   (uint32_t *)nullptr, (uint32_t *)nullptr, (int)cap, 0, 64, s),
                "sort size");
            chk(hipcub::DeviceScan::InclusiveSum(nullptr, cb, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)cap, s),
                "scan size");
            c.dd_cub_bytes = std::max(sb, cb);
            grow(c.dd_cub, c.dd_cub_bytes);
            c.dd_cap = cap;
        }
        uint32_t *nu = (uint32_t *)c.dd_nu;
        chk(hipMemsetAsync(nu, 0, 64 * 4, s), "memset nu");
        uint32_t *iota = (uint32_t *)c.dd_iota, *sidx = (uint32_t *)c.dd_sidx, *flag = (uint32_t *)c.dd_flag,
                 *useq = (uint32_t *)c.dd_useq;
        uint64_t *skeys = (uint64_t *)c.dd_skeys;
        const uint64_t maxlen = *std::max_element(rlen.begin(), rlen.end());
        dd_iota_kernel<<<(unsigned)((maxlen + 255) / 256), 256, 0, s>>>(iota, maxlen);
        for (int i = 0; i < C; ++i) {
            const uint64_t b = P.cb[i], len = rlen[i];
            if (!len) continue;
            const unsigned nb = (unsigned)((len + 255) / 256);
            const uint32_t *cr = d_rids ? d_rids + b : nullptr;
            size_t bytes = c.dd_cub_bytes;
            chk(hipcub::DeviceRadixSort::SortPairs(c.dd_cub, bytes, d_keys + b, skeys, iota, sidx, (int)len, 0, 64, s),
                "dedupe sort");
            dd_heads<<<nb, 256, 0, s>>>(skeys, sidx, cr, len, flag);
            bytes = c.dd_cub_bytes;
            chk(hipcub::DeviceScan::InclusiveSum(c.dd_cub, bytes, flag, useq, (int)len, s), "dedupe scan");
            dd_pack<<<nb, 256, 0, s>>>(skeys, sidx, cr, flag, useq, len, (uint32_t)b, (uint32_t *)c.uidx,
                                       (uint64_t *)c.ukeys, (uint32_t *)c.urids, nu, i);
        }
        chk(hipGetLastError(), "dedupe");
        std::vector<uint32_t> hn(C);
        chk(hipMemcpyAsync(hn.data(), nu, C * 4, hipMemcpyDeviceToHost, s), "nu d2h");
        chk(hipStreamSynchronize(s), "sync");
        for (int i = 0; i < C; ++i) {
            if (hn[i] > rlen[i]) throw std::runtime_error("dedupe: more requests than keys");
            rlen[i] = hn[i];
        }
        rkeys = (const uint64_t *)c.ukeys;
        rrids = d_rids ? (const uint32_t *)c.urids : nullptr;
    }
    uint32_t *counts = (uint32_t *)c.cnt;  // [C][W] send counts
    uint32_t *blk = (uint32_t *)c.cursor, *offs = blk + (uint64_t)W * kRouteBlocks;
    chk(hipMemsetAsync(counts, 0, (uint64_t)C * W * sizeof(uint32_t), s), "memset counts");
    for (int i = 0; i < C; ++i) {
        const uint64_t b = P.cb[i], len = rlen[i];
        if (!len) continue;
        route_hist<<<kRouteBlocks, 256, 0, s>>>(rkeys + b, len, W, (uint8_t *)c.dest + b, blk);
        route_scan<<<1, 1024, 0, s>>>(blk, (uint32_t)(W * kRouteBlocks), W, kRouteBlocks, offs, counts + i * W);
        route_scatter<<<kRouteBlocks, 256, 0, s>>>(rkeys + b, rrids ? rrids + b : nullptr, len, W,
                                                   (const uint8_t *)c.dest + b, offs, (SendRec *)c.send + b,
                                                   (uint32_t *)c.perm + b, (uint32_t)b,
                                                   P.dedupe ? (uint32_t *)c.upos : nullptr);
    }
    chk(hipGetLastError(), "route");
    P.sc.resize((size_t)C * W);
    chk(hipMemcpyAsync(P.sc.data(), counts, (uint64_t)C * W * 4, hipMemcpyDeviceToHost, s), "counts d2h");
    chk(hipStreamSynchronize(s), "sync");
    P.soff.assign((size_t)C * (W + 1), 0);
    for (int i = 0; i < C; ++i) {
        P.soff[i * (W + 1)] = P.cb[i];
        for (int r = 0; r < W; ++r) P.soff[i * (W + 1) + r + 1] = P.soff[i * (W + 1) + r] + P.sc[i * W + r];
    }
    c.last_n = n;
    c.last_routed = c.last_remote = 0;
    for (int i = 0; i < C; ++i)
        for (int r = 0; r < W; ++r) {
            c.last_routed += P.sc[(size_t)i * W + r];
            if (r != c.rank) c.last_remote += P.sc[(size_t)i * W + r];
        }
}

// receive side of the plan from rc (filled by the transport's count exchange)
static void plan_receive(ShardComm &c, Plan &P, uint32_t stride) {
    const int W = P.W, C = P.C;
    P.rb.assign(C + 1, 0);
    P.roff.assign((size_t)C * (W + 1), 0);
    for (int i = 0; i < C; ++i) {
        P.roff[i * (W + 1)] = P.rb[i];
        for (int r = 0; r < W; ++r) P.roff[i * (W + 1) + r + 1] = P.roff[i * (W + 1) + r] + P.rc[i * W + r];
        P.rb[i + 1] = P.roff[i * (W + 1) + W];
    }
    const uint64_t m = P.m();
    if (m > c.cap_remote) {
        const uint64_t cap = m + m / 8 + 1024;
        grow(c.recv, cap * sizeof(SendRec));
        grow(c.rout, cap * sizeof(stage_probe_out_dev));
        grow(c.rrec, cap * stride);
        grow(c.lkeys, cap * 8);
        grow(c.lrids, cap * 4);
        c.cap_remote = cap;
    }
}

// probe what arrived in chunk i
static void chunk_probe(ShardComm &c, const Plan &P, int i, const DevTable &t, const ProbeTuning &tune, bool rows,
                        bool tag, hipStream_t s) {
    const uint64_t b = P.rb[i], m = P.rb[i + 1] - b;
    if (!m) return;
    uint64_t *lk = (uint64_t *)c.lkeys + b;
    uint32_t *lr = (uint32_t *)c.lrids + b;
    unpack_keys<<<(unsigned)((m + 255) / 256), 256, 0, s>>>((const SendRec *)c.recv + b, m, lk, lr);
    chk(launch_probe(t, lk, nullptr, lr, nullptr, m, (stage_probe_out_dev *)c.rout + b,
                     rows ? (uint8_t *)c.rrec + b * (uint64_t)t.stride : nullptr, s, tune),
        "probe");
    if (tag) tag_rows<<<(unsigned)((m + 255) / 256), 256, 0, s>>>((stage_probe_out_dev *)c.rout + b, m, (uint32_t)b);
}

static void chunk_unpermute(ShardComm &c, const Plan &P, int i, uint32_t stride, stage_probe_out_dev *d_out,
                            uint8_t *d_recs, hipStream_t s) {
    const uint64_t p0 = P.cb[i], p1 = P.cb[i + 1];
    const int W = P.W, me = c.rank;
    const uint64_t q0 = P.soff[(size_t)i * (W + 1) + me], q1 = P.soff[(size_t)i * (W + 1) + me + 1];
    const uint64_t ro = P.roff[(size_t)i * (W + 1) + me];  // where the local probe wrote them
    if (P.dedupe) {
        constexpr int R = 4;
        if (p1 > p0)
            expand<R><<<(unsigned)std::min<uint64_t>((p1 - p0 + 4 * R - 1) / (4 * R), 8192), 256, 0, s>>>(
                (const stage_probe_out_dev *)c.bout, (const uint8_t *)c.brec, (const uint32_t *)c.uidx,
                (const uint32_t *)c.upos, p0, p1, stride, d_out, d_recs, q0, q1, (const stage_probe_out_dev *)c.rout + ro,
                (const uint8_t *)c.rrec + ro * stride);
        chk(hipGetLastError(), "expand");
        return;
    }
    constexpr int R = 4;
    if (p1 > p0)
        unpermute<R><<<(unsigned)std::min<uint64_t>((p1 - p0 + 4 * R - 1) / (4 * R), 8192), 256, 0, s>>>(
            (const stage_probe_out_dev *)c.bout, (const uint8_t *)c.brec, (const uint32_t *)c.perm, p0, p1, stride,
            d_out, d_recs, q0, q1, (const stage_probe_out_dev *)c.rout + ro, (const uint8_t *)c.rrec + ro * stride);
    chk(hipGetLastError(), "unpermute");
}

// RCCL path.  Streams: the caller's stream s routes and probes; c.cs carries the RCCL
// transfers; c.us un-permutes.  Order: all key exchanges first (16 B/key), then for each
// chunk the probe (s) and, as soon as it is done, its result exchange (cs) -- so the return
// of chunk i over xGMI overlaps the probe of chunk i+1 in HBM -- and its un-permutation (us).
int shard_probe(ShardComm &c, const DevTable &t, const ProbeTuning &tune, const uint64_t *d_keys,
                const uint32_t *d_rids, uint64_t n, stage_probe_out_dev *d_out, uint8_t *d_recs, int reply,
                hipStream_t s) {
    if (!c.comm) throw std::invalid_argument("not an RCCL communicator");
    const bool owner = reply == STAGE_REPLY_OWNER;
    if (owner) d_recs = nullptr;  // rows stay on the owner
    c.owner_rows = 0;
    const int W = c.world, C = c.chunks;
    const uint32_t stride = t.stride;
    ncclComm_t comm = (ncclComm_t)c.comm;
    Plan P;
    plan_route(c, P, d_keys, d_rids, n, stride, s);
    // count exchange: peer-major [W][C] so one all-to-all of C counts per peer carries all chunks
    uint32_t *cnt = (uint32_t *)c.cnt, *sendT = cnt + (uint64_t)C * W, *recvT = sendT + (uint64_t)C * W;
    std::vector<uint32_t> hT((size_t)C * W);
    for (int i = 0; i < C; ++i)
        for (int r = 0; r < W; ++r) hT[(size_t)r * C + i] = P.sc[(size_t)i * W + r];
    chk(hipMemcpyAsync(sendT, hT.data(), hT.size() * 4, hipMemcpyHostToDevice, s), "counts h2d");
    nchk(ncclAllToAll(sendT, recvT, (size_t)C, ncclUint32, comm, s), "ncclAllToAll counts");
    chk(hipMemcpyAsync(hT.data(), recvT, hT.size() * 4, hipMemcpyDeviceToHost, s), "counts d2h");
    chk(hipStreamSynchronize(s), "sync");
    P.rc.resize((size_t)C * W);
    for (int i = 0; i < C; ++i)
        for (int r = 0; r < W; ++r) P.rc[(size_t)i * W + r] = hT[(size_t)r * C + i];
    plan_receive(c, P, stride);
    hipEvent_t *ev_keys = c.evs.data(), *ev_probe = ev_keys + C, *ev_res = ev_probe + C, ev_start = ev_res[C];
    // the comm stream starts after the routing (done: s was synchronised) -- keys of all chunks
    for (int i = 0; i < C; ++i) {
        nchk(ncclGroupStart(), "group");
        for (int r = 0; r < W; ++r) {
            const uint32_t sn = P.sc[(size_t)i * W + r], rn = P.rc[(size_t)i * W + r];
            if (sn)
                nchk(ncclSend((const SendRec *)c.send + P.soff[(size_t)i * (W + 1) + r], (uint64_t)sn * sizeof(SendRec),
                              ncclUint8, r, comm, c.cs),
                     "send keys");
            if (rn)
                nchk(ncclRecv((SendRec *)c.recv + P.roff[(size_t)i * (W + 1) + r], (uint64_t)rn * sizeof(SendRec),
                              ncclUint8, r, comm, c.cs),
                     "recv keys");
        }
        nchk(ncclGroupEnd(), "group end");
        chk(hipEventRecord(ev_keys[i], c.cs), "event");
    }
    const uint64_t ob = sizeof(stage_probe_out_dev);
    for (int i = 0; i < C; ++i) {
        chk(hipStreamWaitEvent(s, ev_keys[i], 0), "wait keys");
        chunk_probe(c, P, i, t, tune, owner || d_recs != nullptr, owner, s);
        chk(hipEventRecord(ev_probe[i], s), "event");
        chk(hipStreamWaitEvent(c.cs, ev_probe[i], 0), "wait probe");
        nchk(ncclGroupStart(), "group");
        for (int r = 0; r < W; ++r) {
            if (r == c.rank) continue;  // own results are read in place by the un-permutation
            const uint32_t sn = P.sc[(size_t)i * W + r], rn = P.rc[(size_t)i * W + r];
            const uint64_t so = P.soff[(size_t)i * (W + 1) + r], ro = P.roff[(size_t)i * (W + 1) + r];
            if (rn) {
                nchk(ncclSend((const uint8_t *)c.rout + ro * ob, (uint64_t)rn * ob, ncclUint8, r, comm, c.cs), "send out");
                if (d_recs)
                    nchk(ncclSend((const uint8_t *)c.rrec + ro * stride, (uint64_t)rn * stride, ncclUint8, r, comm, c.cs),
                         "send rows");
            }
            if (sn) {
                nchk(ncclRecv((uint8_t *)c.bout + so * ob, (uint64_t)sn * ob, ncclUint8, r, comm, c.cs), "recv out");
                if (d_recs)
                    nchk(ncclRecv((uint8_t *)c.brec + so * stride, (uint64_t)sn * stride, ncclUint8, r, comm, c.cs),
                         "recv rows");
            }
        }
        nchk(ncclGroupEnd(), "group end");
        chk(hipEventRecord(ev_res[i], c.cs), "event");
        chk(hipStreamWaitEvent(c.us, ev_res[i], 0), "wait results");
        chunk_unpermute(c, P, i, stride, d_out, d_recs, c.us);
    }
    // the caller's stream completes after the last un-permutation
    chk(hipEventRecord(ev_start, c.us), "event");
    chk(hipStreamWaitEvent(s, ev_start, 0), "join");
    if (owner) c.owner_rows = P.m();
    return STAGE_OK;
}

// The same plan for W shards held by one process on one device, with device-to-device copies
// where shard_probe has RCCL transfers (same chunks, same offsets), all on one stream.
int shard_probe_loopback(const std::vector<ShardComm *> &cs, const std::vector<const DevTable *> &ts,
                         const ProbeTuning &tune, const std::vector<const uint64_t *> &keys,
                         const std::vector<const uint32_t *> &rids, const std::vector<uint64_t> &n,
                         const std::vector<stage_probe_out_dev *> &outs, std::vector<uint8_t *> recs, int reply,
                         hipStream_t s) {
    const int W = (int)cs.size();
    const uint32_t stride = ts[0]->stride;
    const bool owner = reply == STAGE_REPLY_OWNER;
    if (owner)
        for (auto &r : recs) r = nullptr;
    for (int r = 0; r < W; ++r)
        if (ts[r]->stride != stride || cs[r]->world != W || cs[r]->rank != r || cs[r]->chunks != cs[0]->chunks)
            throw std::invalid_argument("loopback shards disagree on stride / rank / world / chunks");
    const int C = cs[0]->chunks;
    const bool rows = recs[0] != nullptr;
    std::vector<Plan> P(W);
    for (int r = 0; r < W; ++r) plan_route(*cs[r], P[r], keys[r], rids[r], n[r], stride, s);
    for (int r = 0; r < W; ++r) {
        P[r].rc.resize((size_t)C * W);
        for (int i = 0; i < C; ++i)
            for (int q = 0; q < W; ++q) P[r].rc[(size_t)i * W + q] = P[q].sc[(size_t)i * W + r];
        plan_receive(*cs[r], P[r], stride);
    }
    auto copy = [&](void *dst, const void *src, uint64_t bytes, const char *what) {
        if (bytes) chk(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s), what);
    };
    for (int i = 0; i < C; ++i)  // keys: q's chunk-i segment for r -> r's chunk-i segment from q
        for (int r = 0; r < W; ++r)
            for (int q = 0; q < W; ++q)
                copy((SendRec *)cs[r]->recv + P[r].roff[(size_t)i * (W + 1) + q],
                     (const SendRec *)cs[q]->send + P[q].soff[(size_t)i * (W + 1) + r],
                     (uint64_t)P[q].sc[(size_t)i * W + r] * sizeof(SendRec), "loopback keys");
    const uint64_t ob = sizeof(stage_probe_out_dev);
    for (int i = 0; i < C; ++i) {
        for (int r = 0; r < W; ++r) chunk_probe(*cs[r], P[r], i, *ts[r], tune, rows || owner, owner, s);
        for (int q = 0; q < W; ++q)  // results: owner q's chunk-i segment for r -> r's chunk-i slots of q
            for (int r = 0; r < W; ++r) {
                if (r == q) continue;  // as shard_probe: own results are read in place
                const uint64_t cnt = P[q].rc[(size_t)i * W + r];
                const uint64_t ro = P[q].roff[(size_t)i * (W + 1) + r], so = P[r].soff[(size_t)i * (W + 1) + q];
                copy((uint8_t *)cs[r]->bout + so * ob, (const uint8_t *)cs[q]->rout + ro * ob, cnt * ob, "loopback out");
                if (rows)
                    copy((uint8_t *)cs[r]->brec + so * stride, (const uint8_t *)cs[q]->rrec + ro * stride,
                         cnt * stride, "loopback rows");
            }
        for (int r = 0; r < W; ++r) chunk_unpermute(*cs[r], P[r], i, stride, outs[r], recs[r], s);
    }
    for (int r = 0; r < W; ++r) cs[r]->owner_rows = owner ? P[r].m() : 0;
    return STAGE_OK;
}

}  // namespace stage
