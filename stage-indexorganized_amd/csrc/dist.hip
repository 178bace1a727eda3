// dist.hip -- multi-GPU YCSB-C front-end: route every key to shard
// MurmurHash64A(key, 8, 0) % world (misc/murmur/MurmurHash2.cpp:99-147 as the router),
// exchange keys with one RCCL all-to-all-v (grouped ncclSend/ncclRecv over xGMI), probe the
// local shard, return results with the reverse all-to-all-v and fan them out into the caller's
// order.  The reference has no distributed layer; this is the build's own
// exchange step for the 8-GPU config.  Result semantics per key are those of the single-table
// probe (BTree::Read + IndexScanExecutor visibility, include/execute/executor.h:374-454).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstdio>
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

struct alignas(16) SendRec {
    uint64_t key;
    uint32_t rid;
    uint32_t first;  // the request's first caller position (STAGE_REPLY_DIRECT's row destination)
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
// scatter that claims positions with LDS atomics inside each block's range.  The number of
// keys routed is read on the device (n_dev: the chunk's coalesced request count), so the
// host does not wait for the coalescing before it enqueues the routing.
constexpr int kRouteBlocks = 1024;
constexpr int kMaxWorld = 64;
constexpr int kMaxChunks = 64;
constexpr int kDefaultChunks = 4;  // sharded batches are exchanged in this many overlapped chunks
// caller positions served by one coalesced request at most: a hot key's run is cut into
// requests of <= 64 callers, so no single probe or fan-out copy stores more than 64 rows
constexpr uint32_t kFanCap = 64;

// chunk i of C over the routed items [0, total): [total*i/C, total*(i+1)/C); total is the batch
// size, or the coalesced request count read on the device (total_dev)
struct ChunkSpan {
    uint64_t lo, hi;
};
__device__ __forceinline__ ChunkSpan chunk_span(uint64_t total_max, const uint32_t *total_dev, int i, int C) {
    const uint64_t total = total_dev ? *total_dev : total_max;
    return ChunkSpan{total * (uint64_t)i / (uint64_t)C, total * (uint64_t)(i + 1) / (uint64_t)C};
}

__global__ __launch_bounds__(256) void route_hist(const uint64_t *__restrict__ keys, uint64_t total_max,
                                                  const uint32_t *__restrict__ total_dev, int chunk, int nchunks,
                                                  int world, uint8_t *__restrict__ dest, uint32_t *__restrict__ blk) {
    __shared__ uint32_t h[kMaxWorld];
    if (threadIdx.x < (unsigned)world) h[threadIdx.x] = 0;
    __syncthreads();
    const ChunkSpan cs = chunk_span(total_max, total_dev, chunk, nchunks);
    const uint64_t n = cs.hi - cs.lo;
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = cs.lo + b0 + threadIdx.x; i < cs.lo + b1; i += blockDim.x) {
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

// send[lo + pos] = item i's key record (i in the chunk [lo, hi), pos its place in the chunk,
// grouped by destination) with its first caller position; perm[lo + pos] = i; fan[lo + pos] =
// the caller positions it serves: urange[i] (coalesced: a run of flist) or {i, i + 1} (one
// caller, the item itself)
__global__ __launch_bounds__(256) void route_scatter(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ rids,
                                                     uint64_t total_max, const uint32_t *__restrict__ total_dev,
                                                     int chunk, int nchunks, int world,
                                                     const uint8_t *__restrict__ dest, const uint32_t *__restrict__ offs,
                                                     SendRec *__restrict__ send, uint32_t *__restrict__ perm,
                                                     uint32_t *__restrict__ upos, const FanRange *__restrict__ urange,
                                                     const uint32_t *__restrict__ flist, FanRange *__restrict__ fan) {
    __shared__ uint32_t cur[kMaxWorld];
    if (threadIdx.x < (unsigned)world) cur[threadIdx.x] = offs[threadIdx.x * gridDim.x + blockIdx.x];
    __syncthreads();
    const ChunkSpan cs = chunk_span(total_max, total_dev, chunk, nchunks);
    const uint64_t n = cs.hi - cs.lo;
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = cs.lo + b0 + threadIdx.x; i < cs.lo + b1; i += blockDim.x) {
        const uint32_t pos = (uint32_t)cs.lo + atomicAdd(&cur[dest[i]], 1u);
        const uint32_t idx = (uint32_t)i;
        const FanRange fr = urange ? urange[idx] : FanRange{idx, idx + 1};
        send[pos] = SendRec{keys[i], rids ? rids[i] : 0xFFFFFFFEu, urange ? flist[fr.lo] : idx};
        perm[pos] = idx;
        if (upos) upos[idx] = pos;  // where request idx was sent (owner-reply expand)
        fan[pos] = fr;
    }
}

// [C][W] send counts -> [W][C] (peer-major: one all-to-all of C counts per peer)
__global__ void transpose_counts(const uint32_t *__restrict__ cw, int C, int W, uint32_t *__restrict__ wc) {
    for (int k = threadIdx.x; k < C * W; k += blockDim.x) wc[(k % W) * C + k / W] = cw[k];
}

// ---- request coalescing of the whole batch: its keys are radix-sorted with their positions (by
// (key, read id): read ids first, then a stable sort by key); a sorted entry starts a request
// when its key or read id differs from its predecessor's, or at every kFanCap-th sorted
// position; requests are numbered by an inclusive scan and packed at [0, nu).  The exchange
// chunks then cut the requests, not the callers: a key asked in two chunks travels once.
__global__ void dd_iota_kernel(uint32_t *__restrict__ v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

__global__ void dd_gather_keys(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ idx, uint64_t n,
                               uint64_t *__restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[j] = keys[idx[j]];
}

// Narrow sort keys (requests without read ids, coalescing width <= 32 bits): the batch's low
// 32 key bits and the positions; hi[0] |= any key's upper half, so the sorted low words stand
// for the keys themselves only when every key fits 32 bits (else the keys are gathered back
// by position -- a sort on fewer bits than the keys hold only coalesces less, see key_bits).
__global__ __launch_bounds__(256) void dd_narrow_iota(const uint64_t *__restrict__ keys, uint64_t n,
                                                      uint32_t *__restrict__ k32, uint32_t *__restrict__ iota,
                                                      uint32_t *__restrict__ hi) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t k = 0;
    if (i < n) {
        k = keys[i];
        k32[i] = (uint32_t)k;
        iota[i] = (uint32_t)i;
    }
    if (__builtin_amdgcn_ballot_w64((k >> 32) != 0) != 0 && (threadIdx.x & 63) == 0) atomicOr(hi, 1u);
}

// the key of sorted entry j: the sorted 64-bit key, or the narrow one (widened, or gathered
// by position when some key exceeds 32 bits)
struct SortedKeys {
    const uint64_t *k64;   // 64-bit sort: the sorted keys
    const uint32_t *k32;   // 32-bit sort: the sorted low words
    const uint64_t *keys;  // 32-bit sort: the caller's keys (gathered when *hi)
    const uint32_t *hi;
    __device__ __forceinline__ uint64_t at(uint64_t j, const uint32_t *sidx, bool wide) const {
        if (k64) return k64[j];
        return wide ? keys[sidx[j]] : (uint64_t)k32[j];
    }
};

__global__ void dd_heads(SortedKeys sk, const uint32_t *__restrict__ sidx,
                         const uint32_t *__restrict__ rids, uint64_t n, uint32_t cap, uint32_t *__restrict__ flag) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const bool wide = !sk.k64 && *sk.hi != 0;
    bool head = j % cap == 0 || sk.at(j, sidx, wide) != sk.at(j - 1, sidx, wide);
    if (!head && rids) head = rids[sidx[j]] != rids[sidx[j - 1]];
    flag[j] = head ? 1u : 0u;
}

// uidx[b + p] = b + request number of the caller position p (owner reply; may be null); flist[b + j] = the caller position
// of sorted entry j; urange[b + u] = request u's run [b + first, b + last + 1) of flist; the
// request's key / read id packed at b + u; nu[chunk] = the request count (the sharded probe
// coalesces its whole batch at once: b = 0, chunk 0)
__global__ void dd_pack(SortedKeys sk, const uint32_t *__restrict__ sidx,
                        const uint32_t *__restrict__ rids, const uint32_t *__restrict__ flag,
                        const uint32_t *__restrict__ useq, uint64_t n, uint32_t b, uint32_t *__restrict__ uidx,
                        uint32_t *__restrict__ flist, FanRange *__restrict__ urange, uint64_t *__restrict__ ukeys,
                        uint32_t *__restrict__ urids, uint32_t *__restrict__ nu, int chunk) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t u = useq[j] - 1u, p = sidx[j];
    if (uidx) uidx[b + p] = b + u;  // owner-reply mode only
    flist[b + j] = b + p;
    if (flag[j]) {
        ukeys[b + u] = sk.k64 ? sk.k64[j] : *sk.hi ? sk.keys[p] : (uint64_t)sk.k32[j];
        if (rids) urids[b + u] = rids[p];
        urange[b + u].lo = b + (uint32_t)j;
    }
    if (j == n - 1 || flag[j + 1]) urange[b + u].hi = b + (uint32_t)j + 1u;
    if (j == n - 1) nu[chunk] = useq[j];
}

__global__ void unpack_keys(const SendRec *__restrict__ recv, uint64_t n, uint64_t *__restrict__ keys,
                            uint32_t *__restrict__ rids, uint32_t *__restrict__ firsts) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = recv[i].key;
    rids[i] = recv[i].rid;
    if (firsts) firsts[i] = recv[i].first;
}

__device__ __forceinline__ void st_nt(u32x4 v, uint8_t *p) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p)); }

// Fan-out of results that arrived (or were probed) in request order: the result of request
// position p in [p0, p1) -- status record sout[p - p0], row srec + (p - p0) * stride -- is
// stored at each of its caller positions flist[k], k in fan[p] (flist null: k itself).  A wave
// takes R request positions per pass with their R rows in flight together, then stores each
// row once per caller (the rows are read once per request, not once per caller).
template <int R>
__global__ __launch_bounds__(256) void fan_copy(const stage_probe_out_dev *__restrict__ sout,
                                                const uint8_t *__restrict__ srec, uint64_t p0, uint64_t p1,
                                                const FanRange *__restrict__ fan, const uint32_t *__restrict__ flist,
                                                uint32_t stride, stage_probe_out_dev *__restrict__ out,
                                                uint8_t *__restrict__ recs) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t chunks = recs ? stride >> 4 : 0u;
    for (uint64_t pb = p0 + w * R; pb < p1; pb += nw * R) {
        FanRange fr[R];
        u32x4 so[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool in = pb + r < p1;
            const uint64_t q = (in ? pb + r : p1 - 1) - p0;
            fr[r] = in ? fan[pb + r] : FanRange{0u, 0u};
            so[r] = lane < 2 ? reinterpret_cast<const u32x4 *>(sout + q)[lane] : u32x4{0, 0, 0, 0};
        }
        // the first 64 caller positions of each request, in flight with the rows below
        uint32_t mine0[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t kk = fr[r].lo + lane;
            mine0[r] = kk < fr[r].hi ? (flist ? flist[kk] : kk) : 0u;
        }
        for (uint32_t c0 = 0; c0 < (chunks ? chunks : 1u); c0 += 64) {
            const uint32_t c = c0 + lane;
            u32x4 v[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint64_t q = (pb + r < p1 ? pb + r : p1 - 1) - p0;
                v[r] = c < chunks ? reinterpret_cast<const u32x4 *>(srec + q * stride)[c] : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                for (uint32_t k0 = fr[r].lo; k0 < fr[r].hi; k0 += 64) {
                    const uint32_t kk = k0 + lane;
                    const uint32_t mine = k0 == fr[r].lo ? mine0[r] : kk < fr[r].hi ? (flist ? flist[kk] : kk) : 0u;
                    const uint32_t kn = fr[r].hi - k0 < 64u ? fr[r].hi - k0 : 64u;
                    for (uint32_t k = 0; k < kn; ++k) {
                        const uint64_t pos = rl32(mine, (int)k);
                        if (c < chunks) st_nt(v[r], recs + pos * stride + c * 16u);
                        if (c0 == 0 && lane < 2) st_nt(so[r], reinterpret_cast<uint8_t *>(out + pos) + lane * 16u);
                    }
                }
            }
        }
    }
}

// STAGE_REPLY_DIRECT, the caller's side: request p in [p0, p1) was probed by its owner straight
// into caller position flist[fan[p].lo] (status record and row); its other caller positions
// flist[k], k in (fan[p].lo, fan[p].hi), take copies of that position.  A wave per R requests,
// their R rows in flight together as fan_copy; requests with one caller cost one load of fan.
template <int R>
__global__ __launch_bounds__(256) void dup_copy(uint64_t p0, uint64_t p1, const FanRange *__restrict__ fan,
                                                const uint32_t *__restrict__ flist, uint32_t stride,
                                                stage_probe_out_dev *__restrict__ out, uint8_t *__restrict__ recs) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t chunks = stride >> 4;
    for (uint64_t pb = p0 + w * R; pb < p1; pb += nw * R) {
        FanRange fr[R];
        uint32_t first[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            fr[r] = pb + r < p1 ? fan[pb + r] : FanRange{0u, 0u};
            first[r] = fr[r].hi - fr[r].lo > 1 ? flist[fr[r].lo] : 0u;
        }
        bool any = false;
#pragma unroll
        for (int r = 0; r < R; ++r) any = any || fr[r].hi - fr[r].lo > 1;
        if (!any) continue;  // wave-uniform
        uint32_t mine0[R];
        u32x4 so[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool dup = fr[r].hi - fr[r].lo > 1;
            const uint32_t kk = fr[r].lo + 1 + lane;
            mine0[r] = dup && kk < fr[r].hi ? flist[kk] : 0u;
            so[r] = dup && lane < 2 ? reinterpret_cast<const u32x4 *>(out + first[r])[lane] : u32x4{0, 0, 0, 0};
        }
        for (uint32_t c0 = 0; c0 < chunks; c0 += 64) {
            const uint32_t c = c0 + lane;
            u32x4 v[R];
#pragma unroll
            for (int r = 0; r < R; ++r)
                v[r] = fr[r].hi - fr[r].lo > 1 && c < chunks
                           ? reinterpret_cast<const u32x4 *>(recs + (uint64_t)first[r] * stride)[c]
                           : u32x4{0, 0, 0, 0};
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (fr[r].hi - fr[r].lo <= 1) continue;
                for (uint32_t k0 = fr[r].lo + 1; k0 < fr[r].hi; k0 += 64) {
                    const uint32_t kk = k0 + lane;
                    const uint32_t mine = k0 == fr[r].lo + 1 ? mine0[r] : kk < fr[r].hi ? flist[kk] : 0u;
                    const uint32_t kn = fr[r].hi - k0 < 64u ? fr[r].hi - k0 : 64u;
                    for (uint32_t k = 0; k < kn; ++k) {
                        const uint64_t pos = rl32(mine, (int)k);
                        if (c < chunks) st_nt(v[r], recs + pos * stride + c * 16u);
                        if (c0 == 0 && lane < 2) st_nt(so[r], reinterpret_cast<uint8_t *>(out + pos) + lane * 16u);
                    }
                }
            }
        }
    }
}

// owner-reply mode, back in the caller's order: out[perm[p]] = bout[p] for p in [p0, p1).
// Positions [q0, q1) are this rank's own keys: they never left the device, so they are read
// straight from the local probe's output (qout).  Status records only (rows stay on the owner).
__global__ __launch_bounds__(256) void unpermute_status(const stage_probe_out_dev *__restrict__ bout,
                                                        const uint32_t *__restrict__ perm, uint64_t p0, uint64_t p1,
                                                        stage_probe_out_dev *__restrict__ out, uint64_t q0, uint64_t q1,
                                                        const stage_probe_out_dev *__restrict__ qout) {
    const uint64_t p = p0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= p1) return;
    const bool own = p >= q0 && p < q1;
    out[perm[p]] = own ? qout[p - q0] : bout[p];
}

// owner-reply mode with coalesced requests, once every chunk is back: caller position o takes
// the status record of its request, sent from position p = upos[uidx[o]].  p's chunk i is the
// last whose base cb[i] <= p; own requests of chunk i, [q0[i], q1[i]), are read in place from
// the local probe's output (rout + ro[i]).
struct OwnSegs {
    uint32_t cb[kMaxChunks], q0[kMaxChunks], q1[kMaxChunks], ro[kMaxChunks];
    int C;
};
__global__ __launch_bounds__(256) void expand_status(const stage_probe_out_dev *__restrict__ bout,
                                                     const uint32_t *__restrict__ uidx, const uint32_t *__restrict__ upos,
                                                     uint64_t n, stage_probe_out_dev *__restrict__ out, OwnSegs own,
                                                     const stage_probe_out_dev *__restrict__ rout) {
    const uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n) return;
    const uint32_t p = upos[uidx[o]];
    int i = 0;
    while (i + 1 < own.C && own.cb[i + 1] <= p) ++i;
    const bool mine = p >= own.q0[i] && p < own.q1[i];
    out[o] = mine ? rout[own.ro[i] + (p - own.q0[i])] : bout[p];
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

unsigned blocks_for(uint64_t n, unsigned per_block) { return (unsigned)std::max<uint64_t>(1, (n + per_block - 1) / per_block); }

// The 32-bit coalescing sort (u32 keys, u32 positions): hipcub's onesweep, 8 bits a pass
// (rocprim's onesweep at 10 / 11 bits a pass -- 3 passes instead of 4 over 25-30 key bits -- was
// measured no faster, DESIGN §6, and retired).  temp == nullptr: storage size query.
hipError_t sort32(void *temp, size_t &bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                  uint32_t *vout, int n, int bits, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(temp, bytes, kin, kout, vin, vout, n, 0, bits, s);
}

}  // namespace

ShardComm::~ShardComm() {
    for (void *p : opened) (void)hipIpcCloseMemHandle(p);
    for (auto &v : dopen)
        for (void *p : v) (void)hipIpcCloseMemHandle(p);
    for (void *p : {prow[0], prow[1], hbuf})
        if (p) (void)hipFree(p);
    if (cs) (void)hipStreamSynchronize(cs), (void)hipStreamDestroy(cs);
    if (us) (void)hipStreamSynchronize(us), (void)hipStreamDestroy(us);
    if (ps) (void)hipStreamSynchronize(ps), (void)hipStreamDestroy(ps);
    for (hipEvent_t e : {ev_fork, ev_own})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    if (comm) ncclCommDestroy((ncclComm_t)comm);
    for (void *p : {dest, cursor, perm, send, recv, rout, rrec, bout, brec, cnt, lkeys, lrids, fan, dd_skeys, dd_iota,
                    dd_sidx, dd_flag, dd_useq, uidx, ukeys, urids, upos, urange, flist, dd_cub, dd_nu, ctl, lpads,
                    fdest})
        if (p) (void)hipFree(p);
    if (fdest_h) (void)hipHostFree(fdest_h);
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

// The RCCL this process runs (ncclGetVersion through the library's own binding, and the file
// that symbol resolved to) against the headers the library was compiled with.  Two RCCL builds
// can coexist in one process (e.g. PyTorch's copy); the sharded front-end refuses to run on one
// whose major.minor differs from its headers unless STAGE_RCCL_ALLOW_MISMATCH=1.
int shard_rccl_info(int *runtime_code, int *header_code, char *path, uint64_t path_len) {
    int v = 0;
    nchk(ncclGetVersion(&v), "ncclGetVersion");
    if (runtime_code) *runtime_code = v;
    if (header_code) *header_code = NCCL_VERSION_CODE;
    if (path && path_len) {
        Dl_info info{};
        const char *f = dladdr(reinterpret_cast<void *>(&ncclGetVersion), &info) && info.dli_fname ? info.dli_fname : "?";
        std::strncpy(path, f, path_len - 1);
        path[path_len - 1] = 0;
    }
    return STAGE_OK;
}

static void check_rccl_version() {
    int rt = 0, hd = 0;
    char path[512];
    shard_rccl_info(&rt, &hd, path, sizeof path);
    const char *e = std::getenv("STAGE_RCCL_ALLOW_MISMATCH");
    if (rt / 100 != hd / 100 && !(e && e[0] == '1'))
        throw std::runtime_error("RCCL " + std::to_string(rt) + " loaded from " + path + " but libstage_hip was built "
                                 "against RCCL headers " + std::to_string(hd) +
                                 " (load libstage_hip before another RCCL copy, or STAGE_RCCL_ALLOW_MISMATCH=1)");
}

static void init_common(ShardComm &c, int rank, int world, int chunks) {
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
    if (chunks < 1 || chunks > kMaxChunks) throw std::invalid_argument("chunks must be 1..64");
    c.rank = rank;
    c.world = world;
    c.chunks = chunks;
    c.dedupe = shard_default_dedupe();
    grow(c.cnt, 4ull * sizeof(uint32_t) * (uint64_t)world * chunks);
    grow(c.cursor, (2ull * world * kRouteBlocks + 16) * sizeof(uint32_t));
    chk(hipStreamCreateWithFlags(&c.cs, hipStreamNonBlocking), "comm stream");
    chk(hipStreamCreateWithFlags(&c.us, hipStreamNonBlocking), "fan-out stream");
    chk(hipStreamCreateWithFlags(&c.ps, hipStreamNonBlocking), "own-probe stream");
    chk(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming), "event");
    chk(hipEventCreateWithFlags(&c.ev_own, hipEventDisableTiming), "event");
    c.evs.resize(3 * chunks + 2);
    for (auto &e : c.evs) chk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
}

// exchange chunks: STAGE_SHARD_CHUNKS, else 4 (the result return of chunk i overlaps the probe
// of chunk i + 1), or 1 at world 1, where nothing crosses xGMI to overlap
static int env_chunks(int world) {
    const char *e = std::getenv("STAGE_SHARD_CHUNKS");
    return e ? std::max(1, std::min(kMaxChunks, std::atoi(e))) : world == 1 ? 1 : kDefaultChunks;
}

int shard_default_chunks(int world) { return env_chunks(world); }

int shard_init(ShardComm &c, const uint8_t *id128, int rank, int world, int chunks) {
    check_rccl_version();
    init_common(c, rank, world, chunks > 0 ? chunks : env_chunks(world));
    ncclUniqueId id;
    std::memcpy(&id, id128, 128);
    ncclComm_t comm;
    nchk(ncclCommInitRank(&comm, world, id, rank), "ncclCommInitRank");
    c.comm = comm;
    return STAGE_OK;
}

int shard_init_loopback(ShardComm &c, int rank, int world, int chunks) {
    init_common(c, rank, world, chunks > 0 ? chunks : env_chunks(world));
    c.comm = nullptr;
    return STAGE_OK;
}

// ---- control plane over the communicator (host values, e.g. the bench's barrier and its
// max-over-ranks step time): small allreduce / allgather of doubles on the comm stream
static double *ctl_buf(ShardComm &c, uint64_t doubles) {
    if (doubles > c.ctl_cap) {
        grow(c.ctl, doubles * sizeof(double));
        c.ctl_cap = doubles;
    }
    return (double *)c.ctl;
}

int shard_allreduce_f64(ShardComm &c, double *v, uint64_t n, int op) {
    if (!c.comm) throw std::invalid_argument("not an RCCL communicator");
    if (n == 0) return STAGE_OK;
    double *d = ctl_buf(c, n);
    const ncclRedOp_t ro = op == 1 ? ncclMax : op == 2 ? ncclMin : ncclSum;
    chk(hipMemcpyAsync(d, v, n * sizeof(double), hipMemcpyHostToDevice, c.cs), "ctl h2d");
    nchk(ncclAllReduce(d, d, n, ncclFloat64, ro, (ncclComm_t)c.comm, c.cs), "ncclAllReduce");
    chk(hipMemcpyAsync(v, d, n * sizeof(double), hipMemcpyDeviceToHost, c.cs), "ctl d2h");
    chk(hipStreamSynchronize(c.cs), "ctl sync");
    return STAGE_OK;
}

int shard_allgather_f64(ShardComm &c, const double *in, uint64_t n, double *out) {
    if (!c.comm) throw std::invalid_argument("not an RCCL communicator");
    if (n == 0) return STAGE_OK;
    double *d = ctl_buf(c, n * (uint64_t)(c.world + 1));
    chk(hipMemcpyAsync(d, in, n * sizeof(double), hipMemcpyHostToDevice, c.cs), "ctl h2d");
    nchk(ncclAllGather(d, d + n, n, ncclFloat64, (ncclComm_t)c.comm, c.cs), "ncclAllGather");
    chk(hipMemcpyAsync(out, d + n, n * (uint64_t)c.world * sizeof(double), hipMemcpyDeviceToHost, c.cs), "ctl d2h");
    chk(hipStreamSynchronize(c.cs), "ctl sync");
    return STAGE_OK;
}

// ---- the plan of one sharded probe, shared by the RCCL path and the loopback rehearsal.
// What is routed is the caller's batch, or -- coalesced -- its distinct requests (one pass over
// the whole batch, so a key asked in two chunks travels once).  The routed items [0, total) are
// cut into C chunks (C is the same on every rank, fixed at init, so the ranks issue matching
// transfers); chunk i's items [cb_i, cb_{i+1}) take send/perm positions [cb_i, cb_{i+1}),
// grouped by destination; what arrives lands in recv positions [rb_i, rb_{i+1}), grouped by
// source.  All offsets are absolute.  total is known to the host only after the count
// exchange (the coalesced count is read back with the counts).
struct Plan {
    int W = 1, C = 1;
    uint64_t n = 0, total = 0;              // caller positions, routed items
    std::vector<uint64_t> cb, rb;           // chunk bases (send side / receive side), C+1
    std::vector<uint32_t> sc, rc;           // [i*W + r] counts sent to / received from r
    std::vector<uint64_t> soff, roff;       // [i*(W+1) + r] absolute segment starts
    bool dedupe = false;                    // routed items are coalesced requests (c.dd_nu[0] of them)
    uint64_t m() const { return rb[C]; }
};

// coalescing + routing of every chunk, enqueued on the caller stream s (no host wait); the
// send counts [C][W] are left in c.cnt, the coalesced request count in c.dd_nu[0]
static void plan_route(ShardComm &c, Plan &P, const uint64_t *d_keys, const uint32_t *d_rids, uint64_t n,
                       uint32_t stride, bool owner, hipStream_t s) {
    const int W = c.world, C = c.chunks;
    if (n > 0xFFFFFFFFull) throw std::invalid_argument("batch too large");
    if (n > c.cap_local || stride != c.rec_stride) {
        const uint64_t cap = n + n / 8 + 1024;
        grow(c.dest, cap);
        grow(c.perm, cap * 4);
        grow(c.send, cap * sizeof(SendRec));
        grow(c.fan, cap * sizeof(FanRange));
        grow(c.bout, cap * sizeof(stage_probe_out_dev));
        grow(c.brec, cap * stride);
        c.cap_local = cap;
        c.rec_stride = stride;
        c.cap_remote = 0;  // remote buffers follow the stride too
    }
    P.W = W;
    P.C = C;
    P.n = n;
    P.total = n;
    P.dedupe = c.dedupe && n > 0 && n < (1ull << 31);
    // what is routed: the caller's keys, or the coalesced requests packed at [0, nu)
    const uint64_t *rkeys = d_keys;
    const uint32_t *rrids = d_rids;
    const uint32_t *nu = nullptr;
    if (!c.dd_nu) grow(c.dd_nu, 64 * 4);
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
            grow(c.urange, cap * sizeof(FanRange));
            grow(c.flist, cap * 4);
            c.dd_cap = cap;
            c.dd_cub_items = 0;
        }
        // temporary storage of the sorts and the scan
        if (n > c.dd_cub_items) {
            const int items = (int)n;
            size_t sb = 0, sr = 0, cb = 0, s32 = 0;
            chk(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                                   (uint32_t *)nullptr, (uint32_t *)nullptr, items, 0, 64, s),
                "sort size");
            chk(hipcub::DeviceRadixSort::SortPairs(nullptr, sr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                   (uint32_t *)nullptr, (uint32_t *)nullptr, items, 0, 32, s),
                "rid sort size");
            chk(sort32(nullptr, s32, nullptr, nullptr, nullptr, nullptr, items, 32, s), "narrow sort size");
            chk(hipcub::DeviceScan::InclusiveSum(nullptr, cb, (uint32_t *)nullptr, (uint32_t *)nullptr, items, s),
                "scan size");
            c.dd_cub_bytes = std::max(std::max(std::max(sb, sr), cb), s32);
            grow(c.dd_cub, c.dd_cub_bytes);
            c.dd_cub_items = n;
        }
        uint32_t *nuw = (uint32_t *)c.dd_nu;
        uint32_t *iota = (uint32_t *)c.dd_iota, *sidx = (uint32_t *)c.dd_sidx, *flag = (uint32_t *)c.dd_flag,
                 *useq = (uint32_t *)c.dd_useq;
        uint64_t *skeys = (uint64_t *)c.dd_skeys;
        const int bits = c.key_bits >= 1 && c.key_bits <= 64 ? c.key_bits : 64;
        const unsigned nb = blocks_for(n, 256);
        size_t bytes = c.dd_cub_bytes;
        SortedKeys sk{skeys, nullptr, nullptr, nullptr};
        if (!d_rids && bits <= 32) {
            // narrow sort: low words (in flag until the heads overwrite it) + positions; the
            // sorted low words land in skeys' storage
            uint32_t *k32 = flag, *sk32 = reinterpret_cast<uint32_t *>(skeys), *hi = nuw + 32;
            chk(hipMemsetAsync(hi, 0, 4, s), "memset hi");
            dd_narrow_iota<<<nb, 256, 0, s>>>(d_keys, n, k32, iota, hi);
            chk(sort32(c.dd_cub, bytes, k32, sk32, iota, sidx, (int)n, bits, s), "dedupe narrow sort");
            sk = SortedKeys{nullptr, sk32, d_keys, hi};
        } else if (d_rids) {
            dd_iota_kernel<<<nb, 256, 0, s>>>(iota, n);
            // (key, read id) order: sort by read id, then stably by key (LSD radix sorts are
            // stable); flag / useq serve as scratch until the heads are computed
            uint32_t *srid = flag, *sidx1 = useq;
            uint64_t *gk = (uint64_t *)c.ukeys;  // the packed keys are written after this sort
            chk(hipcub::DeviceRadixSort::SortPairs(c.dd_cub, bytes, d_rids, srid, iota, sidx1, (int)n, 0, 32, s),
                "dedupe rid sort");
            dd_gather_keys<<<nb, 256, 0, s>>>(d_keys, sidx1, n, gk);
            bytes = c.dd_cub_bytes;
            chk(hipcub::DeviceRadixSort::SortPairs(c.dd_cub, bytes, gk, skeys, sidx1, sidx, (int)n, 0, bits, s),
                "dedupe key sort");
        } else {
            dd_iota_kernel<<<nb, 256, 0, s>>>(iota, n);
            chk(hipcub::DeviceRadixSort::SortPairs(c.dd_cub, bytes, d_keys, skeys, iota, sidx, (int)n, 0, bits, s),
                "dedupe sort");
        }
        dd_heads<<<nb, 256, 0, s>>>(sk, sidx, d_rids, n, kFanCap, flag);
        bytes = c.dd_cub_bytes;
        chk(hipcub::DeviceScan::InclusiveSum(c.dd_cub, bytes, flag, useq, (int)n, s), "dedupe scan");
        dd_pack<<<nb, 256, 0, s>>>(sk, sidx, d_rids, flag, useq, n, 0u, owner ? (uint32_t *)c.uidx : nullptr,
                                   (uint32_t *)c.flist, (FanRange *)c.urange, (uint64_t *)c.ukeys, (uint32_t *)c.urids,
                                   nuw, 0);
        chk(hipGetLastError(), "dedupe");
        rkeys = (const uint64_t *)c.ukeys;
        rrids = d_rids ? (const uint32_t *)c.urids : nullptr;
        nu = nuw;
    } else {
        chk(hipMemsetAsync(c.dd_nu, 0, 4, s), "memset nu");  // read back with the counts: unused
    }
    uint32_t *counts = (uint32_t *)c.cnt;  // [C][W] send counts
    uint32_t *blk = (uint32_t *)c.cursor, *offs = blk + (uint64_t)W * kRouteBlocks;
    chk(hipMemsetAsync(counts, 0, (uint64_t)C * W * sizeof(uint32_t), s), "memset counts");
    if (n == 0) return;
    for (int i = 0; i < C; ++i) {
        route_hist<<<kRouteBlocks, 256, 0, s>>>(rkeys, n, nu, i, C, W, (uint8_t *)c.dest, blk);
        route_scan<<<1, 1024, 0, s>>>(blk, (uint32_t)(W * kRouteBlocks), W, kRouteBlocks, offs, counts + i * W);
        route_scatter<<<kRouteBlocks, 256, 0, s>>>(rkeys, rrids, n, nu, i, C, W, (const uint8_t *)c.dest, offs,
                                                   (SendRec *)c.send, (uint32_t *)c.perm,
                                                   P.dedupe && owner ? (uint32_t *)c.upos : nullptr,
                                                   P.dedupe ? (const FanRange *)c.urange : nullptr,
                                                   P.dedupe ? (const uint32_t *)c.flist : nullptr, (FanRange *)c.fan);
    }
    chk(hipGetLastError(), "route");
}

// the send side of the plan from P.sc and P.total (filled by the caller from the device counts)
static void plan_send(ShardComm &c, Plan &P) {
    const int W = P.W, C = P.C;
    if (!P.dedupe) P.total = P.n;
    if (P.total > P.n) throw std::runtime_error("routing: more requests than keys");
    P.cb.resize(C + 1);
    for (int i = 0; i <= C; ++i) P.cb[i] = P.total * (uint64_t)i / (uint64_t)C;
    P.soff.assign((size_t)C * (W + 1), 0);
    for (int i = 0; i < C; ++i) {
        P.soff[i * (W + 1)] = P.cb[i];
        for (int r = 0; r < W; ++r) P.soff[i * (W + 1) + r + 1] = P.soff[i * (W + 1) + r] + P.sc[i * W + r];
        if (P.soff[i * (W + 1) + W] != P.cb[i + 1]) throw std::runtime_error("routing: counts disagree with the chunk");
    }
    c.last_n = P.n;
    c.last_routed = c.last_remote = c.last_received = 0;
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
    c.last_received = m;
    if (m > c.cap_remote) {
        const uint64_t cap = m + m / 8 + 1024;
        grow(c.recv, cap * sizeof(SendRec));
        grow(c.rout, cap * sizeof(stage_probe_out_dev));
        grow(c.rrec, cap * stride);
        grow(c.lkeys, cap * 8);
        grow(c.lrids, cap * 4);
        grow(c.lpads, cap * 4);
        c.cap_remote = cap;
    }
}

static void fan_launch(const stage_probe_out_dev *sout, const uint8_t *srec, uint64_t p0, uint64_t p1, const ShardComm &c,
                       const Plan &P, uint32_t stride, stage_probe_out_dev *d_out, uint8_t *d_recs, hipStream_t s) {
    if (p1 <= p0) return;
    constexpr int R = 4;
    fan_copy<R><<<(unsigned)std::min<uint64_t>((p1 - p0 + 4 * R - 1) / (4 * R), 8192), 256, 0, s>>>(
        sout, srec, p0, p1, (const FanRange *)c.fan, P.dedupe ? (const uint32_t *)c.flist : nullptr, stride, d_out,
        d_recs);
    chk(hipGetLastError(), "fan copy");
}

// STAGE_REPLY_DIRECT: from this many ranks on, a rank's own requests (1/W of a chunk) are probed
// in the chunk's one launch with the remote ones; below it, on their own stream beside the remote
// probes, where they overlap the key exchange.  Measured: W = 8 loopback 16.6 → 12.8
// ms per 2^24 lookups merged; the 2-rank RCCL rehearsal 26.7-28.7 merged vs 24.2-25.4 ms apart
constexpr int kDirectMergeFrom = 4;
static inline bool direct_merge(int W) { return W >= kDirectMergeFrom; }

// Probe what chunk i holds for this rank.  The remote segments arrived in recv; this rank's own
// requests never left the device (no self transfer): they are read from the send buffer.
// Full reply: own requests are probed in fan-out form, straight to their caller positions in
// d_out / d_recs, on their own stream c.ps beside the remote probes (a chunk's own share is a
// small launch whose latency the remote probes hide; joined by own_join); tables of other
// geometries: probed into rout / rrec, then fanned out.  The remote segments are probed into
// rout / rrec for the return transfer.  Owner reply: everything into rout / rrec, rows tagged
// with their owner-local index.  Direct reply: the chunk, one segment per source rank q, is probed
// in fan-out form straight into caller q's d_out / d_records (c.dpeer), each request at its first
// caller position (c.lpads) -- from kDirectMergeFrom ranks on in one launch with this rank's own
// requests as one more segment, below it in two (the ranks below / above this one) with the own
// requests as in the full reply.
static void chunk_probe(ShardComm &c, const Plan &P, int i, const DevTable &t, const ProbeTuning &tune, bool owner,
                        stage_probe_out_dev *d_out, uint8_t *d_recs, hipStream_t s, uint8_t *rows_buf = nullptr,
                        bool direct = false) {
    const int W = P.W, me = c.rank;
    const uint64_t b = P.rb[i], e = P.rb[i + 1];
    if (e == b) return;
    const uint64_t r0 = P.roff[(size_t)i * (W + 1) + me], r1 = P.roff[(size_t)i * (W + 1) + me + 1];
    const uint64_t q0 = P.soff[(size_t)i * (W + 1) + me];
    uint64_t *lk = (uint64_t *)c.lkeys;
    uint32_t *lr = (uint32_t *)c.lrids, *lp = (uint32_t *)c.lpads;
    auto unpack = [&](const SendRec *src, uint64_t at, uint64_t m) {
        if (m) unpack_keys<<<blocks_for(m, 256), 256, 0, s>>>(src, m, lk + at, lr + at, direct ? lp + at : nullptr);
    };
    unpack((const SendRec *)c.recv + b, b, r0 - b);
    unpack((const SendRec *)c.send + q0, r0, r1 - r0);
    unpack((const SendRec *)c.recv + r1, r1, e - r1);
    stage_probe_out_dev *rout = (stage_probe_out_dev *)c.rout;
    uint8_t *rrec = rows_buf ? rows_buf : (uint8_t *)c.rrec;  // peer reply: this call's exported row buffer
    const bool rows = owner || d_recs != nullptr;
    auto probe = [&](uint64_t a, uint64_t z) {
        if (z > a)
            chk(launch_probe(t, lk + a, nullptr, lr + a, nullptr, z - a, rout + a, rows ? rrec + a * (uint64_t)t.stride : nullptr,
                             s, tune),
                "probe");
    };
    if (owner) {
        probe(b, e);
        tag_rows<<<blocks_for(e - b, 256), 256, 0, s>>>(rout + b, e - b, (uint32_t)b);
        return;
    }
    if (direct) {  // direct_tables: [2i] the whole chunk (merged) or the ranks below, [2i + 1] those above
        const FanDest *fd = (const FanDest *)c.fdest + 2 * (size_t)i;
        if (direct_merge(W)) {
            chk(launch_probe_fanout(t, lk + b, lr + b, e - b, nullptr, lp + b, nullptr, nullptr, s, tune, fd),
                "direct probe");
            return;
        }
        if (r0 > b)
            chk(launch_probe_fanout(t, lk + b, lr + b, r0 - b, nullptr, lp + b, nullptr, nullptr, s, tune, fd),
                "direct probe");
        if (e > r1)
            chk(launch_probe_fanout(t, lk + r1, lr + r1, e - r1, nullptr, lp + r1, nullptr, nullptr, s, tune, fd + 1),
                "direct probe");
    } else {
        probe(b, r0);
        probe(r1, e);
    }
    if (r1 == r0) return;
    if (d_recs && probe_fanout_supported(t)) {
        hipStream_t os = c.ps;  // beside the remote probes (on s: slower)
        chk(hipEventRecord(c.ev_fork, s), "fork");  // the unpacked keys
        chk(hipStreamWaitEvent(os, c.ev_fork, 0), "fork");
        chk(launch_probe_fanout(t, lk + r0, lr + r0, r1 - r0, (const FanRange *)c.fan + q0,
                                P.dedupe ? (const uint32_t *)c.flist : nullptr, d_out, d_recs, os, tune),
            "fan-out probe");
    } else {
        probe(r0, r1);
        fan_launch(rout + r0, rrec + r0 * (uint64_t)t.stride, q0, q0 + (r1 - r0), c, P, t.stride, d_out, d_recs, s);
    }
}

// the caller's stream waits for the own-request probes of every chunk
static void own_join(ShardComm &c, hipStream_t s) {
    chk(hipEventRecord(c.ev_own, c.ps), "own join");
    chk(hipStreamWaitEvent(s, c.ev_own, 0), "own join");
}

// chunk i's results that came back from other ranks (bout / brec, at their send positions) to
// their caller positions; owner reply: status records of every position (own ones read in place)
// -- coalesced, once all chunks are back (owner_expand: a caller's request may sit in any chunk)
static void chunk_return(ShardComm &c, const Plan &P, int i, uint32_t stride, bool owner, stage_probe_out_dev *d_out,
                         uint8_t *d_recs, hipStream_t s) {
    const int W = P.W, me = c.rank;
    const uint64_t p0 = P.cb[i], pz = P.soff[(size_t)i * (W + 1) + W];
    const uint64_t q0 = P.soff[(size_t)i * (W + 1) + me], q1 = P.soff[(size_t)i * (W + 1) + me + 1];
    const stage_probe_out_dev *bout = (const stage_probe_out_dev *)c.bout;
    const uint8_t *brec = (const uint8_t *)c.brec;
    if (!owner) {
        fan_launch(bout + p0, brec + p0 * (uint64_t)stride, p0, q0, c, P, stride, d_out, d_recs, s);
        fan_launch(bout + q1, brec + q1 * (uint64_t)stride, q1, pz, c, P, stride, d_out, d_recs, s);
        return;
    }
    if (P.dedupe) return;
    const uint64_t ro = P.roff[(size_t)i * (W + 1) + me];  // where the local probe wrote the own results
    const stage_probe_out_dev *qout = (const stage_probe_out_dev *)c.rout + ro;
    if (pz > p0) {
        unpermute_status<<<blocks_for(pz - p0, 256), 256, 0, s>>>(bout, (const uint32_t *)c.perm, p0, pz, d_out, q0, q1,
                                                                  qout);
    }
    chk(hipGetLastError(), "owner-reply return");
}

// ---- STAGE_REPLY_PEER.  Every rank knows every rank's send counts S[q][i][r] (an allgather in
// place of the count all-to-all), hence where owner q put the rows of the requests rank r sent it
// in chunk i: q's receive layout is chunk-major, then by source rank (plan_receive), so
//   peer_row_off(q, i, r) = sum_{i' < i} sum_{r'} S[r'][i'][q] + sum_{r' < r} S[r'][i][q].
// Each rank's two row buffers hold m_q = sum_{i, r} S[r][i][q] rows; every rank applies the same
// growth rule to every rank's size, so all of them know when the buffers moved and re-exchange
// the IPC handles together (an allgather of 2 handles per rank).
struct PeerCounts {
    int W, C;
    std::vector<uint32_t> S;  // [q][i][r]: q sends r in chunk i
    uint32_t at(int q, int i, int r) const { return S[((size_t)q * C + i) * W + r]; }
    uint64_t row_off(int q, int i, int r) const {
        uint64_t o = 0;
        for (int i2 = 0; i2 < i; ++i2)
            for (int r2 = 0; r2 < W; ++r2) o += at(r2, i2, q);
        for (int r2 = 0; r2 < r; ++r2) o += at(r2, i, q);
        return o;
    }
    uint64_t received(int q) const {
        uint64_t m = 0;
        for (int i = 0; i < C; ++i)
            for (int r = 0; r < W; ++r) m += at(r, i, q);
        return m;
    }
};

// the growth rule every rank applies to every rank's row buffers; true when one of them grows.
// The buffers hold rows of the call's stride (every rank's table has the same output stride, as
// the rows reply's transfers assume): a stride change (stage_set_output_layout between calls)
// re-plans every rank's buffers from zero, so they are reallocated and their handles exchanged
// again on every rank together.
static bool peer_grow_plan(ShardComm &c, const PeerCounts &pc, uint32_t stride) {
    if ((int)c.peer_cap.size() != pc.W || c.peer_stride != stride) {
        c.peer_cap.assign(pc.W, 0);
        c.peer_stride = stride;
    }
    bool grew = false;
    for (int q = 0; q < pc.W; ++q) {
        const uint64_t m = pc.received(q);
        if (m > c.peer_cap[q]) {
            c.peer_cap[q] = m + m / 8 + 1024;
            grew = true;
        }
    }
    return grew;
}

// this rank's row buffers at the size the plan says (the old ones are freed: their readers are
// done -- every rank's fan-out of the previous call ended before this call's count exchange)
static void peer_alloc_own(ShardComm &c, uint32_t stride) {
    const uint64_t cap = c.peer_cap[c.rank];
    if (cap == c.prow_cap && stride == c.prow_stride && c.prow[0]) return;
    for (int k = 0; k < 2; ++k) grow(c.prow[k], cap * stride);
    c.prow_cap = cap;
    c.prow_stride = stride;
}

static void *hbuf(ShardComm &c, uint64_t bytes) {
    if (bytes > c.hbuf_cap) {
        grow(c.hbuf, bytes);
        c.hbuf_cap = bytes;
    }
    return c.hbuf;
}

// the IPC handles of every rank's two row buffers, exchanged over the communicator; the peers'
// buffers opened here (own buffers used in place).  The ranks agree on the outcome (an allreduce
// of an ok flag) before any of them goes on, so a runtime that refuses the mapping on one rank
// makes the call fail on every rank, with nothing left mapped -- not a rank hanging in the
// exchange that follows; the next peer call tries again.
static void peer_exchange(ShardComm &c, hipStream_t s) {
    const int W = c.world;
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
    std::vector<hipIpcMemHandle_t> mine(2), all((size_t)2 * W);
    std::memset(mine.data(), 0, 128);
    hipError_t e = hipSuccess;
    const char *what = "hipIpcGetMemHandle";
    for (int k = 0; k < 2 && !e; ++k) e = hipIpcGetMemHandle(&mine[k], c.prow[k]);
    uint8_t *d = (uint8_t *)hbuf(c, (uint64_t)(W + 1) * 128 + 8);
    chk(hipMemcpyAsync(d, mine.data(), 128, hipMemcpyHostToDevice, s), "handles h2d");
    nchk(ncclAllGather(d, d + 128, 128, ncclUint8, (ncclComm_t)c.comm, s), "ncclAllGather handles");
    chk(hipMemcpyAsync(all.data(), d + 128, (size_t)128 * W, hipMemcpyDeviceToHost, s), "handles d2h");
    chk(hipStreamSynchronize(s), "handles sync");
    for (void *p : c.opened) (void)hipIpcCloseMemHandle(p);
    c.opened.clear();
    for (int k = 0; k < 2; ++k) c.peer_row[k].assign(W, nullptr);
    if (!e) what = "hipIpcOpenMemHandle";
    for (int q = 0; q < W && !e; ++q)
        for (int k = 0; k < 2 && !e; ++k) {
            if (q == c.rank) {
                c.peer_row[k][q] = c.prow[k];
                continue;
            }
            void *p = nullptr;
            e = hipIpcOpenMemHandle(&p, all[(size_t)2 * q + k], hipIpcMemLazyEnablePeerAccess);
            if (!e) {
                c.opened.push_back(p);
                c.peer_row[k][q] = p;
            }
        }
    if (e) (void)hipGetLastError();  // the refusal is reported below, not by a later call
    int32_t ok = e ? 0 : 1, all_ok = 0;
    int32_t *dok = (int32_t *)(d + (uint64_t)(W + 1) * 128);
    chk(hipMemcpyAsync(dok, &ok, 4, hipMemcpyHostToDevice, s), "ok h2d");
    nchk(ncclAllReduce(dok, dok, 1, ncclInt32, ncclMin, (ncclComm_t)c.comm, s), "ncclAllReduce ok");
    chk(hipMemcpyAsync(&all_ok, dok, 4, hipMemcpyDeviceToHost, s), "ok d2h");
    chk(hipStreamSynchronize(s), "ok sync");
    if (all_ok) return;
    for (void *p : c.opened) (void)hipIpcCloseMemHandle(p);
    c.opened.clear();
    for (int k = 0; k < 2; ++k) c.peer_row[k].assign(W, nullptr);
    c.peer_cap.clear();  // every rank: the next peer call plans and exchanges afresh
    throw std::runtime_error(std::string("peer reply unavailable: ") +
                             (e ? std::string(what) + " failed on this rank: " + hipGetErrorString(e)
                                : std::string("another rank could not map the row buffers")));
}

// A system-scope acquire on every XCD (256 one-wave workgroups land on all 8): the peers' row
// buffers are mapped non-coherently, so a line this device's L2 kept from an earlier call with
// the same buffer parity could be stale; `buffer_inv sc0 sc1` drops such lines before the
// fan-out reads the rows the owners wrote since (their kernels' end released them to memory,
// and the status records that precede this fan-out were sent after those kernels).
__global__ void peer_acquire_kernel() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate has completed
}

// The owner side's counterpart: a system-scope release on every XCD after the chunk's probe has
// stored its rows into this rank's IPC-exported row buffer, before the status records leave over
// RCCL -- each XCD's L2 writes its dirty lines of the buffer back to HBM, where the peers' reads
// over xGMI find them (kernel-boundary fences alone give device scope only).
__global__ void peer_release_kernel() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// peer reply, chunk i: the status records that came back from every other rank, with each row read
// where its owner left it (peer_row) and stored at the caller positions
static void chunk_return_peer(ShardComm &c, const Plan &P, const PeerCounts &pc, int i, uint32_t stride,
                              stage_probe_out_dev *d_out, uint8_t *d_recs, hipStream_t s) {
    const int W = P.W, me = c.rank;
    peer_acquire_kernel<<<256, 64, 0, s>>>();
    const stage_probe_out_dev *bout = (const stage_probe_out_dev *)c.bout;
    for (int q = 0; q < W; ++q) {
        if (q == me) continue;  // own requests: probed straight to their caller positions
        const uint64_t p0 = P.soff[(size_t)i * (W + 1) + q], sn = P.sc[(size_t)i * W + q];
        if (!sn) continue;
        const uint8_t *rows = (const uint8_t *)c.peer_row[c.parity][q] + pc.row_off(q, i, me) * (uint64_t)stride;
        fan_launch(bout + p0, rows, p0, p0 + sn, c, P, stride, d_out, d_recs, s);
    }
}

// ---- STAGE_REPLY_DIRECT.  The caller's side of chunk i once every owner's token for it is in:
// a system-scope acquire (its L2 may hold lines of d_out / d_records the owners have written
// since), then the duplicates of each coalesced request copied from its first caller position.
static void chunk_return_direct(ShardComm &c, const Plan &P, int i, uint32_t stride, stage_probe_out_dev *d_out,
                                uint8_t *d_recs, hipStream_t s) {
    const int W = P.W;
    peer_acquire_kernel<<<256, 64, 0, s>>>();
    if (!P.dedupe) return;  // one caller per request: nothing to copy
    constexpr int R = 4;
    // the requests of the chunk, send positions [p0, pz) -- without this rank's own ones, [q0, q1),
    // when they were probed straight to every caller position (below kDirectMergeFrom ranks)
    const uint64_t p0 = P.cb[i], pz = P.soff[(size_t)i * (W + 1) + W];
    uint64_t q0 = P.soff[(size_t)i * (W + 1) + c.rank], q1 = P.soff[(size_t)i * (W + 1) + c.rank + 1];
    if (direct_merge(W)) q0 = q1 = pz;
    for (const auto &rg : {std::make_pair(p0, q0), std::make_pair(q1, pz)})
        if (rg.second > rg.first)
            dup_copy<R><<<(unsigned)std::min<uint64_t>((rg.second - rg.first + 4 * R - 1) / (4 * R), 8192), 256, 0, s>>>(
                rg.first, rg.second, (const FanRange *)c.fan, (const uint32_t *)c.flist, stride, d_out, d_recs);
    chk(hipGetLastError(), "direct duplicates");
}

// the FanDest tables of every chunk, one segment per source rank q -- from kDirectMergeFrom ranks
// on [2i] covers receive positions [b, e) (the own segment, read from the send buffer, in its
// place between the ranks below and above); below it [2i] covers [b, r0) from the ranks below
// this one and [2i + 1] [r1, e) from those above -- from the plan and c.dpeer, staged in pinned
// memory and copied to the device on s (the staging is rewritten only after the next call's count
// exchange has synchronised s)
static void direct_tables(ShardComm &c, const Plan &P, hipStream_t s) {
    const int W = P.W, C = P.C, me = c.rank;
    static_assert(kMaxWorld <= kFanDests, "a segment per source rank");
    const size_t bytes = (size_t)2 * kMaxChunks * sizeof(FanDest);
    if (!c.fdest) {
        grow(c.fdest, bytes);
        chk(hipHostMalloc(&c.fdest_h, bytes, hipHostMallocDefault), "hipHostMalloc");
    }
    FanDest *h = (FanDest *)c.fdest_h;
    const bool merge = direct_merge(W);
    for (int i = 0; i < C; ++i)
        for (int side = 0; side < 2; ++side) {
            FanDest &d = h[2 * i + side];
            d.nseg = 0;
            const int qa = merge ? (side ? W : 0) : (side ? me + 1 : 0), qz = merge ? W : (side ? W : me);
            const uint64_t start = P.roff[(size_t)i * (W + 1) + qa];
            for (int q = qa; q < qz; ++q) {
                d.end[d.nseg] = (uint32_t)(P.roff[(size_t)i * (W + 1) + q + 1] - start);
                d.out[d.nseg] = (stage_probe_out_dev *)c.dpeer[0][q];
                d.recs[d.nseg] = (uint8_t *)c.dpeer[1][q];
                ++d.nseg;
            }
        }
    chk(hipMemcpyAsync(c.fdest, h, (size_t)2 * C * sizeof(FanDest), hipMemcpyHostToDevice, s), "direct tables");
}

// this rank's d_out / d_records as another process opens it: the allocation's IPC handle and the
// buffer's offset in it; off = ~0 when the runtime refuses (reported on every rank once the pairs
// are exchanged).  Taken on every call, not cached per pointer: memory freed and allocated again
// at the same address gets a new handle (hipIpcGetMemHandle), which is how the other ranks see
// that their mapping of it is stale.
static ShardComm::DirectBuf direct_export(const void *p) {
    ShardComm::DirectBuf b{};
    b.off = ~0ull;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipIpcMemHandle_t h;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && base &&
        hipIpcGetMemHandle(&h, (void *)base) == hipSuccess) {
        std::memcpy(b.handle, &h, sizeof b.handle);
        b.off = (uint64_t)((const uint8_t *)p - (const uint8_t *)base);
    } else {
        (void)hipGetLastError();
    }
    return b;
}

// every rank's pairs (all[2 * q + k], the same table on every rank) -> c.dpeer.  A rank whose
// allocation handles changed since the last call has its mappings reopened (an offset change
// alone reuses them); when any rank's changed, every rank takes part in agreeing on the outcome
// (an allreduce, as peer_exchange), so a refusal on one rank fails the call on all of them.
static void direct_map(ShardComm &c, const std::vector<ShardComm::DirectBuf> &all, stage_probe_out_dev *d_out,
                       uint8_t *d_recs, hipStream_t s) {
    const int W = c.world;
    for (int j = 0; j < 2 * W; ++j)
        if (all[j].off == ~0ull)
            throw std::runtime_error("direct reply unavailable: rank " + std::to_string(j / 2) +
                                     " could not export its output buffers (hipIpcGetMemHandle)");
    auto same_h = [](const ShardComm::DirectBuf &a, const ShardComm::DirectBuf &b) {
        return std::memcmp(a.handle, b.handle, sizeof a.handle) == 0;
    };
    if ((int)c.dseen.size() != 2 * W) {  // nothing mapped yet
        for (auto &v : c.dopen)
            for (void *p : v) (void)hipIpcCloseMemHandle(p);
        c.dopen.assign(W, {});
        c.dbase.assign(2 * W, nullptr);
        c.dseen.assign(2 * W, ShardComm::DirectBuf{});
        for (auto &b : c.dseen) b.off = ~0ull;  // matches no handle below
    }
    std::vector<char> moved(W, 0);
    bool any = false;
    for (int q = 0; q < W; ++q) {
        moved[q] = c.dseen[2 * q].off == ~0ull || !same_h(all[2 * q], c.dseen[2 * q]) ||
                   !same_h(all[2 * q + 1], c.dseen[2 * q + 1]);
        any = any || moved[q];
    }
    hipError_t e = hipSuccess;
    for (int q = 0; q < W && !e; ++q) {
        if (!moved[q] || q == c.rank) continue;
        for (void *p : c.dopen[q]) (void)hipIpcCloseMemHandle(p);
        c.dopen[q].clear();
        c.dbase[2 * q] = c.dbase[2 * q + 1] = nullptr;
        for (int k = 0; k < 2 && !e; ++k) {
            if (k == 1 && same_h(all[2 * q + 1], all[2 * q])) {  // both buffers in one allocation
                c.dbase[2 * q + 1] = c.dbase[2 * q];
                break;
            }
            hipIpcMemHandle_t h;
            std::memcpy(&h, all[2 * q + k].handle, sizeof h);
            void *b = nullptr;
            e = hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess);
            if (!e) {
                c.dopen[q].push_back(b);
                c.dbase[2 * q + k] = b;
            } else {
                std::fprintf(stderr, "[direct] rank %d: hipIpcOpenMemHandle(rank %d, %s) failed: %s\n", c.rank, q,
                             k ? "d_records" : "d_out", hipGetErrorString(e));
            }
        }
    }
    if (e) (void)hipGetLastError();
    if (any) {
        int32_t ok = e ? 0 : 1, all_ok = 0;
        int32_t *dok = (int32_t *)hbuf(c, 8);
        chk(hipMemcpyAsync(dok, &ok, 4, hipMemcpyHostToDevice, s), "ok h2d");
        nchk(ncclAllReduce(dok, dok, 1, ncclInt32, ncclMin, (ncclComm_t)c.comm, s), "ncclAllReduce ok");
        chk(hipMemcpyAsync(&all_ok, dok, 4, hipMemcpyDeviceToHost, s), "ok d2h");
        chk(hipStreamSynchronize(s), "ok sync");
        if (!all_ok) {
            for (auto &v : c.dopen)
                for (void *p : v) (void)hipIpcCloseMemHandle(p);
            c.dopen.assign(W, {});
            c.dseen.clear();  // every rank: the next direct call maps afresh
            throw std::runtime_error(std::string("direct reply unavailable: ") +
                                     (e ? std::string("hipIpcOpenMemHandle failed on this rank: ") + hipGetErrorString(e)
                                        : std::string("another rank could not map the output buffers")));
        }
    }
    c.dseen = all;
    for (int k = 0; k < 2; ++k) c.dpeer[k].assign(W, nullptr);
    for (int q = 0; q < W; ++q)
        for (int k = 0; k < 2; ++k)
            c.dpeer[k][q] = q == c.rank ? (k ? (void *)d_recs : (void *)d_out)
                                        : (void *)((uint8_t *)c.dbase[2 * q + k] + all[2 * q + k].off);
}

static void owner_expand(ShardComm &c, const Plan &P, stage_probe_out_dev *d_out, hipStream_t s) {
    if (!P.dedupe || P.n == 0) return;
    const int W = P.W, me = c.rank;
    OwnSegs own{};
    own.C = P.C;
    for (int i = 0; i < P.C; ++i) {
        own.cb[i] = (uint32_t)P.cb[i];
        own.q0[i] = (uint32_t)P.soff[(size_t)i * (W + 1) + me];
        own.q1[i] = (uint32_t)P.soff[(size_t)i * (W + 1) + me + 1];
        own.ro[i] = (uint32_t)P.roff[(size_t)i * (W + 1) + me];
    }
    expand_status<<<blocks_for(P.n, 256), 256, 0, s>>>((const stage_probe_out_dev *)c.bout, (const uint32_t *)c.uidx,
                                                        (const uint32_t *)c.upos, P.n, d_out, own,
                                                        (const stage_probe_out_dev *)c.rout);
    chk(hipGetLastError(), "owner-reply expand");
}

// RCCL path.  Streams: the caller's stream s routes and probes; c.cs carries the RCCL
// transfers; c.us fans the returned results out.  One host wait per call: the send counts are
// transposed and exchanged on the device (ncclAllToAll), and the send and receive counts come
// back together.  Then all key exchanges (16 B/request, own requests stay), and for each chunk
// the probe (s) and, as soon as it is done, its result exchange (cs) -- so the return of chunk i
// over xGMI overlaps the probe of chunk i+1 in HBM -- and its fan-out (us).
int shard_probe(ShardComm &c, const DevTable &t, const ProbeTuning &tune, const uint64_t *d_keys,
                const uint32_t *d_rids, uint64_t n, stage_probe_out_dev *d_out, uint8_t *d_recs, int reply,
                hipStream_t s) {
    if (!c.comm) throw std::invalid_argument("not an RCCL communicator");
    const bool owner = reply == STAGE_REPLY_OWNER;
    const bool peer = reply == STAGE_REPLY_PEER && c.world > 1 && d_recs != nullptr;
    const bool direct = reply == STAGE_REPLY_DIRECT && c.world > 1 && d_recs != nullptr;
    if (direct && !probe_fanout_supported(t))
        throw std::invalid_argument("STAGE_REPLY_DIRECT: tables of the YCSB geometry (8-byte keys, 64-slot leaves, rows <= 1024 B)");
    if (owner) d_recs = nullptr;  // rows stay on the owner
    c.owner_rows = 0;
    const int W = c.world, C = c.chunks;
    const uint32_t stride = t.stride;
    ncclComm_t comm = (ncclComm_t)c.comm;
    Plan P;
    plan_route(c, P, d_keys, d_rids, n, stride, owner, s);
    // direct: this device's L2 writes back its dirty lines of d_out / d_records before any owner
    // writes them over xGMI (done before the count exchange's synchronisation below)
    if (direct) peer_release_kernel<<<256, 64, 0, s>>>();
    uint32_t *cnt = (uint32_t *)c.cnt, *sendT = cnt + (uint64_t)C * W, *recvT = sendT + (uint64_t)C * W;
    PeerCounts pc{W, C, {}};
    if (peer) {
        // every rank's [C][W] send counts (the peer fan-out needs the owners' receive layouts),
        // then the coalesced request count
        uint32_t *all = (uint32_t *)hbuf(c, ((uint64_t)W * C * W + 1) * 4);
        nchk(ncclAllGather(cnt, all, (size_t)C * W, ncclUint32, comm, s), "ncclAllGather counts");
        std::vector<uint32_t> hc((size_t)W * C * W + 1);
        chk(hipMemcpyAsync(hc.data(), all, (size_t)W * C * W * 4, hipMemcpyDeviceToHost, s), "counts d2h");
        chk(hipMemcpyAsync(hc.data() + (size_t)W * C * W, c.dd_nu, 4, hipMemcpyDeviceToHost, s), "nu d2h");
        chk(hipStreamSynchronize(s), "sync");
        pc.S.assign(hc.begin(), hc.begin() + (size_t)W * C * W);
        P.sc.assign(pc.S.begin() + (size_t)c.rank * C * W, pc.S.begin() + (size_t)(c.rank + 1) * C * W);
        P.total = hc[(size_t)W * C * W];
        P.rc.resize((size_t)C * W);
        for (int i = 0; i < C; ++i)
            for (int r = 0; r < W; ++r) P.rc[(size_t)i * W + r] = pc.at(r, i, c.rank);
        if (peer_grow_plan(c, pc, stride)) {  // the same decision on every rank
            peer_alloc_own(c, stride);
            peer_exchange(c, s);
        }
        c.parity ^= 1;
    } else if (direct) {
        // every rank's [C][W] send counts and its (handle, offset) of d_out / d_records in one
        // allgather, then the coalesced request count
        const ShardComm::DirectBuf mine[2] = {direct_export(d_out), direct_export(d_recs)};
        const uint64_t cw = (uint64_t)C * W * 4, rec = (cw + sizeof mine + 15) & ~15ull;
        uint8_t *d = (uint8_t *)hbuf(c, (uint64_t)(W + 1) * rec);
        chk(hipMemcpyAsync(d, cnt, cw, hipMemcpyDeviceToDevice, s), "counts");
        chk(hipMemcpyAsync(d + cw, mine, sizeof mine, hipMemcpyHostToDevice, s), "buffers h2d");
        nchk(ncclAllGather(d, d + rec, rec, ncclUint8, comm, s), "ncclAllGather counts + buffers");
        std::vector<uint8_t> h((size_t)W * rec + 4);
        chk(hipMemcpyAsync(h.data(), d + rec, (size_t)W * rec, hipMemcpyDeviceToHost, s), "counts d2h");
        chk(hipMemcpyAsync(h.data() + (size_t)W * rec, c.dd_nu, 4, hipMemcpyDeviceToHost, s), "nu d2h");
        chk(hipStreamSynchronize(s), "sync");
        auto S = [&](int q, int i, int r) {
            uint32_t v;
            std::memcpy(&v, h.data() + (size_t)q * rec + ((size_t)i * W + r) * 4, 4);
            return v;
        };
        P.sc.resize((size_t)C * W);
        P.rc.resize((size_t)C * W);
        for (int i = 0; i < C; ++i)
            for (int r = 0; r < W; ++r) {
                P.sc[(size_t)i * W + r] = S(c.rank, i, r);
                P.rc[(size_t)i * W + r] = S(r, i, c.rank);
            }
        uint32_t nu;
        std::memcpy(&nu, h.data() + (size_t)W * rec, 4);
        P.total = nu;
        std::vector<ShardComm::DirectBuf> all((size_t)2 * W);
        for (int q = 0; q < W; ++q) std::memcpy(&all[(size_t)2 * q], h.data() + (size_t)q * rec + cw, sizeof mine);
        direct_map(c, all, d_out, d_recs, s);
    } else {
        transpose_counts<<<1, 256, 0, s>>>(cnt, C, W, sendT);
        nchk(ncclAllToAll(sendT, recvT, (size_t)C, ncclUint32, comm, s), "ncclAllToAll counts");
        // [C][W] send counts, then [W][C] receive counts, then the coalesced request count
        std::vector<uint32_t> hc((size_t)2 * C * W + 1);
        chk(hipMemcpyAsync(hc.data(), cnt, (size_t)C * W * 4, hipMemcpyDeviceToHost, s), "counts d2h");
        chk(hipMemcpyAsync(hc.data() + (size_t)C * W, recvT, (size_t)C * W * 4, hipMemcpyDeviceToHost, s), "counts d2h");
        chk(hipMemcpyAsync(hc.data() + (size_t)2 * C * W, c.dd_nu, 4, hipMemcpyDeviceToHost, s), "nu d2h");
        chk(hipStreamSynchronize(s), "sync");
        P.sc.assign(hc.begin(), hc.begin() + (size_t)C * W);
        P.total = hc[(size_t)2 * C * W];
        P.rc.resize((size_t)C * W);
        for (int i = 0; i < C; ++i)
            for (int r = 0; r < W; ++r) P.rc[(size_t)i * W + r] = hc[(size_t)C * W + (size_t)r * C + i];
    }
    plan_send(c, P);
    plan_receive(c, P, stride);
    if (direct) direct_tables(c, P, s);
    hipEvent_t *ev_keys = c.evs.data(), *ev_probe = ev_keys + C, *ev_res = ev_probe + C, ev_start = ev_res[C];
    // the comm stream starts after the routing (done: s was synchronised) -- keys of all chunks
    for (int i = 0; i < C; ++i) {
        nchk(ncclGroupStart(), "group");
        for (int r = 0; r < W; ++r) {
            if (r == c.rank) continue;  // own requests are probed from the send buffer
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
        chunk_probe(c, P, i, t, tune, owner, d_out, d_recs, s, peer ? (uint8_t *)c.prow[c.parity] : nullptr, direct);
        // peer / direct: the rows this device stored for other ranks leave its L2 (system-scope
        // release on every XCD) before the status records / tokens that announce them
        if (peer || direct) peer_release_kernel<<<256, 64, 0, s>>>();
        chk(hipEventRecord(ev_probe[i], s), "event");
        chk(hipStreamWaitEvent(c.cs, ev_probe[i], 0), "wait probe");
        nchk(ncclGroupStart(), "group");
        for (int r = 0; r < W; ++r) {
            if (r == c.rank) continue;  // own results are already in place
            const uint32_t sn = P.sc[(size_t)i * W + r], rn = P.rc[(size_t)i * W + r];
            const uint64_t so = P.soff[(size_t)i * (W + 1) + r], ro = P.roff[(size_t)i * (W + 1) + r];
            const bool send_rows = d_recs && !peer;  // peer reply: the rows stay here, read in place
            if (direct) {  // the results are in the callers' buffers already: a 16-B token each way
                if (rn) nchk(ncclSend((const uint8_t *)c.rout + ro * ob, 16, ncclUint8, r, comm, c.cs), "send token");
                if (sn) nchk(ncclRecv((uint8_t *)c.bout + so * ob, 16, ncclUint8, r, comm, c.cs), "recv token");
                continue;
            }
            if (rn) {
                nchk(ncclSend((const uint8_t *)c.rout + ro * ob, (uint64_t)rn * ob, ncclUint8, r, comm, c.cs), "send out");
                if (send_rows)
                    nchk(ncclSend((const uint8_t *)c.rrec + ro * stride, (uint64_t)rn * stride, ncclUint8, r, comm, c.cs),
                         "send rows");
            }
            if (sn) {
                nchk(ncclRecv((uint8_t *)c.bout + so * ob, (uint64_t)sn * ob, ncclUint8, r, comm, c.cs), "recv out");
                if (send_rows)
                    nchk(ncclRecv((uint8_t *)c.brec + so * stride, (uint64_t)sn * stride, ncclUint8, r, comm, c.cs),
                         "recv rows");
            }
        }
        nchk(ncclGroupEnd(), "group end");
        chk(hipEventRecord(ev_res[i], c.cs), "event");
        chk(hipStreamWaitEvent(c.us, ev_res[i], 0), "wait results");
        if (peer) chunk_return_peer(c, P, pc, i, stride, d_out, d_recs, c.us);
        else if (direct) chunk_return_direct(c, P, i, stride, d_out, d_recs, c.us);
        else chunk_return(c, P, i, stride, owner, d_out, d_recs, c.us);
    }
    if (owner) owner_expand(c, P, d_out, c.us);
    // the caller's stream completes after the last fan-out and the own-request probes
    chk(hipEventRecord(ev_start, c.us), "event");
    chk(hipStreamWaitEvent(s, ev_start, 0), "join");
    own_join(c, s);
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
    const bool peer = reply == STAGE_REPLY_PEER && W > 1 && recs[0] != nullptr;
    const bool direct = reply == STAGE_REPLY_DIRECT && W > 1 && recs[0] != nullptr;
    if (direct && !probe_fanout_supported(*ts[0]))
        throw std::invalid_argument("STAGE_REPLY_DIRECT: tables of the YCSB geometry (8-byte keys, 64-slot leaves, rows <= 1024 B)");
    if (owner)
        for (auto &r : recs) r = nullptr;
    for (int r = 0; r < W; ++r)
        if (ts[r]->stride != stride || cs[r]->world != W || cs[r]->rank != r || cs[r]->chunks != cs[0]->chunks)
            throw std::invalid_argument("loopback shards disagree on stride / rank / world / chunks");
    const int C = cs[0]->chunks;
    const bool rows = recs[0] != nullptr;
    std::vector<Plan> P(W);
    std::vector<uint32_t> tot(W);
    for (int r = 0; r < W; ++r) {
        plan_route(*cs[r], P[r], keys[r], rids[r], n[r], stride, owner, s);
        P[r].sc.resize((size_t)C * W);
        chk(hipMemcpyAsync(P[r].sc.data(), cs[r]->cnt, (size_t)C * W * 4, hipMemcpyDeviceToHost, s), "counts d2h");
        chk(hipMemcpyAsync(&tot[r], cs[r]->dd_nu, 4, hipMemcpyDeviceToHost, s), "nu d2h");
    }
    chk(hipStreamSynchronize(s), "sync");
    for (int r = 0; r < W; ++r) {
        P[r].total = tot[r];
        plan_send(*cs[r], P[r]);
    }
    for (int r = 0; r < W; ++r) {
        P[r].rc.resize((size_t)C * W);
        for (int i = 0; i < C; ++i)
            for (int q = 0; q < W; ++q) P[r].rc[(size_t)i * W + q] = P[q].sc[(size_t)i * W + r];
        plan_receive(*cs[r], P[r], stride);
    }
    // peer reply: every shard's counts (what the allgather gives each rank), the same growth rule,
    // and the other shards' row buffers used in place (one process: no IPC)
    PeerCounts pc{W, C, {}};
    if (peer) {
        pc.S.resize((size_t)W * C * W);
        for (int q = 0; q < W; ++q) std::copy(P[q].sc.begin(), P[q].sc.end(), pc.S.begin() + (size_t)q * C * W);
        for (int r = 0; r < W; ++r)
            if (peer_grow_plan(*cs[r], pc, stride)) peer_alloc_own(*cs[r], stride);
        for (int r = 0; r < W; ++r) {
            for (int k = 0; k < 2; ++k) {
                cs[r]->peer_row[k].resize(W);
                for (int q = 0; q < W; ++q) cs[r]->peer_row[k][q] = cs[q]->prow[k];
            }
            cs[r]->parity ^= 1;
        }
    }
    if (direct)  // one process: the callers' buffers themselves
        for (int r = 0; r < W; ++r) {
            for (int k = 0; k < 2; ++k) {
                cs[r]->dpeer[k].resize(W);
                for (int q = 0; q < W; ++q) cs[r]->dpeer[k][q] = k ? (void *)recs[q] : (void *)outs[q];
            }
            direct_tables(*cs[r], P[r], s);
        }
    auto copy = [&](void *dst, const void *src, uint64_t bytes, const char *what) {
        if (bytes) chk(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s), what);
    };
    for (int i = 0; i < C; ++i)  // keys: q's chunk-i segment for r -> r's chunk-i segment from q
        for (int r = 0; r < W; ++r)
            for (int q = 0; q < W; ++q) {
                if (q == r) continue;  // as shard_probe: own requests are probed from the send buffer
                copy((SendRec *)cs[r]->recv + P[r].roff[(size_t)i * (W + 1) + q],
                     (const SendRec *)cs[q]->send + P[q].soff[(size_t)i * (W + 1) + r],
                     (uint64_t)P[q].sc[(size_t)i * W + r] * sizeof(SendRec), "loopback keys");
            }
    const uint64_t ob = sizeof(stage_probe_out_dev);
    for (int i = 0; i < C; ++i) {
        for (int r = 0; r < W; ++r)
            chunk_probe(*cs[r], P[r], i, *ts[r], tune, owner, outs[r], recs[r], s,
                        peer ? (uint8_t *)cs[r]->prow[cs[r]->parity] : nullptr, direct);
        for (int q = 0; q < W && !direct; ++q)  // results: owner q's chunk-i segment for r -> r's chunk-i slots of q
            for (int r = 0; r < W; ++r) {
                if (r == q) continue;  // as shard_probe: own results are already in place
                const uint64_t cnt = P[q].rc[(size_t)i * W + r];
                const uint64_t ro = P[q].roff[(size_t)i * (W + 1) + r], so = P[r].soff[(size_t)i * (W + 1) + q];
                copy((uint8_t *)cs[r]->bout + so * ob, (const uint8_t *)cs[q]->rout + ro * ob, cnt * ob, "loopback out");
                if (rows && !peer)
                    copy((uint8_t *)cs[r]->brec + so * stride, (const uint8_t *)cs[q]->rrec + ro * stride,
                         cnt * stride, "loopback rows");
            }
        for (int r = 0; r < W; ++r) {
            if (peer) chunk_return_peer(*cs[r], P[r], pc, i, stride, outs[r], recs[r], s);
            else if (direct) chunk_return_direct(*cs[r], P[r], i, stride, outs[r], recs[r], s);
            else chunk_return(*cs[r], P[r], i, stride, owner, outs[r], recs[r], s);
        }
    }
    if (owner)
        for (int r = 0; r < W; ++r) owner_expand(*cs[r], P[r], outs[r], s);
    for (int r = 0; r < W; ++r) own_join(*cs[r], s);
    for (int r = 0; r < W; ++r) cs[r]->owner_rows = owner ? P[r].m() : 0;
    return STAGE_OK;
}

}  // namespace stage
