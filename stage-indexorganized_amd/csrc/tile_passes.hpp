// tile_passes.hpp -- the device write path's sort and scans as passes of independent 256-thread
// workgroups (.hip translation units only).
//
// In write-overlap mode an epoch's kernels run beside the previous epoch's read probe, which
// holds every CU it can get.  rocprim's onesweep sort and lookback scans did not overlap it: a
// onesweep pass sat ~3.7 ms behind the probe (r05 c3 trace) and the scans after it ran only once
// the probe had drained, so ~0.7 ms of each epoch was exposed.  Here every workgroup of a pass
// works on its own 4096-item tile and waits for no other workgroup (no decoupled lookback), with
// the probe's own workgroup shape (256 threads, a few KB of LDS), so a pass's workgroups are
// dispatched as the probe's retire and it progresses beside it:
//   sort  LSD radix sort of (u64 key, u32 value) pairs, 8 bits a pass, stable: per pass a tile
//         digit histogram (tile_hist), their exclusive scan in digit-major order (scan_*), and
//         the scatter (tile_scatter), which ranks a tile's items by wave, round and lane with
//         8 ballots per round (the lanes holding the same digit) -- item order within a digit;
//   scan  inclusive / exclusive scans (sum, max) as reduce-then-scan: tile totals
//         (scan_reduce), their scan in one workgroup (scan_partials), the tiles rescanned with
//         their offsets (scan_down).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace stage {
namespace tiles {

constexpr int kThreads = 256;
constexpr int kItems = 16;                              // per thread
constexpr uint32_t kTile = kThreads * kItems;           // items per workgroup
constexpr uint32_t kSub = kTile / (kThreads / 64);      // items per wave
constexpr int kRadixBits = 8;
constexpr uint32_t kDigits = 1u << kRadixBits;
static_assert(kDigits == (uint32_t)kThreads, "a thread per digit in the histogram passes");

inline uint64_t tiles_for(uint64_t n) { return (n + kTile - 1) / kTile; }

struct SumOp {
    template <class T>
    __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
    template <class T>
    __device__ __forceinline__ static T identity() { return T(0); }
};
struct MaxOp {
    template <class T>
    __device__ __forceinline__ T operator()(T a, T b) const { return a > b ? a : b; }
    template <class T>
    __device__ __forceinline__ static T identity() { return T(0); }  // unsigned values
};

// the lanes of the wave whose `valid` item carries digit d (8 ballots)
__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid) {
    uint64_t m = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
    for (int b = 0; b < kRadixBits; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __builtin_amdgcn_ballot_w64(valid && bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) { return lane ? ~0ull >> (64 - lane) : 0ull; }

// item j of this thread's wave: wave w of tile b holds items [b * kTile + w * kSub, .. + kSub),
// round j lane l the item at + j * 64 + l (tile order = wave, round, lane)
__device__ __forceinline__ uint64_t item_of(uint32_t tile, uint32_t wv, int j, uint32_t lane) {
    return (uint64_t)tile * kTile + (uint64_t)wv * kSub + (uint64_t)j * 64 + lane;
}

// hist[d * ntiles + b] = items of tile b whose digit (bits [sh, sh + 8)) is d
__global__ __launch_bounds__(kThreads) void tile_hist(const uint64_t *__restrict__ keys, uint64_t n, uint32_t sh,
                                                      uint32_t *__restrict__ hist, uint32_t ntiles) {
    __shared__ uint32_t cnt[kDigits];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    cnt[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < kItems; ++j) {
        const uint64_t i = item_of(blockIdx.x, wv, j, lane);
        const bool valid = i < n;
        const uint32_t d = valid ? (uint32_t)(keys[i] >> sh) & (kDigits - 1) : 0u;
        const uint64_t peers = digit_peers(d, valid);
        // one atomic per distinct digit of the round (a hot key's run adds once)
        if (valid && lane == (uint32_t)__builtin_ctzll(peers)) atomicAdd(&cnt[d], (uint32_t)__builtin_popcountll(peers));
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = cnt[threadIdx.x];
}

// stable scatter of tile b: offs[d * ntiles + b] = the exclusive-scanned histogram (where tile
// b's first item of digit d goes)
__global__ __launch_bounds__(kThreads) void tile_scatter(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                         uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                         uint64_t n, uint32_t sh, const uint32_t *__restrict__ offs,
                                                         uint32_t ntiles) {
    __shared__ uint32_t wbase[kThreads / 64][kDigits];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) wbase[w][threadIdx.x] = 0;
    __syncthreads();
    uint64_t k[kItems];
    uint32_t v[kItems];
    // counts per wave (each wave writes only its own row; a round's leaders hold distinct digits)
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint64_t i = item_of(blockIdx.x, wv, j, lane);
        const bool valid = i < n;
        k[j] = valid ? kin[i] : 0ull;
        v[j] = valid ? vin[i] : 0u;
        const uint32_t d = (uint32_t)(k[j] >> sh) & (kDigits - 1);
        const uint64_t peers = digit_peers(d, valid);
        if (valid && lane == (uint32_t)__builtin_ctzll(peers)) wbase[wv][d] += (uint32_t)__builtin_popcountll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {  // per-wave bases: thread t owns digit t
        uint32_t run = offs[(uint64_t)threadIdx.x * ntiles + blockIdx.x];
#pragma unroll
        for (int w = 0; w < kThreads / 64; ++w) {
            const uint32_t c = wbase[w][threadIdx.x];
            wbase[w][threadIdx.x] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint64_t i = item_of(blockIdx.x, wv, j, lane);
        const bool valid = i < n;
        const uint32_t d = (uint32_t)(k[j] >> sh) & (kDigits - 1);
        const uint64_t peers = digit_peers(d, valid);
        const uint32_t base = valid ? wbase[wv][d] : 0u;
        __builtin_amdgcn_wave_barrier();  // every lane has read its base before a leader moves it
        if (valid) {
            const uint32_t pos = base + (uint32_t)__builtin_popcountll(peers & lanes_below(lane));
            if (pos < n) {  // always (the offsets partition [0, n)); a guard against a bad histogram
                kout[pos] = k[j];
                vout[pos] = v[j];
            }
            if (lane == (uint32_t)__builtin_ctzll(peers)) wbase[wv][d] = base + (uint32_t)__builtin_popcountll(peers);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- scans: tile b covers items [b * kTile, (b + 1) * kTile), thread t the kItems consecutive
// items from b * kTile + t * kItems

template <class T, class Op>
__device__ __forceinline__ T wave_incl_scan(T x, uint32_t lane) {
    Op op;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x = op(x, y);
    }
    return x;
}

// exclusive prefix of each thread's total across the workgroup (LDS for the 4 wave totals);
// *block_total = the workgroup's total
template <class T, class Op>
__device__ __forceinline__ T block_excl_scan(T x, T *lds4, T *block_total) {
    Op op;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const T incl = wave_incl_scan<T, Op>(x, lane);
    if (lane == 63) lds4[wv] = incl;
    __syncthreads();
    T wpre = Op::template identity<T>(), tot = Op::template identity<T>();
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        if ((uint32_t)w < wv) wpre = op(wpre, lds4[w]);
        tot = op(tot, lds4[w]);
    }
    __syncthreads();  // lds4 may be reused by the caller
    *block_total = tot;
    const T excl_in_wave = __shfl_up(incl, 1, 64);
    return lane ? op(wpre, excl_in_wave) : wpre;
}

template <class T, class Op>
__global__ __launch_bounds__(kThreads) void scan_reduce(const T *__restrict__ in, uint64_t n, T *__restrict__ partial) {
    __shared__ T lds4[kThreads / 64];
    Op op;
    const uint64_t b0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
    T s = Op::template identity<T>();
#pragma unroll
    for (int j = 0; j < kItems; ++j)
        if (b0 + j < n) s = op(s, in[b0 + j]);
    T tot;
    (void)block_excl_scan<T, Op>(s, lds4, &tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

// exclusive scan of m values in place by one workgroup (thread t: a contiguous run)
template <class T, class Op>
__global__ __launch_bounds__(kThreads) void scan_partials(T *__restrict__ p, uint64_t m) {
    __shared__ T lds4[kThreads / 64];
    Op op;
    const uint64_t per = (m + kThreads - 1) / kThreads;
    const uint64_t b0 = (uint64_t)threadIdx.x * per, b1 = b0 + per < m ? b0 + per : m;
    T s = Op::template identity<T>();
    for (uint64_t i = b0; i < b1; ++i) s = op(s, p[i]);
    T tot;
    T run = block_excl_scan<T, Op>(s, lds4, &tot);
    for (uint64_t i = b0; i < b1; ++i) {
        const T x = p[i];
        p[i] = run;
        run = op(run, x);
    }
}

template <class T, class Op, bool INCL>
__global__ __launch_bounds__(kThreads) void scan_down(const T *__restrict__ in, T *__restrict__ out, uint64_t n,
                                                      const T *__restrict__ partial) {
    __shared__ T lds4[kThreads / 64];
    Op op;
    const uint64_t b0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
    T x[kItems];
    T s = Op::template identity<T>();
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        x[j] = b0 + j < n ? in[b0 + j] : Op::template identity<T>();
        s = op(s, x[j]);
    }
    T tot;
    T run = op(partial[blockIdx.x], block_excl_scan<T, Op>(s, lds4, &tot));
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const T nx = op(run, x[j]);
        if (b0 + j < n) out[b0 + j] = INCL ? nx : run;
        run = nx;
    }
}

// scratch bytes of a scan of n items (the tile totals)
template <class T>
inline uint64_t scan_scratch(uint64_t n) { return ((tiles_for(n) * sizeof(T)) + 255) & ~255ull; }

// in -> out (may be the same array); `tmp`: scan_scratch<T>(n) bytes
template <class T, class Op, bool INCL>
inline void scan(const T *in, T *out, uint64_t n, void *tmp, hipStream_t s) {
    if (n == 0) return;
    const uint32_t nt = (uint32_t)tiles_for(n);
    T *part = (T *)tmp;
    scan_reduce<T, Op><<<nt, kThreads, 0, s>>>(in, n, part);
    scan_partials<T, Op><<<1, kThreads, 0, s>>>(part, nt);
    scan_down<T, Op, INCL><<<nt, kThreads, 0, s>>>(in, out, n, part);
}

// scratch bytes of sort_pairs_tiles over n items: the digit histograms and their scan's totals
inline uint64_t sort_scratch(uint64_t n) {
    const uint64_t m = tiles_for(n) * kDigits;
    return ((m * 4 + 255) & ~255ull) + scan_scratch<uint32_t>(m);
}

// stable sort of (ka[i], va[i]) by key bits [0, end_bit), using kb / vb as the other buffers;
// returns true when the result is in kb / vb, false when in ka / va
inline bool sort_pairs_tiles(uint64_t *ka, uint32_t *va, uint64_t *kb, uint32_t *vb, uint64_t n, int end_bit,
                             void *tmp, hipStream_t s) {
    if (n == 0) return false;
    const uint32_t nt = (uint32_t)tiles_for(n);
    const uint64_t m = (uint64_t)nt * kDigits;
    auto *hist = (uint32_t *)tmp;
    void *stmp = (uint8_t *)tmp + ((m * 4 + 255) & ~255ull);
    bool in_b = false;
    for (int sh = 0; sh < end_bit; sh += kRadixBits) {
        const uint64_t *ki = in_b ? kb : ka;
        const uint32_t *vi = in_b ? vb : va;
        uint64_t *ko = in_b ? ka : kb;
        uint32_t *vo = in_b ? va : vb;
        tile_hist<<<nt, kThreads, 0, s>>>(ki, n, (uint32_t)sh, hist, nt);
        scan<uint32_t, SumOp, false>(hist, hist, m, stmp, s);
        tile_scatter<<<nt, kThreads, 0, s>>>(ki, vi, ko, vo, n, (uint32_t)sh, hist, nt);
        in_b = !in_b;
    }
    return in_b;
}

}  // namespace tiles
}  // namespace stage
