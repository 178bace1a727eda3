// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access
// shapes probe_kernel uses (MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of a wide coalesced
// streaming read; "other access widths are uncalibrated").  Each kernel touches a known
// number of bytes in a 32 GiB buffer (far beyond the 256 MiB Infinity Cache), at random
// aligned positions, in the shape named by the kernel:
//   calib_stream16      64 lanes x 16 B coalesced, streaming          (reference shape)
//   calib_rand64_b1     one random 64-B sector per wave, 1 B per lane  (probe: fingerprint sector)
//   calib_rand64_b16    one random 64-B sector per 4 lanes, 16 B/lane  (probe: bottom separator node)
//   calib_rand32_b16    one random 32-B word per 2 lanes, 16 B/lane    (probe: candidate slot word)
//   calib_rand128_b16   one random 128-B line per 8 lanes, 16 B/lane   (probe: inner separator node)
//   calib_rand1024_b16  one random 1024-B row per wave, 16 B/lane      (probe: heap row)
//   calib_wstream16     64 lanes x 16 B streaming nontemporal stores   (probe: output rows)
//   calib_wrand32       one random 32-B record per 2 lanes, 16 B/lane stores (status records)
// Prints one JSON line per kernel: {"kernel", "bytes_per_launch", "launches", "ms"}; the PMC
// pass divides FETCH_SIZE (or WRITE_SIZE) per dispatch by bytes_per_launch.
//   fetch_calib [gib=32] [launches=3]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

// unit u (a sector / word / line / row of `bytes` B) at a random aligned offset in [0, span)
__device__ __forceinline__ uint64_t unit_off(uint64_t u, uint64_t span, uint32_t bytes, uint64_t seed) {
    return (mix(u * 0x9E3779B97F4A7C15ull + seed) % (span / bytes)) * bytes;
}

__global__ void calib_stream16(const u32x4 *__restrict__ p, uint64_t n16, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void calib_rand64_b1(const uint8_t *__restrict__ p, uint64_t span, uint64_t units, uint64_t seed,
                                uint32_t *__restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t acc = 0;
    for (uint64_t u = w0; u < units; u += nw) acc += p[unit_off(u, span, 64, seed) + lane];
    if (acc == 0x12345678u) sink[0] = acc;
}

template <uint32_t BYTES>
__global__ void calib_rand_b16(const uint8_t *__restrict__ p, uint64_t span, uint64_t units, uint64_t seed,
                               uint32_t *__restrict__ sink) {
    constexpr uint32_t L = BYTES / 16;  // lanes per unit
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t ng = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t t = g; t < units * L; t += ng) {
        const uint64_t u = t / L;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(p + unit_off(u, span, BYTES, seed) + (t % L) * 16);
        acc ^= v.x ^ v.z;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void calib_wstream16(u32x4 *__restrict__ p, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(u32x4{(uint32_t)i, 1u, 2u, 3u}, p + i);
}

__global__ void calib_wrand32(uint8_t *__restrict__ p, uint64_t span, uint64_t units, uint64_t seed) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t ng = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = g; t < units * 2; t += ng) {
        const uint64_t u = t / 2;
        *reinterpret_cast<u32x4 *>(p + unit_off(u, span, 32, seed) + (t % 2) * 16) = u32x4{(uint32_t)t, 0u, 0u, 0u};
    }
}

int main(int argc, char **argv) {
    const uint64_t gib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 32;
    const int launches = argc > 2 ? std::atoi(argv[2]) : 3;
    const uint64_t span = gib << 30;
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr;
    CK(hipMalloc(&buf, span));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, span));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = 16384, block = 256;
    const uint64_t units = 1ull << 24;  // random units per launch (>> Infinity Cache lines)
    auto run = [&](const char *name, uint64_t bytes, auto launch) {
        launch(0);  // warm-up, not reported
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < launches; ++i) launch(i + 1);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        std::printf("{\"kernel\": \"%s\", \"bytes_per_launch\": %llu, \"launches\": %d, \"ms_per_launch\": %.4f, "
                    "\"GBps\": %.1f}\n",
                    name, (unsigned long long)bytes, launches, ms / launches, bytes / (ms / launches * 1e-3) / 1e9);
    };
    const uint64_t n16 = span / 16 / 4;  // stream over a quarter of the buffer (8 GiB)
    run("calib_stream16", n16 * 16, [&](int) { calib_stream16<<<grid, block>>>((const u32x4 *)buf, n16, sink); });
    run("calib_rand64_b1", units * 64,
        [&](int s) { calib_rand64_b1<<<grid, block>>>(buf, span, units, 0x1000 + s, sink); });
    run("calib_rand64_b16", units * 64,
        [&](int s) { calib_rand_b16<64><<<grid, block>>>(buf, span, units, 0x2000 + s, sink); });
    run("calib_rand32_b16", units * 32,
        [&](int s) { calib_rand_b16<32><<<grid, block>>>(buf, span, units, 0x3000 + s, sink); });
    run("calib_rand128_b16", units * 128,
        [&](int s) { calib_rand_b16<128><<<grid, block>>>(buf, span, units, 0x4000 + s, sink); });
    run("calib_rand1024_b16", (units / 8) * 1024,
        [&](int s) { calib_rand_b16<1024><<<grid, block>>>(buf, span, units / 8, 0x5000 + s, sink); });
    run("calib_wstream16", n16 * 16, [&](int) { calib_wstream16<<<grid, block>>>((u32x4 *)buf, n16); });
    run("calib_wrand32", units * 32, [&](int s) { calib_wrand32<<<grid, block>>>(buf, span, units, 0x6000 + s); });
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
