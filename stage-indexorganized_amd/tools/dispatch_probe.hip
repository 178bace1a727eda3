// dispatch_probe.hip -- which workgroups get dispatched beside a CU-filling, HBM-bound kernel?
//
// in write-overlap mode the device write path's sort scatter (rocprim's onesweep
// pass, and three tile-scatter forms) did not run beside the read probe -- it ended when the
// probe ended -- while histogram and scan passes of the same grid did.  This tool reproduces
// the setting without the table: a "hog" kernel shaped like probe_kernel (256-thread blocks, a
// 16384-block grid-stride loop, random 16-B loads and streaming stores, no LDS) runs on a
// normal-priority stream; after it has filled the chip, small "guest" kernels (200 blocks of
// 256 threads, trivial work) are launched one after another on a high-priority stream, each
// with a given dynamic LDS size and number of block barriers.  Each guest's time on the guest
// stream is printed next to its time alone.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void hog(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t nsrc,
                                           uint64_t iters) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
    uint64_t h = gid * 0x9E3779B97F4A7C15ull + 1;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t it = 0; it < iters; ++it) {
        u32x4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            h ^= h >> 33;
            h *= 0xff51afd7ed558ccdull;
            v[k] = src[(h >> 7) % nsrc];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) acc += v[k];
        __builtin_nontemporal_store(acc, dst + ((gid + it * nth) % nsrc));
    }
}

// guest: NB block barriers, `dyn` bytes of dynamic LDS touched once
template <int NB>
__global__ __launch_bounds__(256) void guest(uint32_t *__restrict__ out, uint32_t n) {
    extern __shared__ uint32_t lds[];
    const uint32_t t = threadIdx.x;
    uint32_t v = t + blockIdx.x;
    lds[t] = v;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        __syncthreads();
        v += lds[(t + 1 + b) & 255];
    }
    const uint32_t i = blockIdx.x * 256 + t;
    if (i < n) out[i] = v;
}

// writer guests: 200 x 256 threads x 16 items of 8 B (the sort scatter's volume per pass) into a
// 6.7-MB array -- at hashed (scattered) or consecutive positions, with ordinary or nontemporal
// stores
template <bool SCATTER, bool NT>
__global__ __launch_bounds__(256) void writer(uint64_t *__restrict__ out, uint32_t m) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll 1
    for (int j = 0; j < 16; ++j) {
        const uint32_t i = t * 16 + j;
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        const uint32_t pos = SCATTER ? (uint32_t)(h % m) : (i % m);
        if (NT) __builtin_nontemporal_store((uint64_t)i, out + pos);
        else out[pos] = i;
    }
}

int main() {
    CK(hipSetDevice(0));
    const uint64_t nsrc = (6ull << 30) / 16;  // 6 GiB of 16-B items
    u32x4 *src, *dst;
    uint32_t *gout;
    CK(hipMalloc(&src, nsrc * 16));
    CK(hipMalloc(&dst, nsrc * 16));
    CK(hipMalloc(&gout, 200 * 256 * 4));
    CK(hipMemset(src, 1, nsrc * 16));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t sh, sg;
    CK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&sg, hipStreamNonBlocking, hi));
    hipEvent_t h0, h1;
    CK(hipEventCreate(&h0));
    CK(hipEventCreate(&h1));
    struct V {
        int nb;
        uint32_t lds;
    };
    std::vector<V> vs = {{0, 1024}, {2, 1024}, {3, 1024}, {0, 4096}, {3, 4096}, {0, 16384}, {3, 16384}, {3, 55296}};
    auto launch_guest = [&](const V &v, hipStream_t s) {
        if (v.nb == 0) guest<0><<<200, 256, v.lds, s>>>(gout, 200 * 256);
        else if (v.nb == 2) guest<2><<<200, 256, v.lds, s>>>(gout, 200 * 256);
        else guest<3><<<200, 256, v.lds, s>>>(gout, 200 * 256);
    };
    // the hog alone
    const uint64_t iters = 6;  // ~9 ms
    hog<<<16384, 256, 0, sh>>>(src, dst, nsrc, iters);
    CK(hipStreamSynchronize(sh));
    CK(hipEventRecord(h0, sh));
    hog<<<16384, 256, 0, sh>>>(src, dst, nsrc, iters);
    CK(hipEventRecord(h1, sh));
    CK(hipStreamSynchronize(sh));
    float hog_ms = 0;
    CK(hipEventElapsedTime(&hog_ms, h0, h1));
    std::printf("hog alone: %.3f ms\n", hog_ms);
    for (const V &v : vs) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        // alone
        launch_guest(v, sg);
        CK(hipEventRecord(a, sg));
        launch_guest(v, sg);
        CK(hipEventRecord(b, sg));
        CK(hipStreamSynchronize(sg));
        float alone = 0;
        CK(hipEventElapsedTime(&alone, a, b));
        // beside the hog, launched ~1 ms after it started
        CK(hipEventRecord(h0, sh));
        hog<<<16384, 256, 0, sh>>>(src, dst, nsrc, iters);
        CK(hipEventRecord(h1, sh));
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        CK(hipEventRecord(a, sg));
        launch_guest(v, sg);
        CK(hipEventRecord(b, sg));
        CK(hipDeviceSynchronize());
        float beside = 0, hog2 = 0, from_hog = 0;
        CK(hipEventElapsedTime(&beside, a, b));
        CK(hipEventElapsedTime(&hog2, h0, h1));
        CK(hipEventElapsedTime(&from_hog, h0, b));
        std::printf("guest barriers %d lds %6u B: alone %.3f ms, beside the hog %.3f ms (ends %.3f ms after the hog's start; hog %.3f ms)\n",
                    v.nb, v.lds, alone, beside, from_hog, hog2);
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
    }
    uint64_t *wout;
    const uint32_t m = 838000;
    CK(hipMalloc(&wout, (uint64_t)m * 8));
    auto launch_writer = [&](int kind, hipStream_t s) {
        if (kind == 0) writer<true, false><<<200, 256, 0, s>>>(wout, m);
        else if (kind == 1) writer<true, true><<<200, 256, 0, s>>>(wout, m);
        else writer<false, false><<<200, 256, 0, s>>>(wout, m);
    };
    const char *names[3] = {"scattered ordinary stores", "scattered nontemporal stores", "consecutive ordinary stores"};
    for (int kind = 0; kind < 3; ++kind) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        launch_writer(kind, sg);
        CK(hipEventRecord(a, sg));
        launch_writer(kind, sg);
        CK(hipEventRecord(b, sg));
        CK(hipStreamSynchronize(sg));
        float alone = 0;
        CK(hipEventElapsedTime(&alone, a, b));
        CK(hipEventRecord(h0, sh));
        hog<<<16384, 256, 0, sh>>>(src, dst, nsrc, iters);
        CK(hipEventRecord(h1, sh));
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        CK(hipEventRecord(a, sg));
        launch_writer(kind, sg);
        CK(hipEventRecord(b, sg));
        CK(hipDeviceSynchronize());
        float beside = 0, hog2 = 0, from_hog = 0;
        CK(hipEventElapsedTime(&beside, a, b));
        CK(hipEventElapsedTime(&hog2, h0, h1));
        CK(hipEventElapsedTime(&from_hog, h0, b));
        std::printf("writer, %s: alone %.3f ms, beside the hog %.3f ms (ends %.3f ms after the hog's start; hog %.3f ms)\n",
                    names[kind], alone, beside, from_hog, hog2);
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
    }
    return 0;
}
