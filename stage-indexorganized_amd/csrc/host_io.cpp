// host_io.cpp -- host-buffer entry points of the boundary (include/stage_hip.h):
//
//  * stage_probe_host: the batch probe for callers whose keys and result buffers live in host
//    memory.  Chunks of the batch rotate over three streams so the H2D of chunk i+1, the probe
//    of chunk i and the D2H of chunk i-1 overlap (PCIe in both directions + HBM at once).
//  * stage_reader_*: the single-key adapter of SURVEY §8(b) "Threading".  The reference calls
//    BTree::Read (b_tree.cpp:2066-2129) one key at a time from every worker thread
//    (IndexScanExecutor::Execute, executor.h:374-454); a reader coalesces those concurrent
//    calls into one device batch (group probe): callers append to the open batch and block,
//    a dispatcher thread ships a batch when it is full, when its oldest request has waited
//    `max_wait_us` or when arrivals have paused, and fills every caller's result before
//    waking it.  The batch is one probe launch reading keys from and writing results to
//    pinned, device-mapped host memory (no separate copies).  While one batch is on the
//    device the next one fills.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <climits>
#include <cstring>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <mutex>
#include <thread>
#include <vector>

#include "handle.hpp"

using namespace stage_capi;

namespace stage {

constexpr int kPipeLanes = 3;
constexpr uint64_t kPipeChunk = 1ull << 17;  // probes per chunk (128 MiB of rows per lane)

struct PipeLane {
    hipStream_t s = nullptr;
    uint8_t *d = nullptr;  // keys | lens | read ids | out | rows
};

struct HostPipe {
    int device = 0;
    uint64_t stride = 0;
    uint32_t kw = 1;  // u64 key words per probe
    PipeLane lane[kPipeLanes];
};

static uint64_t lane_bytes(uint64_t stride, uint32_t kw) { return kPipeChunk * (8ull * kw + 2 + 4 + 32 + stride); }

void host_pipe_release(HostPipe *p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    for (auto &l : p->lane) {
        if (l.s) (void)hipStreamSynchronize(l.s), (void)hipStreamDestroy(l.s);
        if (l.d) (void)hipFree(l.d);
    }
    delete p;
}

static HostPipe *get_pipe(stage_table *t) {
    const uint64_t stride = t->out_stride ? t->out_stride : t->dev.view.stride;
    const uint32_t kw = host(t).key_words();
    if (t->pipe && t->pipe->stride == stride && t->pipe->kw == kw && t->pipe->device == t->dev.device)
        return t->pipe.get();
    t->pipe.reset();
    std::unique_ptr<HostPipe, HostPipeDeleter> p(new HostPipe);
    p->device = t->dev.device;
    p->stride = stride;
    p->kw = kw;
    for (auto &l : p->lane) {
        hip_check(hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking), "pipe stream");
        hip_check(hipMalloc(&l.d, lane_bytes(stride, kw)), "pipe buffers");
    }
    t->pipe = std::move(p);
    return t->pipe.get();
}

}  // namespace stage

namespace {

// one probe of n <= kPipeChunk keys on a lane: H2D inputs, probe, D2H results (all async)
hipError_t pipe_chunk(stage_table *t, stage::PipeLane &l, uint64_t stride, uint32_t kw, const uint64_t *keys,
                      const uint16_t *lens, const uint32_t *rids, uint64_t n, stage_probe_out *out, uint8_t *rows) {
    using stage::kPipeChunk;
    uint8_t *dk = l.d, *dl = dk + 8ull * kw * kPipeChunk, *dr = dl + 2 * kPipeChunk, *dout = dr + 4 * kPipeChunk,
            *drow = dout + 32 * kPipeChunk;
    hipError_t e = hipMemcpyAsync(dk, keys, 8ull * kw * n, hipMemcpyHostToDevice, l.s);
    if (!e && lens) e = hipMemcpyAsync(dl, lens, 2 * n, hipMemcpyHostToDevice, l.s);
    if (!e && rids) e = hipMemcpyAsync(dr, rids, 4 * n, hipMemcpyHostToDevice, l.s);
    if (e) return e;
    stage::DevTable view = t->dev.view;
    view.stride = (uint32_t)stride;
    e = stage::launch_probe(view, (const uint64_t *)dk, lens ? (const uint16_t *)dl : nullptr,
                            rids ? (const uint32_t *)dr : nullptr, nullptr, n, (stage::stage_probe_out_dev *)dout,
                            rows ? drow : nullptr, l.s, t->tune);
    if (!e) e = hipMemcpyAsync(out, dout, 32 * n, hipMemcpyDeviceToHost, l.s);
    if (!e && rows) e = hipMemcpyAsync(rows, drow, stride * n, hipMemcpyDeviceToHost, l.s);
    return e;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// the coalescing reader

namespace {

long futex(std::atomic<uint32_t> *addr, int op, uint32_t val) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t *>(addr), op, val, nullptr, nullptr, 0);
}

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace

struct stage_reader {
    struct Req {
        uint64_t key;
        uint16_t len;
        uint32_t rid;
        stage_probe_out *out;
        uint8_t *rec;
        int *rc;
    };
    // one batch buffer: a pinned, device-mapped block the probe kernel reads the keys from and
    // writes the results to directly over PCIe (zero-copy: one launch, no copies)
    struct Slot {
        hipStream_t s = nullptr;
        hipEvent_t ev = nullptr;
        uint8_t *h = nullptr;   // keys | lens | read ids | out | rows
        uint8_t *hd = nullptr;  // the same block as the device sees it
        std::vector<Req> reqs;
        uint32_t seq = 0;
        bool busy = false;
    };
    static constexpr int kSlots = 2;

    stage_table *t = nullptr;
    uint32_t max_batch = 0;
    uint32_t max_wait_us = 0;
    uint32_t row_bytes = 0;  // bytes handed to a caller: key padded to 8 + payload
    uint64_t stride = 0;

    std::mutex mu;  // guards open/stop; callers hold it only to append
    std::condition_variable cv_work, cv_space;
    std::vector<Req> open;
    uint32_t open_seq = 1;  // sequence number the open batch will carry
    std::atomic<uint32_t> open_count{0};
    std::atomic<int64_t> first_arrival_ns{0}, last_arrival_ns{0};
    std::atomic<uint32_t> done_seq{0};  // every batch with seq <= done_seq is complete (futex word)
    bool stop = false;
    std::thread worker;
    Slot slot[kSlots];

    std::atomic<uint64_t> n_batches{0}, n_reads{0}, n_full{0};

    void run();
    void launch(Slot &sl);
    void complete(Slot &sl);
};

void stage_reader::launch(Slot &sl) {
    const uint64_t n = sl.reqs.size(), mb = max_batch;
    uint64_t *keys = (uint64_t *)sl.h;
    uint16_t *lens = (uint16_t *)(sl.h + 8 * mb);
    uint32_t *rids = (uint32_t *)(sl.h + 10 * mb);
    for (uint64_t i = 0; i < n; ++i) {
        keys[i] = sl.reqs[i].key;
        lens[i] = sl.reqs[i].len;
        rids[i] = sl.reqs[i].rid;
    }
    stage::DevTable view = t->dev.view;
    view.stride = (uint32_t)stride;
    hipError_t e = stage_capi::need_synced(t) ? hipErrorInvalidValue : hipSuccess;
    const int stale = e != hipSuccess;
    if (!e)
        e = stage::launch_probe(view, (const uint64_t *)sl.hd, (const uint16_t *)(sl.hd + 8 * mb),
                                (const uint32_t *)(sl.hd + 10 * mb), nullptr, n,
                                (stage::stage_probe_out_dev *)(sl.hd + 14 * mb), sl.hd + 46 * mb, sl.s, t->tune);
    if (!e) e = hipEventRecord(sl.ev, sl.s);
    if (e) {  // fail the batch now; complete() only delivers
        for (auto &r : sl.reqs) *r.rc = stale ? STAGE_E_STATE : STAGE_E_HIP;
        sl.reqs.clear();
    }
    sl.busy = true;
}

void stage_reader::complete(Slot &sl) {
    const uint64_t n = sl.reqs.size(), mb = max_batch;
    const stage_probe_out *out = (const stage_probe_out *)(sl.h + 14 * mb);
    const uint8_t *rows = sl.h + 46 * mb;
    if (n && hipEventSynchronize(sl.ev) != hipSuccess) {
        for (auto &r : sl.reqs) *r.rc = STAGE_E_HIP;
    } else {
        for (uint64_t i = 0; i < n; ++i) {
            const Req &r = sl.reqs[i];
            if (r.out) *r.out = out[i];
            if (r.rec) std::memcpy(r.rec, rows + i * stride, row_bytes);
            *r.rc = STAGE_OK;
        }
    }
    n_batches++;
    n_reads += n;
    if (n >= max_batch) n_full++;
    sl.reqs.clear();
    sl.busy = false;
    done_seq.store(sl.seq, std::memory_order_release);
    futex(&done_seq, FUTEX_WAKE_PRIVATE, INT32_MAX);
}

// Dispatch rule: a batch leaves when it is full, when its oldest request has waited
// max_wait_us, or when no request has arrived for kGapNs (the callers of the previous batch
// have come back).  Two batches can be in flight; they complete in launch order.  The
// dispatcher sleeps only when nothing is open or in flight.
constexpr int64_t kGapNs = 3000;

void stage_reader::run() {
    (void)hipSetDevice(t->dev.device);
    int next = 0;  // slot the next batch goes to (slots are used round robin)
    int oldest = 0;
    for (;;) {
        // deliver the oldest in-flight batch once its event has fired
        if (slot[oldest].busy && (slot[oldest].reqs.empty() || hipEventQuery(slot[oldest].ev) != hipErrorNotReady)) {
            complete(slot[oldest]);
            oldest ^= 1;
            continue;
        }
        const bool any_busy = slot[0].busy || slot[1].busy;
        const uint32_t cnt = open_count.load(std::memory_order_acquire);
        if (cnt == 0) {
            if (any_busy) {
                std::this_thread::yield();
                continue;
            }
            std::unique_lock<std::mutex> lk(mu);
            cv_work.wait(lk, [&] { return stop || !open.empty(); });
            if (open.empty() && stop) return;
            continue;
        }
        if (slot[next].busy) {  // both slots in flight: wait for the oldest
            std::this_thread::yield();
            continue;
        }
        const int64_t now = now_ns();
        if (cnt < max_batch && now < first_arrival_ns.load(std::memory_order_acquire) + (int64_t)max_wait_us * 1000 &&
            now - last_arrival_ns.load(std::memory_order_acquire) < kGapNs) {
            std::this_thread::yield();
            continue;
        }
        Slot &sl = slot[next];
        {
            std::lock_guard<std::mutex> lk(mu);
            sl.reqs.swap(open);
            sl.seq = open_seq++;
            open_count.store(0, std::memory_order_release);
        }
        cv_space.notify_all();
        launch(sl);
        next ^= 1;
    }
}

extern "C" {

int stage_host_alloc(uint64_t bytes, void **ptr) {
    if (!ptr) return fail(STAGE_E_ARG, "null pointer");
    return hip_rc(hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocDefault), "hipHostMalloc");
}

int stage_host_free(void *ptr) { return hip_rc(hipHostFree(ptr), "hipHostFree"); }

int stage_probe_host(stage_table *t, const uint64_t *keys, const uint16_t *lens, const uint32_t *read_ids, uint64_t n,
                     stage_probe_out *out, uint8_t *records) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (n && (!keys || !out)) return fail(STAGE_E_ARG, "null host buffer");
    if (n == 0) return STAGE_OK;
    std::lock_guard<std::mutex> lk(t->pipe_mu);
    return guarded([&] {
        stage::hip_check(hipSetDevice(t->dev.device), "hipSetDevice");
        stage::HostPipe *p = stage::get_pipe(t);
        const uint64_t chunks = (n + stage::kPipeChunk - 1) / stage::kPipeChunk;
        for (uint64_t c = 0; c < chunks; ++c) {
            stage::PipeLane &l = p->lane[c % stage::kPipeLanes];
            if (c >= (uint64_t)stage::kPipeLanes) stage::hip_check(hipStreamSynchronize(l.s), "pipe lane");
            const uint64_t b = c * stage::kPipeChunk, m = std::min<uint64_t>(stage::kPipeChunk, n - b);
            stage::hip_check(pipe_chunk(t, l, p->stride, p->kw, keys + b * p->kw, lens ? lens + b : nullptr,
                                        read_ids ? read_ids + b : nullptr, m, out + b,
                                        records ? records + b * p->stride : nullptr),
                             "probe_host chunk");
        }
        for (auto &l : p->lane) stage::hip_check(hipStreamSynchronize(l.s), "pipe drain");
        return STAGE_OK;
    });
}

int stage_reader_create(stage_table *t, uint32_t max_batch, uint32_t max_wait_us, stage_reader **out) {
    if (!t || !out || max_batch == 0 || max_batch > (1u << 20)) return fail(STAGE_E_ARG, "bad reader arguments");
    if (host(t).key_words() != 1) return fail(STAGE_E_ARG, "the single-key reader takes keys of <= 8 bytes");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<stage_reader> r(new stage_reader);
        r->t = t;
        r->max_batch = max_batch;
        r->max_wait_us = max_wait_us;
        r->stride = host(t).stride();
        r->row_bytes = 8 + host(t).params().payload_size;
        const uint64_t mb = max_batch, bytes = mb * (8 + 2 + 4 + 32 + r->stride);
        stage::hip_check(hipSetDevice(t->dev.device), "hipSetDevice");
        for (auto &sl : r->slot) {
            stage::hip_check(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking), "reader stream");
            stage::hip_check(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming), "reader event");
            stage::hip_check(hipHostMalloc((void **)&sl.h, bytes, hipHostMallocMapped | hipHostMallocPortable),
                             "reader pinned");
            stage::hip_check(hipHostGetDevicePointer((void **)&sl.hd, sl.h, 0), "reader mapped pointer");
            sl.reqs.reserve(max_batch);
        }
        r->open.reserve(max_batch);
        stage_reader *raw = r.get();
        r->worker = std::thread([raw] { raw->run(); });
        *out = r.release();
        return STAGE_OK;
    });
}

int stage_reader_read(stage_reader *r, uint64_t key, uint16_t key_size, uint32_t read_id, stage_probe_out *out,
                      uint8_t *record) {
    if (!r) return fail(STAGE_E_ARG, "null reader");
    if (key_size == 0 || key_size > 8) return fail(STAGE_E_ARG, "key_size must be 1..8");
    int rc = STAGE_E_STATE;
    uint32_t seq;
    {
        std::unique_lock<std::mutex> lk(r->mu);
        r->cv_space.wait(lk, [&] { return r->stop || r->open.size() < r->max_batch; });
        if (r->stop) return fail(STAGE_E_STATE, "reader is closing");
        r->open.push_back({key, key_size, read_id, out, record, &rc});
        const int64_t now = now_ns();
        if (r->open.size() == 1) r->first_arrival_ns.store(now, std::memory_order_release);
        r->last_arrival_ns.store(now, std::memory_order_release);
        r->open_count.store((uint32_t)r->open.size(), std::memory_order_release);
        seq = r->open_seq;
        if (r->open.size() == 1) r->cv_work.notify_one();
    }
    for (;;) {  // wait for batch `seq` (sequence numbers wrap: compare as a signed distance)
        const uint32_t d = r->done_seq.load(std::memory_order_acquire);
        if ((int32_t)(d - seq) >= 0) break;
        futex(&r->done_seq, FUTEX_WAIT_PRIVATE, d);
    }
    if (rc) return fail(rc, rc == STAGE_E_STATE ? "device image is stale: call stage_sync after host writes"
                                                : "reader batch failed on the device");
    return STAGE_OK;
}

int stage_reader_stats(stage_reader *r, uint64_t *stats) {
    if (!r || !stats) return fail(STAGE_E_ARG, "null argument");
    stats[0] = r->n_batches.load();
    stats[1] = r->n_reads.load();
    stats[2] = r->n_full.load();
    return STAGE_OK;
}

int stage_reader_destroy(stage_reader *r) {
    if (!r) return STAGE_OK;
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->stop = true;
    }
    r->cv_work.notify_all();
    r->cv_space.notify_all();
    if (r->worker.joinable()) r->worker.join();
    (void)hipSetDevice(r->t->dev.device);
    for (auto &sl : r->slot) {
        if (sl.s) (void)hipStreamSynchronize(sl.s), (void)hipStreamDestroy(sl.s);
        if (sl.ev) (void)hipEventDestroy(sl.ev);
        if (sl.h) (void)hipHostFree(sl.h);
    }
    delete r;
    return STAGE_OK;
}

}  // extern "C"
