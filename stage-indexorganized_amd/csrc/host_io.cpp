// host_io.cpp -- host-buffer entry points of the boundary (include/stage_hip.h):
//
//  * stage_probe_host: the batch probe for callers whose keys and result buffers live in host
//    memory.  Chunks of the batch rotate over three streams so the H2D of chunk i+1, the probe
//    of chunk i and the D2H of chunk i-1 overlap (PCIe in both directions + HBM at once).
//  * stage_reader_*: the single-key adapter of SURVEY §8(b) "Threading".  The reference calls
//    BTree::Read (b_tree.cpp:2066-2129) one key at a time from every worker thread
//    (IndexScanExecutor::Execute, executor.h:374-454); a reader coalesces those concurrent
//    calls into one device batch (group probe): callers append to the open batch and block,
//    a dispatcher thread ships a batch when it is full or its oldest request has waited
//    `max_wait_us`, and fills every caller's result before waking it.  While one batch is on
//    the device the next one fills, so the device and the callers overlap.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
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
    PipeLane lane[kPipeLanes];
};

static uint64_t lane_bytes(uint64_t stride) { return kPipeChunk * (8 + 2 + 4 + 32 + stride); }

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
    if (t->pipe && t->pipe->stride == stride && t->pipe->device == t->dev.device) return t->pipe.get();
    t->pipe.reset();
    std::unique_ptr<HostPipe, HostPipeDeleter> p(new HostPipe);
    p->device = t->dev.device;
    p->stride = stride;
    for (auto &l : p->lane) {
        hip_check(hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking), "pipe stream");
        hip_check(hipMalloc(&l.d, lane_bytes(stride)), "pipe buffers");
    }
    t->pipe = std::move(p);
    return t->pipe.get();
}

}  // namespace stage

namespace {

// one probe of n <= kPipeChunk keys on a lane: H2D inputs, probe, D2H results (all async)
hipError_t pipe_chunk(stage_table *t, stage::PipeLane &l, uint64_t stride, const uint64_t *keys, const uint16_t *lens,
                      const uint32_t *rids, uint64_t n, stage_probe_out *out, uint8_t *rows) {
    using stage::kPipeChunk;
    uint8_t *dk = l.d, *dl = dk + 8 * kPipeChunk, *dr = dl + 2 * kPipeChunk, *dout = dr + 4 * kPipeChunk,
            *drow = dout + 32 * kPipeChunk;
    hipError_t e = hipMemcpyAsync(dk, keys, 8 * n, hipMemcpyHostToDevice, l.s);
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

struct stage_reader {
    struct Req {
        uint64_t key;
        uint16_t len;
        uint32_t rid;
        stage_probe_out *out;
        uint8_t *rec;
        int *rc;
    };

    stage_table *t = nullptr;
    uint32_t max_batch = 0;
    uint32_t max_wait_us = 0;
    uint32_t row_bytes = 0;  // bytes handed to a caller: key padded to 8 + payload
    uint64_t stride = 0;

    std::mutex mu;
    std::condition_variable cv_work, cv_space, cv_done;
    std::vector<Req> open;
    std::chrono::steady_clock::time_point open_since;
    uint64_t open_gen = 1, done_gen = 0;
    bool stop = false;
    std::thread worker;

    hipStream_t s = nullptr;
    uint64_t *h_keys = nullptr;
    uint16_t *h_lens = nullptr;
    uint32_t *h_rids = nullptr;
    stage_probe_out *h_out = nullptr;
    uint8_t *h_rows = nullptr;
    uint8_t *d = nullptr;

    uint64_t n_batches = 0, n_reads = 0, n_full = 0;

    void run();
    int ship(std::vector<Req> &cur);
};

int stage_reader::ship(std::vector<Req> &cur) {
    const uint64_t n = cur.size();
    for (uint64_t i = 0; i < n; ++i) {
        h_keys[i] = cur[i].key;
        h_lens[i] = cur[i].len;
        h_rids[i] = cur[i].rid;
    }
    const uint64_t mb = max_batch;
    uint8_t *dk = d, *dl = dk + 8 * mb, *dr = dl + 2 * mb, *dout = dr + 4 * mb, *drow = dout + 32 * mb;
    hipError_t e = hipSetDevice(t->dev.device);
    if (!e) e = hipMemcpyAsync(dk, h_keys, 8 * n, hipMemcpyHostToDevice, s);
    if (!e) e = hipMemcpyAsync(dl, h_lens, 2 * n, hipMemcpyHostToDevice, s);
    if (!e) e = hipMemcpyAsync(dr, h_rids, 4 * n, hipMemcpyHostToDevice, s);
    if (!e) {
        stage::DevTable view = t->dev.view;
        view.stride = (uint32_t)stride;
        e = stage::launch_probe(view, (const uint64_t *)dk, (const uint16_t *)dl, (const uint32_t *)dr, nullptr, n,
                                (stage::stage_probe_out_dev *)dout, drow, s, t->tune);
    }
    if (!e) e = hipMemcpyAsync(h_out, dout, 32 * n, hipMemcpyDeviceToHost, s);
    if (!e) e = hipMemcpyAsync(h_rows, drow, stride * n, hipMemcpyDeviceToHost, s);
    if (!e) e = hipStreamSynchronize(s);
    if (e) return STAGE_E_HIP;
    for (uint64_t i = 0; i < n; ++i) {
        if (cur[i].out) *cur[i].out = h_out[i];
        if (cur[i].rec) std::memcpy(cur[i].rec, h_rows + i * stride, row_bytes);
    }
    return STAGE_OK;
}

void stage_reader::run() {
    std::vector<Req> cur;
    cur.reserve(max_batch);
    for (;;) {
        uint64_t gen;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_work.wait(lk, [&] { return stop || !open.empty(); });
            if (open.empty() && stop) return;
            const auto deadline = open_since + std::chrono::microseconds(max_wait_us);
            cv_work.wait_until(lk, deadline, [&] { return stop || open.size() >= max_batch; });
            cur.swap(open);
            gen = open_gen++;
        }
        cv_space.notify_all();
        const int rc = stage_capi::need_synced(t) ? STAGE_E_STATE : ship(cur);
        for (auto &r : cur) *r.rc = rc;
        {
            std::lock_guard<std::mutex> lk(mu);
            done_gen = gen;
            ++n_batches;
            n_reads += cur.size();
            if (cur.size() >= max_batch) ++n_full;
        }
        cv_done.notify_all();
        cur.clear();
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
            stage::hip_check(pipe_chunk(t, l, p->stride, keys + b, lens ? lens + b : nullptr,
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
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<stage_reader> r(new stage_reader);
        r->t = t;
        r->max_batch = max_batch;
        r->max_wait_us = max_wait_us;
        r->stride = t->host->stride();
        r->row_bytes = 8 + t->host->params().payload_size;
        const uint64_t mb = max_batch;
        stage::hip_check(hipSetDevice(t->dev.device), "hipSetDevice");
        stage::hip_check(hipStreamCreateWithFlags(&r->s, hipStreamNonBlocking), "reader stream");
        stage::hip_check(hipHostMalloc((void **)&r->h_keys, 8 * mb, hipHostMallocDefault), "reader pinned");
        stage::hip_check(hipHostMalloc((void **)&r->h_lens, 2 * mb, hipHostMallocDefault), "reader pinned");
        stage::hip_check(hipHostMalloc((void **)&r->h_rids, 4 * mb, hipHostMallocDefault), "reader pinned");
        stage::hip_check(hipHostMalloc((void **)&r->h_out, 32 * mb, hipHostMallocDefault), "reader pinned");
        stage::hip_check(hipHostMalloc((void **)&r->h_rows, r->stride * mb, hipHostMallocDefault), "reader pinned");
        stage::hip_check(hipMalloc((void **)&r->d, mb * (8 + 2 + 4 + 32 + r->stride)), "reader device");
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
    {
        std::unique_lock<std::mutex> lk(r->mu);
        r->cv_space.wait(lk, [&] { return r->stop || r->open.size() < r->max_batch; });
        if (r->stop) return fail(STAGE_E_STATE, "reader is closing");
        if (r->open.empty()) r->open_since = std::chrono::steady_clock::now();
        r->open.push_back({key, key_size, read_id, out, record, &rc});
        const uint64_t gen = r->open_gen;
        if (r->open.size() == 1 || r->open.size() >= r->max_batch) r->cv_work.notify_one();
        r->cv_done.wait(lk, [&] { return r->done_gen >= gen; });
    }
    if (rc) return fail(rc, rc == STAGE_E_STATE ? "device image is stale: call stage_sync after host writes"
                                                : "reader batch failed on the device");
    return STAGE_OK;
}

int stage_reader_stats(stage_reader *r, uint64_t *stats) {
    if (!r || !stats) return fail(STAGE_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(r->mu);
    stats[0] = r->n_batches;
    stats[1] = r->n_reads;
    stats[2] = r->n_full;
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
    if (r->s) (void)hipStreamDestroy(r->s);
    for (void *p : {(void *)r->h_keys, (void *)r->h_lens, (void *)r->h_rids, (void *)r->h_out, (void *)r->h_rows})
        if (p) (void)hipHostFree(p);
    if (r->d) (void)hipFree(r->d);
    delete r;
    return STAGE_OK;
}

}  // extern "C"
