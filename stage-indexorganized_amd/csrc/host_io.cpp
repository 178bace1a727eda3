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
//  * stage_reader_create_resident: the same adapter with the device side resident
//    (resident_reader_kernel, kernels.hip) polling a request ring in pinned host memory -- a
//    read costs no launch, no event and no thread hand-off, only PCIe round trips.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <climits>
#include <cstring>
#include <immintrin.h>
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
    const uint32_t kw = facts(t).key_words();
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
    stage::ProbeTuning tune = t->tune;
    tune.status_bytes = t->status_bytes;  // 16: stage_probe_out16 records, packed
    e = stage::launch_probe(view, (const uint64_t *)dk, lens ? (const uint16_t *)dl : nullptr,
                            rids ? (const uint32_t *)dr : nullptr, nullptr, n, (stage::stage_probe_out_dev *)dout,
                            rows ? drow : nullptr, l.s, tune);
    if (!e) e = hipMemcpyAsync(out, dout, (uint64_t)tune.status_bytes * n, hipMemcpyDeviceToHost, l.s);
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

// the resident form: request ring + keeper thread (see stage_reader_create_resident)
struct ResidentReader {
    stage_table *t = nullptr;
    uint32_t slots = 0, waves = 0, row_bytes = 0;
    uint64_t stride = 0, life_ticks = 0;
    uint8_t *h = nullptr, *hd = nullptr;  // ring block, host and device view
    stage::ReaderReq *req = nullptr;
    uint32_t *done = nullptr, *stop = nullptr;
    stage_probe_out *out = nullptr;
    uint8_t *rows = nullptr;
    stage_probe_ident *ident = nullptr;   // per slot: the read's location / next handles
    uint64_t *dpos = nullptr;             // device: next ticket per wave
    stage::ReaderRing ring{};             // device pointers
    std::unique_ptr<std::atomic<uint64_t>[]> freed;  // per slot: ticket + 1 of its last finished reader
    std::atomic<uint64_t> tail{0};
    std::atomic<int> dead{0};             // STAGE_E_STATE / STAGE_E_HIP once the device side ended
    std::atomic<bool> closing{false}, quit{false};
    std::atomic<uint64_t> n_inst{0}, n_reads{0};
    hipStream_t s = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    std::thread keeper;
    void run();
};

void ResidentReader::run() {
    (void)hipSetDevice(t->dev.device);
    int k = 0;
    bool queued[2] = {false, false};
    while (!quit.load(std::memory_order_acquire)) {
        if (queued[k]) {  // two instances queued: wait for the older one before adding a third
            if (hipEventSynchronize(ev[k]) != hipSuccess) {
                dead.store(STAGE_E_HIP);
                break;
            }
            queued[k] = false;
            if (quit.load(std::memory_order_acquire)) break;
        }
        if (stage_capi::need_synced(t)) {
            dead.store(STAGE_E_STATE);
            break;
        }
        stage::DevTable view = t->dev.view;
        view.stride = (uint32_t)stride;
        hipError_t e = stage::launch_resident_reader(view, ring, s);
        if (!e) e = hipEventRecord(ev[k], s);
        if (e) {
            dead.store(STAGE_E_HIP);
            break;
        }
        queued[k] = true;
        n_inst++;
        k ^= 1;
    }
    __atomic_store_n(stop, 1u, __ATOMIC_RELEASE);  // running instances end at their next poll
    (void)hipStreamSynchronize(s);
    if (!dead.load()) dead.store(STAGE_E_STATE);
}

struct stage_reader {
    std::unique_ptr<ResidentReader> res;  // set for the resident kind
    struct Req {
        uint64_t key;
        uint16_t len;
        uint32_t rid;
        bool for_update;
        stage_probe_out *out;
        uint8_t *rec;
        stage_probe_ident *ident;
        int *rc;
    };
    // one batch buffer: a pinned, device-mapped block the probe kernel reads the keys from and
    // writes the results to directly over PCIe (zero-copy: one launch + the ident pass, no copies)
    struct Slot {
        hipStream_t s = nullptr;
        hipEvent_t ev = nullptr;
        uint8_t *h = nullptr;   // keys | lens | read ids | out | rows | ident
        uint8_t *hd = nullptr;  // the same block as the device sees it
        std::vector<Req> reqs;
        uint32_t seq = 0;
        bool busy = false;
    };
    static constexpr int kSlots = 2;
    // byte offsets of a slot block's arrays, each 16-B aligned (the kernels store 16-B records
    // and 8-B ident pairs there whatever max_batch is)
    struct Layout {
        uint64_t lens, rids, fu, out, rows, ident, bytes;
    };
    Layout lay{};

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
    const uint64_t n = sl.reqs.size();
    uint64_t *keys = (uint64_t *)sl.h;
    uint16_t *lens = (uint16_t *)(sl.h + lay.lens);
    uint32_t *rids = (uint32_t *)(sl.h + lay.rids);
    uint8_t *fu = sl.h + lay.fu;
    bool any_fu = false;
    for (uint64_t i = 0; i < n; ++i) {
        keys[i] = sl.reqs[i].key;
        lens[i] = sl.reqs[i].len;
        rids[i] = sl.reqs[i].rid;
        fu[i] = sl.reqs[i].for_update ? 1 : 0;
        any_fu = any_fu || sl.reqs[i].for_update;
    }
    stage::DevTable view = t->dev.view;
    view.stride = (uint32_t)stride;
    hipError_t e = stage_capi::need_synced(t) ? hipErrorInvalidValue : hipSuccess;
    const int stale = e != hipSuccess;
    auto *dout = (stage::stage_probe_out_dev *)(sl.hd + lay.out);
    if (!e)
        e = stage::launch_probe(view, (const uint64_t *)sl.hd, (const uint16_t *)(sl.hd + lay.lens),
                                (const uint32_t *)(sl.hd + lay.rids), nullptr, n, dout, sl.hd + lay.rows, sl.s, t->tune);
    if (!e && any_fu)  // the batch's is_for_update reads (BTree::Read(..., true)) re-answered
        e = stage::launch_for_update(view, sl.hd + lay.fu, (const uint32_t *)(sl.hd + lay.rids), n, dout,
                                     sl.hd + lay.rows, sl.s);
    if (!e) e = stage::launch_ident(view, dout, n, (uint32_t *)(sl.hd + lay.ident), sl.s);
    if (!e) e = hipEventRecord(sl.ev, sl.s);
    if (e) {  // fail the batch now; complete() only delivers
        for (auto &r : sl.reqs) *r.rc = stale ? STAGE_E_STATE : STAGE_E_HIP;
        sl.reqs.clear();
    }
    sl.busy = true;
}

void stage_reader::complete(Slot &sl) {
    const uint64_t n = sl.reqs.size();
    const stage_probe_out *out = (const stage_probe_out *)(sl.h + lay.out);
    const uint8_t *rows = sl.h + lay.rows;
    const stage_probe_ident *ident = (const stage_probe_ident *)(sl.h + lay.ident);
    if (n && hipEventSynchronize(sl.ev) != hipSuccess) {
        for (auto &r : sl.reqs) *r.rc = STAGE_E_HIP;
    } else {
        for (uint64_t i = 0; i < n; ++i) {
            const Req &r = sl.reqs[i];
            if (r.out) *r.out = out[i];
            if (r.rec) std::memcpy(r.rec, rows + i * stride, row_bytes);
            if (r.ident) *r.ident = ident[i];
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
    // mapped: kernels may write results straight into it (stage_ch_query2_batch's `out`)
    return hip_rc(hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocMapped), "hipHostMalloc");
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
            // out: n records of the table's status layout (32 or 16 B)
            auto *ob = reinterpret_cast<stage_probe_out *>(reinterpret_cast<uint8_t *>(out) + b * (uint64_t)t->status_bytes);
            stage::hip_check(pipe_chunk(t, l, p->stride, p->kw, keys + b * p->kw, lens ? lens + b : nullptr,
                                        read_ids ? read_ids + b : nullptr, m, ob,
                                        records ? records + b * p->stride : nullptr),
                             "probe_host chunk");
        }
        for (auto &l : p->lane) stage::hip_check(hipStreamSynchronize(l.s), "pipe drain");
        return STAGE_OK;
    });
}

int stage_reader_create(stage_table *t, uint32_t max_batch, uint32_t max_wait_us, stage_reader **out) {
    if (!t || !out || max_batch == 0 || max_batch > (1u << 20)) return fail(STAGE_E_ARG, "bad reader arguments");
    if (facts(t).key_words() != 1) return fail(STAGE_E_ARG, "the single-key reader takes keys of <= 8 bytes");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<stage_reader> r(new stage_reader);
        r->t = t;
        r->max_batch = max_batch;
        r->max_wait_us = max_wait_us;
        r->stride = facts(t).stride();
        r->row_bytes = 8 + facts(t).params().payload_size;
        const uint64_t mb = max_batch;
        auto al = [](uint64_t x) { return (x + 15) & ~15ull; };
        auto &L = r->lay;
        L.lens = al(8 * mb);
        L.rids = L.lens + al(2 * mb);
        L.fu = L.rids + al(4 * mb);
        L.out = L.fu + al(mb);
        L.rows = L.out + al(32 * mb);
        L.ident = L.rows + al(r->stride * mb);
        L.bytes = L.ident + al(8 * mb);
        const uint64_t bytes = L.bytes;
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

static int resident_read(ResidentReader &R, uint64_t key, uint16_t key_size, uint32_t read_id, bool for_update,
                         stage_probe_out *out, uint8_t *record, stage_probe_ident *ident) {
    if (R.closing.load(std::memory_order_acquire) || R.dead.load(std::memory_order_acquire))
        return fail(STAGE_E_STATE, "resident reader has ended");
    const uint64_t q = R.tail.fetch_add(1, std::memory_order_acq_rel);
    const uint32_t per = R.slots / R.waves;  // wave q % W, its (q / W)-th ticket
    const uint32_t slot = (uint32_t)(q % R.waves) * per + (uint32_t)((q / R.waves) % per);
    const uint64_t prev = q >= R.slots ? q - R.slots + 1 : 0;
    // spin about the length of a read (a few microseconds), then yield: more callers than
    // CPUs must not hold the CPUs the finished ones need
    auto wait = [&](auto ready) {
        for (uint64_t i = 0; !ready(); ++i) {
            if (R.dead.load(std::memory_order_acquire)) return false;
            if (i < 256) _mm_pause();
            else std::this_thread::yield();
        }
        return true;
    };
    if (!wait([&] { return R.freed[slot].load(std::memory_order_acquire) == prev; }))
        return fail(R.dead.load(), "resident reader has ended");
    stage::ReaderReq &rq = R.req[slot];
    rq.key = key;
    rq.rid = read_id;
    // tag: ticket + 1 above 4 bits of key length - 1 (1..8 bytes) and is_for_update
    const uint32_t low = ((uint32_t)(key_size - 1) & 7u) | (for_update ? 8u : 0u);
    __atomic_store_n(&rq.tag, (uint32_t)(((q + 1) << 4) | low), __ATOMIC_RELEASE);
    if (!wait([&] { return __atomic_load_n(R.done + slot, __ATOMIC_ACQUIRE) == (uint32_t)(q + 1); }))
        return fail(R.dead.load(), R.dead.load() == STAGE_E_STATE ? "device image is stale: the resident reader ended"
                                                                  : "resident reader failed on the device");
    if (out) *out = R.out[slot];
    if (record) std::memcpy(record, R.rows + (uint64_t)slot * R.stride, R.row_bytes);
    if (ident) *ident = R.ident[slot];
    R.freed[slot].store(q + 1, std::memory_order_release);
    R.n_reads.fetch_add(1, std::memory_order_relaxed);
    return STAGE_OK;
}

int stage_reader_create_resident(stage_table *t, uint32_t ring_slots, uint32_t waves, uint32_t life_us,
                                 stage_reader **out) {
    if (!t || !out || waves == 0 || waves > 1024 || ring_slots == 0 || ring_slots % (64 * waves) ||
        ring_slots > (1u << 22) || life_us == 0 || life_us > 1000000)
        return fail(STAGE_E_ARG, "bad resident reader arguments (ring_slots: a multiple of 64 * waves; waves "
                                 "1..1024; life_us 1..1e6)");
    if (facts(t).key_words() != 1) return fail(STAGE_E_ARG, "the single-key reader takes keys of <= 8 bytes");
    if (int rc = need_synced(t)) return rc;
    const uint32_t cap = t->dev.view.cap;
    if (t->dev.view.key_width == 0 ? cap > 128 : cap > 1024)
        return fail(STAGE_E_ARG, "resident reader: leaf geometry not supported");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<stage_reader> r(new stage_reader);
        r->t = t;
        r->res.reset(new ResidentReader);
        ResidentReader &R = *r->res;
        R.t = t;
        R.slots = ring_slots;
        R.waves = waves;
        R.stride = facts(t).stride();
        R.row_bytes = 8 + facts(t).params().payload_size;
        stage::hip_check(hipSetDevice(t->dev.device), "hipSetDevice");
        int khz = 0;
        stage::hip_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, t->dev.device), "clock rate");
        R.life_ticks = (uint64_t)(khz > 0 ? khz : 100000) * life_us / 1000;
        const uint64_t S = ring_slots;
        // requests | done | stop | out | ident | rows (each array 64-B aligned)
        auto al = [](uint64_t x) { return (x + 63) & ~63ull; };
        const uint64_t o_done = al(sizeof(stage::ReaderReq) * S), o_stop = o_done + al(4 * S), o_out = o_stop + 64,
                       o_ident = o_out + al(32 * S), o_rows = o_ident + al(8 * S), bytes = o_rows + S * R.stride;
        stage::hip_check(hipHostMalloc((void **)&R.h, bytes, hipHostMallocMapped | hipHostMallocCoherent |
                                                                 hipHostMallocPortable),
                         "resident ring");
        std::memset(R.h, 0, bytes);
        stage::hip_check(hipHostGetDevicePointer((void **)&R.hd, R.h, 0), "resident ring device pointer");
        R.req = (stage::ReaderReq *)R.h;
        R.done = (uint32_t *)(R.h + o_done);
        R.stop = (uint32_t *)(R.h + o_stop);
        R.out = (stage_probe_out *)(R.h + o_out);
        R.rows = R.h + o_rows;
        R.ident = (stage_probe_ident *)(R.h + o_ident);
        R.freed.reset(new std::atomic<uint64_t>[S]);
        for (uint64_t i = 0; i < S; ++i) R.freed[i].store(0);
        std::vector<uint64_t> pos(waves, 0);
        stage::hip_check(hipMalloc((void **)&R.dpos, 8ull * waves), "resident positions");
        stage::hip_check(hipMemcpy(R.dpos, pos.data(), 8ull * waves, hipMemcpyHostToDevice), "resident positions");
        stage::hip_check(hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking), "resident stream");
        for (auto &e : R.ev) stage::hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync),
                                              "resident event");
        R.ring = stage::ReaderRing{(const stage::ReaderReq *)R.hd, (uint32_t *)(R.hd + o_done), (stage::stage_probe_out_dev *)(R.hd + o_out),
                                   R.hd + o_rows, (const uint32_t *)(R.hd + o_stop), R.dpos, ring_slots, waves,
                                   R.life_ticks, (uint32_t *)(R.hd + o_ident)};
        ResidentReader *raw = &R;
        R.keeper = std::thread([raw] { raw->run(); });
        *out = r.release();
        return STAGE_OK;
    });
}

static void resident_destroy(ResidentReader &R) {
    R.closing.store(true, std::memory_order_release);
    // the reads already holding a ticket finish (bounded: the keeper keeps instances queued
    // until they are done or the device side has ended)
    const uint64_t issued = R.tail.load(std::memory_order_acquire);
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t per = R.slots / R.waves;
    for (uint64_t q = issued > R.slots ? issued - R.slots : 0; q < issued; ++q)
        while (R.freed[(q % R.waves) * per + (q / R.waves) % per].load(std::memory_order_acquire) < q + 1 &&
               !R.dead.load() &&
               std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
            std::this_thread::yield();
    R.quit.store(true, std::memory_order_release);
    if (R.keeper.joinable()) R.keeper.join();
    (void)hipSetDevice(R.t->dev.device);
    if (R.s) (void)hipStreamSynchronize(R.s), (void)hipStreamDestroy(R.s);
    for (auto &e : R.ev)
        if (e) (void)hipEventDestroy(e);
    if (R.dpos) (void)hipFree(R.dpos);
    if (R.h) (void)hipHostFree(R.h);
}

int stage_reader_read(stage_reader *r, uint64_t key, uint16_t key_size, uint32_t read_id, stage_probe_out *out,
                      uint8_t *record) {
    return stage_reader_read_ex(r, key, key_size, read_id, 0, out, record, nullptr);
}

int stage_reader_read_ident(stage_reader *r, uint64_t key, uint16_t key_size, uint32_t read_id, stage_probe_out *out,
                            uint8_t *record, stage_probe_ident *ident) {
    return stage_reader_read_ex(r, key, key_size, read_id, 0, out, record, ident);
}

int stage_reader_read_ex(stage_reader *r, uint64_t key, uint16_t key_size, uint32_t read_id, int is_for_update,
                         stage_probe_out *out, uint8_t *record, stage_probe_ident *ident) {
    if (!r) return fail(STAGE_E_ARG, "null reader");
    if (key_size == 0 || key_size > 8) return fail(STAGE_E_ARG, "key_size must be 1..8");
    const bool fu = is_for_update != 0;
    if (r->res) return resident_read(*r->res, key, key_size, read_id, fu, out, record, ident);
    int rc = STAGE_E_STATE;
    uint32_t seq;
    {
        std::unique_lock<std::mutex> lk(r->mu);
        r->cv_space.wait(lk, [&] { return r->stop || r->open.size() < r->max_batch; });
        if (r->stop) return fail(STAGE_E_STATE, "reader is closing");
        r->open.push_back({key, key_size, read_id, fu, out, record, ident, &rc});
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
    if (r->res) {
        stats[0] = r->res->n_inst.load();
        stats[1] = r->res->n_reads.load();
        stats[2] = 0;
        return STAGE_OK;
    }
    stats[0] = r->n_batches.load();
    stats[1] = r->n_reads.load();
    stats[2] = r->n_full.load();
    return STAGE_OK;
}

int stage_reader_destroy(stage_reader *r) {
    if (!r) return STAGE_OK;
    if (r->res) {
        resident_destroy(*r->res);
        delete r;
        return STAGE_OK;
    }
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
