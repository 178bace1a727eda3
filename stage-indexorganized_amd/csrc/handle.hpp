// handle.hpp -- the table handle behind the C-ABI and the error helpers shared by the
// translation units that implement include/stage_hip.h (capi.cpp, host_io.cpp).
#pragma once
#include <hip/hip_runtime_api.h>

#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <atomic>
#include <chrono>
#include <thread>

#include "../../include/stage_hip.h"
#include "device_image.hpp"
#include "dist.hpp"
#include "host_table.hpp"
#include "kernel_api.hpp"

namespace stage {
struct HostPipe;  // host_io.cpp: pinned staging + streams of stage_probe_host
void host_pipe_release(HostPipe *p);
struct HostPipeDeleter {
    void operator()(HostPipe *p) const { host_pipe_release(p); }
};
}  // namespace stage

// CH-Q2's captured batch (chq2.hip): replayed while its key -- every argument of the captured
// launches -- stays the same
struct Q2Graph {
    hipGraphExec_t exec = nullptr;
    std::string key, last_key;
    bool failed = false;
};
// a CH-Q2 batch enqueued by stage_ch_query2_batch_async and not yet waited for (per slot)
struct Q2Pending {
    bool active = false;
    hipEvent_t ev = nullptr;  // after the batch's last copy (its records' copy, when split)
    hipStream_t stream = nullptr;  // the stream it was enqueued on
    uint8_t *pq = nullptr;    // its page-locked staging: counts at q_cn, aborted flags at q_ab
    uint64_t q_cn = 0, q_ab = 0, n_max = 0, m_max = 0;
    uint32_t nq = 0;
    // split emit (async batches into page-locked `out`): the records are finished into this
    // slot's own device buffer and leave over PCIe by a copy on the table's q2_side stream, so
    // the next batch's kernels run while they cross; `fin` marks the end of the batch's kernels
    // (the shared scratch is free again), `ev` the end of the copy
    bool split = false;
    hipEvent_t fin = nullptr;
    uint8_t *dbuf = nullptr;  // the records, row pitch n_max
    uint64_t dcap = 0;
    uint64_t cols = 0, max_out = 0;  // columns (records per query) the 2-D copy to `out` takes
    stage_q2_rec *out = nullptr, *slot_out = nullptr;
};

struct stage_table {
    std::unique_ptr<stage::HostTable> host;
    stage::DeviceImage dev;
    stage::ProbeTuning tune;
    stage::ScanTuning scan_tune;
    uint32_t out_stride = 0;  // 0 = stride of the canonical row (stage_set_output_layout / STAGE_OUT_STRIDE)
    int status_bytes = 32;    // stage_probe_batch's status records: 32 or 16 (stage_set_output_layout)
    std::unique_ptr<stage::ShardComm> comm;
    std::unique_ptr<stage::ShardComm> loop_comm;  // stage_probe_sharded_loopback state
    int shard_chunks = 0;                          // 0 = STAGE_SHARD_CHUNKS or the default
    int shard_dedupe = -1;                         // -1 = STAGE_SHARD_DEDUPE or on
    int shard_key_bits = 64;                       // coalescing sort width (stage_set_shard_key_bits)
    int wp_overlap = 0;                            // stage_set_write_overlap (0 or 1)
    uint64_t q2_hint[2] = {0, 0};                  // CH-Q2's last visited suppliers / STOCK keys (launch shapes)
    Q2Graph q2g[2];     // per CH-Q2 slot (stage_ch_query2_batch_async); slot 0 also serves the synchronous calls
    Q2Pending q2p[2];
    hipStream_t q2_side = nullptr;  // the split batches' record copies (created on first use)
    std::mutex pipe_mu;  // serialises stage_probe_host calls on this table
    std::unique_ptr<stage::HostPipe, stage::HostPipeDeleter> pipe;
    // the device write path hands its epoch's bookkeeping (new copy / version headers, slot
    // words) to the host table on a thread of its own while the device goes on (write_path.hip);
    // every entry point that reads or writes the host table settles it first (host()).
    // Adoptions are pipelined: epoch e + 1's kernels are enqueued while epoch e is still being
    // adopted (the device keeps its own append counters); epoch e + 1's adoption thread joins
    // epoch e's before it touches the host table, so epochs are adopted in order.  adopt_mu
    // guards `adopt` (the newest thread): settle() may run on any caller thread while the writer
    // starts the next adoption.  A failed adoption is sticky: the host table missed an epoch of
    // the device, so every later host-table call (the writer's included) reports it.
    std::mutex adopt_mu;
    std::thread adopt;
    std::exception_ptr adopt_err;        // written by an adoption thread, read after its join
    uint64_t wp_started = 0;             // device epochs enqueued (the writer's count)
    std::atomic<uint64_t> wp_adopted{0}; // device epochs adopted (or failed) -- in order
    std::atomic<bool> adopt_failed{false};
    std::atomic<uint64_t> adopted_sz[3] = {{0}, {0}, {0}};  // host copies / versions / images after the last adoption
    uint64_t wp_epoch_n[stage::kWpDepth] = {};                       // ops of the writer's last epochs (by epoch % kWpDepth)
    void settle() {
        std::lock_guard<std::mutex> g(adopt_mu);
        if (adopt.joinable()) adopt.join();
        if (adopt_err) std::rethrow_exception(adopt_err);
    }
    // starts the adoption of epoch `epoch`: a thread that first joins the previous adoption
    template <class F>
    void start_adoption(uint64_t epoch, F &&fn) {
        std::lock_guard<std::mutex> g(adopt_mu);
        std::thread prev = std::move(adopt);
        adopt = std::thread([this, epoch, prev = std::move(prev), fn = std::forward<F>(fn)]() mutable {
            if (prev.joinable()) prev.join();
            if (!adopt_err) {
                try {
                    fn();
                } catch (...) {
                    adopt_err = std::current_exception();
                    adopt_failed.store(true, std::memory_order_release);
                }
            }
            wp_adopted.store(epoch, std::memory_order_release);
        });
    }
    // the writer waits until epoch `epoch` is adopted (its kWpDepth-buffered outputs are free)
    void wait_adopted(uint64_t epoch) {
        while (wp_adopted.load(std::memory_order_acquire) < epoch) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    ~stage_table() {
        std::lock_guard<std::mutex> g(adopt_mu);
        if (adopt.joinable()) adopt.join();
        for (int k = 0; k < 2; ++k) {
            if (q2p[k].active && q2p[k].ev) (void)hipEventSynchronize(q2p[k].ev);
            if (q2p[k].ev) (void)hipEventDestroy(q2p[k].ev);
            if (q2p[k].fin) (void)hipEventDestroy(q2p[k].fin);
            if (q2g[k].exec) (void)hipGraphExecDestroy(q2g[k].exec);
        }
        if (q2_side) (void)hipStreamSynchronize(q2_side);
        for (int k = 0; k < 2; ++k)
            if (q2p[k].dbuf) (void)hipFree(q2p[k].dbuf);
        if (q2_side) (void)hipStreamDestroy(q2_side);
    }
};

namespace stage_capi {
extern thread_local std::string g_err;

inline int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

template <class F>
int guarded(F fn) {
    try {
        return fn();
    } catch (const std::bad_alloc &) {
        return fail(STAGE_E_NOMEM, "host allocation failed");
    } catch (const std::invalid_argument &e) {
        return fail(STAGE_E_ARG, e.what());
    } catch (const std::exception &e) {
        return fail(STAGE_E_HIP, e.what());
    }
}

// the host table, after any pending device-epoch adoption (stage_table::settle)
inline stage::HostTable &host(stage_table *t) {
    t->settle();
    return *t->host;
}

// geometry facts fixed at stage_open (key width / words, payload size, stride, leaf capacity):
// read without settling a pending adoption, so read-only paths never wait for the writer
inline const stage::HostTable &facts(stage_table *t) { return *t->host; }

// device entry points check the host's dirty flag without settling: a pending adoption never
// touches layout_dirty_, and the device image is already current
inline int need_synced(stage_table *t) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    if (!t->dev.valid || t->host->layout_dirty_)
        return fail(STAGE_E_STATE, "device image is stale: call stage_sync after host writes");
    return STAGE_OK;
}

// device-written heap rows (stage_update_batch_device) are pulled into the host arena before a
// host-side path reads payloads (write_path.hip)
void ensure_host_rows(stage_table *t);

inline hipStream_t pick(stage_table *t, void *stream) { return stream ? (hipStream_t)stream : t->dev.stream; }

inline int hip_rc(hipError_t e, const char *what) {
    if (e == hipSuccess) return STAGE_OK;
    return fail(STAGE_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace stage_capi
