// handle.hpp -- the table handle behind the C-ABI and the error helpers shared by the
// translation units that implement include/stage_hip.h (capi.cpp, host_io.cpp).
#pragma once
#include <hip/hip_runtime_api.h>

#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
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
    std::mutex pipe_mu;  // serialises stage_probe_host calls on this table
    std::unique_ptr<stage::HostPipe, stage::HostPipeDeleter> pipe;
    // the device write path hands its epoch's bookkeeping (new copy / version headers, slot
    // words) to the host table on this thread while the device goes on (write_path.hip);
    // every entry point that reads or writes the host table settles it first (host()).
    // adopt_mu guards `adopt`: settle() may run on any caller thread while the writer (the
    // thread calling stage_update_batch_device) starts the next adoption.  A failed adoption
    // is sticky: the host table missed an epoch of the device, so every later host-table call
    // (the writer's included) reports it.
    std::mutex adopt_mu;
    std::thread adopt;
    std::exception_ptr adopt_err;  // written by the adoption thread before it ends, read after join
    void settle() {
        std::lock_guard<std::mutex> g(adopt_mu);
        if (adopt.joinable()) adopt.join();
        if (adopt_err) std::rethrow_exception(adopt_err);
    }
    // starts the adoption of an epoch (after settle(): no adoption is running)
    template <class F>
    void start_adoption(F &&fn) {
        std::lock_guard<std::mutex> g(adopt_mu);
        if (adopt.joinable()) adopt.join();
        adopt = std::thread(std::forward<F>(fn));
    }
    ~stage_table() {
        std::lock_guard<std::mutex> g(adopt_mu);
        if (adopt.joinable()) adopt.join();
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
