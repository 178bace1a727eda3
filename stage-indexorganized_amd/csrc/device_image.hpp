// device_image.hpp -- the HBM image of one table and its publication from the host layout.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "host_table.hpp"
#include "kernel_api.hpp"
#include "stage_core.hpp"

namespace stage {

struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
};

// device write-path epochs in flight: epoch e's outputs are reused by epoch e + kWpDepth, whose
// call waits for e's host adoption.  Three: an epoch is adopted ~2.7 epochs after its call starts
// (its kernels run beside the previous epoch's probe, its export beside its own, then ~3.7 ms
// of host work), so with two the next-but-one call waited for it and its kernels reached the
// device too late to hide under the probe (§5r6)
constexpr int kWpDepth = 3;
constexpr int kQ2Pinned = kWpDepth;  // first pinned staging slot of CH-Q2

struct DeviceImage {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf head, okey, slot, tree, tree_len, heap, chdr, vhdr, arena, descs, patch;
    DevBuf scratch;     // per-call scratch of stock-level / CH-Q2 / scans (scratch_bytes)
    DevBuf wp_scratch;  // the device write path's own scratch (wp_scratch_bytes): an overlapped
                        // epoch runs beside the caller's later work on the shared scratch
    // the device write path's per-epoch outputs, kWpDepth-buffered by epoch: epoch e's background
    // adoption reads wp_out[e % kWpDepth] / pinned[e % kWpDepth] while epochs e + 1, e + 2 run
    DevBuf wp_out[kWpDepth];  // slot words + totals
    DevBuf wp_bases;   // the next epoch's copy / version / image indices (device-side append counters)
    uint64_t wp_ub[3] = {0, 0, 0};       // upper bounds of those counters (copies, versions, images)
    hipStream_t adopt_stream = nullptr;  // the adoption's D2H copies (beside the caller's stream)
    hipEvent_t adopt_ev[kWpDepth] = {};   // end of an epoch's write-path kernels
    hipEvent_t export_ev[kWpDepth] = {};  // end of its export into pinned host memory
    // write-overlap mode (stage_set_write_overlap): an epoch's kernels up to the publish run on
    // wp_stream after the previous epoch's publish (wp_pub_ev), beside the caller's later work;
    // the publish joins the caller's stream (wp_pre_ev).  wp_pub_valid: wp_pub_ev marks the
    // last change of the device image (cleared by sync_device and every other republish)
    hipStream_t wp_stream = nullptr;
    hipEvent_t wp_pub_ev = nullptr, wp_pre_ev = nullptr;
    bool wp_pub_valid = false;
    std::vector<uint8_t> staging;  // host staging of incremental patches
    // pinned host staging: [0, kWpDepth) the write path's epoch results (by epoch % kWpDepth);
    // [kQ2Pinned, kQ2Pinned + 2) CH-Q2's two batch slots (scan rows, supplier list, records)
    void *pinned[kQ2Pinned + 2] = {};
    uint64_t pinned_cap[kQ2Pinned + 2] = {};
    uint64_t heap_rows = 0;  // rows the heap buffer can hold
    DevTable view{};
    std::vector<uint32_t> host_to_dev;  // host leaf id -> leaf index in key order
    std::vector<uint32_t> dev_to_host;  // leaf index in key order -> host leaf id
    bool valid = false;
    double last_sync_seconds = 0;
    bool last_sync_incremental = false;
    uint64_t last_patch_leaves = 0, last_patch_slots = 0;

    ~DeviceImage();
    void release();
};

// Publish `h` into `d` (allocates/grows device buffers, uploads the layout, fills new
// record-heap rows).  Throws std::runtime_error on HIP failure.
void sync_device(HostTable &h, DeviceImage &d);

void hip_check(hipError_t e, const char *what);

// scratch of at least `bytes` (grown with hipMalloc after draining the device; reused by the
// next call on the same table).  Stream-ordered pool memory (hipMallocAsync) is not used: on
// gfx950 its reuse across calls showed stale reads on other XCDs between kernels of a stream.
uint8_t *scratch_bytes(DeviceImage &d, uint64_t bytes);
// A multi-table operation's users of the tables' per-call scratch: each table's scratch is one
// buffer handed out from offset 0 (scratch_bytes), so within one operation it may have one user.
// Round 5's fault (781d36d) broke exactly that: CH-Q2's batch buffers were carved from NATION's
// scratch while it held the NATION scan rows.  An operation lists its users by the table role
// they live in (kQ2Scratch, kStockLevelScratch); check_scratch_uses refuses two users on one
// table -- the roles' tables when given (a caller passing one table for two roles), else the
// roles themselves (the plan as written).
struct ScratchUse {
    int role;
    const char *what;
};
inline void check_scratch_uses(const ScratchUse *u, int n, const void *const *tables = nullptr) {
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {
            const bool same = tables ? tables[u[i].role] == tables[u[j].role] : u[i].role == u[j].role;
            if (same)
                throw std::invalid_argument(std::string("scratch alias: ") + u[i].what + " and " + u[j].what +
                                            " would share one table's per-call scratch");
        }
}

// the same for the device write path alone (write_path.hip)
uint8_t *wp_scratch_bytes(DeviceImage &d, uint64_t bytes);
// pinned host buffer `k` (0/1) of at least `bytes` (grown with hipHostMalloc; reused by later calls)
uint8_t *pinned_bytes(DeviceImage &d, uint64_t bytes, int k = 0);
// the write path's own output buffer `k` (0/1; not shared with scratch_bytes users: its
// background adoption reads it after the call returned)
uint8_t *wp_out_bytes(DeviceImage &d, uint64_t bytes, int k = 0);

// grow the record heap and the copy / version header arrays so that `extra_*` more entries fit
// after the host's current counts (device write path); refreshes the DevTable view
void reserve_device_rows(HostTable &h, DeviceImage &d, uint64_t extra_images, uint64_t extra_copies,
                         uint64_t extra_versions, hipStream_t s);

}  // namespace stage
