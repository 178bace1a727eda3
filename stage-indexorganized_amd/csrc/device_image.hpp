// device_image.hpp -- the HBM image of one table and its publication from the host layout.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <vector>

#include "host_table.hpp"
#include "kernel_api.hpp"
#include "stage_core.hpp"

namespace stage {

struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
};

struct DeviceImage {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf head, okey, slot, tree, tree_len, heap, chdr, vhdr, arena, descs, patch;
    std::vector<uint8_t> staging;  // host staging of incremental patches
    uint64_t heap_rows = 0;  // rows the heap buffer can hold
    DevTable view{};
    std::vector<uint32_t> host_to_dev;  // host leaf id -> leaf index in key order
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

}  // namespace stage
