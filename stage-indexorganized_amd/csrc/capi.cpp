// capi.cpp -- the extern "C" boundary (include/stage_hip.h).  No exception crosses it.
#include <hip/hip_runtime_api.h>

#include <execinfo.h>
#include <unistd.h>

#include <csignal>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "handle.hpp"

namespace stage_capi {
thread_local std::string g_err;
}
using namespace stage_capi;

extern "C" {

const char *stage_last_error(void) { return g_err.c_str(); }

// STAGE_SEGV_TRACE=1: a host-side SIGSEGV / SIGABRT prints the native backtrace of the faulting
// thread to stderr before the default action (host-code debugging on the GPU box, where no
// debugger is available)
namespace {
void segv_trace(int sig) {
    void *frames[64];
    const int n = backtrace(frames, 64);
    const char msg[] = "stage: fatal signal, native backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(frames, n, 2);
    std::signal(sig, SIG_DFL);
    raise(sig);
}
struct SegvTraceInit {
    SegvTraceInit() {
        if (std::getenv("STAGE_SEGV_TRACE")) {
            std::signal(SIGSEGV, segv_trace);
            std::signal(SIGABRT, segv_trace);
        }
    }
} segv_trace_init;
}  // namespace
const char *stage_version(void) { return "stage-hip 0.1 (gfx950)"; }

int stage_table_create(const stage_params *params, stage_table **out) {
    if (!params || !out) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        auto t = std::make_unique<stage_table>();
        t->host = std::make_unique<stage::HostTable>(*params);
        t->dev.device = params->device;
        if (const char *g = std::getenv("STAGE_OUT_STRIDE")) {
            uint32_t v = (uint32_t)std::atoi(g);
            if (v >= ((t->host->key_pad() + t->host->params().payload_size + 15) & ~15u) && v % 16 == 0)
                t->out_stride = v;
        }
        *out = t.release();
        return STAGE_OK;
    });
}

int stage_table_destroy(stage_table *t) {
    if (!t) return STAGE_OK;
    return guarded([&] {
        if (t->dev.stream) (void)hipSetDevice(t->dev.device);
        delete t;
        return STAGE_OK;
    });
}

int stage_insert(stage_table *t, uint64_t key, uint16_t key_size, const uint8_t *payload, uint64_t gen_rowid,
                 int payload_mode, uint32_t commit_id, uint8_t *rc_out) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        int rc = host(t).insert(key, key_size, payload, gen_rowid, payload_mode, commit_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_load_ycsb(stage_table *t, uint64_t begin_rowid, uint64_t end_rowid, uint32_t key_size, int payload_mode,
                    uint64_t *inserted) {
    if (!t || key_size == 0 || key_size > 8) return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        uint64_t n = host(t).load_ycsb(begin_rowid, end_rowid, key_size, payload_mode);
        if (inserted) *inserted = n;
        return STAGE_OK;
    });
}

int stage_load_keys(stage_table *t, const uint64_t *keys, uint64_t n, uint32_t key_size, int payload_mode,
                    uint64_t *inserted) {
    if (!t || (!keys && n) || key_size == 0 || key_size > 8) return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        uint64_t c = host(t).load_keys(keys, n, key_size, payload_mode);
        if (inserted) *inserted = c;
        return STAGE_OK;
    });
}

int stage_update(stage_table *t, uint64_t key, uint16_t key_size, uint32_t payload_off, const uint8_t *delta,
                 uint32_t delta_len, uint32_t writer_id, uint8_t *rc_out) {
    if (!t || (!delta && delta_len)) return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        ensure_host_rows(t);
        int rc = host(t).update(key, key_size, payload_off, delta, delta_len, writer_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_commit_update(stage_table *t, uint64_t key, uint16_t key_size, uint32_t commit_id, uint32_t sstamp,
                        uint8_t *rc_out) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        int rc = host(t).commit_update(key, key_size, commit_id, sstamp);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_update_batch(stage_table *t, const void *keys, uint32_t key_stride, uint64_t n, uint16_t key_size,
                       uint32_t payload_off, const uint8_t *deltas, uint32_t delta_len, const uint32_t *writer_ids,
                       const uint32_t *commit_ids, const uint32_t *sstamps, uint8_t *rc_out, uint64_t *n_ok) {
    if (!t || (n && (!keys || !writer_ids || (!deltas && delta_len))) || key_stride < key_size)
        return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        ensure_host_rows(t);
        uint64_t ok = host(t).update_batch((const uint8_t *)keys, key_stride, n, key_size, payload_off, deltas,
                                            delta_len, writer_ids, commit_ids, sstamps, rc_out);
        if (n_ok) *n_ok = ok;
        return STAGE_OK;
    });
}

int stage_finalize_update(stage_table *t, uint64_t key, uint16_t key_size, uint32_t commit_id, uint8_t *rc_out) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        int rc = host(t).finalize_update(key, key_size, commit_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_delete(stage_table *t, uint64_t key, uint16_t key_size, uint32_t commit_id, uint8_t *rc_out) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        int rc = host(t).remove(key, key_size, commit_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

// ---- byte-key forms (any key width of the table, up to 32 bytes)
int stage_insert_key(stage_table *t, const uint8_t *key, uint16_t key_size, const uint8_t *payload, uint32_t commit_id,
                     uint8_t *rc_out) {
    if (!t || !key || !payload) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).insert(key, key_size, payload, 0, 0, commit_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_insert_key_inflight(stage_table *t, const uint8_t *key, uint16_t key_size, const uint8_t *payload,
                              uint32_t writer_id, uint8_t *rc_out) {
    if (!t || !key || !payload) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).insert(key, key_size, payload, 0, 0, writer_id, true);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_commit_insert_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t commit_id,
                            uint8_t *rc_out) {
    if (!t || !key) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).commit_insert(key, key_size, commit_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_load_rows(stage_table *t, const uint8_t *keys, uint32_t key_stride, uint16_t key_size,
                    const uint8_t *payloads, uint32_t payload_stride, uint64_t n, uint32_t commit_id,
                    uint8_t *rc_out, uint64_t *inserted) {
    if (!t || (n && (!keys || !payloads)) || key_stride < key_size) return fail(STAGE_E_ARG, "bad arguments");
    if (payload_stride < host(t).params().payload_size) return fail(STAGE_E_ARG, "payload stride < payload size");
    return guarded([&] {
        uint64_t c = host(t).load_rows(keys, key_stride, key_size, payloads, payload_stride, n, commit_id, rc_out);
        if (inserted) *inserted = c;
        return STAGE_OK;
    });
}

int stage_update_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t payload_off,
                     const uint8_t *delta, uint32_t delta_len, uint32_t writer_id, uint8_t *rc_out) {
    if (!t || !key || (!delta && delta_len)) return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        ensure_host_rows(t);
        int rc = host(t).update(key, key_size, payload_off, delta, delta_len, writer_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_commit_update_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t commit_id,
                            uint32_t sstamp, uint8_t *rc_out) {
    if (!t || !key) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).commit_update(key, key_size, commit_id, sstamp);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_update_key_owned(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t payload_off,
                           const uint8_t *delta, uint32_t delta_len, uint32_t writer_id, uint8_t *rc_out) {
    if (!t || !key || (!delta && delta_len)) return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        ensure_host_rows(t);
        int rc = host(t).update_owned(key, key_size, payload_off, delta, delta_len, writer_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_delete_key_owned(stage_table *t, const uint8_t *key, uint16_t key_size, uint8_t *rc_out) {
    if (!t || !key) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).remove_owned(key, key_size);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_delete_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint32_t commit_id, uint8_t *rc_out) {
    if (!t || !key) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).remove(key, key_size, commit_id);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_abort_update_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint8_t *rc_out) {
    if (!t || !key) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).abort_update(key, key_size);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_abort_insert_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint8_t *rc_out) {
    if (!t || !key) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        int rc = host(t).abort_insert(key, key_size);
        if (rc_out) *rc_out = (uint8_t)rc;
        return STAGE_OK;
    });
}

int stage_settle(stage_table *t) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        t->settle();
        return STAGE_OK;
    });
}

uint32_t stage_key_words(stage_table *t) { return t ? facts(t).key_words() : 0; }

int stage_sync(stage_table *t) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        stage::sync_device(host(t), t->dev);
        return STAGE_OK;
    });
}

int stage_sync_info(stage_table *t, double *seconds, uint64_t *info) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    if (seconds) *seconds = t->dev.last_sync_seconds;
    if (info) {
        info[0] = t->dev.last_sync_incremental ? 1 : 0;
        info[1] = t->dev.last_patch_leaves;
        info[2] = t->dev.last_patch_slots;
    }
    return STAGE_OK;
}

int stage_stats(stage_table *t, uint64_t *stats) {
    if (!t || !stats) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        host(t).stats(stats);
        return STAGE_OK;
    });
}

uint32_t stage_record_stride(stage_table *t) { return t ? (t->out_stride ? t->out_stride : facts(t).stride()) : 0; }
uint32_t stage_leaf_capacity(stage_table *t) { return t ? facts(t).cap() : 0; }

int stage_traverse_batch(stage_table *t, const uint64_t *keys, const uint16_t *lens, uint64_t n, int le_child,
                         uint32_t *leaf_out) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    if ((!keys || !leaf_out) && n) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        // leaf index in key order: from the published image, or recomputed if host writes
        // happened since (the traversal itself never needs the device)
        std::vector<uint32_t> local;
        const std::vector<uint32_t> *map = &t->dev.host_to_dev;
        if (!t->dev.valid || host(t).layout_dirty_) {
            std::vector<uint32_t> order;
            host(t).key_order(order);
            local.assign(host(t).leaves_.size(), 0xFFFFFFFFu);
            for (size_t i = 0; i < order.size(); ++i) local[order[i]] = (uint32_t)i;
            map = &local;
        }
        const uint32_t width = host(t).params().key_width, kwords = host(t).key_words();
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t len = width ? width : (lens ? lens[i] : 8u);
            const stage::Key k = host(t).key_of(reinterpret_cast<const uint8_t *>(keys + i * kwords), len);
            leaf_out[i] = (*map)[host(t).route(k, le_child != 0)];
        }
        return STAGE_OK;
    });
}

int64_t stage_export_leaves(stage_table *t, uint32_t cap, uint64_t max_leaves, uint32_t *rc, uint32_t *sc,
                            uint64_t *meta, uint64_t *keyw) {
    if (!t || !rc || !sc || !meta || !keyw || cap == 0) return fail(STAGE_E_ARG, "null argument");
    try {
        const int64_t n = host(t).export_leaves(cap, max_leaves, rc, sc, meta, keyw);
        if (n < 0) return fail(STAGE_E_ARG, "max_leaves is smaller than the leaf count (stage_stats[2])");
        return n;
    } catch (const std::bad_alloc &) {
        return fail(STAGE_E_NOMEM, "host allocation failed");
    } catch (const std::exception &e) {
        return fail(STAGE_E_HIP, e.what());
    }
}

int64_t stage_export_leaf_images(stage_table *t, uint64_t max_leaves, uint8_t *blocks, uint64_t *sep_keys,
                                 uint16_t *sep_lens) {
    if (!t || !blocks || (!sep_keys != !sep_lens)) return fail(STAGE_E_ARG, "bad arguments");
    try {
        ensure_host_rows(t);
        const int64_t n = host(t).export_leaf_images(max_leaves, blocks, sep_keys, sep_lens);
        if (n < 0) return fail(STAGE_E_ARG, "max_leaves is smaller than the leaf count (stage_stats[2])");
        return n;
    } catch (const std::bad_alloc &) {
        return fail(STAGE_E_NOMEM, "host allocation failed");
    } catch (const std::exception &e) {
        return fail(STAGE_E_HIP, e.what());
    }
}

int64_t stage_export_locations(stage_table *t, uint64_t max, uint64_t *handles, uint32_t *leaf, uint16_t *slot) {
    if (!t || (max && (!handles || !leaf || !slot))) return fail(STAGE_E_ARG, "bad arguments");
    try {
        return (int64_t)host(t).export_locations(max, handles, leaf, slot);
    } catch (const std::bad_alloc &) {
        return fail(STAGE_E_NOMEM, "host allocation failed");
    } catch (const std::exception &e) {
        return fail(STAGE_E_HIP, e.what());
    }
}

int stage_resolve_locations(stage_table *t, const uint64_t *handles, uint64_t n, uint32_t *leaf, uint16_t *slot) {
    if (!t || (n && (!handles || !leaf || !slot))) return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        host(t).resolve_locations(handles, n, leaf, slot);
        return STAGE_OK;
    });
}

// ---- what the kept transaction manager reads through a Record (stage_hip.h) ----------------

}  // extern "C"

// the SSN state of copy `id` under its mutex; a copy the device wrote in an epoch the host has
// not adopted yet is waited for (stage_table::settle) once
template <class F>
static int with_copy(stage_table *t, uint32_t id, F fn) {
    stage::CopySsnTable &s = t->host->ssn_;
    {
        std::unique_lock<std::mutex> g(s.mu);
        if (id < s.e.size()) return fn(s, s.e[id]);
    }
    int rc = guarded([&] {
        t->settle();
        return STAGE_OK;
    });
    if (rc) return rc;
    std::unique_lock<std::mutex> g(s.mu);
    if (id >= s.e.size()) return fail(STAGE_E_ARG, "no such overwrite copy");
    return fn(s, s.e[id]);
}

extern "C" {

int stage_probe_identify(stage_table *t, const stage_probe_out *d_out, uint64_t n, stage_probe_ident *d_ident,
                      void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (n && (!d_out || !d_ident)) return fail(STAGE_E_ARG, "null device buffer");
    if (t->status_bytes != 32) return fail(STAGE_E_STATE, "stage_probe_identify reads 32-B status records (leaf, slot)");
    hipError_t e = hipSetDevice(t->dev.device);
    if (e != hipSuccess) return hip_rc(e, "hipSetDevice");
    e = stage::launch_ident(t->dev.view, reinterpret_cast<const stage::stage_probe_out_dev *>(d_out), n,
                            reinterpret_cast<uint32_t *>(d_ident), pick(t, stream));
    return hip_rc(e, "ident kernel");
}

int stage_record_meta_key(stage_table *t, const uint8_t *key, uint16_t key_size, uint64_t *meta,
                          stage_probe_ident *ident, uint8_t *rc_out) {
    if (!t || !key || !meta || !ident) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] {
        stage::HostTable &h = host(t);
        uint32_t leaf, slot;
        *meta = 0;
        *ident = stage_probe_ident{0, 0};
        if (h.find(key, key_size, &leaf, &slot) < 0) {
            if (rc_out) *rc_out = STAGE_RC_NOT_FOUND;
            return STAGE_OK;
        }
        const size_t i = (size_t)leaf * h.cap() + slot;
        *meta = h.meta_[i];
        *ident = stage_probe_ident{h.loc_[i], h.next_[i]};
        if (rc_out) *rc_out = STAGE_RC_OK;
        return STAGE_OK;
    });
}

int stage_location_cells(stage_table *t) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        host(t).enable_cells();
        return STAGE_OK;
    });
}

int stage_location_cell(stage_table *t, uint64_t handle, const void **cell) {
    if (!t || !cell) return fail(STAGE_E_ARG, "null argument");
    stage::HostTable &h = *t->host;  // no settle: a cell is read while the writer goes on
    if (!h.cells_.on()) return fail(STAGE_E_STATE, "location cells are off: call stage_location_cells first");
    if (handle == 0 || (handle >> stage::LocCells::kChunkBits) >= stage::LocCells::kDir)
        return fail(STAGE_E_ARG, "location handle out of range");
    return guarded([&] {
        h.cells_.ensure(handle);
        *cell = h.cells_.find(handle);
        return STAGE_OK;
    });
}

int stage_copy_get(stage_table *t, const uint32_t *copy_ids, uint64_t n, stage_copy_state *out) {
    if (!t || (n && (!copy_ids || !out))) return fail(STAGE_E_ARG, "bad arguments");
    for (uint64_t i = 0; i < n; ++i) {
        const int rc = with_copy(t, copy_ids[i], [&](stage::CopySsnTable &s, stage::CopySsn &c) {
            auto it = s.readers.find(copy_ids[i]);
            out[i] = stage_copy_state{c.cstamp, c.pstamp, c.rstamp, c.sstamp,
                                      it == s.readers.end() ? 0u : (uint32_t)it->second.size(), c.count, c.waiting, 0};
            return STAGE_OK;
        });
        if (rc) return rc;
    }
    return STAGE_OK;
}

int stage_copy_readers(stage_table *t, uint32_t copy_id, uint32_t *read_ids, uint32_t max, uint32_t *count) {
    if (!t || !count || (max && !read_ids)) return fail(STAGE_E_ARG, "bad arguments");
    return with_copy(t, copy_id, [&](stage::CopySsnTable &s, stage::CopySsn &) {
        auto it = s.readers.find(copy_id);
        const uint32_t k = it == s.readers.end() ? 0u : (uint32_t)it->second.size();
        for (uint32_t i = 0; i < k && i < max; ++i) read_ids[i] = it->second[i];
        *count = k;
        return STAGE_OK;
    });
}

// EphemeralPool::OverwriteVersionHeader::AddReader (ephemeral_pool.h:61-65), called by BTree::Read
// for a read served from the copy (b_tree.cpp:2104-2105)
int stage_copy_add_reader(stage_table *t, uint32_t copy_id, uint32_t read_id) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return with_copy(t, copy_id, [&](stage::CopySsnTable &s, stage::CopySsn &) {
        return guarded([&] {
            s.readers[copy_id].push_back(read_id);
            return STAGE_OK;
        });
    });
}

// IncreaseWRCount (+1: AddCount, refused once the header is waiting) / DecreaseWRCount (-1:
// SubCount), ephemeral_pool.cpp:69-103
int stage_copy_wr_count(stage_table *t, uint32_t copy_id, int delta, int *ok) {
    if (!t || !ok || (delta != 1 && delta != -1)) return fail(STAGE_E_ARG, "bad arguments");
    return with_copy(t, copy_id, [&](stage::CopySsnTable &, stage::CopySsn &c) {
        if (delta > 0) {
            *ok = c.waiting ? 0 : 1;
            if (*ok) ++c.count;
        } else {
            --c.count;
            *ok = 1;
        }
        return STAGE_OK;
    });
}

// UpdatePs (ephemeral_pool.cpp:194-205)
int stage_copy_update_ps(stage_table *t, uint32_t copy_id, uint32_t pstamp) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return with_copy(t, copy_id, [&](stage::CopySsnTable &, stage::CopySsn &c) {
        c.pstamp = pstamp;
        return STAGE_OK;
    });
}

int stage_import_leaf_images(stage_table *t, const uint8_t *blocks, uint64_t n_leaves, uint32_t block_size,
                             const uint64_t *sep_keys, const uint16_t *sep_lens, uint64_t *n_records) {
    if (!t || !blocks || (!sep_keys != !sep_lens)) return fail(STAGE_E_ARG, "bad arguments");
    return guarded([&] {
        const uint64_t n = host(t).import_leaf_images(blocks, n_leaves, block_size, sep_keys, sep_lens);
        if (n_records) *n_records = n;
        return STAGE_OK;
    });
}

int stage_probe_batch(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens, const uint32_t *d_read_ids,
                      const uint32_t *d_leaf_ids, uint64_t n, stage_probe_out *d_out, uint8_t *d_records,
                      void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (n && (!d_keys || !d_out)) return fail(STAGE_E_ARG, "null device buffer");
    hipError_t e = hipSetDevice(t->dev.device);
    if (e != hipSuccess) return hip_rc(e, "hipSetDevice");
    stage::DevTable view = t->dev.view;
    if (t->out_stride) view.stride = t->out_stride;
    stage::ProbeTuning tune = t->tune;
    tune.status_bytes = t->status_bytes;
    e = stage::launch_probe(view, d_keys, d_lens, d_read_ids, d_leaf_ids, n,
                            reinterpret_cast<stage::stage_probe_out_dev *>(d_out), d_records, pick(t, stream), tune);
    return hip_rc(e, "probe kernel");
}

int stage_probe_batch_ex(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens, const uint32_t *d_read_ids,
                         const uint32_t *d_leaf_ids, const uint8_t *d_for_update, uint64_t n, stage_probe_out *d_out,
                         uint8_t *d_records, void *stream) {
    if (!d_for_update) return stage_probe_batch(t, d_keys, d_lens, d_read_ids, d_leaf_ids, n, d_out, d_records, stream);
    if (!t) return fail(STAGE_E_ARG, "null table");
    if (t->status_bytes != 32)
        return fail(STAGE_E_UNSUPPORTED, "is_for_update probes need the 32-B status records (stage_set_output_layout)");
    int rc = stage_probe_batch(t, d_keys, d_lens, d_read_ids, d_leaf_ids, n, d_out, d_records, stream);
    if (rc) return rc;
    stage::DevTable view = t->dev.view;
    if (t->out_stride) view.stride = t->out_stride;
    return hip_rc(stage::launch_for_update(view, d_for_update, d_read_ids, n,
                                           reinterpret_cast<stage::stage_probe_out_dev *>(d_out), d_records,
                                           pick(t, stream)),
                  "for-update kernel");
}

int stage_set_output_layout(stage_table *t, uint32_t row_stride, uint32_t status_bytes) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    const uint32_t row = (host(t).key_pad() + host(t).params().payload_size + 15) & ~15u;
    if (row_stride && (row_stride < row || row_stride % 16))
        return fail(STAGE_E_ARG, "row_stride: 0 or a multiple of 16 of at least the row bytes (key pad + payload)");
    if (status_bytes != 32 && status_bytes != 16) return fail(STAGE_E_ARG, "status_bytes: 32 or 16");
    if (status_bytes == 16 && (host(t).params().key_width == 0 || host(t).key_words() != 1 || host(t).cap() != 64))
        return fail(STAGE_E_ARG, "16-B status records: fixed-width keys of <= 8 bytes in 64-slot leaves");
    t->out_stride = row_stride;
    t->status_bytes = (int)status_bytes;
    return STAGE_OK;
}

int stage_scan_batch(stage_table *t, const uint64_t *d_start_keys, const uint16_t *d_lens, uint64_t n,
                     uint32_t scan_size, uint32_t *d_counts, uint8_t *d_records, void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (n && (!d_start_keys || !d_counts || (!d_records && scan_size))) return fail(STAGE_E_ARG, "null device buffer");
    hipError_t e = hipSetDevice(t->dev.device);
    if (e != hipSuccess) return hip_rc(e, "hipSetDevice");
    e = stage::launch_scan(t->dev.view, d_start_keys, d_lens, n, scan_size, d_counts, d_records, pick(t, stream),
                          t->scan_tune);
    return hip_rc(e, "scan kernel");
}

int stage_index_scan_batch(stage_table *t, const uint64_t *d_start_keys, const uint16_t *d_lens,
                           const uint32_t *d_read_ids, uint64_t n, uint32_t scan_size, uint32_t *d_counts,
                           uint8_t *d_records, uint8_t *d_row_status, void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (n && (!d_start_keys || !d_counts || (scan_size && (!d_records || !d_row_status))))
        return fail(STAGE_E_ARG, "null device buffer");
    hipError_t e = hipSetDevice(t->dev.device);
    if (e != hipSuccess) return hip_rc(e, "hipSetDevice");
    e = stage::launch_scan(t->dev.view, d_start_keys, d_lens, n, scan_size, d_counts, d_records, pick(t, stream),
                           t->scan_tune, d_read_ids, d_row_status);
    return hip_rc(e, "index scan kernel");
}

int stage_index_scan_first_batch(stage_table *t, const uint64_t *d_start_keys, const uint32_t *d_read_ids,
                                 uint64_t n, uint32_t scan_size, uint32_t prefix_words, uint32_t *d_image,
                                 uint8_t *d_status, void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (t->dev.view.key_width == 0) return fail(STAGE_E_ARG, "first-tuple scans need fixed-width keys");
    if (scan_size == 0 || scan_size > 63) return fail(STAGE_E_ARG, "scan_size must be 1..63");
    if (prefix_words > t->dev.view.key_words) return fail(STAGE_E_ARG, "prefix_words exceeds the key's words");
    if (n && (!d_start_keys || !d_image || !d_status)) return fail(STAGE_E_ARG, "null device buffer");
    hipError_t e = hipSetDevice(t->dev.device);
    if (e != hipSuccess) return hip_rc(e, "hipSetDevice");
    e = stage::launch_scan_first(t->dev.view, d_start_keys, n, scan_size, d_read_ids, prefix_words, d_image, d_status,
                                 pick(t, stream), t->scan_tune);
    return hip_rc(e, "first-tuple scan kernel");
}

int stage_resolve_batch(stage_table *t, const uint64_t *d_keys, const uint16_t *d_lens, uint64_t n, int le_child,
                        uint32_t *d_leaf, void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (n && (!d_keys || !d_leaf)) return fail(STAGE_E_ARG, "null device buffer");
    hipError_t e = hipSetDevice(t->dev.device);
    if (e != hipSuccess) return hip_rc(e, "hipSetDevice");
    e = stage::launch_resolve(t->dev.view, d_keys, d_lens, n, le_child, d_leaf, pick(t, stream));
    return hip_rc(e, "resolve kernel");
}

int stage_set_probe_tuning(stage_table *t, int group, int max_blocks) {
    if (!t || (group != 1 && group != 2 && group != 4 && group != 8) || max_blocks < 0)
        return fail(STAGE_E_ARG, "bad tuning");
    t->tune.group = group;
    t->tune.max_blocks = max_blocks;
    return STAGE_OK;
}

int stage_set_probe_store(stage_table *t, int policy) {
    if (!t || policy < STAGE_STORE_TEMPORAL || policy > STAGE_STORE_WRITE_THROUGH)
        return fail(STAGE_E_ARG, "bad store policy");
    t->tune.store = policy;
    return STAGE_OK;
}

int stage_murmur64a_batch(const void *d_keys, uint32_t key_len, uint32_t key_stride, uint64_t seed, uint64_t n,
                          uint64_t *d_out, void *stream) {
    if (n && (!d_keys || !d_out || key_stride < key_len)) return fail(STAGE_E_ARG, "bad arguments");
    return hip_rc(stage::launch_murmur(d_keys, key_len, key_stride, seed, n, d_out, (hipStream_t)stream),
                  "murmur kernel");
}

// ---- plumbing
int stage_set_device(int device) { return hip_rc(hipSetDevice(device), "hipSetDevice"); }
int stage_device_count(int *count) { return hip_rc(hipGetDeviceCount(count), "hipGetDeviceCount"); }
int stage_dev_alloc(uint64_t bytes, void **ptr) { return hip_rc(hipMalloc(ptr, bytes ? bytes : 16), "hipMalloc"); }
int stage_dev_free(void *ptr) { return hip_rc(hipFree(ptr), "hipFree"); }
int stage_dev_memset(void *ptr, int value, uint64_t bytes, void *stream) {
    return hip_rc(hipMemsetAsync(ptr, value, bytes, (hipStream_t)stream), "hipMemsetAsync");
}
int stage_memcpy_h2d(void *dst, const void *src, uint64_t bytes, void *stream) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return hip_rc(e, "h2d");
}
int stage_memcpy_d2h(void *dst, const void *src, uint64_t bytes, void *stream) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return hip_rc(e, "d2h");
}
int stage_stream_create(void **stream) {
    return hip_rc(hipStreamCreateWithFlags((hipStream_t *)stream, hipStreamNonBlocking), "hipStreamCreate");
}
int stage_stream_destroy(void *stream) { return hip_rc(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy"); }
int stage_stream_sync(void *stream) { return hip_rc(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize"); }
int stage_device_sync(void) { return hip_rc(hipDeviceSynchronize(), "hipDeviceSynchronize"); }
int stage_event_create(void **ev) { return hip_rc(hipEventCreate((hipEvent_t *)ev), "hipEventCreate"); }
int stage_event_destroy(void *ev) { return hip_rc(hipEventDestroy((hipEvent_t)ev), "hipEventDestroy"); }
int stage_event_record(void *ev, void *stream) {
    return hip_rc(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "hipEventRecord");
}
int stage_event_elapsed(void *a, void *b, float *ms) {
    hipError_t e = hipEventSynchronize((hipEvent_t)b);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b);
    return hip_rc(e, "hipEventElapsedTime");
}

// ---- multi-GPU
int stage_comm_unique_id(uint8_t *id128) {
    if (!id128) return fail(STAGE_E_ARG, "null argument");
    return guarded([&] { return stage::shard_unique_id(id128); });
}

int stage_comm_init(stage_table *t, const uint8_t *id128, int rank, int world) {
    if (!t || !id128 || world < 1 || rank < 0 || rank >= world) return fail(STAGE_E_ARG, "bad arguments");
    if (facts(t).key_words() != 1) return fail(STAGE_E_ARG, "the sharded front-end routes keys of <= 8 bytes");
    return guarded([&] {
        (void)hipSetDevice(t->dev.device);
        t->comm = std::make_unique<stage::ShardComm>();
        const int rc = stage::shard_init(*t->comm, id128, rank, world, t->shard_chunks);
        if (t->shard_dedupe >= 0) t->comm->dedupe = t->shard_dedupe != 0;
        t->comm->key_bits = t->shard_key_bits;
        return rc;
    });
}

int stage_set_shard_dedupe(stage_table *t, int on) {
    if (!t || on < -1 || on > 1) return fail(STAGE_E_ARG, "dedupe must be -1, 0 or 1");
    t->shard_dedupe = on;
    const bool v = on < 0 ? stage::shard_default_dedupe() : on != 0;
    if (t->comm) t->comm->dedupe = v;
    if (t->loop_comm) t->loop_comm->dedupe = v;
    return STAGE_OK;
}

int stage_set_write_overlap(stage_table *t, int on) {
    if (!t || on < 0 || on > 1) return fail(STAGE_E_ARG, "write overlap must be 0 or 1");
    t->wp_overlap = on;
    return STAGE_OK;
}

int stage_set_shard_key_bits(stage_table *t, int bits) {
    if (!t || bits < 0 || bits > 64) return fail(STAGE_E_ARG, "bits must be 0..64");
    t->shard_key_bits = bits ? bits : 64;
    if (t->comm) t->comm->key_bits = t->shard_key_bits;
    if (t->loop_comm) t->loop_comm->key_bits = t->shard_key_bits;
    return STAGE_OK;
}

int stage_rccl_info(int *runtime_version, int *header_version, char *path, uint64_t path_len) {
    return guarded([&] { return stage::shard_rccl_info(runtime_version, header_version, path, path_len); });
}

int stage_sharded_stats(stage_table *t, int loopback, uint64_t *n_keys, uint64_t *n_routed, uint64_t *n_remote) {
    if (!t || !n_keys || !n_routed || !n_remote) return fail(STAGE_E_ARG, "null argument");
    stage::ShardComm *c = loopback ? t->loop_comm.get() : t->comm.get();
    if (!c) return fail(STAGE_E_STATE, "no sharded probe has run");
    *n_keys = c->last_n;
    *n_routed = c->last_routed;
    *n_remote = c->last_remote;
    return STAGE_OK;
}

int stage_sharded_stats_ex(stage_table *t, int loopback, uint64_t *v, int nv) {
    if (!t || !v || nv < 0) return fail(STAGE_E_ARG, "bad arguments");
    stage::ShardComm *c = loopback ? t->loop_comm.get() : t->comm.get();
    if (!c) return fail(STAGE_E_STATE, "no sharded probe has run");
    const uint64_t all[4] = {c->last_n, c->last_routed, c->last_remote, c->last_received};
    for (int i = 0; i < nv && i < 4; ++i) v[i] = all[i];
    return STAGE_OK;
}

int stage_comm_allreduce_f64(stage_table *t, double *values, uint64_t n, int op) {
    if (!t || (!values && n) || op < 0 || op > 2) return fail(STAGE_E_ARG, "bad arguments");
    if (!t->comm) return fail(STAGE_E_STATE, "stage_comm_init first");
    return guarded([&] {
        (void)hipSetDevice(t->dev.device);
        return stage::shard_allreduce_f64(*t->comm, values, n, op);
    });
}

int stage_comm_allgather_f64(stage_table *t, const double *in, uint64_t n, double *out) {
    if (!t || ((!in || !out) && n)) return fail(STAGE_E_ARG, "bad arguments");
    if (!t->comm) return fail(STAGE_E_STATE, "stage_comm_init first");
    return guarded([&] {
        (void)hipSetDevice(t->dev.device);
        return stage::shard_allgather_f64(*t->comm, in, n, out);
    });
}

int stage_set_shard_chunks(stage_table *t, int chunks) {
    if (!t || chunks < 0 || chunks > 64) return fail(STAGE_E_ARG, "chunks must be 0..64");
    t->shard_chunks = chunks;
    return STAGE_OK;
}

int stage_comm_destroy(stage_table *t) {
    if (!t) return fail(STAGE_E_ARG, "null table");
    return guarded([&] {
        t->comm.reset();
        return STAGE_OK;
    });
}

int stage_probe_sharded(stage_table *t, const uint64_t *d_keys, const uint32_t *d_read_ids, uint64_t n,
                        stage_probe_out *d_out, uint8_t *d_records, void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (!t->comm) return fail(STAGE_E_STATE, "stage_comm_init first");
    return guarded([&] {
        (void)hipSetDevice(t->dev.device);
        // the caller's row stride (stage_set_output_layout) is also the stride the rows travel
        // at: one row layout from the owner's probe to the caller's position
        stage::DevTable view = t->dev.view;
        if (t->out_stride) view.stride = t->out_stride;
        return stage::shard_probe(*t->comm, view, t->tune, d_keys, d_read_ids, n,
                                  reinterpret_cast<stage::stage_probe_out_dev *>(d_out), d_records, STAGE_REPLY_ROWS,
                                  pick(t, stream));
    });
}

int stage_probe_sharded_ex(stage_table *t, const uint64_t *d_keys, const uint32_t *d_read_ids, uint64_t n,
                           stage_probe_out *d_out, uint8_t *d_records, int reply_mode, void *stream) {
    int rc = need_synced(t);
    if (rc) return rc;
    if (!t->comm) return fail(STAGE_E_STATE, "stage_comm_init first");
    if (reply_mode != STAGE_REPLY_ROWS && reply_mode != STAGE_REPLY_OWNER && reply_mode != STAGE_REPLY_PEER &&
        reply_mode != STAGE_REPLY_DIRECT)
        return fail(STAGE_E_ARG, "bad reply mode");
    return guarded([&] {
        (void)hipSetDevice(t->dev.device);
        // the caller's row stride (stage_set_output_layout) is also the stride the rows travel
        // at: one row layout from the owner's probe to the caller's position
        stage::DevTable view = t->dev.view;
        if (t->out_stride) view.stride = t->out_stride;
        return stage::shard_probe(*t->comm, view, t->tune, d_keys, d_read_ids, n,
                                  reinterpret_cast<stage::stage_probe_out_dev *>(d_out), d_records, reply_mode,
                                  pick(t, stream));
    });
}

int stage_sharded_owner_rows(stage_table *t, int loopback, uint8_t **d_rows, uint64_t *n_rows) {
    if (!t || !d_rows || !n_rows) return fail(STAGE_E_ARG, "null argument");
    stage::ShardComm *c = loopback ? t->loop_comm.get() : t->comm.get();
    if (!c) return fail(STAGE_E_STATE, "no sharded probe has run");
    *d_rows = (uint8_t *)c->rrec;
    *n_rows = c->owner_rows;
    return STAGE_OK;
}

int stage_probe_sharded_loopback(stage_table *const *shards, int world, const uint64_t *const *d_keys,
                                 const uint32_t *const *d_read_ids, const uint64_t *n, stage_probe_out *const *d_out,
                                 uint8_t *const *d_records, int reply_mode, void *stream) {
    if (!shards || world < 1 || !d_keys || !n || !d_out || !d_records) return fail(STAGE_E_ARG, "null argument");
    if (reply_mode != STAGE_REPLY_ROWS && reply_mode != STAGE_REPLY_OWNER && reply_mode != STAGE_REPLY_PEER &&
        reply_mode != STAGE_REPLY_DIRECT)
        return fail(STAGE_E_ARG, "bad reply mode");
    for (int r = 0; r < world; ++r) {
        int rc = need_synced(shards[r]);
        if (rc) return rc;
        if (facts(shards[r]).key_words() != 1) return fail(STAGE_E_ARG, "the sharded front-end routes keys of <= 8 bytes");
        if (shards[r]->dev.device != shards[0]->dev.device) return fail(STAGE_E_ARG, "shards on different devices");
        if ((d_records[r] == nullptr) != (d_records[0] == nullptr)) return fail(STAGE_E_ARG, "rows for all or none");
    }
    return guarded([&] {
        (void)hipSetDevice(shards[0]->dev.device);
        std::vector<stage::ShardComm *> cs(world);
        std::vector<const stage::DevTable *> ts(world);
        std::vector<stage::DevTable> views(world);
        std::vector<const uint64_t *> ks(world);
        std::vector<const uint32_t *> rs(world);
        std::vector<uint64_t> ns(world);
        std::vector<stage::stage_probe_out_dev *> os(world);
        std::vector<uint8_t *> recs(world);
        for (int r = 0; r < world; ++r) {
            stage_table *t = shards[r];
            const int want = shards[0]->shard_chunks > 0 ? shards[0]->shard_chunks : stage::shard_default_chunks(world);
            if (!t->loop_comm || t->loop_comm->world != world || t->loop_comm->rank != r ||
                t->loop_comm->chunks != want) {
                t->loop_comm = std::make_unique<stage::ShardComm>();
                stage::shard_init_loopback(*t->loop_comm, r, world, want);
            }
            if (t->shard_dedupe >= 0) t->loop_comm->dedupe = t->shard_dedupe != 0;
            t->loop_comm->key_bits = t->shard_key_bits;
            cs[r] = t->loop_comm.get();
            views[r] = t->dev.view;
            if (shards[0]->out_stride) views[r].stride = shards[0]->out_stride;  // as stage_probe_sharded_ex
            ts[r] = &views[r];
            ks[r] = d_keys[r];
            rs[r] = d_read_ids ? d_read_ids[r] : nullptr;
            ns[r] = n[r];
            os[r] = reinterpret_cast<stage::stage_probe_out_dev *>(d_out[r]);
            recs[r] = d_records[r];
        }
        return stage::shard_probe_loopback(cs, ts, shards[0]->tune, ks, rs, ns, os, recs, reply_mode,
                                           pick(shards[0], stream));
    });
}

}  // extern "C"

namespace stage {
void set_error(const std::string &msg) { g_err = msg; }
}  // namespace stage
