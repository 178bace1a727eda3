// adapter_drive.cpp -- the reference-side adapter (include/stage_btree_adapter.hpp) driven
// through the C-ABI, written against the two public headers only (what a reference BTree
// facade compiles against).
//
//   adapter_drive probe <out.bin>
//       builds a YCSB table (4-byte keys, 1000-B payload, 5000 rows) through the C-ABI, writes
//       the version-chain scenarios below on the host write path, publishes, probes a fixed
//       list of (key, read id) pairs with stage_probe_batch + stage_probe_identify and frames
//       every result
//   adapter_drive frame <in.bin> <out.bin>
//       frames stage_probe_out records + stage_probe_ident records + rows read from in.bin (n u64,
//       n keys u64, n read ids u32, n x 32-B records, n x 8-B idents, n x 1008-B rows) -- the same
//       adapter calls without a device
//
// The Record's loc_ptr is written as the location handle itself (a facade puts its
// LocationTable::get(handle) there; the bytes are compared, so the handle stands for it).
// out.bin: n u64, then per result: key u64, read id u32, status u8, ReturnCode u8, ResultType
// u8, perform_read u8, tuple u8, retired u8, read_via_copy u8, record length u16, record bytes,
// 1004 tuple bytes.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/stage_btree_adapter.hpp"
#include "../../include/stage_hip.h"

#define CK(x)                                                                             \
    do {                                                                                  \
        int rc_ = (x);                                                                    \
        if (rc_) {                                                                        \
            std::fprintf(stderr, "%s failed: rc=%d %s\n", #x, rc_, stage_last_error()); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

namespace {
constexpr uint32_t kPayload = 1000, kRow = 1008;

void frame_all(const std::vector<uint64_t> &keys, const std::vector<uint32_t> &rids,
               const std::vector<stage_probe_out> &outs, const std::vector<stage_probe_ident> &ids,
               const std::vector<uint8_t> &rows, FILE *f) {
    const uint64_t n = keys.size();
    std::fwrite(&n, 8, 1, f);
    for (uint64_t i = 0; i < n; ++i) {
        const stage_probe_out &o = outs[i];
        const uint8_t *row = rows.data() + i * kRow;
        const std::vector<uint8_t> rec = stage_adapter::make_record(o, ids[i], ids[i].loc, row, kPayload);
        const stage_adapter::PointLookup p = stage_adapter::point_lookup(o);
        uint8_t tup[stage_adapter::kYcsbTupleInt] = {};
        stage_adapter::ycsb_tuple_int(o, row, tup);
        const uint8_t hdr[8] = {o.status, (uint8_t)stage_adapter::read_return_code(o), (uint8_t)p.result,
                                (uint8_t)p.perform_read, (uint8_t)p.tuple, (uint8_t)p.retired,
                                (uint8_t)stage_adapter::read_via_copy(o, ids[i]), 0};
        const uint16_t len = (uint16_t)rec.size();
        std::fwrite(&keys[i], 8, 1, f);
        std::fwrite(&rids[i], 4, 1, f);
        std::fwrite(hdr, 1, 7, f);
        std::fwrite(&len, 2, 1, f);
        std::fwrite(rec.data(), 1, rec.size(), f);
        std::fwrite(tup, 1, sizeof tup, f);
    }
}

int probe_mode(const char *path) {
    stage_params p{16 * 1024, 32 * 1024, 64 * 1024, kPayload, 4, 0};
    stage_table *t = nullptr;
    CK(stage_table_create(&p, &t));
    uint64_t loaded = 0;
    CK(stage_load_ycsb(t, 0, 5000, 4, 0, &loaded));
    uint8_t rc = 0;
    std::vector<uint8_t> d7(100, 7), d9(100, 9), d5(100, 55), d1(100, 11);
    // SURVEY App. B scenario, key 3: update at read id 1 / commit 2, update at 5 / commit 6
    CK(stage_update(t, 3, 4, 0, d7.data(), 100, 1, &rc));
    CK(stage_commit_update(t, 3, 4, 2, 2, &rc));
    CK(stage_update(t, 3, 4, 0, d9.data(), 100, 5, &rc));
    CK(stage_commit_update(t, 3, 4, 6, 6, &rc));
    // key 5: an update left in flight (writer 8)
    CK(stage_update(t, 5, 4, 0, d5.data(), 100, 8, &rc));
    // key 9042 inserted at commit 10, updated at 11 / commit 12: read id 5 sees no version
    std::vector<uint8_t> pay(kPayload, 0x42);
    CK(stage_insert(t, 9042, 4, pay.data(), 0, 0, 10, &rc));
    CK(stage_update(t, 9042, 4, 0, d1.data(), 100, 11, &rc));
    CK(stage_commit_update(t, 9042, 4, 12, 12, &rc));
    CK(stage_sync(t));
    const std::vector<uint64_t> keys = {3, 3, 3, 3, 5, 5, 9042, 9042, 9042, 77, 123456, 4999};
    const std::vector<uint32_t> rids = {0xFFFFFFFEu, 4, 1, 0, 10, 3, 5, 11, 13, 100, 7, 1};
    const uint64_t n = keys.size();
    std::vector<stage_probe_out> outs(n);
    std::vector<stage_probe_ident> ids(n);
    const uint32_t stride = stage_record_stride(t);  // output row pitch (>= 8 + payload)
    std::vector<uint8_t> wide(n * stride), rows(n * kRow);
    void *dk, *dr, *dout, *did, *drow;
    CK(stage_dev_alloc(8 * n, &dk));
    CK(stage_dev_alloc(4 * n, &dr));
    CK(stage_dev_alloc(32 * n, &dout));
    CK(stage_dev_alloc(8 * n, &did));
    CK(stage_dev_alloc((uint64_t)stride * n, &drow));
    CK(stage_memcpy_h2d(dk, keys.data(), 8 * n, nullptr));
    CK(stage_memcpy_h2d(dr, rids.data(), 4 * n, nullptr));
    CK(stage_probe_batch(t, (const uint64_t *)dk, nullptr, (const uint32_t *)dr, nullptr, n, (stage_probe_out *)dout,
                         (uint8_t *)drow, nullptr));
    CK(stage_probe_identify(t, (const stage_probe_out *)dout, n, (stage_probe_ident *)did, nullptr));
    CK(stage_device_sync());  // the probe ran on the table's stream, the copies use the null stream
    CK(stage_memcpy_d2h(outs.data(), dout, 32 * n, nullptr));
    CK(stage_memcpy_d2h(ids.data(), did, 8 * n, nullptr));
    CK(stage_memcpy_d2h(wide.data(), drow, (uint64_t)stride * n, nullptr));
    for (void *p : {dk, dr, dout, did, drow}) CK(stage_dev_free(p));
    for (size_t i = 0; i < n; ++i) std::memcpy(&rows[i * kRow], &wide[i * stride], kRow);
    FILE *f = std::fopen(path, "wb");
    if (!f) return 1;
    frame_all(keys, rids, outs, ids, rows, f);
    std::fclose(f);
    CK(stage_table_destroy(t));
    return 0;
}

int frame_mode(const char *in, const char *out) {
    FILE *f = std::fopen(in, "rb");
    if (!f) return 1;
    uint64_t n = 0;
    if (std::fread(&n, 8, 1, f) != 1) return 1;
    std::vector<uint64_t> keys(n);
    std::vector<uint32_t> rids(n);
    std::vector<stage_probe_out> outs(n);
    std::vector<stage_probe_ident> ids(n);
    std::vector<uint8_t> rows(n * kRow);
    if (std::fread(keys.data(), 8, n, f) != n || std::fread(rids.data(), 4, n, f) != n ||
        std::fread(outs.data(), sizeof(stage_probe_out), n, f) != n ||
        std::fread(ids.data(), sizeof(stage_probe_ident), n, f) != n || std::fread(rows.data(), 1, n * kRow, f) != n * kRow)
        return 1;
    std::fclose(f);
    FILE *g = std::fopen(out, "wb");
    if (!g) return 1;
    frame_all(keys, rids, outs, ids, rows, g);
    std::fclose(g);
    return 0;
}
}  // namespace

int main(int argc, char **argv) {
    static_assert(sizeof(stage_probe_out) == 32, "32-B probe records");
    if (argc >= 3 && !std::strcmp(argv[1], "probe")) return probe_mode(argv[2]);
    if (argc >= 4 && !std::strcmp(argv[1], "frame")) return frame_mode(argv[2], argv[3]);
    std::fprintf(stderr, "usage: %s probe <out.bin> | frame <in.bin> <out.bin>\n", argv[0]);
    return 2;
}
