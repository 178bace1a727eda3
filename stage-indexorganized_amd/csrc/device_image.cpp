// device_image.cpp -- builds the HBM image of a table from its host layout.
#include "device_image.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace stage {

void hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static void dev_ensure(DevBuf &b, uint64_t bytes, const char *what) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return;
    if (b.p) hip_check(hipFree(b.p), "hipFree");
    b.p = nullptr;
    b.cap = 0;
    hip_check(hipMalloc(&b.p, bytes), what);
    b.cap = bytes;
}

DeviceImage::~DeviceImage() { release(); }

void DeviceImage::release() {
    for (DevBuf *b :
         {&head, &okey, &slot, &tree, &tree_len, &heap, &chdr, &vhdr, &arena, &descs, &patch, &scratch, &wp_scratch, &wp_bases}) {
        if (b->p) (void)hipFree(b->p);
        b->p = nullptr;
        b->cap = 0;
    }
    for (DevBuf *b = wp_out; b != wp_out + kWpDepth; ++b) {
        if (b->p) (void)hipFree(b->p);
        b->p = nullptr;
        b->cap = 0;
    }
    for (int k = 0; k < kQ2Pinned + 2; ++k) {
        if (pinned[k]) (void)hipHostFree(pinned[k]);
        pinned[k] = nullptr;
        pinned_cap[k] = 0;
    }
    for (int k = 0; k < kWpDepth; ++k) {
        if (adopt_ev[k]) (void)hipEventDestroy(adopt_ev[k]);
        adopt_ev[k] = nullptr;
        if (export_ev[k]) (void)hipEventDestroy(export_ev[k]);
        export_ev[k] = nullptr;
    }
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
    if (adopt_stream) (void)hipStreamDestroy(adopt_stream);
    adopt_stream = nullptr;
    if (wp_pub_ev) (void)hipEventDestroy(wp_pub_ev);
    if (wp_pre_ev) (void)hipEventDestroy(wp_pre_ev);
    wp_pub_ev = wp_pre_ev = nullptr;
    wp_pub_valid = false;
    if (wp_stream) (void)hipStreamDestroy(wp_stream);
    wp_stream = nullptr;
    valid = false;
}

template <class F>
static void parallel_for(uint64_t n, F fn) {
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < (1u << 16)) nt = 1;
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nt; ++k)
        th.emplace_back([=] {
            uint64_t b = n * k / nt, e = n * (k + 1) / nt;
            for (uint64_t i = b; i < e; ++i) fn(i);
        });
    for (auto &x : th) x.join();
}

static void upload(DevBuf &b, const void *src, uint64_t bytes, hipStream_t s, const char *what) {
    dev_ensure(b, bytes, what);
    if (bytes) hip_check(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s), what);
}

// One leaf's head (fingerprints + visible mask), key planes and slot words, reference slot
// order.  okey points at the leaf's KW planes of cap words.
static void build_leaf(const HostTable &h, uint32_t hl, uint8_t *hd, uint64_t *okey, SlotInfo *slot) {
    const stage_params &p = h.params();
    const uint32_t kw = h.key_words(), cap = h.cap(), spl = cap / 64, hb = leaf_head_bytes(cap, kw);
    const uint64_t hbase = (uint64_t)hl * cap;
    const uint32_t count = h.leaves_[hl].count;
    std::memset(hd, 0, hb);
    uint64_t vis[16] = {0};  // up to 1024 slots
    for (uint32_t s = 0; s < cap; ++s) {
        const bool live = s < count;
        const uint64_t m = live ? h.meta_[hbase + s] : 0;
        uint64_t w[kMaxKeyWords] = {0, 0, 0, 0};
        if (live)
            for (uint32_t j = 0; j < kw; ++j) w[j] = h.okey_[(hbase + s) * kw + j];
        for (uint32_t j = 0; j < kw; ++j) okey[(uint64_t)j * cap + s] = w[j];
        slot[s].okey = w[0];
        slot[s].meta = m;
        slot[s].next = live ? h.next_[hbase + s] : 0;
        slot[s].image = live ? h.image_[hbase + s] : 0;
        slot[s].loc = live ? h.loc_[hbase + s] : 0;
        slot[s].pad = 0;
        if (meta_visible(m) && (p.key_width == 0 || meta_keylen(m) == p.key_width)) {
            vis[s / 64] |= 1ull << (s % 64);
            hd[s] = (uint8_t)key_fp_words(w, kw);
        }
    }
    std::memcpy(hd + cap, vis, 8 * spl);
    // group max keys over live slots (lexicographic on the order words)
    uint64_t *gm = reinterpret_cast<uint64_t *>(hd + head_gmax_offset(cap));
    for (uint32_t g = 0; g < spl; ++g) {
        uint64_t best[kMaxKeyWords] = {0, 0, 0, 0};
        for (uint32_t s = g * 64; s < g * 64 + 64 && s < count; ++s) {
            const uint64_t *w = h.okey_.data() + (hbase + s) * kw;
            bool gt = false;
            for (uint32_t j = 0; j < kw; ++j)
                if (w[j] != best[j]) {
                    gt = w[j] > best[j];
                    break;
                }
            if (gt)
                for (uint32_t j = 0; j < kw; ++j) best[j] = w[j];
        }
        for (uint32_t j = 0; j < kw; ++j) std::memcpy(gm + g * kw + j, &best[j], 8);
    }
    // info word: count | mp << 16, mp = the longest slot prefix with strictly increasing keys
    uint32_t mp = count ? 1u : 0u;
    while (mp < count) {
        const uint64_t *a = h.okey_.data() + (hbase + mp - 1) * kw, *b = a + kw;
        bool lt = false;
        for (uint32_t j = 0; j < kw; ++j)
            if (a[j] != b[j]) {
                lt = a[j] < b[j];
                break;
            }
        if (!lt) break;
        ++mp;
    }
    const uint32_t info = count | (mp << 16);
    std::memcpy(hd + head_info_offset(cap, kw), &info, 4);
}

// grow a device buffer to `bytes`, keeping its first `keep` bytes
static void grow_keep(DevBuf &b, uint64_t bytes, uint64_t keep, const char *what, hipStream_t s) {
    if (b.cap >= bytes && b.p) return;
    DevBuf nb;
    // doubling: the header arrays grow by one epoch at a time, and each growth synchronises
    const uint64_t want = std::max<uint64_t>(2 * bytes, 4096);
    hip_check(hipMalloc(&nb.p, want), what);
    nb.cap = want;
    if (b.p && keep) hip_check(hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, s), what);
    hip_check(hipStreamSynchronize(s), what);
    if (b.p) hip_check(hipFree(b.p), "hipFree");
    b = nb;
}

// record heap able to hold `rows` rows (the first images_synced_ rows are kept)
static void grow_heap(HostTable &h, DeviceImage &d, uint64_t rows_needed, hipStream_t s) {
    if (rows_needed <= d.heap_rows) return;
    const uint32_t stride = h.hstride();
    // first allocation: 1/16 spare rows; a heap that had to grow is being written (e.g. a device
    // write-path epoch appends one image per successful update): 1/8, so that the copy of the
    // whole heap a growth costs comes half as often (the old and the new heap coexist during
    // the copy: 2.1x the rows at the peak)
    const uint64_t rows = rows_needed + std::max<uint64_t>(rows_needed / (d.heap.p ? 8 : 16), 1024);
    DevBuf nb;
    hip_check(hipMalloc(&nb.p, rows * stride), "record heap");
    nb.cap = rows * stride;
    if (d.heap.p && h.images_synced_) {
        hip_check(hipMemcpyAsync(nb.p, d.heap.p, h.images_synced_ * stride, hipMemcpyDeviceToDevice, s), "heap grow");
        hip_check(hipStreamSynchronize(s), "heap grow sync");
    }
    if (d.heap.p) hip_check(hipFree(d.heap.p), "hipFree heap");
    d.heap = nb;
    d.heap_rows = rows;
}

static uint8_t *grow_scratch(DevBuf &b, uint64_t bytes, const char *what) {
    if (b.cap < bytes) {
        if (b.p) {
            hip_check(hipDeviceSynchronize(), what);
            hip_check(hipFree(b.p), what);
        }
        b.p = nullptr;
        b.cap = 0;
        const uint64_t want = bytes + bytes / 8 + 4096;
        hip_check(hipMalloc(&b.p, want), what);
        b.cap = want;
    }
    return (uint8_t *)b.p;
}

uint8_t *scratch_bytes(DeviceImage &d, uint64_t bytes) { return grow_scratch(d.scratch, bytes, "scratch"); }

uint8_t *wp_scratch_bytes(DeviceImage &d, uint64_t bytes) { return grow_scratch(d.wp_scratch, bytes, "write-path scratch"); }

uint8_t *pinned_bytes(DeviceImage &d, uint64_t bytes, int k) {
    if (d.pinned_cap[k] < bytes) {
        if (d.pinned[k]) hip_check(hipHostFree(d.pinned[k]), "hipHostFree staging");
        d.pinned[k] = nullptr;
        d.pinned_cap[k] = 0;
        const uint64_t want = bytes + bytes / 4 + 4096;
        hip_check(hipHostMalloc(&d.pinned[k], want, hipHostMallocDefault), "pinned staging");
        d.pinned_cap[k] = want;
    }
    return (uint8_t *)d.pinned[k];
}

uint8_t *wp_out_bytes(DeviceImage &d, uint64_t bytes, int k) {
    DevBuf &b = d.wp_out[k];
    if (b.cap < bytes) {
        if (b.p) {
            hip_check(hipDeviceSynchronize(), "wp_out drain");
            hip_check(hipFree(b.p), "hipFree wp_out");
        }
        b.p = nullptr;
        b.cap = 0;
        const uint64_t want = bytes + bytes / 8 + 4096;
        hip_check(hipMalloc(&b.p, want), "wp_out");
        b.cap = want;
    }
    return (uint8_t *)b.p;
}

void reserve_device_rows(HostTable &h, DeviceImage &d, uint64_t extra_images, uint64_t extra_copies,
                         uint64_t extra_versions, hipStream_t s) {
    d.wp_pub_valid = false;  // the grown arrays are filled on s: an overlapped epoch waits for s
    grow_heap(h, d, h.images_.size() + extra_images, s);
    grow_keep(d.chdr, (h.copies_.size() + extra_copies) * sizeof(CopyHdr), h.copies_synced_ * sizeof(CopyHdr), "chdr",
              s);
    grow_keep(d.vhdr, (h.versions_.size() + extra_versions) * sizeof(VersionHdr),
              h.versions_synced_ * sizeof(VersionHdr), "vhdr", s);
    d.view.heap = (const uint8_t *)d.heap.p;
    d.view.chdr = (const CopyHdr *)d.chdr.p;
    d.view.vhdr = (const VersionHdr *)d.vhdr.p;
}

// Copy/version headers: append the new tail, re-send the rewritten range of copy headers.
static void sync_headers(HostTable &h, DeviceImage &d, hipStream_t s) {
    const uint64_t nc = h.copies_.size(), nv = h.versions_.size();
    grow_keep(d.chdr, nc * sizeof(CopyHdr), h.copies_synced_ * sizeof(CopyHdr), "chdr", s);
    grow_keep(d.vhdr, nv * sizeof(VersionHdr), h.versions_synced_ * sizeof(VersionHdr), "vhdr", s);
    const uint64_t c0 = std::min<uint64_t>(h.copies_synced_, h.copies_dirty_from_);
    if (nc > c0)
        hip_check(hipMemcpyAsync((CopyHdr *)d.chdr.p + c0, h.copies_.data() + c0, (nc - c0) * sizeof(CopyHdr),
                                 hipMemcpyHostToDevice, s),
                  "chdr upload");
    if (nv > h.versions_synced_)
        hip_check(hipMemcpyAsync((VersionHdr *)d.vhdr.p + h.versions_synced_, h.versions_.data() + h.versions_synced_,
                                 (nv - h.versions_synced_) * sizeof(VersionHdr), hipMemcpyHostToDevice, s),
                  "vhdr upload");
    h.copies_synced_ = nc;
    h.versions_synced_ = nv;
    h.copies_dirty_from_ = ~0ull;
}

// Incremental publish (no split since the last publish): leaf order and separators are
// unchanged, so only the written slots and their leaves' heads are patched in place.
static void patch_device(HostTable &h, DeviceImage &d, hipStream_t s) {
    const uint32_t cap = h.cap(), hb = leaf_head_bytes(cap, h.key_words());
    std::vector<uint64_t> &ds = h.dirty_slots_;
    std::sort(ds.begin(), ds.end());
    ds.erase(std::unique(ds.begin(), ds.end()), ds.end());
    std::vector<uint32_t> leaves;
    std::vector<uint64_t> first;  // first dirty slot of each leaf in ds
    for (uint64_t k = 0; k < ds.size(); ++k)
        if (leaves.empty() || leaves.back() != ds[k] / cap) {
            leaves.push_back((uint32_t)(ds[k] / cap));
            first.push_back(k);
        }
    first.push_back(ds.size());
    const uint64_t nl = leaves.size(), ns = ds.size();
    if (nl == 0) return;
    // staging: [dev leaf u32 ...][heads nl*hb][slot idx u64 ...][SlotInfo ...][key words ns*kw],
    // 32-B aligned parts
    const uint32_t kw = h.key_words();
    auto al = [](uint64_t x) { return (x + 31) & ~31ull; };
    const uint64_t o_head = al(nl * 4), o_idx = o_head + al(nl * hb), o_src = o_idx + al(ns * 8);
    const uint64_t o_words = o_src + al(ns * sizeof(SlotInfo));
    const uint64_t bytes = o_words + ns * kw * 8;
    d.staging.resize(bytes);
    uint8_t *st = d.staging.data();
    uint32_t *dleaf = (uint32_t *)st;
    uint64_t *sidx = (uint64_t *)(st + o_idx);
    SlotInfo *ssrc = (SlotInfo *)(st + o_src);
    uint64_t *swords = (uint64_t *)(st + o_words);
    parallel_for(nl, [&](uint64_t li) {
        thread_local std::vector<uint64_t> okey_tmp;
        thread_local std::vector<SlotInfo> slot_tmp;
        okey_tmp.resize((uint64_t)cap * kw);
        slot_tmp.resize(cap);
        const uint32_t hl = leaves[li], dl = d.host_to_dev[hl];
        dleaf[li] = dl;
        build_leaf(h, hl, st + o_head + li * hb, okey_tmp.data(), slot_tmp.data());
        for (uint64_t k = first[li]; k < first[li + 1]; ++k) {
            const uint32_t sl = (uint32_t)(ds[k] % cap);
            sidx[k] = (uint64_t)dl * cap + sl;
            ssrc[k] = slot_tmp[sl];
            for (uint32_t j = 0; j < kw; ++j) swords[k * kw + j] = okey_tmp[(uint64_t)j * cap + sl];
        }
    });
    upload(d.patch, st, bytes, s, "patch staging");
    uint8_t *dp = (uint8_t *)d.patch.p;
    hip_check(launch_patch((uint8_t *)d.head.p, (uint64_t *)d.okey.p, (SlotInfo *)d.slot.p, hb, cap, kw,
                           (const uint32_t *)dp, dp + o_head, nl, (const uint64_t *)(dp + o_idx),
                           (const SlotInfo *)(dp + o_src), (const uint64_t *)(dp + o_words), ns, s),
              "patch");
    d.last_patch_leaves = nl;
    d.last_patch_slots = ns;
}

// ---- record heap: fill the rows of images created since the last sync
static void sync_heap(HostTable &h, DeviceImage &d, hipStream_t s) {
    const stage_params &p = h.params();
    const uint32_t stride = h.hstride();
    const uint64_t nimg = h.images_.size();
    grow_heap(h, d, nimg, s);
    if (h.arena_.size() > h.arena_synced_) {
        // the device arena mirrors the host arena; grow keeps the already uploaded prefix
        if (d.arena.cap < h.arena_.size()) {
            DevBuf nb;
            const uint64_t bytes = h.arena_.size() + h.arena_.size() / 4 + 4096;
            hip_check(hipMalloc(&nb.p, bytes), "arena");
            nb.cap = bytes;
            if (d.arena.p && h.arena_synced_)
                hip_check(hipMemcpyAsync(nb.p, d.arena.p, h.arena_synced_, hipMemcpyDeviceToDevice, s), "arena grow");
            hip_check(hipStreamSynchronize(s), "arena sync");
            if (d.arena.p) hip_check(hipFree(d.arena.p), "hipFree arena");
            d.arena = nb;
        }
        h.arena_.segments(h.arena_synced_, h.arena_.size(), [&](uint64_t off, const uint8_t *src, uint64_t bytes) {
            hip_check(hipMemcpyAsync((uint8_t *)d.arena.p + off, src, bytes, hipMemcpyHostToDevice, s),
                      "arena upload");
        });
        h.arena_synced_ = h.arena_.size();
    }
    const uint64_t first = h.images_synced_, count = nimg - first;
    if (count) {
        // identity run (LoadYCSBRows): image r = rowid0 + r, key = rowid, one payload mode
        const ImageDesc &d0 = h.images_[first];
        bool ident = d0.kind == 0;
        uint32_t kw = 8;
        if (ident) {
            const uint64_t kmask_bits = d0.key_le;
            (void)kmask_bits;
            kw = p.key_width ? p.key_width : 8;
            const uint64_t kmask = kw >= 8 ? ~0ull : ((1ull << (8 * kw)) - 1);
            for (uint64_t r = 0; r < count && ident; ++r) {
                const ImageDesc &e = h.images_[first + r];
                ident = e.kind == 0 && e.mode == d0.mode && e.arg == d0.arg + r && e.key_le == (e.arg & kmask);
            }
        }
        if (ident) {
            hip_check(launch_fill((uint8_t *)d.heap.p, stride, p.payload_size, h.key_pad() + p.payload_size, nullptr,
                                  nullptr, first, count, d0.arg, kw, (int)d0.mode, s),
                      "fill (identity)");
        } else {
            std::vector<ImageDescDev> dd(count);
            for (uint64_t r = 0; r < count; ++r) {
                const ImageDesc &e = h.images_[first + r];
                dd[r] = ImageDescDev{e.key_le, e.arg, e.kind, e.mode};
            }
            upload(d.descs, dd.data(), count * sizeof(ImageDescDev), s, "descs");
            hip_check(launch_fill((uint8_t *)d.heap.p, stride, p.payload_size, h.key_pad() + p.payload_size,
                                  (const ImageDescDev *)d.descs.p, (const uint8_t *)d.arena.p, first, count, 0, 0, 0,
                                  s),
                      "fill");
            hip_check(hipStreamSynchronize(s), "fill sync");  // dd is pageable and local
        }
        h.images_synced_ = nimg;
    }
}

void sync_device(HostTable &h, DeviceImage &d) {
    auto t0 = std::chrono::steady_clock::now();
    d.wp_pub_valid = false;  // the next overlapped write-path epoch waits for this publish
    hip_check(hipSetDevice(d.device), "hipSetDevice");
    if (!d.stream) hip_check(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking), "hipStreamCreate");
    hipStream_t s = d.stream;
    if (d.valid && !h.structure_dirty_ && d.host_to_dev.size() == h.leaves_.size()) {
        patch_device(h, d, s);
        sync_headers(h, d, s);
        sync_heap(h, d, s);
        hip_check(hipStreamSynchronize(s), "sync");
        d.view.heap = (const uint8_t *)d.heap.p;
        d.view.chdr = (const CopyHdr *)d.chdr.p;
        d.view.vhdr = (const VersionHdr *)d.vhdr.p;
        h.dirty_slots_.clear();
        h.layout_dirty_ = false;
        d.last_sync_incremental = true;
        d.last_sync_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return;
    }
    const stage_params &p = h.params();
    const uint32_t cap = h.cap();

    // ---- leaves in key order
    std::vector<uint32_t> order;
    h.key_order(order);
    const uint64_t L = order.size();
    d.host_to_dev.assign(h.leaves_.size(), 0xFFFFFFFFu);
    for (uint64_t i = 0; i < L; ++i) d.host_to_dev[order[i]] = (uint32_t)i;
    d.dev_to_host = order;

    const uint32_t kw = h.key_words(), hb = leaf_head_bytes(cap, kw);
    std::vector<uint64_t> okey(L * cap * kw);
    std::vector<uint8_t> head(L * hb, 0);
    std::vector<SlotInfo> slot(L * cap);
    parallel_for(L, [&](uint64_t di) {
        build_leaf(h, order[di], head.data() + di * hb, okey.data() + di * cap * kw, slot.data() + di * cap);
    });

    // ---- implicit separator tree: level 0 = separators in 8-entry nodes (a probe's bottom
    // node is one 64-B sector for 8-B keys), level k+1 = max of each node of level k in
    // 16-entry nodes (one 128-B line), every level padded with +inf, top level one node.  An
    // entry is kw order words (entry-major); lengths ride along for variable-length tables.
    const uint64_t S = L ? L - 1 : 0;
    std::vector<std::vector<uint64_t>> lv;
    std::vector<std::vector<uint8_t>> lvlen;
    {
        const uint64_t n0 = (S + 1 + kLeafFanout - 1) / kLeafFanout * kLeafFanout;
        std::vector<uint64_t> l0(n0 * kw, ~0ull);
        std::vector<uint8_t> l0len(n0, 0xFF);
        for (uint64_t i = 0; i < S; ++i) {
            const auto &sep = h.leaves_[order[i]].sep;
            for (uint32_t j = 0; j < kw; ++j) l0[i * kw + j] = sep.w[j];
            l0len[i] = (uint8_t)sep.len;
        }
        lv.push_back(std::move(l0));
        lvlen.push_back(std::move(l0len));
        while (lvlen.back().size() > (uint64_t)tree_fanout((int)lv.size() - 1)) {
            const uint64_t f = (uint64_t)tree_fanout((int)lv.size() - 1);
            const auto &prev = lv.back();
            const auto &prevlen = lvlen.back();
            const uint64_t nodes = prevlen.size() / f;
            const uint64_t nn = (nodes + kTreeFanout - 1) / kTreeFanout * kTreeFanout;
            std::vector<uint64_t> nx(nn * kw, ~0ull);
            std::vector<uint8_t> nxlen(nn, 0xFF);
            for (uint64_t j = 0; j < nodes; ++j) {
                const uint64_t last = j * f + f - 1;
                for (uint32_t w = 0; w < kw; ++w) nx[j * kw + w] = prev[last * kw + w];
                nxlen[j] = prevlen[last];
            }
            lv.push_back(std::move(nx));
            lvlen.push_back(std::move(nxlen));
        }
    }
    if (lv.size() > (size_t)kMaxTreeLevels) throw std::runtime_error("separator tree too deep");
    std::vector<uint64_t> tree;
    std::vector<uint8_t> tree_len;
    uint64_t level_off[kMaxTreeLevels] = {0};
    for (size_t k = 0; k < lv.size(); ++k) {
        level_off[k] = tree_len.size();  // in entries
        tree.insert(tree.end(), lv[k].begin(), lv[k].end());
        tree_len.insert(tree_len.end(), lvlen[k].begin(), lvlen[k].end());
    }

    upload(d.head, head.data(), head.size(), s, "head");
    upload(d.okey, okey.data(), okey.size() * 8, s, "okey");
    upload(d.slot, slot.data(), slot.size() * sizeof(SlotInfo), s, "slot");
    upload(d.tree, tree.data(), tree.size() * 8, s, "tree");
    upload(d.tree_len, tree_len.data(), tree_len.size(), s, "tree_len");
    sync_headers(h, d, s);
    sync_heap(h, d, s);
    hip_check(hipStreamSynchronize(s), "sync");

    DevTable &v = d.view;
    v.head = (const uint8_t *)d.head.p;
    v.okey = (const uint64_t *)d.okey.p;
    v.slot = (const SlotInfo *)d.slot.p;
    v.tree = (const uint64_t *)d.tree.p;
    v.tree_len = (const uint8_t *)d.tree_len.p;
    v.heap = (const uint8_t *)d.heap.p;
    v.chdr = (const CopyHdr *)d.chdr.p;
    v.vhdr = (const VersionHdr *)d.vhdr.p;
    for (int k = 0; k < kMaxTreeLevels; ++k) v.level_off[k] = level_off[k];
    v.levels = (uint32_t)lv.size();
    v.nleaves = (uint32_t)L;
    v.nseps = (uint32_t)S;
    v.cap = cap;
    v.stride = h.stride();
    v.hstride = h.hstride();
    v.head_bytes = hb;
    v.payload_size = p.payload_size;
    v.key_width = p.key_width;
    v.key_words = kw;
    h.layout_dirty_ = false;
    h.structure_dirty_ = false;
    h.dirty_slots_.clear();
    d.valid = true;
    d.last_sync_incremental = false;
    d.last_patch_leaves = d.last_patch_slots = 0;
    d.last_sync_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace stage
