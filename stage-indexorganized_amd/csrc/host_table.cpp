// host_table.cpp -- reference-exact leaf layout, built in structure-of-arrays form.
//
// Leaf contents, slot order, sorted_count and RecordMetadata words follow the reference's
// single-loader write path:
//   LeafNode::Insert       src/vstore/b_tree.cpp:809-947   (append in slot order, offsets
//                                                            grow down from leaf_node_size)
//   BTree::Insert          src/vstore/b_tree.cpp:1849-2020 (split on NotEnoughSpace, retry)
//   LeafNode::PrepareForSplit / CopyFrom  b_tree.cpp:1558-1690, 1486-1545
//   FinalizeForInsert      include/vstore/record_meta.h:128-137
// The inner levels are not materialised: a leaf's key range is (previous separator,
// own separator], which is exactly what InternalNode::GetChildIndex resolves to
// (b_tree.cpp:664-702: an equal key goes to the left child with le_child, right without).
#include "host_table.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace stage {

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void gen_payload(uint64_t rowid, int mode, uint8_t *dst, uint32_t payload_size) {
    if (mode == 0) {  // memset(tuple.cols[i], rowid, ...)  (ycsb_loader.cpp:149-150)
        std::memset(dst, (int)(rowid & 0xFF), payload_size);
        return;
    }
    for (uint32_t j = 0; j * 8 < payload_size; j++) {
        uint64_t w = splitmix64((rowid << 8) ^ j);
        uint32_t nb = std::min<uint32_t>(8, payload_size - j * 8);
        std::memcpy(dst + j * 8, &w, nb);
    }
}

static uint64_t key_mask(uint32_t len) { return len >= 8 ? ~0ull : ((1ull << (8 * len)) - 1); }

Key make_key(const uint8_t *bytes, uint32_t len, bool uns) {
    Key k = key_zero();
    k.len = len;
    for (uint32_t j = 0; j < (uint32_t)kMaxKeyWords && 8 * j < len; ++j) {
        const uint32_t nb = std::min<uint32_t>(8, len - 8 * j);
        uint64_t w = 0;
        std::memcpy(&w, bytes + 8 * j, nb);
        k.w[j] = order_word(w, len, j, uns);
    }
    return k;
}

void key_to_bytes(const Key &k, uint8_t *out, bool uns) {
    for (uint32_t j = 0; 8 * j < k.len; ++j) {
        const uint32_t nb = std::min<uint32_t>(8, k.len - 8 * j);
        const uint64_t w = uns ? bswap64(k.w[j]) : key_bytes_from_order(k.w[j], nb);
        std::memcpy(out + 8 * j, &w, nb);
    }
}

HostTable::HostTable(const stage_params &p) : p_(p) {
    if (p.payload_size == 0 || p.leaf_node_size < 256 || p.key_width > kMaxKeyBytes)
        throw std::invalid_argument("bad table parameters");
    kw_ = table_key_words(p.key_width);
    uns_ = key_order_unsigned(p.key_width);
    kpad_ = p.key_width > 8 ? pad8(p.key_width) : 8u;  // keys of <= 8 bytes pad to 8
    const uint32_t rec = kpad_ + p.payload_size;
    // largest record count c with 40 + c*(24+rec) < leaf_node_size (the Insert space check)
    const uint32_t room = p.leaf_node_size - 40;
    max_records_ = (room + (24 + rec) - 1) / (24 + rec) - 1;
    if (max_records_ < 3) throw std::invalid_argument("leaf holds fewer than 3 records");
    // slots per device leaf: 64 * a power of two (the kernels' slot groups); variable-length
    // keys up to 128, fixed-width keys (small TPC-C / CH rows) up to 1024
    cap_ = 64;
    while (cap_ < max_records_) cap_ *= 2;
    if (cap_ > (p.key_width == 0 ? 128u : 1024u))
        throw std::invalid_argument("too many records per leaf for the device layout (payload too small)");
    // output/heap row: [key padded to 8][payload], 16-B multiple; rows above 128 B are
    // 128-B multiples so every row starts on an L2 line (a 1008-B tuple = 8 whole lines)
    stride_ = (kpad_ + p.payload_size + 15) & ~15u;
    if (stride_ > 128) stride_ = (stride_ + 127) & ~127u;
    buckets_.resize(1u << 16);
    uint32_t root = alloc_leaf();
    head_ = (int32_t)root;
    for (auto &b : buckets_) b.push_back(RouteEntry{key_inf(), root});
}

bool HostTable::key_ok(uint32_t len) const {
    if (len == 0 || len > kMaxKeyBytes) return false;
    if (p_.key_width) return len == p_.key_width;
    return len <= 8;  // variable-length tables hold keys of 1..8 bytes
}

uint32_t HostTable::alloc_leaf() {
    uint32_t id;
    if (!free_leaves_.empty()) {
        id = free_leaves_.back();
        free_leaves_.pop_back();
        leaves_[id] = Leaf();
    } else {
        id = (uint32_t)leaves_.size();
        leaves_.emplace_back();
        size_t n = (size_t)leaves_.size() * cap_;
        okey_.resize(n * kw_, 0);
        meta_.resize(n, 0);
        next_.resize(n, 0);
        image_.resize(n, 0);
        loc_.resize(n, 0);
    }
    size_t b = (size_t)id * cap_;
    std::fill(okey_.begin() + b * kw_, okey_.begin() + (b + cap_) * kw_, 0);
    std::fill(meta_.begin() + b, meta_.begin() + b + cap_, 0);
    std::fill(next_.begin() + b, next_.begin() + b + cap_, 0);
    std::fill(image_.begin() + b, image_.begin() + b + cap_, 0);
    std::fill(loc_.begin() + b, loc_.begin() + b + cap_, 0);
    leaves_[id].live = true;
    nleaves_live_++;
    return id;
}

uint32_t HostTable::route(const Key &k, bool le_child) const {
    for (uint32_t b = bucket_of(k); b < buckets_.size(); ++b) {
        const auto &v = buckets_[b];
        auto it = le_child ? std::lower_bound(v.begin(), v.end(), k, entry_lt_key)
                           : std::upper_bound(v.begin(), v.end(), k,
                                              [](const Key &kk, const RouteEntry &e) { return key_lt(kk, e.sep); });
        if (it != v.end()) return it->leaf;
    }
    return buckets_.back().back().leaf;  // the +inf leaf
}

// First visible slot holding k.  Equivalent to BaseNode::SearchRecordMeta with
// check_concurrency (b_tree.cpp:61-121): the sorted pass and the unsorted pass both accept
// only visible slots whose key bytes and key size equal the probe, first in slot order.
int64_t HostTable::search(uint32_t leaf, const Key &k) const {
    const Leaf &L = leaves_[leaf];
    const size_t b = (size_t)leaf * cap_;
    const uint64_t *ok = okey_.data() + b * kw_;
    for (uint32_t s = 0; s < L.count; ++s) {
        const uint64_t *w = ok + (size_t)s * kw_;
        if (w[0] != k.w[0]) continue;
        bool eq = true;
        for (uint32_t j = 1; j < kw_; ++j) eq &= w[j] == k.w[j];
        if (!eq) continue;
        uint64_t m = meta_[b + s];
        if (meta_visible(m) && meta_keylen(m) == k.len) return s;
    }
    return -1;
}

uint32_t HostTable::new_image(const uint8_t *key, uint32_t len, const uint8_t *payload, uint64_t gen_rowid,
                              int mode) {
    ImageDesc d;
    d.key_le = 0;
    d.mode = (uint32_t)mode;
    if (len > 8) {  // wide key: the arena holds the whole row [key padded][payload]
        if (!payload) throw std::invalid_argument("keys above 8 bytes need an explicit payload");
        d.kind = 2;
        d.arg = arena_.alloc(kpad_ + p_.payload_size);
        uint8_t *row = arena_.at(d.arg);
        std::memset(row, 0, kpad_);
        std::memcpy(row, key, len);
        std::memcpy(row + kpad_, payload, p_.payload_size);
    } else {
        std::memcpy(&d.key_le, key, len);
        if (payload) {
            d.kind = 1;
            d.arg = arena_.alloc(p_.payload_size);
            std::memcpy(arena_.at(d.arg), payload, p_.payload_size);
        } else {
            d.kind = 0;
            d.arg = gen_rowid;
        }
    }
    images_.push_back(d);
    if (images_.size() > kNextIndexMask) throw std::runtime_error("record heap index overflow");
    return (uint32_t)(images_.size() - 1);
}

void HostTable::image_payload(uint32_t img, uint8_t *dst) const {
    const ImageDesc &d = images_[img];
    if (d.kind == 0) gen_payload(d.arg, (int)d.mode, dst, p_.payload_size);
    else if (d.kind == 1) std::memcpy(dst, arena_.at(d.arg), p_.payload_size);
    else if (d.kind == 2) std::memcpy(dst, arena_.at(d.arg) + kpad_, p_.payload_size);
    else throw std::logic_error("device-written heap row read before materialize_device_rows");
}

void HostTable::reserve_adoption(uint64_t add) {
    auto room = [](auto &v, uint64_t k) {
        if (v.capacity() < v.size() + k) v.reserve(std::max<uint64_t>(v.size() + k, 2 * v.capacity()));
    };
    room(copies_, add);
    room(copy_live_, add);
    room(versions_, add);
    std::lock_guard<std::mutex> g(ssn_.mu);
    room(ssn_.e, add);
}

void HostTable::adopt_device_epoch(const CopyHdr *copies, const uint32_t *writers, uint64_t nc,
                                   const VersionHdr *versions, uint64_t nv, uint64_t nimages, const SlotWords *slots,
                                   uint64_t nslots) {
    if (copies_.size() + nc > kNextIndexMask || versions_.size() + nv > kNextIndexMask ||
        images_.size() + nimages > kNextIndexMask)
        throw std::runtime_error("copy / version / image index overflow");
    const bool trace = std::getenv("STAGE_WP_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (trace)
            std::fprintf(stderr, "[adopt] %s %.2f ms\n", what,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    // grow 4x (at least 4M entries) instead of doubling: each epoch appends ~n headers, and a
    // reallocation copies (and page-faults in) every earlier one
    auto room = [](auto &v, uint64_t add) {
        if (v.capacity() < v.size() + add) v.reserve(std::max<uint64_t>(v.size() + add, 4 * v.capacity() + (1u << 22)));
    };
    room(copies_, nc);
    room(copy_live_, nc);
    room(versions_, nv);
    const uint64_t c0 = copies_.size(), v0 = versions_.size();
    copies_.resize(c0 + nc);  // uninitialised (HugeAllocNoInit): filled below, in parallel
    versions_.resize(v0 + nv);
    copy_live_.resize(copies_.size(), 1);
    parallel_chunks(std::max(nc, nv), [&](uint64_t b, uint64_t e) {
        if (b < nc) std::memcpy(copies_.data() + c0 + b, copies + b, (std::min(e, nc) - b) * sizeof(CopyHdr));
        if (b < nv) std::memcpy(versions_.data() + v0 + b, versions + b, (std::min(e, nv) - b) * sizeof(VersionHdr));
    });
    {
        std::lock_guard<std::mutex> g(ssn_.mu);
        room(ssn_.e, nc);  // not reserve(c0 + nc): an exact reserve reallocates every epoch
        // the epoch's copies are c0 .. c0 + nc - 1: their SSN state goes at the same ids
        if (ssn_.e.size() > c0) throw std::runtime_error("adopt_device_epoch: SSN state ahead of the copies");
        ssn_.e.resize(c0 + nc);  // uninitialised (HugeAllocNoInit): every entry is written below, in parallel
        CopySsn *dst = ssn_.e.data() + c0;
        parallel_chunks(nc, [&](uint64_t b, uint64_t e) {
            for (uint64_t k = b; k < e; ++k) {
                const uint32_t w = writers ? writers[k] : 0;
                dst[k] = CopySsn{w, w, copies[k].rstamp, copies[k].sstamp, 0, (uint8_t)(copies[k].sstamp != kMaxCid), 0};
            }
        });
    }
    lap("headers");
    if (nimages) {
        device_rows_.emplace_back(images_.size(), nimages);
        const uint64_t i0 = images_.size();
        images_.resize(i0 + nimages);
        parallel_chunks(nimages, [&](uint64_t b, uint64_t e) {
            for (uint64_t k = b; k < e; ++k) images_[i0 + k] = ImageDesc{0, 0, 3, 0};
        });
    }
    lap("images");
    // one slot word per touched record (distinct indices): scattered writes in parallel, after a
    // parallel bounds check of every index
    std::atomic<bool> bad{false};
    const uint64_t nmeta = meta_.size();
    parallel_chunks(nslots, [&](uint64_t b, uint64_t e) {
        for (uint64_t k = b; k < e; ++k)
            if (slots[k].idx != ~0ull && slots[k].idx >= nmeta) bad.store(true, std::memory_order_relaxed);
    });
    if (bad.load()) throw std::runtime_error("adopt_device_epoch: slot index outside the table");
    parallel_chunks(nslots, [&](uint64_t b, uint64_t e) {
        for (uint64_t k = b; k < e; ++k) {
            const SlotWords &w = slots[k];
            if (w.idx == ~0ull) continue;
            meta_[w.idx] = w.meta;
            next_[w.idx] = w.next;
            image_[w.idx] = w.image;
            cell(w.idx);
        }
    });
    lap("slots");
    // the device already holds all of it
    copies_synced_ = copies_.size();
    versions_synced_ = versions_.size();
    images_synced_ = images_.size();
}

LocCells::~LocCells() {
    for (auto &d : dir_) delete[] d.load();
}

void LocCells::ensure(uint64_t handle) {
    const uint64_t k = handle >> kChunkBits;
    if (k >= kDir) throw std::runtime_error("location cell directory exhausted");
    if (dir_[k].load(std::memory_order_acquire)) return;
    Cell *c = new Cell[1u << kChunkBits];
    for (uint32_t i = 0; i < (1u << kChunkBits); ++i) {
        c[i].meta.store(0, std::memory_order_relaxed);
        c[i].next.store(0, std::memory_order_relaxed);
        c[i].loc.store(((uint64_t)k << kChunkBits) + i, std::memory_order_relaxed);
    }
    Cell *expect = nullptr;
    if (!dir_[k].compare_exchange_strong(expect, c, std::memory_order_acq_rel)) delete[] c;  // another thread won
}

void CopySsnTable::created(uint64_t id, uint32_t writer, uint32_t rstamp) {
    std::lock_guard<std::mutex> g(mu);
    if (e.size() <= id) e.resize(id + 1, CopySsn{0, 0, 0, kMaxCid, 0, 0, 0});
    e[id] = CopySsn{writer, writer, rstamp, kMaxCid, 0, 0, 0};
}

void CopySsnTable::committed(uint64_t id, uint32_t sstamp) {
    std::lock_guard<std::mutex> g(mu);
    if (id < e.size()) e[id].sstamp = sstamp, e[id].waiting = 1;
}

void CopySsnTable::aborted(uint64_t id) {
    std::lock_guard<std::mutex> g(mu);
    if (id < e.size()) e[id].sstamp = kMaxCid, e[id].waiting = 1;
}

// builds every cell from the current layout; afterwards each write keeps them current
void HostTable::enable_cells() {
    if (cells_.on()) return;
    if (!locpos_.empty()) cells_.ensure(locpos_.size());
    for (uint64_t h = 1; h <= locpos_.size(); h += 1u << LocCells::kChunkBits) cells_.ensure(h);
    cells_.enable();
    for (uint32_t l = 0; l < leaves_.size(); ++l) {
        if (!leaves_[l].live) continue;
        for (uint32_t s = 0; s < leaves_[l].count; ++s) cell((size_t)l * cap_ + s);
    }
}

void HostTable::parallel_chunks(uint64_t n, const std::function<void(uint64_t, uint64_t)> &fn) {
    const unsigned nt = n < 65536 ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (nt == 1) {
        if (n) fn(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back([&, t] { fn(n * t / nt, n * (t + 1) / nt); });
    for (auto &x : th) x.join();
}

void HostTable::materialize_device_rows(const std::function<void(uint64_t, uint64_t, uint8_t *)> &fetch) {
    const uint64_t row = kpad_ + p_.payload_size, chunk = 1u << 14;
    std::vector<uint8_t> buf(chunk * stride_);
    for (const auto &r : device_rows_) {
        for (uint64_t b = 0; b < r.second; b += chunk) {
            const uint64_t cnt = std::min(chunk, r.second - b);
            fetch(r.first + b, cnt, buf.data());
            for (uint64_t k = 0; k < cnt; ++k) {
                const uint8_t *src = buf.data() + k * stride_;
                ImageDesc &d = images_[r.first + b + k];
                d.mode = 0;
                if (kw_ > 1) {  // wide keys: the whole row
                    d.kind = 2;
                    d.key_le = 0;
                    d.arg = arena_.alloc(row);
                    std::memcpy(arena_.at(d.arg), src, row);
                } else {        // key word + payload
                    d.kind = 1;
                    std::memcpy(&d.key_le, src, 8);
                    d.arg = arena_.alloc(p_.payload_size);
                    std::memcpy(arena_.at(d.arg), src + 8, p_.payload_size);
                }
            }
        }
    }
    device_rows_.clear();
}

int HostTable::insert(const uint8_t *key, uint32_t len, const uint8_t *payload, uint64_t gen_rowid, int mode,
                      uint32_t commit_id, bool inflight) {
    if (!key_ok(len)) return STAGE_RC_INVALID;
    const Key k = make_key(key, len, uns_);
    const uint32_t rec = (len > 8 ? pad8(len) : 8u) + p_.payload_size;
    for (int guard = 0; guard < 64; ++guard) {
        uint32_t leaf = route(k, true);
        const uint64_t lid = locpos_.size();  // RecordIndirectLocation, every attempt (b_tree.cpp:1865-1866)
        if (lid >= 0xFFFFFFFFull) throw std::runtime_error("location index overflow");
        locpos_.push_back(kNoPos);
        int64_t hit = search(leaf, k);  // CheckUnique (b_tree.cpp:1395-1417)
        if (hit >= 0) {
            if (meta_inserting(meta_[(size_t)leaf * cap_ + hit])) return STAGE_RC_INVALID;  // ReCheck path
            return STAGE_RC_KEY_EXISTS;
        }
        Leaf &L = leaves_[leaf];
        if (used_space(L) + 24u + rec >= p_.leaf_node_size) {  // NotEnoughSpace (b_tree.cpp:829-836)
            if (!split(leaf)) return STAGE_RC_RETRY_FAILURE;
            continue;
        }
        const uint32_t slot = L.count++;
        L.block += rec;
        const uint64_t offset = p_.leaf_node_size - L.block;
        const size_t i = (size_t)leaf * cap_ + slot;
        set_slot_key(i, k);
        // PrepareForInsert (b_tree.cpp:860-864), then -- unless the inserting transaction is
        // still in flight -- FinalizeInsert: control bit cleared, cstamp = commit_id
        meta_[i] = ((uint64_t)len << 48) | kMetaVisible | (offset << 32) | commit_id | (inflight ? kMetaControl : 0);
        next_[i] = 0;
        image_[i] = new_image(key, len, payload, gen_rowid, mode);
        loc_[i] = (uint32_t)(lid + 1);
        locpos_[lid] = (uint64_t)leaf << 16 | slot;
        if (cells_.on()) {
            cells_.ensure(lid + 1);
            cell(i);
        }
        touch(leaf, slot);
        return STAGE_RC_OK;
    }
    return STAGE_RC_RETRY_FAILURE;
}

bool HostTable::split(uint32_t p) {
    if (leaves_[p].count < 3) return false;
    struct Rec {
        Key key;
        uint64_t meta;
        uint32_t next, image, loc;
    };
    const size_t pb = (size_t)p * cap_;
    std::vector<Rec> v;
    v.reserve(leaves_[p].count);
    uint32_t total = 0;
    for (uint32_t s = 0; s < leaves_[p].count; ++s) {
        uint64_t m = meta_[pb + s];
        if (m != 0 && meta_visible(m) && meta_keylen(m) > 0) {
            v.push_back(Rec{slot_key(pb + s), m, next_[pb + s], image_[pb + s], loc_[pb + s]});
            total += pad8(meta_keylen(m)) + p_.payload_size;
        }
    }
    if (total == 0) return false;
    for (uint32_t s = 0; s < leaves_[p].count; ++s) {  // CopyFrom drops these: their locations dangle
        const uint64_t m = meta_[pb + s];
        if (!(m != 0 && meta_visible(m) && meta_keylen(m) > 0) && loc_[pb + s]) {
            locpos_[loc_[pb + s] - 1] = kNoPos;
            cell_drop(loc_[pb + s]);
        }
    }
    std::sort(v.begin(), v.end(), [](const Rec &a, const Rec &b) { return key_lt(a.key, b.key); });
    int32_t left_size = (int32_t)(total / 2);
    uint32_t nleft = 0;
    for (size_t i = 0; i < v.size(); ++i) {
        ++nleft;
        left_size -= (int32_t)(pad8(meta_keylen(v[i].meta)) + p_.payload_size);
        if (left_size <= 0) break;
    }
    const Key sep = v[nleft - 1].key;
    const Key hi = leaves_[p].sep;
    const Key lo = leaves_[p].prev >= 0 ? leaves_[leaves_[p].prev].sep : key_zero();

    const uint32_t r = alloc_leaf();  // may reallocate the arrays
    auto fill = [&](uint32_t leaf, size_t from, size_t to) {
        Leaf &L = leaves_[leaf];
        const size_t b = (size_t)leaf * cap_;
        uint32_t offset = p_.leaf_node_size, n = 0;
        for (size_t i = from; i < to; ++i) {
            const uint32_t kl = meta_keylen(v[i].meta);
            offset -= pad8(kl) + p_.payload_size;
            set_slot_key(b + n, v[i].key);
            meta_[b + n] = ((uint64_t)kl << 48) | kMetaVisible | ((uint64_t)offset << 32) | meta_cstamp(v[i].meta);
            next_[b + n] = v[i].next;
            image_[b + n] = v[i].image;
            loc_[b + n] = v[i].loc;
            if (v[i].loc) locpos_[v[i].loc - 1] = (uint64_t)leaf << 16 | n;  // loc->record_meta_ptr
            cell(b + n);
            ++n;
        }
        for (uint32_t s = n; s < cap_; ++s) {
            clear_slot_key(b + s);
            meta_[b + s] = 0;
            next_[b + s] = 0;
            image_[b + s] = 0;
            loc_[b + s] = 0;
        }
        L.count = L.sorted = n;
        L.block = p_.leaf_node_size - offset;
        L.deleted = 0;
    };
    fill(p, 0, nleft);
    fill(r, nleft, v.size());
    Leaf &P = leaves_[p];
    Leaf &R = leaves_[r];
    R.sep = hi;
    P.sep = sep;
    R.prev = (int32_t)p;
    R.next = P.next;
    if (P.next >= 0) leaves_[P.next].prev = (int32_t)r;
    P.next = (int32_t)r;
    route_split(p, r, lo, sep, hi);
    layout_dirty_ = true;
    structure_dirty_ = true;
    dirty_slots_.clear();
    return true;
}

void HostTable::route_split(uint32_t p, uint32_t r, const Key &lo, const Key &s, const Key &hi) {
    const uint32_t b_lo = bucket_of(lo);
    const uint32_t b_hi = key_is_inf(hi) ? (uint32_t)buckets_.size() - 1 : bucket_of(hi);
    const uint32_t b_s = bucket_of(s);
    for (uint32_t b = b_lo; b <= b_hi; ++b) {
        auto &v = buckets_[b];
        auto it = std::lower_bound(v.begin(), v.end(), hi, entry_lt_key);
        while (it != v.end() && it->leaf != p) ++it;
        if (it == v.end()) continue;  // p does not reach this bucket
        if (b < b_s) {
            it->sep = s;
        } else if (b > b_s) {
            it->leaf = r;
        } else {
            it->leaf = r;
            v.insert(it, RouteEntry{s, p});
        }
    }
}

uint64_t HostTable::load_ycsb(uint64_t begin, uint64_t end, uint32_t key_size, int mode) {
    if (key_size > 8) return 0;
    if (end > begin) {
        images_.reserve(images_.size() + (end - begin));
        locpos_.reserve(locpos_.size() + (end - begin) + (end - begin) / 32);
    }
    uint64_t ok = 0;
    for (uint64_t rowid = begin; rowid < end; ++rowid)
        if (insert(rowid & key_mask(key_size), key_size, nullptr, rowid, mode, kInvalidCid) == STAGE_RC_OK) ++ok;
    return ok;
}

uint64_t HostTable::load_keys(const uint64_t *keys, uint64_t n, uint32_t key_size, int mode) {
    if (key_size > 8) return 0;
    images_.reserve(images_.size() + n);
    uint64_t ok = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (insert(keys[i] & key_mask(key_size), key_size, nullptr, keys[i], mode, kInvalidCid) == STAGE_RC_OK) ++ok;
    return ok;
}

uint64_t HostTable::load_rows(const uint8_t *keys, uint32_t key_stride, uint32_t key_size, const uint8_t *payloads,
                              uint32_t payload_stride, uint64_t n, uint32_t commit_id, uint8_t *rc_out) {
    images_.reserve(images_.size() + n);
    uint64_t ok = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const int rc = insert(keys + i * (uint64_t)key_stride, key_size, payloads + i * (uint64_t)payload_stride, 0, 0,
                              commit_id);
        if (rc == STAGE_RC_OK) ++ok;
        if (rc_out) rc_out[i] = (uint8_t)rc;
    }
    return ok;
}

int HostTable::find(const uint8_t *key, uint32_t len, uint32_t *leaf, uint32_t *slot) const {
    if (!key_ok(len)) return -1;
    const Key k = make_key(key, len, uns_);
    uint32_t lf = route(k, true);
    int64_t s = search(lf, k);
    if (s < 0) return -1;
    *leaf = lf;
    *slot = (uint32_t)s;
    return 0;
}

// LeafNode::Update, b_tree.cpp:1061-1163 (is_for_update == false): the old image becomes the
// overwrite copy (its image row is immutable), the record gets a new patched image.
int HostTable::update(const uint8_t *key, uint32_t len, uint32_t payload_off, const uint8_t *delta,
                      uint32_t delta_len, uint32_t writer_id) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    const uint64_t m = meta_[i];
    if (meta_inserting(m)) return STAGE_RC_DIRTY;
    if ((uint64_t)payload_off + delta_len > p_.payload_size) return STAGE_RC_INVALID;
    std::vector<uint8_t> pay(p_.payload_size);
    image_payload(image_[i], pay.data());
    if (std::memcmp(pay.data() + payload_off, delta, delta_len) == 0) return STAGE_RC_NOT_NEEDED_UPDATE;
    if (meta_cstamp(m) > writer_id) return STAGE_RC_NOT_NEEDED_UPDATE;
    meta_[i] = m | kMetaControl | kMetaVisible;  // PrepareForUpdate
    CopyHdr c;
    c.rstamp = meta_cstamp(m);
    c.sstamp = kMaxCid;
    c.next = next_[i];
    c.image = image_[i];
    copies_.push_back(c);
    copy_live_.push_back(1);
    if (copies_.size() > kNextIndexMask) throw std::runtime_error("copy index overflow");
    next_[i] = kNextCopy | (uint32_t)(copies_.size() - 1);
    ssn_.created(copies_.size() - 1, writer_id, c.rstamp);
    std::memcpy(pay.data() + payload_off, delta, delta_len);  // CopyPayload
    image_[i] = new_image(key, len, pay.data(), 0, 0);
    cell(i);
    touch(leaf, slot);
    return STAGE_RC_OK;
}

// LeafNode::Update with is_for_update = true (b_tree.cpp:1061-1163): the transaction updates a
// record it owns (its own in-flight update or insert, or a record it locked for update): no Dirty
// check (:1077), the same ComparePayload / newer-writer NotNeededUpdate checks (:1086-1100), and
// CopyPayload in place -- no overwrite copy, no PrepareForUpdate (:1101-1104).  The record gets
// a new image row (rows are immutable); its meta word, next handle and any copy stay.
int HostTable::update_owned(const uint8_t *key, uint32_t len, uint32_t payload_off, const uint8_t *delta,
                            uint32_t delta_len, uint32_t writer_id) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    const uint64_t m = meta_[i];
    if ((uint64_t)payload_off + delta_len > p_.payload_size) return STAGE_RC_INVALID;
    std::vector<uint8_t> pay(p_.payload_size);
    image_payload(image_[i], pay.data());
    if (std::memcmp(pay.data() + payload_off, delta, delta_len) == 0) return STAGE_RC_NOT_NEEDED_UPDATE;
    if (meta_cstamp(m) > writer_id) return STAGE_RC_NOT_NEEDED_UPDATE;
    std::memcpy(pay.data() + payload_off, delta, delta_len);  // CopyPayload
    image_[i] = new_image(key, len, pay.data(), 0, 0);
    touch(leaf, slot);
    return STAGE_RC_OK;
}

// LeafNode::Delete with is_for_update = true (b_tree.cpp:1171-1251): the record's meta word is
// cleared (vacant; the reference's copy allocation at :1195-1203 is reachable from nothing), no
// deleted-size accounting (PointDeleteExecutor skips PerformDelete, so no FinalizeDelete runs).
// BTree::Delete's merge check then sees the leaf's unchanged live size (RC_INVALID as remove()).
int HostTable::remove_owned(const uint8_t *key, uint32_t len) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    meta_[i] = 0;
    cell(i);
    Leaf &L = leaves_[leaf];
    touch(leaf, slot);
    if (nleaves_live_ > 1 && used_space(L) - L.deleted <= p_.merge_threshold) return STAGE_RC_INVALID;
    return STAGE_RC_OK;
}

// CommitTransaction UPDATE entry (transaction_manager.cpp:610-676), single writer.
int HostTable::commit_update(const uint8_t *key, uint32_t len, uint32_t commit_id, uint32_t sstamp) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    if (!meta_inserting(meta_[i]) || (next_[i] & kNextKindMask) != kNextCopy) return STAGE_RC_NOT_FOUND;
    const uint64_t ci = next_[i] & kNextIndexMask;
    CopyHdr &c = copies_[ci];
    c.sstamp = sstamp;
    if (ci < copies_dirty_from_) copies_dirty_from_ = ci;
    VersionHdr v;
    v.begin_id = c.rstamp;
    v.comm_id = c.sstamp;
    v.next = c.next;
    v.image = c.image;
    versions_.push_back(v);
    if (versions_.size() > kNextIndexMask) throw std::runtime_error("version index overflow");
    uint64_t m = (meta_[i] & ~kMetaTxn) | commit_id;  // FinalizeForUpdate(t_cstamp)
    meta_[i] = m & ~kMetaControl;
    next_[i] = kNextVersion | (uint32_t)(versions_.size() - 1);
    ssn_.committed(ci, sstamp);
    cell(i);
    touch(leaf, slot);
    return STAGE_RC_OK;
}

// AbortTransaction UPDATE entry (transaction_manager.cpp:846-921): the record gets its old
// image back (the overwrite copy's immutable heap row), FinalizeForUpdate() clears the control
// bit (cstamp untouched), next := the chain the update found; the copy is released.
int HostTable::abort_update(const uint8_t *key, uint32_t len) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    if (!meta_inserting(meta_[i]) || (next_[i] & kNextKindMask) != kNextCopy) return STAGE_RC_NOT_FOUND;
    const uint64_t ci = next_[i] & kNextIndexMask;
    image_[i] = copies_[ci].image;
    next_[i] = copies_[ci].next;
    meta_[i] = (meta_[i] & ~kMetaControl) | kMetaVisible;
    copy_live_[ci] = 0;
    ssn_.aborted(ci);
    cell(i);
    touch(leaf, slot);
    return STAGE_RC_OK;
}

// AbortTransaction INSERT entry (transaction_manager.cpp:949-979): FinalizeForDelete (meta 0)
// and StatusWord::FailForInsert (count - 1, block - record size, version_store.h:214-217).
// FailForInsert drops the leaf's last slot, so the aborted insert must be that slot.
int HostTable::abort_insert(const uint8_t *key, uint32_t len) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    Leaf &L = leaves_[leaf];
    if (slot + 1 != L.count || slot < L.sorted) return STAGE_RC_INVALID;
    const size_t i = (size_t)leaf * cap_ + slot;
    L.block -= pad8(meta_keylen(meta_[i])) + p_.payload_size;
    L.count -= 1;
    meta_[i] = 0;
    next_[i] = 0;
    image_[i] = 0;
    if (loc_[i]) locpos_[loc_[i] - 1] = kNoPos;
    cell_drop(loc_[i]);
    loc_[i] = 0;
    clear_slot_key(i);
    touch(leaf, slot);
    return STAGE_RC_OK;
}

// CommitTransaction INSERT entry (transaction_manager.cpp:677-695): FinalizeForInsert(offset,
// key_len, t_cstamp) on a record an in-flight insert left PrepareForInsert.
int HostTable::commit_insert(const uint8_t *key, uint32_t len, uint32_t commit_id) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    if (!meta_inserting(meta_[i]) || next_[i] != 0) return STAGE_RC_NOT_FOUND;
    meta_[i] = ((meta_[i] & ~kMetaTxn) | commit_id | kMetaVisible) & ~kMetaControl;
    cell(i);
    touch(leaf, slot);
    return STAGE_RC_OK;
}

// BTree::FinalizeUpdate (b_tree.cpp:2252-2268): cstamp := commit_id, next untouched.
int HostTable::finalize_update(const uint8_t *key, uint32_t len, uint32_t commit_id) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    meta_[i] = ((meta_[i] & ~kMetaTxn) | commit_id) & ~kMetaControl;
    cell(i);
    touch(leaf, slot);
    return STAGE_RC_OK;
}

// LeafNode::Delete (b_tree.cpp:1171-1251) + FinalizeDelete (b_tree.cpp:2275-2310).  Sibling
// merges (BaseNode::CheckMerge) are not supported: such a delete reports RC_INVALID.
int HostTable::remove(const uint8_t *key, uint32_t len, uint32_t commit_id) {
    uint32_t leaf, slot;
    if (find(key, len, &leaf, &slot) < 0) return STAGE_RC_NOT_FOUND;
    const size_t i = (size_t)leaf * cap_ + slot;
    const uint64_t m = meta_[i];
    if (meta_inserting(m)) return STAGE_RC_DIRTY;
    CopyHdr c;
    c.rstamp = meta_cstamp(m);
    c.sstamp = kMaxCid;
    c.next = next_[i];
    c.image = image_[i];
    copies_.push_back(c);
    copy_live_.push_back(1);
    next_[i] = kNextCopy | (uint32_t)(copies_.size() - 1);
    ssn_.created(copies_.size() - 1, commit_id, c.rstamp);
    meta_[i] = 0;
    cell(i);
    Leaf &L = leaves_[leaf];
    L.deleted += pad8(meta_keylen(m)) + p_.payload_size;
    touch(leaf, slot);
    (void)commit_id;
    if (nleaves_live_ > 1 && used_space(L) - L.deleted <= p_.merge_threshold) return STAGE_RC_INVALID;
    return STAGE_RC_OK;
}

// Batched epoch writes.  Small batches run the per-key path.  Large ones run in parallel:
// (A) locate every key (read-only: updates never move records), (B) group the operations by
// slot (an update of a key followed by another of the same key stays in batch order), (C)
// process slot groups on worker threads, each appending its overwrite copies, versions and
// images to thread-local buffers with references tagged "local", then (D) concatenate the
// buffers in thread order and relocate the tagged references.  The result is the per-key
// path's layout up to the order in which new copies / versions / images are numbered.
namespace {
constexpr uint32_t kLocalRef = 1u << 29;   // local copy / version index inside a tagged next handle
constexpr uint32_t kLocalImg = 1u << 31;   // local image index
struct LocalWrites {
    std::vector<CopyHdr> copies;
    std::vector<uint32_t> writers;  // writer id per copy
    std::vector<VersionHdr> versions;
    std::vector<ImageDesc> images;
    std::vector<uint8_t> arena;
    std::vector<uint64_t> touched;  // host slot indices written
    uint64_t copies_dirty_from = ~0ull;
    uint64_t ok = 0;
};
uint32_t reloc_next(uint32_t nx, uint64_t cbase, uint64_t vbase) {
    if (!(nx & kLocalRef) || (nx & kNextKindMask) == 0) return nx;
    const uint32_t kind = nx & kNextKindMask, idx = nx & (kLocalRef - 1);
    return kind | (uint32_t)(idx + (kind == kNextCopy ? cbase : vbase));
}
uint32_t reloc_img(uint32_t im, uint64_t ibase) { return (im & kLocalImg) ? (uint32_t)((im & ~kLocalImg) + ibase) : im; }
}  // namespace

uint64_t HostTable::update_batch(const uint8_t *keys, uint32_t key_stride, uint64_t n, uint32_t len,
                                 uint32_t payload_off, const uint8_t *deltas, uint32_t delta_len,
                                 const uint32_t *writer_ids, const uint32_t *commit_ids, const uint32_t *sstamps,
                                 uint8_t *rc_out) {
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const bool small = n < 8192 || nt == 1 || copies_.size() + n >= kLocalRef || versions_.size() + n >= kLocalRef ||
                       images_.size() + n >= (1ull << 30);
    if (small) {
        uint64_t ok = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint8_t *k = keys + i * (uint64_t)key_stride;
            int rc = update(k, len, payload_off, deltas + i * (uint64_t)delta_len, delta_len, writer_ids[i]);
            if (rc == STAGE_RC_OK && commit_ids && commit_ids[i])
                rc = commit_update(k, len, commit_ids[i], sstamps ? sstamps[i] : commit_ids[i]);
            if (rc == STAGE_RC_OK) ++ok;
            if (rc_out) rc_out[i] = (uint8_t)rc;
        }
        return ok;
    }
    const bool timing = std::getenv("STAGE_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_0 = now();
    auto lap = [&](const char *what) {
        if (!timing) return;
        const auto t = now();
        std::fprintf(stderr, "[update_batch] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t_0).count());
        t_0 = t;
    };
    auto par = [&](uint64_t count, auto fn) {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&, t] { fn(t, count * t / nt, count * (t + 1) / nt); });
        for (auto &x : th) x.join();
    };
    // (A) locate
    std::vector<uint64_t> loc(n);
    std::vector<uint8_t> rc(n, STAGE_RC_NOT_FOUND);
    const bool bad_range = (uint64_t)payload_off + delta_len > p_.payload_size;
    par(n, [&](unsigned, uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; ++i) {
            uint32_t lf, sl;
            loc[i] = find(keys + i * (uint64_t)key_stride, len, &lf, &sl) < 0 ? ~0ull : (uint64_t)lf * cap_ + sl;
        }
    });
    lap("locate");
    // (B) group by slot, batch order inside a group: bucket by leaf range (one bucket per
    // worker, so a slot group never straddles two workers), then sort each bucket in parallel
    const uint64_t span = (uint64_t)leaves_.size() * cap_;
    std::vector<uint64_t> bcount(nt + 1, 0);
    auto bucket = [&](uint64_t l) { return (unsigned)(l * nt / span); };
    for (uint64_t i = 0; i < n; ++i)
        if (loc[i] != ~0ull) bcount[bucket(loc[i]) + 1]++;
    for (unsigned t = 0; t < nt; ++t) bcount[t + 1] += bcount[t];
    const uint64_t m = bcount[nt];
    std::vector<std::pair<uint64_t, uint32_t>> ord(m);
    {
        std::vector<uint64_t> pos(bcount.begin(), bcount.end() - 1);
        for (uint64_t i = 0; i < n; ++i)
            if (loc[i] != ~0ull) ord[pos[bucket(loc[i])]++] = {loc[i], (uint32_t)i};
    }
    par(nt, [&](unsigned, uint64_t tb, uint64_t te) {
        for (uint64_t t = tb; t < te; ++t) std::sort(ord.begin() + bcount[t], ord.begin() + bcount[t + 1]);
    });
    const std::vector<uint64_t> &cut = bcount;
    lap("group");
    // (C) per-thread processing with local appends
    std::vector<LocalWrites> lw(nt);
    par(nt, [&](unsigned, uint64_t tb, uint64_t te) {
        for (uint64_t t = tb; t < te; ++t) {
            LocalWrites &L = lw[t];
            const uint64_t nops = cut[t + 1] - cut[t];
            L.copies.reserve(nops);
            L.versions.reserve(commit_ids ? nops : 0);
            L.images.reserve(nops);
            L.touched.reserve(nops);
            L.arena.reserve(nops * (uint64_t)(kpad_ + p_.payload_size));
            std::vector<uint8_t> pay(p_.payload_size);
            auto payload_of = [&](uint32_t img, uint8_t *dst) {
                if (img & kLocalImg) {
                    const ImageDesc &d = L.images[img & ~kLocalImg];
                    std::memcpy(dst, L.arena.data() + d.arg + (d.kind == 2 ? kpad_ : 0), p_.payload_size);
                } else {
                    image_payload(img, dst);
                }
            };
            for (uint64_t q = cut[t]; q < cut[t + 1]; ++q) {
                const uint32_t op = ord[q].second;
                const uint64_t i = ord[q].first;
                const uint8_t *key = keys + op * (uint64_t)key_stride;
                const uint8_t *delta = deltas + op * (uint64_t)delta_len;
                const uint64_t mw = meta_[i];
                // LeafNode::Update (b_tree.cpp:1061-1163)
                if (meta_inserting(mw)) { rc[op] = STAGE_RC_DIRTY; continue; }
                if (bad_range) { rc[op] = STAGE_RC_INVALID; continue; }
                payload_of(image_[i], pay.data());
                if (std::memcmp(pay.data() + payload_off, delta, delta_len) == 0 || meta_cstamp(mw) > writer_ids[op]) {
                    rc[op] = STAGE_RC_NOT_NEEDED_UPDATE;
                    continue;
                }
                meta_[i] = mw | kMetaControl | kMetaVisible;
                L.copies.push_back(CopyHdr{meta_cstamp(mw), kMaxCid, next_[i], image_[i]});
                L.writers.push_back(writer_ids[op]);
                next_[i] = kNextCopy | kLocalRef | (uint32_t)(L.copies.size() - 1);
                std::memcpy(pay.data() + payload_off, delta, delta_len);
                ImageDesc d;
                d.key_le = 0;
                d.mode = 0;
                d.arg = L.arena.size();
                if (len > 8) {
                    d.kind = 2;
                    L.arena.resize(L.arena.size() + kpad_ + p_.payload_size, 0);
                    std::memcpy(L.arena.data() + d.arg, key, len);
                    std::memcpy(L.arena.data() + d.arg + kpad_, pay.data(), p_.payload_size);
                } else {
                    d.kind = 1;
                    std::memcpy(&d.key_le, key, len);
                    L.arena.insert(L.arena.end(), pay.begin(), pay.end());
                }
                L.images.push_back(d);
                image_[i] = kLocalImg | (uint32_t)(L.images.size() - 1);
                // once per slot (a slot's ops are consecutive here): the relocation below must
                // run once per slot word -- the small-batch gate keeps global indices below
                // kLocalRef, this keeps it independent of that gate
                if (L.touched.empty() || L.touched.back() != i) L.touched.push_back(i);
                rc[op] = STAGE_RC_OK;
                // CommitTransaction UPDATE entry (transaction_manager.cpp:610-676)
                const uint32_t cid = commit_ids ? commit_ids[op] : 0;
                if (cid) {
                    CopyHdr &c = L.copies.back();
                    c.sstamp = sstamps ? sstamps[op] : cid;
                    L.versions.push_back(VersionHdr{c.rstamp, c.sstamp, c.next, c.image});
                    meta_[i] = ((meta_[i] & ~kMetaTxn) | cid) & ~kMetaControl;
                    next_[i] = kNextVersion | kLocalRef | (uint32_t)(L.versions.size() - 1);
                }
                ++L.ok;
            }
        }
    });
    lap("process");
    // (D) concatenate in thread order, relocate the tagged references
    std::vector<uint64_t> cb(nt), vb(nt), ib(nt);
    uint64_t c0 = copies_.size(), v0 = versions_.size(), i0 = images_.size(), ok = 0;
    for (unsigned t = 0; t < nt; ++t) {
        cb[t] = c0, vb[t] = v0, ib[t] = i0;
        c0 += lw[t].copies.size(), v0 += lw[t].versions.size(), i0 += lw[t].images.size();
        ok += lw[t].ok;
    }
    if (c0 > kNextIndexMask || v0 > kNextIndexMask || i0 > kNextIndexMask)
        throw std::runtime_error("copy / version / image index overflow");
    // arena rows keep their order; each gets a global offset that does not straddle a chunk
    std::vector<std::vector<uint64_t>> row_at(nt);
    for (unsigned t = 0; t < nt; ++t) {
        row_at[t].resize(lw[t].images.size());
        for (size_t k = 0; k < lw[t].images.size(); ++k)
            row_at[t][k] = arena_.alloc(lw[t].images[k].kind == 2 ? kpad_ + p_.payload_size : p_.payload_size);
    }
    copies_.resize(c0);
    copy_live_.resize(c0, 1);
    versions_.resize(v0);
    images_.resize(i0);
    lap("resize");
    par(nt, [&](unsigned, uint64_t tb, uint64_t te) {
        for (uint64_t t = tb; t < te; ++t) {
            const LocalWrites &L = lw[t];
            for (size_t k = 0; k < L.copies.size(); ++k) {
                CopyHdr c = L.copies[k];
                c.next = reloc_next(c.next, cb[t], vb[t]);
                c.image = reloc_img(c.image, ib[t]);
                copies_[cb[t] + k] = c;
            }
            for (size_t k = 0; k < L.versions.size(); ++k) {
                VersionHdr v = L.versions[k];
                v.next = reloc_next(v.next, cb[t], vb[t]);
                v.image = reloc_img(v.image, ib[t]);
                versions_[vb[t] + k] = v;
            }
            for (size_t k = 0; k < L.images.size(); ++k) {
                ImageDesc d = L.images[k];
                const uint64_t bytes = d.kind == 2 ? kpad_ + p_.payload_size : p_.payload_size;
                std::memcpy(arena_.at(row_at[t][k]), L.arena.data() + d.arg, bytes);
                d.arg = row_at[t][k];
                images_[ib[t] + k] = d;
            }
            for (uint64_t i : L.touched) {
                next_[i] = reloc_next(next_[i], cb[t], vb[t]);
                image_[i] = reloc_img(image_[i], ib[t]);
            }
        }
    });
    lap("concat");
    {
        // each copy's SSN state at its copy id (cb[t] + k), not appended: the two arrays must
        // never drift apart (a copy id indexes both)
        std::lock_guard<std::mutex> g(ssn_.mu);
        if (nt && ssn_.e.size() > cb[0]) throw std::runtime_error("update_batch: SSN state ahead of the copies");
        if (ssn_.e.capacity() < copies_.size())
            ssn_.e.reserve(std::max<size_t>(copies_.size(), 2 * ssn_.e.capacity()));
        ssn_.e.resize(copies_.size(), CopySsn{0, 0, 0, kMaxCid, 0, 0, 0});
        for (unsigned t = 0; t < nt; ++t)
            for (size_t k = 0; k < lw[t].copies.size(); ++k) {
                const CopyHdr &c = lw[t].copies[k];
                ssn_.e[cb[t] + k] = CopySsn{lw[t].writers[k], lw[t].writers[k], c.rstamp, c.sstamp, 0,
                                            (uint8_t)(c.sstamp != kMaxCid), 0};
            }
    }
    for (unsigned t = 0; t < nt; ++t) {
        for (uint64_t i : lw[t].touched) {
            touch((uint32_t)(i / cap_), (uint32_t)(i % cap_));
            cell(i);
        }
        copies_dirty_from_ = std::min(copies_dirty_from_, lw[t].copies_dirty_from);
    }
    if (rc_out) std::memcpy(rc_out, rc.data(), n);
    lap("touch");
    return ok;
}

void HostTable::key_order(std::vector<uint32_t> &order) const {
    order.clear();
    order.reserve(nleaves_live_);
    for (int32_t l = head_; l >= 0; l = leaves_[l].next) order.push_back((uint32_t)l);
}

void HostTable::stats(uint64_t *out) const {
    for (int i = 0; i < 8; ++i) out[i] = 0;
    std::vector<uint32_t> order;
    key_order(order);
    out[2] = order.size();
    for (uint32_t l : order) {
        const Leaf &L = leaves_[l];
        for (uint32_t s = 0; s < L.count; ++s)
            if (meta_visible(meta_[(size_t)l * cap_ + s])) {
                out[3]++;
                if (s < L.sorted) out[4]++;
                else out[5]++;
            }
        out[6] = std::max<uint64_t>(out[6], L.count);
    }
    out[7] = versions_.size();
}

// keyw: the first 8 key bytes of each slot (the whole key for keys of <= 8 bytes)
int64_t HostTable::export_leaves(uint32_t cap, uint64_t max_leaves, uint32_t *rc, uint32_t *sc, uint64_t *meta,
                                 uint64_t *keyw) const {
    std::vector<uint32_t> order;
    key_order(order);
    if (order.size() > max_leaves) return -(int64_t)order.size();
    for (size_t d = 0; d < order.size(); ++d) {
        const Leaf &L = leaves_[order[d]];
        rc[d] = L.count;
        sc[d] = L.sorted;
        for (uint32_t s = 0; s < cap; ++s) {
            uint64_t m = 0, kw = 0;
            if (s < L.count && s < cap_) {
                const size_t i = (size_t)order[d] * cap_ + s;
                m = meta_[i];
                if (m) {
                    uint8_t kb[kMaxKeyBytes] = {0};
                    key_to_bytes(slot_key(i), kb, uns_);
                    std::memcpy(&kw, kb, 8);
                    if (meta_keylen(m) < 8) kw &= (1ull << (8 * meta_keylen(m))) - 1;
                }
            }
            meta[d * cap + s] = m;
            keyw[d * cap + s] = kw;
        }
    }
    return (int64_t)order.size();
}

// RecordLocation handles -> (leaf index in key order = the device leaf index, slot)
uint64_t HostTable::export_locations(uint64_t max, uint64_t *handles, uint32_t *leaf, uint16_t *slot) const {
    std::vector<uint32_t> order, rank(leaves_.size(), 0xFFFFFFFFu);
    key_order(order);
    for (size_t d = 0; d < order.size(); ++d) rank[order[d]] = (uint32_t)d;
    uint64_t k = 0;
    for (uint64_t id = 0; id < locpos_.size(); ++id) {
        if (locpos_[id] == kNoPos) continue;
        if (k < max) {
            handles[k] = id + 1;
            leaf[k] = rank[locpos_[id] >> 16];
            slot[k] = (uint16_t)(locpos_[id] & 0xFFFF);
        }
        ++k;
    }
    return k;
}

void HostTable::resolve_locations(const uint64_t *handles, uint64_t n, uint32_t *leaf, uint16_t *slot) const {
    std::vector<uint32_t> order, rank(leaves_.size(), 0xFFFFFFFFu);
    key_order(order);
    for (size_t d = 0; d < order.size(); ++d) rank[order[d]] = (uint32_t)d;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t h = handles[i];
        const uint64_t pos = (h == 0 || h > locpos_.size()) ? kNoPos : locpos_[h - 1];
        leaf[i] = pos == kNoPos ? 0xFFFFFFFFu : rank[pos >> 16];
        slot[i] = pos == kNoPos ? 0xFFFF : (uint16_t)(pos & 0xFFFF);
    }
}

// ---- leaf-level snapshot in the reference's block format --------------------------------
// Block = LeafNode (b_tree.h:571-740): [vptr 8][is_leaf 1 + pad 7][NodeHeader: size u32,
// sorted_count u32, next_record_slot u32 + pad 4, StatusWord u64 (version_store.h:158-231:
// frozen bit 60, record count 44-59, block size 22-43, delete size 0-21)], then
// RecordMetadata{meta, next_ptr, loc_ptr} (record_meta.h:30-60) per slot, records
// [key][pad to 8][payload] at meta.offset growing down from `size`.  Canonical form (the
// oracle's orc_export_leaf_images uses the same): next_ptr = 0, loc_ptr = the record's
// RecordLocation handle (location id + 1, 0 = none), record bytes not referenced by a non-zero
// meta word = 0.  Separators: key_words() u64 words of key bytes
// per leaf (little-endian), length 0xFFFF = +inf.
static constexpr uint32_t kLeafHdr = 40, kOffIsLeaf = 8, kOffSize = 16, kOffSorted = 20, kOffStatus = 32;

int64_t HostTable::export_leaf_images(uint64_t max_leaves, uint8_t *blocks, uint64_t *sep_key_le,
                                      uint16_t *sep_len) const {
    std::vector<uint32_t> order;
    key_order(order);
    if (order.size() > max_leaves) return -(int64_t)order.size();
    const uint32_t B = p_.leaf_node_size;
    std::vector<uint8_t> pay(p_.payload_size);
    uint8_t kb[kMaxKeyBytes];
    for (size_t d = 0; d < order.size(); ++d) {
        const Leaf &L = leaves_[order[d]];
        uint8_t *dst = blocks + d * (uint64_t)B;
        std::memset(dst, 0, B);
        dst[kOffIsLeaf] = 1;
        std::memcpy(dst + kOffSize, &B, 4);
        std::memcpy(dst + kOffSorted, &L.sorted, 4);
        const uint64_t status = ((uint64_t)L.count << 44) | ((uint64_t)L.block << 22) | L.deleted;
        std::memcpy(dst + kOffStatus, &status, 8);
        const size_t b = (size_t)order[d] * cap_;
        for (uint32_t s = 0; s < L.count; ++s) {
            const uint64_t m = meta_[b + s];
            const uint64_t lp = loc_[b + s];  // loc_ptr: the record's location handle
            std::memcpy(dst + kLeafHdr + 24 * s, &m, 8);
            std::memcpy(dst + kLeafHdr + 24 * s + 16, &lp, 8);
            if (!m) continue;
            const uint32_t off = meta_offset(m), kl = meta_keylen(m);
            key_to_bytes(slot_key(b + s), kb, uns_);
            std::memcpy(dst + off, kb, kl);
            image_payload(image_[b + s], pay.data());
            std::memcpy(dst + off + pad8(kl), pay.data(), p_.payload_size);
        }
        if (sep_key_le) {
            uint64_t *sw = sep_key_le + d * kw_;
            for (uint32_t w = 0; w < kw_; ++w) sw[w] = 0;
            if (!key_is_inf(L.sep)) key_to_bytes(L.sep, reinterpret_cast<uint8_t *>(sw), uns_);
            sep_len[d] = key_is_inf(L.sep) ? (uint16_t)kInfLen : (uint16_t)L.sep.len;
        }
    }
    return (int64_t)order.size();
}

uint64_t HostTable::import_leaf_images(const uint8_t *blocks, uint64_t n, uint32_t block_size,
                                       const uint64_t *sep_key_le, const uint16_t *sep_len) {
    auto bad = [](const std::string &w) { throw std::invalid_argument("leaf image import: " + w); };
    if (nleaves_live_ != 1 || head_ != 0 || leaves_.size() != 1 || leaves_[0].count != 0 || !images_.empty())
        bad("the table must be empty");
    if (block_size != p_.leaf_node_size) bad("block size differs from the table's leaf_node_size");
    if (n == 0) bad("no leaves");
    if (n > 0x7FFFFFFFull) bad("too many leaves");
    // separators: given (the inner-node keys) or derived as each leaf's largest visible key
    std::vector<Key> sep(n, key_inf());
    uint64_t nrec = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *blk = blocks + i * (uint64_t)block_size;
        uint32_t size, sorted;
        uint64_t status;
        std::memcpy(&size, blk + kOffSize, 4);
        std::memcpy(&sorted, blk + kOffSorted, 4);
        std::memcpy(&status, blk + kOffStatus, 8);
        const uint32_t count = (uint32_t)((status >> 44) & 0xFFFF);
        if (!blk[kOffIsLeaf]) bad("block " + std::to_string(i) + " is not a leaf");
        if (size != block_size) bad("block " + std::to_string(i) + ": header size != block size");
        if ((status >> 60) & 1) bad("block " + std::to_string(i) + " is frozen (mid-split)");
        if (count > cap_ || count > max_records_ || sorted > count) bad("block " + std::to_string(i) + ": bad counts");
        Key mx = key_zero(), mn = key_zero();
        bool any = false;
        for (uint32_t s = 0; s < count; ++s) {
            uint64_t m;
            std::memcpy(&m, blk + kLeafHdr + 24 * s, 8);
            if (!m) continue;
            if (m & kMetaControl) bad("block " + std::to_string(i) + ": in-flight record (control bit)");
            const uint32_t kl = meta_keylen(m), off = meta_offset(m);
            if (!key_ok(kl)) bad("block " + std::to_string(i) + ": key length not valid for this table");
            if (off < kLeafHdr + 24 * count || (uint64_t)off + pad8(kl) + p_.payload_size > size)
                bad("block " + std::to_string(i) + ": record offset out of range");
            if (!meta_visible(m)) continue;
            const Key k = make_key(blk + off, kl, uns_);
            if (!any || key_lt(mx, k)) mx = k;
            if (!any || key_lt(k, mn)) mn = k;
            any = true;
            ++nrec;
        }
        if (i + 1 < n) {
            if (sep_key_le) {
                if (!key_ok(sep_len[i])) bad("separator " + std::to_string(i) + ": length");
                sep[i] = make_key(reinterpret_cast<const uint8_t *>(sep_key_le + i * kw_), sep_len[i], uns_);
            } else {
                if (!any) bad("block " + std::to_string(i) + ": empty leaf needs an explicit separator");
                sep[i] = mx;
            }
            if (i > 0 && !key_lt(sep[i - 1], sep[i])) bad("separators are not increasing");
        }
        if (any && !key_le(mx, sep[i])) bad("block " + std::to_string(i) + ": key above its separator");
        if (any && i > 0 && !key_lt(sep[i - 1], mn)) bad("block " + std::to_string(i) + ": key below its range");
    }
    // second pass: fill the SoA leaves and images (first leaf reuses the empty root)
    images_.reserve(nrec);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t id = i == 0 ? (uint32_t)head_ : alloc_leaf();
        const uint8_t *blk = blocks + i * (uint64_t)block_size;
        uint32_t sorted;
        uint64_t status;
        std::memcpy(&sorted, blk + kOffSorted, 4);
        std::memcpy(&status, blk + kOffStatus, 8);
        Leaf &L = leaves_[id];
        L.count = (uint32_t)((status >> 44) & 0xFFFF);
        L.sorted = sorted;
        L.block = (uint32_t)((status >> 22) & 0x3FFFFF);
        L.deleted = (uint32_t)(status & 0x3FFFFF);
        L.sep = sep[i];
        L.prev = i == 0 ? -1 : (int32_t)(id - 1);
        L.next = -1;
        if (i > 0) leaves_[id - 1].next = (int32_t)id;
        const size_t b = (size_t)id * cap_;
        for (uint32_t s = 0; s < L.count; ++s) {
            uint64_t m, lp;
            std::memcpy(&m, blk + kLeafHdr + 24 * s, 8);
            std::memcpy(&lp, blk + kLeafHdr + 24 * s + 16, 8);
            meta_[b + s] = m;
            next_[b + s] = 0;
            // the block's loc_ptr is kept as the record's location handle (0: a new one)
            if (m || lp) {
                if (lp == 0) {
                    locpos_.push_back(kNoPos);
                    lp = locpos_.size();
                }
                if (lp >= 0xFFFFFFFFull) bad("location handle out of range");
                if (locpos_.size() < lp) locpos_.resize(lp, kNoPos);
                if (locpos_[lp - 1] != kNoPos) bad("location handle " + std::to_string(lp) + " used twice");
                locpos_[lp - 1] = (uint64_t)id << 16 | s;
                loc_[b + s] = (uint32_t)lp;
            }
            if (!m) {
                clear_slot_key(b + s);
                image_[b + s] = 0;
                continue;
            }
            const uint32_t kl = meta_keylen(m), off = meta_offset(m);
            set_slot_key(b + s, make_key(blk + off, kl, uns_));
            image_[b + s] = new_image(blk + off, kl, blk + off + pad8(kl), 0, 0);
        }
    }
    // router: every bucket lists, in key order, each leaf whose range (sep[i-1], sep[i]] meets it
    for (auto &v : buckets_) v.clear();
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t id = (uint32_t)(head_ + i);
        const uint32_t b_lo = i == 0 ? 0 : bucket_of(sep[i - 1]);
        const uint32_t b_hi = key_is_inf(sep[i]) ? (uint32_t)buckets_.size() - 1 : bucket_of(sep[i]);
        for (uint32_t bk = b_lo; bk <= b_hi; ++bk) buckets_[bk].push_back(RouteEntry{sep[i], id});
    }
    if (cells_.on()) {  // rebuild every cell from the imported layout
        for (uint64_t h = 1; h <= locpos_.size(); h += 1u << LocCells::kChunkBits) cells_.ensure(h);
        if (!locpos_.empty()) cells_.ensure(locpos_.size());
        for (uint32_t l = 0; l < leaves_.size(); ++l)
            if (leaves_[l].live)
                for (uint32_t s = 0; s < leaves_[l].count; ++s) cell((size_t)l * cap_ + s);
    }
    layout_dirty_ = true;
    structure_dirty_ = true;
    dirty_slots_.clear();
    return nrec;
}

}  // namespace stage
