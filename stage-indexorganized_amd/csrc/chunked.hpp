// chunked.hpp -- append-only host stores that grow without moving what they hold.
//
// The record-image descriptors and the explicit-payload arena grow by one YCSB-B epoch at a
// time (hundreds of MB); a std::vector would copy the whole store on every reallocation.
// Chunks keep old elements in place, and an arena row never straddles two chunks, so a
// global byte offset is valid on the host and, unchanged, in the contiguous device arena.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "huge_alloc.hpp"

namespace stage {

template <class T, size_t kChunk>
class ChunkedVector {
public:
    size_t size() const { return size_; }
    bool empty() const { return size_ == 0; }
    T &operator[](size_t i) { return chunks_[i / kChunk][i % kChunk]; }
    const T &operator[](size_t i) const { return chunks_[i / kChunk][i % kChunk]; }
    void push_back(const T &v) {
        ensure(size_ + 1);
        (*this)[size_++] = v;
    }
    // grow (new elements are not initialised: callers write them) or shrink the logical size
    void resize(size_t n) {
        ensure(n);
        size_ = n;
    }
    void reserve(size_t n) { ensure(n); }

    ChunkedVector() = default;
    ChunkedVector(const ChunkedVector &) = delete;
    ChunkedVector &operator=(const ChunkedVector &) = delete;
    ~ChunkedVector() {
        for (T *c : chunks_) HugeAlloc<T>().deallocate(c, kChunk);
    }

private:
    // chunks on huge pages (a chunk of image descriptors is 24 MiB): an epoch's appends fault
    // in a few 2-MiB pages instead of thousands of 4-KiB ones
    void ensure(size_t n) {
        while (chunks_.size() * kChunk < n) {
            static_assert(std::is_trivially_copyable<T>::value, "chunk elements are raw storage");
            chunks_.push_back(HugeAlloc<T>().allocate(kChunk));
        }
    }
    std::vector<T *> chunks_;
    size_t size_ = 0;
};

class ChunkedArena {
public:
    static constexpr uint64_t kChunk = 64ull << 20;
    uint64_t size() const { return size_; }
    // room for n contiguous bytes (n <= kChunk); returns their global offset
    uint64_t alloc(uint64_t n) {
        if (n > kChunk) throw std::invalid_argument("arena row larger than a chunk");
        if ((size_ % kChunk) + n > kChunk) size_ = (size_ / kChunk + 1) * kChunk;
        const uint64_t off = size_;
        size_ += n;
        while (chunks_.size() * kChunk < size_) chunks_.emplace_back(new uint8_t[kChunk]);
        return off;
    }
    uint8_t *at(uint64_t off) { return chunks_[off / kChunk].get() + off % kChunk; }
    const uint8_t *at(uint64_t off) const { return chunks_[off / kChunk].get() + off % kChunk; }
    // contiguous host segments covering [b, e): fn(offset, pointer, bytes)
    template <class F>
    void segments(uint64_t b, uint64_t e, F fn) const {
        while (b < e) {
            const uint64_t ce = (b / kChunk + 1) * kChunk, se = ce < e ? ce : e;
            fn(b, at(b), se - b);
            b = se;
        }
    }

private:
    std::vector<std::unique_ptr<uint8_t[]>> chunks_;
    uint64_t size_ = 0;
};

}  // namespace stage
