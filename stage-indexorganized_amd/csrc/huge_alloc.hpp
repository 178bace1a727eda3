// huge_alloc.hpp -- allocator for the host table's per-slot arrays (GBs at 100M rows, written
// and read at random slots): blocks of 8 MiB and more are 2-MiB aligned and marked for
// transparent huge pages (madvise; the kernel's THP mode on these hosts is "madvise"), so a
// random slot access does not also miss the TLB.  Measured on scattered slot-word writes of a
// device epoch (840K records into 131M-slot arrays, 16 threads): 1.7x faster.
#pragma once
#include <sys/mman.h>

#include <cstddef>
#include <cstdlib>
#include <new>

namespace stage {

template <class T>
struct HugeAlloc {
    using value_type = T;
    static constexpr size_t kHuge = 2u << 20, kMin = 8u << 20;
    HugeAlloc() = default;
    template <class U>
    HugeAlloc(const HugeAlloc<U> &) {}
    T *allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < kMin) return static_cast<T *>(::operator new(bytes));
        const size_t r = (bytes + kHuge - 1) & ~(kHuge - 1);
        void *p = std::aligned_alloc(kHuge, r);
        if (!p) throw std::bad_alloc();
        (void)madvise(p, r, MADV_HUGEPAGE);
        return static_cast<T *>(p);
    }
    void deallocate(T *p, size_t n) {
        if (n * sizeof(T) < kMin) ::operator delete(p);
        else std::free(p);
    }
    template <class U>
    bool operator==(const HugeAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const HugeAlloc<U> &) const { return false; }
};

}  // namespace stage
