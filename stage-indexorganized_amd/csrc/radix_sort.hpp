// radix_sort.hpp -- key/value radix sorts of the device paths (.hip translation units only).
// rocprim's default dispatch sorts up to 2^20 items with its merge sort (block sort + merge
// passes); a device write-path epoch (~0.84 M ops) or a CH-Q2 batch (~0.4 M keys) then pays
// ~1.5 ms / ~0.1 ms of merge passes that the onesweep radix sort does in a fraction of it.  This
// config keeps the single-block sort for tiny inputs and uses onesweep from 4096 items on.
#pragma once
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

namespace stage {

using OnesweepFrom4K = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                  rocprim::default_config, 4096>;

// 64-bit keys (the device write path's (slot, op) sort): 256-thread workgroups in both onesweep
// kernels.  rocprim's gfx950 default uses 512-thread ones; beside C3's read probe (256-thread
// workgroups filling every CU) a 512-thread workgroup needs two retired probe workgroups on one
// CU before the next probe workgroup takes the slot, so the sort's scatter pass waited for the
// probe to finish dispatching
template <class K>
struct SortConfig {
    using type = OnesweepFrom4K;
};
template <>
struct SortConfig<uint64_t> {
    using type = rocprim::radix_sort_config<
        rocprim::default_config, rocprim::default_config,
        rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 16>, rocprim::kernel_config<256, 8>, 8,
                                            rocprim::block_radix_rank_algorithm::match>,
        4096>;
};

// temp == nullptr: storage size query
template <class K, class V>
inline hipError_t sort_pairs(void *temp, size_t &bytes, const K *kin, K *kout, const V *vin, V *vout, uint64_t n,
                             int begin_bit, int end_bit, hipStream_t s) {
    return rocprim::radix_sort_pairs<typename SortConfig<K>::type>(temp, bytes, kin, kout, vin, vout, (size_t)n,
                                                                   (unsigned)begin_bit, (unsigned)end_bit, s);
}

}  // namespace stage
