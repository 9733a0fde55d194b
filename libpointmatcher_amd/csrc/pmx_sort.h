// pmx_sort.h — the radix sorts of the setup, the filters and VarTrimmed.
//
// rocPRIM's radix sort picks a merge sort for up to 2^20 items (its default
// radix_sort_config merge_sort_limit): at the 1M points of a C3 cloud that is
// ~21 launches (a block sort, then ten merge-path partition + merge pairs,
// ~180 us per 26-bit sort measured on MI355X).  The onesweep algorithm sorts
// the same keys in one histogram launch plus one launch per 8-bit digit.  The
// limit is set to 0 here: onesweep above the single-block size (both are
// stable radix orders, so the output is the same).
#pragma once

#include <rocprim/device/device_radix_sort.hpp>

namespace pmx {

using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;

template <typename K, typename V>
inline hipError_t pmx_sort_pairs(void* temp, size_t& bytes, const K* kin, K* kout, const V* vin, V* vout, int n,
                                 int begin_bit = 0, int end_bit = 8 * sizeof(K), hipStream_t st = 0) {
    return rocprim::radix_sort_pairs<OnesweepSort>(temp, bytes, kin, kout, vin, vout, (size_t)n,
                                                   (unsigned)begin_bit, (unsigned)end_bit, st);
}

template <typename K>
inline hipError_t pmx_sort_keys(void* temp, size_t& bytes, const K* kin, K* kout, int n, int begin_bit = 0,
                                int end_bit = 8 * sizeof(K), hipStream_t st = 0) {
    return rocprim::radix_sort_keys<OnesweepSort>(temp, bytes, kin, kout, (size_t)n, (unsigned)begin_bit,
                                                  (unsigned)end_bit, st);
}

}  // namespace pmx
