// sortkeys.hip — device radix sort of (f32 key, int32 value) pairs for the
// symmetric K1 sweep (rows ordered by their phase-1 threshold).  rocPRIM's
// device radix sort (header-only, gfx950), behind a plain internal entry so
// the K1 translation unit does not instantiate it.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace mn {

hipError_t sort_f32_pairs(const float *keys_in, float *keys_out, const int *vals_in, int *vals_out,
                          int64_t n, hipStream_t s) {
    size_t bytes = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, bytes, keys_in, keys_out, vals_in, vals_out,
                                             (unsigned)n, 0, 32, s);
    if (e != hipSuccess) return e;
    void *tmp = scratch(kSlotSortTmp, bytes + 256);
    if (!tmp) return hipErrorOutOfMemory;
    return rocprim::radix_sort_pairs(tmp, bytes, keys_in, keys_out, vals_in, vals_out,
                                     (unsigned)n, 0, 32, s);
}

}  // namespace mn
