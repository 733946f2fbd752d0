// sparsify.hip — K5: degree-scored edge pruning on directed neighbour rows.
//
// Reference semantics:
//   SF-GRASS  src_legacy/sparsification.rs:32-113 — avg = sum len / n; if
//     avg < 10 the rows are returned unchanged; deg_i = len(row_i); per row
//     score = w * sqrt((deg_i * deg_j) as f64), sorted descending (the
//     reference's sort_unstable leaves ties unspecified: the contract here is
//     ascending input position), keep min(max(ceil(len * ratio), 1), len)
//     entries in score order.
//   INLINE    src_legacy/laplacian.rs:216-282 — inside _build_adjacency:
//     sparsify iff avg degree > 10 (strict); rows with len > 2 keep
//     max(len / 2, 1) entries by the same score.
//
// GPU design: one wave per row (k <= 64, one slot per lane): a count pass
// (row lengths + global total by atomics), then a pass that reads the total
// (so the avg-degree switch needs no host round trip), scores every slot in
// f64 (sqrt is correctly rounded on gfx950, verified in DESIGN.md), sorts the
// row with a wave bitonic on (-score, position) and writes the kept prefix.
#include <algorithm>
#include <climits>

#include "common.hpp"

namespace mn {
namespace sparsify {

__global__ __launch_bounds__(256) void k_row_len(const int32_t *__restrict__ idx, int64_t n,
                                                 int k, int32_t *__restrict__ len,
                                                 unsigned long long *__restrict__ total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int c = 0;
    for (int r = 0; r < k; ++r) {
        const int32_t j = idx[i * k + r];
        c += (j >= 0 && j < n) ? 1 : 0;
    }
    len[i] = c;
    atomicAdd(total, (unsigned long long)c);
}

__global__ __launch_bounds__(256) void k_sparsify_rows(
    const int32_t *__restrict__ idx, const double *__restrict__ w, int64_t n, int k,
    double ratio, int mode, const int32_t *__restrict__ len,
    const unsigned long long *__restrict__ total, int32_t *__restrict__ out_idx,
    double *__restrict__ out_w, int *__restrict__ applied) {
    const int lane = threadIdx.x & 63;
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i >= n) return;
    const double avg = (double)(*total) / (double)n;
    const bool active = (mode == MN_SPARSIFY_SFGRASS) ? !(avg < 10.0) : (avg > 10.0);
    if (i == 0 && lane == 0) *applied = active ? 1 : 0;
    // compacted position of this slot among the row's valid entries
    const int32_t j = lane < k ? idx[i * k + lane] : -1;
    const double wv = lane < k ? w[i * k + lane] : 0.0;
    const bool valid = j >= 0 && j < n;  // out-of-range ids are treated as empty
    const uint64_t vm = __ballot(valid);
    const int pos = (int)__popcll(vm & ((1ull << lane) - 1ull));
    const int m = (int)__popcll(vm);
    int keep = m;
    bool do_sort = false;
    if (active && m > 0) {
        if (mode == MN_SPARSIFY_SFGRASS) {
            const double kc = ceil((double)m * ratio);
            keep = (int)fmin(fmax(kc, 1.0), (double)m);
            do_sort = true;
        } else if (m > 2) {
            keep = max(m / 2, 1);
            do_sort = true;
        }
    }
    double key[1];
    int pk[1];
    if (do_sort) {
        const double di = (double)len[i];
        const double score = valid ? wv * sqrt(di * (double)len[j]) : 0.0;
        // descending score (NaN compares Equal in the reference: kept after
        // every number here), ties by input position
        key[0] = valid ? (score == score ? -score : __builtin_inf()) : __builtin_inf();
        pk[0] = valid ? pos : INT_MAX;  // (key, pos) is unique per valid entry
        wave_bitonic_sort<1>(key, pk);
        // element e (this lane) now holds the e-th kept candidate's position
        const int src_pos = pk[0];
        // gather (j, w) of the entry whose compacted position is src_pos
        const uint64_t pos_lane_mask = vm;  // valid lanes in slot order
        int src_lane = 64;
        if (src_pos != INT_MAX) {
            // the valid lane with popcount-rank == src_pos
            uint64_t mm = pos_lane_mask;
            for (int t = 0; t < src_pos; ++t) mm &= mm - 1;
            src_lane = (int)__builtin_ctzll(mm);
        }
        const int gj = __shfl(j, src_lane & 63);
        const double gw = __shfl(wv, src_lane & 63);
        if (lane < k) {
            const bool kept = lane < keep;
            out_idx[i * k + lane] = kept ? gj : -1;
            out_w[i * k + lane] = kept ? gw : 0.0;
        }
    } else {
        // pass-through, compacted (valid entries first, in slot order)
        int32_t cj = -1;
        double cw = 0.0;
        // lane e takes the e-th valid slot
        int src_lane = 64;
        if (lane < m) {
            uint64_t mm = vm;
            for (int t = 0; t < lane; ++t) mm &= mm - 1;
            src_lane = (int)__builtin_ctzll(mm);
        }
        cj = __shfl(j, src_lane & 63);
        cw = __shfl(wv, src_lane & 63);
        if (lane < k) {
            out_idx[i * k + lane] = lane < m ? cj : -1;
            out_w[i * k + lane] = lane < m ? cw : 0.0;
        }
    }
}

}  // namespace sparsify
}  // namespace mn

extern "C" int mn_sparsify_rows(const int32_t *nbr_idx, const double *nbr_w, int64_t n,
                                int32_t k, double ratio, int32_t mode, int32_t *out_idx,
                                double *out_w, int32_t *applied_host, void *stream) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(n >= 1 && k >= 1 && k <= 64, MN_EINVAL, "mn_sparsify_rows: n>=1, 1<=k<=64");
    MN_REQUIRE(nbr_idx && nbr_w && out_idx && out_w, MN_EINVAL, "mn_sparsify_rows: NULL pointer");
    MN_REQUIRE(mode == MN_SPARSIFY_SFGRASS || mode == MN_SPARSIFY_INLINE, MN_EINVAL,
               "mn_sparsify_rows: unknown mode");
    MN_REQUIRE(nbr_idx != out_idx, MN_EINVAL, "mn_sparsify_rows: in-place not supported");
    hipStream_t s = (hipStream_t)stream;
    char *g = (char *)scratch(kSlotGeneric3, (size_t)n * 4 + 64);
    MN_REQUIRE(g, MN_ENOMEM, "mn_sparsify_rows: scratch allocation failed");
    unsigned long long *total = (unsigned long long *)g;
    int *applied = (int *)(g + 8);
    int32_t *len = (int32_t *)(g + 64);
    MN_HIP_TRY(hipMemsetAsync(g, 0, 16, s));
    hipLaunchKernelGGL(sparsify::k_row_len, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       nbr_idx, n, k, len, total);
    hipLaunchKernelGGL(sparsify::k_sparsify_rows, dim3((unsigned)((n * 64 + 255) / 256)),
                       dim3(256), 0, s, nbr_idx, nbr_w, n, k, ratio, mode, len, total, out_idx,
                       out_w, applied);
    MN_HIP_TRY(hipGetLastError());
    int ha = 0;
    MN_HIP_TRY(hipMemcpyAsync(&ha, applied, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (applied_host) *applied_host = ha;
    return MN_OK;
}
