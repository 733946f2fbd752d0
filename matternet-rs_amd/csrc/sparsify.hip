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
#include "scan.hpp"

namespace mn {
namespace sparsify {

// deg_i = row length (deg == NULL), or the caller's degrees (the inline
// pruning's eps-valid neighbour counts, laplacian.rs:219-229); total = sum
__global__ __launch_bounds__(256) void k_row_len(const int32_t *__restrict__ idx, int64_t n,
                                                 int k, const int32_t *__restrict__ deg,
                                                 int32_t *__restrict__ len,
                                                 unsigned long long *__restrict__ total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int c = 0;
    if (i < n) {
        if (deg) {
            c = deg[i];
        } else {
            for (int r = 0; r < k; ++r) {
                const int32_t j = idx[i * k + r];
                c += (j >= 0 && j < n) ? 1 : 0;
            }
        }
        len[i] = c;
    }
    // one atomic per wave
    unsigned long long t = (unsigned long long)(int64_t)c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if ((threadIdx.x & 63) == 0 && t) atomicAdd(total, t);
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
                                int32_t k, double ratio, int32_t mode, const int32_t *degrees,
                                int32_t *out_idx, double *out_w, int32_t *applied_host,
                                void *stream) {
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
                       nbr_idx, n, k, degrees, len, total);
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

namespace mn {
namespace sparsify {

// ---------------------------------------------------------------------------
// SF-GRASS over CSR rows of any length (SURVEY.md §8(b) mn_sparsify_sfgrass;
// SfGrassSparsifier::sparsify_graph, src_legacy/sparsification.rs:32-101, on
// &[Vec<(usize, f64)>]: e.g. a symmetrised adjacency whose hub rows hold
// thousands of entries).
//
//   1. k_sf_keep     per row: keep_i = min(max(ceil(len_i ratio), 1), len_i)
//                    (0 for an empty row), or len_i when pruning is off
//   2. scan          output row pointers
//   3. k_sf_rows     one wave per row of <= 512 entries: f64 scores
//                    w * sqrt((deg_i deg_j) as f64), register bitonic on
//                    (-score, position), the kept prefix written in score order
//   4. k_sf_big      one 1024-thread block per longer row: the same sort in LDS
//                    (<= 8192 entries) or, for hub rows, in a global scratch
//                    image (block-wide bitonic network, agent release/acquire
//                    between the steps)
// Bandwidth: nnz (12 B in) + kept (12 B out) + 2 (n + 1) 8 B row pointers.
// ---------------------------------------------------------------------------
constexpr int SF_WAVE_CAP = 512;
constexpr int SF_LDS_CAP = 8192;

__global__ __launch_bounds__(256) void k_sf_keep(const int64_t *__restrict__ indptr, int64_t n,
                                                 double ratio, int active,
                                                 int32_t *__restrict__ keep,
                                                 int *__restrict__ too_long) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t len = indptr[i + 1] - indptr[i];
    // the row sorts index a row with int positions and a power-of-two pad
    if (len > ((int64_t)1 << 30)) atomicOr(too_long, 1);
    int64_t kc = len;
    if (active && len > 0) {
        // ((len as f64 * ratio).ceil() as usize).max(1).min(len)
        const double c = ceil((double)len * ratio);
        kc = !(c == c) || c < 1.0 ? 1 : (c >= (double)len ? len : (int64_t)c);  // NaN as usize: 0
    }
    keep[i] = (int32_t)kc;
}

// score of entry p of row i (deg = row lengths); NaN sorts after every number
// (the reference's partial_cmp().unwrap_or(Equal) has no total order there)
__device__ __forceinline__ double sf_key(const int64_t *__restrict__ indptr,
                                         const int32_t *__restrict__ idx,
                                         const double *__restrict__ w, int64_t n, int64_t di,
                                         int64_t p) {
    const int32_t j = idx[p];
    const int64_t dj = (j >= 0 && j < n) ? indptr[j + 1] - indptr[j] : 0;
    const double sc = w[p] * sqrt((double)(uint64_t)(di * dj));
    return sc == sc ? -sc : __builtin_inf();
}

template <int NR>
__device__ __forceinline__ void sf_row_wave(const int64_t *__restrict__ indptr,
                                            const int32_t *__restrict__ idx,
                                            const double *__restrict__ w, int64_t n, int64_t i,
                                            const int64_t *__restrict__ optr,
                                            int32_t *__restrict__ oidx, double *__restrict__ ow) {
    const int lane = threadIdx.x & 63;
    const int64_t o = indptr[i];
    const int m = (int)(indptr[i + 1] - o);
    const int64_t oo = optr[i];
    const int keep = (int)(optr[i + 1] - oo);
    double key[NR];
    int pk[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        key[r] = e < m ? sf_key(indptr, idx, w, n, m, o + e) : __builtin_inf();
        pk[r] = e < m ? e : INT_MAX;
    }
    wave_bitonic_sort<NR>(key, pk);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        if (e < keep) {
            oidx[oo + e] = idx[o + pk[r]];
            ow[oo + e] = w[o + pk[r]];
        }
    }
}

__global__ __launch_bounds__(256) void k_sf_rows(const int64_t *__restrict__ indptr,
                                                 const int32_t *__restrict__ idx,
                                                 const double *__restrict__ w, int64_t n,
                                                 const int64_t *__restrict__ optr,
                                                 int32_t *__restrict__ oidx,
                                                 double *__restrict__ ow,
                                                 int32_t *__restrict__ big_list,
                                                 int *__restrict__ big_count) {
    const int lane = threadIdx.x & 63;
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i >= n) return;
    const int64_t m = indptr[i + 1] - indptr[i];
    if (m == 0) return;
    if (m <= 64) sf_row_wave<1>(indptr, idx, w, n, i, optr, oidx, ow);
    else if (m <= 128) sf_row_wave<2>(indptr, idx, w, n, i, optr, oidx, ow);
    else if (m <= 256) sf_row_wave<4>(indptr, idx, w, n, i, optr, oidx, ow);
    else if (m <= SF_WAVE_CAP) sf_row_wave<8>(indptr, idx, w, n, i, optr, oidx, ow);
    else if (lane == 0) big_list[atomicAdd(big_count, 1)] = (int32_t)i;
}

__device__ __forceinline__ bool sf_less(double ka, int pa, double kb, int pb) {
    return ka < kb || (ka == kb && pa < pb);
}

__device__ __forceinline__ void sf_sync_global() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

struct alignas(16) SfBigSmem {
    double k[SF_LDS_CAP];
    int p[SF_LDS_CAP];
};

// rows of > SF_WAVE_CAP entries; gk / gp: per big-row global scratch images of
// the padded length (hub rows only), at gofs[b]
__global__ __launch_bounds__(1024) void k_sf_big(const int64_t *__restrict__ indptr,
                                                 const int32_t *__restrict__ idx,
                                                 const double *__restrict__ w, int64_t n,
                                                 const int64_t *__restrict__ optr,
                                                 const int32_t *__restrict__ big_list,
                                                 const int *__restrict__ big_count,
                                                 double *__restrict__ gk, int *__restrict__ gp,
                                                 const int64_t *__restrict__ gofs,
                                                 int32_t *__restrict__ oidx,
                                                 double *__restrict__ ow) {
    __shared__ SfBigSmem sm;
    const int t = threadIdx.x;
    const int nb = *big_count;
    for (int b = blockIdx.x; b < nb; b += gridDim.x) {
        const int64_t i = big_list[b];
        const int64_t o = indptr[i];
        const int m = (int)(indptr[i + 1] - o);
        const int64_t oo = optr[i];
        const int keep = (int)(optr[i + 1] - oo);
        int P = 1;
        while (P < m) P <<= 1;
        const bool lds = P <= SF_LDS_CAP;
        double *K = lds ? sm.k : gk + gofs[b];
        int *Pp = lds ? sm.p : gp + gofs[b];
        for (int e = t; e < P; e += blockDim.x) {
            K[e] = e < m ? sf_key(indptr, idx, w, n, m, o + e) : __builtin_inf();
            Pp[e] = e < m ? e : INT_MAX;
        }
        if (lds) __syncthreads();
        else sf_sync_global();
        for (int kk = 2; kk <= P; kk <<= 1) {
            for (int j = kk >> 1; j > 0; j >>= 1) {
                for (int q = t; q < P / 2; q += blockDim.x) {
                    const int e = ((q & ~(j - 1)) << 1) | (q & (j - 1));  // bit j clear
                    const int pe = e | j;
                    const bool asc = (e & kk) == 0;
                    const double ke = K[e], kp = K[pe];
                    const int pe_ = Pp[e], pp = Pp[pe];
                    const bool sw = asc ? sf_less(kp, pp, ke, pe_) : sf_less(ke, pe_, kp, pp);
                    if (sw) {
                        K[e] = kp; Pp[e] = pp;
                        K[pe] = ke; Pp[pe] = pe_;
                    }
                }
                if (lds) __syncthreads();
                else sf_sync_global();
            }
        }
        for (int e = t; e < keep; e += blockDim.x) {
            const int src = Pp[e];
            oidx[oo + e] = idx[o + src];
            ow[oo + e] = w[o + src];
        }
        __syncthreads();
    }
}

// padded image offsets of the hub rows (P > SF_LDS_CAP), listed in big_list
// order; gofs[nb] = total elements
__global__ void k_sf_hub_offsets(const int64_t *__restrict__ indptr,
                                 const int32_t *__restrict__ big_list,
                                 const int *__restrict__ big_count, int64_t *__restrict__ gofs) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int nb = *big_count;
    int64_t acc = 0;
    for (int b = 0; b < nb; ++b) {
        gofs[b] = acc;
        const int64_t i = big_list[b];
        const int64_t m = indptr[i + 1] - indptr[i];
        int64_t P = 1;
        while (P < m) P <<= 1;
        if (P > SF_LDS_CAP) acc += P;
    }
    gofs[nb] = acc;
}

}  // namespace sparsify

static int sfgrass_impl(const mn_csr *in, int64_t n_nodes, double ratio, mn_csr *out,
                        int32_t *applied_host, void *stream) {
    using namespace sparsify;
    clear_error();
    MN_REQUIRE(in && out, MN_EINVAL, "mn_sparsify_sfgrass: NULL in/out");
    const mn_csr given = *out;
    const bool caller = given.caller_owned == 1;
    *out = mn_csr{};
    const int64_t n = in->n_rows;
    MN_REQUIRE(n >= 1 && n < INT_MAX && in->indptr && (in->nnz == 0 || (in->indices && in->values)),
               MN_EINVAL, "mn_sparsify_sfgrass: bad input CSR (n_rows=%lld)", (long long)n);
    MN_REQUIRE(in->value_type == MN_F64, MN_EINVAL,
               "mn_sparsify_sfgrass: values must be f64 (Vec<(usize, f64)>)");
    if (caller)
        MN_REQUIRE(given.indptr && given.indices && given.values && given.nnz >= 0 &&
                       given.value_type == MN_F64, MN_EINVAL,
                   "mn_sparsify_sfgrass: caller-owned output needs indptr/indices/f64 values");
    const int64_t nn = n_nodes > 0 ? n_nodes : n;
    hipStream_t s = (hipStream_t)stream;
    int64_t ends[2] = {0, 0};
    MN_HIP_TRY(hipMemcpyAsync(&ends[0], in->indptr, 8, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipMemcpyAsync(&ends[1], in->indptr + n, 8, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(ends[0] == 0 && ends[1] >= 0, MN_EINVAL,
               "mn_sparsify_sfgrass: indptr must start at 0");
    const int64_t orig = ends[1];
    // sparsification.rs:41-51: avg = orig_edges / n_nodes; skip if < 10
    const double avg = (double)orig / (double)nn;
    const int active = !(avg < 10.0);
    const double r = ratio;
    char *g = (char *)scratch(kSlotGeneric3, (size_t)n * 4 + (size_t)(n + 2) * 8 +
                                                 ((size_t)n / scan::SB + 4) * 8 + 256);
    int *flags = (int *)scratch(kSlotFlags, 64);
    MN_REQUIRE(g && flags, MN_ENOMEM, "mn_sparsify_sfgrass: scratch allocation failed");
    int32_t *keep = (int32_t *)g;
    int64_t *part = (int64_t *)(g + (((size_t)n * 4 + 15) & ~(size_t)15));
    int32_t *big_list = (int32_t *)scratch(kSlotGeneric2, (size_t)n * 4 + (size_t)n * 8 + 256);
    MN_REQUIRE(big_list, MN_ENOMEM, "mn_sparsify_sfgrass: scratch allocation failed");
    int64_t *gofs = (int64_t *)(((uintptr_t)(big_list + n) + 15) & ~(uintptr_t)15);
    // output row pointers first (their last entry is the output nnz)
    int64_t *optr = caller ? given.indptr : nullptr;
    if (!caller) MN_HIP_TRY(hipMalloc(&optr, sizeof(int64_t) * (n + 1)));
    hipError_t e = hipMemsetAsync(flags + 4, 0, 4, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_sf_keep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                           in->indptr, n, r, active, keep, flags + 4);
        e = scan::exclusive_scan(keep, n, optr, part, s);
    }
    int64_t nnz = 0;
    int too_long = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&nnz, optr + n, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&too_long, flags + 4, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        if (!caller) (void)hipFree(optr);
        set_error("mn_sparsify_sfgrass: %s", hipGetErrorString(e));
        return MN_EHIP;
    }
    if (too_long) {
        if (!caller) (void)hipFree(optr);
        set_error("mn_sparsify_sfgrass: a row longer than 2^30 entries");
        return MN_ENOTSUP;
    }
    if (caller && nnz > given.nnz) {
        out->nnz = nnz;
        set_error("mn_sparsify_sfgrass: output capacity %lld < nnz %lld", (long long)given.nnz,
                  (long long)nnz);
        return MN_ECAP;
    }
    int32_t *oidx = caller ? given.indices : nullptr;
    double *ow = caller ? (double *)given.values : nullptr;
    if (!caller && (hipMalloc(&oidx, sizeof(int32_t) * std::max<int64_t>(nnz, 1)) != hipSuccess ||
                    hipMalloc(&ow, sizeof(double) * std::max<int64_t>(nnz, 1)) != hipSuccess)) {
        (void)hipFree(optr); (void)hipFree(oidx); (void)hipFree(ow);
        set_error("mn_sparsify_sfgrass: output allocation (%lld entries) failed", (long long)nnz);
        return MN_ENOMEM;
    }
    auto fail = [&](const char *what, hipError_t er) {
        if (!caller) { (void)hipFree(optr); (void)hipFree(oidx); (void)hipFree(ow); }
        set_error("mn_sparsify_sfgrass: %s: %s", what, hipGetErrorString(er));
        return MN_EHIP;
    };
    if (!active) {  // sparsification.rs:48-53: the rows unchanged
        if (nnz > 0) {
            if ((e = hipMemcpyAsync(oidx, in->indices, 4 * (size_t)nnz, hipMemcpyDeviceToDevice, s)) != hipSuccess ||
                (e = hipMemcpyAsync(ow, in->values, 8 * (size_t)nnz, hipMemcpyDeviceToDevice, s)) != hipSuccess)
                return fail("copy", e);
        }
    } else {
        if ((e = hipMemsetAsync(flags, 0, 8, s)) != hipSuccess) return fail("memset", e);
        hipLaunchKernelGGL(k_sf_rows, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, s,
                           in->indptr, in->indices, (const double *)in->values, n, optr, oidx, ow,
                           big_list, flags);
        hipLaunchKernelGGL(k_sf_hub_offsets, dim3(1), dim3(64), 0, s, in->indptr, big_list, flags,
                           gofs);
        int64_t hub_elems = 0;
        int nbig = 0;
        if ((e = hipGetLastError()) != hipSuccess) return fail("k_sf_rows", e);
        if ((e = hipMemcpyAsync(&nbig, flags, 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return fail("sync", e);
        if (nbig > 0) {
            if ((e = hipMemcpyAsync(&hub_elems, gofs + nbig, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                (e = hipStreamSynchronize(s)) != hipSuccess)
                return fail("sync", e);
            char *hb = (char *)scratch(kSlotGeneric1, (size_t)hub_elems * 12 + 256);
            if (!hb) {
                if (!caller) { (void)hipFree(optr); (void)hipFree(oidx); (void)hipFree(ow); }
                set_error("mn_sparsify_sfgrass: hub-row scratch (%lld entries) failed",
                          (long long)hub_elems);
                return MN_ENOMEM;
            }
            double *gk = (double *)hb;
            int *gp = (int *)(hb + (size_t)hub_elems * 8);
            hipLaunchKernelGGL(k_sf_big, dim3((unsigned)std::min(nbig, 1024)), dim3(1024), 0, s,
                               in->indptr, in->indices, (const double *)in->values, n, optr,
                               big_list, flags, gk, gp, gofs, oidx, ow);
            if ((e = hipGetLastError()) != hipSuccess) return fail("k_sf_big", e);
        }
    }
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail("sync", e);
    if (applied_host) *applied_host = active;
    out->n_rows = n;
    out->n_cols = in->n_cols;
    out->nnz = nnz;
    out->indptr = optr;
    out->indices = oidx;
    out->values = ow;
    out->value_type = MN_F64;
    out->caller_owned = caller ? 1 : 0;
    return MN_OK;
}

}  // namespace mn

extern "C" int mn_sparsify_sfgrass(const mn_csr *in, int64_t n_nodes, double ratio, mn_csr *out,
                                   int32_t *applied_host, void *stream) {
    return mn::sfgrass_impl(in, n_nodes, ratio, out, applied_host, stream);
}
