// knn_f64.hip — the reference's f64 Euclidean kNN call sites, exact folds.
//
//   topk_by_l2            src_legacy/energymaps.rs:875-892   d = sum (a-b)*(a-b)
//                         (sequential f64 fold), j != i, stable sort, top k
//   prepare_query_item    src_legacy/core.rs:872-909          sqrt'd distance,
//                         1-NN with strict '<' (lowest index among ties)
//   estimate_intrinsic_dimension  src_legacy/clustering.rs:132-195  sqrt'd
//                         distances of <= 500 sampled rows, d1 and d2
//
// These sizes are small next to K1 (hundreds of queries, or N items against
// S sub-centroids), so the exact fold is evaluated for EVERY pair — no Gram
// filter: a block = 32 queries x 256 corpus rows, each thread 4 x 8 pairs
// (32 independent sequential f64 chains, operands broadcast from LDS slabs of
// 16 features); the tile's 256 distances per query are sorted by one wave
// (bitonic, (dist, idx)) and its best k kept; a merge kernel folds the tiles'
// lists 8 at a time.  (dist, idx) is a total order, so per-tile selection +
// merges equal the reference's stable sort truncated to k.
#include <algorithm>
#include <climits>
#include <vector>

#include "common.hpp"

namespace mn {
namespace kf64 {

constexpr int TQ = 32;   // queries per block
constexpr int TC = 256;  // corpus rows per block
constexpr int DS = 16;   // features per LDS slab
constexpr int KMAX = 64;

struct alignas(16) Smem {
    union {
        struct {
            double q[DS][TQ];       // transposed slabs: 4 consecutive queries = 2 x b128
            double c[DS][TC + 2];   // +2: the 8-row groups of a wave hit distinct banks
        } s;
        double dist[TQ][TC + 1];    // tile distances (after the folds)
    } u;
    int flag;
};

template <typename T>
__device__ __forceinline__ double ld(const T *p) { return (double)*p; }

// grid: (corpus tiles, query blocks).  cand [nq][ntiles][k] (dist, idx).
template <typename T>
__global__ __launch_bounds__(256) void k_l2_tile(const T *__restrict__ Q, int64_t nq,
                                                 const T *__restrict__ C, int64_t nc, int d,
                                                 const int64_t *__restrict__ q_ids, int k,
                                                 int use_sqrt, double *__restrict__ cand_d,
                                                 int32_t *__restrict__ cand_i,
                                                 int *__restrict__ nan_flag) {
    __shared__ Smem sm;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int qg = tid & 7, cg = tid >> 3;  // queries 4qg.., corpus rows 8cg..
    const int64_t tile = blockIdx.x, ntiles = gridDim.x;
    const int64_t q0 = (int64_t)blockIdx.y * TQ, c0 = tile * TC;
    double acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = -0.0;  // Rust >= 1.83 float Sum
    for (int t0 = 0; t0 < d; t0 += DS) {
        __syncthreads();
        // stage: queries 32 x 16 (2 per thread), corpus 256 x 16 (16 per thread)
        for (int e = tid; e < TQ * DS; e += 256) {
            const int r = e / DS, t = e % DS;
            const int64_t q = min(q0 + r, nq - 1);
            sm.u.s.q[t][r] = t0 + t < d ? ld(Q + q * d + t0 + t) : 0.0;
        }
        for (int e = tid; e < TC * DS; e += 256) {
            const int r = e / DS, t = e % DS;
            const int64_t c = min(c0 + r, nc - 1);
            sm.u.s.c[t][r] = t0 + t < d ? ld(C + c * d + t0 + t) : 0.0;
        }
        __syncthreads();
        const int tn = min(DS, d - t0);
        for (int t = 0; t < tn; ++t) {
            const double2 qa = *reinterpret_cast<const double2 *>(&sm.u.s.q[t][4 * qg]);
            const double2 qb = *reinterpret_cast<const double2 *>(&sm.u.s.q[t][4 * qg + 2]);
            const double qv[4] = {qa.x, qa.y, qb.x, qb.y};
            double cv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) cv[j] = sm.u.s.c[t][8 * cg + j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const double df = qv[i] - cv[j];
                    acc[i][j] = acc[i][j] + df * df;  // no contraction (-ffp-contract=off)
                }
        }
    }
    __syncthreads();  // slabs dead: the union now holds distances
    bool nan = false;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            double v = use_sqrt ? __builtin_sqrt(acc[i][j]) : acc[i][j];  // f64 sqrt: IEEE
            nan |= v != v;
            sm.u.dist[4 * qg + i][8 * cg + j] = v;
        }
    if (nan) atomicOr(nan_flag, 1);
    __syncthreads();
    // each wave sorts 8 queries' 256 distances and keeps the best k
    for (int qq = wv; qq < TQ; qq += 4) {
        const int64_t q = q0 + qq;
        if (q >= nq) break;
        const int64_t self = q_ids ? q_ids[q] : -1;
        double dv[4];
        int ix[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int cc = lane + 64 * r;
            const int64_t c = c0 + cc;
            const bool ok = c < nc && c != self;
            dv[r] = ok ? sm.u.dist[qq][cc] : __builtin_inf();
            ix[r] = ok ? (int)c : INT_MAX;
        }
        wave_bitonic_sort<4>(dv, ix);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = lane + 64 * r;
            if (e < k) {
                cand_d[(q * ntiles + tile) * k + e] = dv[r];
                cand_i[(q * ntiles + tile) * k + e] = ix[r];
            }
        }
    }
}

// One wave per (query, group of 8 lists): merge 8 sorted k-lists (512 slots)
// and keep the best k.  Final level writes out_idx (-1 pad) / out_dist.
__global__ __launch_bounds__(256) void k_l2_merge(const double *__restrict__ ind,
                                                  const int32_t *__restrict__ ini, int64_t nq,
                                                  int64_t nlists, int k, double *__restrict__ outd,
                                                  int32_t *__restrict__ outi, int final_,
                                                  int32_t *__restrict__ out_idx,
                                                  double *__restrict__ out_dist) {
    const int lane = threadIdx.x & 63;
    const int64_t ngroups = (nlists + 7) / 8;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nq * ngroups) return;
    const int64_t q = w / ngroups, g = w % ngroups;
    double dv[8];
    int ix[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int e = lane + 64 * r;  // list g*8 + e / k, slot e % k
        const int64_t l = g * 8 + e / k;
        const int s = e % k;
        const bool ok = e < 8 * k && l < nlists;
        dv[r] = ok ? ind[(q * nlists + l) * k + s] : __builtin_inf();
        ix[r] = ok ? ini[(q * nlists + l) * k + s] : INT_MAX;
    }
    wave_bitonic_sort<8>(dv, ix);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int e = lane + 64 * r;
        if (e >= k) continue;
        if (final_) {
            const bool ok = ix[r] != INT_MAX;
            out_idx[q * k + e] = ok ? ix[r] : -1;
            out_dist[q * k + e] = ok ? dv[r] : __builtin_inf();
        } else {
            outd[(q * ngroups + g) * k + e] = dv[r];
            outi[(q * ngroups + g) * k + e] = ix[r];
        }
    }
}

}  // namespace kf64
}  // namespace mn

extern "C" int mn_knn_l2_f64(const void *Q, int64_t nq, const void *C, int64_t nc, int32_t d,
                             int32_t x_is_f64, const int64_t *q_ids, int32_t k,
                             int32_t use_sqrt, int32_t *out_idx, double *out_dist,
                             void *stream) {
    using namespace mn;
    using namespace mn::kf64;
    clear_error();
    MN_REQUIRE(Q && C && out_idx && out_dist, MN_EINVAL, "mn_knn_l2_f64: NULL pointer argument");
    MN_REQUIRE(nq >= 0 && nc >= 0 && d >= 1, MN_EINVAL, "mn_knn_l2_f64: bad shape");
    MN_REQUIRE(k >= 1 && k <= KMAX, MN_ENOTSUP, "mn_knn_l2_f64: k=%d outside [1,%d]", k, KMAX);
    MN_REQUIRE(nc <= INT_MAX, MN_EINVAL, "mn_knn_l2_f64: corpus ids must fit int32");
    hipStream_t s = (hipStream_t)stream;
    if (nq == 0) return MN_OK;
    const int64_t ntiles = nc > 0 ? (nc + TC - 1) / TC : 0;
    const int64_t nqb = (nq + TQ - 1) / TQ;
    MN_REQUIRE(nqb < 65536 || ntiles == 0, MN_ENOTSUP,
               "mn_knn_l2_f64: nq=%lld exceeds 65535*32 (batch the queries)", (long long)nq);
    if (ntiles == 0) {
        // no corpus rows: every slot empty
        MN_HIP_TRY(hipMemsetAsync(out_idx, 0xff, sizeof(int32_t) * (size_t)nq * k, s));
        std::vector<double> inf((size_t)nq * k, __builtin_inf());
        MN_HIP_TRY(hipMemcpyAsync(out_dist, inf.data(), inf.size() * 8, hipMemcpyHostToDevice, s));
        MN_HIP_TRY(hipStreamSynchronize(s));
        return MN_OK;
    }
    const size_t per = (size_t)nq * ntiles * k;
    char *g = (char *)scratch(kSlotGeneric0, per * 24 + (size_t)nq * ((ntiles + 7) / 8) * k * 12 + 256);
    int *flag = (int *)scratch(kSlotFlags, 64);
    MN_REQUIRE(g && flag, MN_ENOMEM, "mn_knn_l2_f64: scratch allocation failed");
    double *cd = (double *)g;
    int32_t *ci = (int32_t *)(cd + per);
    // (16-B aligned whatever the parity of per: the merge reads f64 pairs)
    double *cd2 = (double *)(g + ((per * 12 + 64 + 15) & ~(size_t)15));
    int32_t *ci2 = (int32_t *)(cd2 + (size_t)nq * ((ntiles + 7) / 8) * k);
    MN_HIP_TRY(hipMemsetAsync(flag, 0, 4, s));
    const dim3 grid((unsigned)ntiles, (unsigned)nqb);
    if (x_is_f64)
        hipLaunchKernelGGL(k_l2_tile<double>, grid, dim3(256), 0, s, (const double *)Q, nq,
                           (const double *)C, nc, d, q_ids, k, use_sqrt, cd, ci, flag);
    else
        hipLaunchKernelGGL(k_l2_tile<float>, grid, dim3(256), 0, s, (const float *)Q, nq,
                           (const float *)C, nc, d, q_ids, k, use_sqrt, cd, ci, flag);
    MN_KCHECK(s, "k_l2_tile");
    // merge levels: 8 lists per wave until one is left
    int64_t nl = ntiles;
    double *ad = cd, *bd = cd2;
    int32_t *ai = ci, *bi = ci2;
    for (;;) {
        const int64_t ng = (nl + 7) / 8;
        const bool fin = ng == 1;
        const int64_t waves = nq * ng;
        hipLaunchKernelGGL(k_l2_merge, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, ad, ai,
                           nq, nl, k, bd, bi, fin ? 1 : 0, out_idx, out_dist);
        MN_KCHECK(s, "k_l2_merge");
        if (fin) break;
        nl = ng;
        std::swap(ad, bd);
        std::swap(ai, bi);
    }
    int hf = 0;
    MN_HIP_TRY(hipMemcpyAsync(&hf, flag, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hf == 0, MN_ENONFINITE,
               "mn_knn_l2_f64: NaN distance (the reference's partial_cmp().unwrap() panics)");
    return MN_OK;
}
