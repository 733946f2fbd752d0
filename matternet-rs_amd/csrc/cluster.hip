// cluster.hip — the batch nearest-centroid step of the clustering stage
// (surfface-pipeline/src/stages/clustering.rs:42-63): per item of a batch,
// the nearest current centroid by the Gram-form Euclidean distance
//
//     d(i, j) = sqrt(|x_i|^2 + |c_j|^2 - 2 x_i . c_j)      (f32)
//
// then min_dim / argmin over j.  The stage's incremental centroid logic
// (:65-88) stays on the host, as in the reference (which downloads every
// batch's results to the CPU for it).
//
// Parity: Burn evaluates |x|^2 (powf_scalar(2).sum_dim), the matmul and the
// reductions in a backend-defined order, so the reference's bits are not
// reproducible from its source (parity-unpinned).  This kernel fixes the
// order — sequential non-contracted f32 folds over the features for the norms
// and the dot, (|x|^2 + |c|^2) - 2 dot, a correctly rounded sqrt, the FIRST
// index of the minimum (NaN from a negative radicand never wins) — and is
// bit-exact against the oracle's restatement of exactly that.
//
// GPU design: 64 x 64 (item, centroid) tiles, 32-feature LDS stages of both
// row blocks (transposed, padded), 4 x 4 pairs per thread folded in feature
// order (VALU, like mst.hip); the B x C distances go to HBM and one wave per
// item takes the argmin.
#include <algorithm>
#include <climits>

#include "common.hpp"

namespace mn {
namespace clu {

constexpr int T = 64;
constexpr int FK = 32;

// sequential f32 sum of squares of each row
__global__ void k_row_sq(const float *__restrict__ X, int64_t n, int F, float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.0f;
    for (int f = 0; f < F; ++f) {
        const float x = X[i * F + f];
        s = s + x * x;
    }
    out[i] = s;
}

__global__ __launch_bounds__(256) void k_gram_dist(const float *__restrict__ Xb, int64_t B,
                                                   const float *__restrict__ Cm, int64_t C, int F,
                                                   int64_t ntj, const float *__restrict__ bn,
                                                   const float *__restrict__ cn,
                                                   float *__restrict__ D) {
    __shared__ float xa[FK][T + 1], ca[FK][T + 1];
    const int64_t bi = blockIdx.x / ntj, bj = blockIdx.x % ntj;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float dot[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) dot[a][b] = 0.0f;
    for (int f0 = 0; f0 < F; f0 += FK) {
        for (int e = threadIdx.x; e < FK * T; e += 256) {
            const int r = e / FK, fe = e % FK, f = f0 + fe;
            const int64_t gi = bi * T + r, gj = bj * T + r;
            xa[fe][r] = (f < F && gi < B) ? Xb[gi * F + f] : 0.f;
            ca[fe][r] = (f < F && gj < C) ? Cm[gj * F + f] : 0.f;
        }
        __syncthreads();
        const int fn = min(FK, F - f0);
        for (int fe = 0; fe < fn; ++fe) {
            float xv[4], cv[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) xv[a] = xa[fe][4 * ty + a];
#pragma unroll
            for (int b = 0; b < 4; ++b) cv[b] = ca[fe][4 * tx + b];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) dot[a][b] = dot[a][b] + xv[a] * cv[b];
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int64_t i = bi * T + 4 * ty + a, j = bj * T + 4 * tx + b;
            if (i >= B || j >= C) continue;
            const float v = (bn[i] + cn[j]) - 2.0f * dot[a][b];
            D[i * C + j] = sqrt_rn_f32(v);  // NaN for v < 0 (as the reference's sqrt)
        }
}

// one wave per item: first index of the minimum (NaN never wins)
__global__ __launch_bounds__(256) void k_row_argmin(const float *__restrict__ D, int64_t B,
                                                    int64_t C, int32_t *__restrict__ out_idx,
                                                    float *__restrict__ out_dist) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= B) return;
    float best = __builtin_nanf("");
    int bj = INT_MAX;
    for (int64_t j = lane; j < C; j += 64) {
        const float v = D[i * C + j];
        if (v == v && (best != best || v < best)) { best = v; bj = (int)j; }  // j ascends per lane
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o);
        const int oj = __shfl_xor(bj, o);
        const bool take = (ob == ob) && (best != best || ob < best || (ob == best && oj < bj));
        if (take) { best = ob; bj = oj; }
    }
    if (lane == 0) {
        out_idx[i] = bj == INT_MAX ? 0 : (int32_t)bj;
        out_dist[i] = bj == INT_MAX ? D[i * C] : best;
    }
}

inline unsigned grid(int64_t n, int t) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

}  // namespace clu

static int nearest_centroid_impl(const float *batch, int64_t B, const float *cents, int64_t C,
                                 int32_t F, int32_t *out_idx, float *out_dist, void *stream) {
    using namespace clu;
    clear_error();
    MN_REQUIRE(batch && cents && out_idx && out_dist, MN_EINVAL,
               "mn_nearest_centroid_f32: NULL pointer");
    MN_REQUIRE(B >= 1 && C >= 1 && F >= 1, MN_EINVAL, "mn_nearest_centroid_f32: empty input");
    MN_REQUIRE(C <= (int64_t)INT_MAX, MN_ENOTSUP, "mn_nearest_centroid_f32: too many centroids");
    hipStream_t s = (hipStream_t)stream;
    float *D = (float *)scratch(kSlotGeneric0, sizeof(float) * ((size_t)B * C + B + C) + 64);
    MN_REQUIRE(D, MN_ENOMEM, "mn_nearest_centroid_f32: scratch allocation failed");
    float *bn = D + (size_t)B * C, *cn = bn + B;
    hipLaunchKernelGGL(k_row_sq, dim3(grid(B, 256)), dim3(256), 0, s, batch, B, F, bn);
    hipLaunchKernelGGL(k_row_sq, dim3(grid(C, 256)), dim3(256), 0, s, cents, C, F, cn);
    MN_KCHECK(s, "k_row_sq");
    const int64_t nti = (B + T - 1) / T, ntj = (C + T - 1) / T;
    MN_REQUIRE(nti * ntj < INT_MAX, MN_ENOTSUP, "mn_nearest_centroid_f32: grid too large");
    hipLaunchKernelGGL(k_gram_dist, dim3((unsigned)(nti * ntj)), dim3(256), 0, s, batch, B, cents, C,
                       F, ntj, bn, cn, D);
    MN_KCHECK(s, "k_gram_dist");
    hipLaunchKernelGGL(k_row_argmin, dim3(grid(B, 4)), dim3(256), 0, s, D, B, C, out_idx, out_dist);
    MN_KCHECK(s, "k_row_argmin");
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

}  // namespace mn

extern "C" int mn_nearest_centroid_f32(const float *batch, int64_t b, const float *centroids,
                                       int64_t c, int32_t f, int32_t *out_idx, float *out_dist,
                                       void *stream) {
    return mn::nearest_centroid_impl(batch, b, centroids, c, f, out_idx, out_dist, stream);
}
