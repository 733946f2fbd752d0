// bc.hip — Stage C feature kNN by Bhattacharyya coefficient (§8(f) rank 3).
//
// Reference semantics (f32 throughout):
//   surfface-core/src/distance.rs:260-290 bhattacharyya_coefficient
//     for c in 0..C (sequential f32 fold):
//       vi = max(var_i[c], reg); vj = max(var_j[c], reg); v = vi + vj
//       db += (mu_i[c] - mu_j[c])^2 / (4 v) + 0.5 ln(v / (2 sqrt(vi vj)))
//     BC = clamp(exp(-db), 0, 1)
//   surfface-core/src/laplacian.rs:254-298 compute_bhattacharyya_weights
//     nodes = the F feature columns of the [C, F] centroid means / variances
//     (transpose_to_feature_profiles, :233-238); per node i every j != i with
//     BC > weight_threshold, sorted by BC descending (sort_unstable: ties
//     unspecified — here j ascending), truncated to k = min(k, F - 1).
//
// Parity: the fold order, every +, *, / and the square root are the
// reference's (sqrt correctly rounded via mn::sqrt_rn_f32, f32 division is
// correctly rounded); ln / exp are glibc's logf / expf restated on the device
// (glibc_f32.hpp: bit-identical to the platform libm the reference's f32::ln /
// f32::exp call, checked on every f32 input), so BC and the neighbour sets are
// bit-exact.
//
// GPU design: BC is symmetric bit for bit (every operation commutes in i, j),
// so only the upper 64 x 64 tiles are computed; a block stages a 32-centroid
// chunk of both tiles' means and floored variances in LDS and every thread
// folds a 4 x 4 pair block in centroid order (VALU / transcendental bound:
// ~2 divisions, a sqrt and a log per term — not a Gram, no MFMA).  Then one
// wave per node selects its top k with a register bitonic sort on
// (-BC, j).
#include <algorithm>
#include <climits>

#include "common.hpp"
#include "glibc_f32.hpp"

namespace mn {
namespace bc {

constexpr int T = 64;    // node tile
constexpr int CK = 32;   // centroids per LDS stage
constexpr int FMAXB = 4096;

__global__ __launch_bounds__(256) void k_bc_matrix(const float *__restrict__ mu,
                                                   const float *__restrict__ var, int64_t C, int F,
                                                   int ntile, float reg, float *__restrict__ BC,
                                                   int *__restrict__ nonfinite) {
    __shared__ float mi[CK][T], vi_[CK][T], mj[CK][T], vj_[CK][T];
    int t = blockIdx.x, bi = 0;
    while (t >= ntile - bi) { t -= ntile - bi; ++bi; }
    const int bj = bi + t;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i0 = bi * T + 4 * ty, j0 = bj * T + 4 * tx;
    float db[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) db[a][b] = 0.0f;
    for (int64_t c0 = 0; c0 < C; c0 += CK) {
        // stage: 32 centroid rows x 64 nodes of each tile (coalesced along F)
        for (int e = threadIdx.x; e < CK * T; e += 256) {
            const int cr = e / T, col = e % T;
            const int64_t c = c0 + cr;
            const int gi = bi * T + col, gj = bj * T + col;
            float a = 0.f, va = 1.f, b = 0.f, vb = 1.f;
            if (c < C) {
                if (gi < F) { a = mu[c * F + gi]; va = fmaxf(var[c * F + gi], reg); }
                if (gj < F) { b = mu[c * F + gj]; vb = fmaxf(var[c * F + gj], reg); }
            }
            mi[cr][col] = a; vi_[cr][col] = va;
            mj[cr][col] = b; vj_[cr][col] = vb;
        }
        __syncthreads();
        const int cn = (int)min<int64_t>(CK, C - c0);
        for (int cr = 0; cr < cn; ++cr) {
            float ma[4], va[4], mb[4], vb[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) { ma[a] = mi[cr][4 * ty + a]; va[a] = vi_[cr][4 * ty + a]; }
#pragma unroll
            for (int b = 0; b < 4; ++b) { mb[b] = mj[cr][4 * tx + b]; vb[b] = vj_[cr][4 * tx + b]; }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const float vs = va[a] + vb[b];
                    const float d = ma[a] - mb[b];
                    const float mean_term = (d * d) / (4.0f * vs);
                    const float log_term =
                        0.5f * glibc::logf(vs / (2.0f * sqrt_rn_f32(va[a] * vb[b])));
                    db[a][b] = db[a][b] + (mean_term + log_term);
                }
        }
        __syncthreads();
    }
    bool bad = false;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int i = i0 + a, j = j0 + b;
            if (i >= F || j >= F) continue;
            float w = glibc::expf(-db[a][b]);
            bad |= (w != w);
            w = w < 0.f ? 0.f : (w > 1.f ? 1.f : w);  // NaN stays NaN
            BC[(int64_t)i * F + j] = w;
            BC[(int64_t)j * F + i] = w;
        }
    if (bad) atomicOr(nonfinite, 1);
}

// per node: the k largest BC > thr over j != i, ordered (BC desc, j asc)
template <int NR>
__global__ __launch_bounds__(256) void k_bc_select(const float *__restrict__ BC, int F, int k,
                                                   float thr, int32_t *__restrict__ out_idx,
                                                   float *__restrict__ out_w) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= F) return;
    float key[NR];
    int ix[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int j = lane + 64 * r;
        const float w = (j < F && j != i) ? BC[(int64_t)i * F + j] : 0.f;
        const bool ok = j < F && j != i && w > thr;
        key[r] = ok ? -w : __builtin_inff();
        ix[r] = ok ? j : INT_MAX;
    }
    wave_bitonic_sort<NR>(key, ix);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;  // sorted position
        if (e < k) {
            const bool ok = ix[r] != INT_MAX;
            out_idx[(int64_t)i * k + e] = ok ? ix[r] : -1;
            out_w[(int64_t)i * k + e] = ok ? -key[r] : 0.f;
        }
    }
    for (int e = 64 * NR + lane; e < k; e += 64) {  // k beyond the F - 1 candidates
        out_idx[(int64_t)i * k + e] = -1;
        out_w[(int64_t)i * k + e] = 0.f;
    }
}

inline unsigned grid(int64_t n, int t) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

}  // namespace bc

static int bc_knn_impl(const float *means, const float *vars, int64_t C, int32_t F, int32_t k,
                       float reg, float thr, int32_t *out_idx, float *out_w, void *stream) {
    using namespace bc;
    clear_error();
    MN_REQUIRE(means && vars && out_idx && out_w, MN_EINVAL, "mn_bc_knn_f32: NULL pointer");
    MN_REQUIRE(C >= 1 && F >= 2 && F <= FMAXB, MN_EINVAL,
               "mn_bc_knn_f32: need C >= 1 and 2 <= F <= %d", FMAXB);
    MN_REQUIRE(k >= 1, MN_EINVAL, "mn_bc_knn_f32: k must be >= 1");
    hipStream_t s = (hipStream_t)stream;
    const int kk = std::min(k, F - 1);  // laplacian.rs:260 k.min(F - 1)
    float *BCm = (float *)scratch(kSlotGeneric0, sizeof(float) * (size_t)F * F + 64);
    int *flags = (int *)scratch(kSlotFlags, 64);
    MN_REQUIRE(BCm && flags, MN_ENOMEM, "mn_bc_knn_f32: scratch allocation failed");
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 16, s));
    const int ntile = (F + T - 1) / T;
    hipLaunchKernelGGL(k_bc_matrix, dim3((unsigned)(ntile * (ntile + 1) / 2)), dim3(256), 0, s,
                       means, vars, C, F, ntile, reg, BCm, flags);
    MN_KCHECK(s, "k_bc_matrix");
    int hf = 0;
    MN_HIP_TRY(hipMemcpyAsync(&hf, flags, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hf == 0, MN_ENONFINITE,
               "mn_bc_knn_f32: NaN coefficient (the reference panics in partial_cmp().unwrap())");
    const int nr = (F + 63) / 64;
    // k slots per row: at most kk = min(k, F - 1) valid, the rest -1 / 0
    (void)kk;
#define MN_BS(NRV) hipLaunchKernelGGL(k_bc_select<NRV>, dim3(grid(F, 4)), dim3(256), 0, s, BCm, F, k, thr, out_idx, out_w)
    if (nr <= 1) MN_BS(1); else if (nr <= 2) MN_BS(2); else if (nr <= 4) MN_BS(4);
    else if (nr <= 8) MN_BS(8); else if (nr <= 16) MN_BS(16); else if (nr <= 32) MN_BS(32);
    else MN_BS(64);
#undef MN_BS
    MN_KCHECK(s, "k_bc_select");
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

}  // namespace mn

extern "C" int mn_bc_knn_f32(const float *means, const float *vars, int64_t c, int32_t f,
                             int32_t k, float var_reg, float weight_thr, int32_t *out_idx,
                             float *out_w, void *stream) {
    return mn::bc_knn_impl(means, vars, c, f, k, var_reg, weight_thr, out_idx, out_w, stream);
}
