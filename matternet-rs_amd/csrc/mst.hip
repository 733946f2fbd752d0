// mst.hip — the MST stage's k-NN candidate graph with its default metric
// (surfface-core/src/mst.rs:312-363 build_candidate_graph, DistanceMetric::
// Bhattacharyya) and the thickness-weighted edge costs (mst.rs:400-412).
//
// Reference semantics (f32 throughout):
//   distance.rs:78-108 bhattacharyya_distance_diagonal, per feature k in order:
//     si = var_i[k].max(1e-10); sj = var_j[k].max(1e-10)
//     ss = si + sj; sp = si * sj; md = mean_i[k] - mean_j[k]
//     mahal = 0.25 * (md * md) / ss
//     log_term = 0.25 * (ss / (2 * sqrt(sp))).max(1e-10).ln()
//     distance += mahal + log_term
//   mst.rs:330-344: every j != i, sort_by(partial_cmp) (stable: ties keep j
//   ascending), truncate to k = min(k_neighbors, C - 1).
//   mst.rs:400-412 cost = distance * phi(t_i, t_j), phi by ThicknessWeight
//   (None: cost = distance); thickness = the mean variance of the centroid
//   (centroid.rs:107-109).
//
// Parity: the fold order and every +, *, / are the reference's; the square
// root is correctly rounded (mn::sqrt_rn_f32) like Rust's f32::sqrt, and ln is
// glibc's logf restated on the device (glibc_f32.hpp: bit-identical to the
// platform libm the reference's f32::ln calls, checked on every f32 input).
// Distances and neighbour lists are therefore bit-exact.
//
// GPU design: D(i, j) is symmetric bit for bit (md is negated, squared; ss,
// sp commute), so only the upper 64 x 64 node tiles are computed; a block
// stages a 32-feature chunk of both tiles' means and floored variances in LDS
// (transposed, padded) and every thread folds a 4 x 4 pair block in feature
// order (VALU / transcendental bound: a division pair, a sqrt and a table
// log per term — not a Gram).  The C x C f32 matrix lives in HBM (C <= 65536:
// <= 16 GiB of 288).  Then one wave per node keeps its k best (dist, j) in
// registers over 1024-slot passes of a wave bitonic sort (the carried prefix
// plus the next row chunk), and writes edges + costs.
#include <algorithm>
#include <climits>

#include "common.hpp"
#include "glibc_f32.hpp"

namespace mn {
namespace mst {

constexpr int T = 64;       // node tile
constexpr int FK = 32;      // features per LDS stage
constexpr int NR = 16;      // selection pass: 64 * NR slots
constexpr int KMAX = 512;   // carried neighbours (k) per row
constexpr int64_t CMAX = 65536;
constexpr float EPS = 1e-10f;

__device__ __forceinline__ float bd_term(float mi, float si, float mj, float sj) {
    const float ss = si + sj;
    const float sp = si * sj;
    const float md = mi - mj;
    const float mahal = (0.25f * (md * md)) / ss;
    const float r = fmaxf(ss / (2.0f * sqrt_rn_f32(sp)), EPS);
    const float lt = 0.25f * glibc::logf(r);
    return mahal + lt;
}

__global__ __launch_bounds__(256) void k_bd_matrix(const float *__restrict__ mu,
                                                   const float *__restrict__ var, int64_t C,
                                                   int F, int ntile, float *__restrict__ D) {
    __shared__ float mi[FK][T + 1], si[FK][T + 1], mj[FK][T + 1], sj[FK][T + 1];
    int t = blockIdx.x, bi = 0;
    while (t >= ntile - bi) { t -= ntile - bi; ++bi; }
    const int bj = bi + t;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t i0 = (int64_t)bi * T + 4 * ty, j0 = (int64_t)bj * T + 4 * tx;
    float dd[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) dd[a][b] = 0.0f;
    for (int f0 = 0; f0 < F; f0 += FK) {
        // stage: 64 nodes x 32 features of each tile (coalesced along F)
        for (int e = threadIdx.x; e < FK * T; e += 256) {
            const int node = e / FK, fe = e % FK;
            const int f = f0 + fe;
            const int64_t gi = (int64_t)bi * T + node, gj = (int64_t)bj * T + node;
            float a = 0.f, va = 1.f, b = 0.f, vb = 1.f;
            if (f < F) {
                if (gi < C) { a = mu[gi * F + f]; va = fmaxf(var[gi * F + f], EPS); }
                if (gj < C) { b = mu[gj * F + f]; vb = fmaxf(var[gj * F + f], EPS); }
            }
            mi[fe][node] = a; si[fe][node] = va;
            mj[fe][node] = b; sj[fe][node] = vb;
        }
        __syncthreads();
        const int fn = min(FK, F - f0);
        for (int fe = 0; fe < fn; ++fe) {
            float ma[4], va[4], mb[4], vb[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) { ma[a] = mi[fe][4 * ty + a]; va[a] = si[fe][4 * ty + a]; }
#pragma unroll
            for (int b = 0; b < 4; ++b) { mb[b] = mj[fe][4 * tx + b]; vb[b] = sj[fe][4 * tx + b]; }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) dd[a][b] = dd[a][b] + bd_term(ma[a], va[a], mb[b], vb[b]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int64_t i = i0 + a, j = j0 + b;
            if (i >= C || j >= C) continue;
            D[i * C + j] = dd[a][b];
            D[j * C + i] = dd[a][b];
        }
}

__device__ __forceinline__ float edge_cost(float dist, float ti, float tj, int tw) {
    float phi;
    switch (tw) {
    case MN_TW_MEAN: phi = (ti + tj) / 2.0f; break;
    case MN_TW_MIN: phi = fminf(ti, tj); break;
    case MN_TW_MAX: phi = fmaxf(ti, tj); break;
    case MN_TW_GEOMEAN: phi = sqrt_rn_f32(ti * tj); break;
    default: return dist;  // MN_TW_NONE
    }
    return dist * phi;
}

// per node i: the kk best (dist, j), j != i, of row i of D, ascending
__global__ __launch_bounds__(256) void k_bd_select(const float *__restrict__ D, int64_t C, int kk,
                                                   const float *__restrict__ th, int tw,
                                                   int32_t *__restrict__ out_v,
                                                   float *__restrict__ out_dist,
                                                   float *__restrict__ out_cost,
                                                   int *__restrict__ nonfinite) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= C) return;
    const float *row = D + i * C;
    float key[NR];
    int ix[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) { key[r] = __builtin_inff(); ix[r] = INT_MAX; }
    bool bad = false;
    int carry = 0;
    for (int64_t j0 = 0; j0 < C;) {
        const int fresh = 64 * NR - carry;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int e = lane + 64 * r;
            if (e >= carry) {
                const int64_t j = j0 + (e - carry);
                const bool ok = j < C && j != i;
                const float v = ok ? row[j] : __builtin_inff();
                bad |= (v != v);
                key[r] = ok ? v : __builtin_inff();
                ix[r] = ok ? (int)j : INT_MAX;
            }
        }
        wave_bitonic_sort<NR>(key, ix);
        j0 += fresh;
        carry = kk;
    }
    if (__any(bad)) {
        if (lane == 0) atomicOr(nonfinite, 1);
        return;
    }
    const float ti = th[i];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        if (e < kk) {
            const int j = ix[r];
            out_v[i * kk + e] = j;
            out_dist[i * kk + e] = key[r];
            out_cost[i * kk + e] = edge_cost(key[r], ti, th[j], tw);
        }
    }
}

// centroid.rs:107-109 get_thickness = variances.mean_dim(1): sequential f32
// sum over the row, then / F (Burn's summation order is backend-defined:
// parity of this helper is unpinned; callers may pass their own thickness)
__global__ void k_thickness(const float *__restrict__ var, int64_t C, int F,
                            float *__restrict__ th) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C) return;
    float s = 0.0f;
    for (int f = 0; f < F; ++f) s = s + var[i * F + f];
    th[i] = s / (float)F;
}

__global__ void k_l2_costs(const int32_t *__restrict__ v, const float *__restrict__ dist,
                           int64_t n, int kk, const float *__restrict__ th, int tw,
                           float *__restrict__ cost) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * kk) return;
    cost[e] = edge_cost(dist[e], th[e / kk], th[v[e]], tw);
}

inline unsigned grid(int64_t n, int t) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

}  // namespace mst

static int mst_candidates_impl(const float *means, const float *vars, int64_t C, int32_t F,
                               int32_t k_neighbors, int32_t metric, int32_t tw,
                               const float *thickness, float *out_thickness, int32_t *out_v,
                               float *out_dist, float *out_cost, void *stream) {
    using namespace mst;
    clear_error();
    MN_REQUIRE(means && out_v && out_dist && out_cost, MN_EINVAL,
               "mn_mst_candidate_graph_f32: NULL pointer");
    MN_REQUIRE(C >= 2 && F >= 1, MN_EINVAL, "mn_mst_candidate_graph_f32: need C >= 2, F >= 1");
    MN_REQUIRE(k_neighbors >= 1, MN_EINVAL, "mn_mst_candidate_graph_f32: k_neighbors >= 1");
    MN_REQUIRE(metric >= MN_MST_BHATTACHARYYA && metric <= MN_MST_SQEUCLIDEAN, MN_EINVAL,
               "mn_mst_candidate_graph_f32: bad metric %d", metric);
    MN_REQUIRE(tw >= MN_TW_MEAN && tw <= MN_TW_NONE, MN_EINVAL,
               "mn_mst_candidate_graph_f32: bad thickness weight %d", tw);
    MN_REQUIRE(thickness || vars, MN_EINVAL,
               "mn_mst_candidate_graph_f32: thickness needs the variances");
    const int64_t kk = std::min<int64_t>(k_neighbors, C - 1);  // mst.rs:317
    hipStream_t s = (hipStream_t)stream;
    // thickness (after the kNN of the L2 metrics: it uses the generic scratch slots)
    float *th = nullptr;
    auto thickness_pass = [&]() -> int {
        th = (float *)scratch(kSlotGeneric1, sizeof(float) * (size_t)C + 64);
        MN_REQUIRE(th, MN_ENOMEM, "mn_mst_candidate_graph_f32: scratch allocation failed");
        if (thickness) {
            MN_HIP_TRY(hipMemcpyAsync(th, thickness, sizeof(float) * (size_t)C,
                                      hipMemcpyDeviceToDevice, s));
        } else {
            hipLaunchKernelGGL(k_thickness, dim3(grid(C, 256)), dim3(256), 0, s, vars, C, F, th);
            MN_KCHECK(s, "k_thickness");
        }
        if (out_thickness)
            MN_HIP_TRY(hipMemcpyAsync(out_thickness, th, sizeof(float) * (size_t)C,
                                      hipMemcpyDeviceToDevice, s));
        return MN_OK;
    };
    if (metric != MN_MST_BHATTACHARYYA) {
        // mst.rs:383-397: the squared-L2 fold (Euclidean: its f32 sqrt) — the K1 kNN
        mn_knn_opts o{};
        o.k = (int32_t)kk;
        o.metric = metric == MN_MST_EUCLIDEAN ? MN_L2 : MN_L2SQ;
        o.exclude_self = 1;
        o.stream = stream;
        int rc = mn_knn_f32(means, C, F, &o, out_v, out_dist);
        if (rc != MN_OK) return rc;
        rc = thickness_pass();
        if (rc != MN_OK) return rc;
        hipLaunchKernelGGL(k_l2_costs, dim3(grid(C * kk, 256)), dim3(256), 0, s, out_v, out_dist,
                           C, (int)kk, th, tw, out_cost);
        MN_KCHECK(s, "k_l2_costs");
        MN_HIP_TRY(hipStreamSynchronize(s));
        return MN_OK;
    }
    MN_REQUIRE(vars, MN_EINVAL, "mn_mst_candidate_graph_f32: Bhattacharyya needs variances");
    MN_REQUIRE(C <= CMAX, MN_ENOTSUP, "mn_mst_candidate_graph_f32: C <= %lld centroids",
               (long long)CMAX);
    MN_REQUIRE(kk <= KMAX, MN_ENOTSUP, "mn_mst_candidate_graph_f32: k <= %d", KMAX);
    {
        const int rc = thickness_pass();
        if (rc != MN_OK) return rc;
    }
    int *flags = (int *)scratch(kSlotFlags, 64);
    float *D = (float *)scratch(kSlotGeneric0, sizeof(float) * (size_t)C * C + 64);
    MN_REQUIRE(D && flags, MN_ENOMEM, "mn_mst_candidate_graph_f32: %lld x %lld matrix allocation failed",
               (long long)C, (long long)C);
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 16, s));
    const int64_t ntile = (C + T - 1) / T;
    hipLaunchKernelGGL(k_bd_matrix, dim3((unsigned)(ntile * (ntile + 1) / 2)), dim3(256), 0, s,
                       means, vars, C, F, (int)ntile, D);
    MN_KCHECK(s, "k_bd_matrix");
    hipLaunchKernelGGL(k_bd_select, dim3(grid(C, 4)), dim3(256), 0, s, D, C, (int)kk, th, tw,
                       out_v, out_dist, out_cost, flags);
    MN_KCHECK(s, "k_bd_select");
    int hf = 0;
    MN_HIP_TRY(hipMemcpyAsync(&hf, flags, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hf == 0, MN_ENONFINITE,
               "mn_mst_candidate_graph_f32: NaN distance (the reference panics in "
               "partial_cmp().unwrap())");
    return MN_OK;
}

}  // namespace mn

extern "C" int mn_mst_candidate_graph_f32(const float *means, const float *vars, int64_t c,
                                          int32_t f, int32_t k_neighbors, int32_t metric,
                                          int32_t thickness_weight, const float *thickness,
                                          float *out_thickness, int32_t *out_v, float *out_dist,
                                          float *out_cost, void *stream) {
    return mn::mst_candidates_impl(means, vars, c, f, k_neighbors, metric, thickness_weight,
                                   thickness, out_thickness, out_v, out_dist, out_cost, stream);
}
