// search.hip — §8(f) rank 2: the lambda-aware query path (batched).
//
// Reference semantics (src_legacy/core.rs):
//   search_lambda_aware(query, k, alpha)  :1156-1193
//     for i in 0..nitems: s_i = query.lambda_similarity(item_i, alpha)
//     results.sort_by(|a, b| b.1.partial_cmp(&a.1).unwrap()); truncate(k)
//   lambda_similarity :162-179  = alpha*cos + (1-alpha)*lambda_sim
//   lambda_component_similarity :141-144 = 1 - min(|lq - li|, 1)
//   cosine_similarity :233-244 = dot / (norm(q)*norm(x)) if that product > 0 else 0
//   norm :210-214 (sequential f64 sum of x*x, sqrt), dot :196-205 (sequential
//   f64 sum of a*b) — no FMA contraction (Makefile: -ffp-contract=off).
//   sort_by is stable over ascending i => order = (score desc, i asc).
//
// GPU design (HBM stream of X, f64 VALU chains):
//   k_lambda_scores: one block = 256 items x 32 queries.  Items stream through
//     LDS in 32-feature slabs (row-coalesced loads, stored transposed), the
//     query slab beside them; each lane owns a 4-item x 8-query register
//     micro-tile (one 16-B item read + 8 broadcast query reads per 32 f64
//     mul/add) and one item-norm chain, all folded in the reference's order.
//     Each wave then sorts its queries' 256 (-score, i) keys straight from
//     registers (bitonic, key_less) and writes the top k.
//   k_topk_reduce: waves sort 512-candidate chunks and keep the top k until one
//     chunk is left (k <= 256 => each level at least halves the candidates).
//   (score desc, i asc) is a total order, so per-tile selection + merges give
//   exactly the reference's truncated stable sort.
#include <climits>
#include <cmath>
#include <type_traits>

#include "common.hpp"

namespace mn {
namespace srch {

constexpr int kTile = 256;  // items per block
constexpr int kSlab = 32;   // features per LDS slab
constexpr int kQB = 32;     // queries per block (8 per wave)
constexpr int kChunk = 512; // candidates per reduce wave
constexpr int kMaxK = 256;

enum : int { kFlagNan = 1, kFlagZeroLambda = 2 };

__global__ void k_query_norms(const double *__restrict__ Q, int64_t nq, int32_t f,
                              const double *__restrict__ lq, double *__restrict__ qn,
                              int *__restrict__ flag) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const double *a = Q + q * f;
    double s = 0.0;
    for (int32_t t = 0; t < f; ++t) s = s + a[t] * a[t];
    qn[q] = __builtin_sqrt(s);
    if (lq[q] == 0.0) atomicOr(flag, kFlagZeroLambda);  // core.rs:1169-1172 assert_ne!
}

template <typename T>
__global__ __launch_bounds__(256) void k_lambda_scores(
    const T *__restrict__ X, int64_t n, int32_t f, const double *__restrict__ lambdas,
    const double *__restrict__ Q, const double *__restrict__ qn, const double *__restrict__ lq,
    int64_t nq, double alpha, int32_t kk, int64_t ntiles, double *__restrict__ ck,
    int32_t *__restrict__ ci, int *__restrict__ flag) {
    // xs: the item slab transposed, [feature][item] (+4 pad: 16-B aligned rows,
    // two-way bank aliasing on the transposing stores); qs: [feature][query]
    __shared__ __attribute__((aligned(16))) T xs[kSlab][kTile + 4];
    __shared__ __attribute__((aligned(16))) double qs[kSlab][kQB];
    __shared__ double xns[kTile];

    const int t = threadIdx.x;
    const int w = t >> 6, lane = t & 63;
    const int64_t tile = blockIdx.x;
    const int64_t i0 = tile * kTile;
    const int64_t q0 = (int64_t)blockIdx.y * kQB;
    const int nqb = (int)min((int64_t)kQB, nq - q0);
    // micro-tile: items 4*lane .. 4*lane+3 x queries kQW*w .. kQW*w+kQW-1
    constexpr int kQW = kQB / 4;

    double acc[4][kQW];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int q = 0; q < kQW; ++q) acc[a][q] = 0.0;
    double nrm = 0.0;  // norm chain of item 4*lane + w

    // slab element p of thread t: row 8p + t/32, feature t%32 (two 128-B row
    // segments per wave load).  The next slab's loads are issued before the
    // current slab's chains so their latency hides under the f64 VALU work.
    const int lc = t & (kSlab - 1), lr = t >> 5;
    // buffer descriptor over this tile's rows (wave-uniform inputs made
    // provably uniform): rows >= n fall outside num_records and read as 0
    const uint64_t tb = (uint64_t)(X + i0 * (int64_t)f);
    const int32_t nbytes = __builtin_amdgcn_readfirstlane(
        (int32_t)(min((int64_t)kTile, n - i0) * f * (int64_t)sizeof(T)));
    const uint64_t tbu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(tb >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)tb);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)tbu, (short)0, nbytes, 0x00020000);
    T v[kSlab];
    auto load_slab = [&](int32_t f0) {
        const int cc = min(lc, f - f0 - 1);
        const int voff = (lr * f + cc) * (int)sizeof(T);
#pragma unroll
        for (int p = 0; p < kSlab; ++p) {
            const int soff = (8 * p * f + f0) * (int)sizeof(T);
            if constexpr (sizeof(T) == 4)
                v[p] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
            else
                v[p] = __longlong_as_double(
                    (long long)__builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
        }
    };
    load_slab(0);
    for (int32_t f0 = 0; f0 < f; f0 += kSlab) {
        const int cn = min(kSlab, f - f0);
#pragma unroll
        for (int p = 0; p < kSlab; ++p) {
            const bool ok = (i0 + 8 * p + lr < n) && lc < cn;
            xs[lc][8 * p + lr] = ok ? v[p] : T(0);
        }
        for (int e = t; e < kSlab * kQB; e += kTile) {
            const int c = e / kQB, q = e % kQB;
            qs[c][q] = (q < nqb && c < cn) ? Q[(q0 + q) * f + f0 + c] : 0.0;
        }
        __syncthreads();
        if (f0 + kSlab < f) load_slab(f0 + kSlab);
        for (int c = 0; c < cn; ++c) {
            T xv[4];
            *reinterpret_cast<typename std::conditional<sizeof(T) == 4, float4, double4>::type *>(xv) =
                *reinterpret_cast<const typename std::conditional<sizeof(T) == 4, float4,
                                                                  double4>::type *>(&xs[c][4 * lane]);
            double qv[kQW];
#pragma unroll
            for (int q = 0; q < kQW; ++q) qv[q] = qs[c][kQW * w + q];
            const double xw = (double)xv[w & 3];
            nrm = nrm + xw * xw;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const double x = (double)xv[a];
                double pr[kQW];  // products first, then the chain adds
#pragma unroll
                for (int q = 0; q < kQW; ++q) pr[q] = qv[q] * x;
#pragma unroll
                for (int q = 0; q < kQW; ++q) acc[a][q] = acc[a][q] + pr[q];
            }
        }
        __syncthreads();
    }
    xns[4 * lane + w] = __builtin_sqrt(nrm);
    __syncthreads();

    int nan = 0;
    double d[kQW][4];
    int ix[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int64_t i = i0 + 4 * lane + a;
        const bool live = i < n;
        ix[a] = live ? (int)i : INT_MAX;
        const double xn = xns[4 * lane + a];
        const double li = live ? lambdas[i] : 0.0;
#pragma unroll
        for (int q = 0; q < kQW; ++q) {
            const int qq = kQW * w + q;
            double key = INFINITY;  // sorts after every live item
            if (live && qq < nqb) {
                const double denom = qn[q0 + qq] * xn;
                const double cs = denom > 0.0 ? acc[a][q] / denom : 0.0;
                const double ls = 1.0 - fmin(fabs(lq[q0 + qq] - li), 1.0);
                const double sc = alpha * cs + (1.0 - alpha) * ls;
                nan |= (sc != sc);
                key = -sc;
            }
            d[q][a] = key;
        }
    }
    if (nan) atomicOr(flag, kFlagNan);
    // each wave holds its queries' 256 keys in registers (4 per lane): sort
    // them in place (positions are irrelevant to the selection) and write the
    // top kk
#pragma unroll
    for (int q = 0; q < kQW; ++q) {
        const int qq = kQW * w + q;
        if (qq >= nqb) break;  // wave-uniform
        int jx[4] = {ix[0], ix[1], ix[2], ix[3]};
        wave_bitonic_sort<4>(d[q], jx);
        double *okey = ck + ((q0 + qq) * ntiles + tile) * kk;
        int32_t *oidx = ci + ((q0 + qq) * ntiles + tile) * kk;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = lane + 64 * r;
            if (e < kk) { okey[e] = d[q][r]; oidx[e] = jx[r]; }
        }
    }
}

// One wave per 512-candidate chunk of one query.  Not final: keep the chunk's
// top kk as the next level's input.  Final (one chunk per query): write the
// first min(k, n) results as (i, score), padding with (-1, NaN).
__global__ __launch_bounds__(256) void k_topk_reduce(
    const double *__restrict__ ink, const int32_t *__restrict__ ini, int64_t m, int64_t nq,
    int32_t kk, int64_t nchunks, double *__restrict__ outk, int32_t *__restrict__ outi,
    int32_t final_, int32_t k, int64_t n, int64_t *__restrict__ out_idx,
    double *__restrict__ out_score) {
    const int lane = threadIdx.x & 63;
    const int64_t chunk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t q = blockIdx.y;
    if (chunk >= nchunks || q >= nq) return;
    double d[8];
    int ix[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int64_t e = chunk * kChunk + lane + 64 * r;
        if (e < m) { d[r] = ink[q * m + e]; ix[r] = ini[q * m + e]; }
        else { d[r] = INFINITY; ix[r] = INT_MAX; }
    }
    wave_bitonic_sort<8>(d, ix);
    if (!final_) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int e = lane + 64 * r;
            if (e < kk) {
                outk[(q * nchunks + chunk) * kk + e] = d[r];
                outi[(q * nchunks + chunk) * kk + e] = ix[r];
            }
        }
        return;
    }
    const int64_t c = min((int64_t)k, n);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int e = lane + 64 * r;
        if (e < k) {
            const bool ok = e < c;
            out_idx[q * k + e] = ok ? (int64_t)ix[r] : -1;
            out_score[q * k + e] = ok ? -d[r] : NAN;
        }
    }
}

}  // namespace srch
}  // namespace mn

extern "C" int mn_search_lambda_aware(const void *X, int32_t x_is_f64, int64_t n, int32_t f,
                                      const double *lambdas, const double *Q,
                                      const double *lambda_q, int64_t nq, int32_t k, double alpha,
                                      int64_t *out_idx, double *out_score, void *stream) {
    using namespace mn::srch;
    mn::clear_error();
    MN_REQUIRE(n >= 0 && f >= 0 && nq >= 0 && k >= 0, MN_EINVAL,
               "mn_search_lambda_aware: bad sizes");
    MN_REQUIRE(k <= kMaxK, MN_ENOTSUP, "mn_search_lambda_aware: k=%d > %d", k, kMaxK);
    MN_REQUIRE(n < INT_MAX, MN_ENOTSUP, "mn_search_lambda_aware: n >= 2^31");
    MN_REQUIRE((int64_t)kTile * f * 8 < INT_MAX, MN_ENOTSUP,
               "mn_search_lambda_aware: f too large for 32-bit tile offsets");
    MN_REQUIRE(nq == 0 || k == 0 || (Q && lambda_q && out_idx && out_score &&
                                     (n == 0 || (X && lambdas))),
               MN_EINVAL, "mn_search_lambda_aware: NULL pointer");
    MN_REQUIRE(std::isfinite(alpha), MN_EINVAL, "mn_search_lambda_aware: alpha not finite");
    if (nq == 0 || k == 0) return MN_OK;
    hipStream_t s = (hipStream_t)stream;

    const int64_t ntiles = (n + kTile - 1) / kTile;
    const int32_t kk = (int32_t)std::min<int64_t>(k, kTile);
    int *flag = (int *)mn::scratch(mn::kSlotFlags, sizeof(int));
    double *qn = (double *)mn::scratch(mn::kSlotNorms, sizeof(double) * (size_t)nq);
    MN_REQUIRE(flag && qn, MN_ENOMEM, "mn_search_lambda_aware: scratch");
    MN_HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), s));
    hipLaunchKernelGGL(k_query_norms, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, Q, nq,
                       f, lambda_q, qn, flag);
    MN_KCHECK(s, "k_query_norms");

    int64_t m = ntiles * kk;  // candidates per query
    const size_t cap = (size_t)nq * (size_t)std::max<int64_t>(m, 1);
    double *ka = (double *)mn::scratch(mn::kSlotGeneric0, sizeof(double) * cap);
    int32_t *ia = (int32_t *)mn::scratch(mn::kSlotGeneric1, sizeof(int32_t) * cap);
    double *kb = (double *)mn::scratch(mn::kSlotGeneric2, sizeof(double) * cap);
    int32_t *ib = (int32_t *)mn::scratch(mn::kSlotGeneric3, sizeof(int32_t) * cap);
    MN_REQUIRE(ka && ia && kb && ib, MN_ENOMEM, "mn_search_lambda_aware: scratch");

    if (n > 0) {
        const dim3 g((unsigned)ntiles, (unsigned)((nq + kQB - 1) / kQB));
        if (x_is_f64)
            hipLaunchKernelGGL(k_lambda_scores<double>, g, dim3(kTile), 0, s, (const double *)X,
                               n, f, lambdas, Q, qn, lambda_q, nq, alpha, kk, ntiles, ka, ia,
                               flag);
        else
            hipLaunchKernelGGL(k_lambda_scores<float>, g, dim3(kTile), 0, s, (const float *)X, n,
                               f, lambdas, Q, qn, lambda_q, nq, alpha, kk, ntiles, ka, ia, flag);
        MN_KCHECK(s, "k_lambda_scores");
    }
    // reduce levels until one chunk per query is left, then the final pass
    while (true) {
        const int64_t nchunks = (m + kChunk - 1) / kChunk;
        const bool fin = nchunks <= 1;
        const dim3 g((unsigned)((std::max<int64_t>(nchunks, 1) + 3) / 4), (unsigned)nq);
        hipLaunchKernelGGL(k_topk_reduce, g, dim3(256), 0, s, ka, ia, m, nq, kk,
                           std::max<int64_t>(nchunks, 1), kb, ib, fin ? 1 : 0, k, n, out_idx,
                           out_score);
        MN_KCHECK(s, "k_topk_reduce");
        if (fin) break;
        m = nchunks * kk;
        std::swap(ka, kb);
        std::swap(ia, ib);
    }
    int hflag = 0;
    MN_HIP_TRY(hipMemcpyAsync(&hflag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(!(hflag & kFlagZeroLambda), MN_EINVAL,
               "Lambda of the item is 0.0, prepare the item before searching (core.rs:1169)");
    MN_REQUIRE(!(hflag & kFlagNan), MN_ENONFINITE,
               "mn_search_lambda_aware: NaN score (reference: partial_cmp().unwrap() panics)");
    return MN_OK;
}
