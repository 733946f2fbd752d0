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
    double s = -0.0;  // Rust >= 1.83 float Sum starts at -0.0
    for (int32_t t = 0; t < f; ++t) s = s + a[t] * a[t];
    qn[q] = __builtin_sqrt(s);
    if (lq[q] == 0.0) atomicOr(flag, kFlagZeroLambda);  // core.rs:1169-1172 assert_ne!
}

// Per-tile candidate lists of up to three selections (NK = 1: the lambda
// score; NK = 3, the hybrid search: + cosine > 0.9999, + best cosine).
struct Cand {
    double *k[3];
    int32_t *i[3];
};

template <typename T, int NK>
__global__ __launch_bounds__(256) void k_lambda_scores(
    const T *__restrict__ X, int64_t n, int32_t f, const double *__restrict__ lambdas,
    const double *__restrict__ Q, const double *__restrict__ qn, const double *__restrict__ lq,
    int64_t nq, double alpha, int32_t kk, int64_t ntiles, Cand cand, int *__restrict__ flag) {
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
        for (int q = 0; q < kQW; ++q) acc[a][q] = -0.0;  // Rust float Sum's start value
    double nrm = -0.0;  // norm chain of item 4*lane + w

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
#pragma unroll
    for (int kind = 0; kind < NK; ++kind) {
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
                double key = INFINITY;  // sorts after every live item / absent
                if (live && qq < nqb) {
                    const double denom = qn[q0 + qq] * xn;
                    const double cs = denom > 0.0 ? acc[a][q] / denom : 0.0;
                    if (kind == 0) {
                        const double ls = 1.0 - fmin(fabs(lq[q0 + qq] - li), 1.0);
                        const double sc = alpha * cs + (1.0 - alpha) * ls;
                        nan |= (sc != sc);
                        key = -sc;
                    } else if (kind == 1) {
                        key = cs > 0.9999 ? -cs : INFINITY;  // core.rs:1198,1230-1232
                    } else {
                        key = -cs;
                    }
                }
                d[q][a] = key;
            }
        }
        // each wave holds its queries' 256 keys in registers (4 per lane):
        // sort them in place (positions are irrelevant to the selection) and
        // write the top kk
#pragma unroll
        for (int q = 0; q < kQW; ++q) {
            const int qq = kQW * w + q;
            if (qq >= nqb) break;  // wave-uniform
            int jx[4] = {ix[0], ix[1], ix[2], ix[3]};
            wave_bitonic_sort<4>(d[q], jx);
            double *okey = cand.k[kind] + ((q0 + qq) * ntiles + tile) * kk;
            int32_t *oidx = cand.i[kind] + ((q0 + qq) * ntiles + tile) * kk;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int e = lane + 64 * r;
                if (e < kk) { okey[e] = d[q][r]; oidx[e] = jx[r]; }
            }
        }
    }
    if (nan) atomicOr(flag, kFlagNan);
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
            const bool ok = e < c && d[r] < INFINITY;  // INF: absent (hybrid lists)
            out_idx[q * k + e] = ok ? (int64_t)ix[r] : -1;
            out_score[q * k + e] = ok ? -d[r] : NAN;
        }
    }
}

// Hybrid union (core.rs:1282-1314), one wave per query: high-semantic
// entries (score = cosine) first, then the lambda top-k (lambda score) where
// the index is new, then the best-cosine item where new; the union sorted by
// score descending (sort_unstable: ties here by ascending index), first k.
// Inputs per query: B (cos > 0.9999 top k), A (lambda top k), C (best cos),
// -1 padded.  Needs 2k + 1 <= 512.
// Hybrid, lambda top k (list A): an item whose cosine is > 0.9999 was inserted
// with its COSINE first (high_semantic_vec, core.rs:1289-1293; or_insert keeps
// it, :1296-1299), even when it falls outside list B's top k.  Re-evaluate
// each A entry's cosine with the score kernel's exact folds (sequential f64
// norm and dot, same order) and substitute it.  One thread per (query, entry).
template <typename T>
__global__ __launch_bounds__(256) void k_hybrid_cos_fix(const T *__restrict__ X, int32_t f,
                                                        const double *__restrict__ Q,
                                                        const double *__restrict__ qn, int64_t nq,
                                                        int32_t k, const int64_t *__restrict__ ai,
                                                        double *__restrict__ as) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq * k) return;
    const int64_t q = t / k, i = ai[t];
    if (i < 0) return;
    const T *x = X + i * f;
    const double *a = Q + q * f;
    double dot = -0.0, nrm = -0.0;
    for (int32_t c = 0; c < f; ++c) {
        const double xv = (double)x[c];
        nrm = nrm + xv * xv;
        dot = dot + a[c] * xv;
    }
    const double denom = qn[q] * __builtin_sqrt(nrm);
    const double cs = denom > 0.0 ? dot / denom : 0.0;
    if (cs > 0.9999) as[t] = cs;
}

__global__ __launch_bounds__(64) void k_hybrid_union(
    const int64_t *__restrict__ ai, const double *__restrict__ as, const int64_t *__restrict__ bi,
    const double *__restrict__ bs, const int64_t *__restrict__ ci, const double *__restrict__ cs,
    int64_t nq, int32_t k, int64_t *__restrict__ out_idx, double *__restrict__ out_score) {
    __shared__ int64_t eidx[kChunk];
    __shared__ double escore[kChunk];
    __shared__ int keep[kChunk];
    const int lane = threadIdx.x;
    const int64_t q = blockIdx.x;
    if (q >= nq) return;
    double d[8];
    int ix[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int e = lane + 64 * r;
        int64_t id = -1;
        double sc = 0.0;
        int prio = 3;
        if (e < k) { id = bi[q * k + e]; sc = bs[q * k + e]; prio = 0; }
        else if (e < 2 * k) { id = ai[q * k + e - k]; sc = as[q * k + e - k]; prio = 1; }
        else if (e == 2 * k) { id = ci[q]; sc = cs[q]; prio = 2; }
        eidx[e] = id;
        escore[e] = sc;
        // first sort: by (index, priority); absent entries last
        d[r] = id >= 0 ? (double)id * 4.0 + prio : INFINITY;
        ix[r] = e;
    }
    wave_bitonic_sort<8>(d, ix);
    // sorted position p = lane + 64 r holds entry ix[r]; keep the first of
    // each index run (the highest-priority insertion, as HashMap::entry
    // .or_insert keeps the first)
#pragma unroll
    for (int r = 0; r < 8; ++r) keep[lane + 64 * r] = ix[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int p = lane + 64 * r;
        const int e = keep[p];
        const bool present = d[r] < INFINITY;
        const bool first = p == 0 || eidx[keep[p - 1]] != eidx[e];
        const bool use = present && first;
        d[r] = use ? -escore[e] : INFINITY;
        ix[r] = use ? (int)eidx[e] : INT_MAX;
    }
    wave_bitonic_sort<8>(d, ix);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int e = lane + 64 * r;
        if (e < k) {
            const bool ok = d[r] < INFINITY;
            out_idx[q * k + e] = ok ? (int64_t)ix[r] : -1;
            out_score[q * k + e] = ok ? -d[r] : NAN;
        }
    }
}

}  // namespace srch
}  // namespace mn

namespace {

// One selection's candidate lists -> final (idx, score) [nq][k] rows.
int reduce_lists(double *ka, int32_t *ia, double *kb, int32_t *ib, int64_t m, int64_t nq,
                 int32_t kk, int32_t k, int64_t n, int64_t *out_idx, double *out_score,
                 hipStream_t s) {
    using namespace mn::srch;
    while (true) {
        const int64_t nchunks = (m + kChunk - 1) / kChunk;
        const bool fin = nchunks <= 1;
        const dim3 g((unsigned)((std::max<int64_t>(nchunks, 1) + 3) / 4), (unsigned)nq);
        hipLaunchKernelGGL(k_topk_reduce, g, dim3(256), 0, s, ka, ia, m, nq, kk,
                           std::max<int64_t>(nchunks, 1), kb, ib, fin ? 1 : 0, k, n, out_idx,
                           out_score);
        MN_KCHECK(s, "k_topk_reduce");
        if (fin) return MN_OK;
        m = nchunks * kk;
        std::swap(ka, kb);
        std::swap(ia, ib);
    }
}

int search_batch(const void *X, int32_t x_is_f64, int64_t n, int32_t f, const double *lambdas,
                 const double *Q, const double *lambda_q, int64_t nq, int32_t k, double alpha,
                 int64_t *out_idx, double *out_score, void *stream, bool hybrid);

// Queries run in batches that keep the reduce grid (one row of blocks per
// query, gridDim.y <= 65535) and the candidate scratch (nq x tiles x k
// entries per selection) bounded.
int search_impl(const void *X, int32_t x_is_f64, int64_t n, int32_t f, const double *lambdas,
                const double *Q, const double *lambda_q, int64_t nq, int32_t k, double alpha,
                int64_t *out_idx, double *out_score, void *stream, bool hybrid) {
    using namespace mn::srch;
    const int64_t ntiles = std::max<int64_t>((n + kTile - 1) / kTile, 1);
    const int64_t kk = std::max<int64_t>(std::min<int64_t>(k, kTile), 1);
    const int64_t per_q = ntiles * kk * 24 * (hybrid ? 3 : 1);
    const int64_t budget = (int64_t)4 << 30;
    const int64_t qb = std::max<int64_t>(kQB, std::min<int64_t>(65535, budget / per_q) / kQB * kQB);
    if (nq <= qb)
        return search_batch(X, x_is_f64, n, f, lambdas, Q, lambda_q, nq, k, alpha, out_idx,
                            out_score, stream, hybrid);
    for (int64_t a = 0; a < nq; a += qb) {
        const int64_t b = std::min(nq, a + qb);
        const int rc = search_batch(X, x_is_f64, n, f, lambdas, Q + a * f, lambda_q + a, b - a, k,
                                    alpha, out_idx + a * k, out_score + a * k, stream, hybrid);
        if (rc != MN_OK) return rc;
    }
    return MN_OK;
}

int search_batch(const void *X, int32_t x_is_f64, int64_t n, int32_t f, const double *lambdas,
                 const double *Q, const double *lambda_q, int64_t nq, int32_t k, double alpha,
                 int64_t *out_idx, double *out_score, void *stream, bool hybrid) {
    using namespace mn::srch;
    const char *fn = hybrid ? "mn_search_lambda_aware_hybrid" : "mn_search_lambda_aware";
    MN_REQUIRE(n >= 0 && f >= 0 && nq >= 0 && k >= 0, MN_EINVAL, "%s: bad sizes", fn);
    const int kmax = hybrid ? (kChunk - 1) / 2 : kMaxK;
    MN_REQUIRE(k <= kmax, MN_ENOTSUP, "%s: k=%d > %d", fn, k, kmax);
    MN_REQUIRE(n < INT_MAX, MN_ENOTSUP, "%s: n >= 2^31", fn);
    MN_REQUIRE((int64_t)kTile * f * 8 < INT_MAX, MN_ENOTSUP,
               "%s: f too large for 32-bit tile offsets", fn);
    MN_REQUIRE(nq == 0 || k == 0 || (Q && lambda_q && out_idx && out_score &&
                                     (n == 0 || (X && lambdas))),
               MN_EINVAL, "%s: NULL pointer", fn);
    MN_REQUIRE(std::isfinite(alpha), MN_EINVAL, "%s: alpha not finite", fn);
    if (nq == 0 || k == 0) return MN_OK;
    hipStream_t s = (hipStream_t)stream;

    const int NK = hybrid ? 3 : 1;
    const int64_t ntiles = (n + kTile - 1) / kTile;
    const int32_t kk = (int32_t)std::min<int64_t>(k, kTile);
    int *flag = (int *)mn::scratch(mn::kSlotFlags, sizeof(int));
    double *qn = (double *)mn::scratch(mn::kSlotNorms, sizeof(double) * (size_t)nq);
    MN_REQUIRE(flag && qn, MN_ENOMEM, "%s: scratch", fn);
    MN_HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), s));
    hipLaunchKernelGGL(k_query_norms, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, Q, nq,
                       f, lambda_q, qn, flag);
    MN_KCHECK(s, "k_query_norms");

    // per selection: two ping-pong candidate buffers of nq * ntiles * kk
    const int64_t m = ntiles * kk;
    const size_t cap = (size_t)nq * (size_t)std::max<int64_t>(m, 1);
    const size_t per = cap * (2 * sizeof(double) + 2 * sizeof(int32_t));
    // hybrid: + the three selections' final rows, [nq][k] (idx, score) each
    const size_t fin = hybrid ? (size_t)nq * (size_t)k * 3 * (sizeof(int64_t) + sizeof(double)) : 0;
    char *base = (char *)mn::scratch(mn::kSlotGeneric0, per * (size_t)NK + fin);
    MN_REQUIRE(base, MN_ENOMEM, "%s: scratch", fn);
    Cand cand{};
    double *kb[3];
    int32_t *ib[3];
    for (int c = 0; c < NK; ++c) {
        char *p = base + per * (size_t)c;
        cand.k[c] = (double *)p;
        kb[c] = (double *)(p + cap * sizeof(double));
        cand.i[c] = (int32_t *)(p + 2 * cap * sizeof(double));
        ib[c] = (int32_t *)(p + 2 * cap * sizeof(double) + cap * sizeof(int32_t));
    }
    if (n > 0) {
        const dim3 g((unsigned)ntiles, (unsigned)((nq + kQB - 1) / kQB));
#define MN_SCORES(T, NKV)                                                                     \
    hipLaunchKernelGGL((k_lambda_scores<T, NKV>), g, dim3(kTile), 0, s, (const T *)X, n, f,    \
                       lambdas, Q, qn, lambda_q, nq, alpha, kk, ntiles, cand, flag)
        if (x_is_f64) {
            if (hybrid) MN_SCORES(double, 3); else MN_SCORES(double, 1);
        } else {
            if (hybrid) MN_SCORES(float, 3); else MN_SCORES(float, 1);
        }
#undef MN_SCORES
        MN_KCHECK(s, "k_lambda_scores");
    }
    if (!hybrid) {
        int rc = reduce_lists(cand.k[0], cand.i[0], kb[0], ib[0], m, nq, kk, k, n, out_idx,
                              out_score, s);
        if (rc != MN_OK) return rc;
    } else {
        char *fp = base + per * (size_t)NK;
        int64_t *fi[3];
        double *fs[3];
        for (int c = 0; c < 3; ++c) {
            fi[c] = (int64_t *)(fp + (size_t)c * nq * k * sizeof(int64_t));
            fs[c] = (double *)(fp + 3 * (size_t)nq * k * sizeof(int64_t) +
                               (size_t)c * nq * k * sizeof(double));
        }
        // A = lambda top k, B = cos > 0.9999 top k, C = best cosine (k = 1)
        for (int c = 0; c < 3; ++c) {
            int rc = reduce_lists(cand.k[c], cand.i[c], kb[c], ib[c], m, nq, kk, c == 2 ? 1 : k,
                                  n, fi[c], fs[c], s);
            if (rc != MN_OK) return rc;
        }
        if (n > 0) {
            const unsigned gb = (unsigned)((nq * k + 255) / 256);
            if (x_is_f64)
                hipLaunchKernelGGL(k_hybrid_cos_fix<double>, dim3(gb), dim3(256), 0, s,
                                   (const double *)X, f, Q, qn, nq, k, fi[0], fs[0]);
            else
                hipLaunchKernelGGL(k_hybrid_cos_fix<float>, dim3(gb), dim3(256), 0, s,
                                   (const float *)X, f, Q, qn, nq, k, fi[0], fs[0]);
            MN_KCHECK(s, "k_hybrid_cos_fix");
        }
        hipLaunchKernelGGL(k_hybrid_union, dim3((unsigned)nq), dim3(64), 0, s, fi[0], fs[0], fi[1],
                           fs[1], fi[2], fs[2], nq, k, out_idx, out_score);
        MN_KCHECK(s, "k_hybrid_union");
    }
    int hflag = 0;
    MN_HIP_TRY(hipMemcpyAsync(&hflag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hybrid || !(hflag & kFlagZeroLambda), MN_EINVAL,
               "Lambda of the item is 0.0, prepare the item before searching (core.rs:1169)");
    MN_REQUIRE(!(hflag & kFlagNan), MN_ENONFINITE,
               "%s: NaN score (reference: partial_cmp().unwrap() panics)", fn);
    return MN_OK;
}

}  // namespace

extern "C" int mn_search_lambda_aware(const void *X, int32_t x_is_f64, int64_t n, int32_t f,
                                      const double *lambdas, const double *Q,
                                      const double *lambda_q, int64_t nq, int32_t k, double alpha,
                                      int64_t *out_idx, double *out_score, void *stream) {
    mn::clear_error();
    return search_impl(X, x_is_f64, n, f, lambdas, Q, lambda_q, nq, k, alpha, out_idx, out_score,
                       stream, false);
}

extern "C" int mn_search_lambda_aware_hybrid(const void *X, int32_t x_is_f64, int64_t n,
                                             int32_t f, const double *lambdas, const double *Q,
                                             const double *lambda_q, int64_t nq, int32_t k,
                                             double alpha, int64_t *out_idx, double *out_score,
                                             void *stream) {
    mn::clear_error();
    return search_impl(X, x_is_f64, n, f, lambdas, Q, lambda_q, nq, k, alpha, out_idx, out_score,
                       stream, true);
}
