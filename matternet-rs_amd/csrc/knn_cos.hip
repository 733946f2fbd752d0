// knn_cos.hip — K1 (cosine): rectified-cosine kNN of the FEATURE columns of
// X [n][f] (the feature graph of graph.rs:214, built on the transposed data),
// bit-exact vs the reference's f64 arithmetic.
//
// Reference semantics (src_legacy/tests/test_helpers.rs:77-126, the
// brute-force spec of build_adjacency; production _build_adjacency
// laplacian.rs:245-290 uses the same distance and weight):
//   norm_i = sqrt(sum_t x_ti^2)          sequential f64 over the profile
//   dot_ij = sum_t x_ti x_tj             sequential f64 (products exact)
//   cos = norm_i*norm_j > 1e-12 ? clamp(dot/(norm_i norm_j), -1, 1) : 0
//   dist = 1 - max(cos, 0); keep dist <= eps and w = 1/(1+(dist/sigma)^p) >
//   1e-12; sort by (dist, j); truncate topk.
//
// MI355X design (profiles are long: n ~ 1e6, f ~ 768):
//   1. k_transpose        X -> XT [f][n] (LDS-tiled) so every profile streams.
//   2. k_col_norms        exact sequential f64 norms (one wave per column:
//                         squares formed lane-parallel, the ordered chain of
//                         adds reads them back from LDS as broadcasts).
//   3. k_gram_f64         G = X^T X on MFMA v_mfma_f64_16x16x4_f64 (f32 inputs
//                         widened: products exact), upper 64x64 block tiles,
//                         split-K over rows, f64 atomics into G.
//   4. k_cos_select       per node (one wave): approximate distances from G,
//                         wave bitonic sort, top-L candidates + the (L+1)-th.
//   5. k_cos_exact_q      sixteen (node, candidate) pairs a wave, four lanes a
//                         pair: the reference's sequential f64 dot over the
//                         full profile (products exact and lane-parallel, the
//                         chain of adds ordered; k_cos_exact_wave: the round-4
//                         four-pairs-a-wave form).
//                         Only candidates that can reach the top k are
//                         evaluated: the first topk by approximate distance,
//                         then those whose lower bound d~ - delta does not
//                         exceed the worst of those (k_extra_pairs).
//   6. k_cos_finish       per node: sort exact (dist, j), certify
//                         (|d~ - d| <= 2(n+16)2^-53), filter, write; nodes
//                         that fail go to the exact all-pairs fallback.
#include <algorithm>
#include <climits>
#include <vector>

#include "common.hpp"
#include "glibc_f64.hpp"

namespace mn {
namespace kcos {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int FMAXC = 4096;  // features (nodes) limit
constexpr int LMAXC = 64;    // candidate list length limit

// ---- 1. transpose -------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_transpose(const T *__restrict__ X, int64_t n, int f,
                                                   T *__restrict__ XT) {
    __shared__ T tile[64][65];
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    const int c0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int64_t row = r0 + r;
        const int col = c0 + tx;
        tile[r][tx] = (row < n && col < f) ? X[row * f + col] : (T)0;
    }
    __syncthreads();
    for (int c = ty; c < 64; c += 4) {
        const int col = c0 + c;
        const int64_t row = r0 + tx;
        if (col < f && row < n) XT[(int64_t)col * n + row] = tile[tx][c];
    }
}

// ---- 2. exact sequential norms / dots (one wave per ordered f64 chain) ------
// The reference folds sum_t a_t b_t in t order (f64, products exact for f32
// inputs).  One wave streams 256-element chunks of both profiles (float4 per
// lane, the next chunk in flight), forms the 256 products lane-parallel into
// LDS, and the ordered chain of adds reads them back as broadcast
// ds_read_b128: the VALU issues little but the adds.
constexpr int CH = 256;

constexpr int PF = 4;  // chunks in flight ahead of the chain

__device__ __forceinline__ double ordered_dot(const float *__restrict__ a,
                                              const float *__restrict__ b, int64_t n,
                                              double (*buf)[CH]) {
    const int lane = threadIdx.x & 63;
    const int64_t nfull = n / CH;
    const bool vec = ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0;
    float4 ra[PF], rb[PF];
    auto fetch = [&](int64_t c, float4 &pa, float4 &pb) {
        const int64_t o = c * CH + 4 * lane;
        if (vec) {
            pa = *reinterpret_cast<const float4 *>(a + o);
            pb = *reinterpret_cast<const float4 *>(b + o);
        } else {
            pa = make_float4(a[o], a[o + 1], a[o + 2], a[o + 3]);
            pb = make_float4(b[o], b[o + 1], b[o + 2], b[o + 3]);
        }
    };
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (u < nfull) fetch(u, ra[u], rb[u]);
    double acc = -0.0;
    for (int64_t c0 = 0; c0 < nfull; c0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int64_t c = c0 + u;
            if (c >= nfull) break;
            double *bb = buf[u & 1];
            bb[4 * lane + 0] = (double)ra[u].x * (double)rb[u].x;
            bb[4 * lane + 1] = (double)ra[u].y * (double)rb[u].y;
            bb[4 * lane + 2] = (double)ra[u].z * (double)rb[u].z;
            bb[4 * lane + 3] = (double)ra[u].w * (double)rb[u].w;
            if (c + PF < nfull) fetch(c + PF, ra[u], rb[u]);
            __builtin_amdgcn_wave_barrier();
            acc = lds_chain_f64<CH>(acc, bb);
            __builtin_amdgcn_wave_barrier();
        }
    }
    for (int64_t t = nfull * CH; t < n; ++t) acc = acc + (double)a[t] * (double)b[t];
    return acc;
}

// Four ordered chains per wave (lanes 16g..16g+15 run chain g): each group
// loads its 256-element chunk of both profiles (16 per lane, next chunk in
// flight), forms the products lane-parallel into its LDS buffer, and folds it
// with group-broadcast LDS reads — one VALU add serves four chains, so the
// redundant-lane issue cost of a single-chain wave is cut by four.
constexpr int CHP = CH + 2;  // buffer stride (16 B pad: the 4 groups hit different banks)

// 16 consecutive values per lane (f32: 4 x float4, f64: 8 x double2)
__device__ __forceinline__ void load16(const float *p, bool vec, float (&o)[16]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        float4 x;
        if (vec) x = *reinterpret_cast<const float4 *>(p + 4 * u);
        else x = make_float4(p[4 * u], p[4 * u + 1], p[4 * u + 2], p[4 * u + 3]);
        o[4 * u] = x.x; o[4 * u + 1] = x.y; o[4 * u + 2] = x.z; o[4 * u + 3] = x.w;
    }
}
__device__ __forceinline__ void load16(const double *p, bool vec, double (&o)[16]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        double2 x;
        if (vec) x = *reinterpret_cast<const double2 *>(p + 2 * u);
        else x = make_double2(p[2 * u], p[2 * u + 1]);
        o[2 * u] = x.x; o[2 * u + 1] = x.y;
    }
}

// The products are the reference's fl(a*b) in f64 (exact for f32 inputs).
// PFD chunks of both profiles in flight ahead of the chain (registers); SQ:
// a == b (the norms: one load, the square)
template <typename T, int PFD = 2, bool SQ = false>
__device__ __forceinline__ double ordered_dot4(const T *__restrict__ a,
                                               const T *__restrict__ b, int64_t n,
                                               double (*buf)[4][CHP]) {
    const int lane = threadIdx.x & 63, g = lane >> 4, gl = lane & 15;
    const int64_t nfull = n / CH;
    const bool vec = ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0;
    T ra[PFD][16], rb[SQ ? 1 : PFD][16];
    auto fetch = [&](int64_t c, T (&pa)[16], T (&pb)[16]) {
        const int64_t o = c * CH + 16 * gl;
        load16(a + o, vec, pa);
        if constexpr (!SQ) load16(b + o, vec, pb);
    };
#pragma unroll
    for (int h = 0; h < PFD; ++h)
        if (nfull > h) fetch(h, ra[h], rb[SQ ? 0 : h]);
    double acc = -0.0;
    for (int64_t c0 = 0; c0 < nfull; c0 += PFD) {
#pragma unroll
        for (int h = 0; h < PFD; ++h) {
            const int64_t c = c0 + h;
            if (c >= nfull) break;
            double *bb = buf[h & 1][g];
#pragma unroll
            for (int u = 0; u < 16; ++u)
                bb[16 * gl + u] = (double)ra[h][u] * (double)(SQ ? ra[h][u] : rb[SQ ? 0 : h][u]);
            if (c + PFD < nfull) fetch(c + PFD, ra[h], rb[SQ ? 0 : h]);
            __builtin_amdgcn_wave_barrier();
            acc = lds_chain_f64<CH>(acc, bb);
            __builtin_amdgcn_wave_barrier();
        }
    }
    for (int64_t t = nfull * CH; t < n; ++t) acc = acc + (double)a[t] * (double)b[t];
    return acc;
}

// four columns per wave
template <typename T>
__global__ __launch_bounds__(64) void k_col_norms(const T *__restrict__ XT, int64_t n, int f,
                                                  double *__restrict__ nrm) {
    __shared__ double buf[2][4][CHP];
    const int g = threadIdx.x >> 4;
    const int i = blockIdx.x * 4 + g;
    const T *p = XT + (int64_t)min(i, f - 1) * n;
    const double acc = ordered_dot4<T, 4, true>(p, p, n, buf);
    if ((threadIdx.x & 15) == 0 && i < f) nrm[i] = __builtin_sqrt(acc);
}

// ---- 3. Gram on f64 MFMA --------------------------------------------------
constexpr int GT = 64;  // output tile
constexpr int GK = 16;  // rows per LDS stage

template <typename T>
__global__ __launch_bounds__(256) void k_gram_f64(const T *__restrict__ X, int64_t n, int f,
                                                  int ntile, int64_t kchunk, int nchunk,
                                                  double *__restrict__ G) {
    // rows GT + 16 apart (round 6; was GT + 4): the fragment reads take 16
    // consecutive columns of four rows, and a row stride of 16 (mod 32)
    // words for f32 / 32 (mod 64) for f64 puts a lane group's rows on
    // disjoint banks (GT + 4: 3.2 bank-conflict cycles per LDS instruction)
    __shared__ T As[GK][GT + 16];
    __shared__ T Bs[GK][GT + 16];
    // blockIdx.x = chunk-major over upper-triangle tiles (concurrent blocks share rows)
    const int ntri = ntile * (ntile + 1) / 2;
    const int chunk = blockIdx.x / ntri;
    int t = blockIdx.x % ntri, bi = 0;
    while (t >= ntile - bi) { t -= ntile - bi; ++bi; }
    const int bj = bi + t;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int64_t k0 = (int64_t)chunk * kchunk;
    const int64_t k1 = min(n, k0 + kchunk);
    f64x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int lr = threadIdx.x >> 4, lc4 = (threadIdx.x & 15) * 4;  // 16 rows x 16 x 4 values
    const int ca = bi * GT + lc4, cb = bj * GT + lc4;
    // the next stage's rows are loaded while this stage computes (round 4b)
    auto load = [&](int64_t kb, T (&va)[4], T (&vb)[4]) {
        const int64_t row = kb + lr;
#pragma unroll
        for (int u = 0; u < 4; ++u) va[u] = vb[u] = (T)0;
        if (row < k1) {
            const T *pr = X + row * f;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                va[u] = ca + u < f ? pr[ca + u] : (T)0;
                vb[u] = cb + u < f ? pr[cb + u] : (T)0;
            }
        }
    };
    T va[4], vb[4];
    if (k0 < k1) load(k0, va, vb);
    for (int64_t kb = k0; kb < k1; kb += GK) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            As[lr][lc4 + u] = va[u];
            Bs[lr][lc4 + u] = vb[u];
        }
        __syncthreads();
        if (kb + GK < k1) load(kb + GK, va, vb);
#pragma unroll
        for (int s = 0; s < GK / 4; ++s) {
            const int kr = s * 4 + (lane >> 4);
            double a[2], b[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) a[m] = (double)As[kr][wr * 32 + m * 16 + (lane & 15)];
#pragma unroll
            for (int m = 0; m < 2; ++m) b[m] = (double)Bs[kr][wc * 32 + m * 16 + (lane & 15)];
#pragma unroll
            for (int ma = 0; ma < 2; ++ma)
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
                    acc[ma][mb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ma], b[mb], acc[ma][mb],
                                                                       0, 0, 0);
        }
    }
    // C/D (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int ma = 0; ma < 2; ++ma)
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = bi * GT + wr * 32 + ma * 16 + (lane >> 4) + 4 * r;
                const int gj = bj * GT + wc * 32 + mb * 16 + (lane & 15);
                if (gi < f && gj < f) atomicAdd(&G[(int64_t)gi * f + gj], acc[ma][mb][r]);
            }
}

// ---- 3b. Gram on f32 MFMA with an f64 fold (round 5, f32 profiles) ----------
// G~ = X^T X on v_mfma_f32_16x16x4_f32 (f32 inputs as they are), upper
// 128 x 128 block tiles (four waves of 64 x 64), split-K over row chunks: the
// f32 accumulators are folded into f64 every G3F rows, the chunk's f64 tile
// is added into G.  Error (selection only; the exact chains decide): per fold
// window the f32 sum of G3F products is within (G3F + 8) 2^-24 sum |x_i x_j|
// (<= n_i n_j), the f64 folds add (n / G3F + nchunk + 8) 2^-53 — valid while
// no product or partial leaves the f32 normal range: every column's max |x|
// (atomicMax into colmax) must lie in [2^-20, 2^40] or be 0, else the driver
// recomputes G with k_gram_f64.
constexpr int G3T = 128;  // block tile
constexpr int G3K = 32;   // rows per LDS stage
constexpr int G3F = 256;  // rows per f32 window before the f64 fold
constexpr int G3P = G3T + 16;  // row stride: 4 rows of a fragment read on 4 bank quarters
typedef float f32x4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_gram_f32m(const float *__restrict__ X, int64_t n, int f,
                                                   int ntile, int64_t kchunk,
                                                   double *__restrict__ G,
                                                   unsigned *__restrict__ colmax) {
    __shared__ __attribute__((aligned(16))) float As[G3K][G3P];
    __shared__ __attribute__((aligned(16))) float Bs[G3K][G3P];
    const int ntri = ntile * (ntile + 1) / 2;
    const int chunk = blockIdx.x / ntri;  // chunk-major: concurrent blocks share rows
    int t = blockIdx.x % ntri, bi = 0;
    while (t >= ntile - bi) { t -= ntile - bi; ++bi; }
    const int bj = bi + t;
    const bool diag = bi == bj;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int64_t k0 = (int64_t)chunk * kchunk;
    const int64_t k1 = min(n, k0 + kchunk);
    f32x4v acc[4][4];
    double fold[4][4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) fold[a][b][r] = 0.0;
        }
    // stage loads: 32 rows x 128 columns of A (and B): thread -> row tid / 8,
    // 16 consecutive columns (4 x float4 when the row slice is aligned)
    const int lr = tid >> 3, lc = (tid & 7) * 16;
    const int ca = bi * G3T + lc, cb = bj * G3T + lc;
    const bool vec = (f & 3) == 0;
    float va[16], vb[16];
    float ma = 0.f, mb = 0.f;  // this thread's max |x| over its columns (fmaxf drops NaN:
    bool nan_a = false, nan_b = false;  // tracked apart)
    auto load = [&](int64_t kb) {
        const int64_t row = kb + lr;
        const bool rin = row < k1;
        const float *pr = X + (rin ? row : k0) * (int64_t)f;
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
            if (vec && ca + u + 3 < f) {
                const float4 x = *reinterpret_cast<const float4 *>(pr + ca + u);
                va[u] = x.x; va[u + 1] = x.y; va[u + 2] = x.z; va[u + 3] = x.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) va[u + e] = ca + u + e < f ? pr[ca + u + e] : 0.f;
            }
            if (!diag) {
                if (vec && cb + u + 3 < f) {
                    const float4 x = *reinterpret_cast<const float4 *>(pr + cb + u);
                    vb[u] = x.x; vb[u + 1] = x.y; vb[u + 2] = x.z; vb[u + 3] = x.w;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) vb[u + e] = cb + u + e < f ? pr[cb + u + e] : 0.f;
                }
            }
        }
        if (!rin) {
#pragma unroll
            for (int u = 0; u < 16; ++u) va[u] = vb[u] = 0.f;
        }
    };
    int since_fold = 0;
    if (k0 < k1) load(k0);
    for (int64_t kb = k0; kb < k1; kb += G3K) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
            *reinterpret_cast<float4 *>(&As[lr][lc + u]) = make_float4(va[u], va[u + 1], va[u + 2], va[u + 3]);
            if (!diag)
                *reinterpret_cast<float4 *>(&Bs[lr][lc + u]) = make_float4(vb[u], vb[u + 1], vb[u + 2], vb[u + 3]);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            ma = fmaxf(ma, __builtin_fabsf(va[u]));
            nan_a |= va[u] != va[u];
            if (!diag) {
                mb = fmaxf(mb, __builtin_fabsf(vb[u]));
                nan_b |= vb[u] != vb[u];
            }
        }
        __syncthreads();
        if (kb + G3K < k1) load(kb + G3K);
        const float (*Bp)[G3P] = diag ? As : Bs;
#pragma unroll
        for (int ks = 0; ks < G3K / 4; ++ks) {
            const int kr = ks * 4 + (lane >> 4);
            float a[4], b[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) a[m] = As[kr][wr * 64 + m * 16 + (lane & 15)];
#pragma unroll
            for (int m = 0; m < 4; ++m) b[m] = Bp[kr][wc * 64 + m * 16 + (lane & 15)];
#pragma unroll
            for (int ma_ = 0; ma_ < 4; ++ma_)
#pragma unroll
                for (int mb_ = 0; mb_ < 4; ++mb_)
                    acc[ma_][mb_] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ma_], b[mb_], acc[ma_][mb_],
                                                                         0, 0, 0);
        }
        since_fold += G3K;
        if (since_fold >= G3F) {
            since_fold = 0;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) fold[a][b][r] += (double)acc[a][b][r];
                    acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
                }
        }
    }
    // C/D (f32 16x16x4): row = 4 * (lane >> 4) + reg, col = lane & 15
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double v = fold[a][b][r] + (double)acc[a][b][r];
                const int gi = bi * G3T + wr * 64 + a * 16 + 4 * (lane >> 4) + r;
                const int gj = bj * G3T + wc * 64 + b * 16 + (lane & 15);
                if (gi < f && gj < f) atomicAdd(&G[(int64_t)gi * f + gj], v);
            }
    // column maxima (NaN propagates through the unsigned order: NaN bits > inf)
    const unsigned mra = nan_a ? 0x7FC00000u : __float_as_uint(ma);
    const unsigned mrb = nan_b ? 0x7FC00000u : __float_as_uint(mb);
    // fold over the 32 row-threads of each column group (lanes tid & 7 equal)
    __shared__ unsigned cm[2][G3T];
    if (tid < 2 * G3T) (&cm[0][0])[tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        atomicMax(&cm[0][lc + u], mra);
        if (!diag) atomicMax(&cm[1][lc + u], mrb);
    }
    __syncthreads();
    if (tid < G3T) {
        if (bi * G3T + tid < f) atomicMax(&colmax[bi * G3T + tid], cm[0][tid]);
        if (!diag && bj * G3T + tid < f) atomicMax(&colmax[bj * G3T + tid], cm[1][tid]);
    }
}

// 1 in *bad when a column max leaves [2^-20, 2^40] (zero columns are exact)
// or is not finite: the f32 Gram's error bound does not hold
__global__ void k_colmax_check(const unsigned *__restrict__ colmax, int f, int *__restrict__ bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= f) return;
    const unsigned u = colmax[i];
    const float m = __uint_as_float(u);
    const bool ok = u == 0u || (u < 0x7F800000u && m >= 0x1p-20f && m <= 0x1p40f);
    if (!ok) *bad = 1;
}

__device__ __forceinline__ double gram_at(const double *G, int f, int i, int j) {
    return ((i / GT) <= (j / GT)) ? G[(int64_t)i * f + j] : G[(int64_t)j * f + i];
}

// the reference's distance from (dot, norms)
__device__ __forceinline__ double cos_dist(double dot, double ni, double nj) {
    const double denom = ni * nj;
    double cs = 0.0;
    if (denom > 1e-12) {
        cs = dot / denom;
        cs = cs < -1.0 ? -1.0 : (cs > 1.0 ? 1.0 : cs);  // NaN stays NaN
    }
    return 1.0 - (cs > 0.0 ? cs : 0.0);
}

// ---- 4. per node candidate selection ---------------------------------------
template <int NR>
__global__ __launch_bounds__(256) void k_cos_select(const double *__restrict__ G,
                                                    const double *__restrict__ nrm, int f, int L,
                                                    int32_t *__restrict__ cand,
                                                    double *__restrict__ capx,
                                                    double *__restrict__ gnext, double amb) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= f) return;
    double d[NR];
    int ix[NR];
    const double ni = nrm[i];
    bool nan = false;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int j = lane + 64 * r;
        if (j < f && j != i) {
            d[r] = cos_dist(gram_at(G, f, i, j), ni, nrm[j]);
            if (d[r] != d[r]) { d[r] = 2.0; nan = true; }  // non-finite data
            // n_i n_j at the reference's 1e-12 cut: approximate norms may fall
            // on the other side of it — the node takes the exact path
            if (__builtin_fabs(ni * nrm[j] - 1e-12) <= amb) nan = true;
            ix[r] = j;
        } else {
            d[r] = __builtin_inf();
            ix[r] = INT_MAX;
        }
    }
    const bool any_nan = __any(nan);
    wave_bitonic_sort<NR>(d, ix);
    if (lane < L) {
        cand[(int64_t)i * L + lane] = ix[0];
        capx[(int64_t)i * L + lane] = any_nan ? -__builtin_inf() : d[0];
    }
    double gn = (L < f - 1) ? wave_elem<NR>(d, L) : __builtin_inf();
    if (any_nan) gn = -__builtin_inf();  // the bound argument fails: exact path
    if (lane == 0) gnext[i] = gn;
}

// ---- 5. exact sequential dot for (node, candidate) ---------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_cos_exact(const T *__restrict__ XT, int64_t n,
                                                   const int32_t *__restrict__ pi,
                                                   const int32_t *__restrict__ pj, int64_t npairs,
                                                   const double *__restrict__ nrm,
                                                   double *__restrict__ dist) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npairs) return;
    const int i = pi[q], j = pj[q];
    if (i < 0 || j < 0) { dist[q] = __builtin_inf(); return; }
    const double denom = nrm[i] * nrm[j];
    if (!(denom > 1e-12)) { dist[q] = 1.0; return; }  // cos = 0 without a dot
    const T *a = XT + (int64_t)i * n;
    const T *b = XT + (int64_t)j * n;
    double acc = -0.0;
    int64_t t = 0;
    for (; t + 8 <= n; t += 8) {
        T va[8], vb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { va[u] = a[t + u]; vb[u] = b[t + u]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + (double)va[u] * (double)vb[u];
    }
    for (; t < n; ++t) acc = acc + (double)a[t] * (double)b[t];
    dist[q] = cos_dist(acc, nrm[i], nrm[j]);
}

// one wave per listed pair q: (node i = pi[q], candidate slot) -> dist[slot]
// four listed pairs per wave, pair q = (node i, candidate slot) -> dist[slot]
template <typename T, int PFD = 2>
__global__ __launch_bounds__(256) void k_cos_exact_wave(const T *__restrict__ XT, int64_t n,
                                                        const int32_t *__restrict__ plist,
                                                        const int *__restrict__ pcount,
                                                        int64_t pmax, const int32_t *__restrict__ cand,
                                                        int L, const double *__restrict__ nrm,
                                                        double *__restrict__ dist) {
    __shared__ double buf[4][2][4][CHP];
    const int w = threadIdx.x >> 6, g = (threadIdx.x & 63) >> 4;
    const int64_t np = pcount ? (int64_t)*pcount : pmax;
    const int64_t wq = ((int64_t)blockIdx.x * 4 + w) * 4;
    if (wq >= np) return;  // wave-uniform
    const int64_t q = wq + g;
    int slot = -1, i = 0, j = 0;
    bool act = false;
    double denom = 0.0;
    if (q < np) {
        slot = plist ? plist[q] : (int)q;  // slot = i * L + r
        i = slot / L;
        j = cand[slot];
        if (j != INT_MAX) {
            denom = nrm[i] * nrm[j];
            act = true;
        }
    }
    const bool dot = act && denom > 1e-12;  // else cos = 0 without a dot
    const T *pa = XT + (int64_t)(dot ? i : 0) * n, *pb = XT + (int64_t)(dot ? j : 0) * n;
    const double acc = ordered_dot4<T, PFD>(pa, pb, n, buf[w]);
    if ((threadIdx.x & 15) == 0 && act) dist[slot] = dot ? cos_dist(acc, nrm[i], nrm[j]) : 1.0;
}

// Round 5: sixteen listed pairs per wave (lanes 4g..4g+3 run pair g) in
// 64-element chunks.  The four-chains-per-wave form above reads every product
// back as a 16-lane broadcast (1 KB of LDS returned per two elements and
// chain): with ~3.5 waves a CU the LDS return path, not the add chain, set the
// pace (~16 cycles an element).  Here a ds_read_b128 serves sixteen chains
// (the 16 chain buffers sit 528 B apart: bank offsets 4g, conflict-free), the
// products of a chunk are formed by the chain's four lanes (16 each), and
// PFD chunks of both profiles are in flight (one wave a CU).
constexpr int CQ = 64;        // chunk (elements of one profile)
constexpr int CQP = CQ + 2;   // chain buffer stride in doubles (528 B)
// Round 6 (LPC 8): a lane's EPL = 8 products were written as four 16-B
// pieces 64 B apart per lane — in a ds_write_b128 lane group (8 lanes, banks
// (a / 4) mod 32) lanes gl and gl + 2 hit the same banks: 4-way conflicts
// (SQ_LDS_BANK_CONFLICT 4.8 cycles per LDS instruction, profiles/r05_legs).
// Segments of 8 products are now 10 doubles apart (80 B: the 8 lanes' pieces
// of one store cover all 32 banks) and chain buffers 84 doubles apart (672 B:
// the four chains of a ds_read_b128 lane group read distinct 16-B slots).
constexpr int CQS = 10;               // segment stride (8 products + 2 pad)
constexpr int CQP8 = 8 * CQS + 4;     // chain buffer stride, LPC 8 (672 B)

// The ordered fold over one chunk in the segmented layout (element e at
// b[(e / 8) CQS + e % 8]): lds_chain_f64<64> with the segment gaps skipped.
__device__ __forceinline__ double lds_chain_f64_seg(double acc, const double *b) {
    const double2 *b2 = reinterpret_cast<const double2 *>(b);
    double2 v[2][16];
    // batch bt = elements 32 bt .. 32 bt + 31 = segments 4 bt .. 4 bt + 3
#pragma unroll
    for (int q = 0; q < 16; ++q) v[0][q] = b2[(q >> 2) * (CQS / 2) + (q & 3)];
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
    for (int q = 0; q < 16; ++q) v[1][q] = b2[(4 + (q >> 2)) * (CQS / 2) + (q & 3)];
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
    for (int bt = 0; bt < 2; ++bt) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            acc = acc + v[bt][q].x;
            acc = acc + v[bt][q].y;
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 32, 0);
    }
    return acc;
}
// RAW (round 5): the chains of the listed pairs write their raw dot into
// dist[slot] (k_cos_dist turns it into the distance once the norms exist) and
// fnorm more chains follow the np listed ones: chain np + c folds column c
// with itself -> nrm[c] = sqrt (the reference's sequential norm).
// LPC lanes a chain (4: sixteen chains a wave; 8: eight chains, half the
// product work a lane and twice the waves), EPL = 64 / LPC elements a lane
// per chunk.
template <int N>
__device__ __forceinline__ void loadn(const float *p, bool vec, float (&o)[N]) {
#pragma unroll
    for (int u = 0; u < N; u += 4) {
        float4 x;
        if (vec) x = *reinterpret_cast<const float4 *>(p + u);
        else x = make_float4(p[u], p[u + 1], p[u + 2], p[u + 3]);
        o[u] = x.x; o[u + 1] = x.y; o[u + 2] = x.z; o[u + 3] = x.w;
    }
}
template <int N>
__device__ __forceinline__ void loadn(const double *p, bool vec, double (&o)[N]) {
#pragma unroll
    for (int u = 0; u < N; u += 2) {
        double2 x;
        if (vec) x = *reinterpret_cast<const double2 *>(p + u);
        else x = make_double2(p[u], p[u + 1]);
        o[u] = x.x; o[u + 1] = x.y;
    }
}
template <typename T, int PFD, bool RAW = false, int LPC = 4>
__global__ __launch_bounds__(64) void k_cos_exact_q(const T *__restrict__ XT, int64_t n,
                                                    const int32_t *__restrict__ plist,
                                                    const int *__restrict__ pcount, int64_t pmax,
                                                    const int32_t *__restrict__ cand, int L,
                                                    int fnorm, double *__restrict__ nrm,
                                                    double *__restrict__ dist) {
    constexpr int CPW = 64 / LPC, EPL = CQ / LPC;
    constexpr bool SEG = LPC == 8;  // the segmented, conflict-free layout
    __shared__ __attribute__((aligned(16))) double buf[2][CPW][SEG ? CQP8 : CQP];
    const int lane = threadIdx.x & 63, g = lane / LPC, gl = lane % LPC;
    const int64_t np = pcount ? (int64_t)*pcount : pmax;
    const int64_t wq = (int64_t)blockIdx.x * CPW;
    if (wq >= np + (RAW ? fnorm : 0)) return;  // wave-uniform
    const int64_t q = wq + g;
    int slot = -1, i = 0, j = 0, ncol = -1;
    bool act = false;
    double denom = 0.0;
    if (q < np) {
        slot = plist ? plist[q] : (int)q;  // slot = i * L + r
        i = slot / L;
        j = cand[slot];
        if (j != INT_MAX) {
            if constexpr (!RAW) denom = nrm[i] * nrm[j];
            act = true;
        }
    } else if (RAW && q < np + fnorm) {
        ncol = (int)(q - np);
        i = j = ncol;
    }
    // else cos = 0 without a dot (RAW: every listed pair and norm chain folds)
    const bool dot = RAW ? (act || ncol >= 0) : (act && denom > 1e-12);
    const T *a = XT + (int64_t)(dot ? i : 0) * n, *b = XT + (int64_t)(dot ? j : 0) * n;
    const int64_t nfull = n / CQ;
    const bool vec = ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0;
    // Straight-line loop body: the loads are unconditional (past the last
    // full chunk they re-read it) and the main loop runs whole groups of PFD
    // chunks, so the wait before a chunk's products counts only the loads
    // issued after its own (vmcnt(N)); with the loads behind a branch the
    // compiler waited for all of them (vmcnt(0)) at every group.
    T ra[PFD][EPL], rb[PFD][EPL];
#define MN_QFETCH(C, H)                                  \
    do {                                                 \
        const int64_t o_ = (C) * CQ + EPL * gl;          \
        loadn<EPL>(a + o_, vec, ra[H]);                  \
        loadn<EPL>(b + o_, vec, rb[H]);                  \
    } while (0)
#define MN_QCHUNK(H)                                                                     \
    do {                                                                                 \
        double *bb_ = buf[(H) & 1][g];                                                   \
        _Pragma("unroll") for (int u = 0; u < EPL; u += 2)                              \
            *reinterpret_cast<double2 *>(bb_ + (SEG ? CQS : EPL) * gl + u) =             \
                make_double2((double)ra[H][u] * (double)rb[H][u],                        \
                             (double)ra[H][u + 1] * (double)rb[H][u + 1]);               \
    } while (0)
    double acc = -0.0;
    if (nfull > 0) {
#pragma unroll
        for (int h = 0; h < PFD; ++h) MN_QFETCH(min((int64_t)h, nfull - 1), h);
        const int64_t nmain = nfull / PFD * PFD;
        for (int64_t c0 = 0; c0 < nmain; c0 += PFD) {
#pragma unroll
            for (int h = 0; h < PFD; ++h) {
                MN_QCHUNK(h);
                MN_QFETCH(min(c0 + h + PFD, nfull - 1), h);
                __builtin_amdgcn_wave_barrier();
                if constexpr (SEG) acc = lds_chain_f64_seg(acc, buf[h & 1][g]);
                else acc = lds_chain_f64<CQ>(acc, buf[h & 1][g]);
                __builtin_amdgcn_wave_barrier();
            }
        }
        const int rem = (int)(nfull - nmain);  // < PFD chunks, already in ra[0..rem)
#pragma unroll
        for (int h = 0; h < PFD - 1; ++h) {
            if (h < rem) {
                MN_QCHUNK(h);
                __builtin_amdgcn_wave_barrier();
                if constexpr (SEG) acc = lds_chain_f64_seg(acc, buf[h & 1][g]);
                else acc = lds_chain_f64<CQ>(acc, buf[h & 1][g]);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
#undef MN_QFETCH
#undef MN_QCHUNK
    for (int64_t t = nfull * CQ; t < n; ++t) acc = acc + (double)a[t] * (double)b[t];
    if (gl == 0) {
        if constexpr (RAW) {
            if (act) dist[slot] = acc;
            else if (ncol >= 0) nrm[ncol] = __builtin_sqrt(acc);
        } else if (act) {
            dist[slot] = dot ? cos_dist(acc, nrm[i], nrm[j]) : 1.0;
        }
    }
}

// the listed pairs' distances from their raw dots (k_cos_exact_q RAW) and
// the exact norms: the reference's cos = dot / (n_i n_j) if n_i n_j > 1e-12
__global__ void k_cos_dist(const int32_t *__restrict__ plist, const int *__restrict__ pcount,
                           const int32_t *__restrict__ cand, int L,
                           const double *__restrict__ nrm, double *__restrict__ dist) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)*pcount) return;
    const int slot = plist[q];
    const int i = slot / L, j = cand[slot];
    if (j == INT_MAX) return;
    const double denom = nrm[i] * nrm[j];
    dist[slot] = denom > 1e-12 ? cos_dist(dist[slot], nrm[i], nrm[j]) : 1.0;
}

// sqrt(G_ii): the selection's norms when the exact ones come with the exact
// pass (|G_ii - n_i^2| <= gamma_n n_i^2, like every G_ij)
__global__ void k_gram_diag_norms(const double *__restrict__ G, int f, double *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < f) out[i] = __builtin_sqrt(gram_at(G, f, i, i));
}

// slots of the first kq candidates of every node (they are always evaluated)
__global__ void k_first_pairs(int f, int L, int kq, int32_t *__restrict__ plist) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)f * kq) return;
    plist[q] = (int32_t)((q / kq) * L + q % kq);
}

// the other candidates of node i that can still reach its top k: their lower
// bound d~ - delta does not exceed Dp <= d~_{kq-1} + delta, the upper bound of
// the worst exact distance among the first kq (NaN-safe: -inf approximate
// distances flag non-finite data, everything is evaluated then)
__global__ void k_extra_pairs(const int32_t *__restrict__ cand, const double *__restrict__ capx,
                              int f, int L, int kq, double delta, int32_t *__restrict__ plist,
                              int *__restrict__ pcount) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= f) return;
    const double ak = capx[(int64_t)i * L + kq - 1];
    const double Dp = (ak == -__builtin_inf()) ? __builtin_inf() : ak + delta;
    for (int r = kq; r < L; ++r) {
        const int64_t slot = (int64_t)i * L + r;
        if (cand[slot] == INT_MAX) continue;
        if (!(capx[slot] - delta > Dp)) plist[atomicAdd(pcount, 1)] = (int32_t)slot;
    }
}

__global__ void k_all_cand(int f, int32_t *__restrict__ cand) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)f * f) return;
    const int i = (int)(q / f), j = (int)(q % f);
    cand[q] = i == j ? INT_MAX : j;
}

__global__ void k_iota32(int32_t *__restrict__ v, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

__global__ void k_fill_f64(double *__restrict__ p, int64_t n, double v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void k_cand_pairs(const int32_t *__restrict__ cand, int f, int L,
                             int32_t *__restrict__ pi, int32_t *__restrict__ pj) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)f * L) return;
    pi[q] = (int32_t)(q / L);
    const int c = cand[q];
    pj[q] = c == INT_MAX ? -1 : c;
}

__device__ __forceinline__ double weight_of(double d, double sigma, double p) {
    const double x = d / sigma;
    const double pw = glibc::pow_glibc(x, p);  // glibc pow (glibc_f64.hpp), every p
    return 1.0 / (1.0 + pw);
}

// ---- 6. exact sort + certification + filter ----------------------------------
__global__ __launch_bounds__(256) void k_cos_finish(const int32_t *__restrict__ cand,
                                                    const double *__restrict__ cdist,
                                                    const double *__restrict__ gnext, int f, int L,
                                                    int topk, double eps, double sigma, double p,
                                                    double delta, int32_t *__restrict__ out_idx,
                                                    double *__restrict__ out_dist,
                                                    double *__restrict__ out_w,
                                                    int *__restrict__ fb_count,
                                                    int32_t *__restrict__ fb_list) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= f) return;
    double d[1];
    int ix[1];
    const bool ok = lane < L && cand[(int64_t)i * L + lane] != INT_MAX;
    d[0] = ok ? cdist[(int64_t)i * L + lane] : __builtin_inf();
    ix[0] = ok ? cand[(int64_t)i * L + lane] : INT_MAX;
    wave_bitonic_sort<1>(d, ix);
    const int M = min(L, f - 1);
    const int keff = min(topk, M);
    const double gn = gnext[i];
    bool cert = true;
    if (gn < __builtin_inf() && keff > 0) {
        const double Dk = wave_elem<1>(d, keff - 1);
        cert = (gn - delta) > Dk;
    }
    if (!cert) {
        if (lane == 0) fb_list[atomicAdd(fb_count, 1)] = i;
        return;
    }
    // filter (dist <= eps, w > 1e-12) is monotone in dist: a prefix survives
    const double wv = weight_of(d[0], sigma, p);
    const bool keep = lane < keff && d[0] <= eps && wv > 1e-12;
    const uint64_t km = __ballot(keep);
    const int nkeep = __popcll(~km) == 0 ? 64 : (int)__builtin_ctzll(~km);  // prefix length
    if (lane < topk) {
        const bool k2 = lane < nkeep;
        out_idx[(int64_t)i * topk + lane] = k2 ? ix[0] : -1;
        out_dist[(int64_t)i * topk + lane] = k2 ? d[0] : __builtin_inf();
        if (out_w) out_w[(int64_t)i * topk + lane] = k2 ? wv : 0.0;
    }
}

// ---- fallback: exact all-pairs for uncertified nodes -----------------------------
__global__ void k_fb_pairs(const int32_t *__restrict__ fb_list, const int *__restrict__ fb_count,
                           int f, int32_t *__restrict__ pi, int32_t *__restrict__ pj) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)(*fb_count) * f;
    if (q >= total) return;
    const int node = fb_list[q / f];
    const int j = (int)(q % f);
    pi[q] = node;
    pj[q] = j == node ? -1 : j;
}

template <int NR>
__global__ __launch_bounds__(256) void k_fb_finish(const int32_t *__restrict__ fb_list,
                                                   const int *__restrict__ fb_count,
                                                   const double *__restrict__ fdist, int f,
                                                   int topk, double eps, double sigma, double p,
                                                   int32_t *__restrict__ out_idx,
                                                   double *__restrict__ out_dist,
                                                   double *__restrict__ out_w) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= *fb_count) return;
    const int i = fb_list[b];
    double d[NR];
    int ix[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int j = lane + 64 * r;
        const bool ok = j < f && j != i;
        d[r] = ok ? fdist[(int64_t)b * f + j] : __builtin_inf();
        ix[r] = ok ? j : INT_MAX;
    }
    wave_bitonic_sort<NR>(d, ix);
    const int keff = min(topk, f - 1);
    // the filter is monotone in dist: a prefix of the sorted list survives
    // (element e = lane + 64 r); topk may exceed 64 here (every register)
    int nkeep = 0;
    bool open = true;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        const double wv = weight_of(d[r], sigma, p);
        const bool keep = e < keff && d[r] <= eps && wv > 1e-12;
        const uint64_t km = __ballot(keep);
        if (open) {
            const int run = __popcll(~km) == 0 ? 64 : (int)__builtin_ctzll(~km);
            nkeep += run;
            open = run == 64;
        }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        if (e < topk) {
            const bool k2 = e < nkeep;
            out_idx[(int64_t)i * topk + e] = k2 ? ix[r] : -1;
            out_dist[(int64_t)i * topk + e] = k2 ? d[r] : __builtin_inf();
            if (out_w) out_w[(int64_t)i * topk + e] = k2 ? weight_of(d[r], sigma, p) : 0.0;
        }
    }
    for (int e = 64 * NR + lane; e < topk; e += 64) {  // topk beyond the f - 1 nodes
        out_idx[(int64_t)i * topk + e] = -1;
        out_dist[(int64_t)i * topk + e] = __builtin_inf();
        if (out_w) out_w[(int64_t)i * topk + e] = 0.0;
    }
}

// StandardScaler on the columns of X [n][m] (f64): smartcore's
// StandardScaler::fit/transform as build_laplacian_matrix applies it when
// GraphParams.normalise is set (src_legacy/laplacian.rs:143-150).  smartcore
// is not in the reference tree, so its exact arithmetic is parity-unpinned;
// restated as mean = sequential sum / n, std = sqrt(sequential sum of
// (x - mean)^2 / n), out = (x - mean) / std (std == 0: x - mean).  One thread
// per column, rows streamed (adjacent threads read adjacent columns).
__global__ void k_standardize_cols(const double *__restrict__ X, int64_t n, int m,
                                   double *__restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= m) return;
    double s = 0.0;
    for (int64_t r = 0; r < n; ++r) s = s + X[r * m + c];
    const double mean = s / (double)n;
    double v = 0.0;
    for (int64_t r = 0; r < n; ++r) {
        const double t = X[r * m + c] - mean;
        v = v + t * t;
    }
    const double sd = __builtin_sqrt(v / (double)n);
    for (int64_t r = 0; r < n; ++r) {
        const double t = X[r * m + c] - mean;
        out[r * m + c] = sd > 0.0 ? t / sd : t;
    }
}

inline unsigned grid(int64_t n, int t = 256) {
    return (unsigned)std::max<int64_t>(1, (n + t - 1) / t);
}

}  // namespace kcos

static thread_local mn_knn_stats t_cos_stats{};

template <typename T>
static int knn_cos_columns_impl(const T *X, int64_t n, int32_t f, const mn_cos_opts *o,
                                int32_t *out_idx, double *out_dist, double *out_w) {
    using namespace kcos;
    clear_error();
    t_cos_stats = mn_knn_stats{};
    MN_REQUIRE(o && X && out_idx && out_dist, MN_EINVAL, "mn_knn_cos_columns: NULL argument");
    MN_REQUIRE(n >= 1 && f >= 2 && f <= FMAXC, MN_EINVAL,
               "mn_knn_cos_columns_f32: need n >= 1 and 2 <= f <= %d", FMAXC);
    MN_REQUIRE(o->topk >= 1, MN_EINVAL, "mn_knn_cos_columns_f32: topk >= 1");
    // topk > 64 (graph.rs topk is any usize): every node through the exact
    // all-pairs path (k_fb_finish writes any topk <= f - 1, padding beyond)
    const bool all_exact = o->topk > 64;
    MN_REQUIRE(o->sigma > 0.0, MN_EINVAL, "mn_knn_cos_columns_f32: sigma must be > 0");
    const int margin = o->margin > 0 ? o->margin : 16;
    const int L = std::min(std::min(o->topk + margin, LMAXC), f - 1);
    hipStream_t s = (hipStream_t)o->stream;
    const int ntile = (f + GT - 1) / GT;
    const int ntri = ntile * (ntile + 1) / 2;
    // ~8192 Gram blocks (round 6; was 2048).  Tuning build: MN_COS_GBLK = the
    // target block count (C3, same process, bit-identical: 8192 -> Gram phase
    // 13.35 ms vs 14.6 at 2048, 4096 13.8, 1024 16.1 —
    // profiles/r05/r05_c3_gblk_ab.log)
    const int64_t gblk = knob_int("MN_COS_GBLK", 8192);
    int nchunk = (int)std::max<int64_t>(1, std::min<int64_t>((gblk + ntri - 1) / ntri, (n + 255) / 256));
    int64_t kchunk = (n + nchunk - 1) / nchunk;
    kchunk = ((kchunk + GK - 1) / GK) * GK;
    nchunk = (int)((n + kchunk - 1) / kchunk);

    T *XT = (T *)scratch(kSlotGeneric0, sizeof(T) * (size_t)n * f);
    // layout (bytes): G f^2 x 8, nrm / gnext f x 8 each, flags 64, cand / pi /
    // pj f L x 4 each, (16-aligned) cdist / capx f L x 8 each, fb_list f x 4,
    // (16-aligned) nrmA f x 8, colmax f x 4
    const size_t gbytes = 8 * ((size_t)f * f + 2 * (size_t)f) + 64 + 28 * (size_t)f * L + 16 +
                          4 * (size_t)f + 16 + 12 * (size_t)f + 64;
    char *g = (char *)scratch(kSlotGeneric1, gbytes);
    MN_REQUIRE(XT && g, MN_ENOMEM, "mn_knn_cos_columns_f32: scratch allocation failed");
    double *G = (double *)g;
    double *nrm = G + (size_t)f * f;
    double *gnext = nrm + f;
    int *flags = (int *)(gnext + f);
    int32_t *cand = (int32_t *)(flags + 16);
    int32_t *pi = cand + (size_t)f * L;
    int32_t *pj = pi + (size_t)f * L;
    double *cdist = (double *)(((uintptr_t)(pj + (size_t)f * L) + 15) & ~(uintptr_t)15);
    double *capx = cdist + (size_t)f * L;
    int32_t *fb_list = (int32_t *)(capx + (size_t)f * L);
    double *nrmA = (double *)(((uintptr_t)(fb_list + f) + 15) & ~(uintptr_t)15);
    unsigned *colmax = (unsigned *)(nrmA + f);

    Timer tm;
    tm.start(o->timing != 0, s);
    MN_HIP_TRY(hipMemsetAsync(G, 0, sizeof(double) * (size_t)f * f, s));
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 64, s));
    // the transpose runs on the side stream while the Gram (it reads X itself)
    // occupies the MFMAs (round 4b).  Round 5: the exact norms (768 latency-
    // bound chains) join the exact pass as chains of their own (k_cos_exact_q
    // RAW); the candidate selection takes sqrt(G_ii) instead (error folded into
    // delta).  On the side stream beside the Gram they took 13.7 ms and held
    // the Gram phase at 20.5 ms.  The all-exact path (topk > 64) still needs
    // them first: k_col_norms on the side stream.
    hipStream_t side = side_stream();
    MN_REQUIRE(side, MN_EHIP, "mn_knn_cos_columns_f32: side stream creation failed");
    MN_HIP_TRY(stream_wait(side, s));
    hipLaunchKernelGGL(k_transpose<T>, dim3(grid(n, 64), (unsigned)((f + 63) / 64)), dim3(256), 0, side,
                       X, n, f, XT);
    MN_KCHECK(side, "k_transpose");
    const bool norms_in_pass = !all_exact && knob_int("MN_COS_NORMS_SIDE", 0) == 0;
    if (!norms_in_pass) {
        hipLaunchKernelGGL(k_col_norms<T>, dim3((unsigned)((f + 3) / 4)), dim3(64), 0, side, XT, n,
                           f, nrm);
        MN_KCHECK(side, "k_col_norms");
    }
    const int nr = (f + 63) / 64;
    if (all_exact) {
        MN_HIP_TRY(stream_wait(s, side));
        tm.mark();
        hipLaunchKernelGGL(k_iota32, dim3(grid(f)), dim3(256), 0, s, fb_list, f);
        MN_HIP_TRY(hipMemcpyAsync(flags, &f, 4, hipMemcpyHostToDevice, s));
        MN_HIP_TRY(hipGetLastError());
    } else {
        // Tuning build, MN_COS_GRAM = 1: the f32-MFMA Gram (k_gram_f32m, f64
        // fold every G3F rows) when the exact norms come with the exact pass;
        // its bound needs every column max in [2^-20, 2^40] (or 0) — checked
        // on the device, else G is recomputed on f64 MFMA.  C3 (same process,
        // profiles/r05/r05_c3_gram32_ab.log): Gram phase 13.5 vs 14.4 ms, but
        // the wider delta adds ~1 exact chain per node (exact pass 8.1 -> 9.4
        // ms): slower overall, not the default.
        bool f32g = false;
        double e32 = 0.0;  // |G~_ij - dot_ij| <= e32 n_i n_j (f32 Gram)
        if (sizeof(T) == 4 && norms_in_pass && knob_int("MN_COS_GRAM", 0) == 1) {
            const int nt3 = (f + G3T - 1) / G3T;
            const int ntri3 = nt3 * (nt3 + 1) / 2;
            int nch3 = (int)std::max<int64_t>(1, std::min<int64_t>((1024 + ntri3 - 1) / ntri3,
                                                                   (n + G3F - 1) / G3F));
            int64_t kch3 = (n + nch3 - 1) / nch3;
            kch3 = (kch3 + G3F - 1) / G3F * G3F;  // fold windows aligned to the chunk
            nch3 = (int)((n + kch3 - 1) / kch3);
            MN_HIP_TRY(hipMemsetAsync(colmax, 0, 4 * (size_t)f, s));
            hipLaunchKernelGGL(k_gram_f32m, dim3((unsigned)(ntri3 * nch3)), dim3(256), 0, s,
                               (const float *)X, n, f, nt3, kch3, G, colmax);
            MN_KCHECK(s, "k_gram_f32m");
            hipLaunchKernelGGL(k_colmax_check, dim3(grid(f)), dim3(256), 0, s, colmax, f, flags + 3);
            int bad = 0;
            MN_HIP_TRY(hipMemcpyAsync(&bad, flags + 3, 4, hipMemcpyDeviceToHost, s));
            MN_HIP_TRY(hipStreamSynchronize(s));
            if (!bad) {
                f32g = true;
                e32 = (double)(G3F + 8) * 0x1p-24 +
                      ((double)n / G3F + (double)nch3 + 8.0) * 0x1p-53;
            } else {
                MN_HIP_TRY(hipMemsetAsync(G, 0, sizeof(double) * (size_t)f * f, s));
            }
        }
        // (measured and dropped: the same f64 arithmetic on 128 x 128 tiles,
        // 21 instead of 78 upper tiles — 20.7 vs 14.5 ms,
        // profiles/r05/r05_c3_gram_tiles_ab.log)
        if (!f32g)
            hipLaunchKernelGGL(k_gram_f64<T>, dim3((unsigned)(ntri * nchunk)), dim3(256), 0, s, X, n,
                               f, ntile, kchunk, nchunk, G);
        MN_HIP_TRY(hipGetLastError());
        MN_HIP_TRY(stream_wait(s, side));
        tm.mark();
        // the selection's band around the reference's 1e-12 cut (relative)
        // (f64 Gram: |G_ii - n_i^2| <= gamma_n n_i^2 grows like n u, so the
        // band scales with n once 4 (n + 16) 2^-53 passes 1e-8, n ~ 9e7)
        const double amb_rel = f32g ? 4.0 * e32 : std::max(1e-8, 4.0 * ((double)n + 16.0) * 0x1p-53);
        // approximate norms sqrt(G_ii) for the selection when the exact ones
        // come with the exact pass
        if (norms_in_pass)
            hipLaunchKernelGGL(k_gram_diag_norms, dim3(grid(f)), dim3(256), 0, s, G, f, nrmA);
        const double *nsel = norms_in_pass ? nrmA : nrm;
    #define MN_SEL(NRV) hipLaunchKernelGGL(k_cos_select<NRV>, dim3(grid(f, 4)), dim3(256), 0, s, G, nsel, f, L, cand, capx, gnext, 1e-12 * amb_rel)
        if (nr <= 1) MN_SEL(1); else if (nr <= 2) MN_SEL(2); else if (nr <= 4) MN_SEL(4);
        else if (nr <= 8) MN_SEL(8); else if (nr <= 16) MN_SEL(16); else if (nr <= 32) MN_SEL(32);
        else MN_SEL(64);
    #undef MN_SEL
        // exact distances: the first kq candidates of every node, then the ones
        // whose lower bound can still reach the top k (the rest stay +inf)
        // |d~ - d| bound: f64 accumulation of n products (f64 inputs: each product
        // rounded once more), norms and the quotient, with a factor-2 margin
        // With the norms from G_ii (error <= the Gram's own, gamma_n each) the
        // bound doubles: 4 (n + 16) u keeps the factor-2 margin.
        // The f32 Gram: |cos~ - cos| <= 2 e32 / (1 - e32) (dot and norms), x 2
        // margin, plus the f64 rounding of the distance itself.
        const double delta =
            f32g ? 4.02 * e32 + 64.0 * 0x1p-53
                 : (norms_in_pass ? 4.0 : 2.0) * ((double)n + (sizeof(T) == 8 ? 17.0 : 16.0)) * 0x1p-53 +
                       1e-300;
        const int kq = std::min(o->topk, L);
        const int fkq = f * kq;
        hipLaunchKernelGGL(k_fill_f64, dim3(grid((int64_t)f * L)), dim3(256), 0, s, cdist,
                           (int64_t)f * L, __builtin_inf());
        // one pass over one list: [first kq of every node | near ties], the
        // count of the latter appended on the device (flags[1])
        hipLaunchKernelGGL(k_first_pairs, dim3(grid((int64_t)f * kq)), dim3(256), 0, s, f, L, kq, pi);
        MN_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(flags + 1), fkq, 1, s));
        if (L > kq)
            hipLaunchKernelGGL(k_extra_pairs, dim3(grid(f)), dim3(256), 0, s, cand, capx, f, L, kq,
                               delta, pi, flags + 1);
        // chunks in flight ahead of the chains: 4 (C3, same process,
        // profiles/r04/r04_c3_pf_ab.log: exact pass 8.33-8.42 ms vs 8.44-8.68 at
        // 2 — the chains are bound by their adds, not by the loads); tuning build: MN_COS_PF
        // round 5: sixteen chains a wave (k_cos_exact_q);
        // tuning build: MN_COS_EXACT = 0 runs the four-chain form
        const int pfd = knob_int("MN_COS_PF", 4);
        if (norms_in_pass) {
            // the listed pairs' raw dots (into cdist) and the f norm chains
            // (into nrm) in one pass, then the distances
            // (measured and dropped: a producer / consumer pair of waves per
            // sixteen chains, one barrier a 64-element chunk — 11.4 vs 8.15 ms
            // with __syncthreads and with a raw s_barrier alike,
            // profiles/r05/r05_c3_pc_ab.log, r05_c3_pc2_ab.log)
            // lanes a chain: 8 — eight chains a wave, twice the waves of the
            // sixteen-chain form (C3 exact pass 8.17 -> 7.6 ms, same process,
            // profiles/r05/r05_c3_lpc_ab.log); tuning build: MN_COS_LPC = 4 / 16
            const int lpc = knob_int("MN_COS_LPC", 8);
            auto kq = k_cos_exact_q<T, 4, true, 8>;
            if (lpc == 4) kq = pfd == 8 ? k_cos_exact_q<T, 8, true, 4> : k_cos_exact_q<T, 4, true, 4>;
            if (lpc == 16) kq = k_cos_exact_q<T, 4, true, 16>;
            const int cpw = 64 / (lpc == 4 ? 4 : (lpc == 16 ? 16 : 8));
            hipLaunchKernelGGL(kq, dim3(grid((int64_t)f * L + f, cpw)), dim3(64), 0, s, XT, n, pi,
                               flags + 1, (int64_t)f * L, cand, L, f, nrm, cdist);
            hipLaunchKernelGGL(k_cos_dist, dim3(grid((int64_t)f * L)), dim3(256), 0, s, pi, flags + 1,
                               cand, L, nrm, cdist);
        } else if (knob_int("MN_COS_EXACT", 1) == 1) {
            // chunks in flight: 4 (C3: 8.13 ms; 8: 9.0 ms, the four-chain
            // form 8.36 ms — profiles/r05/r05_c3_exact_ab.log)
            auto kq8 = k_cos_exact_q<T, 4>;
            if (pfd == 8) kq8 = k_cos_exact_q<T, 8>;
            hipLaunchKernelGGL(kq8, dim3(grid((int64_t)f * L, 16)), dim3(64), 0, s, XT, n, pi,
                               flags + 1, (int64_t)f * L, cand, L, 0, nrm, cdist);
        } else {
            auto kx = k_cos_exact_wave<T, 2>;
            if (pfd == 4) kx = k_cos_exact_wave<T, 4>;
            hipLaunchKernelGGL(kx, dim3(grid((int64_t)f * L, 16)), dim3(256), 0, s, XT, n, pi,
                               flags + 1, (int64_t)f * L, cand, L, nrm, cdist);
        }
        hipLaunchKernelGGL(k_cos_finish, dim3(grid(f, 4)), dim3(256), 0, s, cand, cdist, gnext, f, L,
                           o->topk, o->eps, o->sigma, o->p, delta, out_idx, out_dist, out_w, flags,
                           fb_list);
        MN_HIP_TRY(hipGetLastError());
    }
    tm.mark();
    int nfb = 0;
    MN_HIP_TRY(hipMemcpyAsync(&nfb, flags, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (nfb > 0) {  // exact all-pairs for the uncertified nodes
        const int64_t np = (int64_t)nfb * f;
        int32_t *fpi = nullptr, *fpj = nullptr;
        double *fd = nullptr;
        MN_HIP_TRY(hipMalloc(&fpi, 4 * np));
        MN_HIP_TRY(hipMalloc(&fpj, 4 * np));
        MN_HIP_TRY(hipMalloc(&fd, 8 * np));
        if (all_exact) {
            // every ordered pair: the wave form (four ordered LDS chains a wave),
            // node i = slot / f (fb_list is the identity here), cand = j or
            // INT_MAX on the diagonal
            hipLaunchKernelGGL(k_all_cand, dim3(grid(np)), dim3(256), 0, s, f, fpj);
            hipLaunchKernelGGL((k_cos_exact_q<T, 4>), dim3(grid(np, 16)), dim3(64), 0, s, XT, n,
                               (const int32_t *)nullptr, (const int *)nullptr, np, fpj, f, 0, nrm, fd);
        } else {
            hipLaunchKernelGGL(k_fb_pairs, dim3(grid(np)), dim3(256), 0, s, fb_list, flags, f, fpi, fpj);
            hipLaunchKernelGGL(k_cos_exact<T>, dim3(grid(np)), dim3(256), 0, s, XT, n, fpi, fpj, np, nrm, fd);
        }
#define MN_FB(NRV) hipLaunchKernelGGL(k_fb_finish<NRV>, dim3(grid(nfb, 4)), dim3(256), 0, s, fb_list, flags, fd, f, o->topk, o->eps, o->sigma, o->p, out_idx, out_dist, out_w)
        if (nr <= 1) MN_FB(1); else if (nr <= 2) MN_FB(2); else if (nr <= 4) MN_FB(4);
        else if (nr <= 8) MN_FB(8); else if (nr <= 16) MN_FB(16); else if (nr <= 32) MN_FB(32);
        else MN_FB(64);
#undef MN_FB
        MN_HIP_TRY(hipGetLastError());
        MN_HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(fpi); (void)hipFree(fpj); (void)hipFree(fd);
    }
    tm.mark();
    MN_HIP_TRY(hipStreamSynchronize(s));
    t_cos_stats.n_queries = f;
    t_cos_stats.n_uncertified = nfb;
    t_cos_stats.slices = nchunk;
    t_cos_stats.list_len = L;
    if (tm.on) {
        t_cos_stats.ms_gram = tm.ms(0, 1);
        t_cos_stats.ms_rerank = tm.ms(1, 2);
        t_cos_stats.ms_fallback = tm.ms(2, 3);
        t_cos_stats.ms_total = tm.ms(0, 3);
    }
    return MN_OK;
}

}  // namespace mn

extern "C" {

int mn_knn_cos_columns_f32(const float *X, int64_t n_rows, int32_t f, const mn_cos_opts *opts,
                           int32_t *out_idx, double *out_dist, double *out_w) {
    return mn::knn_cos_columns_impl<float>(X, n_rows, f, opts, out_idx, out_dist, out_w);
}

int mn_knn_cos_columns_f64(const double *X, int64_t n_rows, int32_t f, const mn_cos_opts *opts,
                           int32_t *out_idx, double *out_dist, double *out_w) {
    return mn::knn_cos_columns_impl<double>(X, n_rows, f, opts, out_idx, out_dist, out_w);
}

int mn_standardize_columns_f64(const double *X, int64_t n_rows, int32_t n_cols, double *out,
                               void *stream) {
    mn::clear_error();
    MN_REQUIRE(X && out && n_rows >= 1 && n_cols >= 1, MN_EINVAL,
               "mn_standardize_columns_f64: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mn::kcos::k_standardize_cols, dim3(mn::kcos::grid(n_cols)), dim3(256), 0,
                       s, X, n_rows, n_cols, out);
    MN_KCHECK(s, "k_standardize_cols");
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

int mn_cos_last_stats(mn_knn_stats *out) {
    if (!out) return MN_EINVAL;
    *out = mn::t_cos_stats;
    return MN_OK;
}

}  // extern "C"
