// knn_f32.hip — K1: brute-force L2^2 kNN on gfx950, bit-exact vs the reference.
//
// Reference semantics (what the output must equal, bit for bit):
//   surfface-core/src/distance.rs:206-213  d(a,b) = sequential f32 fold of
//       (a_t - b_t)^2, no FMA;
//   surfface-core/src/mst.rs:330-360       for every row i, all j != i, stable
//       sort by d (=> ties by ascending j), keep min(k, n-1).
//
// MI355X design:
//   1. k_row_norms      one wave per row: ||x||^2 (f32), max corpus norm,
//                       non-finite input flag (reference panics on NaN).
//   2. k_gram_topk      candidate generation.  A 128-query x 256-corpus tile of
//                       the Gram matrix on MFMA v_mfma_f32_16x16x4_f32 (exact
//                       f32 products, f32 accumulate), operands staged through
//                       LDS (register staging, double buffer, padded rows =>
//                       conflict-free ds_read_b128).  The epilogue forms
//                       d~ = |q|^2 + |c|^2 - 2 q.c and filters it against a
//                       per-query threshold tau (the current L-th best);
//                       survivors go to an LDS queue per query; a full queue is
//                       merged into the query's sorted top-L list (global
//                       memory, wave-wide bitonic sort).  The N x N matrix is
//                       never materialised.
//   3. k_rerank         one wave per query: the L (x slices) candidates are
//                       re-ranked with the REFERENCE arithmetic (sequential f32
//                       fold, contraction off: the library is compiled with
//                       -ffp-contract=off), sorted by (dist, idx) and
//                       certified: every non-candidate has d~ >= tau_L, and
//                       |d~ - d| <= delta = 2(4d+16)u(|q|^2 + max|c|^2), so
//                       tau_L - delta > D_k proves the top-k is exact.
//   4. k_fallback       uncertified rows (massive exact ties, overflow) are
//                       recomputed by an exact brute-force scan.
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "gram_bf16.hpp"
#include "gram_sweep2.hpp"
#include "gram_sweep3.hpp"
#include "shard_sym.hpp"

namespace mn {

// sortkeys.hip
hipError_t sort_f32_pairs(const float *keys_in, float *keys_out, const int *vals_in,
                          int *vals_out, int64_t n, hipStream_t s);

namespace knn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128;             // query rows per block (8 waves x 16 rows)
constexpr int BN = 256;             // corpus rows per tile (16 column tiles of 16)
constexpr int BK = 16;              // feature depth per LDS stage
constexpr int LDK = BK + 8;         // padded row stride (floats, 96 B): conflict-free b128 reads
constexpr int NWAVES = 8;
constexpr int NT = 64 * NWAVES;
constexpr int NCT = BN / 16;        // column tiles per corpus tile
constexpr int QCAP = 48;            // LDS candidate queue per query
constexpr int QPRE = QCAP - 16;     // merge before a column tile if cnt > QPRE
constexpr int LMAX = 128 - QCAP;    // L + QCAP <= 128 (two elements per lane)
constexpr int KMAX = 64;            // k limit of the C ABI
constexpr int KBIG = 512;           // k limit of the exact split-scan path (k > KMAX)
constexpr int KLIST = KMAX + 8;     // internal list limit (MN_L2's extended L2^2 list;
                                    // the fallback keeps it per thread in LDS)
constexpr int FB_THREADS = 128;

struct alignas(16) GramSmem {
    float A[2][BM][LDK];
    float B[2][BN][LDK];
    float qd[BM][QCAP];
    int qi[BM][QCAP];
    float cn[2][BN];
    float qn[BM];
    float tau[BM];
    int cnt[BM];
    int lsz[BM];
    int ovf[BM];  // a valid pair had a non-finite d~ (overflow): force the exact path
};

// ---------------------------------------------------------------------------
// 1. row norms + input validation
// ---------------------------------------------------------------------------
template <bool VEC4>
__global__ __launch_bounds__(256) void k_row_norms(const float *__restrict__ X, int64_t n,
                                                   int d, float *__restrict__ nrm,
                                                   unsigned *__restrict__ maxbits,
                                                   int *__restrict__ nonfinite) {
    const int lane = threadIdx.x & 63;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    unsigned mx = 0u;  // max |x|^2 bits (one atomic per wave)
    for (int64_t row = wave0; row < n; row += nwaves) {
        const float *p = X + row * (int64_t)d;
        float s = 0.f;
        bool bad = false;
        if (VEC4) {
            for (int t = lane * 4; t < d; t += 256) {
                const float4 v = *reinterpret_cast<const float4 *>(p + t);
                s = __builtin_fmaf(v.x, v.x, s);
                s = __builtin_fmaf(v.y, v.y, s);
                s = __builtin_fmaf(v.z, v.z, s);
                s = __builtin_fmaf(v.w, v.w, s);
                bad |= !(__builtin_isfinite(v.x) && __builtin_isfinite(v.y) &&
                         __builtin_isfinite(v.z) && __builtin_isfinite(v.w));
            }
        } else {
            for (int t = lane; t < d; t += 64) {
                const float v = p[t];
                s = __builtin_fmaf(v, v, s);
                bad |= !__builtin_isfinite(v);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        const bool anybad = __any(bad);
        if (lane == 0) {
            nrm[row] = s;
            if (anybad) atomicOr(nonfinite, 1);
            mx = max(mx, __builtin_isfinite(s) ? __float_as_uint(s) : 0x7f800000u);
        }
    }
    wave_atomic_umax(maxbits, mx);
}

// ---------------------------------------------------------------------------
// 2. Gram (MFMA) + threshold filter + per-query top-L lists
// ---------------------------------------------------------------------------
template <bool VEC4>
__device__ __forceinline__ float4 load4(const float *__restrict__ X, int64_t row, int64_t nrows,
                                        int d, int k) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row >= nrows) return v;
    const float *p = X + row * (int64_t)d + k;
    if (VEC4) {
        if (k < d) v = *reinterpret_cast<const float4 *>(p);
    } else {
        if (k + 0 < d) v.x = p[0];
        if (k + 1 < d) v.y = p[1];
        if (k + 2 < d) v.z = p[2];
        if (k + 3 < d) v.w = p[3];
    }
    return v;
}

// Merge the LDS queue of `row` into its sorted top-L list (global).  Wave-wide.
__device__ __forceinline__ void merge_row(GramSmem &sm, int row, int L, float *__restrict__ ld,
                                          int *__restrict__ li) {
    const int lane = threadIdx.x & 63;
    const int s = sm.lsz[row];
    const int c = sm.cnt[row];
    float d[2];
    int ix[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        if (e < s) {
            d[r] = ld[e];
            ix[r] = li[e];
        } else if (e < s + c) {
            d[r] = sm.qd[row][e - s];
            ix[r] = sm.qi[row][e - s];
        } else {
            d[r] = __builtin_inff();
            ix[r] = INT_MAX;
        }
    }
    wave_bitonic_sort<2>(d, ix);
    const int ns = min(L, s + c);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        if (e < ns) {
            ld[e] = d[r];
            li[e] = ix[r];
        }
    }
    const float tl = wave_elem<2>(d, L - 1);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        sm.lsz[row] = ns;
        sm.cnt[row] = 0;
        sm.tau[row] = (ns == L) ? tl : __builtin_inff();
    }
    __builtin_amdgcn_wave_barrier();
}

template <bool VEC4>
__global__ __launch_bounds__(NT) void k_gram_topk(
    const float *__restrict__ Q, int64_t nq, const float *__restrict__ C, int64_t nc, int d,
    int64_t q_off, int64_t c_off, int excl, const float *__restrict__ qnrm,
    const float *__restrict__ cnrm, int L, int S, int64_t chunk, float *__restrict__ list_d,
    int *__restrict__ list_i, int *__restrict__ out_lsz, float *__restrict__ out_tau) {
    __shared__ GramSmem sm;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int g = lane >> 4;   // MFMA row group (C/D: row = 4g + reg)
    const int cl = lane & 15;  // MFMA column within a 16-wide tile
    const int64_t q0 = (int64_t)blockIdx.x * BM;
    const int sl = blockIdx.y;
    const int64_t cbeg = (int64_t)sl * chunk;
    const int64_t cend = min(nc, cbeg + chunk);

    for (int r = tid; r < BM; r += NT) {
        sm.qn[r] = (q0 + r < nq) ? qnrm[q0 + r] : 0.f;
        sm.tau[r] = __builtin_inff();
        sm.cnt[r] = 0;
        sm.lsz[r] = 0;
        sm.ovf[r] = 0;
    }
    __syncthreads();

    const int nk = (d + BK - 1) / BK;
    // staging map: A = 128 rows x 4 float4 (1 per thread), B = 256 x 4 (2 per thread)
    const int a_row = tid >> 2, a_c4 = tid & 3;
    int tile_par = 0;

    for (int64_t c0 = cbeg; c0 < cend; c0 += BN, tile_par ^= 1) {
        if (tid < BN) sm.cn[tile_par][tid] = (c0 + tid < cend) ? cnrm[c0 + tid] : 0.f;

        f32x4 acc[NCT];
#pragma unroll
        for (int t = 0; t < NCT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

        float4 ra, rb0, rb1;
        ra = load4<VEC4>(Q, q0 + a_row, nq, d, 4 * a_c4);
        rb0 = load4<VEC4>(C, c0 + a_row, cend, d, 4 * a_c4);
        rb1 = load4<VEC4>(C, c0 + 128 + a_row, cend, d, 4 * a_c4);
        *reinterpret_cast<float4 *>(&sm.A[0][a_row][4 * a_c4]) = ra;
        *reinterpret_cast<float4 *>(&sm.B[0][a_row][4 * a_c4]) = rb0;
        *reinterpret_cast<float4 *>(&sm.B[0][128 + a_row][4 * a_c4]) = rb1;
        __syncthreads();

        for (int kt = 0; kt < nk; ++kt) {
            const int cur = kt & 1;
            const bool more = kt + 1 < nk;
            if (more) {
                const int k = (kt + 1) * BK + 4 * a_c4;
                ra = load4<VEC4>(Q, q0 + a_row, nq, d, k);
                rb0 = load4<VEC4>(C, c0 + a_row, cend, d, k);
                rb1 = load4<VEC4>(C, c0 + 128 + a_row, cend, d, k);
            }
            const float4 a = *reinterpret_cast<const float4 *>(&sm.A[cur][16 * w + cl][4 * g]);
#pragma unroll
            for (int t = 0; t < NCT; ++t) {
                const float4 b = *reinterpret_cast<const float4 *>(&sm.B[cur][16 * t + cl][4 * g]);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc[t], 0, 0, 0);
            }
            if (more) {
                *reinterpret_cast<float4 *>(&sm.A[cur ^ 1][a_row][4 * a_c4]) = ra;
                *reinterpret_cast<float4 *>(&sm.B[cur ^ 1][a_row][4 * a_c4]) = rb0;
                *reinterpret_cast<float4 *>(&sm.B[cur ^ 1][128 + a_row][4 * a_c4]) = rb1;
            }
            __syncthreads();
        }

        // ---- epilogue: filter + queue + merge (this wave's 16 rows only) ----
#pragma unroll 1
        for (int t = 0; t < NCT; ++t) {
            {   // pre-merge rows that could overflow while taking 16 more candidates
                const int myrow = 16 * w + cl;
                const int c = sm.cnt[myrow];
                uint64_t need = __ballot(lane < 16 && c > QPRE);
                while (need) {
                    const int rr = __builtin_ctzll(need);
                    need &= need - 1;
                    const int row = 16 * w + rr;
                    const int64_t base = ((q0 + row) * S + sl) * (int64_t)L;
                    merge_row(sm, row, L, list_d + base, list_i + base);
                }
            }
            f32x4 curv;
            switch (t) {
#define MN_CASE(T) case T: curv = acc[T]; break;
                MN_CASE(0) MN_CASE(1) MN_CASE(2) MN_CASE(3) MN_CASE(4) MN_CASE(5) MN_CASE(6)
                MN_CASE(7) MN_CASE(8) MN_CASE(9) MN_CASE(10) MN_CASE(11) MN_CASE(12)
                MN_CASE(13) MN_CASE(14) MN_CASE(15)
#undef MN_CASE
                default: curv = acc[0];
            }
            const int64_t col = c0 + 16 * t + cl;
            const bool colok = col < cend;
            const float cv = sm.cn[tile_par][16 * t + cl];
            const int64_t gcol = c_off + col;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int lrow = 16 * w + 4 * g + i;
                const int64_t q = q0 + lrow;
                const float tv = sm.tau[lrow];
                const float dd = __builtin_fmaf(-2.f, curv[i], sm.qn[lrow] + cv);
                const bool valid = colok && (q < nq) && !(excl && (q_off + q) == gcol);
                const bool pass = valid && (dd < tv);
                if (__ballot(valid && !(dd < __builtin_inff()))) {
                    // d~ overflowed (or NaN): the threshold argument no longer
                    // covers this pair, so the row is resolved exactly later.
                    if (valid && !(dd < __builtin_inff())) sm.ovf[lrow] = 1;
                    __builtin_amdgcn_wave_barrier();
                }
                const uint64_t m = __ballot(pass);
                if (m) {
#pragma unroll
                    for (int gg = 0; gg < 4; ++gg) {
                        const uint32_t mg = (uint32_t)(m >> (16 * gg)) & 0xFFFFu;
                        if (!mg) continue;
                        const int row = 16 * w + 4 * gg + i;
                        const int c = sm.cnt[row];
                        if (g == gg && pass) {
                            const int pos = c + __popc(mg & ((1u << cl) - 1u));
                            sm.qd[row][pos] = dd;
                            sm.qi[row][pos] = (int)gcol;
                        }
                        __builtin_amdgcn_wave_barrier();
                        if (lane == 0) sm.cnt[row] = c + __popc(mg);
                        __builtin_amdgcn_wave_barrier();
                    }
                }
            }
        }
    }

    // ---- flush the queues, publish list sizes and thresholds ----
    for (int rr = 0; rr < 16; ++rr) {
        const int row = 16 * w + rr;
        if (sm.cnt[row] > 0) {
            const int64_t base = ((q0 + row) * S + sl) * (int64_t)L;
            merge_row(sm, row, L, list_d + base, list_i + base);
        }
    }
    if (lane < 16) {
        const int row = 16 * w + lane;
        const int64_t q = q0 + row;
        if (q < nq) {
            out_lsz[q * S + sl] = sm.lsz[row];
            out_tau[q * S + sl] = sm.ovf[row] ? -__builtin_inff() : sm.tau[row];
        }
    }
}

// ---------------------------------------------------------------------------
// 3. exact re-rank + certification
// ---------------------------------------------------------------------------

// The reference fold (distance.rs:206-213): acc starts at -0.0 and adds each
// (a-b)^2 in feature order; -ffp-contract=off keeps mul and add separate.
constexpr int EXU = 4;  // (8: 47 vs 43 ms at C2, profiles/r03n_rerank_unroll.log)
template <bool VEC4>
__device__ __forceinline__ float exact_l2sq(const float *__restrict__ a,
                                            const float *__restrict__ b, int d) {
    float acc = -0.0f;
    if (VEC4) {
        const float4 *a4 = reinterpret_cast<const float4 *>(a);
        const float4 *b4 = reinterpret_cast<const float4 *>(b);
        const int d4 = d >> 2;
        int t = 0;
        // EXU float4 of the (random) candidate row in flight per lane ahead of
        // the ordered adds (a one-at-a-time loop waits on each gather)
        for (; t + EXU <= d4; t += EXU) {
            float4 y[EXU], x[EXU];
#pragma unroll
            for (int u = 0; u < EXU; ++u) y[u] = b4[t + u];
#pragma unroll
            for (int u = 0; u < EXU; ++u) x[u] = a4[t + u];
#pragma unroll
            for (int u = 0; u < EXU; ++u) {
                float df = x[u].x - y[u].x; acc = acc + df * df;
                df = x[u].y - y[u].y; acc = acc + df * df;
                df = x[u].z - y[u].z; acc = acc + df * df;
                df = x[u].w - y[u].w; acc = acc + df * df;
            }
        }
        for (; t < d4; ++t) {
            const float4 x = a4[t], y = b4[t];
            float df = x.x - y.x; acc = acc + df * df;
            df = x.y - y.y; acc = acc + df * df;
            df = x.z - y.z; acc = acc + df * df;
            df = x.w - y.w; acc = acc + df * df;
        }
    } else {
        for (int t = 0; t < d; ++t) {
            const float df = a[t] - b[t];
            acc = acc + df * df;
        }
    }
    return acc;
}

template <int NR, bool VEC4>
__global__ __launch_bounds__(256) void k_rerank(
    const float *__restrict__ Q, int64_t nq, const float *__restrict__ C, int64_t nc, int d,
    int64_t c_off, const float *__restrict__ qnrm, const unsigned *__restrict__ cmax_bits,
    int S, int L, const float *__restrict__ list_d, const int *__restrict__ list_i,
    const int *__restrict__ lsz, const float *__restrict__ ltau, int k, float cert_c,
    int32_t *__restrict__ out_idx, float *__restrict__ out_dist, int *__restrict__ fb_count,
    int *__restrict__ fb_list) {
    (void)list_d;
    (void)nc;
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    float dd[NR];
    int ix[NR];
    int M = 0;
    float G = __builtin_inff();
    bool forced = false;
    for (int s = 0; s < S; ++s) {
        const int sz = lsz[q * S + s];
        const float ts = ltau[q * S + s];
        forced |= (ts == -__builtin_inff());
        if (sz >= L) G = fminf(G, ts);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int e = lane + 64 * r;
            if (s == 0) ix[r] = -1;
            if (e >= M && e < M + sz) ix[r] = list_i[(q * S + s) * (int64_t)L + (e - M)];
        }
        M += sz;
    }
    const float *qrow = Q + q * (int64_t)d;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if (ix[r] >= 0) {
            dd[r] = exact_l2sq<VEC4>(qrow, C + ((int64_t)ix[r] - c_off) * d, d);
        } else {
            dd[r] = __builtin_inff();
            ix[r] = INT_MAX;
        }
    }
    wave_bitonic_sort<NR>(dd, ix);
    const int keff = min(k, M);
    if (forced) {
        if (lane == 0) {
            const int pos = atomicAdd(fb_count, 1);
            fb_list[pos] = (int)q;
        }
    } else if (G < __builtin_inff()) {  // some slice rejected candidates: certify
        const float Dk = keff > 0 ? wave_elem<NR>(dd, keff - 1) : -__builtin_inff();
        const float cmax = __uint_as_float(*cmax_bits);
        const float delta = cert_c * (qnrm[q] + cmax) + 1e-38f;
        const bool cert = (G - delta) > Dk;  // NaN/inf-safe: false => fallback
        if (!cert && lane == 0) {
            const int pos = atomicAdd(fb_count, 1);
            fb_list[pos] = (int)q;
        }
    }
    wave_store_list<NR>(dd, ix, k, keff, out_idx + q * k, out_dist + q * k);
}

// ---------------------------------------------------------------------------
// 2b. bf16-split candidate path (default): split + buffer-based exact re-rank.
//     The Gram runs on bf16 MFMA (gram_bf16.hpp, GM_L2) at 16x the f32 MFMA
//     rate per instruction, three instructions per 16 features.
// ---------------------------------------------------------------------------

// Corpus visiting order of the running-threshold generators: a fixed
// pseudo-random bijection perm(i) = (A i + B) mod n (A ~ 0.618 n, coprime
// with n).  Corpora stored in a sorted order (rows sorted along a coordinate)
// would otherwise make nearly every pair beat the running L-th best and
// overflow the candidate buffers; in a golden-ratio order the threshold
// updates behave as for random order (about L (1 + ln(m / L)) writes).
__global__ __launch_bounds__(256) void k_perm_init(int *__restrict__ perm, int *__restrict__ ipos,
                                                   int64_t n, uint64_t a, uint64_t b) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = (int)((a * (uint64_t)i + b) % (uint64_t)n);  // a, b < n < 2^31
    perm[i] = r;
    if (ipos) ipos[r] = (int)i;
}
__global__ __launch_bounds__(256) void k_gather_f32(const float *__restrict__ src,
                                                    const int *__restrict__ perm, int64_t n,
                                                    float *__restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}

// f32 -> bf16, round to nearest even (finite inputs; values beyond the bf16
// range round to +-inf, which the Gram epilogue flags as unusable).
__device__ __forceinline__ uint32_t bf16_rne(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// X [n][d] f32 -> XS [n][2 dp] bf16, per 32-feature group [hi 32 | lo 32]:
// hi = bf16(x), lo = bf16(x - hi) (x - hi is exact in f32), so
// |x - hi - lo| <= 2^-16 |x|.  Subnormal parts are flushed here (the bf16
// MFMA may flush them anyway), which adds at most 2^-126 per term: covered by
// the absolute slack of the certification bound.  Features d..dp-1 are 0.
__global__ __launch_bounds__(256) void k_split_bf16(const float *__restrict__ X, int64_t n, int d,
                                                    int dp, uint16_t *__restrict__ XS,
                                                    const int *__restrict__ perm) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int per = dp >> 3;
    if (e >= n * per) return;
    const int64_t orow = e / per;
    const int64_t row = perm ? (int64_t)perm[orow] : orow;  // source row
    const int f0 = (int)(e - orow * per) * 8;
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
        uint32_t hp[2], lp[2];
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int f = f0 + u + v;
            const float x = f < d ? X[row * (int64_t)d + f] : 0.f;
            uint32_t hb = 0, lb = 0;
            if (__builtin_fabsf(x) >= 0x1p-126f) {
                hb = bf16_rne(x);
                const float r = x - __uint_as_float(hb << 16);
                lb = __builtin_fabsf(r) >= 0x1p-126f ? bf16_rne(r) : 0u;
            }
            hp[v] = hb;
            lp[v] = lb;
        }
        hw[u >> 1] = hp[0] | (hp[1] << 16);
        lw[u >> 1] = lp[0] | (lp[1] << 16);
    }
    uint16_t *o = XS + orow * (int64_t)(2 * dp) + 64 * (f0 >> 5) + (f0 & 31);
    *reinterpret_cast<uint4 *>(o) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    *reinterpret_cast<uint4 *>(o + 32) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
}

// One wave per query: gather the buffered candidates of every slice (key <=
// the slice's final tau), order them by key, evaluate the reference fold for
// the best kq and then for every other candidate whose lower bound key - delta
// does not exceed the worst of those (the rest cannot enter the top k), sort by
// (dist, idx) and certify: every pair never buffered (or dropped) had key >=
// T = min_s tau_s, so T - delta > D_k proves the top k exact.
//   delta = cert_c (|q|^2 + max|c|^2) + 2^-100 bounds |d~ - d| (split
//   residuals and the dropped lo.lo term <= 3 2^-16 sum|q_t c_t|, f32
//   accumulation of 3 dp exact products, the two norms, the final fma; sum
//   |q_t c_t| <= (|q|^2 + |c|^2)/2; 2^-100 covers flushed subnormal parts).
// |d~ - d_ref| bound of the split generator for query q (bf16x3):
//   dot error  <= (3 2^-16 + gamma) sum|q_t c_t| (1 + 2^-6),  gamma = 6 dp u
//   (3 dp exact products accumulated in f32; 2x the round-to-nearest bound,
//   so any internal rounding of the MFMA adder is covered), sum|q_t c_t| <=
//   |q| max|c| (Cauchy-Schwarz); key = |q|^2 + |c|^2 - 2 dot~: x2, plus the
//   norms' lane-parallel f32 folds and the final fma (24 u (|q|^2 + max|c|^2));
//   plus the reference fold's own error (d + 3) u (Mkey + base) where Mkey
//   bounds the keys the bound is applied to.  Evaluated in f64, rounded up.
__device__ __forceinline__ float delta_x3(float qn, float cmax, int dp, int d, float mkey) {
    const double u = 0x1p-24;
    const double qa = __builtin_sqrt((double)qn) * (1.0 + 0x1p-40);
    const double ca = __builtin_sqrt((double)cmax) * (1.0 + 0x1p-40);
    const double base = 2.0 * (3.0 * 0x1p-16 + 6.0 * dp * u) * (1.0 + 0x1p-6) * qa * ca +
                        24.0 * u * ((double)qn + (double)cmax);
    const double dl = base + (d + 3.0) * u * ((double)mkey + base) + 0x1p-100;
    const double v = dl * (1.0 + 0x1p-20);
    float f = (float)v;
    if ((double)f < v) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}

template <int NR, bool VEC4>
__global__ __launch_bounds__(256) void k_rerank_buf(
    const float *__restrict__ Q, int64_t nq, const float *__restrict__ C, int d, int64_t c_off,
    const float *__restrict__ qnrm, const unsigned *__restrict__ cmax_bits, int S, int cap,
    const uint2 *__restrict__ buf, const int *__restrict__ bcnt, const float *__restrict__ btau,
    int k, int64_t nvalid_max, int dp, const int *__restrict__ perm, int64_t q_off, int excl,
    int32_t *__restrict__ out_idx, float *__restrict__ out_dist, int *__restrict__ fb_count,
    int *__restrict__ fb_list) {
    __shared__ int cand[4][64 * NR];
    __shared__ float candk[4][64 * NR];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t q = (int64_t)blockIdx.x * 4 + wid;
    if (q >= nq) return;
    int M = 0;
    float T = __builtin_inff();
    bool forced = false;
    for (int s = 0; s < S; ++s) {
        const int cnt = bcnt[q * S + s];
        const float ts = btau[q * S + s];
        forced |= (ts == -__builtin_inff());
        T = fminf(T, ts);
        const uint2 *bp = buf + (q * S + s) * (int64_t)cap;
        for (int e0 = 0; e0 < cnt; e0 += 64) {
            const int e = e0 + lane;
            const uint2 v = e < cnt ? bp[e] : make_uint2(0x7f800000u, 0u);
            // ids are positions in the permuted corpus copy: map them back,
            // and drop the query's own row (the kernel ran without exclusion)
            int64_t gid = (int64_t)v.y;
            if (perm && e < cnt) gid = c_off + perm[gid - c_off];
            const bool pass = e < cnt && __uint_as_float(v.x) <= ts && !(excl && gid == q_off + q);
            const uint64_t pm = __ballot(pass);
            const int pos = M + (int)__popcll(pm & ((1ull << lane) - 1ull));
            if (pass && pos < 64 * NR) {
                cand[wid][pos] = (int)gid;
                candk[wid][pos] = __uint_as_float(v.x);
            }
            M += (int)__popcll(pm);
        }
    }
    forced |= M > 64 * NR;
    M = min(M, 64 * NR);
    __builtin_amdgcn_wave_barrier();
    float kk[NR];
    int ix[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        kk[r] = e < M ? candk[wid][e] : __builtin_inff();
        ix[r] = e < M ? cand[wid][e] : INT_MAX;
    }
    wave_bitonic_sort<NR>(kk, ix);
    float mkey = T < __builtin_inff() ? __builtin_fabsf(T) : 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r)
        if (lane + 64 * r < M && __builtin_isfinite(kk[r])) mkey = fmaxf(mkey, __builtin_fabsf(kk[r]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mkey = fmaxf(mkey, __shfl_xor(mkey, o));
    const float delta = delta_x3(qnrm[q], __uint_as_float(*cmax_bits), dp, d, mkey);
    const float *qrow = Q + q * (int64_t)d;
    const int kq = min(k, M);
    float dd[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        dd[r] = __builtin_inff();
        if (e < kq) dd[r] = exact_l2sq<VEC4>(qrow, C + ((int64_t)ix[r] - c_off) * d, d);
    }
    float Dp = -__builtin_inff();
#pragma unroll
    for (int r = 0; r < NR; ++r) Dp = fmaxf(Dp, (lane + 64 * r) < kq ? dd[r] : -__builtin_inff());
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) Dp = fmaxf(Dp, __shfl_xor(Dp, o));
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        // NaN-safe: evaluated unless the lower bound provably exceeds Dp
        if (e >= kq && e < M && !(kk[r] - delta > Dp))
            dd[r] = exact_l2sq<VEC4>(qrow, C + ((int64_t)ix[r] - c_off) * d, d);
    }
    // skipped candidates keep +inf: strictly beyond D_k, so neither the order
    // of the top k nor the certification below can see them
#pragma unroll
    for (int r = 0; r < NR; ++r)
        if (lane + 64 * r >= M) ix[r] = INT_MAX;
    wave_bitonic_sort<NR>(dd, ix);
    const int keff = (int)min((int64_t)min(k, M), nvalid_max);
    bool cert = !forced;
    if (cert && T < __builtin_inff() && keff > 0) {
        const float Dk = wave_elem<NR>(dd, keff - 1);
        cert = (T - delta) > Dk;  // NaN/inf-safe: false => exact rescan
    }
    if (!cert) {
        if (lane == 0) fb_list[atomicAdd(fb_count, 1)] = (int)q;
        return;
    }
    wave_store_list<NR>(dd, ix, k, keff, out_idx + q * k, out_dist + q * k);
}


// ---------------------------------------------------------------------------
// 2c. two-phase single-bf16 candidates (MN_KNN_BF16X1, the default at scale)
//
//   k_prep_x1    one wave per row: hi = bf16(x) (RNE, subnormals flushed) in
//                two layouts (row-major for the phase-1 Gram, KB32 for the
//                sweep), |x|^2 (f64 sum rounded to f32), and exact-residual
//                bounds |hi| and |x - hi| (f64, rounded UP to f32).
//   phase 1      gram_bf16.hpp GM_L2H on the first m0 corpus rows (a sample)
//                with list length L1: tau0(q) = min over slices of the L1-th
//                best key.
//   k_tau_x1     tau0, tq = (tau0 - |q|^2)/2 and the certification bound
//                delta(q) (below).
//   phase 2      gram_sweep2.hpp over rows m0..nc-1: every pair with
//                key < tau0(q) is buffered.
//   k_rerank_x1  exact re-rank + certification over both buffers.
//
// Certification: every pair never buffered (or dropped) has approximate key
// >= T = tau0(q), and |key - d_ref| <= delta(q), so T - delta > D_k proves the
// top k exact.  With q = qh + rq, c = ch + rc (exact residuals):
//   |q.c - qh.ch| <= |qh||rc| + |rq||ch| + |rq||rc|        (Cauchy-Schwarz)
// bounded over the corpus by max|ch|, max|rc|; plus the f32 accumulation of
// dp products and the accumulator's start value (gamma (M + |qh| max|ch|),
// gamma = (4 dp + 64) u), the roundings of the norms, tq, acc0 and the stored
// key (4 u M), M = |T| + |q|^2 + max|c|^2; and the reference fold's own error
// (d + 3) u (|T| + 2E).
// ---------------------------------------------------------------------------

// element offset of (row, k-block kb) in a KB32 copy of n rows: k-block-major
// [nkb][n][32], or tile-major (tm = the panel stride in k-blocks, >= nkb;
// gram_sweep2.hpp TM) [n/256][tm][256][32]
__device__ __forceinline__ int64_t kb32_at(int64_t row, int kb, int64_t n, int tm) {
    return tm ? ((((row >> 8) * tm + kb) << 13) + ((row & 255) << 5))
              : (((int64_t)kb * n + row) << 5);
}

// bounds must never round down: v >= 0
__device__ __forceinline__ float f32_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}

// One wave per PAIR of rows (lanes 0-31: row r, 32-63: row r+1), so the
// KB32 stores of the two rows fill whole 128-B lines.
// Output position `row` holds source row perm[row] (perm == NULL: row): the
// corpus copies are written in the visiting order, the query copies in place.
template <bool VEC4>
__global__ __launch_bounds__(256) void k_prep_x1(const float *__restrict__ X, int64_t n, int d,
                                                 int dp, const int *__restrict__ perm,
                                                 uint16_t *__restrict__ XR,
                                                 uint16_t *__restrict__ XK, float *__restrict__ nrm,
                                                 float *__restrict__ hcv, float *__restrict__ hn,
                                                 float *__restrict__ rn,
                                                 unsigned *__restrict__ maxbits,
                                                 int *__restrict__ flags, int corpus, int tm,
                                                 unsigned *__restrict__ amax) {
    const int lane = threadIdx.x & 63, hl = lane >> 5, ll = lane & 31;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    float am = 0.f;  // max |x| (amax != NULL: the fp16 sweep's scale)
    unsigned mx0 = 0u, mx1 = 0u, mx2 = 0u;  // corpus maxima (one atomic per wave)
    for (int64_t r2 = 2 * wave0; r2 < n; r2 += 2 * nwaves) {
        const int64_t row = r2 + hl;
        const bool live = row < n;
        const int64_t srow = perm ? (int64_t)perm[min(row, n - 1)] : min(row, n - 1);
        const float *p = X + srow * (int64_t)d;
        double s = 0.0, sh = 0.0, sr = 0.0;
        bool bad = false;
        for (int t0 = 8 * ll; t0 < dp; t0 += 256) {
            uint32_t wv[4];
            float xv[8];
            if (VEC4 && t0 + 8 <= d) {
                const float4 a = *reinterpret_cast<const float4 *>(p + t0);
                const float4 b = *reinterpret_cast<const float4 *>(p + t0 + 4);
                xv[0] = a.x; xv[1] = a.y; xv[2] = a.z; xv[3] = a.w;
                xv[4] = b.x; xv[5] = b.y; xv[6] = b.z; xv[7] = b.w;
            } else {
#pragma unroll
                for (int u = 0; u < 8; ++u) xv[u] = t0 + u < d ? p[t0 + u] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                uint32_t hb2[2];
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const float x = xv[u + v];
                    bad |= !__builtin_isfinite(x);
                    if (live) am = fmaxf(am, __builtin_fabsf(x));
                    const uint32_t hb = __builtin_fabsf(x) >= 0x1p-126f ? bf16_rne(x) : 0u;
                    const float hf = __uint_as_float(hb << 16);
                    const float r = x - hf;  // exact
                    s += (double)x * (double)x;
                    sh += (double)hf * (double)hf;
                    sr += (double)r * (double)r;
                    hb2[v] = hb;
                }
                wv[u >> 1] = hb2[0] | (hb2[1] << 16);
            }
            if (live) {
                const uint4 pk = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                if (XR) *reinterpret_cast<uint4 *>(XR + row * (int64_t)dp + t0) = pk;
                if (XK)
                    *reinterpret_cast<uint4 *>(XK + kb32_at(row, t0 >> 5, n, tm) + (t0 & 31)) =
                        pk;
            }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {
            s += __shfl_xor(s, o);
            sh += __shfl_xor(sh, o);
            sr += __shfl_xor(sr, o);
        }
        bad = bad && live;
        const bool anybad = __any(bad);
        if (ll == 0 && live) {
            const float nf = (float)s;
            if (nrm) nrm[row] = nf;
            if (hcv) hcv[row] = 0.5f * nf;
            const float hf = f32_up(__builtin_sqrt(sh) * (1.0 + 0x1p-50));
            const float rf = f32_up(__builtin_sqrt(sr) * (1.0 + 0x1p-50));
            if (hn) hn[row] = hf;
            if (rn) rn[row] = rf;
            if (anybad) atomicOr(flags, 1);
            // keys stay far from f32 overflow (and bf16(x) finite) below 2^100
            if (!(s <= 0x1p100)) atomicOr(flags + 1, 1);
            if (corpus) {
                mx0 = max(mx0, __float_as_uint(nf));
                mx1 = max(mx1, __float_as_uint(hf));
                mx2 = max(mx2, __float_as_uint(rf));
            }
        }
    }
    if (corpus) {
        wave_atomic_umax(maxbits + 0, mx0);
        wave_atomic_umax(maxbits + 1, mx1);
        wave_atomic_umax(maxbits + 2, mx2);
    }
    if (amax) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
        if (lane == 0 && am > 0.f) atomicMax(amax, __float_as_uint(am));
    }
}

// fp16 copy for the symmetric sweep (gram_sweep2.hpp F16) with a PER-ROW
// exponent: h = fp16(x 2^e) with e = 14 - E, max|x| < 2^E (the row's largest
// value lands in [2^13, 2^14); |e| <= 100), round to nearest even, |x 2^e| <
// 2^-14 flushed to 0 (the MFMA never sees a subnormal), stored tile-major KB32
// like k_prep_x1 (XK may be NULL: the statistics pass).  Per position, in
// UNSCALED units: |h 2^-e| and |x - h 2^-e| (the residual is exact), rounded
// up, and the scale s = 2^e (hn may be NULL: no statistics).  A row's own
// exponent keeps its relative precision whatever the other rows' magnitudes
// (one global exponent let a single huge row flush every small one).
// Position `row` holds source row perm[row].
template <bool VEC4>
__global__ __launch_bounds__(256) void k_prep_f16r(const float *__restrict__ X, int64_t n, int d,
                                                   int dp, const int *__restrict__ perm,
                                                   uint16_t *__restrict__ XK,
                                                   float *__restrict__ hn, float *__restrict__ rn,
                                                   float *__restrict__ sc, int tm) {
    const int lane = threadIdx.x & 63, hl = lane >> 5, ll = lane & 31;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r2 = 2 * wave0; r2 < n; r2 += 2 * nwaves) {
        const int64_t row = r2 + hl;
        const bool live = row < n;
        const int64_t srow = perm ? (int64_t)perm[min(row, n - 1)] : min(row, n - 1);
        const float *p = X + srow * (int64_t)d;
        auto load8 = [&](int t0, float (&xv)[8]) {
            if (VEC4 && t0 + 8 <= d) {
                const float4 a = *reinterpret_cast<const float4 *>(p + t0);
                const float4 b = *reinterpret_cast<const float4 *>(p + t0 + 4);
                xv[0] = a.x; xv[1] = a.y; xv[2] = a.z; xv[3] = a.w;
                xv[4] = b.x; xv[5] = b.y; xv[6] = b.z; xv[7] = b.w;
            } else {
#pragma unroll
                for (int u = 0; u < 8; ++u) xv[u] = t0 + u < d ? p[t0 + u] : 0.f;
            }
        };
        // the row's exponent (half-wave max over its 32 lanes)
        float am = 0.f;
        for (int t0 = 8 * ll; t0 < dp; t0 += 256) {
            float xv[8];
            load8(t0, xv);
#pragma unroll
            for (int u = 0; u < 8; ++u) am = fmaxf(am, __builtin_fabsf(xv[u]));
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
        int E = 0;
        if (am > 0.f) frexpf(am, &E);  // am < 2^E
        const int e = am > 0.f ? min(max(14 - E, -100), 100) : 0;
        double sh = 0.0, sr = 0.0;
        for (int t0 = 8 * ll; t0 < dp; t0 += 256) {
            uint32_t wv[4];
            float xv[8];
            load8(t0, xv);
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                uint32_t hb2[2];
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const float x = xv[u + v];
                    const float xs = __builtin_ldexpf(x, e);  // exact: |x 2^e| < 2^14
                    _Float16 h = __builtin_fabsf(xs) >= 0x1p-14f ? (_Float16)xs : (_Float16)0.f;
                    uint16_t hbits;
                    __builtin_memcpy(&hbits, &h, 2);
                    const double hf = __builtin_ldexp((double)(float)h, -e);  // exact in f64
                    const double r = (double)x - hf;                          // exact in f64
                    sh += hf * hf;
                    sr += r * r;
                    hb2[v] = hbits;
                }
                wv[u >> 1] = hb2[0] | (hb2[1] << 16);
            }
            if (live && XK) {
                const uint4 pk = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                *reinterpret_cast<uint4 *>(XK + kb32_at(row, t0 >> 5, n, tm) + (t0 & 31)) = pk;
            }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {
            sh += __shfl_xor(sh, o);
            sr += __shfl_xor(sr, o);
        }
        if (ll == 0 && live && hn) {
            // f64 sums of squares: relative error <= (dp + 1) 2^-53, covered by
            // the 2^-40 margin (dp <= 2^12)
            hn[row] = f32_up(__builtin_sqrt(sh * (1.0 + 0x1p-40)) * (1.0 + 0x1p-50));
            rn[row] = f32_up(__builtin_sqrt(sr * (1.0 + 0x1p-40)) * (1.0 + 0x1p-50));
            sc[row] = __builtin_ldexpf(1.f, e);
        }
    }
}

// ---------------------------------------------------------------------------
// 2d. refill of the rows the bf16x1 bound could not certify (dense clusters:
// the bound scales with |q||c|, not with the neighbour distances)
//
// The bf16x3 product q.c ~ qh.ch + qh.cl + ql.ch is ONE dot product of length
// 3 dp: [qh | qh | ql] . [ch | cl | ch].  So the same sweep kernel, given KB32
// copies of those concatenated rows, evaluates the split Gram with a
// per-query fixed threshold and NO list-length limit.  Each uncertified row
// already holds an upper bound ub >= D_k (the k-th exact distance among its
// re-ranked candidates); the refill buffers every pair with key < T = ub +
// 1.125 delta3(ub), so every pair with d <= ub is buffered and the re-rank
// certifies T - delta3(T) > D_k by construction (buffer overflow aside).
//
// delta3: with x = h + l + r2 (hi = bf16(x), lo = bf16(x - hi), r2 exact),
//   omitted products  <= |ql| max|cl| + (|qh|+|ql|+|q2|) max|c2| + |q2|(max|ch|+max|cl|)
//   f32 accumulation of the 3 dp exact products on top of acc0:
//                        (6 dp + 64) u (M + (|qh|+|ql|)(max|ch|+max|cl|))
//                        (2x the round-to-nearest bound, acc0 <= M / 2)
//   norms, tq, acc0, stored key: 4 u M, M = |T| + |q|^2 + max|c|^2
//   and the reference fold's own error (d + 3) u (|T| + 2E), as in k_tau_x1.
// ---------------------------------------------------------------------------

// KB32 rows of width 3 dp (nkb3 = 3 dp / 32 blocks): queries [hi | hi | lo],
// corpus [hi | lo | hi].  Output position `row` holds source row rows[row]
// (queries gathered by the fallback list) or perm[row] (corpus, visiting
// order).  One wave per pair of rows, like k_prep_x1.
template <bool VEC4>
__global__ __launch_bounds__(256) void k_prep_x3(const float *__restrict__ X, int64_t n, int d,
                                                 int dp, const int *__restrict__ src,
                                                 uint16_t *__restrict__ XK, int corpus,
                                                 float *__restrict__ nrm, float *__restrict__ hn,
                                                 float *__restrict__ ln, float *__restrict__ r2n,
                                                 unsigned *__restrict__ cmax3, int tm) {
    const int lane = threadIdx.x & 63, hl = lane >> 5, ll = lane & 31;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int nkb = dp >> 5;
    unsigned mx[4] = {0u, 0u, 0u, 0u};  // corpus maxima (one atomic per wave)
    for (int64_t r2 = 2 * wave0; r2 < n; r2 += 2 * nwaves) {
        const int64_t row = r2 + hl;
        const bool live = row < n;
        const int64_t srow = src ? (int64_t)src[min(row, n - 1)] : min(row, n - 1);
        const float *p = X + srow * (int64_t)d;
        double s = 0.0, sh = 0.0, sl = 0.0, s2 = 0.0;
        for (int t0 = 8 * ll; t0 < dp; t0 += 256) {
            float xv[8];
            if (VEC4 && t0 + 8 <= d) {
                const float4 a = *reinterpret_cast<const float4 *>(p + t0);
                const float4 b = *reinterpret_cast<const float4 *>(p + t0 + 4);
                xv[0] = a.x; xv[1] = a.y; xv[2] = a.z; xv[3] = a.w;
                xv[4] = b.x; xv[5] = b.y; xv[6] = b.z; xv[7] = b.w;
            } else {
#pragma unroll
                for (int u = 0; u < 8; ++u) xv[u] = t0 + u < d ? p[t0 + u] : 0.f;
            }
            uint32_t hw[4], lw[4];
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                uint32_t hb2[2], lb2[2];
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const float x = xv[u + v];
                    uint32_t hb = 0, lb = 0;
                    if (__builtin_fabsf(x) >= 0x1p-126f) hb = bf16_rne(x);
                    const float hf = __uint_as_float(hb << 16);
                    const float r = x - hf;  // exact
                    if (__builtin_fabsf(r) >= 0x1p-126f) lb = bf16_rne(r);
                    const float lf = __uint_as_float(lb << 16);
                    const float rr = r - lf;  // exact
                    s += (double)x * (double)x;
                    sh += (double)hf * (double)hf;
                    sl += (double)lf * (double)lf;
                    s2 += (double)rr * (double)rr;
                    hb2[v] = hb;
                    lb2[v] = lb;
                }
                hw[u >> 1] = hb2[0] | (hb2[1] << 16);
                lw[u >> 1] = lb2[0] | (lb2[1] << 16);
            }
            if (live) {
                const uint4 H = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                const uint4 Lo = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                const int kb = t0 >> 5, ko = t0 & 31;
                *reinterpret_cast<uint4 *>(XK + kb32_at(row, kb, n, tm) + ko) = H;
                *reinterpret_cast<uint4 *>(XK + kb32_at(row, kb + nkb, n, tm) + ko) =
                    corpus ? Lo : H;
                *reinterpret_cast<uint4 *>(XK + kb32_at(row, kb + 2 * nkb, n, tm) + ko) =
                    corpus ? H : Lo;
            }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {
            s += __shfl_xor(s, o);
            sh += __shfl_xor(sh, o);
            sl += __shfl_xor(sl, o);
            s2 += __shfl_xor(s2, o);
        }
        if (ll == 0 && live) {
            const float nf = (float)s;
            const float hf = f32_up(__builtin_sqrt(sh) * (1.0 + 0x1p-50));
            const float lf = f32_up(__builtin_sqrt(sl) * (1.0 + 0x1p-50));
            const float rf = f32_up(__builtin_sqrt(s2) * (1.0 + 0x1p-50));
            if (nrm) nrm[row] = nf;
            if (hn) hn[row] = hf;
            if (ln) ln[row] = lf;
            if (r2n) r2n[row] = rf;
            if (corpus) {
                mx[0] = max(mx[0], __float_as_uint(nf));
                mx[1] = max(mx[1], __float_as_uint(hf));
                mx[2] = max(mx[2], __float_as_uint(lf));
                mx[3] = max(mx[3], __float_as_uint(rf));
            }
        }
    }
    if (corpus)
        for (int c = 0; c < 4; ++c) wave_atomic_umax(cmax3 + c, mx[c]);
}

__device__ __forceinline__ double delta3_at(double Tf, double qn, double qh, double ql, double q2,
                                            double Mn, double Mh, double Ml, double M2, int d,
                                            int dp) {
    const double u = 0x1p-24;
    const double M = Tf + qn + Mn;
    const double Eprod = ql * Ml + (qh + ql + q2) * M2 + q2 * (Mh + Ml);
    const double gam = (6.0 * dp + 64.0) * u;
    const double E = Eprod + gam * (M + (qh + ql) * (Mh + Ml)) + 4.0 * u * M;
    return (2.0 * E + (d + 3.0) * u * (Tf + 2.0 * E) + 0x1p-100) * (1.0 + 0x1p-20);
}

// Per refilled row i (query rows[i]): T = ub + 1.125 delta3(|ub|), tq, and
// the certification bound delta3(|T|).  ub = +inf (no k candidates) forces
// the exact scan (T = -inf).
__global__ __launch_bounds__(256) void k_tau_x3(int64_t n, const int *__restrict__ rows,
                                                const float *__restrict__ ub,
                                                const float *__restrict__ qn3,
                                                const float *__restrict__ qh3,
                                                const float *__restrict__ ql3,
                                                const float *__restrict__ q23,
                                                const unsigned *__restrict__ cmax3, int d, int dp,
                                                float *__restrict__ tq, float *__restrict__ tau,
                                                float *__restrict__ delta) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float b = ub[rows[i]];
    if (!(b < __builtin_inff())) {
        tq[i] = -__builtin_inff();
        tau[i] = -__builtin_inff();
        delta[i] = 0.f;
        return;
    }
    const double Mn = __uint_as_float(cmax3[0]), Mh = __uint_as_float(cmax3[1]),
                 Ml = __uint_as_float(cmax3[2]), M2 = __uint_as_float(cmax3[3]);
    const float qnf = qn3[i];
    const double qn = qnf, qh = qh3[i], ql = ql3[i], q2 = q23[i];
    const double d0 = delta3_at(__builtin_fabs((double)b), qn, qh, ql, q2, Mn, Mh, Ml, M2, d, dp);
    const float T = f32_up((double)b + 1.125 * d0);
    tau[i] = T;
    tq[i] = (T - qnf) * 0.5f;
    delta[i] = f32_up(delta3_at(__builtin_fabs((double)T), qn, qh, ql, q2, Mn, Mh, Ml, M2, d, dp));
}

// delta of the bf16x1 bound: Tf = |threshold| magnitude in the
// accumulator terms, qn / qh / qr the row's |q|^2, |bf16(q)|, |q - bf16(q)|,
// Mn the corpus max |c|^2, Mh / Mr the corpus maxima of |ch| / |c - ch|.
// The error of the approximate key d~ = |q|^2 + |c|^2 - 2 (acc0 + qh.ch)
// against the exact distance: the omitted products |q.c - qh.ch| <= |qh||rc|
// + |rq||ch| + |rq||rc| (Cauchy-Schwarz), the f32 accumulation of acc0 and
// the dp exact products, the roundings of the norms / folds / stored key
// (4 u M), and the reference fold's own error (d + 3) u (|T| + 2 E).
//   tight = 0: accumulation gamma (4 dp + 64) u (M + qh Mh) (the original,
//              generous constant);
//   tight = 1: 2 (dp + 33) u (M / 2 + qh Mh): <= 2 u per addition in ANY
//              order (Higham's gamma_n sum |terms| with a factor 2 for a
//              non-nearest internal rounding), |acc0| <= M / 2, sum |products|
//              <= |qh||ch|; the probe scripts/probes/probe_mfma_accum.hip
//              measures the MFMA chains well inside it (profiles/).
__device__ __forceinline__ float delta_x1(double Tf, float qn, double qh, double qr, double Mn,
                                          double Mh, double Mr, int d, int dp, int tight = 0) {
    const double u = 0x1p-24;
    const double M = Tf + (double)qn + Mn;
    const double Eprod = qh * Mr + qr * Mh + qr * Mr;
    const double acc = tight ? 2.0 * (dp + 33.0) * u * (0.5 * M + qh * Mh)
                             : (4.0 * dp + 64.0) * u * (M + qh * Mh);
    const double E = Eprod + acc + 4.0 * u * M;
    const double dl = 2.0 * E + (d + 3.0) * u * (Tf + 2.0 * E) + 0x1p-100;
    return f32_up(dl * (1.0 + 0x1p-20));
}
__device__ __forceinline__ float delta_x1(double Tf, float qn, double qh, double qr,
                                          const unsigned *__restrict__ cmax, int d, int dp) {
    return delta_x1(Tf, qn, qh, qr, __uint_as_float(cmax[0]), __uint_as_float(cmax[1]),
                    __uint_as_float(cmax[2]), d, dp, 0);
}

// Per query: T = min over phase-1 slices of tau (-inf: forced), tq, delta;
// tmax (may be NULL) collects max |T| over the finite T (uint bits).
__global__ __launch_bounds__(256) void k_tau_x1(int64_t nq, int S1, const float *__restrict__ btau1,
                                                const float *__restrict__ nq_f,
                                                const float *__restrict__ hn_q,
                                                const float *__restrict__ rn_q,
                                                const unsigned *__restrict__ cmax, int d, int dp,
                                                float *__restrict__ tq, float *__restrict__ tau0,
                                                float *__restrict__ delta,
                                                unsigned *__restrict__ tmax) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned tb = 0u;
    if (q < nq) {
        float T = __builtin_inff();
        for (int s = 0; s < S1; ++s) T = fminf(T, btau1[q * S1 + s]);
        const float qn = nq_f[q];
        const double Tf = __builtin_isfinite(T) ? __builtin_fabs((double)T) : 0.0;
        const float dl = delta_x1(Tf, qn, hn_q[q], rn_q[q], cmax, d, dp);
        tau0[q] = T;
        tq[q] = (T - qn) * 0.5f;
        delta[q] = dl;
        if (__builtin_isfinite(T)) tb = __float_as_uint(__builtin_fabsf(T));
    }
    if (tmax) wave_atomic_umax(tmax, tb);  // every lane of the wave takes part
}

// f64 -> f32 rounded toward +inf (any sign)
__device__ __forceinline__ float f32_ceil(double v) {
    float f = (float)v;
    if ((double)f < v) {  // one ulp toward +inf (f is finite here)
        const uint32_t b = __float_as_uint(f);
        f = (b & 0x80000000u) ? (b == 0x80000000u ? __uint_as_float(1u) : __uint_as_float(b - 1u))
                              : __uint_as_float(b + 1u);
    }
    return f;
}

// f64 -> f32 rounded toward -inf (any sign)
__device__ __forceinline__ float f32_floor(double v) { return -f32_ceil(-v); }

// SW_SYM folds with a PER-PAIR, separable certification bound (round 4; the
// round-3 bound used corpus maxima of |h| and |x - h|, so one huge row left
// every row uncertified).
//
// For a pair (q, c): keỹ = qn_q + qn_c - 2 P, P = h̄_q . h̄_c (h̄ = h 2^-e, r =
// x - h̄ exact), and the sweep's f32 accumulator acc = s_q s_c (a + b + P) +
// rounding, s = 2^e (per row).  Every term of |d_exact - keỹ| and of the
// accumulator's rounding splits into a per-row part (AM-GM on the cross
// terms, lambda = 2^-12 ~ the fp16 relative precision):
//   |q|^2 - qn_q          <= u qn (1 + 2u)                    (f64 sum -> f32)
//   2|q.c - P|            <= 2(|h̄_q||r_c| + |r_q||h̄_c| + |r_q||r_c|)
//                          <= sum over x in {q, c} of lambda |h̄_x|^2 + |r_x|^2 (1/lambda + 1)
//   2 |acc error| / s_q s_c <= 2 gamma (|a| + |b| + |h̄_q||h̄_c|), gamma = 2 (dp + 33) u + u
//                          (any-order accumulation of acc0 and dp exact products,
//                          <= 2u per addition, + acc0's rounding), |a| + |b| <=
//                          sum over x of (|T_x| + qn_x + 3 alpha_x) / 2
// so alpha_x = [u' qn + lambda hn^2 + rn^2 (1/lambda + 1) + gamma (|T| + qn + hn^2)]
//              / (1 - 3 gamma)   bounds x's share: |d_exact - keỹ| + 2|acc err| <=
// Delta(q, c) = alpha_q + alpha_c.
// Certificate threshold Tc = T - 2 alpha (so the candidates are about those
// with keỹ < T, as with one shared bound: keỹ - alpha_q - alpha_c < Tc_q ~
// keỹ < T + alpha_c - alpha_q), fold threshold Tf = Tc + |Tc| (d + 6) u (the
// reference fold's own (d + 3) u, the key's roundings); the row test is
//   acc0 = U_q s_c + V_c s_q,  U = (Tf + alpha - qn) / 2 s,  V = -(qn - alpha) / 2 s
// (the off-diagonal column test swaps the roles: V_q s_c + U_c s_q; rows are
// sorted by Tf, so Tf(c) >= Tf(q) there).  acc <= 0 => keỹ - Delta >= Tf =>
// d_exact >= Tf => d_ref >= Tc.  So every pair never buffered has d_ref >= Tc
// and the certificate is Tc > D_k; a buffered pair's key kl = Tf - 2 acc /
// (s_q s_c) is a lower bound of d_exact up to f32 roundings (the re-rank's
// relative slack).  U, V, Tf are rounded up (more candidates = safe), Tc down.
// An outlier column's alpha_c only widens its own pairs (their keys ~ |c|^2
// >> alpha_c are still rejected); an outlier row fails its own certificate.

// per row r: alpha, the fold threshold tf (also the sort key) and the
// certificate tc; hn / rn from the statistics pass of k_prep_f16r
__global__ __launch_bounds__(256) void k_sym_row(int64_t n, const float *__restrict__ tau0,
                                                 const float *__restrict__ nq_f,
                                                 const float *__restrict__ hn,
                                                 const float *__restrict__ rn, int d, int dp,
                                                 float *__restrict__ alpha_o,
                                                 float *__restrict__ tf_o,
                                                 float *__restrict__ tc_o) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const double u = 0x1p-24, lam = 0x1p-12;
    const double T = tau0[r], qn = nq_f[r], h = hn[r], rr = rn[r];
    const double gam = 2.0 * (dp + 33.0) * u + u;
    const double Ta = __builtin_isfinite(T) ? __builtin_fabs(T) : 0.0;
    const double base = 1.0000001 * u * qn + lam * h * h + rr * rr * (1.0 / lam + 1.0) +
                        gam * (Ta + qn + h * h);
    const float alpha = f32_up(base / (1.0 - 3.0 * gam) * (1.0 + 0x1p-20));
    const double Tc = T - 2.0 * (double)alpha;  // +inf stays +inf
    const double Tca = __builtin_isfinite(Tc) ? __builtin_fabs(Tc) : 0.0;
    alpha_o[r] = alpha;
    tc_o[r] = __builtin_isfinite(Tc) ? f32_floor(Tc) : (float)Tc;
    tf_o[r] = __builtin_isfinite(Tc) ? f32_ceil(Tc + Tca * (d + 6.0) * u) : (float)Tc;
}

// per position p (row pi[p], sorted by tf): the kernel's folds and keys, the
// re-rank's certificate, hcP = qn / 2 (unscaled: the bf16x3 refill's corpus
// term), the scale by position
__global__ __launch_bounds__(256) void k_sym_pos(int64_t n, const int *__restrict__ pi,
                                                 const float *__restrict__ nq_f,
                                                 const float *__restrict__ alpha,
                                                 const float *__restrict__ tf,
                                                 const float *__restrict__ tc,
                                                 const float *__restrict__ sc_row,
                                                 float *__restrict__ tauP,
                                                 float *__restrict__ teffP,
                                                 float *__restrict__ Uo, float *__restrict__ Vo,
                                                 float *__restrict__ hcP,
                                                 float *__restrict__ scP) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int r = pi[p];
    const double qn = nq_f[r], a = alpha[r], s = sc_row[r];
    const float Tf = tf[r];
    tauP[p] = tc[r];
    teffP[p] = Tf;
    Uo[p] = f32_ceil(((double)Tf + a - qn) * 0.5 * s);
    Vo[p] = f32_ceil(-(qn - a) * 0.5 * s);
    hcP[p] = 0.5f * (float)qn;
    scP[p] = (float)s;
}

__global__ __launch_bounds__(256) void k_fill_empty(int32_t *__restrict__ idx, float *__restrict__ dist,
                                                    int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        idx[i] = -1;
        dist[i] = __builtin_inff();
    }
}

__global__ __launch_bounds__(256) void k_iota(int *__restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (int)i;
}

// One wave per query: gather both phases' buffered candidates with key < T
// (all of them when T = +inf: nothing was rejected), order by key, evaluate
// the reference fold for the best kq and then for every other candidate whose
// lower bound key - delta does not exceed the worst of those, sort by (dist,
// idx), certify T - delta > D_k.  Overflowing buffers force the exact scan.
// Rows with more than 64 NR candidates go to big_list (a second launch with a
// wider NR re-ranks them; without a big_list they are rescanned exactly).
template <int NR, int WPB, bool VEC4>
__global__ __launch_bounds__(64 * WPB) void k_rerank_x1(
    const float *__restrict__ Q, int64_t nq, const float *__restrict__ C, int d, int64_t c_off,
    int S1, int cap1, const uint2 *__restrict__ buf1, const int *__restrict__ cnt1,
    const float *__restrict__ tau0, int S2, int cap2, const uint2 *__restrict__ buf2,
    const int *__restrict__ cnt2, const float *__restrict__ delta, int k, int64_t nvalid_max,
    const int *__restrict__ qlist, const int *__restrict__ qlist_n, int *__restrict__ big_count,
    int *__restrict__ big_list, const int *__restrict__ perm, int64_t q_off, int excl,
    const int *__restrict__ qmap, float *__restrict__ ub, int32_t *__restrict__ out_idx,
    float *__restrict__ out_dist, int *__restrict__ fb_count, int *__restrict__ fb_list,
    float rel, int *__restrict__ why, int m1) {
    __shared__ int cand[WPB][64 * NR];
    __shared__ float candk[WPB][64 * NR];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t wq = (int64_t)blockIdx.x * WPB + wid;
    if (qlist ? wq >= *qlist_n : wq >= nq) return;
    const int64_t q = qlist ? qlist[wq] : wq;
    // qo: the row of Q / the output (refill: the buffers are per refilled row)
    const int64_t qo = qmap ? (int64_t)qmap[q] : q;
#ifdef MN_TUNING
    if (qo < 0 || qo > nvalid_max + 1) {  // (diagnostics)
        if (lane == 0) printf("k_rerank_x1: row %lld maps to %lld\n", (long long)q, (long long)qo);
        return;
    }
#endif
    const float T = tau0[q];
    bool forced = T == -__builtin_inff();
    // rel > 0 (SW_SYM): buffered keys are per-pair LOWER bounds (k_sym_pos),
    // buffered below Teff <= T + rel |T|; a candidate's exact distance is >=
    // key - rel (|key| + |T|), and the certificate is T > D_k (delta = 0)
    const float Tg = (rel > 0.f && __builtin_isfinite(T)) ? T + rel * __builtin_fabsf(T) : T;
    int ovf = 0;  // diagnostics (why != NULL): a buffer overflowed
    int M = 0;
    // ids are positions in the visiting order: map them back (c_off +
    // perm[p]); the generators ran without exclusion, so the query's own row
    // is dropped here
    auto gather = [&](const uint2 *bp, int cnt, bool) {
        for (int e0 = 0; e0 < cnt; e0 += 64) {
            const int e = e0 + lane;
            uint2 v = e < cnt ? bp[e] : make_uint2(0x7f800000u, 0u);
#ifdef MN_TUNING
            // (diagnostics: an id past the corpus is reported and dropped)
            if (e < cnt && (int64_t)v.y > nvalid_max + 1) {
                printf("k_rerank_x1: row %lld (out %lld) entry %d of %d: id %u > %lld, key %g\n",
                       (long long)q, (long long)qo, e, cnt, v.y, (long long)nvalid_max + 1,
                       (double)__uint_as_float(v.x));
                v = make_uint2(0x7f800000u, 0u);
            }
#endif
            int64_t gid = (int64_t)v.y;
            if (e < cnt) gid = c_off + perm[gid];
            const bool pass = e < cnt && __uint_as_float(v.x) < Tg && !(excl && gid == q_off + qo);
            const uint64_t pm = __ballot(pass);
            const int pos = M + (int)__popcll(pm & ((1ull << lane) - 1ull));
            if (pass && pos < 64 * NR) {
                cand[wid][pos] = (int)gid;
                candk[wid][pos] = __uint_as_float(v.x);
            }
            M += (int)__popcll(pm);
        }
    };
    for (int s = 0; s < S1; ++s)
        gather(buf1 + (q * S1 + s) * (int64_t)cap1, cnt1[q * S1 + s], true);
    for (int j = 0; j < S2; ++j) {
        int c = cnt2[q * S2 + j];
        forced |= c < 0 || c > cap2;  // -1: overflow; SW_SYM: a count past cap
        ovf |= (c < 0 || c > cap2) ? 1 : 0;
        c = min(c, cap2);
        if (c > 0) gather(buf2 + (q * S2 + j) * (int64_t)cap2, c, false);
    }
    if (!forced && M > 64 * NR && big_list) {
        if (lane == 0) big_list[atomicAdd(big_count, 1)] = (int)q;
        return;
    }
    forced |= M > 64 * NR;
    M = min(M, 64 * NR);
    __builtin_amdgcn_wave_barrier();
    float kk[NR];
    int ix[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        kk[r] = e < M ? candk[wid][e] : __builtin_inff();
        ix[r] = e < M ? cand[wid][e] : INT_MAX;
    }
    wave_bitonic_sort<NR>(kk, ix);
    const float dlt = delta[q];
    const float *qrow = Q + qo * (int64_t)d;
    const int kq = min(k, M);
    // first pass: the kq1 best keys (round 6: k + m1 of them, k + m1 <= 64 —
    // the lanes the k-best pass left idle — so Dp, the k-th exact distance
    // among them, is tighter and the second pass rarely runs; m1 = 0: k)
    const int kq1 = (m1 > 0 && k + m1 <= 64) ? min(M, k + m1) : kq;
    float dd[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        dd[r] = __builtin_inff();
        if (e < kq1) dd[r] = exact_l2sq<VEC4>(qrow, C + ((int64_t)ix[r] - c_off) * d, d);
    }
    float Dp = -__builtin_inff();
    if (kq1 == kq) {
#pragma unroll
        for (int r = 0; r < NR; ++r) Dp = fmaxf(Dp, (lane + 64 * r) < kq ? dd[r] : -__builtin_inff());
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) Dp = fmaxf(Dp, __shfl_xor(Dp, o));
    } else {  // the kq-th smallest of the kq1 (<= 64: register 0) exact distances
        float t[1] = {lane < kq1 ? dd[0] : __builtin_inff()};
        int ti[1] = {lane};
        wave_bitonic_sort<1>(t, ti);
        Dp = __shfl(t[0], kq - 1);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        const float lb = kk[r] - dlt - rel * (__builtin_fabsf(kk[r]) + __builtin_fabsf(T));
        if (e >= kq1 && e < M && !(lb > Dp))
            dd[r] = exact_l2sq<VEC4>(qrow, C + ((int64_t)ix[r] - c_off) * d, d);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
        if (lane + 64 * r >= M) ix[r] = INT_MAX;
    wave_bitonic_sort<NR>(dd, ix);
    const int keff = (int)min((int64_t)min(k, M), nvalid_max);
    if (!fb_list) {
        // partial mode (one rank's share of a row-sharded symmetric sweep,
        // shard_share): the exact top-k of this share's admitted candidates,
        // certified after the owner's merge (k_merge_certify); a forced row
        // (overflow, too many candidates) is marked idx -2 in slot 0
        if (forced) {
            for (int e = lane; e < k; e += 64) {
                out_idx[qo * k + e] = e == 0 ? -2 : -1;
                out_dist[qo * k + e] = __builtin_inff();
            }
            return;
        }
        wave_store_list<NR>(dd, ix, k, keff, out_idx + qo * k, out_dist + qo * k);
        return;
    }
    bool cert = !forced;
    if (cert && T < __builtin_inff() && keff > 0) {
        const float Dk = wave_elem<NR>(dd, keff - 1);
        cert = (T - dlt) > Dk;  // NaN/inf-safe: false => exact rescan
    }
    const int kneed = (int)min((int64_t)k, nvalid_max);
    if (cert && T < __builtin_inff() && keff < kneed) cert = false;
    if (!cert) {
        if (why && lane == 0) {  // reason counters (MN_X1_DEBUG)
            const int rsn = ovf ? 0 : M > 64 * NR ? 1 : T == -__builtin_inff() ? 2
                          : !(T < __builtin_inff()) ? 3 : keff < kneed ? 4 : 5;
            atomicAdd(&why[rsn], 1);
        }
        if (ub) {
            // any k exact candidate distances bound D_k from above (the refill)
            const float b = (kneed > 0 && keff >= kneed) ? wave_elem<NR>(dd, kneed - 1)
                                                         : __builtin_inff();
            if (lane == 0) ub[qo] = b;
        }
        if (lane == 0) fb_list[atomicAdd(fb_count, 1)] = (int)qo;
        return;
    }
    wave_store_list<NR>(dd, ix, k, keff, out_idx + qo * k, out_dist + qo * k);
}

// sum of buffered entries (statistics only; timing mode)
__global__ __launch_bounds__(256) void k_count_cands(const int *__restrict__ c, int64_t n, int cap,
                                                     unsigned long long *__restrict__ out) {
    __shared__ unsigned long long part[4];
    unsigned long long a = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int v = c[i];
        a += (unsigned long long)(v < 0 ? cap : min(v, cap));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, part[0] + part[1] + part[2] + part[3]);
}

// MN_L2 (distance.rs:195-203; mst.rs:344 stable sort of the ROOTED f32
// distances): two different L2^2 values can round to the same f32 root, and
// then the reference orders them by index, not by the squared value.  The
// L2^2 list is computed k2 = k + 8 long (k2 <= KLIST: two entries a lane); one
// wave per row takes the correctly rounded roots (Rust f32::sqrt; gfx950
// sqrtf is not correctly rounded, common.hpp), re-sorts by (root, idx) —
// which only permutes runs of equal roots — and keeps k.  Entries beyond the
// list have roots >= the last one, so the result is exact unless the run of
// roots equal to the k-th one reaches the end of a full list: those rows go to
// the exact root-keyed scan.
__global__ __launch_bounds__(256) void k_l2_order(const int32_t *__restrict__ idx2,
                                                  const float *__restrict__ d2, int64_t nq, int k2,
                                                  int k, int64_t nc, int64_t q_off, int64_t c_off,
                                                  int excl, int32_t *__restrict__ out_idx,
                                                  float *__restrict__ out_dist,
                                                  int *__restrict__ fb_count,
                                                  int *__restrict__ fb_list) {
    const int lane = threadIdx.x & 63;
    const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (q >= nq) return;
    float key[2];
    int ix[2], m = 0;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        const int id = e < k2 ? idx2[q * k2 + e] : -1;
        const float sq = e < k2 ? d2[q * k2 + e] : __builtin_inff();
        key[r] = id >= 0 ? sqrt_rn_f32(sq) : __builtin_inff();
        ix[r] = id >= 0 ? id : INT_MAX;
        m += (int)__popcll(__ballot(id >= 0));
    }
    wave_bitonic_sort<2>(key, ix);
    const int64_t gq = q_off + q;
    const int64_t valid = nc - ((excl && gq >= c_off && gq < c_off + nc) ? 1 : 0);
    const float rk = wave_elem<2>(key, min(k, m) - 1 < 0 ? 0 : min(k, m) - 1);
    const float rl = wave_elem<2>(key, k2 - 1);
    // k2 > k always (k <= KMAX, k2 = k + 8): the list extends past rank k
    const bool more = m == k2 && (int64_t)k2 < valid;
    if (more && k <= m && rl == rk) {
        if (lane == 0) fb_list[atomicAdd(fb_count, 1)] = (int)q;
        return;
    }
    wave_store_list<2>(key, ix, k, m, out_idx + q * k, out_dist + q * k);
}

// Rows the bf16x1 path leaves uncertified (after its bf16x3 refill) against a
// large corpus: gather them, run the split generator on them with k + 1
// neighbours and self included, then drop the query's own id (d = +0: it is
// in the k + 1 list unless > k exact duplicates precede it, in which case the
// last entry goes).
__global__ __launch_bounds__(256) void k_gather_rows(const float *__restrict__ X, int d,
                                                     const int *__restrict__ rows, int64_t n,
                                                     float *__restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * d) return;
    const int64_t i = e / d;
    out[e] = X[(int64_t)rows[i] * d + (e - i * d)];
}

__global__ __launch_bounds__(256) void k_scatter_escalated(
    const int *__restrict__ rows, int64_t n, int64_t q_off, int excl, int k,
    const int32_t *__restrict__ eidx, const float *__restrict__ edist,
    int32_t *__restrict__ out_idx, float *__restrict__ out_dist) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t q = rows[i], gid = q_off + q;
    int wpos = 0;
    for (int r = 0; r <= k; ++r) {
        const int id = eidx[i * (k + 1) + r];
        if (excl && id >= 0 && id == gid) continue;
        if (wpos < k) {
            out_idx[q * k + wpos] = id;
            out_dist[q * k + wpos] = id >= 0 ? edist[i * (k + 1) + r] : __builtin_inff();
            ++wpos;
        }
    }
    for (; wpos < k; ++wpos) {
        out_idx[q * k + wpos] = -1;
        out_dist[q * k + wpos] = __builtin_inff();
    }
}

// ---------------------------------------------------------------------------
// 4. exact fallback scan for uncertified rows
// ---------------------------------------------------------------------------
struct alignas(16) FallbackSmem {
    float ld[FB_THREADS][KLIST];
    int li[FB_THREADS][KLIST];
    float rd[2];
    int ri[2];
    int rt[2];
};

// SQRT: keys are the correctly rounded f32 roots (MN_L2 rows whose equal-root
// run reaches past the extended list, k_l2_order)
template <bool VEC4, bool SQRT = false>
__global__ __launch_bounds__(FB_THREADS) void k_fallback(
    const float *__restrict__ Q, const float *__restrict__ C, int64_t nc, int d, int64_t q_off,
    int64_t c_off, int excl, int k, const int *__restrict__ fb_count,
    const int *__restrict__ fb_list, int32_t *__restrict__ out_idx,
    float *__restrict__ out_dist) {
    __shared__ FallbackSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nfb = *fb_count;
    for (int f = blockIdx.x; f < nfb; f += gridDim.x) {
        const int64_t q = fb_list[f];
        const int64_t gq = q_off + q;
        const bool self_in = excl && gq >= c_off && gq < c_off + nc;
        const int64_t valid = nc - (self_in ? 1 : 0);
        const int keff = (int)min((int64_t)k, valid);
        const float *qrow = Q + q * (int64_t)d;
        int cnt = 0;
        for (int64_t j = tid; keff > 0 && j < nc; j += FB_THREADS) {
            const int64_t gj = c_off + j;
            if (excl && gj == gq) continue;
            float dist = exact_l2sq<VEC4>(qrow, C + j * (int64_t)d, d);
            if constexpr (SQRT) dist = sqrt_rn_f32(dist);
            const int gi = (int)gj;
            if (cnt == keff && !key_less(dist, gi, sm.ld[tid][keff - 1], sm.li[tid][keff - 1]))
                continue;
            int p = cnt < keff ? cnt : keff - 1;
            while (p > 0 && key_less(dist, gi, sm.ld[tid][p - 1], sm.li[tid][p - 1])) {
                sm.ld[tid][p] = sm.ld[tid][p - 1];
                sm.li[tid][p] = sm.li[tid][p - 1];
                --p;
            }
            sm.ld[tid][p] = dist;
            sm.li[tid][p] = gi;
            if (cnt < keff) ++cnt;
        }
        __syncthreads();
        int head = 0;
        for (int r = 0; r < keff; ++r) {
            float bd = head < cnt ? sm.ld[tid][head] : __builtin_inff();
            int bi = head < cnt ? sm.li[tid][head] : INT_MAX;
            int bt = tid;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const float od = __shfl_xor(bd, o);
                const int oi = __shfl_xor(bi, o);
                const int ot = __shfl_xor(bt, o);
                if (key_less(od, oi, bd, bi)) { bd = od; bi = oi; bt = ot; }
            }
            if (lane == 0) { sm.rd[w] = bd; sm.ri[w] = bi; sm.rt[w] = bt; }
            __syncthreads();
            const bool first = key_less(sm.rd[0], sm.ri[0], sm.rd[1], sm.ri[1]) ||
                               !key_less(sm.rd[1], sm.ri[1], sm.rd[0], sm.ri[0]);
            const int win = first ? 0 : 1;
            if (tid == sm.rt[win]) {
                out_idx[q * k + r] = sm.ri[win];
                out_dist[q * k + r] = sm.rd[win];
                ++head;
            }
            __syncthreads();
        }
        for (int r = keff + tid; r < k; r += FB_THREADS) {
            out_idx[q * k + r] = -1;
            out_dist[q * k + r] = __builtin_inff();
        }
        __syncthreads();
    }
}

// Split exact scan for a FEW uncertified rows (k_fallback gives a whole row
// to one block: ~60 ms per row at 1M x 768).  Launch over a batch of up to
// FSQ rows: block b scans corpus part [b chunk, (b+1) chunk) (chunk <= FSC
// rows) for every row of the batch (the rows in LDS, one corpus row per
// thread, the reference fold per (row, corpus row) in feature order), keeps
// the part's survivors — dist <= ub[row] (an exact upper bound of D_k from
// the re-rank, +inf when none) — and writes the part's best keff by (dist,
// id).  k_fb_merge then reduces groups of part lists to one list per row.
constexpr int FSQ = 16;     // rows per launch (LDS: FSQ d floats + the part's distances)
constexpr int FSC = 1024;   // corpus rows per part (one per thread; one sort of <= FSC survivors)
constexpr int FST = 1024;   // threads
constexpr int FMG = 4096;   // merge: entries per group (sorted in LDS)
constexpr int FMT = 256;    // merge threads

__device__ __forceinline__ void lds_bitonic(float *kd, int *ki, int P) {
    for (int kk = 2; kk <= P; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int e = threadIdx.x; e < P; e += blockDim.x) {
                const int pe = e ^ j;
                if (pe > e) {
                    const bool asc = (e & kk) == 0;
                    const bool sw = asc ? key_less(kd[pe], ki[pe], kd[e], ki[e])
                                        : key_less(kd[e], ki[e], kd[pe], ki[pe]);
                    if (sw) {
                        const float td = kd[e]; kd[e] = kd[pe]; kd[pe] = td;
                        const int ti = ki[e]; ki[e] = ki[pe]; ki[pe] = ti;
                    }
                }
            }
            __syncthreads();
        }
}

// One corpus row per thread (FSC = FST, 16 waves): the row's 16-feature
// pieces are loaded whole (4 float4, one 64-B segment) right before use, so
// no lane relies on L1 keeping its row; the batch's query values are staged
// feature-major in LDS (Qt [d][FSQ]: one broadcast ds_read_b128 per 4
// queries and feature).  (Whole rows per lane with 4 waves per CU ran 13-20
// ms per batch at 1M x 768; scalar-loaded queries spilled SGPRs, 9.7 ms.)
template <bool VEC4, bool SQRT>
__global__ __launch_bounds__(FST) void k_fb_part(
    const float *__restrict__ Qt, const float *__restrict__ C, int64_t nc, int d, int64_t q_off,
    int64_t c_off, int excl, int keff_max, const int *__restrict__ rows, int nb,
    const float *__restrict__ ub, const float *__restrict__ ub2, int64_t chunk,
    float2 *__restrict__ plist, int *__restrict__ pcnt) {
    extern __shared__ float4 fsm4[];
    float4 *qs = fsm4;                              // [d][FSQ / 4]: Qt staged
    float *dv = (float *)(qs + (size_t)d * (FSQ / 4));  // [FSQ][FSC]
    float *sd = dv + FSQ * FSC;                     // [FSC]
    int *si = (int *)(sd + FSC);                    // [FSC]
    int &scnt = si[FSC];
    const int P = gridDim.x, b = blockIdx.x, t = threadIdx.x;
    const int64_t c0 = (int64_t)b * chunk, c1 = min(nc, c0 + chunk);
    const int64_t c = c0 + t;
    for (int e = t; e < d * (FSQ / 4); e += FST) qs[e] = reinterpret_cast<const float4 *>(Qt)[e];
    __syncthreads();
    if (c < c1) {
        const float *crow = C + c * (int64_t)d;
        float acc[FSQ];
#pragma unroll
        for (int r = 0; r < FSQ; ++r) acc[r] = -0.0f;
        auto step = [&](float y, int f) {
            const float4 *qf = qs + (size_t)f * (FSQ / 4);  // LDS broadcast reads
#pragma unroll
            for (int r4 = 0; r4 < FSQ / 4; ++r4) {
                const float4 q4 = qf[r4];
                float df = q4.x - y; acc[4 * r4 + 0] = acc[4 * r4 + 0] + df * df;
                df = q4.y - y; acc[4 * r4 + 1] = acc[4 * r4 + 1] + df * df;
                df = q4.z - y; acc[4 * r4 + 2] = acc[4 * r4 + 2] + df * df;
                df = q4.w - y; acc[4 * r4 + 3] = acc[4 * r4 + 3] + df * df;
            }
        };
        if (VEC4) {
            int f = 0;
            for (; f + 16 <= d; f += 16) {
                const float4 *p4 = reinterpret_cast<const float4 *>(crow + f);
                const float4 v0 = p4[0], v1 = p4[1], v2 = p4[2], v3 = p4[3];
                step(v0.x, f); step(v0.y, f + 1); step(v0.z, f + 2); step(v0.w, f + 3);
                step(v1.x, f + 4); step(v1.y, f + 5); step(v1.z, f + 6); step(v1.w, f + 7);
                step(v2.x, f + 8); step(v2.y, f + 9); step(v2.z, f + 10); step(v2.w, f + 11);
                step(v3.x, f + 12); step(v3.y, f + 13); step(v3.z, f + 14); step(v3.w, f + 15);
            }
            for (; f < d; f += 4) {
                const float4 v = *reinterpret_cast<const float4 *>(crow + f);
                step(v.x, f); step(v.y, f + 1); step(v.z, f + 2); step(v.w, f + 3);
            }
        } else {
            for (int f = 0; f < d; ++f) step(crow[f], f);
        }
#pragma unroll
        for (int r = 0; r < FSQ; ++r) dv[r * FSC + t] = SQRT ? sqrt_rn_f32(acc[r]) : acc[r];
    }
    __syncthreads();
    for (int r = 0; r < nb; ++r) {
        const int64_t q = rows[r], gq = q_off + q;
        const float u = fminf(ub ? ub[q] : __builtin_inff(), ub2 ? ub2[r] : __builtin_inff());
        if (t == 0) scnt = 0;
        __syncthreads();
        if (c < c1) {
            const float dist = dv[r * FSC + t];
            const int64_t gj = c_off + c;
            if (!(excl && gj == gq) && dist <= u) {
                const int p = atomicAdd(&scnt, 1);
                sd[p] = dist;
                si[p] = (int)gj;
            }
        }
        __syncthreads();
        const int m = scnt;
        int keep = m;
        if (m > keff_max) {
            int Pw = 1;
            while (Pw < m) Pw <<= 1;
            for (int e = m + t; e < Pw; e += FST) {
                sd[e] = __builtin_inff();
                si[e] = INT_MAX;
            }
            __syncthreads();
            lds_bitonic(sd, si, Pw);
            keep = keff_max;
        }
        float2 *out = plist + ((int64_t)r * P + b) * keff_max;
        for (int e = t; e < keep; e += FST) out[e] = make_float2(sd[e], __int_as_float(si[e]));
        if (t == 0) pcnt[r * P + b] = keep;
        __syncthreads();
    }
}

// Qt [d][FSQ]: the batch's query rows feature-major (zero past nb)
__global__ __launch_bounds__(256) void k_fb_qt(const float *__restrict__ Q, int d,
                                               const int *__restrict__ rows, int nb,
                                               float *__restrict__ Qt) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)d * FSQ) return;
    const int f = (int)(e / FSQ), r = (int)(e % FSQ);
    Qt[e] = r < nb ? Q[(int64_t)rows[r] * d + f] : 0.f;
}

// groups of gs part lists (<= FMG entries) of each row -> that group's best
// keff; with one group left, the row's output (keff = min(k, valid), padded)
template <bool FINAL>
__global__ __launch_bounds__(FMT) void k_fb_merge(
    const float2 *__restrict__ plist, const int *__restrict__ pcnt, int P, int keff_max, int gs,
    float2 *__restrict__ olist, int *__restrict__ ocnt, const int *__restrict__ rows,
    int64_t nc, int64_t q_off, int64_t c_off, int excl, int k, int32_t *__restrict__ out_idx,
    float *__restrict__ out_dist, float *__restrict__ ub_out = nullptr) {
    __shared__ float sd[FMG];
    __shared__ int si[FMG];
    __shared__ int base[FMG / 8 + 1];
    const int G = (P + gs - 1) / gs;
    const int r = blockIdx.x / G, g = blockIdx.x % G, t = threadIdx.x;
    const int p0 = g * gs, p1 = min(P, p0 + gs);
    if (t == 0) {
        int a = 0;
        for (int p = p0; p < p1; ++p) {
            base[p - p0] = a;
            a += pcnt[r * P + p];
        }
        base[p1 - p0] = a;
    }
    __syncthreads();
    const int m = base[p1 - p0];
    for (int p = p0; p < p1; ++p) {
        const int o = base[p - p0], n = base[p - p0 + 1] - o;
        const float2 *src = plist + ((int64_t)r * P + p) * keff_max;
        for (int e = t; e < n; e += FMT) {
            sd[o + e] = src[e].x;
            si[o + e] = __float_as_int(src[e].y);
        }
    }
    int Pw = 1;
    while (Pw < m) Pw <<= 1;
    for (int e = m + t; e < Pw; e += FMT) {
        sd[e] = __builtin_inff();
        si[e] = INT_MAX;
    }
    __syncthreads();
    lds_bitonic(sd, si, Pw);
    const int keep = min(m, keff_max);
    if constexpr (FINAL) {
        const int64_t q = rows[r], gq = q_off + q;
        const bool self_in = excl && gq >= c_off && gq < c_off + nc;
        const int keff = (int)min((int64_t)k, nc - (self_in ? 1 : 0));
        if (ub_out) {  // probe pass: the k-th exact distance seen (an upper bound of D_k)
            if (t == 0) ub_out[r] = (keff > 0 && keep >= keff) ? sd[keff - 1] : __builtin_inff();
            return;
        }
        for (int e = t; e < k; e += FMT) {
            const bool ok = e < keff && e < keep;
            out_idx[q * k + e] = ok ? si[e] : -1;
            out_dist[q * k + e] = ok ? sd[e] : __builtin_inff();
        }
    } else {
        float2 *out = olist + ((int64_t)r * G + g) * keff_max;
        for (int e = t; e < keep; e += FMT) out[e] = make_float2(sd[e], __int_as_float(si[e]));
        if (t == 0) ocnt[r * G + g] = keep;
    }
}

// Host driver of the split scan: the nfb rows listed (device) in rows, in
// batches; part lists in the kSlotX1Esc scratch.  Returns 1 when the shape is
// outside its limits (the caller keeps its other path).
static int fb_split_scan(const float *Q, const float *C, int64_t nc, int d, int64_t q_off,
                         int64_t c_off, int excl, int k, const int *rows, int nfb,
                         const float *ub, bool sqrt_keys, int32_t *out_idx, float *out_dist,
                         hipStream_t s) {
    const int keff_max = k;
    const size_t ldsmax = 160 * 1024;
    if (nc < 1 || k > KBIG || d < 1 ||
        (size_t)d * FSQ * 4 + (size_t)FSQ * FSC * 4 + (size_t)FSC * 8 + 16 > ldsmax)
        return 1;
    static bool attr = false;  // dynamic LDS beyond 64 KB (once per process)
    if (!attr) {
        for (const void *f : {(const void *)k_fb_part<true, true>, (const void *)k_fb_part<true, false>,
                              (const void *)k_fb_part<false, true>, (const void *)k_fb_part<false, false>})
            MN_HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsmax));
        attr = true;
    }
    const int64_t P = (nc + FSC - 1) / FSC;
    const int64_t chunk = FSC;
    // parts per merge group: their entries fit FMG, their prefix k_fb_merge's
    // base[FMG / 8 + 1] (k < 8 would otherwise put > 512 parts in a group)
    const int gs = std::min(FMG / keff_max, FMG / 8);
    // ping-pong part lists: [FSQ][P][keff] and the first merge level; Qt
    const size_t l0 = (size_t)FSQ * P * keff_max, l1 = (size_t)FSQ * ((P + gs - 1) / gs) * keff_max;
    const size_t b0 = (l0 * 8 + 255) & ~(size_t)255, b1 = (l1 * 8 + 255) & ~(size_t)255;
    const size_t c0b = ((size_t)FSQ * P * 4 + 255) & ~(size_t)255;
    const size_t qtb = ((size_t)d * FSQ * 4 + 255) & ~(size_t)255;
    char *g = (char *)scratch(kSlotX1Esc, b0 + b1 + 2 * c0b + qtb + FSQ * 4 + 256);
    if (!g) return MN_ENOMEM;
    float2 *la = (float2 *)g, *lb = (float2 *)(g + b0);
    int *ca = (int *)(g + b0 + b1), *cb = (int *)(g + b0 + b1 + c0b);
    float *Qt = (float *)(g + b0 + b1 + 2 * c0b);
    const bool vec4 = (d % 4 == 0) && (((uintptr_t)Q | (uintptr_t)C) % 16 == 0);
    float *ub2 = (float *)(g + b0 + b1 + 2 * c0b + qtb);  // [FSQ] probe bounds
    // probe: the first PA parts give every row of the batch an exact upper
    // bound of D_k (rows without one, e.g. exact ties at distance 0 beyond k
    // with no candidates, would otherwise keep every part's full list)
    const int64_t PA = std::min<int64_t>(P, 64);
    auto pass = [&](int r0, int nb, int64_t Pn, const float *u2, float *uo) -> int {
        auto kp = vec4 ? (sqrt_keys ? k_fb_part<true, true> : k_fb_part<true, false>)
                       : (sqrt_keys ? k_fb_part<false, true> : k_fb_part<false, false>);
        const size_t lds = (size_t)d * FSQ * 4 + (size_t)FSQ * FSC * 4 + (size_t)FSC * 8 + 16;
        hipLaunchKernelGGL(kp, dim3((unsigned)Pn), dim3(FST), lds, s, Qt, C, nc, d, q_off, c_off,
                           excl, keff_max, rows + r0, nb, ub, u2, chunk, la, ca);
        MN_KCHECK(s, "k_fb_part");
        int Pl = (int)Pn;
        float2 *src = la, *dst = lb;
        int *sc = ca, *dc = cb;
        while (Pl > gs) {
            const int G = (Pl + gs - 1) / gs;
            hipLaunchKernelGGL(k_fb_merge<false>, dim3((unsigned)(nb * G)), dim3(FMT), 0, s, src,
                               sc, Pl, keff_max, gs, dst, dc, rows + r0, nc, q_off, c_off, excl,
                               k, out_idx, out_dist, (float *)nullptr);
            MN_KCHECK(s, "k_fb_merge");
            std::swap(src, dst);
            std::swap(sc, dc);
            Pl = G;
        }
        hipLaunchKernelGGL(k_fb_merge<true>, dim3((unsigned)nb), dim3(FMT), 0, s, src, sc, Pl,
                           keff_max, gs, dst, dc, rows + r0, nc, q_off, c_off, excl, k, out_idx,
                           out_dist, uo);
        MN_KCHECK(s, "k_fb_merge<final>");
        return MN_OK;
    };
    for (int r0 = 0; r0 < nfb; r0 += FSQ) {
        const int nb = std::min(FSQ, nfb - r0);
        hipLaunchKernelGGL(k_fb_qt, dim3((unsigned)(((int64_t)d * FSQ + 255) / 256)), dim3(256), 0,
                           s, Q, d, rows + r0, nb, Qt);
        const bool probe = P > 4 * PA;
        if (probe) {
            const int rc = pass(r0, nb, PA, (const float *)nullptr, ub2);
            if (rc != MN_OK) return rc;
        }
        const int rc = pass(r0, nb, P, probe ? (const float *)ub2 : (const float *)nullptr,
                            (float *)nullptr);
        if (rc != MN_OK) return rc;
    }
    return MN_OK;
}

// ---------------------------------------------------------------------------
// 5. merge of exact per-shard lists (row-sharded multi-GPU build)
// ---------------------------------------------------------------------------
constexpr int MAX_PARTS = 16;
static_assert(MAX_PARTS == kMaxShardRanks, "the sharded build merges up to MAX_PARTS parts");

__global__ __launch_bounds__(256) void k_merge_parts(const int32_t *__restrict__ pidx,
                                                     const float *__restrict__ pdist, int P,
                                                     int64_t nq, int k,
                                                     int32_t *__restrict__ out_idx,
                                                     float *__restrict__ out_dist) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    int head[MAX_PARTS];
#pragma unroll
    for (int p = 0; p < MAX_PARTS; ++p) head[p] = 0;
    for (int r = 0; r < k; ++r) {
        int bp = -1;
        float bd = __builtin_inff();
        int bi = INT_MAX;
#pragma unroll
        for (int p = 0; p < MAX_PARTS; ++p) {
            if (p >= P) break;
            const int h = head[p];
            if (h >= k) continue;
            const int64_t off = ((int64_t)p * nq + q) * k + h;
            const int ci = pidx[off];
            if (ci < 0) continue;
            const float cd = pdist[off];
            if (bp < 0 || key_less(cd, ci, bd, bi)) { bp = p; bd = cd; bi = ci; }
        }
#pragma unroll
        for (int p = 0; p < MAX_PARTS; ++p)
            if (p == bp) head[p]++;
        out_idx[q * k + r] = bp < 0 ? -1 : bi;
        out_dist[q * k + r] = bp < 0 ? __builtin_inff() : bd;
    }
}

}  // namespace knn

namespace {
thread_local mn_knn_stats t_stats{};
}
mn_knn_stats &knn_stats_ref() { return t_stats; }

// perm = the golden-ratio bijection of k_perm_init over n rows, in scratch slot
// `slot`; with_inverse: ipos = perm + n (position of row r in the order);
// then `extra` bytes for the caller.
static int *make_perm(int64_t n, int slot, size_t extra, hipStream_t s, bool with_inverse = false) {
    const size_t words = (size_t)n * (with_inverse ? 2 : 1);
    int *perm = (int *)scratch(slot, sizeof(int) * words + extra + 256);
    if (!perm || n == 0) return perm;
    uint64_t a = (uint64_t)((double)n * 0.6180339887498949);
    if (a == 0) a = 1;
    auto gcd = [](uint64_t x, uint64_t y) { while (y) { const uint64_t t = x % y; x = y; y = t; } return x; };
    while (gcd(a, (uint64_t)n) != 1) ++a;
    a %= (uint64_t)n;
    if (a == 0) a = 1;
    const uint64_t b = (uint64_t)n / 3;
    hipLaunchKernelGGL(knn::k_perm_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, perm,
                       with_inverse ? perm + n : (int *)nullptr, n, a, b);
    return perm;
}

static int knn_f32_core(const float *Q, int64_t nq, const float *C, int64_t nc, int32_t d,
                        int64_t q_off, int64_t c_off, const mn_knn_opts *opts,
                        int32_t *out_idx, float *out_dist, int algo) {
    using namespace knn;
    const int k = opts->k;
    MN_REQUIRE(k >= 1 && k <= KLIST, MN_ENOTSUP, "mn_knn: k=%d outside [1,%d]", k, KLIST);
    // margin clipped so that L = k + margin <= LMAX (MN_L2's extended lists)
    const int margin = std::min(opts->margin > 0 ? opts->margin : 16, LMAX - k);
    const int L = k + margin;
    MN_REQUIRE(L <= LMAX, MN_ENOTSUP, "mn_knn: k+margin=%d exceeds %d", L, LMAX);
    // candidate generator: bf16-split MFMA or f32 MFMA; both are followed by
    // the same exact re-rank / certification / fallback contract
    MN_REQUIRE(!(algo == MN_KNN_BF16X3 && L > kb16::LMAX), MN_ENOTSUP,
               "mn_knn: bf16-split candidates need k+margin <= %d", kb16::LMAX);
    const bool split = algo == MN_KNN_BF16X3 || (algo == MN_KNN_AUTO && L <= kb16::LMAX);
    t_stats.algo = split ? MN_KNN_BF16X3 : MN_KNN_F32;
    MN_REQUIRE(q_off >= 0 && c_off >= 0 && q_off + nq <= INT_MAX && c_off + nc <= INT_MAX,
               MN_EINVAL, "mn_knn: global ids must fit int32");
    const int excl = opts->exclude_self ? 1 : 0;
    hipStream_t s = (hipStream_t)opts->stream;
    t_stats.n_queries = nq;
    if (nq == 0) return MN_OK;

    const bool vec4 = (d % 4 == 0) && (((uintptr_t)Q | (uintptr_t)C) % 16 == 0);
    const bool same = (Q == C) && (nq == nc) && (q_off == c_off);

    // corpus split: enough blocks to fill 256 CUs, bounded by the re-rank width
    const int64_t blocks_q = (nq + BM - 1) / BM;
    int64_t S = 1;
    if (blocks_q < 512) S = (512 + blocks_q - 1) / blocks_q;
    S = std::min<int64_t>(S, 256 / L);
    S = std::min<int64_t>(S, std::max<int64_t>(1, (nc + BN - 1) / BN));
    S = std::max<int64_t>(S, 1);
    int64_t chunk = (nc + S - 1) / S;
    chunk = ((chunk + BN - 1) / BN) * BN;
    if (chunk == 0) chunk = BN;
    S = std::max<int64_t>(1, (nc + chunk - 1) / chunk);
    const int SL = (int)(S * L);
    const int NR = SL <= 64 ? 1 : (SL <= 128 ? 2 : 4);
    t_stats.slices = (int)S;
    t_stats.list_len = L;

    float *qn = (float *)scratch(kSlotNorms, sizeof(float) * (size_t)nq);
    float *cn = same ? qn : (float *)scratch(kSlotNorms2, sizeof(float) * (size_t)std::max<int64_t>(nc, 1));
    int *flags = (int *)scratch(kSlotFlags, 64);
    const size_t nlist = (size_t)nq * S * L;
    char *lists = (char *)scratch(kSlotLists, nlist * 8);
    char *meta = (char *)scratch(kSlotListMeta, (size_t)nq * S * 8);
    int *fb_list = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nq);
    MN_REQUIRE(qn && cn && flags && lists && meta && fb_list, MN_ENOMEM,
               "mn_knn: device scratch allocation failed");
    float *list_d = (float *)lists;
    int *list_i = (int *)(lists + nlist * 4);
    int *lsz = (int *)meta;
    float *ltau = (float *)(meta + (size_t)nq * S * 4);
    unsigned *maxbits = (unsigned *)flags;
    int *nonfinite = flags + 1;
    int *fb_count = flags + 2;

    Timer tm;
    tm.start(opts->timing != 0, s);
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 64, s));
    auto norms = [&](const float *X, int64_t n, float *out) {
        if (n == 0) return;
        int64_t blocks = std::min<int64_t>((n + 3) / 4, 8192);
        if (vec4)
            hipLaunchKernelGGL(k_row_norms<true>, dim3((unsigned)blocks), dim3(256), 0, s, X, n, d,
                               out, maxbits, nonfinite);
        else
            hipLaunchKernelGGL(k_row_norms<false>, dim3((unsigned)blocks), dim3(256), 0, s, X, n, d,
                               out, maxbits, nonfinite);
    };
    if (!same) {
        norms(Q, nq, qn);
        // query norms must not feed the corpus max: recompute flags after
    }
    MN_HIP_TRY(hipMemsetAsync(maxbits, 0, 4, s));
    norms(C, nc, cn);
    MN_HIP_TRY(hipGetLastError());
    int hflags[4] = {0, 0, 0, 0};
    MN_HIP_TRY(hipMemcpyAsync(hflags, flags, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hflags[1] == 0, MN_ENONFINITE,
               "mn_knn: input contains NaN/inf (the reference panics in partial_cmp().unwrap())");
    tm.mark();

    if (split) {
        // ---- bf16-split candidates (gram_bf16.hpp GM_L2) + buffer re-rank ----
        const int dp = (d + 127) / 128 * 128;  // 2 dp bf16 per row: a multiple of DALIGN
        uint16_t *XSq = (uint16_t *)scratch(kSlotGeneric0, (size_t)nq * dp * 4 + 64);
        uint16_t *XSc = (uint16_t *)scratch(kSlotGeneric1, (size_t)nc * dp * 4 + 64);
        // the corpus copy is stored in the golden-ratio visiting order (see
        // k_perm_init), with its norms; ids are mapped back in the re-rank
        int *perm = make_perm(nc, kSlotPerm, sizeof(float) * (size_t)nc, s);
        MN_REQUIRE(XSq && XSc && perm, MN_ENOMEM, "mn_knn: split copy allocation failed");
        float *cnp = (float *)(perm + nc);
        auto split_rows = [&](const float *X, int64_t n, uint16_t *XS, const int *pm) {
            const int64_t th = n * (dp / 8);
            if (th > 0)
                hipLaunchKernelGGL(k_split_bf16, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s,
                                   X, n, d, dp, XS, pm);
        };
        split_rows(Q, nq, XSq, nullptr);
        split_rows(C, nc, XSc, perm);
        if (nc > 0)
            hipLaunchKernelGGL(k_gather_f32, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, cn,
                               perm, nc, cnp);
        MN_KCHECK(s, "k_split_bf16");
        tm.mark();
        const char *ms = knob("MN_L2_MIN_SLICES");
        const kb16::GramPlan pl = kb16::plan_gram(nq, nc, L, (ms && *ms) ? atoi(ms) : 2);
        t_stats.slices = (int)pl.S;
        const size_t nbuf = (size_t)nq * pl.S * pl.cap;
        uint2 *cbuf = (uint2 *)scratch(kSlotLists, nbuf * sizeof(uint2) + 64);
        char *bmeta = (char *)scratch(kSlotListMeta, (size_t)nq * pl.S * 8 + 64);
        MN_REQUIRE(cbuf && bmeta, MN_ENOMEM, "mn_knn: candidate buffer allocation failed (%zu MB)",
                   (nbuf * sizeof(uint2)) >> 20);
        int *bcnt = (int *)bmeta;
        float *btau = (float *)(bmeta + (size_t)nq * pl.S * 4);
        if (nc > 0) {
            const int64_t bq = (nq + kb16::BM - 1) / kb16::BM;
            auto kern = kb16::k_gram_bf16<kb16::GM_L2, 0>;
#ifdef MN_TUNING
            // MN_L2_PROBE=noepi: timing probe (K loop only; results invalid)
            const char *probe = knob("MN_L2_PROBE");
            if (probe && !strcmp(probe, "noepi")) kern = kb16::k_gram_bf16<kb16::GM_L2, 1>;
#endif
            hipLaunchKernelGGL(kern, dim3((unsigned)(bq * pl.S)),
                               dim3(kb16::NT), 0, s, XSq, nq, XSc, nc, 2 * dp, q_off, c_off, 0, qn,
                               cnp, L, (int)pl.S, pl.chunk, pl.cap, cbuf, bcnt, btau);
        } else {
            MN_HIP_TRY(hipMemsetAsync(bcnt, 0, sizeof(int) * (size_t)nq * pl.S, s));
        }
        MN_KCHECK(s, "k_gram_bf16<L2>");
        tm.mark();
        const int64_t nvalid = same ? nc - 1 : nc;
        const dim3 rgrid((unsigned)((nq + 3) / 4));
#define MN_RRB(NRV, V)                                                                          \
    hipLaunchKernelGGL((k_rerank_buf<NRV, V>), rgrid, dim3(256), 0, s, Q, nq, C, d, c_off, qn,   \
                       maxbits, (int)pl.S, pl.cap, cbuf, bcnt, btau, k,                         \
                       std::max<int64_t>(nvalid, 0), dp, perm, q_off, excl, out_idx, out_dist,  \
                       fb_count, fb_list)
        if (vec4) {
            if (pl.NR == 1) MN_RRB(1, true);
            else if (pl.NR == 2) MN_RRB(2, true);
            else if (pl.NR == 4) MN_RRB(4, true);
            else MN_RRB(8, true);
        } else {
            if (pl.NR == 1) MN_RRB(1, false);
            else if (pl.NR == 2) MN_RRB(2, false);
            else if (pl.NR == 4) MN_RRB(4, false);
            else MN_RRB(8, false);
        }
#undef MN_RRB
        MN_KCHECK(s, "k_rerank_buf");
        tm.mark();
    } else {
        tm.mark();  // no split phase
        if (nc > 0) {
            dim3 grid((unsigned)blocks_q, (unsigned)S);
            if (vec4)
                hipLaunchKernelGGL(k_gram_topk<true>, grid, dim3(NT), 0, s, Q, nq, C, nc, d, q_off,
                                   c_off, excl, qn, cn, L, (int)S, chunk, list_d, list_i, lsz, ltau);
            else
                hipLaunchKernelGGL(k_gram_topk<false>, grid, dim3(NT), 0, s, Q, nq, C, nc, d, q_off,
                                   c_off, excl, qn, cn, L, (int)S, chunk, list_d, list_i, lsz, ltau);
            MN_HIP_TRY(hipGetLastError());
        } else {
            MN_HIP_TRY(hipMemsetAsync(lsz, 0, sizeof(int) * (size_t)nq * S, s));
        }
        tm.mark();

        const float cert_c = 2.0f * (4.0f * (float)d + 16.0f) * 0x1p-24f;
        const dim3 rgrid((unsigned)((nq + 3) / 4));
    #define MN_RERANK(NRV, V)                                                                       \
        hipLaunchKernelGGL((k_rerank<NRV, V>), rgrid, dim3(256), 0, s, Q, nq, C, nc, d, c_off, qn,   \
                           maxbits, (int)S, L, list_d, list_i, lsz, ltau, k, cert_c, out_idx,        \
                           out_dist, fb_count, fb_list)
        if (vec4) {
            if (NR == 1) MN_RERANK(1, true);
            else if (NR == 2) MN_RERANK(2, true);
            else MN_RERANK(4, true);
        } else {
            if (NR == 1) MN_RERANK(1, false);
            else if (NR == 2) MN_RERANK(2, false);
            else MN_RERANK(4, false);
        }
    #undef MN_RERANK
        MN_HIP_TRY(hipGetLastError());
        tm.mark();
    }

    const unsigned fgrid = (unsigned)std::min<int64_t>(nq, 1024);
    if (vec4)
        hipLaunchKernelGGL(k_fallback<true>, dim3(fgrid), dim3(FB_THREADS), 0, s, Q, C, nc, d,
                           q_off, c_off, excl, k, fb_count, fb_list, out_idx, out_dist);
    else
        hipLaunchKernelGGL(k_fallback<false>, dim3(fgrid), dim3(FB_THREADS), 0, s, Q, C, nc, d,
                           q_off, c_off, excl, k, fb_count, fb_list, out_idx, out_dist);
    MN_HIP_TRY(hipGetLastError());
    tm.mark();
    MN_HIP_TRY(hipMemcpyAsync(hflags, flags, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    t_stats.n_uncertified = hflags[2];
    if (tm.on) {
        t_stats.ms_norms = tm.ms(0, 2);  // norms (+ bf16 split)
        t_stats.ms_gram = tm.ms(2, 3);
        t_stats.ms_rerank = tm.ms(3, 4);
        t_stats.ms_fallback = tm.ms(4, 5);
        t_stats.ms_total = tm.ms(0, 5);
    }
    return MN_OK;
}


static int knn_f32_core(const float *Q, int64_t nq, const float *C, int64_t nc, int32_t d,
                        int64_t q_off, int64_t c_off, const mn_knn_opts *opts,
                        int32_t *out_idx, float *out_dist, int algo);

// Host driver of MN_KNN_BF16X1 (section 2c).  Returns 1 (nothing written)
// when some row is too large for the single-bf16 bound: the caller then runs
// the split generator.
// ---- phase 1 as a sweep (round 4) -------------------------------------------
// The list generator (k_gram_bf16<GM_L2H>, ~0.2 of the MFMA peak: 130 ms at
// C2) keeps a sorted list per row while it scans the sample.  Here: (a) the
// list generator on a pre-sample (the first m0 / P1_DIV sample positions, list
// P1_L0) gives each row a threshold T0 = its P1_L0-th best key there; (b) the
// query-major sweep (k_gram_sweep2<SW_L2>, tile-major copies) buffers every
// sample pair with key < T0 (expected ~P1_DIV P1_L0 a row); (c) k_p1_select
// takes each row's L1-th smallest buffered key = the sample's L1-th best key,
// the list generator's threshold (an overflowing buffer gives a larger key:
// still a threshold; correctness rests on the certificate); (d) rows with fewer
// than L1 buffered keys (T0 below the sample's L1-th key) run the list
// generator on their own.  btau1 [nq] (one slice) as before.  C2 (same box,
// profiles/r04/r04_p1_ab.log): 130.7 -> 97.1 ms (pre 23.3, sweep 64.5, select
// 0.8, 48.8k rows to (d)); (4, 16) 104.8 ms, (6, 16) 103.7, (6, 24) 108.9 —
// fewer buffered keys beat a cheaper pre-sample; outputs identical.
constexpr int P1_L0 = 4, P1_DIV = 8;

// one wave per row: the L1-th smallest of the row's buffered keys (repeated
// minimum with multiplicities: exact, <= L1 rounds); fewer than L1 keys: the
// row is listed for (d)
template <int NR>
__global__ __launch_bounds__(256) void k_p1_select(int64_t nq, const int *__restrict__ cnt,
                                                   const uint2 *__restrict__ buf, int cap, int L1,
                                                   float *__restrict__ btau, int *__restrict__ fb_count,
                                                   int *__restrict__ fb_list) {
    const int lane = threadIdx.x & 63;
    const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (q >= nq) return;
    int c = cnt[q];
    c = (c < 0 || c > cap) ? cap : c;  // -1: overflow, the buffer is full
    if (c < L1) {
        if (lane == 0) {
            btau[q] = __builtin_inff();
            fb_list[atomicAdd(fb_count, 1)] = (int)q;
        }
        return;
    }
    float kk[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        kk[r] = e < c ? __uint_as_float(buf[q * (int64_t)cap + e].x) : __builtin_inff();
    }
    float t = -__builtin_inff(), res = __builtin_inff();
    int need = L1;
    for (int it = 0; it < L1; ++it) {
        float m = __builtin_inff();
#pragma unroll
        for (int r = 0; r < NR; ++r) m = fminf(m, kk[r] > t ? kk[r] : __builtin_inff());
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
        int eq = 0;
#pragma unroll
        for (int r = 0; r < NR; ++r) eq += (int)__popcll(__ballot(kk[r] == m));
        if (eq >= need) { res = m; break; }
        need -= eq;
        t = m;
    }
    if (lane == 0) btau[q] = res;
}

__global__ __launch_bounds__(256) void k_gather_bf16_rows(const uint16_t *__restrict__ R, int dp,
                                                          const float *__restrict__ qn,
                                                          const int *__restrict__ rows, int nfb,
                                                          uint16_t *__restrict__ out,
                                                          float *__restrict__ qn_out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < (int64_t)nfb * dp) {
        const int64_t i = e / dp;
        out[e] = R[(int64_t)rows[i] * dp + (e - i * dp)];
    }
    if (e < nfb) qn_out[e] = qn[rows[e]];
}

__global__ __launch_bounds__(256) void k_scatter_tau(const int *__restrict__ rows, int nfb,
                                                     const float *__restrict__ v,
                                                     float *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nfb) out[rows[i]] = v[i];
}

static int sweep_phase1(const uint16_t *QR, const uint16_t *QK, int64_t nq, const uint16_t *CR,
                        const uint16_t *CKs, int64_t m0, int d, int dp, int nkb, int pst1,
                        int64_t q_off, int L1, const float *qn, const float *qhn, const float *qrn,
                        const float *cnv, const float *chc, const unsigned *cmax, float *tq,
                        float *tau0, float *dlt, float *btau1, int *fb_list, int *cntr,
                        hipStream_t s) {
    using namespace knn;
    Timer tdb;  // tuning build, MN_X1_DEBUG: the steps' times
    tdb.start(knob("MN_X1_DEBUG") != nullptr, s);
    // (a) the pre-sample: the list generator, list P1_L0, over the first m00
    const char *l0e = knob("MN_P1_L0"), *dve = knob("MN_P1_DIV");  // tuning build: experiments
    const int L0 = (l0e && *l0e) ? std::min(std::max(atoi(l0e), 2), 32) : P1_L0;
    const int dv = (dve && *dve) ? std::max(2, atoi(dve)) : P1_DIV;
    int64_t m00 = std::max<int64_t>(m0 / dv, (int64_t)64 * L0);
    m00 = std::min<int64_t>(m0, (m00 + 255) / 256 * 256);
    const kb16::GramPlan p0 = kb16::plan_gram(nq, m00, L0, 1, 1);
    // (phase-2 / escalation slots: the caller's phase-1 list slots stay valid
    // for the query-major fallback)
    uint2 *cb0 = (uint2 *)scratch(kSlotX1Esc, (size_t)nq * p0.S * p0.cap * sizeof(uint2) + 64);
    int *bc0 = (int *)scratch(kSlotX1Meta2, (size_t)nq * p0.S * 4 + 64);
    MN_REQUIRE(cb0 && bc0, MN_ENOMEM, "mn_knn: pre-sample buffer allocation failed");
    const int64_t bq = (nq + kb16::BM - 1) / kb16::BM;
    hipLaunchKernelGGL((kb16::k_gram_bf16<kb16::GM_L2H, 0>), dim3((unsigned)(bq * p0.S)),
                       dim3(kb16::NT), 0, s, QR, nq, CR, m00, dp, q_off, (int64_t)0, 0, qn, cnv,
                       L0, (int)p0.S, p0.chunk, p0.cap, cb0, bc0, btau1);
    MN_KCHECK(s, "k_gram_bf16<L2H, pre-sample>");
    hipLaunchKernelGGL(k_tau_x1, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, nq,
                       (int)p0.S, btau1, qn, qhn, qrn, cmax, d, dp, tq, tau0, dlt,
                       (unsigned *)nullptr);
    MN_KCHECK(s, "k_tau_x1<pre-sample>");
    tdb.mark();
    // (b) the sweep of the sample with T0
    const double expect = (double)L0 * (double)m0 / (double)m00;
    const int cap = std::min(512, std::max(64, (int)((2.5 * expect + 64.0 + 15.0) / 16.0) * 16));
    uint2 *cbuf = (uint2 *)scratch(kSlotX1Buf2, (size_t)nq * cap * sizeof(uint2) + 64);
    int *cnt = (int *)scratch(kSlotX1Meta2, (size_t)nq * 4 + 64);
    MN_REQUIRE(cbuf && cnt, MN_ENOMEM, "mn_knn: phase-1 sweep buffer allocation failed");
    MN_HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)nq * 4, s));
    const int64_t nqb = (nq + ksw2::BQ - 1) / ksw2::BQ;
    MN_REQUIRE(nqb < INT_MAX && nq * 32 < INT_MAX, MN_ENOTSUP, "mn_knn: phase-1 sweep grid too large");
    // round 6: gram_sweep3.hpp's schedule in its query-major mode (global
    // per-row counters; tuning build MN_P1_SWEEP3=0: round 5's sweep2)
    auto p1k = ksw2::k_gram_sweep3<0, ksw2::SW_L2, 2>;
#ifdef MN_TUNING
    if (!knob_int("MN_P1_SWEEP3", 1)) p1k = ksw2::k_gram_sweep2<0, ksw2::SW_L2, true>;
#endif
    hipLaunchKernelGGL(p1k, dim3((unsigned)nqb), dim3(ksw2::NT), 0, s, QK, nq, CKs, m0, nkb, q_off,
                       (int64_t)0, 0, tq, tau0, chc, (int64_t)0, 1, m0, cap, cbuf, cnt, pst1,
                       ksw2::SymArgs{});
    MN_KCHECK(s, "k_gram_sweep3<SW_L2, phase 1>");
    tdb.mark();
    // (c) the L1-th smallest buffered key per row
    MN_HIP_TRY(hipMemsetAsync(cntr, 0, 4, s));
    const unsigned g4 = (unsigned)((nq + 3) / 4);
    if (cap <= 128)
        hipLaunchKernelGGL(k_p1_select<2>, dim3(g4), dim3(256), 0, s, nq, cnt, cbuf, cap, L1, btau1, cntr, fb_list);
    else if (cap <= 256)
        hipLaunchKernelGGL(k_p1_select<4>, dim3(g4), dim3(256), 0, s, nq, cnt, cbuf, cap, L1, btau1, cntr, fb_list);
    else
        hipLaunchKernelGGL(k_p1_select<8>, dim3(g4), dim3(256), 0, s, nq, cnt, cbuf, cap, L1, btau1, cntr, fb_list);
    MN_KCHECK(s, "k_p1_select");
    int nfb = 0;
    MN_HIP_TRY(hipMemcpyAsync(&nfb, cntr, 4, hipMemcpyDeviceToHost, s));
    tdb.mark();
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (tdb.on)
        fprintf(stderr, "sweep_phase1: pre-sample %lld, cap %d, rows short of L1 %d; ms pre %.2f sweep %.2f select %.2f\n",
                (long long)m00, cap, nfb, tdb.ms(0, 1), tdb.ms(1, 2), tdb.ms(2, 3));
    if (nfb == 0) return MN_OK;
    // (d) the rows T0 left short: the list generator on them alone
    const kb16::GramPlan pf = kb16::plan_gram(nfb, m0, L1, 1, 1);
    const size_t gb = (size_t)nfb * dp * 2, lb = (size_t)nfb * pf.S * pf.cap * sizeof(uint2);
    char *g = (char *)scratch(kSlotX1Esc, gb + lb + (size_t)nfb * pf.S * 8 + (size_t)nfb * 8 + 1024);
    MN_REQUIRE(g, MN_ENOMEM, "mn_knn: phase-1 fallback allocation failed");
    uint16_t *QRf = (uint16_t *)g;
    uint2 *cbf = (uint2 *)(g + ((gb + 255) & ~(size_t)255));
    int *bcf = (int *)((char *)cbf + ((lb + 255) & ~(size_t)255));
    float *btf = (float *)(bcf + (size_t)nfb * pf.S);
    float *qnf = btf + (size_t)nfb * pf.S;
    hipLaunchKernelGGL(k_gather_bf16_rows, dim3((unsigned)(((int64_t)nfb * dp + 255) / 256)), dim3(256),
                       0, s, QR, dp, qn, fb_list, nfb, QRf, qnf);
    MN_KCHECK(s, "k_gather_bf16_rows");
    const int64_t bqf = (nfb + kb16::BM - 1) / kb16::BM;
    hipLaunchKernelGGL((kb16::k_gram_bf16<kb16::GM_L2H, 0>), dim3((unsigned)(bqf * pf.S)),
                       dim3(kb16::NT), 0, s, QRf, (int64_t)nfb, CR, m0, dp, (int64_t)0, (int64_t)0, 0,
                       qnf, cnv, L1, (int)pf.S, pf.chunk, pf.cap, cbf, bcf, btf);
    MN_KCHECK(s, "k_gram_bf16<L2H, phase-1 fallback>");
    hipLaunchKernelGGL(k_scatter_tau, dim3((unsigned)((nfb + 255) / 256)), dim3(256), 0, s, fb_list,
                       nfb, btf, btau1);
    MN_KCHECK(s, "k_scatter_tau");
    return MN_OK;
}

static int knn_x1(const float *Q, int64_t nq, const float *C, int64_t nc, int32_t d,
                  int64_t q_off, int64_t c_off, const mn_knn_opts *opts, int32_t *out_idx,
                  float *out_dist) {
    using namespace knn;
    const int k = opts->k;
    const int margin = opts->margin > 0 ? opts->margin : 16;
    const int excl = opts->exclude_self ? 1 : 0;
    hipStream_t s = (hipStream_t)opts->stream;
    const bool vec4 = (d % 4 == 0) && (((uintptr_t)Q | (uintptr_t)C) % 16 == 0);
    const bool same = (Q == C) && (nq == nc) && (q_off == c_off);
    const int dp = (d + 255) / 256 * 256;  // kb16 DALIGN; KB32 stages: nkb = dp / 32 >= 8
    const int nkb = dp / 32;
    t_stats.algo = MN_KNN_BF16X1;

    // queries in place (QR row-major for phase 1, QK KB32 for the sweep); the
    // corpus in the golden-ratio visiting order (CR, CK; position p holds row
    // perm[p]), so the phase-1 sample is the contiguous prefix [0, m0) and the
    // sweep covers [m0, nc); ids are mapped back through perm in the re-rank
    uint16_t *QR = (uint16_t *)scratch(kSlotX1QR, (size_t)nq * dp * 2 + 64);
    // sweep2 reads tile-major KB32 (rows padded to whole 256-row panels; the
    // pad rows are never candidates); the legacy sweep the k-block-major form
    const char *tme = knob("MN_X1_TM");  // tuning build: 0 = k-block-major layout (A/B)
    const int tmaj = (tme && *tme == '0') ? 0 : 1;
    // tile-major panel stride: nkb + TM_PAD k-blocks (MN_TM_PAD, default 1)
    const char *tpe = knob("MN_TM_PAD");
    const int tpad = (tpe && *tpe) ? std::max(0, atoi(tpe)) : 1;
    const int pst1 = tmaj ? nkb + tpad : 0, pst3 = tmaj ? 3 * nkb + tpad : 0;
    auto pad256 = [&](int64_t r) { return tmaj ? (r + 255) / 256 * 256 : r; };
    const int64_t kbw1 = tmaj ? (int64_t)pst1 * 32 : dp, kbw3 = tmaj ? (int64_t)pst3 * 32 : 3 * dp;
    uint16_t *QK = (uint16_t *)scratch(kSlotX1QK, (size_t)pad256(nq) * kbw1 * 2 + 64);
    uint16_t *CR = (uint16_t *)scratch(kSlotX1CR, (size_t)nc * dp * 2 + 64);
    uint16_t *CK = (uint16_t *)scratch(kSlotX1CK, (size_t)pad256(nc) * kbw1 * 2 + 64);
    char *aux = (char *)scratch(kSlotX1Aux, (size_t)nq * 28 + (size_t)nc * 8 + 256);
    int *flags = (int *)scratch(kSlotFlags, 128);
    int *fb_list = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nq * 2 + 64);
    int *perm = make_perm(nc, kSlotPerm, 0, s);
    MN_REQUIRE(QR && QK && CR && CK && aux && flags && fb_list && perm, MN_ENOMEM,
               "mn_knn: bf16x1 scratch allocation failed");
    float *qn = (float *)aux, *qhn = qn + nq, *qrn = qhn + nq, *tq = qrn + nq, *tau0 = tq + nq,
          *dlt = tau0 + nq;
    float *cnv = dlt + nq, *chc = cnv + nc;  // corpus norms / half norms, visiting order
    float *ubv = chc + nc;                   // upper bounds of D_k of uncertified rows
    unsigned *cmax = (unsigned *)flags;  // [0..2]: max |c|^2, |ch|, |rc|
    int *fb_count = flags + 5;  // [3]: non-finite input, [4]: too large for bf16x1
    unsigned long long *ncand = (unsigned long long *)(flags + 8);

    // phase-1 sample: the first m0 corpus rows, list length L1 (tau0 ~ the
    // (L1 nc / m0)-th best key); small corpora run phase 1 alone (m0 = nc).
    // The symmetric sweep (self kNN) samples nc/24 with list 12 (same box,
    // profiles/r03h_grid_*.log — uniform C2 / clustered C2 ms: nc/16 x 16
    // 1025 / 1713, nc/24 x 12 978 / 1565, nc/32 x 8 946 / 1976 (its 155k
    // refilled rows), nc/32 x 12 1004 / 1345)
    const char *sye = knob("MN_X1_SYM");  // tuning build: 0 = the query-major sweep (A/B)
    const bool sym_pre = same && excl && tmaj && !(sye && *sye == '0');
    int L1 = sym_pre ? std::min(std::max((3 * k + 3) / 8, 12), 48)
                     : std::min(std::max((k + 1) / 2, 16), 48);
    const char *fl = knob("MN_X1_L1");  // experiments: phase-1 list length
    if (fl && *fl) L1 = std::min(std::max(atoi(fl), 4), 48);
    const char *fs = knob("MN_X1_SAMPLE_DIV");  // experiments: sample = nc / div
    const int64_t div = (fs && *fs) ? std::max(2, atoi(fs)) : (sym_pre ? 24 : 16);
    int64_t m0 = std::max<int64_t>(nc / div, (int64_t)64 * L1);
    m0 = (m0 + 255) / 256 * 256;  // whole phase-1 tiles and whole sweep panels
    const bool two = m0 + 4 * ksw2::BC <= nc;
    if (!two) {
        m0 = nc;
        L1 = std::min(k + margin, kb16::LMAX);
    }
    // self kNN: the symmetric sweep (gram_sweep2.hpp SW_SYM: each unordered
    // pair once, rows in ascending-tau0 order; MN_X1_SYM=0 for the
    // query-major sweep of the rows outside the sample)
    bool sym = sym_pre && two;

    // flags: [0..2] cmax, [3] non-finite input, [4] too large for bf16x1,
    // [5] fb_count, [6] big_count, [7] max |tau0|, [8..9] ncand, [10..13]
    // refill maxima, [14] max |x|, [16..17] fp16 maxima (SW_SYM)
    Timer tm;
    tm.start(opts->timing != 0, s);
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 128, s));
    auto prep = [&](const float *X, int64_t n, const int *pm, uint16_t *R, uint16_t *K, float *nv,
                    float *hcv, float *hv, float *rv, int corpus, unsigned *amax = nullptr) {
        if (n == 0) return;
        const int64_t blocks = std::min<int64_t>((n + 7) / 8, 16384);
        if (vec4)
            hipLaunchKernelGGL(k_prep_x1<true>, dim3((unsigned)blocks), dim3(256), 0, s, X, n, d,
                               dp, pm, R, K, nv, hcv, hv, rv, cmax, flags + 3, corpus, pst1, amax);
        else
            hipLaunchKernelGGL(k_prep_x1<false>, dim3((unsigned)blocks), dim3(256), 0, s, X, n, d,
                               dp, pm, R, K, nv, hcv, hv, rv, cmax, flags + 3, corpus, pst1, amax);
    };
    // phase 1 as a sweep (round 4, SW_SYM only; tuning build: MN_P1_SWEEP=0
    // keeps the list generator): tile-major copies of the rows and the sample
    const char *p1e = knob("MN_P1_SWEEP");
    const bool p1s = sym && !(p1e && *p1e == '0');
    uint16_t *CKs = nullptr;
    if (p1s) {
        CKs = (uint16_t *)scratch(kSlotGeneric3, (size_t)pad256(m0) * kbw1 * 2 + 64);
        MN_REQUIRE(CKs, MN_ENOMEM, "mn_knn: sample copy allocation failed");
    }
    if (sym) {
        // phase 1 only: the rows (maxima over them: Q == C) and the sample;
        // the sweep copy is built in tau0 order below
        prep(Q, nq, nullptr, QR, p1s ? QK : nullptr, qn, nullptr, qhn, qrn, 1);
        prep(C, m0, perm, CR, CKs, cnv, chc, nullptr, nullptr, 0);
    } else {
        prep(Q, nq, nullptr, QR, QK, qn, nullptr, qhn, qrn, 0);
        prep(C, nc, perm, CR, CK, cnv, chc, nullptr, nullptr, 1);
    }
    MN_KCHECK(s, "k_prep_x1");
    int hflags[8] = {0};
    MN_HIP_TRY(hipMemcpyAsync(hflags, flags, 32, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hflags[3] == 0, MN_ENONFINITE,
               "mn_knn: input contains NaN/inf (the reference panics in partial_cmp().unwrap())");
    if (hflags[4] != 0) return 1;
    tm.mark();

    t_stats.sample_rows = m0;
    t_stats.list_len = L1;
    const kb16::GramPlan pl = kb16::plan_gram(nq, m0, L1, 1, two ? 1 : 0);
    t_stats.slices = (int)pl.S;
    const size_t nbuf1 = (size_t)nq * pl.S * pl.cap;
    uint2 *cbuf1 = (uint2 *)scratch(kSlotLists, nbuf1 * sizeof(uint2) + 64);
    char *meta1 = (char *)scratch(kSlotListMeta, (size_t)nq * pl.S * 8 + 64);
    MN_REQUIRE(cbuf1 && meta1, MN_ENOMEM, "mn_knn: phase-1 buffer allocation failed (%zu MB)",
               (nbuf1 * sizeof(uint2)) >> 20);
    int *bcnt1 = (int *)meta1;
    float *btau1 = (float *)(meta1 + (size_t)nq * pl.S * 4);
    if (p1s) {
        const int rc1 = sweep_phase1(QR, QK, nq, CR, CKs, m0, d, dp, nkb, pst1, q_off, L1, qn, qhn, qrn,
                                     cnv, chc, cmax, tq, tau0, dlt, btau1, fb_list, flags + 20, s);
        if (rc1 != MN_OK) return rc1;
    } else {
        const int64_t bq = (nq + kb16::BM - 1) / kb16::BM;
        hipLaunchKernelGGL((kb16::k_gram_bf16<kb16::GM_L2H, 0>), dim3((unsigned)(bq * pl.S)),
                           dim3(kb16::NT), 0, s, QR, nq, CR, m0, dp, q_off, (int64_t)0, 0, qn, cnv,
                           L1, (int)pl.S, pl.chunk, pl.cap, cbuf1, bcnt1, btau1);
        MN_KCHECK(s, "k_gram_bf16<L2H>");
    }
    unsigned *tmaxb = (unsigned *)(flags + 7);  // max |tau0| (SW_SYM bound)
    hipLaunchKernelGGL(k_tau_x1, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, nq,
                       (int)pl.S, btau1, qn, qhn, qrn, cmax, d, dp, tq, tau0, dlt, tmaxb);
    MN_KCHECK(s, "k_tau_x1");
    tm.mark();

    int S2 = 0, cap2 = 0;
    uint2 *cbuf2 = nullptr;
    int *cnt2 = nullptr;
    // what the re-rank reads: per-query thresholds / bounds, the phase-1
    // lists (S1 slices), the id map (positions -> rows) and the row map
    int S1r = (int)pl.S;
    int sym_mark = 0;  // 1: an extra timer mark before the SW_SYM sweep
    const float *tau_r = tau0, *dlt_r = dlt;
    float rel_r = 0.f;  // > 0: keys are per-pair lower bounds (SW_SYM), see k_rerank_x1
    const int *perm_r = perm, *qmap_r = nullptr;
    const float *chc_r = chc;
    // tuning build only: timing probes (noepi = sweep K loop only; nodma /
    // noread = also without the DMA issue / fragment reads): NO outputs
    const char *probe = knob("MN_X1_PROBE");
    if (sym) {
        // rows in ascending fold threshold Tf (position p holds row pi[p],
        // k_sym_row); a non-finite threshold would break the column fold
        const size_t nn = (size_t)nc;
        char *so = (char *)scratch(kSlotSymOrd, nn * 4 * 17 + 8192);
        uint16_t *XK = (uint16_t *)scratch(kSlotX1CK, (size_t)pad256(nc) * kbw1 * 2 + 64);
        MN_REQUIRE(so && XK, MN_ENOMEM, "mn_knn: symmetric-sweep scratch allocation failed");
        auto arr = [&](int i) { return so + (size_t)i * (((nn * 4) + 255) & ~(size_t)255); };
        float *skey = (float *)arr(0);
        int *pi = (int *)arr(1), *iota = (int *)arr(2);
        float *tauP = (float *)arr(3), *teffP = (float *)arr(4), *hcP = (float *)arr(5),
              *Up = (float *)arr(6), *Vp = (float *)arr(7), *zdlt = (float *)arr(8),
              *scP = (float *)arr(9), *h16 = (float *)arr(10), *r16 = (float *)arr(11),
              *s16 = (float *)arr(12), *alr = (float *)arr(13), *tfr = (float *)arr(14),
              *tcr = (float *)arr(15);
        float kmax = 0.f;
        {   // any non-finite threshold: the query-major sweep (below)
            hipLaunchKernelGGL(k_iota, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, iota, nc);
            MN_HIP_TRY(sort_f32_pairs(tau0, skey, iota, pi, nc, s));
            MN_HIP_TRY(hipMemcpyAsync(&kmax, skey + nc - 1, 4, hipMemcpyDeviceToHost, s));
            MN_HIP_TRY(hipStreamSynchronize(s));
        }
        if (!(kmax < __builtin_inff())) {
            // fall back to the query-major sweep: its copies were skipped (and
            // a sweep phase 1 left no sample lists: the list generator)
            sym = false;
            if (p1s) {
                const int64_t bq = (nq + kb16::BM - 1) / kb16::BM;
                hipLaunchKernelGGL((kb16::k_gram_bf16<kb16::GM_L2H, 0>), dim3((unsigned)(bq * pl.S)),
                                   dim3(kb16::NT), 0, s, QR, nq, CR, m0, dp, q_off, (int64_t)0, 0, qn,
                                   cnv, L1, (int)pl.S, pl.chunk, pl.cap, cbuf1, bcnt1, btau1);
                MN_KCHECK(s, "k_gram_bf16<L2H>");
                hipLaunchKernelGGL(k_tau_x1, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, nq,
                                   (int)pl.S, btau1, qn, qhn, qrn, cmax, d, dp, tq, tau0, dlt,
                                   (unsigned *)nullptr);
                MN_KCHECK(s, "k_tau_x1");
            }
            prep(Q, nq, nullptr, nullptr, QK, qn, nullptr, qhn, qrn, 0);
            prep(C, nc, perm, nullptr, CK, cnv, chc, nullptr, nullptr, 1);
            MN_KCHECK(s, "k_prep_x1");
        } else {
            // fp16 operands x 2^e with a per-row e, the per-pair bound folded
            // into the thresholds: statistics by row, the rows' fold / certificate
            // thresholds, rows sorted by the fold threshold, the fp16 copy in
            // that order (k_prep_f16r, k_sym_row, k_sym_pos)
            const int64_t blocks = std::min<int64_t>((nc + 7) / 8, 16384);
            auto f16r = [&](const int *pm, uint16_t *K, float *hv, float *rv, float *sv) {
                if (vec4)
                    hipLaunchKernelGGL(k_prep_f16r<true>, dim3((unsigned)blocks), dim3(256), 0, s, C,
                                       nc, d, dp, pm, K, hv, rv, sv, pst1);
                else
                    hipLaunchKernelGGL(k_prep_f16r<false>, dim3((unsigned)blocks), dim3(256), 0, s, C,
                                       nc, d, dp, pm, K, hv, rv, sv, pst1);
            };
            f16r(nullptr, nullptr, h16, r16, s16);
            MN_KCHECK(s, "k_prep_f16r<stats>");
            hipLaunchKernelGGL(k_sym_row, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s,
                               nc, tau0, qn, h16, r16, d, dp, alr, tfr, tcr);
            MN_KCHECK(s, "k_sym_row");
            hipLaunchKernelGGL(k_iota, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, iota, nc);
            MN_HIP_TRY(sort_f32_pairs(tfr, skey, iota, pi, nc, s));
            f16r(pi, XK, nullptr, nullptr, nullptr);
            MN_KCHECK(s, "k_prep_f16r");
            hipLaunchKernelGGL(k_sym_pos, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s,
                               nc, pi, qn, alr, tfr, tcr, s16, tauP, teffP, Up, Vp, hcP, scP);
            MN_HIP_TRY(hipMemsetAsync(zdlt, 0, nn * 4, s));
            MN_KCHECK(s, "k_sym_pos");
            // block table (gram_sweep2.hpp sym_block_table): order 2 (default,
            // round 4), XCD groups of 4 row blocks x 8 column phases — each
            // XCD's 32 co-resident blocks read 12 panels per tile step instead
            // of 33: C2 sweep 788 -> 720 ms, same process (profiles/
            // r04/r04b_ab_order.log); order 1: column ranges of TPB tiles ordered by
            // range then row (round 3); order 0: ranges from the diagonal
            const int nbk = (int)((nc + ksw2::BC - 1) / ksw2::BC);
            const char *tpe2 = knob("MN_SYM_TPB");
            const int TPB = (tpe2 && *tpe2) ? std::max(1, atoi(tpe2)) : 256;
            const char *ore = knob("MN_SYM_ORDER");
            const int order = (ore && *ore) ? atoi(ore) : 2;
            // 2 x 16 groups (tuning build: MN_SYM_GSHAPE = rows of a 32-block group)
            int4 *dtab = nullptr;
            const std::vector<int4> &tab =
                ksw2::sym_table_device(nbk, TPB, order, knob_int("MN_SYM_GSHAPE", 2), 0, 1, s, &dtab);
            MN_REQUIRE(dtab, MN_ENOMEM, "mn_knn: block table allocation / upload failed");
            // per-row buffers: expect ~ L1 nc / m0 candidates a row
            const double expect = (double)L1 * (double)nc / (double)m0;
            const char *cpe = knob("MN_SYM_CAP");
            cap2 = (cpe && *cpe) ? std::max(64, atoi(cpe))
                                 : std::max(256, (int)((2.5 * expect + 64.0 + 15.0) / 16.0) * 16);
            S2 = 1;
            t_stats.sweep_slices = -1;  // symmetric: one per-row buffer
            t_stats.sweep_cap = cap2;
            cbuf2 = (uint2 *)scratch(kSlotX1Buf2, nn * cap2 * sizeof(uint2) + 64);
            cnt2 = (int *)scratch(kSlotX1Meta2, nn * 4 + 64);
            MN_REQUIRE(cbuf2 && cnt2, MN_ENOMEM,
                       "mn_knn: symmetric sweep buffer allocation failed (%zu MB)",
                       (nn * cap2 * sizeof(uint2)) >> 20);
            MN_HIP_TRY(hipMemsetAsync(cnt2, 0, nn * 4, s));
            MN_REQUIRE(tab.size() < INT_MAX && nc * 32 < INT_MAX, MN_ENOTSUP,
                       "mn_knn: sweep grid too large (split the queries / corpus)");
            tm.mark();  // SW_SYM: sort / fp16 copy / table -> ms_norms
            sym_mark = 1;
            // diagonal tile: acc0 = U_q s_c + V_c s_q (tq = U, hc = V);
            // off-diagonal: V_q s_c + U_c s_q (aoff = V, hoff = U); keys from Teff
            ksw2::SymArgs sa{dtab, Vp, Up, scP};
            // the default: gram_sweep3.hpp's schedule, DMA two k-steps ahead
            auto sk = ksw2::k_gram_sweep3<0, ksw2::SW_SYM, 2>;
#ifdef MN_TUNING
            // MN_SWEEP=2: round 5's k_gram_sweep2 (and its MN_SW_V variants)
            const int sweep_gen = knob_int("MN_SWEEP", 4);
            if (sweep_gen == 2) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true>;
            // timing probes (results invalid): noepi = K loop only, nodma /
            // noread = also without the DMA issue / fragment reads
            // l2res / l2res_noepi = operands L2-resident (panels 0 / 1)
            // MN_SW_V: the DMA-placement variants of gram_sweep2.hpp (default 2)
            const int swv = sweep_gen == 2 ? knob_int("MN_SW_V", 14) : -1;
            if (swv == 0) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true, 0>;
            if (swv == 6) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true, 6>;
            if (swv == 10) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true, 10>;
            if (swv == 2) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true, 2>;
            if (swv == 12) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true, 12>;
            if (swv == 1) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true, 1>;
            if (swv == 3) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true, 3>;
            if (sweep_gen != 2) {
            } else if (probe && *probe && swv >= 0 && swv <= 3)
                sk = swv == 0 ? ksw2::k_gram_sweep2<1, ksw2::SW_SYM, true, true, 0>
                     : swv == 1 ? ksw2::k_gram_sweep2<1, ksw2::SW_SYM, true, true, 1>
                     : swv == 2 ? ksw2::k_gram_sweep2<1, ksw2::SW_SYM, true, true, 2>
                                : ksw2::k_gram_sweep2<1, ksw2::SW_SYM, true, true, 3>;
            else if (probe && *probe)
                sk = !strcmp(probe, "nodma") ? ksw2::k_gram_sweep2<2, ksw2::SW_SYM, true, true>
                     : !strcmp(probe, "noread") ? ksw2::k_gram_sweep2<3, ksw2::SW_SYM, true, true>
                     : !strcmp(probe, "l2res") ? ksw2::k_gram_sweep2<5, ksw2::SW_SYM, true, true>
                     : !strcmp(probe, "l2res_noepi") ? ksw2::k_gram_sweep2<6, ksw2::SW_SYM, true, true>
                                                : ksw2::k_gram_sweep2<1, ksw2::SW_SYM, true, true>;
            // MN_SWEEP=3: gram_sweep3.hpp's schedule (PROBE noepi: K loop only)
            if (sweep_gen == 4 && probe && *probe)
                sk = !strcmp(probe, "nodma")    ? ksw2::k_gram_sweep3<4, ksw2::SW_SYM, 2>
                     : !strcmp(probe, "nobar")  ? ksw2::k_gram_sweep3<5, ksw2::SW_SYM, 2>
                     : !strcmp(probe, "noread") ? ksw2::k_gram_sweep3<6, ksw2::SW_SYM, 2>
                                                : ksw2::k_gram_sweep3<1, ksw2::SW_SYM, 2>;
            if (sweep_gen == 5)  // two windows per k-step and group
                sk = (probe && *probe) ? ksw2::k_gram_sweep3<1, ksw2::SW_SYM, 2, 2>
                                       : ksw2::k_gram_sweep3<0, ksw2::SW_SYM, 2, 2>;
            if (sweep_gen == 3)  // DMA three k-steps ahead
                sk = !(probe && *probe)          ? ksw2::k_gram_sweep3<0, ksw2::SW_SYM>
                     : !strcmp(probe, "initonly") ? ksw2::k_gram_sweep3<2, ksw2::SW_SYM>
                     : !strcmp(probe, "prefilter") ? ksw2::k_gram_sweep3<3, ksw2::SW_SYM>
                                                   : ksw2::k_gram_sweep3<1, ksw2::SW_SYM>;
#endif
            hipLaunchKernelGGL(sk, dim3((unsigned)tab.size()), dim3(ksw2::NT), 0, s, XK, nc, XK,
                               nc, nkb, (int64_t)0, (int64_t)0, 1, Up, teffP, Vp, (int64_t)0, 1,
                               (int64_t)0, cap2, cbuf2, cnt2, pst1, sa);
            MN_KCHECK(s, "k_gram_sweep<SYM>");
            S1r = 0;
            tau_r = tauP;   // the certificate: T > D_k (the bound is in the folds)
            dlt_r = zdlt;
            rel_r = (d + 8.0f) * 0x1p-24f;  // keys are lower bounds up to f32 roundings
            perm_r = pi;
            qmap_r = pi;
            chc_r = hcP;
        }
    }
    if (two && !sym) {
        const double expect = (double)L1 * (double)(nc - m0) / (double)m0;
        const ksw2::SweepPlan p2 = ksw2::plan_sweep(nq, nc - m0, expect);
        S2 = (int)p2.S;
        cap2 = p2.cap;
        t_stats.sweep_slices = S2;
        t_stats.sweep_cap = cap2;
        const size_t nbuf2 = (size_t)nq * S2 * cap2;
        cbuf2 = (uint2 *)scratch(kSlotX1Buf2, nbuf2 * sizeof(uint2) + 64);
        cnt2 = (int *)scratch(kSlotX1Meta2, (size_t)nq * S2 * 4 + 64);
        MN_REQUIRE(cbuf2 && cnt2, MN_ENOMEM, "mn_knn: sweep buffer allocation failed (%zu MB)",
                   (nbuf2 * sizeof(uint2)) >> 20);
        const int64_t nqb = (nq + ksw2::BQ - 1) / ksw2::BQ;
        const int64_t grid = nqb * p2.S;
        MN_REQUIRE(grid < INT_MAX && nq * 32 < INT_MAX && nc * 32 < INT_MAX, MN_ENOTSUP,
                   "mn_knn: sweep grid too large (split the queries / corpus)");
        using ksw2::SW_L2;
        auto kern = tmaj ? ksw2::k_gram_sweep2<0, SW_L2, true> : ksw2::k_gram_sweep2<0, SW_L2, false>;
#ifdef MN_TUNING
        // timing probes: noepi = K loop only; nodma / noread = also without the
        // in-loop DMA issue / fragment reads; nowait = DMA never waited for
        if (probe && *probe)
            kern = !strcmp(probe, "nodma") ? ksw2::k_gram_sweep2<2, SW_L2, true>
                   : !strcmp(probe, "noread") ? ksw2::k_gram_sweep2<3, SW_L2, true>
                   : !strcmp(probe, "nowait") ? ksw2::k_gram_sweep2<4, SW_L2, true>
                                              : ksw2::k_gram_sweep2<1, SW_L2, true>;
#endif
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(ksw2::NT), 0, s, QK, nq, CK, nc,
                           nkb, q_off, (int64_t)0, 0, tq, tau0, chc, m0, S2, p2.chunk, cap2,
                           cbuf2, cnt2, pst1, ksw2::SymArgs{});
        MN_KCHECK(s, "k_gram_sweep");
    }
    tm.mark();
    if (probe && *probe) {  // timing probe: outputs are not produced
        MN_HIP_TRY(hipStreamSynchronize(s));
        if (tm.on) {
            const int o = sym_mark;
            t_stats.ms_norms = tm.ms(0, 1) + (o ? tm.ms(2, 3) : 0.f);
            t_stats.ms_sample = tm.ms(1, 2);
            t_stats.ms_sweep = tm.ms(2 + o, 3 + o);
            t_stats.ms_gram = t_stats.ms_sample + t_stats.ms_sweep;
        }
        return MN_OK;
    }

    const int64_t nvalid = std::max<int64_t>(same ? nc - 1 : nc, 0);
    int *big_count = flags + 6;
    int *big_list = fb_list + nq;  // second half of the fallback-list slot
    // pass 1: up to 512 candidates per row, 4 rows per block; pass 2 (the rare
    // rows with more): up to 1024, one row per block
    // MN_X1_DEBUG=1: why rows stay uncertified (stderr), per re-rank pass
    const char *dbe = getenv("MN_X1_DEBUG");
    int *why = (dbe && *dbe == '1') ? flags + 20 : nullptr;  // [20..25]
    if (why) MN_HIP_TRY(hipMemsetAsync(why, 0, 24, s));
    auto why_print = [&](const char *pass) {
        if (!why) return;
        int h[6] = {0};
        if (hipMemcpyAsync(h, why, 24, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return;
        fprintf(stderr,
                "mn_knn x1 %s: uncertified by overflow %d, >1024 candidates %d, forced %d, "
                "no threshold %d, < k candidates %d, bound %d\n",
                pass, h[0], h[1], h[2], h[3], h[4], h[5]);
        (void)hipMemsetAsync(why, 0, 24, s);
    };
    // the re-rank's first-pass margin (k_rerank_x1 m1; tuning build MN_RR_M1, 0 = round 5;
    // 8 measured best, profiles/r06/r06_c2_rerank_m1_scan*.log)
    const int rr_m1 = knob_int("MN_RR_M1", 8);
#define MN_RRX(NRV, WPB, V, NB, QL, QN, BC, BL)                                                 \
    hipLaunchKernelGGL((k_rerank_x1<NRV, WPB, V>), dim3((unsigned)(NB)), dim3(64 * WPB), 0, s, \
                       Q, nq, C, d, c_off, S1r, pl.cap, cbuf1, bcnt1, tau_r, S2, cap2,          \
                       cbuf2, cnt2, dlt_r, k, nvalid, QL, QN, BC, BL, perm_r, q_off, excl,      \
                       qmap_r, ubv, out_idx, out_dist, fb_count, fb_list, rel_r, why, rr_m1)
    const int64_t nb1 = (nq + 3) / 4;
    if (vec4) MN_RRX(8, 4, true, nb1, (const int *)nullptr, (const int *)nullptr, big_count, big_list);
    else MN_RRX(8, 4, false, nb1, (const int *)nullptr, (const int *)nullptr, big_count, big_list);
    MN_KCHECK(s, "k_rerank_x1<8>");
    int nbig = 0;
    MN_HIP_TRY(hipMemcpyAsync(&nbig, big_count, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (nbig > 0) {
        if (vec4) MN_RRX(16, 1, true, nbig, big_list, big_count, (int *)nullptr, (int *)nullptr);
        else MN_RRX(16, 1, false, nbig, big_list, big_count, (int *)nullptr, (int *)nullptr);
    }
#undef MN_RRX
    MN_KCHECK(s, "k_rerank_x1");
    why_print("re-rank");
    tm.mark();
    // statistics of the buffers now: an escalation below reuses (and may
    // reallocate) the scratch slots that hold them
    if (tm.on) {
        if (S1r > 0)
            hipLaunchKernelGGL(k_count_cands, dim3(1024), dim3(256), 0, s, bcnt1, nq * pl.S,
                               pl.cap, ncand);
        if (two)
            hipLaunchKernelGGL(k_count_cands, dim3(1024), dim3(256), 0, s, cnt2, nq * S2, cap2,
                               ncand);
        MN_KCHECK(s, "k_count_cands");
    }
    int64_t hpre[8] = {0};
    MN_HIP_TRY(hipMemcpyAsync(hpre, flags, 64, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    const int nfb = ((const int *)hpre)[5];
    const int64_t n_cand = hpre[4];
    // many uncertified rows: refill them with the bf16x3 sweep (section 2d)
    // instead of the exact scan, whose cost is O(nc d) per row.  No x1 buffer
    // (phase-1 / sweep lists, sample) is read after this point; perm, chc and
    // ubv stay live.
    // tuning build: MN_X1_NOREFILL=1 sends every uncertified row to the exact
    // scan (diagnostics of the refill)
    if (nfb > 256 && !knob_int("MN_X1_NOREFILL", 0)) {
        Timer te;
        te.start(true, s);
        const int nkb3 = 3 * nkb;
        char *eb = (char *)scratch(kSlotX1Esc, (size_t)nfb * 32 + 256);
        // the row-major phase-1 copies are dead: their slots hold the 3 dp copies
        uint16_t *CK3 = (uint16_t *)scratch(kSlotX1CR, (size_t)pad256(nc) * kbw3 * 2 + 64);
        uint16_t *QK3 = (uint16_t *)scratch(kSlotX1QR, (size_t)pad256(nfb) * kbw3 * 2 + 64);
        MN_REQUIRE(eb && CK3 && QK3, MN_ENOMEM, "mn_knn: refill scratch allocation failed");
        int *erows = (int *)eb;
        float *qn3 = (float *)(eb + (((size_t)nfb * 4 + 15) & ~(size_t)15));
        float *qh3 = qn3 + nfb, *ql3 = qh3 + nfb, *q23 = ql3 + nfb, *tq3 = q23 + nfb,
              *tau3 = tq3 + nfb, *dlt3 = tau3 + nfb;
        unsigned *cmax3 = (unsigned *)(flags + 10);  // [10..13]: max |c|^2, |ch|, |cl|, |c2|
        MN_HIP_TRY(hipMemcpyAsync(erows, fb_list, sizeof(int) * (size_t)nfb, hipMemcpyDeviceToDevice, s));
        MN_HIP_TRY(hipMemsetAsync(cmax3, 0, 16, s));
        MN_HIP_TRY(hipMemsetAsync(fb_count, 0, 8, s));  // fb_count, big_count
        auto prep3 = [&](const float *X, int64_t n, const int *src, uint16_t *K, int corpus,
                         float *nv, float *hv, float *lv, float *rv) {
            const int64_t blocks = std::min<int64_t>((n + 7) / 8, 16384);
            if (vec4)
                hipLaunchKernelGGL(k_prep_x3<true>, dim3((unsigned)blocks), dim3(256), 0, s, X, n,
                                   d, dp, src, K, corpus, nv, hv, lv, rv, cmax3, pst3);
            else
                hipLaunchKernelGGL(k_prep_x3<false>, dim3((unsigned)blocks), dim3(256), 0, s, X, n,
                                   d, dp, src, K, corpus, nv, hv, lv, rv, cmax3, pst3);
        };
        prep3(C, nc, perm_r, CK3, 1, nullptr, nullptr, nullptr, nullptr);
        prep3(Q, nfb, erows, QK3, 0, qn3, qh3, ql3, q23);
        MN_KCHECK(s, "k_prep_x3");
        hipLaunchKernelGGL(k_tau_x3, dim3((unsigned)((nfb + 255) / 256)), dim3(256), 0, s,
                           (int64_t)nfb, erows, ubv, qn3, qh3, ql3, q23, cmax3, d, dp, tq3, tau3,
                           dlt3);
        MN_KCHECK(s, "k_tau_x3");
        // expected candidates per row: those below ub + 1.125 delta3, where ub
        // (the first pass's k-th exact distance) can sit up to its delta above
        // D_k: in dense clusters several hundred rows (clustered C2: 8 (k + 16)
        // overflowed 62.7k of 80k refilled rows); 32 (k + 16), the buffer kept
        // within ~16 GB
        const double ex3 = std::min(32.0 * (k + 16), 16e9 / (20.0 * (double)nfb));
        const ksw2::SweepPlan p3 = ksw2::plan_sweep(nfb, nc, std::max(ex3, 8.0 * (k + 16)));
        const size_t nbuf3 = (size_t)nfb * p3.S * p3.cap;
        uint2 *cbuf3 = (uint2 *)scratch(kSlotX1Buf2, nbuf3 * sizeof(uint2) + 64);
        int *cnt3 = (int *)scratch(kSlotX1Meta2, (size_t)nfb * p3.S * 4 + 64);
        MN_REQUIRE(cbuf3 && cnt3, MN_ENOMEM, "mn_knn: refill buffer allocation failed (%zu MB)",
                   (nbuf3 * sizeof(uint2)) >> 20);
        const int64_t grid3 = ((nfb + ksw2::BQ - 1) / ksw2::BQ) * p3.S;
        MN_REQUIRE(grid3 < INT_MAX, MN_ENOTSUP, "mn_knn: refill grid too large");
        hipLaunchKernelGGL((tmaj ? ksw2::k_gram_sweep2<0, ksw2::SW_L2, true>
                                 : ksw2::k_gram_sweep2<0, ksw2::SW_L2, false>),
                           dim3((unsigned)grid3), dim3(ksw2::NT), 0, s, QK3, (int64_t)nfb, CK3,
                           nc, nkb3, (int64_t)0, (int64_t)0, 0, tq3, tau3, chc_r, (int64_t)0,
                           (int)p3.S, p3.chunk, p3.cap, cbuf3, cnt3, pst3, ksw2::SymArgs{});
        MN_KCHECK(s, "k_gram_sweep<x3>");
        int *big_count3 = flags + 6;
        int *big_list3 = fb_list + nq;
#define MN_RR3(NRV, WPB, V, NB, QL, QN, BC, BL)                                                 \
    hipLaunchKernelGGL((k_rerank_x1<NRV, WPB, V>), dim3((unsigned)(NB)), dim3(64 * WPB), 0, s, \
                       Q, (int64_t)nfb, C, d, c_off, 0, 0, (const uint2 *)nullptr,            \
                       (const int *)nullptr, tau3, (int)p3.S, p3.cap, cbuf3, cnt3, dlt3, k,    \
                       nvalid, QL, QN, BC, BL, perm_r, q_off, excl, erows, (float *)nullptr,     \
                       out_idx, out_dist, fb_count, fb_list, 0.f, why, rr_m1)
        const int64_t nb3 = (nfb + 3) / 4;
        if (vec4) MN_RR3(8, 4, true, nb3, (const int *)nullptr, (const int *)nullptr, big_count3, big_list3);
        else MN_RR3(8, 4, false, nb3, (const int *)nullptr, (const int *)nullptr, big_count3, big_list3);
        MN_KCHECK(s, "k_rerank_x1<refill>");
        int nbig3 = 0;
        MN_HIP_TRY(hipMemcpyAsync(&nbig3, big_count3, 4, hipMemcpyDeviceToHost, s));
        MN_HIP_TRY(hipStreamSynchronize(s));
        if (nbig3 > 0) {
            if (vec4) MN_RR3(16, 1, true, nbig3, big_list3, big_count3, (int *)nullptr, (int *)nullptr);
            else MN_RR3(16, 1, false, nbig3, big_list3, big_count3, (int *)nullptr, (int *)nullptr);
            MN_KCHECK(s, "k_rerank_x1<refill, wide>");
        }
#undef MN_RR3
        why_print("bf16x3 refill");
        te.mark();
        t_stats.n_escalated = nfb;
        t_stats.ms_escalate = te.ms(0, 1);
    }
    // rows still uncertified: against a large corpus, gather them and run the
    // split generator (k + 1 neighbours, self included, then the query's own
    // id dropped) — one batched, certified Gram pass instead of an O(nc d)
    // exact scan per row on one CU (15 rows cost 228 ms that way at C2);
    // small corpora keep the exact scan
    int nfb2 = 0;
    MN_HIP_TRY(hipMemcpyAsync(&nfb2, fb_count, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    // a few rows: the split exact scan (every corpus part in parallel, pruned
    // by the rows' exact upper bounds of D_k), ~1 ms per 8 rows at C2
    int split = 1;
    // MN_FB_SPLIT: the row limit of the split scan (default 4096; 0 = always
    // the batched split-generator pass; A/B and tests)
    const char *fse = knob("MN_FB_SPLIT");
    const int fb_lim = (fse && *fse) ? std::max(0, atoi(fse)) : 4096;
    if (nfb2 > 0 && nfb2 <= fb_lim && nc >= (1 << 16)) {
        split = fb_split_scan(Q, C, nc, d, q_off, c_off, excl, k, fb_list, nfb2, ubv, false,
                              out_idx, out_dist, s);
        if (split < 0) return split;
    }
    if (split == MN_OK) {
        // done
    } else if (nfb2 > 0 && nc >= (1 << 16) && k + 1 <= KLIST) {
        // the refill slot is dead here (knn_f32_core below does not use it):
        // rows, the gathered queries and the (k + 1)-lists, 16-B aligned parts
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const size_t b_rows = al(sizeof(int) * (size_t)nfb2), b_q = al(sizeof(float) * (size_t)nfb2 * d),
                     b_l = al(sizeof(int32_t) * (size_t)nfb2 * (k + 1));
        char *gb = (char *)scratch(kSlotX1Esc, b_rows + b_q + 2 * b_l + 256);
        MN_REQUIRE(gb, MN_ENOMEM, "mn_knn: escalation scratch allocation failed");
        int *rows = (int *)gb;
        float *Qg = (float *)(gb + b_rows);
        int32_t *ei = (int32_t *)(gb + b_rows + b_q);
        float *ed = (float *)(gb + b_rows + b_q + b_l);
        MN_HIP_TRY(hipMemcpyAsync(rows, fb_list, sizeof(int) * (size_t)nfb2,
                                  hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)(((int64_t)nfb2 * d + 255) / 256)),
                           dim3(256), 0, s, Q, d, rows, (int64_t)nfb2, Qg);
        MN_KCHECK(s, "k_gather_rows");
        mn_knn_opts o2 = *opts;
        o2.k = k + 1;
        o2.exclude_self = 0;
        o2.metric = MN_L2SQ;
        o2.timing = 0;
        o2.algo = (k + 1 + margin <= kb16::LMAX) ? MN_KNN_BF16X3 : MN_KNN_F32;
        const mn_knn_stats saved = t_stats;
        const int rc = knn_f32_core(Qg, nfb2, C, nc, d, 0, c_off, &o2, ei, ed, o2.algo);
        t_stats = saved;
        if (rc == MN_OK) {
            hipLaunchKernelGGL(k_scatter_escalated, dim3((unsigned)((nfb2 + 255) / 256)),
                               dim3(256), 0, s, rows, (int64_t)nfb2, q_off, excl, k, ei, ed,
                               out_idx, out_dist);
            MN_KCHECK(s, "k_scatter_escalated");
        }
        MN_HIP_TRY(hipStreamSynchronize(s));
        if (rc != MN_OK) return rc;
    } else if (nfb2 > 0) {
        const unsigned fgrid = (unsigned)std::min<int64_t>(nfb2, 1024);
        if (vec4)
            hipLaunchKernelGGL(k_fallback<true>, dim3(fgrid), dim3(FB_THREADS), 0, s, Q, C, nc, d,
                               q_off, c_off, excl, k, fb_count, fb_list, out_idx, out_dist);
        else
            hipLaunchKernelGGL(k_fallback<false>, dim3(fgrid), dim3(FB_THREADS), 0, s, Q, C, nc,
                               d, q_off, c_off, excl, k, fb_count, fb_list, out_idx, out_dist);
        MN_KCHECK(s, "k_fallback");
    }
    tm.mark();
    MN_HIP_TRY(hipStreamSynchronize(s));
    t_stats.n_uncertified = nfb2;
    if (tm.on) {
        t_stats.n_candidates = n_cand;
        const int o = sym_mark;
        t_stats.ms_norms = tm.ms(0, 1) + (o ? tm.ms(2, 3) : 0.f);
        t_stats.ms_sample = tm.ms(1, 2);
        t_stats.ms_sweep = tm.ms(2 + o, 3 + o);
        t_stats.ms_gram = t_stats.ms_sample + t_stats.ms_sweep;
        t_stats.ms_rerank = tm.ms(3 + o, 4 + o);
        t_stats.ms_fallback = tm.ms(4 + o, 5 + o);
        t_stats.ms_total = tm.ms(0, 5 + o);
    }
    return MN_OK;
}

// ---------------------------------------------------------------------------
// 6. row-sharded symmetric sweep (shard.hip): the SW_SYM
// pipeline of knn_x1 over all N rows, its block table dealt over the ranks
// ---------------------------------------------------------------------------
// Stage A (shard_phase1, per rank): tau0 of the rank's own rows from the
// phase-1 generator against the GLOBAL sample (the first m0 rows of the
// golden-ratio order over all N rows), as knn_x1 computes it.
// Stage B (shard_share, per rank, after the tau0 / norm all-gather): every
// rank builds the same per-row bounds, the same Tf order and the same fp16
// copy of all N rows (deterministic kernels and radix sort), sweeps ITS share
// of the order-2 block table (ksw2::sym_block_table_share: every tile on
// exactly one rank) and re-ranks all N rows in partial mode: per row the exact
// top-k of the candidates its tiles admitted (k_rerank_x1, fb_list == NULL).
// Stage C (shard_finish, per owner, after the exchange): merge the parts of
// the owner's rows and certify them with the row's certificate threshold Tc
// (k_merge_certify) — the union of the parts' admitted candidates is exactly
// the single-GPU sweep's, so the certificate is the same; uncertified rows go
// to the split exact scan against all N rows (X_all is resident on every rank).
static_assert(knn::KMAX == kShardKMax, "shard_plan's k limit is the C ABI's");

static void shard_prep(const float *X, int64_t n, int d, int dp, const int *pm, uint16_t *R,
                       float *nv, float *hcv, float *hv, float *rv, unsigned *cmax, int *flags,
                       hipStream_t s, uint16_t *K = nullptr, int tm = 0) {
    if (n == 0) return;
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)X % 16 == 0);
    const int64_t blocks = std::min<int64_t>((n + 7) / 8, 16384);
    if (vec4)
        hipLaunchKernelGGL(knn::k_prep_x1<true>, dim3((unsigned)blocks), dim3(256), 0, s, X, n, d, dp,
                           pm, R, K, nv, hcv, hv, rv, cmax, flags + 3, 1, tm, (unsigned *)nullptr);
    else
        hipLaunchKernelGGL(knn::k_prep_x1<false>, dim3((unsigned)blocks), dim3(256), 0, s, X, n, d,
                           dp, pm, R, K, nv, hcv, hv, rv, cmax, flags + 3, 1, tm, (unsigned *)nullptr);
}

int shard_phase1(const float *X_all, const ShardPlan &pl, int64_t row0, int64_t nl, hipStream_t s,
                 float *tau0_o, float *qn_o) {
    using namespace knn;
    const int64_t N = pl.N, m0 = pl.m0;
    const int d = pl.d, dp = pl.dp;
    uint16_t *QR = (uint16_t *)scratch(kSlotX1QR, (size_t)nl * dp * 2 + 64);
    uint16_t *CR = (uint16_t *)scratch(kSlotX1CR, (size_t)m0 * dp * 2 + 64);
    char *aux = (char *)scratch(kSlotX1Aux, (size_t)nl * 16 + (size_t)m0 * 8 + 256);
    int *flags = (int *)scratch(kSlotFlags, 128);
    int *perm = make_perm(N, kSlotPerm, 0, s);
    MN_REQUIRE(QR && CR && aux && flags && perm, MN_ENOMEM, "shard_phase1: scratch allocation failed");
    float *qhn = (float *)aux, *qrn = qhn + nl, *tq = qrn + nl, *dlt = tq + nl;
    float *cnv = dlt + nl, *chc = cnv + m0;
    unsigned *cmax = (unsigned *)flags;
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 128, s));
    // phase 1 as knn_x1's symmetric path runs it (round 4b: the sweep with a
    // pre-sample threshold, sweep_phase1; tuning build: MN_P1_SWEEP=0 keeps the
    // list generator): tile-major copies of the rows and the sample
    const bool p1s = knob_int("MN_P1_SWEEP", 1) != 0;
    const int nkb = pl.nkb, pst1 = nkb + 1;
    const int64_t kbw1 = (int64_t)pst1 * 32;
    uint16_t *QK = nullptr, *CKs = nullptr;
    int *fbl = nullptr;
    if (p1s) {
        QK = (uint16_t *)scratch(kSlotX1QK, (size_t)((nl + 255) / 256 * 256) * kbw1 * 2 + 64);
        CKs = (uint16_t *)scratch(kSlotGeneric3, (size_t)((m0 + 255) / 256 * 256) * kbw1 * 2 + 64);
        fbl = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nl + 64);
        MN_REQUIRE(QK && CKs && fbl, MN_ENOMEM, "shard_phase1: sweep copy allocation failed");
    }
    // maxima over the rows and the sample (both enter the phase-1 bound)
    shard_prep(X_all + row0 * (int64_t)d, nl, d, dp, nullptr, QR, qn_o, nullptr, qhn, qrn, cmax,
               flags, s, QK, p1s ? pst1 : 0);
    shard_prep(X_all, m0, d, dp, perm, CR, cnv, chc, nullptr, nullptr, cmax, flags, s, CKs,
               p1s ? pst1 : 0);
    MN_KCHECK(s, "k_prep_x1<shard>");
    int hflags[8] = {0};
    MN_HIP_TRY(hipMemcpyAsync(hflags, flags, 32, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hflags[3] == 0, MN_ENONFINITE,
               "mn_knn_sharded: input contains NaN/inf (the reference panics in partial_cmp().unwrap())");
    if (hflags[4] != 0) return 1;  // too large for the bf16 bound: the per-shard path
    if (p1s) {
        float *bt = (float *)scratch(kSlotListMeta, (size_t)nl * 4 + 64);
        MN_REQUIRE(bt, MN_ENOMEM, "shard_phase1: threshold allocation failed");
        const int rc1 = sweep_phase1(QR, QK, nl, CR, CKs, m0, d, dp, nkb, pst1, row0, pl.L1, qn_o, qhn,
                                     qrn, cnv, chc, cmax, tq, tau0_o, dlt, bt, fbl, flags + 20, s);
        if (rc1 != MN_OK) return rc1;
        hipLaunchKernelGGL(k_tau_x1, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, nl, 1, bt,
                           qn_o, qhn, qrn, cmax, d, dp, tq, tau0_o, dlt, (unsigned *)nullptr);
        MN_KCHECK(s, "k_tau_x1<shard>");
        return MN_OK;
    }
    const kb16::GramPlan gp = kb16::plan_gram(nl, m0, pl.L1, 1, 1);
    const size_t nbuf1 = (size_t)nl * gp.S * gp.cap;
    uint2 *cbuf1 = (uint2 *)scratch(kSlotLists, nbuf1 * sizeof(uint2) + 64);
    char *meta1 = (char *)scratch(kSlotListMeta, (size_t)nl * gp.S * 8 + 64);
    MN_REQUIRE(cbuf1 && meta1, MN_ENOMEM, "shard_phase1: phase-1 buffer allocation failed");
    int *bcnt1 = (int *)meta1;
    float *btau1 = (float *)(meta1 + (size_t)nl * gp.S * 4);
    const int64_t bq = (nl + kb16::BM - 1) / kb16::BM;
    hipLaunchKernelGGL((kb16::k_gram_bf16<kb16::GM_L2H, 0>), dim3((unsigned)(bq * gp.S)),
                       dim3(kb16::NT), 0, s, QR, nl, CR, m0, dp, row0, (int64_t)0, 0, qn_o, cnv,
                       pl.L1, (int)gp.S, gp.chunk, gp.cap, cbuf1, bcnt1, btau1);
    MN_KCHECK(s, "k_gram_bf16<L2H, shard>");
    hipLaunchKernelGGL(k_tau_x1, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, nl,
                       (int)gp.S, btau1, qn_o, qhn, qrn, cmax, d, dp, tq, tau0_o, dlt,
                       (unsigned *)nullptr);
    MN_KCHECK(s, "k_tau_x1<shard>");
    return MN_OK;
}

__global__ __launch_bounds__(256) void k_flag_nonfinite(const float *__restrict__ v, int64_t n,
                                                        int *__restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool bad = i < n && !__builtin_isfinite(v[i]);
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

int shard_share(const float *X_all, const ShardPlan &pl, const float *tau0_all,
                const float *qn_all, int rank, int world, hipStream_t s, int32_t *pidx,
                float *pdist, float *tc_all, int64_t *n_cand) {
    using namespace knn;
    const int64_t N = pl.N;
    const int d = pl.d, dp = pl.dp, nkb = pl.nkb, k = pl.k;
    const size_t nn = (size_t)N;
    const int pst1 = nkb + 1;  // tile-major panel stride (knn_x1's TM_PAD 1)
    const int64_t kbw1 = (int64_t)pst1 * 32;
    const int64_t npad = (N + 255) / 256 * 256;
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)X_all % 16 == 0);
    int *flags = (int *)scratch(kSlotFlags, 128);
    char *so = (char *)scratch(kSlotSymOrd, nn * 4 * 17 + 8192);
    uint16_t *XK = (uint16_t *)scratch(kSlotX1CK, (size_t)npad * kbw1 * 2 + 64);
    int *big_list = (int *)scratch(kSlotFallback, sizeof(int) * nn + 64);
    MN_REQUIRE(flags && so && XK && big_list, MN_ENOMEM, "shard_share: scratch allocation failed");
    auto arr = [&](int i) { return so + (size_t)i * (((nn * 4) + 255) & ~(size_t)255); };
    float *skey = (float *)arr(0);
    int *pi = (int *)arr(1), *iota = (int *)arr(2);
    float *tauP = (float *)arr(3), *teffP = (float *)arr(4), *hcP = (float *)arr(5),
          *Up = (float *)arr(6), *Vp = (float *)arr(7), *zdlt = (float *)arr(8),
          *scP = (float *)arr(9), *h16 = (float *)arr(10), *r16 = (float *)arr(11),
          *s16 = (float *)arr(12), *alr = (float *)arr(13), *tfr = (float *)arr(14);
    const unsigned g256 = (unsigned)((N + 255) / 256);
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 128, s));
    // a non-finite threshold would break the column fold: the per-shard path
    hipLaunchKernelGGL(k_flag_nonfinite, dim3(g256), dim3(256), 0, s, tau0_all, N, flags);
    MN_KCHECK(s, "k_flag_nonfinite");
    int hbad = 0;
    MN_HIP_TRY(hipMemcpyAsync(&hbad, flags, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (hbad) return 1;
    const int64_t blocks = std::min<int64_t>((N + 7) / 8, 16384);
    auto f16r = [&](const int *pm, uint16_t *K, float *hv, float *rv, float *sv) {
        if (vec4)
            hipLaunchKernelGGL(k_prep_f16r<true>, dim3((unsigned)blocks), dim3(256), 0, s, X_all, N,
                               d, dp, pm, K, hv, rv, sv, pst1);
        else
            hipLaunchKernelGGL(k_prep_f16r<false>, dim3((unsigned)blocks), dim3(256), 0, s, X_all,
                               N, d, dp, pm, K, hv, rv, sv, pst1);
    };
    f16r(nullptr, nullptr, h16, r16, s16);
    MN_KCHECK(s, "k_prep_f16r<stats, shard>");
    hipLaunchKernelGGL(k_sym_row, dim3(g256), dim3(256), 0, s, N, tau0_all, qn_all, h16, r16, d,
                       dp, alr, tfr, tc_all);
    MN_KCHECK(s, "k_sym_row<shard>");
    hipLaunchKernelGGL(k_iota, dim3(g256), dim3(256), 0, s, iota, N);
    MN_HIP_TRY(sort_f32_pairs(tfr, skey, iota, pi, N, s));
    f16r(pi, XK, nullptr, nullptr, nullptr);
    MN_KCHECK(s, "k_prep_f16r<shard>");
    hipLaunchKernelGGL(k_sym_pos, dim3(g256), dim3(256), 0, s, N, pi, qn_all, alr, tfr, tc_all,
                       s16, tauP, teffP, Up, Vp, hcP, scP);
    MN_HIP_TRY(hipMemsetAsync(zdlt, 0, nn * 4, s));
    MN_KCHECK(s, "k_sym_pos<shard>");
    const int nbk = (int)((N + ksw2::BC - 1) / ksw2::BC);
    int4 *dtab = nullptr;
    // groups of 8 row blocks x 4 column phases (round 6: largest share 6.23-6.25
    // vs 6.39-6.52 s for 4 x 8 over the 8M C4 in one process, 2 x 16 slower;
    // profiles/r06/r06_c4_gr*_ab.log)
    const std::vector<int4> &tab = ksw2::sym_table_device(nbk, 256, 2, ksw2::kShareGR, rank, world, s, &dtab);
    MN_REQUIRE(dtab, MN_ENOMEM, "shard_share: block table allocation / upload failed");
    MN_REQUIRE(tab.size() < INT_MAX, MN_ENOTSUP, "shard_share: sweep grid too large");
    // per-row buffers: a share holds ~1/world of the ~L1 N / m0 candidates of
    // a row on average, but unevenly (a row's candidates in one column range
    // go to one rank): a 256-entry cap overflowed 0.9% of the rows at C2 with
    // 8 ranks (profiles/r04/r04_shard_probe.log), the single-GPU cap none
    const double expect = (double)pl.L1 * (double)N / (double)pl.m0;
    const char *cpe = knob("MN_SH_CAP");  // tuning build: per-row buffer entries
    const int cap2 = (cpe && *cpe) ? std::max(64, atoi(cpe))
                                   : std::max(256, (int)((2.5 * expect + 64.0 + 15.0) / 16.0) * 16);
    uint2 *cbuf2 = (uint2 *)scratch(kSlotX1Buf2, nn * cap2 * sizeof(uint2) + 64);
    int *cnt2 = (int *)scratch(kSlotX1Meta2, nn * 4 + 64);
    MN_REQUIRE(cbuf2 && cnt2, MN_ENOMEM, "shard_share: sweep buffer allocation failed (%zu MB)",
               (nn * cap2 * sizeof(uint2)) >> 20);
    MN_HIP_TRY(hipMemsetAsync(cnt2, 0, nn * 4, s));
    if (!tab.empty()) {
        ksw2::SymArgs sa{dtab, Vp, Up, scP};
        auto sk = ksw2::k_gram_sweep3<0, ksw2::SW_SYM, 2>;
        if (knob_int("MN_SWEEP", 4) == 2) sk = ksw2::k_gram_sweep2<0, ksw2::SW_SYM, true, true>;
        hipLaunchKernelGGL(sk, dim3((unsigned)tab.size()), dim3(ksw2::NT), 0, s, XK, N, XK, N, nkb,
                           (int64_t)0, (int64_t)0, 1, Up, teffP, Vp, (int64_t)0, 1, (int64_t)0, cap2,
                           cbuf2, cnt2, pst1, sa);
        MN_KCHECK(s, "k_gram_sweep3<SYM, shard>");
    }
    // partial re-rank of every row: 128 candidates a wave first, the rows with
    // more (up to 1024) in a second launch
    int *big_count = flags + 6;
    const float rel = (d + 8.0f) * 0x1p-24f;
    const int64_t nvalid = N - 1;
    const int rr_m1 = knob_int("MN_RR_M1", 8);  // the re-rank's first-pass margin
#define MN_RRS(NRV, WPB, V, NB, QL, QN, BCN, BL)                                                  \
    hipLaunchKernelGGL((k_rerank_x1<NRV, WPB, V>), dim3((unsigned)(NB)), dim3(64 * WPB), 0, s,   \
                       X_all, N, X_all, d, (int64_t)0, 0, 0, (const uint2 *)nullptr,              \
                       (const int *)nullptr, tauP, 1, cap2, cbuf2, cnt2, zdlt, k, nvalid, QL, QN, \
                       BCN, BL, pi, (int64_t)0, 1, pi, (float *)nullptr, pidx, pdist,             \
                       (int *)nullptr, (int *)nullptr, rel, (int *)nullptr, rr_m1)
    const int64_t nb1 = (N + 3) / 4;
    if (vec4) MN_RRS(2, 4, true, nb1, (const int *)nullptr, (const int *)nullptr, big_count, big_list);
    else MN_RRS(2, 4, false, nb1, (const int *)nullptr, (const int *)nullptr, big_count, big_list);
    MN_KCHECK(s, "k_rerank_x1<partial>");
    int nbig = 0;
    MN_HIP_TRY(hipMemcpyAsync(&nbig, big_count, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (nbig > 0) {
        if (vec4) MN_RRS(16, 1, true, nbig, big_list, big_count, (int *)nullptr, (int *)nullptr);
        else MN_RRS(16, 1, false, nbig, big_list, big_count, (int *)nullptr, (int *)nullptr);
        MN_KCHECK(s, "k_rerank_x1<partial, wide>");
    }
#undef MN_RRS
    if (n_cand) {
        unsigned long long *nc64 = (unsigned long long *)(flags + 8);
        MN_HIP_TRY(hipMemsetAsync(nc64, 0, 8, s));
        hipLaunchKernelGGL(k_count_cands, dim3(1024), dim3(256), 0, s, cnt2, N, cap2, nc64);
        MN_KCHECK(s, "k_count_cands<shard>");
        unsigned long long h = 0;
        MN_HIP_TRY(hipMemcpyAsync(&h, nc64, 8, hipMemcpyDeviceToHost, s));
        MN_HIP_TRY(hipStreamSynchronize(s));
        *n_cand = (int64_t)h;
    }
    return MN_OK;
}

// One thread per owned row: merge the parts' exact lists (each (dist, id)
// ordered; part p row q at p * pstride + q * k) and certify the merged top-k
// with the row's certificate Tc > D_k.  A part's idx -2 in slot 0 (a forced
// row) or fewer than kneed entries leave the row uncertified: ub = the merged
// k-th exact distance (an upper bound of D_k) and the row listed.
__global__ __launch_bounds__(256) void k_merge_certify(
    const int32_t *__restrict__ pidx, const float *__restrict__ pdist, int P, int64_t pstride,
    int64_t nl, int k, int kneed, const float *__restrict__ tc, int32_t *__restrict__ out_idx,
    float *__restrict__ out_dist, float *__restrict__ ub, int *__restrict__ fb_count,
    int *__restrict__ fb_list, int *__restrict__ why) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nl) return;
    int head[knn::MAX_PARTS];
    bool forced = false;
#pragma unroll
    for (int p = 0; p < knn::MAX_PARTS; ++p) {
        head[p] = 0;
        if (p < P && pidx[p * pstride + q * k] == -2) forced = true;
    }
    int m = 0;
    float Dk = __builtin_inff();
    for (int r = 0; r < k; ++r) {
        int bp = -1;
        float bd = __builtin_inff();
        int bi = INT_MAX;
#pragma unroll
        for (int p = 0; p < knn::MAX_PARTS; ++p) {
            if (p >= P) break;
            const int h = head[p];
            if (h >= k) continue;
            const int64_t off = p * pstride + q * k + h;
            const int ci = pidx[off];
            if (ci < 0) continue;
            const float cd = pdist[off];
            if (bp < 0 || key_less(cd, ci, bd, bi)) { bp = p; bd = cd; bi = ci; }
        }
#pragma unroll
        for (int p = 0; p < knn::MAX_PARTS; ++p)
            if (p == bp) head[p]++;
        out_idx[q * k + r] = bp < 0 ? -1 : bi;
        out_dist[q * k + r] = bp < 0 ? __builtin_inff() : bd;
        if (bp >= 0) {
            ++m;
            if (r == kneed - 1) Dk = bd;
        }
    }
    bool cert = !forced && m >= kneed;
    if (cert && kneed > 0) cert = tc[q] > Dk;  // NaN-safe: false => exact scan
    if (!cert) {
        ub[q] = (m >= kneed && kneed > 0) ? Dk : __builtin_inff();
        fb_list[atomicAdd(fb_count, 1)] = (int)q;
        if (why) atomicAdd(&why[forced ? 0 : m < kneed ? 1 : 2], 1);
    }
}

int shard_finish(const float *X_all, const ShardPlan &pl, int64_t row0, int64_t nl, int parts,
                 int64_t part_stride, const int32_t *pidx, const float *pdist, const float *tc_all,
                 hipStream_t s, int32_t *out_idx, float *out_dist, int *n_fallback) {
    using namespace knn;
    const int64_t N = pl.N;
    const int d = pl.d, k = pl.k;
    int *flags = (int *)scratch(kSlotFlags, 128);
    char *fb = (char *)scratch(kSlotFallback, sizeof(int) * (size_t)nl * 2 + 256);
    MN_REQUIRE(flags && fb, MN_ENOMEM, "shard_finish: scratch allocation failed");
    int *fb_list = (int *)fb;
    float *ub = (float *)(fb + (((size_t)nl * 4 + 255) & ~(size_t)255));
    int *fb_count = flags + 5;
    MN_HIP_TRY(hipMemsetAsync(fb_count, 0, 4, s));
    const int kneed = (int)std::min<int64_t>(k, N - 1);
    // MN_X1_DEBUG=1: why rows stay uncertified (stderr)
    const char *dbe = getenv("MN_X1_DEBUG");
    int *why = (dbe && *dbe == '1') ? flags + 20 : nullptr;
    if (why) MN_HIP_TRY(hipMemsetAsync(why, 0, 12, s));
    hipLaunchKernelGGL(k_merge_certify, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, pidx,
                       pdist, parts, part_stride, nl, k, kneed, tc_all + row0, out_idx, out_dist, ub,
                       fb_count, fb_list, why);
    MN_KCHECK(s, "k_merge_certify");
    int nfb = 0;
    MN_HIP_TRY(hipMemcpyAsync(&nfb, fb_count, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (why) {
        int h[3] = {0};
        MN_HIP_TRY(hipMemcpy(h, why, 12, hipMemcpyDeviceToHost));
        fprintf(stderr, "mn_knn sharded rows %lld..: uncertified forced %d, < k %d, bound %d\n",
                (long long)row0, h[0], h[1], h[2]);
    }
    if (n_fallback) *n_fallback = nfb;
    if (nfb == 0) return MN_OK;
    const float *Q = X_all + row0 * (int64_t)d;
    int rc = fb_split_scan(Q, X_all, N, d, row0, 0, 1, k, fb_list, nfb, ub, false, out_idx,
                           out_dist, s);
    if (rc < 0) return rc;
    if (rc == 1) {  // outside the split scan's limits: the exact scan per row
        const bool vec4 = (d % 4 == 0) && ((uintptr_t)X_all % 16 == 0);
        const unsigned fgrid = (unsigned)std::min<int64_t>(nfb, 1024);
        if (vec4)
            hipLaunchKernelGGL(k_fallback<true>, dim3(fgrid), dim3(FB_THREADS), 0, s, Q, X_all, N, d,
                               row0, (int64_t)0, 1, k, fb_count, fb_list, out_idx, out_dist);
        else
            hipLaunchKernelGGL(k_fallback<false>, dim3(fgrid), dim3(FB_THREADS), 0, s, Q, X_all, N,
                               d, row0, (int64_t)0, 1, k, fb_count, fb_list, out_idx, out_dist);
        MN_KCHECK(s, "k_fallback<shard>");
    }
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

// Host entry shared by mn_knn_f32 and mn_knn_f32_qc: argument checks, the
// generator choice, and the Euclidean (MN_L2) root.
static int knn_f32_impl(const float *Q, int64_t nq, const float *C, int64_t nc, int32_t d,
                        int64_t q_off, int64_t c_off, const mn_knn_opts *opts,
                        int32_t *out_idx, float *out_dist) {
    using namespace knn;
    clear_error();
    t_stats = mn_knn_stats{};
    MN_REQUIRE(opts, MN_EINVAL, "mn_knn: opts is NULL");
    MN_REQUIRE(Q && C && out_idx && out_dist, MN_EINVAL, "mn_knn: NULL pointer argument");
    MN_REQUIRE(nq >= 0 && nc >= 0 && d >= 1, MN_EINVAL, "mn_knn: bad shape nq=%lld nc=%lld d=%d",
               (long long)nq, (long long)nc, d);
    MN_REQUIRE(opts->metric == MN_L2SQ || opts->metric == MN_L2, MN_ENOTSUP,
               "mn_knn_f32: metric %d not supported here", opts->metric);
    const int k = opts->k;
    MN_REQUIRE(k >= 1 && k <= KBIG, MN_ENOTSUP, "mn_knn: k=%d outside [1,%d]", k, KBIG);
    const int algo = opts->algo;
    MN_REQUIRE(algo >= MN_KNN_AUTO && algo <= MN_KNN_BF16X1, MN_EINVAL, "mn_knn: bad algo %d",
               algo);
    MN_REQUIRE(q_off >= 0 && c_off >= 0 && q_off + nq <= INT_MAX && c_off + nc <= INT_MAX,
               MN_EINVAL, "mn_knn: global ids must fit int32");
    t_stats.n_queries = nq;
    if (k > KMAX) {
        // k beyond the candidate generators' lists (mst.rs:317 takes any k):
        // every row through the exact split scan — every corpus part's best k
        // by the reference fold (rooted for MN_L2), merged by (dist, id)
        t_stats.algo = MN_KNN_F32;
        if (nq == 0) return MN_OK;
        hipStream_t s = (hipStream_t)opts->stream;
        int *rows = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nq + 64);
        MN_REQUIRE(rows, MN_ENOMEM, "mn_knn: row list allocation failed");
        hipLaunchKernelGGL(k_iota, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, rows, nq);
        MN_KCHECK(s, "k_iota");
        const int excl = opts->exclude_self ? 1 : 0;
        const int rc = nc > 0 ? fb_split_scan(Q, C, nc, d, q_off, c_off, excl, k, rows, (int)nq,
                                              nullptr, opts->metric == MN_L2, out_idx, out_dist, s)
                              : 1;
        if (rc < 0) return rc;
        if (rc == 1) {
            MN_REQUIRE(nc == 0, MN_ENOTSUP, "mn_knn: k=%d > %d needs d <= %d", k, KMAX,
                       (int)((160 * 1024 - FSQ * FSC * 4 - FSC * 8 - 16) / (FSQ * 4)));
            hipLaunchKernelGGL(k_fill_empty, dim3((unsigned)((nq * k + 255) / 256)), dim3(256), 0, s,
                               out_idx, out_dist, nq * (int64_t)k);
            MN_KCHECK(s, "k_fill_empty");
        }
        MN_HIP_TRY(hipStreamSynchronize(s));
        return MN_OK;
    }
    // MN_L2: the L2^2 graph k2 = k + 8 long, then k_l2_order (root order)
    const bool l2 = opts->metric == MN_L2 && nq > 0;
    const int k2 = l2 ? k + 8 : k;  // <= KLIST
    mn_knn_opts o2 = *opts;
    o2.k = k2;
    o2.metric = MN_L2SQ;
    int32_t *ri = out_idx;
    float *rd = out_dist;
    if (l2) {
        char *t = (char *)scratch(kSlotL2List, (size_t)nq * k2 * 8 + 256);
        MN_REQUIRE(t, MN_ENOMEM, "mn_knn: MN_L2 list allocation failed");
        ri = (int32_t *)t;
        rd = (float *)(t + (((size_t)nq * k2 * 4 + 255) & ~(size_t)255));
    }
    int rc = 1;
    const bool x1 = algo == MN_KNN_BF16X1 || (algo == MN_KNN_AUTO && nc >= (1 << 17));
    if (x1 && nq > 0 && nc > 0) {
        rc = knn_x1(Q, nq, C, nc, d, q_off, c_off, &o2, ri, rd);
        if (rc < 0) return rc;
    }
    if (rc == 1) {
        int a = algo == MN_KNN_BF16X1 ? MN_KNN_AUTO : algo;
        if (a == MN_KNN_AUTO) {
            const int margin = opts->margin > 0 ? opts->margin : 16;
            a = (k2 + margin <= kb16::LMAX) ? MN_KNN_BF16X3 : MN_KNN_F32;
        }
        rc = knn_f32_core(Q, nq, C, nc, d, q_off, c_off, &o2, ri, rd, a);
        if (rc != MN_OK) return rc;
    }
    if (l2) {
        hipStream_t s = (hipStream_t)opts->stream;
        int *fl = (int *)scratch(kSlotFlags, 64);
        int *fbl = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nq * 2 + 64);
        MN_REQUIRE(fl && fbl, MN_ENOMEM, "mn_knn: MN_L2 scratch allocation failed");
        const int excl = opts->exclude_self ? 1 : 0;
        MN_HIP_TRY(hipMemsetAsync(fl, 0, 4, s));
        hipLaunchKernelGGL(k_l2_order, dim3((unsigned)((nq * 64 + 255) / 256)), dim3(256), 0, s,
                           ri, rd, nq, k2, k, nc, q_off, c_off, excl, out_idx, out_dist, fl, fbl);
        MN_KCHECK(s, "k_l2_order");
        int nfb = 0;
        MN_HIP_TRY(hipMemcpyAsync(&nfb, fl, 4, hipMemcpyDeviceToHost, s));
        MN_HIP_TRY(hipStreamSynchronize(s));
        int split = 1;
        if (nfb > 0 && nfb <= 256 && nc >= (1 << 16)) {
            split = fb_split_scan(Q, C, nc, d, q_off, c_off, excl, k, fbl, nfb, nullptr, true,
                                  out_idx, out_dist, s);
            if (split < 0) return split;
            MN_HIP_TRY(hipStreamSynchronize(s));
        }
        if (nfb > 0 && split != MN_OK) {
            const bool vec4 = (d % 4 == 0) && (((uintptr_t)Q | (uintptr_t)C) % 16 == 0);
            const unsigned fgrid = (unsigned)std::min<int64_t>(nfb, 1024);
            if (vec4)
                hipLaunchKernelGGL((k_fallback<true, true>), dim3(fgrid), dim3(FB_THREADS), 0, s,
                                   Q, C, nc, d, q_off, c_off, excl, k, fl, fbl, out_idx, out_dist);
            else
                hipLaunchKernelGGL((k_fallback<false, true>), dim3(fgrid), dim3(FB_THREADS), 0, s,
                                   Q, C, nc, d, q_off, c_off, excl, k, fl, fbl, out_idx, out_dist);
            MN_KCHECK(s, "k_fallback<sqrt>");
            MN_HIP_TRY(hipStreamSynchronize(s));
        }
        t_stats.n_root_rescan = nfb;  // rows rescanned for the root order
    }
    return MN_OK;
}

}  // namespace mn

extern "C" {

int mn_knn_f32(const float *X, int64_t n, int32_t d, const mn_knn_opts *opts, int32_t *out_idx,
               float *out_dist) {
    return mn::knn_f32_impl(X, n, X, n, d, 0, 0, opts, out_idx, out_dist);
}

int mn_knn_f32_qc(const float *Q, int64_t nq, const float *C, int64_t nc, int32_t d,
                  int64_t q_offset, int64_t c_offset, const mn_knn_opts *opts, int32_t *out_idx,
                  float *out_dist) {
    return mn::knn_f32_impl(Q, nq, C, nc, d, q_offset, c_offset, opts, out_idx, out_dist);
}

int mn_knn_merge_f32(const int32_t *part_idx, const float *part_dist, int32_t parts, int64_t nq,
                     int32_t k, int32_t *out_idx, float *out_dist, void *stream) {
    mn::clear_error();
    MN_REQUIRE(part_idx && part_dist && out_idx && out_dist, MN_EINVAL,
               "mn_knn_merge_f32: NULL pointer");
    MN_REQUIRE(parts >= 1 && parts <= mn::knn::MAX_PARTS && nq >= 0 && k >= 1, MN_EINVAL,
               "mn_knn_merge_f32: bad args parts=%d k=%d", parts, k);
    if (nq == 0) return MN_OK;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mn::knn::k_merge_parts, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0,
                       s, part_idx, part_dist, parts, nq, k, out_idx, out_dist);
    MN_HIP_TRY(hipGetLastError());
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

int mn_knn_last_stats(mn_knn_stats *out) {
    if (!out) return MN_EINVAL;
    *out = mn::t_stats;
    return MN_OK;
}

}  // extern "C"
