// knn_bf16.hip — K1 (C5): rectified-cosine kNN over bf16 item rows, bit-exact
// vs the reference's f64 arithmetic on the exactly-widened bf16 values.
//
// Reference semantics (src_legacy/tests/test_helpers.rs:77-126; production
// _build_adjacency src_legacy/laplacian.rs:245-290 uses the same distance and
// weight): norm_i = sqrt(sum x^2) (sequential f64), dot = sequential f64 sum,
// cos = norm_i*norm_j > 1e-12 ? clamp(dot/(norm_i*norm_j), -1, 1) : 0,
// dist = 1 - max(cos, 0), keep dist <= eps and w = 1/(1+(dist/sigma)^p) > 1e-12,
// order (dist asc, j asc), truncate topk.
//
// MI355X design (bf16 MFMA roofline: 2.5 PFLOP/s dense):
//   k_bf16_norms   exact sequential f64 norms, one lane per row (16-B loads).
//   k_gram_bf16    a block owns 256 queries (8 waves x 32 rows) and sweeps its
//                  corpus slice in 256-row tiles: the 256x256xd Gram on
//                  v_mfma_f32_32x32x16_bf16 (bf16 products exact in f32, f32
//                  accumulate), operands staged through LDS (BK = 32, rows
//                  padded to 80 B: conflict-free ds_read_b128, loads issued two
//                  stages ahead).  Epilogue key = -cos~ = -dot/(n_q n_c) vs the
//                  row's threshold (L-th best key); survivors -> LDS queue ->
//                  wave-wide bitonic merge into the row's top-L list.
//   k_cos_rerank   one wave per query: the reference's sequential f64 dot for
//                  every candidate, sort by (dist, idx), certify with
//                  |cos~ - cos| <= 2(d+12)2^-24 (f32 accumulation of exact
//                  products + two f32 scalings), eps/weight filter (a prefix).
//   k_cos_fallback exact scan for uncertified rows (ties at dist 1, overflow).
//
// Two-phase generator (the default for self graphs at scale, C5): the corpus
// is visited in a golden-ratio order (pos p holds row perm(p)) whose prefix of
// m0 = n/16 rows is the sample.
//   phase 1   k_gram_bf16<GM_COS> of every query against the sample, list
//             length L1: t(q) = -(min over slices of the L1-th best key), the
//             cosine of about the (16 L1)-th neighbour.
//   phase 2   gram_sweep2.hpp SW_COS over positions [m0, n) in KB32 layout:
//             acc = q.c - t |q||c| > 0 buffers the pair (no per-row lists, one
//             compare per product: the same epilogue as the L2 sweep).
//   k_cos_rerank_x1  both buffers -> exact f64 distances, (dist, j) order,
//             certification: every pair never buffered has cos~ <= t, so its
//             exact cos is <= t + delta and its distance >= 1 - max(t+delta, 0).
#include <algorithm>
#include <cmath>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "glibc_f64.hpp"
#include "gram_bf16.hpp"
#include "gram_sweep2.hpp"
#include "gram_sweep3.hpp"

namespace mn {
namespace kb16 {


__device__ __forceinline__ double bf2d(uint16_t b) {
    return (double)__uint_as_float((uint32_t)b << 16);
}

// ---- zero-padded copy (d % 8 != 0 or unaligned input): exact, zeros add +0 ----
__global__ __launch_bounds__(256) void k_pad_rows(const uint16_t *__restrict__ X, int64_t n, int d,
                                                  int d8, uint16_t *__restrict__ Y) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * d8) return;
    const int64_t i = e / d8;
    const int c = (int)(e - i * d8);
    Y[e] = c < d ? X[i * d + c] : (uint16_t)0;
}

// ---- exact sequential norms (reference order) ------------------------------
__global__ __launch_bounds__(256) void k_bf16_norms(const uint16_t *__restrict__ X, int64_t n,
                                                    int d, double *__restrict__ nrm,
                                                    float *__restrict__ inv,
                                                    int *__restrict__ nonfinite) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint16_t *p = X + i * (int64_t)d;
    double acc = -0.0;
    bool bad = false;
    int t = 0;
    if ((d & 7) == 0) {
        for (; t < d; t += 8) {
            const uint4 v = *reinterpret_cast<const uint4 *>(p + t);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double a = bf2d((uint16_t)(w[u] & 0xFFFFu));
                const double b = bf2d((uint16_t)(w[u] >> 16));
                bad |= !isfinite(a) || !isfinite(b);
                acc = __builtin_fma(a, a, acc);  // exact square: same rounding as acc + a*a
                acc = __builtin_fma(b, b, acc);
            }
        }
    } else {
        for (; t < d; ++t) {
            const double a = bf2d(p[t]);
            bad |= !isfinite(a);
            acc = __builtin_fma(a, a, acc);
        }
    }
    const double nv = __builtin_sqrt(acc);
    nrm[i] = nv;
    inv[i] = nv > 0.0 ? (float)(1.0 / nv) : 0.f;
    if (bad) atomicOr(nonfinite, 1);
}


// ---- exact re-rank / certification / filter --------------------------------------
// The reference's `acc + a * b` in f64: a bf16 x bf16 product is exact in f64
// (8 + 8 significant bits), so one fused multiply-add rounds identically.
__device__ __forceinline__ double exact_dot(const uint16_t *__restrict__ a,
                                            const uint16_t *__restrict__ b, int d) {
    double acc = -0.0;
    if ((d & 7) == 0) {
        auto fold8 = [&](const uint4 va, const uint4 vb) {
            const uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = __builtin_fma(bf2d((uint16_t)(wa[u] & 0xFFFFu)),
                                    bf2d((uint16_t)(wb[u] & 0xFFFFu)), acc);
                acc = __builtin_fma(bf2d((uint16_t)(wa[u] >> 16)), bf2d((uint16_t)(wb[u] >> 16)),
                                    acc);
            }
        };
        int t = 0;
        // 4 16-B pieces of the (random) candidate row in flight per lane ahead
        // of the ordered FMAs (one at a time, each waits on its gather)
        for (; t + 32 <= d; t += 32) {
            uint4 va[4], vb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) vb[u] = *reinterpret_cast<const uint4 *>(b + t + 8 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u) va[u] = *reinterpret_cast<const uint4 *>(a + t + 8 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u) fold8(va[u], vb[u]);
        }
        for (; t < d; t += 8)
            fold8(*reinterpret_cast<const uint4 *>(a + t), *reinterpret_cast<const uint4 *>(b + t));
    } else {
        for (int t = 0; t < d; ++t) acc = __builtin_fma(bf2d(a[t]), bf2d(b[t]), acc);
    }
    return acc;
}

__device__ __forceinline__ double cos_dist(double dot, double ni, double nj) {
    const double denom = ni * nj;
    double cs = 0.0;
    if (denom > 1e-12) {
        cs = dot / denom;
        cs = cs < -1.0 ? -1.0 : (cs > 1.0 ? 1.0 : cs);
    }
    return 1.0 - (cs > 0.0 ? cs : 0.0);
}

__device__ __forceinline__ double weight_of(double d, double sigma, double p) {
    const double x = d / sigma;
    const double pw = glibc::pow_glibc(x, p);  // glibc pow (glibc_f64.hpp), every p
    return 1.0 / (1.0 + pw);
}

template <int NR>
__global__ __launch_bounds__(256) void k_cos_rerank(
    const uint16_t *__restrict__ Q, int64_t nq, const uint16_t *__restrict__ C, int d,
    int64_t c_off, const double *__restrict__ qn, const double *__restrict__ cn, int S, int cap,
    const uint2 *__restrict__ buf, const int *__restrict__ bcnt, const float *__restrict__ btau,
    int topk, int64_t nvalid_max, double delta, double eps, double sigma, double p,
    int32_t *__restrict__ out_idx, double *__restrict__ out_dist, double *__restrict__ out_w,
    int *__restrict__ fb_count, int *__restrict__ fb_list) {
    __shared__ int cand[4][64 * NR];
    __shared__ float candk[4][64 * NR];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t q = (int64_t)blockIdx.x * 4 + wid;
    if (q >= nq) return;
    // candidates: every buffered pair of slice s whose key <= tau_s (all of
    // them when the slice never filled its L keys); non-candidates of a full
    // slice have key >= tau_s, so T = min_s tau_s bounds them
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
            const bool pass = e < cnt && __uint_as_float(v.x) <= ts;
            const uint64_t pm = __ballot(pass);
            const int pos = M + (int)__popcll(pm & ((1ull << lane) - 1ull));
            if (pass && pos < 64 * NR) {
                cand[wid][pos] = (int)v.y;
                candk[wid][pos] = __uint_as_float(v.x);
            }
            M += (int)__popcll(pm);
        }
    }
    forced |= M > 64 * NR;
    M = min(M, 64 * NR);
    __builtin_amdgcn_wave_barrier();
    // candidates in approximate order (key, id)
    float kk[NR];
    int ix[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        kk[r] = e < M ? candk[wid][e] : __builtin_inff();
        ix[r] = e < M ? cand[wid][e] : INT_MAX;
    }
    wave_bitonic_sort<NR>(kk, ix);
    // exact distances, pruned: the kq best by key first; their largest exact
    // distance Dp bounds the k-th.  A candidate with key kappa has exact
    // distance >= 1 - max(-kappa + delta, 0) (|cos~ - cos| <= delta); above
    // Dp it cannot reach the top k and is skipped (its distance stays +inf,
    // strictly beyond D_k, so the certification below is unaffected).
    const uint16_t *qrow = Q + q * (int64_t)d;
    const int kq = min(topk, M);
    double dd[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        dd[r] = __builtin_inf();
        if (e < kq) {
            const int64_t c = (int64_t)ix[r] - c_off;
            dd[r] = cos_dist(exact_dot(qrow, C + c * d, d), qn[q], cn[c]);
        }
    }
    double Dp = -__builtin_inf();
#pragma unroll
    for (int r = 0; r < NR; ++r) Dp = fmax(Dp, (lane + 64 * r) < kq ? dd[r] : -__builtin_inf());
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) Dp = fmax(Dp, __shfl_xor(Dp, o));
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        if (e >= kq && e < M) {
            const double cub = -(double)kk[r] + delta;
            const double lb = 1.0 - (cub > 0.0 ? cub : 0.0);
            if (lb <= Dp) {
                const int64_t c = (int64_t)ix[r] - c_off;
                dd[r] = cos_dist(exact_dot(qrow, C + c * d, d), qn[q], cn[c]);
            }
        }
    }
    wave_bitonic_sort<NR>(dd, ix);
    const int keff = (int)min((int64_t)min(topk, M), nvalid_max);
    bool cert = !forced;
    if (cert && T < __builtin_inff() && keff > 0) {
        // every non-candidate had key >= T, i.e. cos~ <= -T  =>  cos <= -T + delta
        const double Dk = wave_elem<NR>(dd, keff - 1);
        const double cmax = -(double)T + delta;
        const double dmin = 1.0 - (cmax > 0.0 ? cmax : 0.0);
        cert = dmin > Dk;
    }
    if (!cert) {
        if (lane == 0) fb_list[atomicAdd(fb_count, 1)] = (int)q;
        return;
    }
    const double wv = weight_of(dd[0], sigma, p);
    const bool keep = lane < keff && dd[0] <= eps && wv > 1e-12;
    const uint64_t km = __ballot(keep);
    const int nkeep = (~km) == 0 ? 64 : (int)__builtin_ctzll(~km);
    if (lane < topk) {
        const bool k2 = lane < nkeep;
        out_idx[q * topk + lane] = k2 ? ix[0] : -1;
        out_dist[q * topk + lane] = k2 ? dd[0] : __builtin_inf();
        if (out_w) out_w[q * topk + lane] = k2 ? wv : 0.0;
    }
}

constexpr int FBT = 128;
static_assert(FBT >= 128, "k_cos_fb_merge: one part list per thread, P <= FBT");
struct alignas(16) FbSmem {
    double ld[FBT][KMAX];
    int li[FBT][KMAX];
    double rd[2];
    int ri[2], rt[2];
};

__global__ __launch_bounds__(FBT) void k_cos_fallback(
    const uint16_t *__restrict__ Q, const uint16_t *__restrict__ C, int64_t nc, int d,
    int64_t q_off, int64_t c_off, int excl, const double *__restrict__ qn,
    const double *__restrict__ cn, int topk, double eps, double sigma, double p,
    const int *__restrict__ fb_count, const int *__restrict__ fb_list,
    int32_t *__restrict__ out_idx, double *__restrict__ out_dist, double *__restrict__ out_w) {
    __shared__ FbSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nfb = *fb_count;
    for (int f = blockIdx.x; f < nfb; f += gridDim.x) {
        const int64_t q = fb_list[f];
        const int64_t gq = q_off + q;
        const bool self_in = excl && gq >= c_off && gq < c_off + nc;
        const int keff = (int)min((int64_t)topk, nc - (self_in ? 1 : 0));
        const uint16_t *qrow = Q + q * (int64_t)d;
        int cnt = 0;
        for (int64_t j = tid; keff > 0 && j < nc; j += FBT) {
            const int64_t gj = c_off + j;
            if (excl && gj == gq) continue;
            const double dist = cos_dist(exact_dot(qrow, C + j * d, d), qn[q], cn[j]);
            const int gi = (int)gj;
            if (cnt == keff && !key_less(dist, gi, sm.ld[tid][keff - 1], sm.li[tid][keff - 1]))
                continue;
            int pp = cnt < keff ? cnt : keff - 1;
            while (pp > 0 && key_less(dist, gi, sm.ld[tid][pp - 1], sm.li[tid][pp - 1])) {
                sm.ld[tid][pp] = sm.ld[tid][pp - 1];
                sm.li[tid][pp] = sm.li[tid][pp - 1];
                --pp;
            }
            sm.ld[tid][pp] = dist;
            sm.li[tid][pp] = gi;
            if (cnt < keff) ++cnt;
        }
        __syncthreads();
        int head = 0;
        bool stop = false;  // the eps/weight filter keeps a prefix
        for (int r = 0; r < keff; ++r) {
            double bd = head < cnt ? sm.ld[tid][head] : __builtin_inf();
            int bi = head < cnt ? sm.li[tid][head] : INT_MAX;
            int bt = tid;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double od = __shfl_xor(bd, o);
                const int oi = __shfl_xor(bi, o), ot = __shfl_xor(bt, o);
                if (key_less(od, oi, bd, bi)) { bd = od; bi = oi; bt = ot; }
            }
            if (lane == 0) { sm.rd[w] = bd; sm.ri[w] = bi; sm.rt[w] = bt; }
            __syncthreads();
            const int win = key_less(sm.rd[1], sm.ri[1], sm.rd[0], sm.ri[0]) ? 1 : 0;
            const double dv = sm.rd[win];
            const double wv = weight_of(dv, sigma, p);
            stop = stop || !(dv <= eps && wv > 1e-12);
            if (tid == sm.rt[win]) {
                ++head;
                out_idx[q * topk + r] = stop ? -1 : sm.ri[win];
                out_dist[q * topk + r] = stop ? __builtin_inf() : dv;
                if (out_w) out_w[q * topk + r] = stop ? 0.0 : wv;
            }
            __syncthreads();
        }
        for (int r = keff + tid; r < topk; r += FBT) {
            out_idx[q * topk + r] = -1;
            out_dist[q * topk + r] = __builtin_inf();
            if (out_w) out_w[q * topk + r] = 0.0;
        }
        __syncthreads();
    }
}

// ---- two-phase generator ------------------------------------------------------
// visiting order: pos p -> row (a p + b) mod n, gcd(a, n) = 1
struct Perm {
    uint64_t a, b, n, ainv;
    __device__ __forceinline__ int64_t operator()(int64_t p) const {
        return (int64_t)((a * (uint64_t)p + b) % n);
    }
    __device__ __forceinline__ int64_t pos(int64_t r) const {  // inverse
        return (int64_t)((ainv * (((uint64_t)r + n - b) % n)) % n);
    }
};

inline Perm make_perm_ab(int64_t n) {
    uint64_t a = (uint64_t)((double)n * 0.6180339887498949);
    if (a == 0) a = 1;
    auto gcd = [](uint64_t x, uint64_t y) { while (y) { const uint64_t t = x % y; x = y; y = t; } return x; };
    while (gcd(a, (uint64_t)n) != 1) ++a;
    a %= (uint64_t)n;
    if (a == 0) a = 1;
    // a^-1 mod n (extended Euclid; n < 2^31 so the products fit 64 bits)
    int64_t r0 = (int64_t)n, r1 = (int64_t)a, t0 = 0, t1 = 1;
    while (r1) {
        const int64_t qq = r0 / r1, r2 = r0 - qq * r1, t2 = t0 - qq * t1;
        r0 = r1; r1 = r2; t0 = t1; t1 = t2;
    }
    const uint64_t ainv = (uint64_t)((t0 % (int64_t)n + (int64_t)n) % (int64_t)n);
    return Perm{a, (uint64_t)n / 3, (uint64_t)n, ainv};
}

// KB32 copy [dp/32][n][32] (zero-padded past d) of rows perm(p) (perm.n == 0:
// identity); one thread per 16 B of output, consecutive threads write
// consecutive bytes of one k-block
// tm > 0: the tile-major variant with panel stride tm k-blocks (gram_sweep2.hpp
// TM; rows padded to 256 with zeros, n_pad = n rounded up)
// pidx (may be NULL): position p holds row pidx[p] (the symmetric sweep's
// threshold order), else Perm pm
__global__ __launch_bounds__(256) void k_to_kb32(const uint16_t *__restrict__ X, int64_t n, int d,
                                                 int dp, Perm pm, uint16_t *__restrict__ XK,
                                                 int tm, const int *__restrict__ pidx = nullptr) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int nkb = dp / 32;
    const int64_t rows = tm ? (n + 255) / 256 * 256 : n;
    const int64_t per_kb = rows * 4;
    if (t >= per_kb * nkb) return;
    int kb, cc;
    int64_t p, o;
    if (tm) {
        cc = (int)(t & 3);
        const int r = (int)((t >> 2) & 255);
        const int64_t pk = t >> 10;  // panel * nkb + kb
        kb = (int)(pk % nkb);
        const int64_t panel = pk / nkb;
        p = panel * 256 + r;
        o = ((panel * tm + kb) << 13) + (r << 5) + 8 * cc;
    } else {
        kb = (int)(t / per_kb);
        const int64_t rem = t - (int64_t)kb * per_kb;
        p = rem >> 2;
        cc = (int)(rem & 3);
        o = ((int64_t)kb * n + p) * 32 + 8 * cc;
    }
    if (p >= n) {  // padded rows (tile-major only)
        *reinterpret_cast<uint4 *>(XK + o) = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    const int64_t src = pidx ? (int64_t)pidx[p] : (pm.n ? pm(p) : p);
    const int e0 = 32 * kb + 8 * cc;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (e0 + 8 <= d) {
        v = *reinterpret_cast<const uint4 *>(X + src * d + e0);  // d % 8 == 0, 16-B aligned rows
    } else if (e0 < d) {
        uint16_t h[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) h[u] = e0 + u < d ? X[src * d + e0 + u] : (uint16_t)0;
        v = make_uint4(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16),
                       h[4] | ((uint32_t)h[5] << 16), h[6] | ((uint32_t)h[7] << 16));
    }
    *reinterpret_cast<uint4 *>(XK + o) = v;
}

// row-major copy of the sample positions [0, m) (stride d), 16 B per thread
__global__ __launch_bounds__(256) void k_sample_rows(const uint16_t *__restrict__ X, int64_t m,
                                                     int d, Perm pm, uint16_t *__restrict__ XR) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int d8 = d / 8;
    if (t >= m * d8) return;
    const int64_t p = t / d8;
    const int c = (int)(t - p * d8);
    *reinterpret_cast<uint4 *>(XR + p * d + 8 * c) =
        *reinterpret_cast<const uint4 *>(X + pm(p) * d + 8 * c);
}

// per position: 1/|c| (phase 1) and -|c| (sweep), f32 of the exact norms
__global__ __launch_bounds__(256) void k_perm_norms(const double *__restrict__ nrm,
                                                    const float *__restrict__ inv, int64_t n,
                                                    Perm pm, float *__restrict__ invp,
                                                    float *__restrict__ negn) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int64_t r = pm(p);
    invp[p] = inv[r];
    negn[p] = -(float)nrm[r];
}

// per query row q: t = -(min over phase-1 slices of the L1-th best key); a
// forced slice (-inf) or no full slice (+inf) -> t = +inf (nothing is
// buffered, the row is rescanned).  tq = t |q| at the query's sweep position.
__global__ __launch_bounds__(256) void k_tau_cos(int64_t nq, int S1, const float *__restrict__ btau1,
                                                 const double *__restrict__ qn, Perm pm,
                                                 float *__restrict__ tcos,
                                                 float *__restrict__ tq_pos) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    float T = __builtin_inff();
    for (int s = 0; s < S1; ++s) T = fminf(T, btau1[q * S1 + s]);
    const bool ok = __builtin_isfinite(T);
    const float t = ok ? -T : __builtin_inff();
    tcos[q] = t;
    tq_pos[pm.pos(q)] = ok ? (float)((double)t * qn[q]) : __builtin_inff();
}

// SW_COS_SYM: sort keys -t (descending thresholds), a non-finite flag
__global__ __launch_bounds__(256) void k_cos_sym_keys(int64_t n, const float *__restrict__ tcos,
                                                      float *__restrict__ key,
                                                      int *__restrict__ iota,
                                                      int *__restrict__ bad) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float t = tcos[r];
    key[r] = -t;
    iota[r] = (int)r;
    if (!__builtin_isfinite(t)) atomicOr(bad, 1);
}

// SW_COS_SYM per position p (row pi[p]): tq = t|x| (diagonal tiles: the
// row's test, as k_tau_cos), ta = |x| and hoff = -t|x| (off-diagonal tiles),
// hc = -|x| (diagonal columns), cn = |x| (the row keys)
__global__ __launch_bounds__(256) void k_cos_sym_pos(int64_t n, const int *__restrict__ pi,
                                                     const float *__restrict__ tcos,
                                                     const double *__restrict__ xn,
                                                     float *__restrict__ tq, float *__restrict__ ta,
                                                     float *__restrict__ hc,
                                                     float *__restrict__ hoff,
                                                     float *__restrict__ cn) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int r = pi[p];
    const double nr = xn[r];
    const float t = tcos[r];
    const float tqv = (float)((double)t * nr);
    tq[p] = tqv;
    ta[p] = (float)nr;
    hc[p] = -(float)nr;
    hoff[p] = -tqv;
    cn[p] = (float)nr;
}

// One wave per query: both buffers' candidates in key = -cos~ order (sweep
// keys mapped back: -cos~ = key / |q| - t), exact distances for the best kq
// and every other candidate whose lower bound does not exceed the worst of
// those, (dist, j) order, certification dist_min(never buffered) > D_k.
// pidx != NULL (SW_COS_SYM): the work items are sweep POSITIONS p (row
// pidx[p]; big_list holds positions), one per-position buffer (S2 = 1, counts
// past cap2 = overflow), candidate ids are positions; no phase-1 lists.
template <int NR>
__global__ __launch_bounds__(256) void k_cos_rerank_x1(
    const uint16_t *__restrict__ X, int64_t n, int d, Perm pm, const int *__restrict__ pidx,
    const double *__restrict__ xn,
    const float *__restrict__ xinv, int S1, int cap1, const uint2 *__restrict__ buf1,
    const int *__restrict__ cnt1, const float *__restrict__ btau1, int S2, int cap2,
    const uint2 *__restrict__ buf2, const int *__restrict__ cnt2, const float *__restrict__ tcos,
    int topk, double delta, double eps, double sigma, double p, const int *__restrict__ qlist,
    const int *__restrict__ qlist_n, int *__restrict__ big_count, int *__restrict__ big_list,
    int32_t *__restrict__ out_idx, double *__restrict__ out_dist, double *__restrict__ out_w,
    int *__restrict__ fb_count, int *__restrict__ fb_list, int m1) {
    __shared__ int cand[4][64 * NR];
    __shared__ float candk[4][64 * NR];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t wq = (int64_t)blockIdx.x * 4 + wid;
    if (qlist ? wq >= *qlist_n : wq >= n) return;
    const int64_t item = qlist ? qlist[wq] : wq;  // a row, or (pidx) a position
    const int64_t q = pidx ? (int64_t)pidx[item] : item;
    const float t = tcos[q];
    bool forced = !(t < __builtin_inff());
    int M = 0;
    const float qi = xinv[q];
    for (int s = 0; s < S1; ++s) {
        const int cnt = cnt1[q * S1 + s];
        const float ts = btau1[q * S1 + s];
        const uint2 *bp = buf1 + (q * S1 + s) * (int64_t)cap1;
        for (int e0 = 0; e0 < cnt; e0 += 64) {
            const int e = e0 + lane;
            const uint2 v = e < cnt ? bp[e] : make_uint2(0x7f800000u, 0u);
            const int64_t gid = e < cnt ? pm((int64_t)v.y) : -1;
            const bool pass = e < cnt && __uint_as_float(v.x) <= ts && gid != q;
            const uint64_t bm = __ballot(pass);
            const int pos = M + (int)__popcll(bm & ((1ull << lane) - 1ull));
            if (pass && pos < 64 * NR) {
                cand[wid][pos] = (int)gid;
                candk[wid][pos] = __uint_as_float(v.x);
            }
            M += (int)__popcll(bm);
        }
    }
    const int64_t qp = pidx ? item : pm.pos(q);  // the sweep ran over positions
    for (int s = 0; s < S2; ++s) {
        int cnt = cnt2[qp * S2 + s];
        forced |= cnt < 0 || cnt > cap2;  // -1 / a count past cap (SW_COS_SYM): overflow
        cnt = min(cnt, cap2);
        const uint2 *bp = buf2 + (qp * S2 + s) * (int64_t)cap2;
        for (int e0 = 0; e0 < cnt; e0 += 64) {
            const int e = e0 + lane;
            const uint2 v = e < cnt ? bp[e] : make_uint2(0u, 0u);
            const int64_t gid = e < cnt ? (pidx ? (int64_t)pidx[v.y] : pm((int64_t)v.y)) : -1;
            const bool pass = e < cnt && gid != q;
            const uint64_t bm = __ballot(pass);
            const int pos = M + (int)__popcll(bm & ((1ull << lane) - 1ull));
            if (pass && pos < 64 * NR) {
                cand[wid][pos] = (int)gid;
                candk[wid][pos] = __uint_as_float(v.x) * qi - t;
            }
            M += (int)__popcll(bm);
        }
    }
    if (!forced && M > 64 * NR && big_list) {
        if (lane == 0) big_list[atomicAdd(big_count, 1)] = (int)item;
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
    const uint16_t *qrow = X + q * (int64_t)d;
    const int kq = min(topk, M);
    // first pass over the kq1 = topk + m1 best keys (<= 64: register 0), the
    // pruning bound the topk-th exact distance among them (as k_rerank_x1,
    // round 6); m1 = 0: the topk best, bound their maximum
    const int kq1 = (m1 > 0 && topk + m1 <= 64) ? min(M, topk + m1) : kq;
    double dd[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        dd[r] = __builtin_inf();
        if (e < kq1) dd[r] = cos_dist(exact_dot(qrow, X + (int64_t)ix[r] * d, d), xn[q], xn[ix[r]]);
    }
    double Dp = -__builtin_inf();
    if (kq1 == kq) {
#pragma unroll
        for (int r = 0; r < NR; ++r) Dp = fmax(Dp, (lane + 64 * r) < kq ? dd[r] : -__builtin_inf());
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) Dp = fmax(Dp, __shfl_xor(Dp, o));
    } else {
        double t[1] = {lane < kq1 ? dd[0] : __builtin_inf()};
        int ti[1] = {lane};
        wave_bitonic_sort<1>(t, ti);
        Dp = __shfl(t[0], kq - 1);
    }
    // pruning bound: the sweep keys carry two extra f32 roundings (2 delta
    // covers them with a wide margin)
    const double dprune = 2.0 * delta + 1e-6;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        if (e >= kq1 && e < M) {
            const double cub = -(double)kk[r] + dprune;
            const double lb = 1.0 - (cub > 0.0 ? cub : 0.0);
            if (lb <= Dp) dd[r] = cos_dist(exact_dot(qrow, X + (int64_t)ix[r] * d, d), xn[q], xn[ix[r]]);
        }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
        if (lane + 64 * r >= M) ix[r] = INT_MAX;
    wave_bitonic_sort<NR>(dd, ix);
    const int keff = (int)min((int64_t)min(topk, M), n - 1);
    const int kneed = (int)min((int64_t)topk, n - 1);
    bool cert = !forced && keff >= kneed;
    if (cert && keff > 0) {
        const double Dk = wave_elem<NR>(dd, keff - 1);
        const double cmax = (double)t + delta;
        const double dmin = 1.0 - (cmax > 0.0 ? cmax : 0.0);
        cert = dmin > Dk;
    }
    if (!cert) {
        if (lane == 0) fb_list[atomicAdd(fb_count, 1)] = (int)q;
        return;
    }
    const double wv = weight_of(dd[0], sigma, p);
    const bool keep = lane < keff && dd[0] <= eps && wv > 1e-12;
    const uint64_t km = __ballot(keep);
    const int nkeep = (~km) == 0 ? 64 : (int)__builtin_ctzll(~km);
    if (lane < topk) {
        const bool k2 = lane < nkeep;
        out_idx[q * topk + lane] = k2 ? ix[0] : -1;
        out_dist[q * topk + lane] = k2 ? dd[0] : __builtin_inf();
        if (out_w) out_w[q * topk + lane] = k2 ? wv : 0.0;
    }
}

// ---- split exact scan (few uncertified rows over a large corpus) ------------
// Block (f, p) scans corpus part p of fallback row f into its keff best
// (dist, id) — the same per-thread insertion lists and block selection as
// k_cos_fallback — and k_cos_fb_merge merges the P part lists of a row (each
// sorted) with the same selection, then applies the eps / weight prefix.
// Block-level selection of the r-th best over the threads' sorted lists.
template <typename Emit>
__device__ void fb_select(FbSmem &sm, int cnt, int keff, Emit emit) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int head = 0;
    for (int r = 0; r < keff; ++r) {
        double bd = head < cnt ? sm.ld[tid][head] : __builtin_inf();
        int bi = head < cnt ? sm.li[tid][head] : INT_MAX;
        int bt = tid;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o);
            const int oi = __shfl_xor(bi, o), ot = __shfl_xor(bt, o);
            if (key_less(od, oi, bd, bi)) { bd = od; bi = oi; bt = ot; }
        }
        if (lane == 0) { sm.rd[w] = bd; sm.ri[w] = bi; sm.rt[w] = bt; }
        __syncthreads();
        const int win = key_less(sm.rd[1], sm.ri[1], sm.rd[0], sm.ri[0]) ? 1 : 0;
        if (tid == sm.rt[win]) {
            ++head;
            emit(r, sm.rd[win], sm.ri[win]);
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(FBT) void k_cos_fb_part(
    const uint16_t *__restrict__ X, int64_t n, int d, const double *__restrict__ xn, int topk,
    int P, int64_t cs, const int *__restrict__ fb_list, double *__restrict__ pd,
    int *__restrict__ pi, int *__restrict__ pc) {
    __shared__ FbSmem sm;
    const int tid = threadIdx.x;
    const int f = blockIdx.x / P, p = blockIdx.x % P;
    const int64_t q = fb_list[f];
    const int keff = (int)min((int64_t)topk, n - 1);
    const int64_t j0 = (int64_t)p * cs, j1 = min(n, j0 + cs);
    const uint16_t *qrow = X + q * (int64_t)d;
    int cnt = 0;
    for (int64_t j = j0 + tid; keff > 0 && j < j1; j += FBT) {
        if (j == q) continue;
        const double dist = cos_dist(exact_dot(qrow, X + j * d, d), xn[q], xn[j]);
        const int gi = (int)j;
        if (cnt == keff && !key_less(dist, gi, sm.ld[tid][keff - 1], sm.li[tid][keff - 1]))
            continue;
        int pp = cnt < keff ? cnt : keff - 1;
        while (pp > 0 && key_less(dist, gi, sm.ld[tid][pp - 1], sm.li[tid][pp - 1])) {
            sm.ld[tid][pp] = sm.ld[tid][pp - 1];
            sm.li[tid][pp] = sm.li[tid][pp - 1];
            --pp;
        }
        sm.ld[tid][pp] = dist;
        sm.li[tid][pp] = gi;
        if (cnt < keff) ++cnt;
    }
    __syncthreads();
    // entries of the part: every valid j in range beyond the query itself
    const int64_t valid = (j1 > j0 ? j1 - j0 : 0) - ((q >= j0 && q < j1) ? 1 : 0);
    const int kp = (int)min((int64_t)keff, max<int64_t>(valid, 0));
    const int64_t o = ((int64_t)f * P + p) * KMAX;
    fb_select(sm, cnt, kp, [&](int r, double dv, int iv) { pd[o + r] = dv; pi[o + r] = iv; });
    if (tid == 0) pc[(int64_t)f * P + p] = kp;
}

__global__ __launch_bounds__(FBT) void k_cos_fb_merge(
    int64_t n, int topk, int P, double eps, double sigma, double p_, const int *__restrict__ fb_list,
    const double *__restrict__ pd, const int *__restrict__ pi, const int *__restrict__ pc,
    int32_t *__restrict__ out_idx, double *__restrict__ out_dist, double *__restrict__ out_w) {
    __shared__ FbSmem sm;
    __shared__ int sstop;
    const int tid = threadIdx.x, f = blockIdx.x;
    const int64_t q = fb_list[f];
    const int keff = (int)min((int64_t)topk, n - 1);
    int cnt = 0;
    if (tid == 0) sstop = 0;
    if (tid < P) {
        const int64_t o = ((int64_t)f * P + tid) * KMAX;
        cnt = pc[(int64_t)f * P + tid];
        for (int r = 0; r < cnt; ++r) {
            sm.ld[tid][r] = pd[o + r];
            sm.li[tid][r] = pi[o + r];
        }
    }
    __syncthreads();
    // the eps / weight filter keeps a prefix: the first failing entry stops
    // the list (sstop: each round's emitter is ordered after the previous
    // round's by fb_select's barrier)
    fb_select(sm, cnt, keff, [&](int r, double dv, int iv) {
        const double wv = weight_of(dv, sigma, p_);
        const bool st = sstop || !(dv <= eps && wv > 1e-12);
        if (st) sstop = 1;
        out_idx[q * topk + r] = st ? -1 : iv;
        out_dist[q * topk + r] = st ? __builtin_inf() : dv;
        if (out_w) out_w[q * topk + r] = st ? 0.0 : wv;
    });
    for (int r = keff + tid; r < topk; r += FBT) {
        out_idx[q * topk + r] = -1;
        out_dist[q * topk + r] = __builtin_inf();
        if (out_w) out_w[q * topk + r] = 0.0;
    }
}

}  // namespace kb16

hipError_t sort_f32_pairs(const float *keys_in, float *keys_out, const int *vals_in,
                          int *vals_out, int64_t n, hipStream_t s);  // sortkeys.hip

static thread_local mn_knn_stats t_bf16_stats{};

// ---- phase 1 as a sweep (round 4; C2's knn_f32.hip sweep_phase1, cosine form)
// (a) the list generator (k_gram_bf16<GM_COS>) on a pre-sample — the first
// m0 / CP1_DIV sample positions, list CP1_L0 — gives each row a cosine
// threshold t0; (b) the query-major SW_COS sweep of every position against the
// sample positions [0, m0) buffers the pairs with cos~ > t0 (keys k = t0|q| -
// q.c/|c|, so -cos~ = k/|q| - t0); (c) k_p1_select_cos takes each position's
// L1-th smallest buffered key -> btau1[row] = k/|q| - t0 = -(the sample's L1-th
// best cos~), the list generator's own output (an overflowing buffer gives a
// lower threshold: more candidates; the certificate does not depend on it);
// (d) rows with fewer than L1 buffered keys run the list generator alone.
// C5 (1M x 3072, same process, profiles/r04/r04_c5_p1_params.log): the list
// generator 501 ms; (L0, div) = (4, 8) 430 ms (135k rows short), (6, 8) 375
// (10k), (8, 8) 380, (8, 6) 396, (6, 12) 361 (1.5k short); outputs identical.
constexpr int CP1_L0 = 6, CP1_DIV = 12;

template <int NR>
__global__ __launch_bounds__(256) void k_p1_select_cos(int64_t n, kb16::Perm pm, const int *__restrict__ cnt,
                                                       const uint2 *__restrict__ buf, int cap, int L1,
                                                       const double *__restrict__ xn,
                                                       const float *__restrict__ t0,
                                                       float *__restrict__ btau,
                                                       int *__restrict__ fb_count,
                                                       int *__restrict__ fb_list) {
    const int lane = threadIdx.x & 63;
    const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (p >= n) return;
    const int64_t r = pm(p);
    int c = cnt[p];
    c = (c < 0 || c > cap) ? cap : c;  // -1: overflow, the buffer is full
    if (c < L1) {
        if (lane == 0) {
            btau[r] = __builtin_inff();
            fb_list[atomicAdd(fb_count, 1)] = (int)r;
        }
        return;
    }
    float kk[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
        const int e = lane + 64 * u;
        kk[u] = e < c ? __uint_as_float(buf[p * (int64_t)cap + e].x) : __builtin_inff();
    }
    float t = -__builtin_inff(), res = __builtin_inff();
    int need = L1;
    for (int it = 0; it < L1; ++it) {
        float m = __builtin_inff();
#pragma unroll
        for (int u = 0; u < NR; ++u) m = fminf(m, kk[u] > t ? kk[u] : __builtin_inff());
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
        int eq = 0;
#pragma unroll
        for (int u = 0; u < NR; ++u) eq += (int)__popcll(__ballot(kk[u] == m));
        if (eq >= need) { res = m; break; }
        need -= eq;
        t = m;
    }
    if (lane == 0) btau[r] = (float)((double)res / xn[r] - (double)t0[r]);
}

__global__ __launch_bounds__(256) void k_gather_rows_bf16(const uint16_t *__restrict__ X, int d,
                                                          const float *__restrict__ xinv,
                                                          const int *__restrict__ rows, int nfb,
                                                          uint16_t *__restrict__ out,
                                                          float *__restrict__ inv_out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 16 B each
    const int d8 = d / 8;
    if (e < (int64_t)nfb * d8) {
        const int64_t i = e / d8;
        const int c = (int)(e - i * d8);
        *reinterpret_cast<uint4 *>(out + i * d + 8 * c) =
            *reinterpret_cast<const uint4 *>(X + (int64_t)rows[i] * d + 8 * c);
    }
    if (e < nfb) inv_out[e] = xinv[rows[e]];
}

// min over the S slices of each fallback row's threshold -> btau[row]
__global__ __launch_bounds__(256) void k_scatter_min(const int *__restrict__ rows, int nfb, int S,
                                                     const float *__restrict__ v,
                                                     float *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nfb) return;
    float m = __builtin_inff();
    for (int q = 0; q < S; ++q) m = fminf(m, v[(int64_t)i * S + q]);
    out[rows[i]] = m;
}

// Phase 1 by sweep: btau1 [n] (one slice) for k_tau_cos; XK holds the
// position-order tile-major copy on return.
static int cos_sweep_phase1(const uint16_t *X, int64_t n, int32_t d, int dp, int nkb, int pst,
                            const kb16::Perm &pm, const uint16_t *XR, int64_t m0, int L1,
                            const double *xn, const float *xinv, const float *invp,
                            const float *negn, float *tcos, float *tq_pos, uint16_t *XK,
                            float *btau1, int *cntr, int *fb_list, hipStream_t s) {
    using namespace kb16;
    const int L0 = knob_int("MN_BF16_P1_L0", CP1_L0);
    const int dv = std::max(2, knob_int("MN_BF16_P1_DIV", CP1_DIV));
    {   // position-order copy of every row (the queries and the sample)
        const int64_t nt = (n + 255) / 256 * 256 * 4 * nkb;
        hipLaunchKernelGGL(k_to_kb32, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, X, n, d,
                           dp, pm, XK, pst, (const int *)nullptr);
        MN_KCHECK(s, "k_to_kb32 (phase 1)");
    }
    // (a) pre-sample
    int64_t m00 = std::max<int64_t>(m0 / dv, (int64_t)64 * L0);
    m00 = std::min<int64_t>(m0, (m00 + 255) / 256 * 256);
    const GramPlan p0 = plan_gram(n, m00, L0, 1, 1);
    uint2 *cb0 = (uint2 *)scratch(kSlotX1Esc, (size_t)n * p0.S * p0.cap * sizeof(uint2) + 64);
    char *m0b = (char *)scratch(kSlotX1Meta2, (size_t)n * p0.S * 8 + 64);
    MN_REQUIRE(cb0 && m0b, MN_ENOMEM, "mn_knn_cos_bf16: pre-sample buffer allocation failed");
    int *bc0 = (int *)m0b;
    float *bt0 = (float *)(m0b + (size_t)n * p0.S * 4);
    const int64_t bq = (n + BM - 1) / BM;
    hipLaunchKernelGGL((k_gram_bf16<GM_COS, 0>), dim3((unsigned)(bq * p0.S)), dim3(NT), 0, s, X, n, XR,
                       m00, d, (int64_t)0, (int64_t)0, 0, xinv, invp, L0, (int)p0.S, p0.chunk, p0.cap,
                       cb0, bc0, bt0);
    MN_KCHECK(s, "k_gram_bf16<COS> (pre-sample)");
    hipLaunchKernelGGL(k_tau_cos, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, (int)p0.S,
                       bt0, xn, pm, tcos, tq_pos);
    MN_KCHECK(s, "k_tau_cos (pre-sample)");
    // (b) the sweep of the sample positions with t0
    const double expect = (double)L0 * (double)m0 / (double)m00;
    const int cap = std::min(512, std::max(64, (int)((2.5 * expect + 64.0 + 15.0) / 16.0) * 16));
    uint2 *cbuf = (uint2 *)scratch(kSlotX1Buf2, (size_t)n * cap * sizeof(uint2) + 64);
    int *cnt = (int *)scratch(kSlotX1Meta2, (size_t)n * 4 + 64);
    MN_REQUIRE(cbuf && cnt, MN_ENOMEM, "mn_knn_cos_bf16: phase-1 sweep buffer allocation failed");
    MN_HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)n * 4, s));
    const int64_t nqb = (n + ksw2::BQ - 1) / ksw2::BQ;
    // round 6: gram_sweep3.hpp's query-major mode (tuning build
    // MN_P1_SWEEP3=0: round 5's sweep2)
    auto p1k = ksw2::k_gram_sweep3<0, ksw2::SW_COS, 2>;
#ifdef MN_TUNING
    if (!knob_int("MN_P1_SWEEP3", 1)) p1k = ksw2::k_gram_sweep2<0, ksw2::SW_COS, true>;
#endif
    hipLaunchKernelGGL(p1k, dim3((unsigned)nqb), dim3(ksw2::NT), 0, s, XK, n, XK, m0, nkb, (int64_t)0,
                       (int64_t)0, 0, tq_pos, tq_pos, negn, (int64_t)0, 1, m0, cap, cbuf, cnt, pst,
                       ksw2::SymArgs{});
    MN_KCHECK(s, "k_gram_sweep3<COS> (phase 1)");
    // (c) the L1-th smallest key per position
    MN_HIP_TRY(hipMemsetAsync(cntr, 0, 4, s));
    const unsigned g4 = (unsigned)((n + 3) / 4);
    if (cap <= 128)
        hipLaunchKernelGGL(k_p1_select_cos<2>, dim3(g4), dim3(256), 0, s, n, pm, cnt, cbuf, cap, L1, xn, tcos, btau1, cntr, fb_list);
    else if (cap <= 256)
        hipLaunchKernelGGL(k_p1_select_cos<4>, dim3(g4), dim3(256), 0, s, n, pm, cnt, cbuf, cap, L1, xn, tcos, btau1, cntr, fb_list);
    else
        hipLaunchKernelGGL(k_p1_select_cos<8>, dim3(g4), dim3(256), 0, s, n, pm, cnt, cbuf, cap, L1, xn, tcos, btau1, cntr, fb_list);
    MN_KCHECK(s, "k_p1_select_cos");
    int nfb = 0;
    MN_HIP_TRY(hipMemcpyAsync(&nfb, cntr, 4, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (knob("MN_BF16_DEBUG"))
        fprintf(stderr, "cos_sweep_phase1: pre-sample %lld, cap %d, rows short of L1 %d\n",
                (long long)m00, cap, nfb);
    if (nfb == 0) return MN_OK;
    // (d) the rows t0 left short: the list generator on them alone
    const GramPlan pf = plan_gram(nfb, m0, L1, 1, 1);
    const size_t gb = (size_t)nfb * d * 2, lb = (size_t)nfb * pf.S * pf.cap * sizeof(uint2);
    char *g = (char *)scratch(kSlotX1Esc, gb + lb + (size_t)nfb * pf.S * 8 + (size_t)nfb * 4 + 1024);
    MN_REQUIRE(g, MN_ENOMEM, "mn_knn_cos_bf16: phase-1 fallback allocation failed");
    uint16_t *Xf = (uint16_t *)g;
    uint2 *cbf = (uint2 *)(g + ((gb + 255) & ~(size_t)255));
    int *bcf = (int *)((char *)cbf + ((lb + 255) & ~(size_t)255));
    float *btf = (float *)(bcf + (size_t)nfb * pf.S);
    float *invf = btf + (size_t)nfb * pf.S;
    hipLaunchKernelGGL(k_gather_rows_bf16, dim3((unsigned)(((int64_t)nfb * (d / 8) + 255) / 256)),
                       dim3(256), 0, s, X, d, xinv, fb_list, nfb, Xf, invf);
    MN_KCHECK(s, "k_gather_rows_bf16");
    const int64_t bqf = (nfb + BM - 1) / BM;
    hipLaunchKernelGGL((k_gram_bf16<GM_COS, 0>), dim3((unsigned)(bqf * pf.S)), dim3(NT), 0, s, Xf,
                       (int64_t)nfb, XR, m0, d, (int64_t)0, (int64_t)0, 0, invf, invp, L1, (int)pf.S,
                       pf.chunk, pf.cap, cbf, bcf, btf);
    MN_KCHECK(s, "k_gram_bf16<COS> (phase-1 fallback)");
    hipLaunchKernelGGL(k_scatter_min, dim3((unsigned)((nfb + 255) / 256)), dim3(256), 0, s, fb_list,
                       nfb, (int)pf.S, btf, btau1);
    MN_KCHECK(s, "k_scatter_min");
    return MN_OK;
}

// Two-phase generator for self graphs (see the header).  X [n][d] row-major
// (d % 8 == 0, 16-B aligned), exact norms xn / 1/|x| xinv by row.  Returns
// MN_OK, or 1 when the inputs do not suit it (the caller runs the one-phase
// generator).
static int knn_cos_bf16_x1(const uint16_t *X, int64_t n, int32_t d, const mn_cos_opts *o,
                           const double *xn, const float *xinv, int *flags, int *fb_list,
                           int32_t *out_idx, double *out_dist, double *out_w, hipStream_t s) {
    using namespace kb16;
    const int topk = o->topk;
    int L1 = std::min(std::max((topk + 1) / 2, 16), 48);
    const char *fl = knob("MN_BF16_L1");  // experiments: phase-1 list length
    if (fl && *fl) L1 = std::min(std::max(atoi(fl), 4), 48);
    // sample = n / div rows: n/24 under the symmetric sweep (its cost does not
    // follow the threshold; C5 1M x 3072: phase 1 726 -> 497 ms, 0 uncertified,
    // profiles/r03k_c5_grid.log), n/16 for the query-major sweep (round 2 grid)
    const char *te0 = knob("MN_BF16_TM"), *sy0 = knob("MN_BF16_SYM");
    const bool sym_planned = !(te0 && *te0 == '0') && !(sy0 && *sy0 == '0');
    const char *fs = knob("MN_BF16_SAMPLE_DIV");  // experiments: sample = n / div
    const int64_t div = (fs && *fs) ? std::max(2, atoi(fs)) : (sym_planned ? 24 : 16);
    int64_t m0 = std::max<int64_t>(n / div, (int64_t)64 * L1);
    m0 = (m0 + 255) / 256 * 256;  // whole sweep tiles (TM) and phase-1 tiles
    if (m0 + 4 * ksw2::BC > n || n * 32 >= INT_MAX || n >= INT_MAX) return 1;
    const int dp = (d + 255) / 256 * 256;  // KB32 k-blocks, nkb >= 8 (sweep2's prefetch)
    const int nkb = dp / 32;
    const Perm pm = make_perm_ab(n);

    const char *te = knob("MN_BF16_TM");  // layout A/B: 0 = k-block-major KB32
    const int tmaj = (te && *te == '0') ? 0 : 1;
    const char *tpe = knob("MN_TM_PAD");  // panel stride nkb + pad k-blocks (default 1)
    const int pst = tmaj ? nkb + ((tpe && *tpe) ? std::max(0, atoi(tpe)) : 1) : 0;
    const int64_t nrows = tmaj ? (n + 255) / 256 * 256 : n;
    uint16_t *XK = (uint16_t *)scratch(kSlotX1CK, (size_t)nrows * (tmaj ? pst * 32 : dp) * 2 + 64);
    uint16_t *XR = (uint16_t *)scratch(kSlotX1CR, (size_t)m0 * d * 2 + 64);
    float *aux = (float *)scratch(kSlotX1Aux, (size_t)n * 16 + 256);
    MN_REQUIRE(XK && XR && aux, MN_ENOMEM, "mn_knn_cos_bf16: two-phase scratch allocation failed");
    float *invp = aux, *negn = aux + n, *tcos = negn + n, *tq_pos = tcos + n;

    Timer tm;
    tm.start(o->timing != 0, s);
    {
        const int64_t ns = m0 * (d / 8);
        hipLaunchKernelGGL(k_sample_rows, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, X, m0,
                           d, pm, XR);
        hipLaunchKernelGGL(k_perm_norms, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, xn,
                           xinv, n, pm, invp, negn);
        MN_KCHECK(s, "k_sample_rows / k_perm_norms");
    }
    // phase 1: every query (rows, in place) against the sample (positions [0, m0))
    const GramPlan pl = plan_gram(n, m0, L1, 1, 1);
    const size_t nbuf1 = (size_t)n * pl.S * pl.cap;
    uint2 *buf1 = (uint2 *)scratch(kSlotLists, nbuf1 * sizeof(uint2) + 64);
    char *meta1 = (char *)scratch(kSlotListMeta, (size_t)n * pl.S * 8 + 64);
    MN_REQUIRE(buf1 && meta1, MN_ENOMEM, "mn_knn_cos_bf16: phase-1 buffer allocation failed");
    int *cnt1 = (int *)meta1;
    float *btau1 = (float *)(meta1 + (size_t)n * pl.S * 4);
    // phase 1 by sweep (round 4; SW_COS_SYM only — the query-major sweep reads
    // the phase-1 lists; tuning build: MN_BF16_P1_SWEEP=0 keeps the list generator)
    const bool p1s = sym_planned && tmaj && knob_int("MN_BF16_P1_SWEEP", 1) != 0;
    auto list_phase1 = [&]() -> int {
        const int64_t bq = (n + BM - 1) / BM;
        hipLaunchKernelGGL((k_gram_bf16<GM_COS, 0>), dim3((unsigned)(bq * pl.S)), dim3(NT), 0, s, X,
                           n, XR, m0, d, (int64_t)0, (int64_t)0, 0, xinv, invp, L1, (int)pl.S,
                           pl.chunk, pl.cap, buf1, cnt1, btau1);
        MN_KCHECK(s, "k_gram_bf16<COS> (sample)");
        hipLaunchKernelGGL(k_tau_cos, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n,
                           (int)pl.S, btau1, xn, pm, tcos, tq_pos);
        MN_KCHECK(s, "k_tau_cos");
        return MN_OK;
    };
    if (p1s) {
        const int rc1 = cos_sweep_phase1(X, n, d, dp, nkb, pst, pm, XR, m0, L1, xn, xinv, invp, negn,
                                         tcos, tq_pos, XK, btau1, flags + 6, fb_list, s);
        if (rc1 != MN_OK) return rc1;
        hipLaunchKernelGGL(k_tau_cos, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, 1,
                           btau1, xn, pm, tcos, tq_pos);
        MN_KCHECK(s, "k_tau_cos");
    } else {
        const int rc1 = list_phase1();
        if (rc1 != MN_OK) return rc1;
    }
    tm.mark();
    // phase 2, SW_COS_SYM (default, MN_BF16_SYM=0: the query-major sweep):
    // positions in descending-threshold order, each unordered pair once; the
    // query-major sweep when a threshold is not finite (a row without a full
    // sample list) or the layout is k-block-major
    const char *sye = knob("MN_BF16_SYM");
    bool sym = tmaj && !(sye && *sye == '0');
    int *pi = nullptr;
    float *tqS = nullptr, *taS = nullptr, *hcS = nullptr, *hoS = nullptr, *cnS = nullptr;
    if (sym) {
        const size_t an = ((size_t)n * 4 + 255) & ~(size_t)255;
        char *so = (char *)scratch(kSlotSymOrd, an * 9 + 256);
        MN_REQUIRE(so, MN_ENOMEM, "mn_knn_cos_bf16: symmetric-sweep scratch allocation failed");
        float *key = (float *)so, *skey = (float *)(so + an);
        int *iota = (int *)(so + 2 * an);
        pi = (int *)(so + 3 * an);
        tqS = (float *)(so + 4 * an);
        taS = (float *)(so + 5 * an);
        hcS = (float *)(so + 6 * an);
        hoS = (float *)(so + 7 * an);
        cnS = (float *)(so + 8 * an);
        hipLaunchKernelGGL(k_cos_sym_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n,
                           tcos, key, iota, flags + 4);
        MN_KCHECK(s, "k_cos_sym_keys");
        int bad = 0;
        MN_HIP_TRY(hipMemcpyAsync(&bad, flags + 4, 4, hipMemcpyDeviceToHost, s));
        MN_HIP_TRY(hipStreamSynchronize(s));
        if (bad) {
            sym = false;
            // the query-major sweep reads the sample lists: the list generator
            if (p1s) {
                const int rc1 = list_phase1();
                if (rc1 != MN_OK) return rc1;
            }
        } else {
            MN_HIP_TRY(sort_f32_pairs(key, skey, iota, pi, n, s));
        }
    }
    {
        const int64_t nt = nrows * 4 * nkb;
        hipLaunchKernelGGL(k_to_kb32, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, X, n, d,
                           dp, pm, XK, pst, sym ? (const int *)pi : (const int *)nullptr);
        MN_KCHECK(s, "k_to_kb32");
        if (sym) {
            hipLaunchKernelGGL(k_cos_sym_pos, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n,
                               pi, tcos, xn, tqS, taS, hcS, hoS, cnS);
            MN_KCHECK(s, "k_cos_sym_pos");
        }
    }
    tm.mark();  // the sweep copy (+ SW_COS_SYM order and per-position folds)
    double expect;
    int S2, cap2;
    ksw2::SweepPlan p2{};
    if (sym) {
        expect = (double)L1 * (double)n / (double)m0;
        S2 = 1;
        cap2 = std::max(256, (int)((2.5 * expect + 64.0 + 15.0) / 16.0) * 16);
    } else {
        expect = (double)L1 * (double)(n - m0) / (double)m0;
        p2 = ksw2::plan_sweep(n, n - m0, expect);
        S2 = (int)p2.S;
        cap2 = p2.cap;
    }
    const size_t nbuf2 = (size_t)n * S2 * cap2;
    uint2 *buf2 = (uint2 *)scratch(kSlotX1Buf2, nbuf2 * sizeof(uint2) + 64);
    int *cnt2 = (int *)scratch(kSlotX1Meta2, (size_t)n * S2 * 4 + 64);
    MN_REQUIRE(buf2 && cnt2, MN_ENOMEM, "mn_knn_cos_bf16: sweep buffer allocation failed");
    if (sym) {
        const int nbk = (int)((n + ksw2::BC - 1) / ksw2::BC);
        // group shape 8 row blocks x 4 column phases (round 6, sweep3: 2510-2524
        // vs 2630-2652 ms for 4 x 8 same process, 2 x 16 2830, 16 x 2 2608;
        // profiles/r06/r06_c5_gr_scan*.log)
        int4 *dtab = nullptr;
        const std::vector<int4> &tab =
            ksw2::sym_table_device(nbk, 256, knob_int("MN_BF16_SYM_ORDER", 2), 8, 0, 1, s, &dtab);
        MN_REQUIRE(dtab, MN_ENOMEM, "mn_knn_cos_bf16: block table allocation / upload failed");
        MN_HIP_TRY(hipMemsetAsync(cnt2, 0, (size_t)n * 4, s));
        MN_REQUIRE(tab.size() < INT_MAX, MN_ENOTSUP, "mn_knn_cos_bf16: sweep grid too large");
        // the default: gram_sweep3.hpp's schedule, DMA two k-steps ahead
        auto kern = ksw2::k_gram_sweep3<0, ksw2::SW_COS_SYM, 2>;
        const char *probe = knob("MN_BF16_PROBE");  // tuning build: noepi = K loop only
#ifdef MN_TUNING
        const int sweep_gen = knob_int("MN_SWEEP", 4);  // 2: round 5's k_gram_sweep2
        const bool noepi = probe && !strcmp(probe, "noepi");
        if (sweep_gen == 4 && noepi) kern = ksw2::k_gram_sweep3<1, ksw2::SW_COS_SYM, 2>;
        if (sweep_gen == 5)
            kern = noepi ? ksw2::k_gram_sweep3<1, ksw2::SW_COS_SYM, 2, 2>
                         : ksw2::k_gram_sweep3<0, ksw2::SW_COS_SYM, 2, 2>;
        if (sweep_gen == 3)
            kern = noepi ? ksw2::k_gram_sweep3<1, ksw2::SW_COS_SYM> : ksw2::k_gram_sweep3<0, ksw2::SW_COS_SYM>;
        if (sweep_gen == 2) {
            kern = noepi ? ksw2::k_gram_sweep2<1, ksw2::SW_COS_SYM, true>
                         : ksw2::k_gram_sweep2<0, ksw2::SW_COS_SYM, true>;
            // MN_SW_V: the DMA-placement variants of gram_sweep2.hpp (default 14)
            if (knob_int("MN_SW_V", 14) == 0) kern = ksw2::k_gram_sweep2<0, ksw2::SW_COS_SYM, true, false, 0>;
            if (knob_int("MN_SW_V", 14) == 2) kern = ksw2::k_gram_sweep2<0, ksw2::SW_COS_SYM, true, false, 2>;
        }
#endif
        hipLaunchKernelGGL(kern, dim3((unsigned)tab.size()), dim3(ksw2::NT), 0, s, XK, n, XK, n, nkb,
                           (int64_t)0, (int64_t)0, 1, tqS, cnS, hcS, (int64_t)0, 1, (int64_t)0,
                           cap2, buf2, cnt2, pst, ksw2::SymArgs{dtab, taS, hoS, 0});
        MN_KCHECK(s, "k_gram_sweep3<COS_SYM>");
        if (probe && *probe) {  // timing probe: no outputs are produced
            tm.mark();
            MN_HIP_TRY(hipStreamSynchronize(s));
            if (tm.on) {
                t_bf16_stats.ms_sample = tm.ms(0, 1);
                t_bf16_stats.ms_norms = tm.ms(1, 2);
                t_bf16_stats.ms_sweep = tm.ms(2, 3);
                t_bf16_stats.ms_gram = t_bf16_stats.ms_sample + t_bf16_stats.ms_sweep;
            }
            t_bf16_stats.sample_rows = m0;
            t_bf16_stats.sweep_slices = -1;
            return MN_OK;
        }
    } else {
        const int64_t grid = (n + ksw2::BQ - 1) / ksw2::BQ * p2.S;
        MN_REQUIRE(grid < INT_MAX, MN_ENOTSUP, "mn_knn_cos_bf16: sweep grid too large");
        auto kern = tmaj ? ksw2::k_gram_sweep2<0, ksw2::SW_COS, true>
                         : ksw2::k_gram_sweep2<0, ksw2::SW_COS, false>;
        const char *probe = knob("MN_BF16_PROBE");  // tuning build: noepi = K loop only
#ifdef MN_TUNING
        if (probe && !strcmp(probe, "noepi"))
            kern = tmaj ? ksw2::k_gram_sweep2<1, ksw2::SW_COS, true>
                        : ksw2::k_gram_sweep2<1, ksw2::SW_COS, false>;
#endif
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(ksw2::NT), 0, s, XK, n, XK, n, nkb,
                           (int64_t)0, (int64_t)0, 0, tq_pos, tq_pos, negn, m0, S2, p2.chunk,
                           cap2, buf2, cnt2, pst, ksw2::SymArgs{});
        MN_KCHECK(s, "k_gram_sweep2<COS>");
        if (probe && *probe) {  // timing probe: no outputs are produced
            tm.mark();
            MN_HIP_TRY(hipStreamSynchronize(s));
            if (tm.on) {
                t_bf16_stats.ms_sample = tm.ms(0, 1);
                t_bf16_stats.ms_norms = tm.ms(1, 2);
                t_bf16_stats.ms_sweep = tm.ms(2, 3);
                t_bf16_stats.ms_gram = t_bf16_stats.ms_sample + t_bf16_stats.ms_sweep;
            }
            t_bf16_stats.sample_rows = m0;
            t_bf16_stats.sweep_slices = S2;
            return MN_OK;
        }
    }
    tm.mark();
    // certification slack (cosine units): phase 1's f32 accumulation of exact
    // products scaled by two f32 inverse norms, 2 (d + 12) u; the sweep's
    // dk + 1 terms (products and acc0 = -t|q||c|, |t| <= 1 + ...) with f32
    // roundings of t|q|, |c| and acc0: 2.5 (dk + 16) u covers both.  dk = d
    // rounded up to the MFMA's 32: the all-zero k-blocks of the padding add
    // exactly 0 to the accumulator
    const int dk = (d + 31) / 32 * 32;
    // SW_COS_SYM: + 24 u for the off-diagonal row key k_q's four f32 roundings
    // (terms |acc|/|q||c| <= 2, |t(c)|, |t(q)| <= 1 in cosine units)
    const double delta = 2.5 * ((double)dk + 16.0) * 0x1p-24 + (sym ? 24.0 * 0x1p-24 : 0.0);
    int *fb_count = flags + 2, *big_count = flags + 3;
    int *big_list = fb_list + n;
    const int *pix = sym ? (const int *)pi : (const int *)nullptr;
    const int S1r = sym ? 0 : (int)pl.S;  // SW_COS_SYM decided the sample pairs too
    // the re-rank's first-pass margin: 0 (C5: 106.8 ms; 4 / 8 / 16: 113 / 158 / 215 ms —
    // profiles/r06/r06_c5_rerank_m1_ab.log: its 6-KB rows make every extra one cost)
    const int crr_m1 = knob_int("MN_CRR_M1", 0);
#define MN_RRC(NRV, NB, QL, QN, BC, BL)                                                          \
    hipLaunchKernelGGL(k_cos_rerank_x1<NRV>, dim3((unsigned)(NB)), dim3(256), 0, s, X, n, d, pm, \
                       pix, xn, xinv, S1r, pl.cap, buf1, cnt1, btau1, S2, cap2, buf2, cnt2,     \
                       tcos, topk, delta, o->eps, o->sigma, o->p, QL, QN, BC, BL, out_idx,      \
                       out_dist, out_w, fb_count, fb_list, crr_m1)
    MN_RRC(8, (n + 3) / 4, (const int *)nullptr, (const int *)nullptr, big_count, big_list);
    MN_KCHECK(s, "k_cos_rerank_x1<8>");
    int hb[4] = {0, 0, 0, 0};
    MN_HIP_TRY(hipMemcpyAsync(hb, flags, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    if (hb[3] > 0) {
        MN_RRC(16, (hb[3] + 3) / 4, (const int *)big_list, (const int *)big_count, (int *)nullptr,
               (int *)nullptr);
        MN_KCHECK(s, "k_cos_rerank_x1<16>");
    }
#undef MN_RRC
    tm.mark();
    MN_HIP_TRY(hipMemcpyAsync(hb, flags, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    const int nfb = hb[2];
    // few rows: each row's exact scan split over P blocks + a merge (one block
    // per row would leave the chip idle); many rows: one block per row
    // (k_cos_fb_merge loads the P part lists one per thread: P <= FBT)
    const int P = (int)std::min<int64_t>(FBT, std::max<int64_t>(1, (2048 + nfb - 1) / std::max(nfb, 1)));
    const char *fse = knob("MN_BF16_FB_SPLIT");  // 0: always one block per row (A/B)
    if (nfb > 0 && P >= 4 && !(fse && *fse == '0')) {
        const int64_t cs = (n + P - 1) / P;
        const size_t np = (size_t)nfb * P;
        char *fbp = (char *)scratch(kSlotGeneric3, np * KMAX * 12 + np * 4 + 256);
        MN_REQUIRE(fbp, MN_ENOMEM, "mn_knn_cos_bf16: split-scan scratch allocation failed");
        double *pd = (double *)fbp;
        int *pix2 = (int *)(pd + np * KMAX), *pc = pix2 + np * KMAX;
        hipLaunchKernelGGL(k_cos_fb_part, dim3((unsigned)np), dim3(FBT), 0, s, X, n, d, xn, topk, P,
                           cs, fb_list, pd, pix2, pc);
        MN_KCHECK(s, "k_cos_fb_part");
        hipLaunchKernelGGL(k_cos_fb_merge, dim3((unsigned)nfb), dim3(FBT), 0, s, n, topk, P, o->eps,
                           o->sigma, o->p, fb_list, pd, pix2, pc, out_idx, out_dist, out_w);
        MN_KCHECK(s, "k_cos_fb_merge");
    } else {
        hipLaunchKernelGGL(k_cos_fallback, dim3((unsigned)std::min<int64_t>(n, 1024)), dim3(FBT), 0,
                           s, X, X, n, d, (int64_t)0, (int64_t)0, 1, xn, xn, topk, o->eps, o->sigma,
                           o->p, fb_count, fb_list, out_idx, out_dist, out_w);
        MN_KCHECK(s, "k_cos_fallback");
    }
    tm.mark();
    MN_HIP_TRY(hipMemcpyAsync(hb, flags, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    t_bf16_stats.n_uncertified = hb[2];
    t_bf16_stats.algo = MN_KNN_BF16X1;
    t_bf16_stats.slices = (int)pl.S;
    t_bf16_stats.list_len = L1;
    t_bf16_stats.sample_rows = m0;
    t_bf16_stats.sweep_slices = sym ? -1 : S2;
    t_bf16_stats.sweep_cap = cap2;
    if (tm.on) {
        t_bf16_stats.ms_sample = tm.ms(0, 1);
        t_bf16_stats.ms_norms = tm.ms(1, 2);
        t_bf16_stats.ms_sweep = tm.ms(2, 3);
        t_bf16_stats.ms_gram = t_bf16_stats.ms_sample + t_bf16_stats.ms_sweep;
        t_bf16_stats.ms_rerank = tm.ms(3, 4);
        t_bf16_stats.ms_fallback = tm.ms(4, 5);
    }
    return MN_OK;
}

static int knn_cos_bf16_impl(const uint16_t *Q, int64_t nq, const uint16_t *C, int64_t nc,
                             int32_t d, int64_t q_off, int64_t c_off, const mn_cos_opts *o,
                             int32_t *out_idx, double *out_dist, double *out_w) {
    using namespace kb16;
    clear_error();
    t_bf16_stats = mn_knn_stats{};
    MN_REQUIRE(o && Q && C && out_idx && out_dist, MN_EINVAL, "mn_knn_cos_bf16: NULL argument");
    MN_REQUIRE(nq >= 0 && nc >= 0 && d >= 1, MN_EINVAL, "mn_knn_cos_bf16: bad shape");
    MN_REQUIRE(o->topk >= 1 && o->topk <= KMAX, MN_ENOTSUP, "mn_knn_cos_bf16: topk in [1,64]");
    MN_REQUIRE(o->sigma > 0.0, MN_EINVAL, "mn_knn_cos_bf16: sigma must be > 0");
    // candidate margin (rows whose bound does not separate rank topk from the
    // margin are rescanned exactly); clipped so that L = topk + margin <= LMAX
    const int margin = std::min(o->margin > 0 ? o->margin : 16, LMAX - o->topk);
    const int L = o->topk + margin;
    MN_REQUIRE(q_off + nq <= INT_MAX && c_off + nc <= INT_MAX, MN_EINVAL,
               "mn_knn_cos_bf16: ids must fit int32");
    hipStream_t s = (hipStream_t)o->stream;
    t_bf16_stats.n_queries = nq;
    if (nq == 0) return MN_OK;
    const bool same = (Q == C) && nq == nc && q_off == c_off;
    const int excl = 1;
    const GramPlan pl = plan_gram(nq, nc, L, (int64_t)knob_int("MN_BF16_MIN_SLICES", 2));
    const int64_t S = pl.S, chunk = pl.chunk;
    const int cap = pl.cap, NR = pl.NR;
    const int64_t blocks_q = (nq + BM - 1) / BM;
    t_bf16_stats.slices = (int)S;
    t_bf16_stats.list_len = L;

    char *g = (char *)scratch(kSlotNorms, (size_t)(nq + nc) * 12 + 256);
    uint2 *cbuf = (uint2 *)scratch(kSlotLists, (size_t)nq * S * cap * sizeof(uint2) + 64);
    char *meta = (char *)scratch(kSlotListMeta, (size_t)nq * S * 8 + 64);
    int *fb_list = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nq * 2 + 64);
    int *flags = (int *)scratch(kSlotFlags, 64);
    MN_REQUIRE(g && cbuf && meta && fb_list && flags, MN_ENOMEM,
               "mn_knn_cos_bf16: scratch allocation failed (candidate buffer %zu MB)",
               (size_t)nq * S * cap * sizeof(uint2) >> 20);
    double *qn = (double *)g;
    double *cn = same ? qn : qn + nq;
    float *qinv = (float *)(qn + nq + (same ? 0 : nc));
    float *cinv = same ? qinv : qinv + nq;
    int *bcnt = (int *)meta;
    float *btau = (float *)(meta + (size_t)nq * S * 4);

    const bool misaligned = ((uintptr_t)Q & 15) || ((uintptr_t)C & 15);
    if ((d % DALIGN) || misaligned) {
        // exact: appended zero features add +0 to every norm and dot
        const int d8 = (d + DALIGN - 1) / DALIGN * DALIGN;
        uint16_t *Qp = (uint16_t *)scratch(kSlotGeneric0, (size_t)nq * d8 * 2 + 64);
        uint16_t *Cp = same ? Qp : (uint16_t *)scratch(kSlotGeneric1, (size_t)nc * d8 * 2 + 64);
        MN_REQUIRE(Qp && Cp, MN_ENOMEM, "mn_knn_cos_bf16: padded copy allocation failed");
        hipLaunchKernelGGL(k_pad_rows, dim3((unsigned)((nq * d8 + 255) / 256)), dim3(256), 0, s, Q,
                           nq, d, d8, Qp);
        if (!same && nc > 0)
            hipLaunchKernelGGL(k_pad_rows, dim3((unsigned)((nc * d8 + 255) / 256)), dim3(256), 0, s,
                               C, nc, d, d8, Cp);
        MN_KCHECK(s, "k_pad_rows");
        Q = Qp;
        C = Cp;
        d = d8;
    }
    Timer tm;
    tm.start(o->timing != 0, s);
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 64, s));
    hipLaunchKernelGGL(k_bf16_norms, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, Q, nq, d,
                       qn, qinv, flags + 1);
    if (!same && nc > 0)
        hipLaunchKernelGGL(k_bf16_norms, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, C, nc,
                           d, cn, cinv, flags + 1);
    MN_KCHECK(s, "k_bf16_norms");
    int hf[4] = {0, 0, 0, 0};
    MN_HIP_TRY(hipMemcpyAsync(hf, flags, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(hf[1] == 0, MN_ENONFINITE, "mn_knn_cos_bf16: input contains NaN/inf");
    tm.mark();
    {
        // self graphs at scale: the two-phase generator (MN_BF16_X1=0: one phase)
        const char *xe = knob("MN_BF16_X1");
        if (same && !(xe && *xe == '0')) {
            const float ms_norms = tm.on ? tm.ms(0, 1) : 0.f;
            const int rc = knn_cos_bf16_x1(Q, nq, d, o, qn, qinv, flags, fb_list, out_idx, out_dist,
                                           out_w, s);
            if (rc != 1) {
                if (tm.on) {  // + the generator's own sweep-copy interval
                    t_bf16_stats.ms_norms = ms_norms + t_bf16_stats.ms_norms;
                    t_bf16_stats.ms_total = t_bf16_stats.ms_norms + t_bf16_stats.ms_gram +
                                            t_bf16_stats.ms_rerank + t_bf16_stats.ms_fallback;
                }
                return rc;
            }
        }
    }
    if (nc > 0) {
        auto kern = k_gram_bf16<GM_COS, 0>;
#ifdef MN_TUNING
        // timing probes (results invalid): noepi = K loop only, filteronly /
        // nomerge = the epilogue without its list updates
        const char *probe = knob("MN_BF16_PROBE");
        if (probe && *probe)
            kern = !strcmp(probe, "noepi") ? k_gram_bf16<GM_COS, 1>
                   : !strcmp(probe, "filteronly") ? k_gram_bf16<GM_COS, 2>
                   : !strcmp(probe, "nomerge") ? k_gram_bf16<GM_COS, 3> : k_gram_bf16<GM_COS, 0>;
#endif
        hipLaunchKernelGGL(kern, dim3((unsigned)(blocks_q * S)), dim3(NT), 0, s, Q, nq,
                           C, nc, d, q_off, c_off, excl, qinv, cinv, L, (int)S, chunk, cap, cbuf,
                           bcnt, btau);
    } else {
        MN_HIP_TRY(hipMemsetAsync(bcnt, 0, sizeof(int) * (size_t)nq * S, s));
    }
    MN_KCHECK(s, "k_gram_bf16");
    tm.mark();
    const double delta = 2.0 * ((double)d + 12.0) * 0x1p-24;
    const int64_t nvalid = same ? nc - 1 : nc;  // qc callers: exclusion inside the shard
    const dim3 rg((unsigned)((nq + 3) / 4));
#define MN_RR(NRV)                                                                              \
    hipLaunchKernelGGL(k_cos_rerank<NRV>, rg, dim3(256), 0, s, Q, nq, C, d, c_off, qn, cn,       \
                       (int)S, cap, cbuf, bcnt, btau, o->topk, std::max<int64_t>(nvalid, 0),     \
                       delta, o->eps, o->sigma, o->p, out_idx, out_dist, out_w, flags + 2,     \
                       fb_list)
    if (NR == 1) MN_RR(1); else if (NR == 2) MN_RR(2); else if (NR == 4) MN_RR(4); else MN_RR(8);
#undef MN_RR
    MN_KCHECK(s, "k_cos_rerank");
    tm.mark();
    hipLaunchKernelGGL(k_cos_fallback, dim3((unsigned)std::min<int64_t>(nq, 1024)), dim3(FBT), 0, s,
                       Q, C, nc, d, q_off, c_off, excl, qn, cn, o->topk, o->eps, o->sigma, o->p,
                       flags + 2, fb_list, out_idx, out_dist, out_w);
    MN_KCHECK(s, "k_cos_fallback");
    tm.mark();
    MN_HIP_TRY(hipMemcpyAsync(hf, flags, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    t_bf16_stats.n_uncertified = hf[2];
    if (tm.on) {
        t_bf16_stats.ms_norms = tm.ms(0, 1);
        t_bf16_stats.ms_gram = tm.ms(1, 2);
        t_bf16_stats.ms_rerank = tm.ms(2, 3);
        t_bf16_stats.ms_fallback = tm.ms(3, 4);
        t_bf16_stats.ms_total = tm.ms(0, 4);
    }
    return MN_OK;
}

}  // namespace mn

extern "C" {

int mn_knn_cos_bf16(const uint16_t *X, int64_t n, int32_t d, const mn_cos_opts *opts,
                    int32_t *out_idx, double *out_dist, double *out_w) {
    return mn::knn_cos_bf16_impl(X, n, X, n, d, 0, 0, opts, out_idx, out_dist, out_w);
}

int mn_knn_cos_bf16_qc(const uint16_t *Q, int64_t nq, const uint16_t *C, int64_t nc, int32_t d,
                       int64_t q_offset, int64_t c_offset, const mn_cos_opts *opts,
                       int32_t *out_idx, double *out_dist, double *out_w) {
    return mn::knn_cos_bf16_impl(Q, nq, C, nc, d, q_offset, c_offset, opts, out_idx, out_dist,
                                 out_w);
}

int mn_bf16_last_stats(mn_knn_stats *out) {
    if (!out) return MN_EINVAL;
    *out = mn::t_bf16_stats;
    return MN_OK;
}

}  // extern "C"
