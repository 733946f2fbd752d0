// sorted_index.hip — K4: the lambda-sorted index (SortedLambdas).
//
// Reference semantics (src_legacy/sorted_index.rs:22-54, core.rs:938-940):
//   build_from(lambdas): for i ascending, zadd(lambda_i, i, i.to_string());
//   BTreeMap<OrderedFloat<f64>, bucket> => ascending OrderedFloat order (all
//   NaN equal and greatest, -0.0 == +0.0); inside a bucket the entries are
//   re-sorted by the decimal-string id after every insert => ties ordered by
//   the string ("10" < "2").  to_vec() yields (bucket key, idx), where the key
//   is the first-inserted (smallest idx) lambda of the bucket.
//   std_dev: laplacian.rs:421-448 std_deviation (f64 sum -> f32 mean, f32
//   squared deviations).
//
// GPU design: every element gets a unique composite key
//   (sortable 64-bit OrderedFloat key of lambda, lexrank(idx)) where
//   lexrank(i) is the rank of i's decimal string among "0".."N-1", computed in
//   closed form per element (digit DP, no strings) — so the BTreeMap +
//   per-insert bucket re-sort (quadratic under ties, Appendix B.10) becomes ONE
//   bitonic sort: LDS-fused stages for j < 2048, global stages above.
//   Bit-exact order given identical lambdas.
#include <algorithm>
#include <climits>
#include <cmath>

#include <cstdlib>

#include "common.hpp"
#include "glibc_f64.hpp"
#include "scan.hpp"

namespace mn {
namespace sidx {

struct alignas(16) Key {
    unsigned long long k1;  // OrderedFloat key
    uint32_t k2;            // lexrank(idx)
    uint32_t idx;
};

__device__ __forceinline__ bool key_lt(const Key &a, const Key &b) {
    return a.k1 < b.k1 || (a.k1 == b.k1 && a.k2 < b.k2);
}

// OrderedFloat<f64> total order: -0 == +0, every NaN equal and greatest
__device__ __forceinline__ unsigned long long of_key(double x) {
    if (x != x) return ~0ull;
    if (x == 0.0) x = 0.0;  // canonicalise -0.0
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// numbers in [0, N) whose decimal string starts with the digits of v (v > 0)
__device__ __forceinline__ int64_t count_with_prefix(int64_t v, int64_t N) {
    int64_t c = 0, lo = v, hi = v;
    while (lo < N) {
        c += min(hi, N - 1) - lo + 1;
        if (lo > (INT64_MAX - 9) / 10) break;
        lo *= 10;
        hi = hi * 10 + 9;
    }
    return c;
}

// rank of str(i) among {str(0), ..., str(N-1)} in byte-lexicographic order
__device__ int64_t lexrank(int64_t i, int64_t N) {
    if (i == 0) return 0;
    int dig[20];
    int L = 0;
    for (int64_t t = i; t > 0; t /= 10) dig[L++] = (int)(t % 10);
    // digits most-significant first: dig[L-1] ... dig[0]
    int64_t r = (L - 1) + 1;  // proper prefixes + "0"
    int64_t pre = 0;
    for (int p = 0; p < L; ++p) {
        const int sp = dig[L - 1 - p];
        for (int c = (p == 0 ? 1 : 0); c < sp; ++c) r += count_with_prefix(pre * 10 + c, N);
        pre = pre * 10 + sp;
    }
    return r;
}

__global__ __launch_bounds__(256) void k_make_keys(const double *__restrict__ lam, int64_t n,
                                                   int64_t P, Key *__restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    Key k;
    if (i < n) {
        k.k1 = of_key(lam[i]);
        k.k2 = (uint32_t)lexrank(i, n);
        k.idx = (uint32_t)i;
    } else {  // padding sorts last
        k.k1 = ~0ull;
        k.k2 = 0xFFFFFFFFu;
        k.idx = 0xFFFFFFFFu;
    }
    keys[i] = k;
}

constexpr int TILE = 2048;  // LDS-fused bitonic tile (32 KB of keys)

// all stages with j < TILE for a given kk (and the full local sort when kk <= TILE)
__global__ __launch_bounds__(1024) void k_bitonic_local(Key *__restrict__ keys, int64_t P,
                                                        int64_t kk_from, int64_t kk_to) {
    __shared__ Key sm[TILE];
    const int64_t base = (int64_t)blockIdx.x * TILE;
    for (int e = threadIdx.x; e < TILE; e += blockDim.x) sm[e] = keys[base + e];
    __syncthreads();
    for (int64_t kk = kk_from; kk <= kk_to; kk <<= 1) {
        const int jstart = (int)((kk >> 1) < (int64_t)(TILE >> 1) ? (kk >> 1) : (TILE >> 1));
        for (int j = jstart; j > 0; j >>= 1) {
            for (int e = threadIdx.x; e < TILE; e += blockDim.x) {
                const int pe = e ^ j;
                if (pe > e) {
                    const int64_t ge = base + e;
                    const bool asc = (ge & kk) == 0;
                    const bool sw = asc ? key_lt(sm[pe], sm[e]) : key_lt(sm[e], sm[pe]);
                    if (sw) { Key t = sm[e]; sm[e] = sm[pe]; sm[pe] = t; }
                }
            }
            __syncthreads();
        }
    }
    for (int e = threadIdx.x; e < TILE; e += blockDim.x) keys[base + e] = sm[e];
}

__global__ __launch_bounds__(256) void k_bitonic_global(Key *__restrict__ keys, int64_t P,
                                                        int64_t kk, int64_t j) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P) return;
    const int64_t pe = e ^ j;
    if (pe <= e) return;
    const bool asc = (e & kk) == 0;
    const Key a = keys[e], b = keys[pe];
    const bool sw = asc ? key_lt(b, a) : key_lt(a, b);
    if (sw) { keys[e] = b; keys[pe] = a; }
}

// run starts (bucket boundaries) + per-run min index for the bucket key
__global__ __launch_bounds__(256) void k_run_flags(const Key *__restrict__ keys, int64_t n,
                                                   int32_t *__restrict__ start) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    start[r] = (r == 0 || keys[r].k1 != keys[r - 1].k1) ? 1 : 0;
}
__global__ __launch_bounds__(256) void k_run_min(const Key *__restrict__ keys, int64_t n,
                                                 const int32_t *__restrict__ start,
                                                 const int64_t *__restrict__ pos,
                                                 unsigned *__restrict__ run_min) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t run = pos[r] + start[r] - 1;  // inclusive scan - 1
    atomicMin(&run_min[run], keys[r].idx);
}
__global__ __launch_bounds__(256) void k_emit(const Key *__restrict__ keys, int64_t n,
                                              const int32_t *__restrict__ start,
                                              const int64_t *__restrict__ pos,
                                              const unsigned *__restrict__ run_min,
                                              const double *__restrict__ lam,
                                              int64_t *__restrict__ order,
                                              double *__restrict__ key_out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    order[r] = keys[r].idx;
    if (key_out) {
        const int64_t run = pos[r] + start[r] - 1;
        key_out[r] = lam[run_min[run]];
    }
}

// laplacian.rs:421-448 std_deviation, reproduced bit-for-bit: the reference
// folds sequentially (f64 sum -> f32 mean, then an f32 sum of squared
// deviations), and no parallel order reproduces that rounding, so the adds
// stay one dependent chain.  What is NOT sequential is everything around it:
// one wave streams 256-value chunks (4 consecutive values per lane, the next
// chunk in flight) into LDS, and the chain reads them back as broadcast
// ds_read_b128 (all lanes, same address: conflict-free), so the VALU issues
// little but the chain's adds (pass 2: the squared deviations are formed
// lane-parallel before the chain).  The host runs it on a side stream,
// concurrent with the sort.
constexpr int STD_CHUNK = 256;  // values per chunk: 64 lanes x 4

constexpr int STD_PF = 4;  // chunks in flight ahead of the chain

// Pass 1 certified in parallel.  Pass 1 only feeds (f32) of the f64 sum, so
// its bits are known whenever every value the sequential fold can take rounds
// to the same f32: the fold lies within gamma_n * sum|x| (u = 2^-53) of the
// exact sum, which a double-double reduction gives to ~n u^2 sum|x|.  When
// that interval straddles an f32 rounding boundary (rarely: its width is
// ~1e-10 relative against an f32 ulp of 6e-8 at n = 1e6), or a value is not
// finite, the sequential pass 1 runs as before.  Pass 2's f32 chain stays
// sequential (its rounding is large and order-dependent).
constexpr int SUM_BLOCKS = 512;

__device__ __forceinline__ void two_sum(double a, double b, double &s, double &e) {
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}
__device__ __forceinline__ void dd_add(double &hi, double &lo, double x) {
    double s, e;
    two_sum(hi, x, s, e);
    e += lo;
    two_sum(s, e, hi, lo);
}

// per block: double-double sum of lam and f64 sum of |lam| (+ non-finite flag)
__global__ __launch_bounds__(256) void k_sum_dd(const double *__restrict__ lam, int64_t n,
                                               double *__restrict__ part) {
    __shared__ double sh[3][256];
    double hi = 0.0, lo = 0.0, ab = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)SUM_BLOCKS * 256) {
        const double v = lam[i];
        dd_add(hi, lo, v);
        ab += __builtin_fabs(v);  // NaN / inf propagate: the check below fails
    }
    sh[0][threadIdx.x] = hi; sh[1][threadIdx.x] = lo; sh[2][threadIdx.x] = ab;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            double h = sh[0][threadIdx.x], l = sh[1][threadIdx.x];
            dd_add(h, l, sh[0][threadIdx.x + o]);
            dd_add(h, l, sh[1][threadIdx.x + o]);
            sh[0][threadIdx.x] = h; sh[1][threadIdx.x] = l;
            sh[2][threadIdx.x] += sh[2][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x] = sh[0][0];
        part[3 * blockIdx.x + 1] = sh[1][0];
        part[3 * blockIdx.x + 2] = sh[2][0];
    }
}

__global__ __launch_bounds__(64) void k_std_exact(const double *__restrict__ lam, int64_t n,
                                                  const double *__restrict__ part,
                                                  float *__restrict__ out, int *__restrict__ seq) {
    __shared__ double b64[2][STD_CHUNK];
    __shared__ float b32[2][STD_CHUNK];
    const int lane = threadIdx.x;
    const int64_t nfull = n / STD_CHUNK;
    double ring[STD_PF][4];
    auto fetch = [&](int64_t c, double (&p)[4]) {
#pragma unroll
        for (int t = 0; t < 4; ++t) p[t] = lam[c * STD_CHUNK + 4 * lane + t];
    };
    // ---- pass 1: s = sum(lam) in index order (f64), certified from the
    // double-double partials when possible ----
    bool certified = false;
    float sf = 0.0f;
    if (part) {
        double hi = 0.0, lo = 0.0, ab = 0.0;
        for (int b = 0; b < SUM_BLOCKS; ++b) {  // every lane the same (uniform)
            dd_add(hi, lo, part[3 * b]);
            dd_add(hi, lo, part[3 * b + 1]);
            ab += part[3 * b + 2];
        }
        const double u = 0x1p-53, nn = (double)n;
        // sequential-fold bound gamma_n * sum|x| plus the double-double
        // reduction's own error, an ulp of hi and |lo|, all inflated
        const double E = (nn * u / (1.0 - nn * u)) * ab * (1.0 + 0x1p-20) +
                         8.0 * (nn + SUM_BLOCKS) * u * u * ab + __builtin_fabs(lo) +
                         __builtin_fabs(hi) * 0x1p-52 + 0x1p-1000;
        if (__builtin_isfinite(hi) && __builtin_isfinite(ab) && __builtin_isfinite(E)) {
            const float a = (float)(hi - E), b = (float)(hi + E);
            if (a == b) { certified = true; sf = a; }
        }
    }
    double s = -0.0;
    if (!certified) {
#pragma unroll
    for (int u = 0; u < STD_PF; ++u)
        if (u < nfull) fetch(u, ring[u]);
    for (int64_t c0 = 0; c0 < nfull; c0 += STD_PF) {
#pragma unroll
        for (int u = 0; u < STD_PF; ++u) {
            const int64_t c = c0 + u;
            if (c >= nfull) break;
            double *bb = b64[u & 1];
#pragma unroll
            for (int t = 0; t < 4; ++t) bb[4 * lane + t] = ring[u][t];
            if (c + STD_PF < nfull) fetch(c + STD_PF, ring[u]);
            __builtin_amdgcn_wave_barrier();
            s = lds_chain_f64<STD_CHUNK>(s, bb);
            __builtin_amdgcn_wave_barrier();
        }
    }
    for (int64_t i = nfull * STD_CHUNK; i < n; ++i) s = s + lam[i];
    sf = (float)s;
    }
    if (threadIdx.x == 0 && seq) *seq = certified ? 0 : 1;
    const float mean = __fdiv_rn(sf, (float)n);
    // ---- pass 2: var = sum((mean - (f32)lam)^2) in index order (f32) ----
    float var = -0.0f;
#pragma unroll
    for (int u = 0; u < STD_PF; ++u)
        if (u < nfull) fetch(u, ring[u]);
    for (int64_t c0 = 0; c0 < nfull; c0 += STD_PF) {
#pragma unroll
        for (int u = 0; u < STD_PF; ++u) {
            const int64_t c = c0 + u;
            if (c >= nfull) break;
            float *bb = b32[u & 1];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float dv = mean - (float)ring[u][t];
                bb[4 * lane + t] = dv * dv;
            }
            if (c + STD_PF < nfull) fetch(c + STD_PF, ring[u]);
            __builtin_amdgcn_wave_barrier();
            var = lds_chain_f32<STD_CHUNK>(var, bb);
            __builtin_amdgcn_wave_barrier();
        }
    }
    for (int64_t i = nfull * STD_CHUNK; i < n; ++i) {
        const float dv = mean - (float)lam[i];
        var = var + dv * dv;
    }
    if (lane == 0) *out = sqrt_rn_f32(__fdiv_rn(var, (float)n));
}

// ---- lambda-aware lookups (sorted_index.rs:64-140) ---------------------------
// keys[] is non-decreasing in OrderedFloat order; searches run on of_key().
__device__ __forceinline__ int64_t lower_rank(const double *keys, int64_t n, unsigned long long kv) {
    int64_t lo = 0, hi = n;  // first rank with key >= kv
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (of_key(keys[mid]) < kv) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int64_t upper_rank(const double *keys, int64_t n, unsigned long long kv) {
    int64_t lo = 0, hi = n;  // first rank with key > kv
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (of_key(keys[mid]) <= kv) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_range_bylambda(const double *__restrict__ keys,
                                                        const int64_t *__restrict__ order,
                                                        int64_t n, double band,
                                                        const double *__restrict__ lq, int64_t nq,
                                                        int k, int64_t *__restrict__ oi,
                                                        double *__restrict__ ol,
                                                        int32_t *__restrict__ oc) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const double q = lq[t];
    const unsigned long long klo = of_key(q - band), khi = of_key(q + band);
    int cnt = 0;
    if (klo > khi) {
        cnt = -1;  // BTreeMap::range panics: start > end
    } else {
        const int64_t r0 = lower_rank(keys, n, klo), r1 = upper_rank(keys, n, khi);
        cnt = (int)min<int64_t>(k, max<int64_t>(0, r1 - r0));
        for (int e = 0; e < cnt; ++e) {
            oi[t * k + e] = order[r0 + e];
            ol[t * k + e] = keys[r0 + e];
        }
    }
    for (int e = max(cnt, 0); e < k; ++e) {
        oi[t * k + e] = -1;
        ol[t * k + e] = __builtin_nan("");
    }
    oc[t] = cnt;
}

__global__ __launch_bounds__(256) void k_nearest_bylambda(
    const double *__restrict__ keys, const int64_t *__restrict__ order, int64_t n, double delta0,
    double growth, double max_delta, const double *__restrict__ lq, int64_t nq, int k,
    int64_t *__restrict__ oi, double *__restrict__ ol, int32_t *__restrict__ oc) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const double q = lq[t];
    double delta = delta0;
    int64_t r0 = 0, r1 = 0;
    int cnt = 0;
    for (;;) {  // sorted_index.rs:110-126 (f64::max / f64::min ignore NaN, like fmax / fmin)
        const double lo = fmax(q - delta, 0.0), hi = fmin(q + delta, 1.0);
        const unsigned long long klo = of_key(lo), khi = of_key(hi);
        if (klo > khi) { cnt = -1; break; }  // BTreeMap::range panics
        r0 = lower_rank(keys, n, klo);
        r1 = upper_rank(keys, n, khi);
        if (r1 - r0 >= k || delta >= max_delta) break;
        delta = fmin(delta * growth, max_delta);
    }
    if (cnt == 0 && r1 > r0) {
        const int64_t m = r1 - r0;
        if (q != q && m >= 2) {
            cnt = -1;  // |lambda - NaN| is NaN: partial_cmp().unwrap() panics
        } else {
            // k smallest |key - q| with ties in rank order: the distance is
            // non-increasing toward q from the left and non-decreasing from the
            // right, so merge outward from q's position, run by run
            auto dist = [&](int64_t r) { return fabs(keys[r] - q); };
            int64_t L = lower_rank(keys, n, of_key(q));
            L = min(max(L, r0), r1) - 1;  // left pointer (descending)
            int64_t R = L + 1;           // right pointer (ascending)
            while (cnt < k && (L >= r0 || R < r1)) {
                const double dl = L >= r0 ? dist(L) : __builtin_inf();
                const double dr = R < r1 ? dist(R) : __builtin_inf();
                const bool take_left = L >= r0 && (R >= r1 || dl <= dr);
                const double d = take_left ? dl : dr;
                if (take_left) {
                    // left run: ranks [Ls, L] with distance d (first rank <= L
                    // whose distance is <= d, by bisection)
                    int64_t a = r0, b = L;
                    while (a < b) {
                        const int64_t mid = (a + b) >> 1;
                        if (dist(mid) <= d) b = mid; else a = mid + 1;
                    }
                    for (int64_t r = a; r <= L && cnt < k; ++r, ++cnt) {
                        oi[t * k + cnt] = order[r];
                        ol[t * k + cnt] = keys[r];
                    }
                    L = a - 1;
                }
                if (R < r1 && (!take_left || dr == d)) {
                    // right run: ranks [R, Re] with distance d
                    int64_t a = R, b = r1 - 1;
                    while (a < b) {
                        const int64_t mid = (a + b + 1) >> 1;
                        if (dist(mid) <= d) a = mid; else b = mid - 1;
                    }
                    for (int64_t r = R; r <= a && cnt < k; ++r, ++cnt) {
                        oi[t * k + cnt] = order[r];
                        ol[t * k + cnt] = keys[r];
                    }
                    R = a + 1;
                }
            }
        }
    }
    for (int e = max(cnt, 0); e < k; ++e) {
        oi[t * k + e] = -1;
        ol[t * k + e] = __builtin_nan("");
    }
    oc[t] = cnt;
}

inline unsigned grid(int64_t n, int t = 256) {
    return (unsigned)std::max<int64_t>(1, (n + t - 1) / t);
}

}  // namespace sidx

static int sorted_index_impl(const double *lam, int64_t n, int64_t *order, double *key_out,
                             double *std_host, void *stream) {
    using namespace sidx;
    clear_error();
    MN_REQUIRE(n >= 0 && (n == 0 || (lam && order)), MN_EINVAL, "mn_sorted_index: bad args");
    MN_REQUIRE(n <= 0xFFFFFFFELL, MN_EINVAL, "mn_sorted_index: n too large");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return MN_OK;
    int64_t P = TILE;
    while (P < n) P <<= 1;
    Key *keys = (Key *)scratch(kSlotGeneric1, sizeof(Key) * (size_t)P);
    char *aux = (char *)scratch(kSlotGeneric2, (size_t)n * 16 + ((size_t)n / scan::SB + 2) * 8 + 64);
    MN_REQUIRE(keys && aux, MN_ENOMEM, "mn_sorted_index: scratch allocation failed");
    int32_t *start = (int32_t *)aux;
    unsigned *run_min = (unsigned *)(start + n);
    int64_t *pos = (int64_t *)(((uintptr_t)(run_min + n) + 15) & ~(uintptr_t)15);
    int64_t *part = pos + (n + 1);
    double *sums = (double *)scratch(kSlotFlags, 64);
    MN_REQUIRE(sums, MN_ENOMEM, "mn_sorted_index: scratch allocation failed");

    // std_deviation is a sequential fold independent of the sort: it runs on
    // the library's side stream (ordered after the caller's prior work on s)
    hipStream_t side = nullptr;
    if (std_host) {
        side = side_stream();
        MN_REQUIRE(side, MN_EHIP, "mn_sorted_index: side stream creation failed");
        MN_HIP_TRY(stream_wait(side, s));
        // pass-1 certificate partials (the sequential pass 1 runs only if it
        // fails); MN_STD_SEQ=1 forces the sequential pass (tests)
        const char *fs = knob("MN_STD_SEQ");
        const bool force_seq = fs && *fs == '1';
        double *part1 = force_seq ? nullptr : (double *)scratch(kSlotNorms2, sizeof(double) * 3 * SUM_BLOCKS + 64);
        if (part1) {
            hipLaunchKernelGGL(k_sum_dd, dim3(SUM_BLOCKS), dim3(256), 0, side, lam, n, part1);
            MN_KCHECK(side, "k_sum_dd");
        }
        hipLaunchKernelGGL(k_std_exact, dim3(1), dim3(64), 0, side, lam, n, (const double *)part1,
                           (float *)sums, (int *)(sums + 1));
        MN_KCHECK(side, "k_std_exact");
    }
    hipLaunchKernelGGL(k_make_keys, dim3(grid(P)), dim3(256), 0, s, lam, n, P, keys);
    // local sort of every TILE, then merge levels: global stages j >= TILE, local j < TILE
    hipLaunchKernelGGL(k_bitonic_local, dim3((unsigned)(P / TILE)), dim3(1024), 0, s, keys, P,
                       (int64_t)2, (int64_t)TILE);
    for (int64_t kk = 2 * TILE; kk <= P; kk <<= 1) {
        for (int64_t j = kk >> 1; j >= TILE; j >>= 1)
            hipLaunchKernelGGL(k_bitonic_global, dim3(grid(P)), dim3(256), 0, s, keys, P, kk, j);
        hipLaunchKernelGGL(k_bitonic_local, dim3((unsigned)(P / TILE)), dim3(1024), 0, s, keys, P,
                           kk, kk);
    }
    MN_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_run_flags, dim3(grid(n)), dim3(256), 0, s, keys, n, start);
    // inclusive run id = exclusive scan + flag
    MN_HIP_TRY(scan::exclusive_scan(start, n, pos, part, s));
    MN_HIP_TRY(hipMemsetAsync(run_min, 0xFF, sizeof(unsigned) * (size_t)n, s));
    hipLaunchKernelGGL(k_run_min, dim3(grid(n)), dim3(256), 0, s, keys, n, start, pos, run_min);
    hipLaunchKernelGGL(k_emit, dim3(grid(n)), dim3(256), 0, s, keys, n, start, pos, run_min, lam,
                       order, key_out);
    if (std_host) {
        MN_HIP_TRY(stream_wait(s, side));
        float sd = 0.f;
        MN_HIP_TRY(hipMemcpyAsync(&sd, sums, 4, hipMemcpyDeviceToHost, s));
        MN_HIP_TRY(hipStreamSynchronize(s));
        *std_host = (double)sd;
    }
    MN_HIP_TRY(hipGetLastError());
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

}  // namespace mn

extern "C" int mn_sorted_index(const double *lambda, int64_t n, int64_t *order_out,
                               double *key_out, double *std_out_host, void *stream) {
    return mn::sorted_index_impl(lambda, n, order_out, key_out, std_out_host, stream);
}

extern "C" int mn_sorted_range_bylambda(const double *keys, const int64_t *order, int64_t n,
                                        double std_dev, const double *lambda_q, int64_t nq,
                                        int32_t k, double p, int64_t *out_idx, double *out_lambda,
                                        int32_t *out_count, void *stream) {
    using namespace mn::sidx;
    mn::clear_error();
    MN_REQUIRE(n >= 0 && nq >= 0 && k >= 0, MN_EINVAL, "mn_sorted_range_bylambda: bad sizes");
    MN_REQUIRE(nq == 0 || (lambda_q && out_idx && out_lambda && out_count && (n == 0 || (keys && order))),
               MN_EINVAL, "mn_sorted_range_bylambda: NULL pointer");
    if (nq == 0) return MN_OK;
    hipStream_t s = (hipStream_t)stream;
    // sorted_index.rs:65 `2.0_f64.powf(p)`: llvm.pow(2.0, p), which LLVM's
    // library-call simplifier rewrites to exp2(p) in an optimised build
    // (replacePowWithExp, no fast-math needed) — the host libm's exp2 here.
    // glibc pow(2, p) and exp2(p) differ in ~0.1 % of fractional p; a debug
    // build of the reference calls pow and may differ there.
    const double band = std_dev / ::exp2(p);
    hipLaunchKernelGGL(k_range_bylambda, dim3(grid(nq)), dim3(256), 0, s, keys, order, n, band,
                       lambda_q, nq, k, out_idx, out_lambda, out_count);
    MN_HIP_TRY(hipGetLastError());
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

extern "C" int mn_sorted_k_nearest_by_lambda(const double *keys, const int64_t *order, int64_t n,
                                             double std_dev, const double *lambda_q, int64_t nq,
                                             int32_t k, double lambda_p, int32_t has_base_delta,
                                             double base_delta, double growth,
                                             double max_multiplier, int64_t *out_idx,
                                             double *out_lambda, int32_t *out_count,
                                             void *stream) {
    using namespace mn::sidx;
    mn::clear_error();
    MN_REQUIRE(n >= 0 && nq >= 0 && k >= 0, MN_EINVAL, "mn_sorted_k_nearest_by_lambda: bad sizes");
    MN_REQUIRE(nq == 0 || (lambda_q && out_idx && out_lambda && out_count && (n == 0 || (keys && order))),
               MN_EINVAL, "mn_sorted_k_nearest_by_lambda: NULL pointer");
    if (nq == 0) return MN_OK;
    hipStream_t s = (hipStream_t)stream;
    if (k == 0 || n == 0) {  // sorted_index.rs:94-96: empty result
        MN_HIP_TRY(hipMemsetAsync(out_count, 0, sizeof(int32_t) * (size_t)nq, s));
        MN_HIP_TRY(hipStreamSynchronize(s));
        return MN_OK;
    }
    // sorted_index.rs:97-106 (f64::max / min: fmax / fmin; abs after unwrap)
    const double delta0 = fabs(has_base_delta ? base_delta : fmax(std_dev * lambda_p, 1e-9));
    const double g = (std::isfinite(growth) && growth > 1.0) ? growth : 1.7;
    const double max_delta = fmin(delta0 * fmax(max_multiplier, 1.0), 1.0);
    hipLaunchKernelGGL(k_nearest_bylambda, dim3(grid(nq)), dim3(256), 0, s, keys, order, n, delta0,
                       g, max_delta, lambda_q, nq, k, out_idx, out_lambda, out_count);
    MN_HIP_TRY(hipGetLastError());
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}
