// energy.hip — K3: per-row Rayleigh energy / Dirichlet dispersion / taumode
// lambda against a sparse F x F feature Laplacian, and lambda normalisation.
//
// Reference semantics (per item row x, f32 storage widened to f64):
//   src_legacy/taumode.rs:261-318 compute_synthetic_lambda
//     zero vector (all |x_t| <= 1e-10) -> lambda 0;  tau = select_tau(x)
//     (:29-70: Fixed / Mean / Median / Percentile over the row's values,
//     floor 1e-10); lambda = tau*E/(E+tau) + (1-tau)*clamp(G,0,1)
//   :326-361 E = max(0, sum_i sum_j x_i L_ij x_j / sum x^2)  (den > 1e-12)
//   :366-408 G = sum over ordered pairs i != j of (e_ij/S)^2,
//            e_ij = max(0,-L_ij)(x_i-x_j)^2, S = sum e_ij (S <= 1e-12 -> 0)
//   src_legacy/energymaps.rs:923-1045 node_energy_and_dispersion: same E,
//     G over j > i only (lambda := E)
//   src_legacy/core.rs:1341-1354 normalise_lambdas (min fold +inf, max fold 0)
//
// Tolerance contract: rel 1e-9 — the reference itself sums E
// in rayon par_bridge order.  Here: G = Q/S^2 with Q = sum e^2 (one pass,
// algebraically identical to sum (e/S)^2, within ~nnz*u relative).
//
// GPU design.  The Laplacian is flattened once per call into two entry lists
// (entry_class below): A = the dispersion's edges (w = -L_ij > 0), which feed
// the Rayleigh numerator, S and Q; B = everything that feeds only the
// numerator.  For an exactly symmetric L only the upper triangle is listed
// (multiplicity 2, applied once per row).  Both lists live in LDS, shared by
// the block's waves.  A wave takes TWO item rows at a time: they are staged
// in LDS (f32) for the x_i / x_j gathers, and each entry read from LDS serves
// both rows (per entry and row: 7 f64 VALU ops, 2 LDS gathers, half an entry
// read).  tau = median via an exact wave-level radix select on the sortable
// f32 keys (no sort).  f64 accumulation throughout.  This orientation is
// compute-bound (F^2-ish entries per F-long row), not HBM-bound: the roofline
// that applies is the f64 VALU rate.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "common.hpp"

namespace mn {
namespace energy {

constexpr int FMAX = 4096;             // row length limit (registers: FMAX/64 per lane)
constexpr size_t LDS_BUDGET = 160 * 1024;
constexpr size_t EDGE_LDS_MAX = 96 * 1024;  // entry lists kept in LDS up to this size

// ---- build the entry lists from CSR --------------------------------------
// Laplacian values: f64 (legacy GraphLaplacian) or f32 (Stage C CsMat<f32>)
struct Vals {
    const void *p;
    int f32;
    __device__ __forceinline__ double operator[](int64_t i) const {
        return f32 ? (double)((const float *)p)[i] : ((const double *)p)[i];
    }
};

// Symmetry / range / order check of an n x n CSR (round 4: one wave per row,
// lanes over the row's entries; the round-3 form — a thread per entry that
// first located its row by an upper-bound search on indptr — spent most of
// its 1.6 ms at C3 on those dependent searches).  Every stored upper entry
// (i, j > i) must find a stored (j, i) with the same value (binary search of
// row j), and the stored upper and lower entry counts must be equal
// (ucount[0] += #upper - #lower per block): the matches map the upper
// entries into the lower ones injectively, so equal counts make it a
// bijection — the same verdict as searching every off-diagonal entry, and a
// stricter one for duplicated entries (an (i, j) stored twice against one
// (j, i) is asymmetric here, as the symmetric lists' multiplicity 2 would
// double-count it).
// asym bit 1: asymmetric; bit 2: a column index out of range; bit 4: a row
// whose columns are not strictly ascending.
__global__ __launch_bounds__(256) void k_check_sym(const int64_t *__restrict__ ip,
                                                   const int32_t *__restrict__ ix, Vals v, int n,
                                                   int *__restrict__ asym,
                                                   unsigned long long *__restrict__ ucount) {
    __shared__ int bal[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    int d = 0;  // +1 upper, -1 lower
    int bad = 0;
    for (int64_t i = (int64_t)blockIdx.x * 4 + wv; i < n; i += nw) {
        const int64_t a0 = ip[i], b0 = ip[i + 1];
        for (int64_t p = a0 + lane; p < b0; p += 64) {
            const int j = ix[p];
            if (p + 1 < b0 && !(ix[p + 1] > j)) bad |= 4;
            if (j < 0 || j >= n) {
                bad |= 2;
            } else if (j < i) {
                d -= 1;
            } else if (j > i) {
                d += 1;
                int64_t a = ip[j], b = ip[j + 1] - 1, hit = -1;
                while (a <= b) {
                    const int64_t mid = (a + b) >> 1;
                    const int c = ix[mid];
                    if (c == i) { hit = mid; break; }
                    if (c < i) a = mid + 1; else b = mid - 1;
                }
                if (hit < 0 || v[hit] != v[p]) bad |= 1;
            }
        }
    }
    // one flag atomic per wave that found something, one balance atomic per block
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        d += __shfl_xor(d, o);
        bad |= __shfl_xor(bad, o);
    }
    if (lane == 0 && bad) atomicOr(asym, bad);
    if (lane == 0) bal[wv] = d;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tb = bal[0] + bal[1] + bal[2] + bal[3];
        if (tb != 0) atomicAdd(ucount, (unsigned long long)(long long)tb);
    }
}

// grid of the check: a wave per row, at most 32768 blocks (grid-stride beyond)
inline unsigned check_sym_grid(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, 32768)); }

// Every stored CSR entry (i, j, v) the reduction needs goes to one list,
// packed (i | j << 16) + an f64 value:
//   A (0)  off-diagonal, w = -v > 0, in the dispersion's pair set: value w;
//          feeds num (as -w), S and Q with the uniform multiplicities
//          (mA_num, mA_g) applied once to the row's sums;
//   B (1)  everything else (the diagonal, v >= 0, pairs outside the
//          dispersion's set): value m * v, feeds num only.
// Symmetric L: only j >= i is listed, off-diagonal multiplicity 2.  Pair set:
// taumode = ordered pairs i != j (taumode.rs:366-408), energymaps = j > i
// (energymaps.rs:990-1030), spectral = ordered pairs with W = max(0, -L)
// (spectral/mod.rs:115-140: the diagonal's (x_f - x_f)^2 term is 0).
//   D (2)  the diagonal, when split_diag (k_energy_rows2): summed per feature
//          into dg[i] and applied from the lane's own row registers.
__device__ __forceinline__ int entry_class(int i, int j, double v, int sym, int g_mode,
                                           int split_diag = 0) {
    if (sym && j < i) return -1;  // covered by (j, i)
    if (i == j) return split_diag ? 2 : 1;
    const bool counts = (g_mode != MN_G_ENERGYMAPS) || sym || j > i;
    return (counts && -v > 0.0) ? 0 : 1;
}

__global__ void k_count_entries(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                                Vals v, int f, int sym, int g_mode, int split_diag,
                                int32_t *__restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= f) return;
    int ca = 0, cb = 0;
    for (int64_t p = ip[i]; p < ip[i + 1]; ++p) {
        const int c = entry_class(i, ix[p], v[p], sym, g_mode, split_diag);
        ca += c == 0;
        cb += c == 1;
    }
    cnt[i] = ca;
    cnt[f + i] = cb;
}

// ident (k_energy_rows3, symmetric L): dg[i] = L_ii - dgA_i with dgA_i = the
// row's list-A weight sum over BOTH triangles (sum of -L_ij > 0, j != i), so
// that the list-A part of x^T L x needs no x_i x_j products (see rows3).
__global__ void k_fill_entries(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                               Vals v, int f, int sym, int g_mode, int split_diag,
                               const int64_t *__restrict__ off, uint32_t *__restrict__ eij,
                               double *__restrict__ ev, double *__restrict__ dg, int ident = 0) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= f) return;
    int64_t qa = off[i], qb = off[f + i];
    double di = 0.0;  // the row's diagonal entries in CSR order (one thread: deterministic)
    double da = 0.0;  // ident: the row's list-A weights, both triangles, CSR order
    for (int64_t p = ip[i]; p < ip[i + 1]; ++p) {
        const int j = ix[p];
        if (ident && j != i && -v[p] > 0.0) da += -v[p];
        const int c = entry_class(i, j, v[p], sym, g_mode, split_diag);
        if (c == 2) {
            di += v[p];
            continue;
        }
        if (c < 0) continue;
        const int64_t q = c == 0 ? qa++ : qb++;
        eij[q] = (uint32_t)i | ((uint32_t)j << 16);
        ev[q] = c == 0 ? -v[p] : ((sym && i != j) ? 2.0 * v[p] : v[p]);
    }
    if (split_diag) dg[i] = ident ? di - da : di;
}

// ---- wave-level exact order statistic on f32 keys -------------------------
__device__ __forceinline__ uint32_t f2key(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return __uint_as_float(u);
}

// rank-th smallest key (0-based) among keys[0..nr) per lane (all lanes' keys)
template <int NR>
__device__ uint32_t wave_select(const uint32_t (&keys)[NR], int nr, int rank, int *hist) {
    const int lane = threadIdx.x & 63;
    uint32_t prefix = 0, mask = 0;
    int target = rank;
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        hist[lane * 4 + 0] = 0; hist[lane * 4 + 1] = 0;
        hist[lane * 4 + 2] = 0; hist[lane * 4 + 3] = 0;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < NR; ++r)
            if (r < nr && (keys[r] & mask) == prefix) atomicAdd(&hist[(keys[r] >> shift) & 255], 1);
        __builtin_amdgcn_wave_barrier();
        const int c0 = hist[lane * 4], c1 = hist[lane * 4 + 1], c2 = hist[lane * 4 + 2],
                  c3 = hist[lane * 4 + 3];
        const int tot = c0 + c1 + c2 + c3;
        int incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const int excl = incl - tot;
        const bool mine = target >= excl && target < incl;
        int bin = 0, before = excl;
        if (mine) {
            if (target < excl + c0) { bin = 0; }
            else if (target < excl + c0 + c1) { bin = 1; before += c0; }
            else if (target < excl + c0 + c1 + c2) { bin = 2; before += c0 + c1; }
            else { bin = 3; before += c0 + c1 + c2; }
        }
        const uint64_t who = __ballot(mine);
        const int src = (int)__builtin_ctzll(who);
        const int b = __shfl(lane * 4 + bin, src);
        const int bf = __shfl(before, src);
        target -= bf;
        prefix |= (uint32_t)b << shift;
        mask |= 255u << shift;
        __builtin_amdgcn_wave_barrier();
    }
    return prefix;
}

// Same result, faster for spread values: one histogram pass over 256 buckets
// LINEAR IN THE VALUE between the row's min and max (b = floor((v - vmin) *
// 256 / (vmax - vmin)), monotone under rounding, so buckets before the
// target's hold only smaller-or-equal values), then the target bucket's
// members (<= 64) are sorted in one wave.  The radix select's first pass
// (sign + exponent byte) piles the keys of a row onto a few LDS addresses;
// these buckets do not.  Falls back to wave_select for a bucket of > 64
// members or non-finite / degenerate ranges.
template <int NR>
__device__ uint32_t wave_select_lin(const uint32_t (&keys)[NR], int f, int rank, int *hist) {
    const int lane = threadIdx.x & 63;
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if (lane + 64 * r < f) {
            kmin = keys[r] < kmin ? keys[r] : kmin;
            kmax = keys[r] > kmax ? keys[r] : kmax;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t a = __shfl_xor(kmin, o), b = __shfl_xor(kmax, o);
        kmin = a < kmin ? a : kmin;
        kmax = b > kmax ? b : kmax;
    }
    if (kmin == kmax) return kmin;
    const float vmin = key2f(kmin), vmax = key2f(kmax);
    const float scale = 256.0f / (vmax - vmin);
    if (!__builtin_isfinite(vmin) || !__builtin_isfinite(vmax) || !(scale < 1e30f))
        return wave_select<NR>(keys, NR, rank, hist);
    hist[lane * 4 + 0] = 0; hist[lane * 4 + 1] = 0;
    hist[lane * 4 + 2] = 0; hist[lane * 4 + 3] = 0;
    __builtin_amdgcn_wave_barrier();
    int bk[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const float v = key2f(keys[r]);
        int b = (int)((v - vmin) * scale);
        b = b < 0 ? 0 : (b > 255 ? 255 : b);
        bk[r] = lane + 64 * r < f ? b : -1;
        if (bk[r] >= 0) atomicAdd(&hist[b], 1);
    }
    __builtin_amdgcn_wave_barrier();
    const int c0 = hist[lane * 4], c1 = hist[lane * 4 + 1], c2 = hist[lane * 4 + 2],
              c3 = hist[lane * 4 + 3];
    const int tot = c0 + c1 + c2 + c3;
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const int excl = incl - tot;
    const bool mine = rank >= excl && rank < incl;
    int bin = 0, before = excl, cb = c0;
    if (mine) {
        if (rank < excl + c0) { bin = 0; cb = c0; }
        else if (rank < excl + c0 + c1) { bin = 1; before += c0; cb = c1; }
        else if (rank < excl + c0 + c1 + c2) { bin = 2; before += c0 + c1; cb = c2; }
        else { bin = 3; before += c0 + c1 + c2; cb = c3; }
    }
    const uint64_t who = __ballot(mine);
    const int src = (int)__builtin_ctzll(who);
    const int B = __shfl(lane * 4 + bin, src);
    const int bef = __shfl(before, src);
    const int cnt = __shfl(cb, src);
    if (cnt > 64) return wave_select<NR>(keys, NR, rank, hist);
    __builtin_amdgcn_wave_barrier();  // histogram read before its words are reused
    uint32_t *cand = (uint32_t *)hist;
    int base = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const bool in = bk[r] == B;
        const uint64_t m = __ballot(in);
        if (in) cand[base + (int)__popcll(m & ((1ull << lane) - 1ull))] = keys[r];
        base += (int)__popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    // bitonic sort of the bucket's keys (unsigned words, one per lane)
    uint32_t u = lane < cnt ? cand[lane] : 0xFFFFFFFFu;
#pragma unroll
    for (int k2 = 2; k2 <= 64; k2 <<= 1) {
#pragma unroll
        for (int j = k2 >> 1; j > 0; j >>= 1) {
            const uint32_t pu = __shfl_xor(u, j);
            const bool asc = (lane & k2) == 0, lower = (lane & j) == 0;
            const bool keep_min = asc == lower;
            u = keep_min ? (pu < u ? pu : u) : (pu > u ? pu : u);
        }
    }
    const uint32_t res = __shfl(u, rank - bef);
    __builtin_amdgcn_wave_barrier();
    return res;
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

// tau of one row (taumode.rs:29-70) from its keys
template <int NR>
__device__ double row_tau(const uint32_t (&keys)[NR], int f, double msum, int tau_mode,
                          double tau_param, int pct_rank, int *hist, int sel = 0) {
    if (tau_mode == MN_TAU_FIXED)
        return (isfinite(tau_param) && tau_param > 0.0) ? tau_param : 1e-10;
    if (tau_mode == MN_TAU_MEAN) return fmax(wave_sum(msum) / (double)f, 1e-10);
    const int lane = threadIdx.x & 63;
    const int rank = (tau_mode == MN_TAU_PERCENTILE) ? pct_rank : ((f % 2 == 1) ? f / 2 : f / 2 - 1);
    // sel 1: value-linear buckets (wave_select_lin), else the radix select
    const uint32_t ka = (sel & 1) ? wave_select_lin<NR>(keys, f, rank, hist)
                                 : wave_select<NR>(keys, NR, rank, hist);
    double med = (double)key2f(ka);
    if (tau_mode == MN_TAU_MEDIAN && f % 2 == 0) {
        // element rank+1: equal to ka if >= rank+2 keys are <= ka, else min{key > ka}
        int le = 0;
        uint32_t nxt = 0xFFFFFFFFu;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int t = lane + 64 * r;
            if (t < f) {
                le += keys[r] <= ka ? 1 : 0;
                if (keys[r] > ka && keys[r] < nxt) nxt = keys[r];
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            le += __shfl_xor(le, o);
            const uint32_t on = __shfl_xor(nxt, o);
            nxt = on < nxt ? on : nxt;
        }
        const double b = (le >= rank + 2) ? med : (double)key2f(nxt);
        med = 0.5 * (med + b);
    }
    return fmax(med, 1e-10);
}

// LDS: [ev f64 x ne | eij u32 x ne] (when in_lds) | xs f32 [waves][ROWS][fpad]
//      | hist int [waves][256]
template <int NR, int ROWS = 2>
__global__ __launch_bounds__(NR <= 16 ? 1024 : 256) void k_energy_rows(
    const float *__restrict__ X, int64_t n, int f, int64_t na, int64_t ne, int in_lds,
    const uint32_t *__restrict__ geij, const double *__restrict__ gev, double mA_num,
    double mA_g, int g_mode, int tau_mode, double tau_param, int pct_rank,
    double *__restrict__ Eo, double *__restrict__ Go, double *__restrict__ Lo, int sel) {
    typedef typename std::conditional<ROWS == 4, float4, float2>::type gat_t;
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int fpad = (f + 3) & ~3;
    const size_t eb = in_lds ? (((size_t)ne * 12 + 15) & ~(size_t)15) : 0;
    double *sev = (double *)dsm;
    uint32_t *seij = (uint32_t *)(dsm + (size_t)ne * 8);
    float *xs = (float *)(dsm + eb) + (size_t)w * ROWS * fpad;
    int *hist = (int *)(dsm + eb + (size_t)nw * ROWS * fpad * 4) + w * 256;
    if (in_lds) {
        for (int64_t p = threadIdx.x; p < ne; p += blockDim.x) {
            seij[p] = geij[p];
            sev[p] = gev[p];
        }
    }
    __syncthreads();
    const uint32_t *EIJ = in_lds ? seij : geij;
    const double *EV = in_lds ? sev : gev;
    const int64_t npass = (n + ROWS - 1) / ROWS;
    for (int64_t ps = (int64_t)blockIdx.x * nw + w; ps < npass; ps += (int64_t)gridDim.x * nw) {
        const int64_t r0 = ps * ROWS;
        uint32_t keys[ROWS][NR];
        double den[ROWS], msum[ROWS];
        bool nonzero[ROWS];
#pragma unroll
        for (int t = 0; t < ROWS; ++t) {
            // a missing last row repeats the previous one (computed, not written)
            // (sel & 16: timing probe, every pass re-reads row 0)
            const float *xr = X + ((sel & 16) ? 0 : min(r0 + t, n - 1)) * (int64_t)f;
            double dn = 0.0, ms = 0.0;
            bool nz = false;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int c = lane + 64 * r;
                const float x = c < f ? xr[c] : 0.f;
                if (c < f) {
                    xs[c * ROWS + t] = x;
                    const double xd = (double)x;
                    dn += xd * xd;
                    ms += xd;
                    nz |= !(fabs(xd) <= 1e-10);
                }
                keys[t][r] = c < f ? f2key(x) : 0xFFFFFFFFu;
            }
            den[t] = wave_sum(dn);
            msum[t] = ms;
            nonzero[t] = __any(nz) != 0;
        }
        __builtin_amdgcn_wave_barrier();
        double nA[ROWS], nB[ROWS], S[ROWS], Q[ROWS];
#pragma unroll
        for (int t = 0; t < ROWS; ++t) nA[t] = nB[t] = S[t] = Q[t] = 0.0;
        // list A: num += v x_i x_j (v = -w), S += e, Q += e^2, e = w (x_i - x_j)^2
        // the ROWS values of one feature are adjacent: one 8-B (16-B) gather
        // per endpoint serves the 2 (4) rows of the pass
        static_assert(ROWS == 2 || ROWS == 4, "gathers are float2 / float4");
        auto unpack = [](const gat_t &g, float (&a)[ROWS]) {
            const float *q = reinterpret_cast<const float *>(&g);
#pragma unroll
            for (int t = 0; t < ROWS; ++t) a[t] = q[t];
        };
#pragma unroll 2
        for (int64_t p = lane; p < na; p += 64) {
            const uint32_t ij = EIJ[p];
            const double wv = EV[p];
            // (sel & 32: timing probe, conflict-free gathers of fixed features)
            const int i = (sel & 32) ? lane : (int)(ij & 0xFFFFu);
            const int j = (sel & 32) ? lane + 64 : (int)(ij >> 16);
            const gat_t gi = *reinterpret_cast<const gat_t *>(&xs[i * ROWS]);
            const gat_t gj = *reinterpret_cast<const gat_t *>(&xs[j * ROWS]);
            float ai[ROWS], aj[ROWS];
            unpack(gi, ai);
            unpack(gj, aj);
#pragma unroll
            for (int t = 0; t < ROWS; ++t) {
                const double xi = (double)ai[t], xj = (double)aj[t];
                nA[t] = __builtin_fma(-wv, xi * xj, nA[t]);
                const double dd = xi - xj;
                const double e = (dd * dd) * wv;
                S[t] += e;
                Q[t] = __builtin_fma(e, e, Q[t]);
            }
        }
        // list B: num only
#pragma unroll 2
        for (int64_t p = na + lane; p < ne; p += 64) {
            const uint32_t ij = EIJ[p];
            const double v = EV[p];
            const int i = (sel & 32) ? lane : (int)(ij & 0xFFFFu);
            const int j = (sel & 32) ? lane + 64 : (int)(ij >> 16);
            const gat_t gi = *reinterpret_cast<const gat_t *>(&xs[i * ROWS]);
            const gat_t gj = *reinterpret_cast<const gat_t *>(&xs[j * ROWS]);
            float ai[ROWS], aj[ROWS];
            unpack(gi, ai);
            unpack(gj, aj);
#pragma unroll
            for (int t = 0; t < ROWS; ++t) {
                const double xi = (double)ai[t], xj = (double)aj[t];
                nB[t] = __builtin_fma(v, xi * xj, nB[t]);
            }
        }
#pragma unroll
        for (int t = 0; t < ROWS; ++t) {
            const double num = wave_sum(mA_num * nA[t] + nB[t]);
            const double Ss = mA_g * wave_sum(S[t]);
            const double Qs = mA_g * wave_sum(Q[t]);
            double e_raw = 0.0, g_raw = 0.0, lam = 0.0;
            if (g_mode == MN_G_SPECTRAL) {
                // spectral/mod.rs:89: clamp(num / (den + 1e-9), -1e6, 1e6); the
                // row energy is kept raw (G) until the global total is known
                const double r = num / (den[t] + 1e-9);
                e_raw = r < -1e6 ? -1e6 : (r > 1e6 ? 1e6 : r);
                g_raw = Ss;
                lam = e_raw;
            } else if (!(g_mode == MN_G_TAUMODE && !nonzero[t])) {  // zero vector: lambda 0
                e_raw = den[t] > 1e-12 ? fmax(num / den[t], 0.0) : 0.0;
                if (Ss > 1e-12) {
                    const double g = Qs / (Ss * Ss);
                    g_raw = g < 0.0 ? 0.0 : (g > 1.0 ? 1.0 : g);
                }
                if (g_mode == MN_G_TAUMODE) {
                    const double tau = row_tau<NR>(keys[t], f, msum[t], tau_mode, tau_param,
                                                   pct_rank, hist, sel);
                    const double ebv = e_raw / (e_raw + tau);
                    lam = tau * ebv + (1.0 - tau) * g_raw;
                } else {
                    lam = e_raw;
                }
            }
            if (lane == 0 && r0 + t < n) {
                if (Eo) Eo[r0 + t] = e_raw;
                if (Go) Go[r0 + t] = g_raw;
                if (Lo) Lo[r0 + t] = lam;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- K3 v2: counted order statistics, diagonal from registers, prefetch ----
// Column c of one row through a buffer resource sized to the row: columns
// >= f read 0 without a branch (a guarded `c < f ? x[c] : 0` compiles to a
// branch with its own vmcnt(0) wait — one serial HBM trip per register).
// `row` must be wave-uniform.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const float *row, int f) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)row, (short)0, f * 4, 0x00020000);
}
__device__ __forceinline__ float row_at(__amdgpu_buffer_rsrc_t rs, int c) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, c * 4, 0, 0));
}

// Wave reductions through DPP (quad_perm xor 1 / xor 2, row half-mirror, row
// mirror, row_bcast15 / row_bcast31): six VALU steps with no LDS round trip
// (a __shfl_xor is a ds_bpermute each).  The total lands in lane 63 and is
// read out wave-uniform.
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ double dpp64(double old, double v) {
    const uint64_t o = __double_as_longlong(old), u = __double_as_longlong(v);
    const uint32_t lo = dpp32<CTRL, RM>((uint32_t)o, (uint32_t)u);
    const uint32_t hi = dpp32<CTRL, RM>((uint32_t)(o >> 32), (uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ uint32_t lane63_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_umin_dpp(uint32_t x) {
    x = min(x, dpp32<0xB1, 0xF>(x, x));
    x = min(x, dpp32<0x4E, 0xF>(x, x));
    x = min(x, dpp32<0x141, 0xF>(x, x));
    x = min(x, dpp32<0x140, 0xF>(x, x));
    x = min(x, dpp32<0x142, 0xA>(x, x));
    x = min(x, dpp32<0x143, 0xC>(x, x));
    return lane63_u32(x);
}
__device__ __forceinline__ uint32_t wave_umax_dpp(uint32_t x) {
    x = max(x, dpp32<0xB1, 0xF>(x, x));
    x = max(x, dpp32<0x4E, 0xF>(x, x));
    x = max(x, dpp32<0x141, 0xF>(x, x));
    x = max(x, dpp32<0x140, 0xF>(x, x));
    x = max(x, dpp32<0x142, 0xA>(x, x));
    x = max(x, dpp32<0x143, 0xC>(x, x));
    return lane63_u32(x);
}
// (`old` = x: lanes a row mask leaves out keep garbage that never reaches
// lane 63 — rows 1 and 3 are written by the bcast15 step, row 3 by bcast31)
__device__ __forceinline__ double wave_sum_dpp(double x) {
    x += dpp64<0xB1, 0xF>(x, x);
    x += dpp64<0x4E, 0xF>(x, x);
    x += dpp64<0x141, 0xF>(x, x);
    x += dpp64<0x140, 0xF>(x, x);
    x += dpp64<0x142, 0xA>(x, x);
    x += dpp64<0x143, 0xC>(x, x);
    const uint64_t u = __double_as_longlong(x);
    const uint32_t lo = lane63_u32((uint32_t)u), hi = lane63_u32((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// keys <= k over the wave's row (pads 0xFFFFFFFF never count: k < 0xFFFFFFFF)
template <int NR>
__device__ __forceinline__ int wave_cle(const uint32_t (&keys)[NR], uint32_t k) {
    int c = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) c += (int)__popcll(__ballot(keys[r] <= k));
    return c;
}

// Exact order statistic `rank` (and rank + 1 when need == 2) of a row's f keys
// (pads 0xFFFFFFFF) without a histogram: a bracket (kA, kB] with
// cle(kA) <= rank and cle(kB) >= rank + need is narrowed by pairs of
// value-interpolated probes (+-hw keys at the bracket's mean density; a probe
// is NR compares + ballot popcounts, no LDS) until it holds <= 20 keys (<= 64
// after 8 rounds); those are compacted into LDS and each lane ranks its own
// candidate by counting over broadcast reads (sorted position t holds the u
// with #(< u) <= t < #(<= u)).  false: the row did not settle (non-finite
// values, > 64 tied keys, skewed rows) — the caller runs the radix select.
template <int NR>
__device__ bool wave_select_cnt(const uint32_t (&keys)[NR], int f, int rank, int need,
                                uint32_t *cand, uint32_t &out0, uint32_t &out1) {
    const int lane = threadIdx.x & 63;
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
#pragma unroll
    for (int r = 0; r < NR; ++r) {  // pads (0xFFFFFFFF) never lower kmin; kept out of kmax
        kmin = min(kmin, keys[r]);
        kmax = max(kmax, lane + 64 * r < f ? keys[r] : 0u);
    }
    kmin = wave_umin_dpp(kmin);
    kmax = wave_umax_dpp(kmax);
    if (kmin == kmax) {
        out0 = out1 = kmin;
        return true;
    }
    if (!__builtin_isfinite(key2f(kmin)) || !__builtin_isfinite(key2f(kmax))) return false;
    uint32_t kA = kmin - 1u, kB = kmax;  // finite keys are >= f2key(-FLT_MAX) > 0
    int cA = 0, cB = f;
    for (int it = 0; it < 8 && cB - cA > 20; ++it) {
        const float vlo = key2f(kA + 1u), vhi = key2f(kB);
        const int m = cB - cA;
        const float span = vhi - vlo;
        if (!(span > 0.f)) break;  // one value left (ties): compact or fall back
        const int hw = m / 6 < 6 ? 6 : (m / 6 > 24 ? 24 : m / 6);
        // estimates only (any probe is exact): approximate reciprocal
        const float rm = __builtin_amdgcn_rcpf((float)m);
        const float est = vlo + span * (((float)(rank - cA) + 0.5f * (float)need) * rm);
        const float half = span * ((float)hw * rm);
        const float p1 = fmaxf(est - half, vlo), p2 = fminf(est + half, vhi);
        const uint32_t k1 = f2key(p1), k2 = f2key(p2);
        const int c1 = wave_cle<NR>(keys, k1), c2 = wave_cle<NR>(keys, k2);
        if (c1 <= rank) {
            if (k1 > kA) { kA = k1; cA = c1; }
        } else if (c1 >= rank + need && k1 < kB) {
            kB = k1; cB = c1;
        }
        if (c2 <= rank) {
            if (k2 > kA) { kA = k2; cA = c2; }
        } else if (c2 >= rank + need && k2 < kB) {
            kB = k2; cB = c2;
        }
    }
    const int m = cB - cA;
    if (m > 64) return false;
    int base = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const bool in = keys[r] > kA && keys[r] <= kB;  // pads exceed kB (finite)
        const uint64_t mk = __ballot(in);
        if (in) cand[base + (int)__popcll(mk & ((1ull << lane) - 1ull))] = keys[r];
        base += (int)__popcll(mk);
    }
    if (lane >= m) cand[lane] = 0xFFFFFFFFu;
    __builtin_amdgcn_wave_barrier();
    const uint32_t u = cand[lane];
    int lt = 0, le = 0;
    for (int q = 0; q < m; q += 4) {
        const uint4 v = *reinterpret_cast<const uint4 *>(&cand[q]);
        lt += (v.x < u) + (v.y < u) + (v.z < u) + (v.w < u);
        le += (v.x <= u) + (v.y <= u) + (v.z <= u) + (v.w <= u);
    }
    const int t0 = rank - cA;
    const uint64_t h0 = __ballot(lane < m && lt <= t0 && t0 < le);
    out0 = (uint32_t)__builtin_amdgcn_readlane((int)u, (int)__builtin_ctzll(h0));
    if (need == 2) {
        const uint64_t h1 = __ballot(lane < m && lt <= t0 + 1 && t0 + 1 < le);
        out1 = (uint32_t)__builtin_amdgcn_readlane((int)u, (int)__builtin_ctzll(h1));
    } else {
        out1 = out0;
    }
    __builtin_amdgcn_wave_barrier();  // cand is reused by the next row
    return true;
}

// Inclusive prefix sum over the wave's 64 lanes through DPP (row_shr 1/2/4/8
// inside each 16-lane row, then row_bcast15 / row_bcast31 carry the row totals
// forward); lanes whose DPP source is out of range add 0 (`old`).
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += (int)dpp32<0x111, 0xF>(0u, (uint32_t)x);
    x += (int)dpp32<0x112, 0xF>(0u, (uint32_t)x);
    x += (int)dpp32<0x114, 0xF>(0u, (uint32_t)x);
    x += (int)dpp32<0x118, 0xF>(0u, (uint32_t)x);
    x += (int)dpp32<0x142, 0xA>(0u, (uint32_t)x);
    x += (int)dpp32<0x143, 0xC>(0u, (uint32_t)x);
    return x;
}

// Exact order statistic `rank` (and rank + 1 when need == 2) of a row's f keys
// (pads 0xFFFFFFFF; vals: the same row as floats) by one value-linear
// histogram pass (round 5): 256 buckets
// b(v) = min(255, (v - vmin) * 255.99 / (vmax - vmin)) — monotone in v, so a
// bucket is a key interval — counted with LDS adds, located by a DPP prefix
// scan over the lanes' four-bucket sums; the keys of the bucket(s) holding the
// two ranks are compacted and ranked as in wave_select_cnt.  No probe rounds
// and no scalar popcount chains.  false: more than 64 keys in those buckets
// (ties, heavy tails) or non-finite values — the caller tries the next select.
template <int NR>
__device__ bool wave_select_hist(const uint32_t (&keys)[NR], const float (&vals)[NR], int f,
                                 int rank, int need, int *hist, uint32_t &out0, uint32_t &out1) {
    const int lane = threadIdx.x & 63;
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        kmin = min(kmin, keys[r]);
        kmax = max(kmax, lane + 64 * r < f ? keys[r] : 0u);
    }
    kmin = wave_umin_dpp(kmin);
    kmax = wave_umax_dpp(kmax);
    if (kmin == kmax) {
        out0 = out1 = kmin;
        return true;
    }
    const float vlo = key2f(kmin), vhi = key2f(kmax);
    if (!__builtin_isfinite(vlo) || !__builtin_isfinite(vhi)) return false;
    const float sc = 255.99f / (vhi - vlo);  // span overflow: sc = 0, one bucket, > 64
    reinterpret_cast<int4 *>(hist)[lane] = make_int4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    uint32_t bk[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        // fminf first: NaN (0 x inf on a denormal span) -> 255, the cast stays defined
        const float d = fminf((vals[r] - vlo) * sc, 255.0f);
        bk[r] = (uint32_t)d;
        if (lane + 64 * r < f) atomicAdd(&hist[bk[r]], 1);
    }
    __builtin_amdgcn_wave_barrier();
    const int4 h = reinterpret_cast<const int4 *>(hist)[lane];
    const int c1 = h.x, c2 = c1 + h.y, c3 = c2 + h.z, tot = c3 + h.w;
    const int incl = wave_incl_scan(tot), excl = incl - tot;
    // bucket holding order statistic q and the count of keys below it
    auto locate = [&](int q, uint32_t &b, int &below, int &upto) {
        const uint64_t hit = __ballot(excl <= q && q < incl);
        const int L = (int)__builtin_ctzll(hit);
        const int sb = (q - excl >= c1) + (q - excl >= c2) + (q - excl >= c3);
        const int lo = excl + (sb == 0 ? 0 : (sb == 1 ? c1 : (sb == 2 ? c2 : c3)));
        const int hi = excl + (sb == 0 ? c1 : (sb == 1 ? c2 : (sb == 2 ? c3 : tot)));
        b = (uint32_t)__builtin_amdgcn_readlane(4 * lane + sb, L);
        below = __builtin_amdgcn_readlane(lo, L);
        upto = __builtin_amdgcn_readlane(hi, L);
    };
    uint32_t b0, b1;
    int cA, e0, cB0, cB;
    locate(rank, b0, cA, e0);
    if (need == 2 && rank + 1 >= e0) locate(rank + 1, b1, cB0, cB);
    else { b1 = b0; cB = e0; }
    const int m = cB - cA;
    if (m > 64) return false;
    __builtin_amdgcn_wave_barrier();  // every lane has read the histogram
    uint32_t *cand = (uint32_t *)hist;
    int base = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const bool in = lane + 64 * r < f && bk[r] >= b0 && bk[r] <= b1;
        const uint64_t mk = __ballot(in);
        if (in) cand[base + (int)__popcll(mk & ((1ull << lane) - 1ull))] = keys[r];
        base += (int)__popcll(mk);
    }
    if (lane >= m) cand[lane] = 0xFFFFFFFFu;
    __builtin_amdgcn_wave_barrier();
    const uint32_t u = cand[lane];
    int lt = 0, le = 0;
    for (int q = 0; q < m; q += 4) {
        const uint4 v = *reinterpret_cast<const uint4 *>(&cand[q]);
        lt += (v.x < u) + (v.y < u) + (v.z < u) + (v.w < u);
        le += (v.x <= u) + (v.y <= u) + (v.z <= u) + (v.w <= u);
    }
    const int t0 = rank - cA;
    const uint64_t h0 = __ballot(lane < m && lt <= t0 && t0 < le);
    out0 = (uint32_t)__builtin_amdgcn_readlane((int)u, (int)__builtin_ctzll(h0));
    if (need == 2) {
        const uint64_t h1 = __ballot(lane < m && lt <= t0 + 1 && t0 + 1 < le);
        out1 = (uint32_t)__builtin_amdgcn_readlane((int)u, (int)__builtin_ctzll(h1));
    } else {
        out1 = out0;
    }
    __builtin_amdgcn_wave_barrier();  // cand is reused by the next row
    return true;
}

// Median / Percentile tau of every row, one wave per row (grid-stride), for
// k_energy_rows2: a lean kernel (keys in registers, 1 KB LDS per wave) at
// high occupancy re-reads X instead of holding the select's registers and
// latency inside the entry-loop kernel (which keeps Fixed / Mean inline).
template <int NR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_row_tau(const float *__restrict__ X, int64_t n, int f,
                                                 int tau_mode, double tau_param, int pct_rank,
                                                 double *__restrict__ tau) {
    __shared__ __attribute__((aligned(16))) int hist_all[4][256];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int *hist = hist_all[w];
    const bool med = tau_mode == MN_TAU_MEDIAN;
    const int rank = med ? ((f % 2 == 1) ? f / 2 : f / 2 - 1) : pct_rank;
    const int need = (med && f % 2 == 0) ? 2 : 1;
    const int64_t rstride = (int64_t)gridDim.x * 4;
    int64_t row = (int64_t)blockIdx.x * 4 + w;
    float xv[NR];
    auto load_row = [&](int64_t rw) {
        const __amdgpu_buffer_rsrc_t rs = row_rsrc(X + rw * (int64_t)f, f);
#pragma unroll
        for (int r = 0; r < NR; ++r) xv[r] = row_at(rs, lane + 64 * r);
        __builtin_amdgcn_sched_barrier(0);  // all loads issue before any use
    };
    if (row < n) load_row(row);
    for (; row < n; row += rstride) {
        uint32_t keys[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            // sortable key (as f2key, branch-free) | all-ones for columns >= f
            const uint32_t u = __float_as_uint(xv[r]);
            const uint32_t k = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
            keys[r] = k | (uint32_t)-(int32_t)(lane + 64 * r >= f);
        }
        if (row + rstride < n) load_row(row + rstride);  // next row in flight during the select
        uint32_t k0, k1;
        double v;
        if (wave_select_cnt<NR>(keys, f, rank, need, (uint32_t *)hist, k0, k1)) {
            v = (double)key2f(k0);
            if (need == 2) v = 0.5 * (v + (double)key2f(k1));
            v = fmax(v, 1e-10);
        } else {
            v = row_tau<NR>(keys, f, 0.0, tau_mode, tau_param, pct_rank, hist);
        }
        if (lane == 0) tau[row] = v;
    }
}

// Two item rows per wave pass (as k_energy_rows), reorganised:
//  - the Laplacian diagonal (class D) is applied from the rows' registers
//    while they are staged (sum dg_c x_c^2): no gathers for it;
//  - the entry lists hold byte offsets of x_i / x_j in the wave's stage
//    (i*8 | j*8 << 16) and are padded to whole 4-entry-per-lane chunks with
//    entries at a zero slot past the row (exact no-ops), so the loop has no
//    tail and issues 4 entry reads, then 8 gathers, per lane at a time;
//  - the next pass's rows are loaded into registers while this pass runs
//    (the HBM latency hides behind the entry loop);
//  - Median / Percentile tau come from k_row_tau (counted selection).
// LDS: eij u32 [neP] | ev f64 [neP] | dg f64 [fpad] | per wave: xs f32
// [fpad + 1][2] (slot fpad = 0).
constexpr int E2_CH = 256;  // entries per chunk (4 per lane)
constexpr int E2_MIN_WAVES = 4;
// k_energy_rows2's LDS: the padded lists + dg, plus `waves` wave stages
static inline size_t e2_lds_bytes(int64_t na, int64_t nb, int f, int waves, bool tk = false) {
    const int64_t neP = (na + E2_CH - 1) / E2_CH * E2_CH + (nb + E2_CH - 1) / E2_CH * E2_CH;
    const size_t fpad = (size_t)((f + 3) & ~3);
    return (((size_t)neP * 4 + 15) & ~(size_t)15) + (size_t)neP * 8 + fpad * 8 +
           (size_t)waves * ((fpad + 4) * 8 + (tk ? 1024 : 0));
}
template <int NR, bool TK>
__global__ __launch_bounds__(1024) void k_energy_rows2(
    const float *__restrict__ X, int64_t n, int f, int64_t na, int64_t naP, int64_t nb,
    int64_t nbP, const uint32_t *__restrict__ geij, const double *__restrict__ gev,
    const double *__restrict__ gdg, double mA_num, double mA_g, int g_mode, int tau_mode,
    double tau_param, int pct_rank, const double *__restrict__ tau_in, double *__restrict__ Eo,
    double *__restrict__ Go, double *__restrict__ Lo) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const int fpad = (f + 3) & ~3;
    const int64_t neP = naP + nbP;
    uint32_t *seij = (uint32_t *)dsm;
    double *sev = (double *)(dsm + (((size_t)neP * 4 + 15) & ~(size_t)15));
    double *sdg = sev + neP;
    const size_t wbytes = (size_t)(fpad + 4) * 8 + (TK ? 1024 : 0);
    float *xs = (float *)((unsigned char *)(sdg + fpad) + (size_t)w * wbytes);
    int *hist = (int *)(xs + 2 * (fpad + 4));  // TK: the select's scratch
    const uint32_t zoff = (uint32_t)fpad * 8u;  // the zero slot
    const uint32_t zpair = zoff | (zoff << 16);
    for (int64_t p = threadIdx.x; p < neP; p += blockDim.x) {
        const int64_t q = p < naP ? p : na + (p - naP);  // source index
        const bool real = p < naP ? p < na : (p - naP) < nb;
        uint32_t e = zpair;
        double v = 0.0;
        if (real) {
            const uint32_t ij = geij[q];
            e = ((ij & 0xFFFFu) * 8u) | (((ij >> 16) * 8u) << 16);
            v = gev[q];
        }
        seij[p] = e;
        sev[p] = v;
    }
    for (int c = threadIdx.x; c < fpad; c += blockDim.x) sdg[c] = c < f ? gdg[c] : 0.0;
    if (lane < 8) xs[2 * fpad + lane] = 0.f;
    __syncthreads();
    const unsigned char *xsb = (const unsigned char *)xs;
    const bool mean_tau = g_mode == MN_G_TAUMODE && tau_mode == MN_TAU_MEAN;
    const int64_t npass = (n + 1) / 2;
    const int64_t pstride = (int64_t)gridDim.x * nw;
    int64_t ps = (int64_t)blockIdx.x * nw + w;
    float cur[2][NR];
    auto load_rows = [&](int64_t pq, float (&dst)[2][NR]) {
        const int64_t r0 = pq * 2;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            // a missing last row repeats (computed, not written)
            const __amdgpu_buffer_rsrc_t rs = row_rsrc(X + min(r0 + t, n - 1) * (int64_t)f, f);
#pragma unroll
            for (int r = 0; r < NR; ++r) dst[t][r] = row_at(rs, lane + 64 * r);
        }
        __builtin_amdgcn_sched_barrier(0);  // all loads issue before any use
    };
    if (ps < npass) load_rows(ps, cur);
    for (; ps < npass; ps += pstride) {
        const int64_t r0 = ps * 2;
        double den[2] = {0.0, 0.0}, msum[2] = {0.0, 0.0}, numD[2] = {0.0, 0.0};
        bool nzr[2] = {false, false};
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int c = lane + 64 * r;
            if (c < f) {
                const double dgc = sdg[c];
                *reinterpret_cast<float2 *>(&xs[2 * c]) = make_float2(cur[0][r], cur[1][r]);
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const double xd = (double)cur[t][r];
                    const double x2 = xd * xd;
                    den[t] += x2;
                    if (mean_tau) msum[t] += xd;
                    numD[t] = __builtin_fma(dgc, x2, numD[t]);
                    nzr[t] |= !(fabs(xd) <= 1e-10);
                }
            }
        }
        // tau: per-row Median / Percentile from k_row_tau (tau_in), in this
        // kernel (TK, MN_ENERGY_TAU=1 A/B), else Fixed / Mean inline
        double tau[2] = {0.0, 0.0};
        uint32_t keys[TK ? 2 : 1][NR];
        if (TK) {
#pragma unroll
            for (int t = 0; t < (TK ? 2 : 1); ++t)
#pragma unroll
                for (int r = 0; r < NR; ++r)
                    keys[t][r] = lane + 64 * r < f ? f2key(cur[t][r]) : 0xFFFFFFFFu;
        }
        // the next pass's rows: in flight during this pass's select + entry loop
        if (ps + pstride < npass) load_rows(ps + pstride, cur);
        if (g_mode == MN_G_TAUMODE) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                if (TK && (tau_mode == MN_TAU_MEDIAN || tau_mode == MN_TAU_PERCENTILE)) {
                    const bool med = tau_mode == MN_TAU_MEDIAN;
                    const int rank = med ? ((f % 2 == 1) ? f / 2 : f / 2 - 1) : pct_rank;
                    const int need = (med && f % 2 == 0) ? 2 : 1;
                    uint32_t k0, k1;
                    if (wave_select_cnt<NR>(keys[TK ? t : 0], f, rank, need, (uint32_t *)hist, k0,
                                            k1)) {
                        double v = (double)key2f(k0);
                        if (need == 2) v = 0.5 * (v + (double)key2f(k1));
                        tau[t] = fmax(v, 1e-10);
                    } else {
                        tau[t] = row_tau<NR>(keys[TK ? t : 0], f, msum[t], tau_mode, tau_param,
                                             pct_rank, hist);
                    }
                } else if (tau_in) {
                    tau[t] = tau_in[min(r0 + t, n - 1)];
                } else if (tau_mode == MN_TAU_MEAN) {
                    tau[t] = fmax(wave_sum_dpp(msum[t]) / (double)f, 1e-10);
                } else {
                    tau[t] = (isfinite(tau_param) && tau_param > 0.0) ? tau_param : 1e-10;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        double nA0 = 0.0, nA1 = 0.0, S0 = 0.0, S1 = 0.0, Q0 = 0.0, Q1 = 0.0;
        for (int64_t p0 = lane; p0 < naP; p0 += E2_CH) {
            uint32_t ij[4];
            double wv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                ij[u] = seij[p0 + 64 * u];
                wv[u] = sev[p0 + 64 * u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float2 gi = *reinterpret_cast<const float2 *>(xsb + (ij[u] & 0xFFFFu));
                const float2 gj = *reinterpret_cast<const float2 *>(xsb + (ij[u] >> 16));
                const double xi0 = (double)gi.x, xj0 = (double)gj.x;
                const double xi1 = (double)gi.y, xj1 = (double)gj.y;
                nA0 = __builtin_fma(-wv[u], xi0 * xj0, nA0);
                nA1 = __builtin_fma(-wv[u], xi1 * xj1, nA1);
                const double d0 = xi0 - xj0, d1 = xi1 - xj1;
                const double e0 = (d0 * d0) * wv[u], e1 = (d1 * d1) * wv[u];
                S0 += e0;
                S1 += e1;
                Q0 = __builtin_fma(e0, e0, Q0);
                Q1 = __builtin_fma(e1, e1, Q1);
            }
        }
        double nB0 = 0.0, nB1 = 0.0;
        for (int64_t p0 = naP + lane; p0 < neP; p0 += E2_CH) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t ij = seij[p0 + 64 * u];
                const double v = sev[p0 + 64 * u];
                const float2 gi = *reinterpret_cast<const float2 *>(xsb + (ij & 0xFFFFu));
                const float2 gj = *reinterpret_cast<const float2 *>(xsb + (ij >> 16));
                nB0 = __builtin_fma(v, (double)gi.x * (double)gj.x, nB0);
                nB1 = __builtin_fma(v, (double)gi.y * (double)gj.y, nB1);
            }
        }
        const double nAs[2] = {nA0, nA1}, nBs[2] = {nB0, nB1}, Sv[2] = {S0, S1}, Qv[2] = {Q0, Q1};
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const double num = wave_sum_dpp(mA_num * nAs[t] + nBs[t] + numD[t]);
            const double Ss = mA_g * wave_sum_dpp(Sv[t]);
            const double Qs = mA_g * wave_sum_dpp(Qv[t]);
            const double dn = wave_sum_dpp(den[t]);
            const bool nonzero = __any(nzr[t]) != 0;
            double e_raw = 0.0, g_raw = 0.0, lam = 0.0;
            if (g_mode == MN_G_SPECTRAL) {
                const double rr = num / (dn + 1e-9);
                e_raw = rr < -1e6 ? -1e6 : (rr > 1e6 ? 1e6 : rr);
                g_raw = Ss;
                lam = e_raw;
            } else if (!(g_mode == MN_G_TAUMODE && !nonzero)) {  // zero vector: lambda 0
                e_raw = dn > 1e-12 ? fmax(num / dn, 0.0) : 0.0;
                if (Ss > 1e-12) {
                    const double g = Qs / (Ss * Ss);
                    g_raw = g < 0.0 ? 0.0 : (g > 1.0 ? 1.0 : g);
                }
                if (g_mode == MN_G_TAUMODE) {
                    const double ebv = e_raw / (e_raw + tau[t]);
                    lam = tau[t] * ebv + (1.0 - tau[t]) * g_raw;
                } else {
                    lam = e_raw;
                }
            }
            if (lane == 0 && r0 + t < n) {
                if (Eo) Eo[r0 + t] = e_raw;
                if (Go) Go[r0 + t] = g_raw;
                if (Lo) Lo[r0 + t] = lam;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- K3 v3: one pass over X (round 4) -------------------------------------
// k_row_tau + k_energy_rows2 read X twice (PMC 6.2 GB per call for 3.1 GB of
// rows).  rows3 streams each row once: a wave takes two rows per pass, selects
// their tau (counted selection, registers), stages them in LDS as f64 pairs
// (no f32 -> f64 converts in the entry loop) and folds the entry lists, while
// the next pass's rows are in flight.  For a symmetric L the list-A part of
// the Rayleigh numerator uses the identity (w = -L_ij > 0, the upper list A)
//     2 sum_A L_ij x_i x_j = sum_A w (x_i - x_j)^2 - sum_c dgA_c x_c^2
// (dgA_c = the A weights at c, both triangles), so
//     x^T L x = sum_c (L_cc - dgA_c) x_c^2 + S_A + sum_B v x_i x_j
// with S_A = sum_A w (x_i - x_j)^2 — the dispersion's own sum: per entry and
// row d = x_i - x_j, e = w d^2, S += e, Q += e^2 (5 f64 ops instead of 7).
// Exact identity; its rounding differs from the reference's fold by O(u) of
// the terms (the 1e-9 contract; tests/test_energy_gpu.py).
// LDS: eij u32 [neP] | ev f64 [neP] | dgm f64 [fpad] | per wave: xs [fpad + 1]
// (slot fpad = 0) of double2 (S64: 8 waves a block) or float2 (16 waves, the
// converts in the loop) | 256 ints (select scratch).
template <bool S64> struct E3 {
    static constexpr int WAVES = S64 ? 8 : 16;
    static constexpr int XB = S64 ? 16 : 8;  // stage bytes per column (two rows)
};
static inline size_t e3_lds_bytes(int64_t neP, int f, int waves, int xb) {
    const size_t fpad = (size_t)((f + 3) & ~3);
    return (((size_t)neP * 4 + 15) & ~(size_t)15) + (size_t)neP * 8 + fpad * 8 +
           (size_t)waves * ((fpad + 1) * xb + 1024);
}
template <int NR, bool S64>
__global__ __launch_bounds__(64 * E3<S64>::WAVES) void k_energy_rows3(
    const float *__restrict__ X, int64_t n, int f, int64_t na, int64_t naP, int64_t nb,
    int64_t nbP, const uint32_t *__restrict__ geij, const double *__restrict__ gev,
    const double *__restrict__ gdgm, double mA_g, int g_mode, int tau_mode, double tau_param,
    int pct_rank, double *__restrict__ Eo, double *__restrict__ Go, double *__restrict__ Lo,
    const int32_t *__restrict__ gperm, int sel_v) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    constexpr int NW = E3<S64>::WAVES, XB = E3<S64>::XB;
    typedef typename std::conditional<S64, double2, float2>::type stage_t;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int fpad = (f + 3) & ~3;
    const int64_t neP = naP + nbP;
    uint32_t *seij = (uint32_t *)dsm;
    double *sev = (double *)(dsm + (((size_t)neP * 4 + 15) & ~(size_t)15));
    double *sdg = sev + neP;
    unsigned char *wbase = (unsigned char *)(sdg + fpad) + (size_t)w * ((fpad + 1) * XB + 1024);
    stage_t *xs = (stage_t *)wbase;                       // [fpad + 1]
    int *hist = (int *)(wbase + (size_t)(fpad + 1) * XB);  // 256 ints
    // entry offsets: byte offsets of x_i / x_j in the stage (XB B per column),
    // packed (i XB) | (j XB) << 16 (fpad XB < 2^16); padding -> zero slot
    const uint32_t zoff = (uint32_t)fpad * XB;
    const uint32_t zpair = zoff | (zoff << 16);
    for (int64_t p = threadIdx.x; p < neP; p += blockDim.x) {
        const int64_t q = p < naP ? p : na + (p - naP);
        const bool real = p < naP ? p < na : (p - naP) < nb;
        uint32_t e = zpair;
        double v = 0.0;
        if (real) {
            const uint32_t ij = geij[q];
            e = ((ij & 0xFFFFu) * XB) | (((ij >> 16) * XB) << 16);
            v = gev[q];
        }
        seij[p] = e;
        sev[p] = v;
    }
    for (int c = threadIdx.x; c < fpad; c += blockDim.x) sdg[c] = c < f ? gdgm[c] : 0.0;
    if (lane == 0) xs[fpad] = stage_t{0, 0};
    // the stage slot of each of this lane's columns (gperm: the bank-balanced
    // column order the conflict-free entry lists were built for)
    int slot[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int c = lane + 64 * r;
        slot[r] = (gperm && c < f) ? gperm[c] : c;
    }
    __syncthreads();
    const unsigned char *xsb = (const unsigned char *)xs;
    const bool mean_tau = g_mode == MN_G_TAUMODE && tau_mode == MN_TAU_MEAN;
    const bool sel_tau = g_mode == MN_G_TAUMODE &&
                         (tau_mode == MN_TAU_MEDIAN || tau_mode == MN_TAU_PERCENTILE);
    const bool med = tau_mode == MN_TAU_MEDIAN;
    const int rank = med ? ((f % 2 == 1) ? f / 2 : f / 2 - 1) : pct_rank;
    const int need = (med && f % 2 == 0) ? 2 : 1;
    const int64_t npass = (n + 1) / 2;
    const int64_t pstride = (int64_t)gridDim.x * NW;
    int64_t ps = (int64_t)blockIdx.x * NW + w;
    float cur[2][NR];
    auto load_rows = [&](int64_t pq, float (&dst)[2][NR]) {
        const int64_t r0 = pq * 2;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            // a missing last row repeats (computed, not written)
            const __amdgpu_buffer_rsrc_t rs = row_rsrc(X + min(r0 + t, n - 1) * (int64_t)f, f);
#pragma unroll
            for (int r = 0; r < NR; ++r) dst[t][r] = row_at(rs, lane + 64 * r);
        }
        __builtin_amdgcn_sched_barrier(0);  // all loads issue before any use
    };
    if (ps < npass) load_rows(ps, cur);
    for (; ps < npass; ps += pstride) {
        const int64_t r0 = ps * 2;
        // stage the pair (f64) and the diagonal part from registers
        double den[2] = {0.0, 0.0}, msum[2] = {0.0, 0.0}, numD[2] = {0.0, 0.0};
        bool nzr[2] = {false, false};
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int c = lane + 64 * r;
            if (c < f) {
                const double x0 = (double)cur[0][r], x1 = (double)cur[1][r];
                if constexpr (S64) xs[slot[r]] = make_double2(x0, x1);
                else xs[slot[r]] = make_float2(cur[0][r], cur[1][r]);
                const double dgc = sdg[c];
                const double q0 = x0 * x0, q1 = x1 * x1;
                den[0] += q0;
                den[1] += q1;
                numD[0] = __builtin_fma(dgc, q0, numD[0]);
                numD[1] = __builtin_fma(dgc, q1, numD[1]);
                if (mean_tau) {
                    msum[0] += x0;
                    msum[1] += x1;
                }
                nzr[0] |= !(fabs(x0) <= 1e-10);
                nzr[1] |= !(fabs(x1) <= 1e-10);
            }
        }
        double tau[2] = {0.0, 0.0};
        if (sel_tau) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                uint32_t keys[NR];
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const uint32_t u = __float_as_uint(cur[t][r]);
                    const uint32_t k = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
                    keys[r] = k | (uint32_t)-(int32_t)(lane + 64 * r >= f);
                }
                uint32_t k0, k1;
                // sel_v 1 (default): histogram select, then the counted
                // selection, then the radix select; 0: the round-4 order
                if ((sel_v == 1 && wave_select_hist<NR>(keys, cur[t], f, rank, need, hist, k0, k1)) ||
                    wave_select_cnt<NR>(keys, f, rank, need, (uint32_t *)hist, k0, k1)) {
                    double v = (double)key2f(k0);
                    if (need == 2) v = 0.5 * (v + (double)key2f(k1));
                    tau[t] = fmax(v, 1e-10);
                } else {
                    tau[t] = row_tau<NR>(keys, f, 0.0, tau_mode, tau_param, pct_rank, hist);
                }
            }
        } else if (g_mode == MN_G_TAUMODE) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
                tau[t] = tau_mode == MN_TAU_MEAN
                             ? fmax(wave_sum_dpp(msum[t]) / (double)f, 1e-10)
                             : ((isfinite(tau_param) && tau_param > 0.0) ? tau_param : 1e-10);
        }
        // the next pass's rows: in flight during this pass's entry loop
        if (ps + pstride < npass) load_rows(ps + pstride, cur);
        __builtin_amdgcn_wave_barrier();
        // list A: S, Q (two accumulator sets: shorter add chains)
        double S0a = 0.0, S1a = 0.0, Q0a = 0.0, Q1a = 0.0;
        double S0b = 0.0, S1b = 0.0, Q0b = 0.0, Q1b = 0.0;
        for (int64_t p0 = lane; p0 < naP; p0 += E2_CH) {
            uint32_t ij[4];
            double wv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                ij[u] = seij[p0 + 64 * u];
                wv[u] = sev[p0 + 64 * u];
            }
            stage_t gi[4], gj[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                gi[u] = *reinterpret_cast<const stage_t *>(xsb + (ij[u] & 0xFFFFu));
                gj[u] = *reinterpret_cast<const stage_t *>(xsb + (ij[u] >> 16));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double d0 = (double)gi[u].x - (double)gj[u].x;
                const double d1 = (double)gi[u].y - (double)gj[u].y;
                const double e0 = wv[u] * (d0 * d0), e1 = wv[u] * (d1 * d1);
                if (u & 1) {
                    S0b += e0; S1b += e1;
                    Q0b = __builtin_fma(e0, e0, Q0b); Q1b = __builtin_fma(e1, e1, Q1b);
                } else {
                    S0a += e0; S1a += e1;
                    Q0a = __builtin_fma(e0, e0, Q0a); Q1a = __builtin_fma(e1, e1, Q1a);
                }
            }
        }
        // list B: numerator-only entries (v x_i x_j, multiplicity in v)
        double nB0 = 0.0, nB1 = 0.0;
        for (int64_t p0 = naP + lane; p0 < neP; p0 += E2_CH) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t ij = seij[p0 + 64 * u];
                const double v = sev[p0 + 64 * u];
                const stage_t gi = *reinterpret_cast<const stage_t *>(xsb + (ij & 0xFFFFu));
                const stage_t gj = *reinterpret_cast<const stage_t *>(xsb + (ij >> 16));
                nB0 = __builtin_fma(v, (double)gi.x * (double)gj.x, nB0);
                nB1 = __builtin_fma(v, (double)gi.y * (double)gj.y, nB1);
            }
        }
        const double SA[2] = {S0a + S0b, S1a + S1b}, QA[2] = {Q0a + Q0b, Q1a + Q1b};
        const double nBs[2] = {nB0, nB1};
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const double SAs = wave_sum_dpp(SA[t]);
            const double num = wave_sum_dpp(numD[t] + nBs[t]) + SAs;
            const double Ss = mA_g * SAs;
            const double Qs = mA_g * wave_sum_dpp(QA[t]);
            const double dn = wave_sum_dpp(den[t]);
            const bool nonzero = __any(nzr[t]) != 0;
            double e_raw = 0.0, g_raw = 0.0, lam = 0.0;
            if (g_mode == MN_G_SPECTRAL) {
                const double rr = num / (dn + 1e-9);
                e_raw = rr < -1e6 ? -1e6 : (rr > 1e6 ? 1e6 : rr);
                g_raw = Ss;
                lam = e_raw;
            } else if (!(g_mode == MN_G_TAUMODE && !nonzero)) {  // zero vector: lambda 0
                e_raw = dn > 1e-12 ? fmax(num / dn, 0.0) : 0.0;
                if (Ss > 1e-12) {
                    const double g = Qs / (Ss * Ss);
                    g_raw = g < 0.0 ? 0.0 : (g > 1.0 ? 1.0 : g);
                }
                if (g_mode == MN_G_TAUMODE) {
                    const double ebv = e_raw / (e_raw + tau[t]);
                    lam = tau[t] * ebv + (1.0 - tau[t]) * g_raw;
                } else {
                    lam = e_raw;
                }
            }
            if (lane == 0 && r0 + t < n) {
                if (Eo) Eo[r0 + t] = e_raw;
                if (Go) Go[r0 + t] = g_raw;
                if (Lo) Lo[r0 + t] = lam;
            }
        }
        __builtin_amdgcn_wave_barrier();  // the stage is rewritten next pass
    }
}

// ---- register-resident entry lists (the C3 shape: ne <= 64 NE) -------------
// The entry lists are the same for every row, so each lane keeps its slots
// p = lane + 64 t in registers for the whole launch (list A padded to whole
// slots with zero-weight entries, then list B from slot tA on): a pass over
// two rows then needs only the two 16-B gathers (f64 pair of both rows) per
// entry, all addresses known up front — no per-entry LDS list reads and no
// load -> gather dependency, which left the LDS-list kernel latency-bound
// (SQ wait_any 0.60).  Rows are staged in LDS as f64 pairs (no per-entry
// conversions).  Same arithmetic as k_energy_rows (f64, the A/B multiplicities
// applied once per row).
template <int NR, int NE>
__global__ __launch_bounds__(NE <= 16 ? 512 : 256) void k_energy_rows_reg(
    const float *__restrict__ X, int64_t n, int f, int64_t na, int64_t ne,
    const uint32_t *__restrict__ geij, const double *__restrict__ gev, double mA_num,
    double mA_g, int g_mode, int tau_mode, double tau_param, int pct_rank,
    double *__restrict__ Eo, double *__restrict__ Go, double *__restrict__ Lo) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    double2 *xs = (double2 *)dsm + (size_t)w * f;
    int *hist = (int *)((double2 *)dsm + (size_t)nw * f) + w * 256;
    // this lane's slots: A (padded to whole slots) then B
    const int tA = (int)((na + 63) / 64);
    const int64_t nb = ne - na;
    uint32_t eij[NE];
    double ev[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) {
        int64_t p;
        bool ok;
        if (t < tA) {
            p = (int64_t)t * 64 + lane;
            ok = p < na;
        } else {
            p = na + (int64_t)(t - tA) * 64 + lane;
            ok = p < ne && (t - tA) * 64 + lane < nb;
        }
        eij[t] = ok ? geij[p] : 0u;
        ev[t] = ok ? gev[p] : 0.0;
    }
    const int64_t npass = (n + 1) / 2;
    for (int64_t ps = (int64_t)blockIdx.x * nw + w; ps < npass; ps += (int64_t)gridDim.x * nw) {
        const int64_t r0 = ps * 2;
        double den[2], msum[2];
        bool nonzero[2];
        {
            const float *x0 = X + r0 * (int64_t)f;
            const float *x1 = X + min(r0 + 1, n - 1) * (int64_t)f;  // a missing last row repeats
            double dn0 = 0.0, dn1 = 0.0, ms0 = 0.0, ms1 = 0.0;
            bool nz0 = false, nz1 = false;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int c = lane + 64 * r;
                if (c < f) {
                    const double a = (double)x0[c], b = (double)x1[c];
                    xs[c] = make_double2(a, b);
                    dn0 += a * a;
                    dn1 += b * b;
                    ms0 += a;
                    ms1 += b;
                    nz0 |= !(fabs(a) <= 1e-10);
                    nz1 |= !(fabs(b) <= 1e-10);
                }
            }
            den[0] = wave_sum(dn0);
            den[1] = wave_sum(dn1);
            msum[0] = ms0;
            msum[1] = ms1;
            nonzero[0] = __any(nz0) != 0;
            nonzero[1] = __any(nz1) != 0;
        }
        __builtin_amdgcn_wave_barrier();
        double nA0 = 0.0, nA1 = 0.0, nB0 = 0.0, nB1 = 0.0, S0 = 0.0, S1 = 0.0, Q0 = 0.0, Q1 = 0.0;
#pragma unroll
        for (int t = 0; t < NE; ++t) {
            const int i = (int)(eij[t] & 0xFFFFu), j = (int)(eij[t] >> 16);
            const double2 gi = xs[i], gj = xs[j];
            if (t < tA) {  // list A: num -= w x_i x_j, e = w (x_i - x_j)^2
                nA0 = __builtin_fma(-ev[t], gi.x * gj.x, nA0);
                nA1 = __builtin_fma(-ev[t], gi.y * gj.y, nA1);
                const double d0 = gi.x - gj.x, d1 = gi.y - gj.y;
                const double e0 = (d0 * d0) * ev[t], e1 = (d1 * d1) * ev[t];
                S0 += e0;
                S1 += e1;
                Q0 = __builtin_fma(e0, e0, Q0);
                Q1 = __builtin_fma(e1, e1, Q1);
            } else {       // list B: num only
                nB0 = __builtin_fma(ev[t], gi.x * gj.x, nB0);
                nB1 = __builtin_fma(ev[t], gi.y * gj.y, nB1);
            }
        }
        const double nAs[2] = {nA0, nA1}, nBs[2] = {nB0, nB1}, Sv[2] = {S0, S1}, Qv[2] = {Q0, Q1};
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const double num = wave_sum(mA_num * nAs[t] + nBs[t]);
            const double Ss = mA_g * wave_sum(Sv[t]);
            const double Qs = mA_g * wave_sum(Qv[t]);
            double e_raw = 0.0, g_raw = 0.0, lam = 0.0;
            if (g_mode == MN_G_SPECTRAL) {
                const double r = num / (den[t] + 1e-9);
                e_raw = r < -1e6 ? -1e6 : (r > 1e6 ? 1e6 : r);
                g_raw = Ss;
                lam = e_raw;
            } else if (!(g_mode == MN_G_TAUMODE && !nonzero[t])) {  // zero vector: lambda 0
                e_raw = den[t] > 1e-12 ? fmax(num / den[t], 0.0) : 0.0;
                if (Ss > 1e-12) {
                    const double g = Qs / (Ss * Ss);
                    g_raw = g < 0.0 ? 0.0 : (g > 1.0 ? 1.0 : g);
                }
                if (g_mode == MN_G_TAUMODE) {
                    uint32_t keys[NR];
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        const int c = lane + 64 * r;
                        keys[r] = c < f ? f2key((float)(t == 0 ? xs[c].x : xs[c].y)) : 0xFFFFFFFFu;
                    }
                    const double tau =
                        row_tau<NR>(keys, f, msum[t], tau_mode, tau_param, pct_rank, hist);
                    const double ebv = e_raw / (e_raw + tau);
                    lam = tau * ebv + (1.0 - tau) * g_raw;
                } else {
                    lam = e_raw;
                }
            }
            if (lane == 0 && r0 + t < n) {
                if (Eo) Eo[r0 + t] = e_raw;
                if (Go) Go[r0 + t] = g_raw;
                if (Lo) Lo[r0 + t] = lam;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- Stage D global normalisation (spectral/mod.rs:137-145, 177) ------------
// total = sum of the row energies: fixed-order two-level reduction
// (deterministic); then D = clamp(row / (total + 1e-12), 0, 1), lambda = R + D.
constexpr int SUM_BLOCKS = 256;
__global__ __launch_bounds__(256) void k_sum_partials(const double *__restrict__ x, int64_t n,
                                                      double *__restrict__ part) {
    __shared__ double red[4];
    const int64_t per = (n + SUM_BLOCKS - 1) / SUM_BLOCKS;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
    double s = 0.0;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) s += x[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}
__global__ __launch_bounds__(256) void k_spectral_finish(const double *__restrict__ part,
                                                         int64_t n, const double *__restrict__ E,
                                                         double *__restrict__ G,
                                                         double *__restrict__ lam) {
    __shared__ double tot;
    if (threadIdx.x < 64) {
        double s = 0.0;
        for (int q = threadIdx.x; q < SUM_BLOCKS; q += 64) s += part[q];
        s = wave_sum(s);
        if (threadIdx.x == 0) tot = s;
    }
    __syncthreads();
    const double total = tot;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double d = G[i] / (total + 1e-12);
        d = d < 0.0 ? 0.0 : (d > 1.0 ? 1.0 : d);
        G[i] = d;
        if (lam) lam[i] = E[i] + d;
    }
}

// ---- normalise_lambdas -------------------------------------------------
__device__ __forceinline__ unsigned long long d2key(double x) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double key2d(unsigned long long k) {
    const unsigned long long u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)u);
}

__global__ __launch_bounds__(256) void k_minmax(const double *__restrict__ lam, int64_t n,
                                                unsigned long long *__restrict__ mm) {
    unsigned long long mn = ~0ull, mx = 0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double v = lam[i];
        if (v != v) continue;  // f64::min / f64::max ignore NaN
        const unsigned long long k = d2key(v);
        mn = k < mn ? k : mn;
        mx = k > mx ? k : mx;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&mm[0], mn);
        atomicMax(&mm[1], mx);
    }
}

__global__ __launch_bounds__(256) void k_normalise(double *__restrict__ lam, int64_t n,
                                                   const unsigned long long *__restrict__ mm,
                                                   double *__restrict__ out3) {
    const double mnv = mm[0] == ~0ull ? __builtin_inf() : key2d(mm[0]);
    double mxv = mm[1] == 0ull ? 0.0 : key2d(mm[1]);
    mxv = fmax(mxv, 0.0);  // core.rs:1343 max fold starts at 0.0
    const double range = fmax(mxv - mnv, 1e-9);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) lam[i] = (lam[i] - mnv) / range;
    if (i == 0 && out3) { out3[0] = mnv; out3[1] = mxv; out3[2] = range; }
}

// ---- diffusion pre-pass / Laplacian matvec (energymaps.rs:518-546,
//      GraphLaplacian::multiply_vector graph.rs:464-501) ----------------------
// Per row x (f64): steps times x <- x - eta * (L x), (L x)_i = the CSR row
// fold sum += L[i,p] * x[col[p]] from +0.0 in stored order (no FMA), or, in
// matvec mode, y = L x once.  One wave per row, the row double-buffered in
// LDS; L (CSR) in LDS when it fits.  Lane-parallel over features i: every
// fold is its own sequential chain, so the result is bit-exact.
constexpr int DF_SW = 16;  // feature sweeps held in registers (f <= 1024)
template <bool XF64>
__global__ __launch_bounds__(512) void k_diffuse_rows(
    const void *__restrict__ Xin, int64_t n, int f, const int64_t *__restrict__ gip,
    const int32_t *__restrict__ gix, const double *__restrict__ gv, int64_t nnz, int l_in_lds,
    const int32_t *__restrict__ gperm, double eta, int steps, int matvec,
    double *__restrict__ Xout) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    // LDS: [val f64 x nnz | col i32 x nnz | ptr i32 x (f+1) | perm i32 x f]
    //      | x [waves][2][f] f64
    // Lane l of sweep g folds feature row perm[64 g + l]: rows ordered by
    // length (host), so a sweep's 64 chains are about equally long
    double *lv = (double *)dsm;
    int32_t *lc = (int32_t *)(dsm + (size_t)nnz * 8);
    int32_t *lp = lc + nnz;
    int32_t *lperm = lp + f + 1;
    const size_t lb = l_in_lds ? ((((size_t)nnz * 12 + (size_t)(2 * f + 1) * 4) + 15) & ~(size_t)15) : 0;
    double *xb = (double *)(dsm + lb) + (size_t)w * 2 * f;
    if (l_in_lds) {
        for (int64_t p = threadIdx.x; p < nnz; p += blockDim.x) {
            lv[p] = gv[p];
            lc[p] = gix[p];
        }
        for (int i = threadIdx.x; i <= f; i += blockDim.x) lp[i] = (int32_t)gip[i];
        for (int i = threadIdx.x; i < f; i += blockDim.x) lperm[i] = gperm[i];
    }
    __syncthreads();
    // lane l of sweep g: feature row si[g] = perm[64 g + l], entries [sp0, sp1)
    int si[DF_SW], sp0[DF_SW], sp1[DF_SW];
#pragma unroll
    for (int g = 0; g < DF_SW; ++g) {
        const int q = min(lane + 64 * g, f - 1);
        si[g] = l_in_lds ? lperm[q] : 0;
        sp0[g] = l_in_lds ? lp[si[g]] : 0;
        sp1[g] = l_in_lds && lane + 64 * g < f ? lp[si[g] + 1] : sp0[g];
    }
    for (int64_t row = (int64_t)blockIdx.x * nw + w; row < n; row += (int64_t)gridDim.x * nw) {
        double *x = xb, *y = xb + f;
        if (!XF64 && f <= 1024) {
            // f32 rows: all 16 loads in flight at once (buffer loads, columns
            // >= f read 0; a guarded strided loop waits on each load in turn)
            const __amdgpu_buffer_rsrc_t rs = row_rsrc((const float *)Xin + row * f, f);
            float v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = row_at(rs, lane + 64 * r);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (lane + 64 * r < f) x[lane + 64 * r] = (double)v[r];
        } else {
            for (int i = lane; i < f; i += 64)
                x[i] = XF64 ? ((const double *)Xin)[row * f + i]
                            : (double)((const float *)Xin)[row * f + i];
        }
        __builtin_amdgcn_wave_barrier();
        const int ns = matvec ? 1 : steps;
        for (int st = 0; st < ns; ++st) {
            if (l_in_lds && f <= 64 * DF_SW) {
                // row-independent sweep metadata from registers (loaded once)
#pragma unroll
                for (int g = 0; g < DF_SW; ++g) {
                    if (64 * g >= f) break;
                    if (lane + 64 * g < f) {
                        double sum = 0.0;
                        for (int p = sp0[g]; p < sp1[g]; ++p) sum = sum + lv[p] * x[lc[p]];
                        y[si[g]] = matvec ? sum : x[si[g]] - eta * sum;
                    }
                }
                __builtin_amdgcn_wave_barrier();
                double *t = x; x = y; y = t;
                continue;
            }
            for (int q = lane; q < f; q += 64) {
                const int i = l_in_lds ? lperm[q] : gperm[q];
                const int64_t p0 = l_in_lds ? lp[i] : gip[i], p1 = l_in_lds ? lp[i + 1] : gip[i + 1];
                double sum = 0.0;
                for (int64_t p = p0; p < p1; ++p) {
                    const double v = l_in_lds ? lv[p] : gv[p];
                    const int c = l_in_lds ? lc[p] : gix[p];
                    sum = sum + v * x[c];
                }
                y[i] = matvec ? sum : x[i] - eta * sum;
            }
            __builtin_amdgcn_wave_barrier();
            double *t = x; x = y; y = t;
        }
        for (int i = lane; i < f; i += 64) Xout[row * f + i] = x[i];
        __builtin_amdgcn_wave_barrier();
    }
}

// Round 4: the same folds with L's entries interleaved on the host by groups
// of DF_G sweeps — slot ((base_G + t) DF_G + u) 64 + l holds entry t of the
// feature row lane l folds in sweep DF_G G + u (rows by length; rows shorter
// than the group's longest padded with (0, f): the zero slot x[f], an exact
// no-op, as a fold from +0.0 never holds -0.0) — so a wave's value / column
// reads are contiguous (conflict-free) and DF_G independent folds advance per
// step with their loads in flight together (no branch between them).
template <bool XF64, int DF_G, int DF_T>
__global__ __launch_bounds__(512) void k_diffuse_rows2(
    const void *__restrict__ Xin, int64_t n, int f, const double *__restrict__ giv,
    const int32_t *__restrict__ gic, int64_t S, const int32_t *__restrict__ gsw,
    const int32_t *__restrict__ gperm, double eta, int steps, int matvec,
    double *__restrict__ Xout) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const int nsw = (f + 63) / 64;
    // LDS: [val f64 x S | col i32 x S] | x [waves][2][f + 1] f64 (slot f = 0)
    double *iv = (double *)dsm;
    int32_t *ic = (int32_t *)(dsm + (size_t)S * 8);
    const size_t lb = (((size_t)S * 12) + 15) & ~(size_t)15;
    double *xb = (double *)(dsm + lb) + (size_t)w * 2 * (f + 1);
    for (int64_t q = threadIdx.x; q < S; q += blockDim.x) {
        iv[q] = giv[q];
        ic[q] = gic[q];
    }
    __syncthreads();
    constexpr int MAXG = (DF_SW + DF_G - 1) / DF_G;
    int si[DF_SW], sb[MAXG], sl[MAXG];
#pragma unroll
    for (int g = 0; g < DF_SW; ++g) si[g] = gperm[min(lane + 64 * g, f - 1)];
    const int ngr = (nsw + DF_G - 1) / DF_G;
#pragma unroll
    for (int G = 0; G < MAXG; ++G) {
        sb[G] = G < ngr ? gsw[2 * G] : 0;
        sl[G] = G < ngr ? gsw[2 * G + 1] : 0;
    }
    if (lane == 0) {
        xb[f] = 0.0;
        xb[f + 1 + f] = 0.0;
    }
    // f32 rows: the next row's values are loaded during this row's steps
    float nxt[DF_SW];
    auto load_row = [&](int64_t r) {
        const __amdgpu_buffer_rsrc_t rs = row_rsrc((const float *)Xin + min(r, n - 1) * f, f);
#pragma unroll
        for (int q = 0; q < DF_SW; ++q) nxt[q] = row_at(rs, lane + 64 * q);
    };
    const int64_t rstride = (int64_t)gridDim.x * nw;
    if (!XF64) load_row((int64_t)blockIdx.x * nw + w);
    for (int64_t row = (int64_t)blockIdx.x * nw + w; row < n; row += rstride) {
        double *x = xb, *y = xb + (f + 1);
        if (!XF64) {
#pragma unroll
            for (int r = 0; r < DF_SW; ++r)
                if (lane + 64 * r < f) x[lane + 64 * r] = (double)nxt[r];
            if (row + rstride < n) load_row(row + rstride);
        } else {
            for (int i = lane; i < f; i += 64) x[i] = ((const double *)Xin)[row * f + i];
        }
        __builtin_amdgcn_wave_barrier();
        const int ns = matvec ? 1 : steps;
        for (int st = 0; st < ns; ++st) {
            // groups of DF_G sweeps advance together, padded to the group's
            // longest row: DF_G independent folds per step, their loads issued
            // ahead with no branch in the way (each fold keeps its order)
#pragma unroll
            for (int G = 0; G < MAXG; ++G) {
                if (G >= ngr) break;
                const int base = __builtin_amdgcn_readfirstlane(sb[G]);
                const int len = __builtin_amdgcn_readfirstlane(sl[G]);
                double sum[DF_G];
#pragma unroll
                for (int u = 0; u < DF_G; ++u) sum[u] = 0.0;
                const double *pv = iv + (size_t)base * (DF_G * 64) + lane;
                const int32_t *pc = ic + (size_t)base * (DF_G * 64) + lane;
                // DF_T entries of each fold per iteration (len is a multiple)
                for (int t = 0; t < len; t += DF_T) {
                    int c[DF_T][DF_G];
                    double v[DF_T][DF_G], xv[DF_T][DF_G];
#pragma unroll
                    for (int e = 0; e < DF_T; ++e)
#pragma unroll
                        for (int u = 0; u < DF_G; ++u) {
                            c[e][u] = pc[((t + e) * DF_G + u) * 64];
                            v[e][u] = pv[((t + e) * DF_G + u) * 64];
                        }
#pragma unroll
                    for (int e = 0; e < DF_T; ++e)
#pragma unroll
                        for (int u = 0; u < DF_G; ++u) xv[e][u] = x[c[e][u]];
#pragma unroll
                    for (int e = 0; e < DF_T; ++e)
#pragma unroll
                        for (int u = 0; u < DF_G; ++u) sum[u] = sum[u] + v[e][u] * xv[e][u];
                }
#pragma unroll
                for (int u = 0; u < DF_G; ++u) {
                    const int g = DF_G * G + u;
                    if (g < DF_SW && g < nsw && lane + 64 * g < f)
                        y[si[g < DF_SW ? g : 0]] = matvec ? sum[u] : x[si[g < DF_SW ? g : 0]] - eta * sum[u];
                }
            }
            __builtin_amdgcn_wave_barrier();
            double *t = x; x = y; y = t;
        }
        for (int i = lane; i < f; i += 64) Xout[row * f + i] = x[i];
        __builtin_amdgcn_wave_barrier();
    }
}

// Round 4b: the same folds with an iteration's E = DF_G x DF_T entries of a
// lane stored contiguously — values as E/2 double2 pieces [it][h][lane],
// columns as int2 / int4 pieces [it][q][lane] — so a lane's values and
// columns come in by ds_read_b128 (b64 for two columns; 16-B lane stride:
// conflict-free) instead of one ds_read_b64 / b32 per entry: the value /
// column reads were 12 of the 20 LDS bytes an entry costs, on the narrow
// instructions, and the kernel is LDS-bound.  Entry k = e DF_G + u of an
// iteration is entry t = DF_T it + e of fold u; pads (0, f) read the zero slot.
// C3 (same process, profiles/r04/r04_diffusion_v3_ab.log, bit-identical):
// rows2 (2, 1) 9.62-9.69 ms -> rows3 (2, 1) 8.94-8.96, (4, 1) 8.80-8.94, (2, 2)
// 8.89-8.92, (2, 4) 9.59, (1, 2) 11.2, (1, 4) 12.0.  What bounds it: ~2.5 KB of
// LDS reads per (2, 1) iteration and wave (a 1-KB value piece, 512-B columns,
// two 512-B x gathers), ~54 iterations per row and step: ~540 GB over the
// 1M rows x 4 steps, ~120 B/clk per CU at 8.9 ms — the LDS array's rate for
// the b64 gathers.
template <bool XF64, int DF_G, int DF_T>
__global__ __launch_bounds__(512) void k_diffuse_rows3(
    const void *__restrict__ Xin, int64_t n, int f, const double *__restrict__ giv,
    const int32_t *__restrict__ gic, int64_t S, const int32_t *__restrict__ gsw,
    const int32_t *__restrict__ gperm, double eta, int steps, int matvec,
    double *__restrict__ Xout) {
    constexpr int E = DF_G * DF_T;
    static_assert(E == 2 || E == 4 || E == 8, "E in {2, 4, 8}");
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const int nsw = (f + 63) / 64;
    // LDS: [val f64 x S | col i32 x S] | x [waves][2][f + 1] f64 (slot f = 0)
    double *iv = (double *)dsm;
    int32_t *ic = (int32_t *)(dsm + (size_t)S * 8);
    const size_t lb = (((size_t)S * 12) + 15) & ~(size_t)15;
    double *xb = (double *)(dsm + lb) + (size_t)w * 2 * (f + 1);
    {   // S is a multiple of 64 E: 16-B pieces
        const double2 *g2 = (const double2 *)giv;
        double2 *l2 = (double2 *)iv;
        for (int64_t q = threadIdx.x; q < S / 2; q += blockDim.x) l2[q] = g2[q];
        const int4 *c4 = (const int4 *)gic;
        int4 *lc4 = (int4 *)ic;
        for (int64_t q = threadIdx.x; q < S / 4; q += blockDim.x) lc4[q] = c4[q];
    }
    __syncthreads();
    constexpr int MAXG = (DF_SW + DF_G - 1) / DF_G;
    int si[DF_SW], sb[MAXG], sl[MAXG];
#pragma unroll
    for (int g = 0; g < DF_SW; ++g) si[g] = gperm[min(lane + 64 * g, f - 1)];
    const int ngr = (nsw + DF_G - 1) / DF_G;
#pragma unroll
    for (int G = 0; G < MAXG; ++G) {
        sb[G] = G < ngr ? gsw[2 * G] : 0;
        sl[G] = G < ngr ? gsw[2 * G + 1] : 0;
    }
    if (lane == 0) {
        xb[f] = 0.0;
        xb[f + 1 + f] = 0.0;
    }
    float nxt[DF_SW];
    auto load_row = [&](int64_t r) {
        const __amdgpu_buffer_rsrc_t rs = row_rsrc((const float *)Xin + min(r, n - 1) * f, f);
#pragma unroll
        for (int q = 0; q < DF_SW; ++q) nxt[q] = row_at(rs, lane + 64 * q);
    };
    const int64_t rstride = (int64_t)gridDim.x * nw;
    if (!XF64) load_row((int64_t)blockIdx.x * nw + w);
    const double2 *iv2 = (const double2 *)iv;
    for (int64_t row = (int64_t)blockIdx.x * nw + w; row < n; row += rstride) {
        double *x = xb, *y = xb + (f + 1);
        if (!XF64) {
#pragma unroll
            for (int r = 0; r < DF_SW; ++r)
                if (lane + 64 * r < f) x[lane + 64 * r] = (double)nxt[r];
            if (row + rstride < n) load_row(row + rstride);
        } else {
            for (int i = lane; i < f; i += 64) x[i] = ((const double *)Xin)[row * f + i];
        }
        __builtin_amdgcn_wave_barrier();
        const int ns = matvec ? 1 : steps;
        for (int st = 0; st < ns; ++st) {
#pragma unroll
            for (int G = 0; G < MAXG; ++G) {
                if (G >= ngr) break;
                const int base = __builtin_amdgcn_readfirstlane(sb[G]);
                const int len = __builtin_amdgcn_readfirstlane(sl[G]);
                double sum[DF_G];
#pragma unroll
                for (int u = 0; u < DF_G; ++u) sum[u] = 0.0;
                for (int it = base; it < base + len; ++it) {
                    double v[E];
                    int c[E];
#pragma unroll
                    for (int h = 0; h < E / 2; ++h) {
                        const double2 t = iv2[((size_t)it * (E / 2) + h) * 64 + lane];
                        v[2 * h] = t.x;
                        v[2 * h + 1] = t.y;
                    }
                    if constexpr (E == 2) {
                        const int2 t = ((const int2 *)ic)[(size_t)it * 64 + lane];
                        c[0] = t.x;
                        c[1] = t.y;
                    } else {
#pragma unroll
                        for (int q = 0; q < E / 4; ++q) {
                            const int4 t = ((const int4 *)ic)[((size_t)it * (E / 4) + q) * 64 + lane];
                            c[4 * q] = t.x; c[4 * q + 1] = t.y; c[4 * q + 2] = t.z; c[4 * q + 3] = t.w;
                        }
                    }
                    double xv[E];
#pragma unroll
                    for (int k = 0; k < E; ++k) xv[k] = x[c[k]];
#pragma unroll
                    for (int e = 0; e < DF_T; ++e)
#pragma unroll
                        for (int u = 0; u < DF_G; ++u)
                            sum[u] = sum[u] + v[e * DF_G + u] * xv[e * DF_G + u];
                }
#pragma unroll
                for (int u = 0; u < DF_G; ++u) {
                    const int g = DF_G * G + u;
                    if (g < DF_SW && g < nsw && lane + 64 * g < f)
                        y[si[g < DF_SW ? g : 0]] = matvec ? sum[u] : x[si[g < DF_SW ? g : 0]] - eta * sum[u];
                }
            }
            __builtin_amdgcn_wave_barrier();
            double *t = x; x = y; y = t;
        }
        for (int i = lane; i < f; i += 64) Xout[row * f + i] = x[i];
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- item-graph orientation: energy of the F feature signals (length n) ----
// node_energy_and_dispersion(X^T, L_items) (energymaps.rs:923-1045 with the
// n x n item Laplacian; SURVEY §8(d) orientation (ii)): per signal s_f =
// X[:, f], E_f = max(0, s^T L s / s^T s) and G_f = sum (e/S)^2 over the
// dispersion's pairs.  One block per contiguous range of graph rows i, 256
// threads over the signals (coalesced row loads of X); per stored entry
// (i, j, v) the row x_j is gathered once and serves every signal.  Block
// partials [block][4][f] (num, den, S, Q) are summed in a fixed order.
// Round 4: an entry's multiplicities and weights are folded into three
// per-entry coefficients (uniform: scalar registers) — num += (m v)(x_i x_j),
// S += (mg w) d^2, Q += (mg w^2) d^4 with w = -v, d = x_i - x_j (the same sums
// as m v x_i x_j, mg e, mg e^2 with e = w d^2, reassociated: 8 f64 operations
// per entry and signal instead of 14, within the 1e-9 tolerance) — entries
// outside the dispersion's pair set carry zero S / Q coefficients (exact
// no-ops: no branch); for a symmetric L with ascending rows (k_check_sym bit
// 4 clear) a row's j < i prefix is skipped by a binary search instead of
// being walked.  NE entries' gathers are issued together (C3, same process,
// profiles/r04/r04_signals_ab.log: NE 4 18.5 ms, 2 18.1-19.5, 8 20.0; the
// round-3 kernel 22.5 ms in the bench).  Measured and dropped: one wave per
// row with dwordx4 gathers (12 signals a lane, the entry's coefficients once
// per wave): 27 ms — 218 VGPRs, two waves a SIMD, the gathers' latency
// exposed.
template <int FPT, int NE>
__global__ __launch_bounds__(256) void k_energy_signals(
    const float *__restrict__ X, int64_t n, int f, const int64_t *__restrict__ ip,
    const int32_t *__restrict__ ix, const double *__restrict__ v, int sym, int skip, int g_mode,
    int64_t rows_per_block, double *__restrict__ part) {
    const int t = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(n, r0 + rows_per_block);
    double num[FPT], den[FPT], S[FPT], Q[FPT];
#pragma unroll
    for (int u = 0; u < FPT; ++u) num[u] = den[u] = S[u] = Q[u] = 0.0;
    const double mnum = sym ? 2.0 : 1.0;
    const double mg = (sym && g_mode == MN_G_TAUMODE) ? 2.0 : 1.0;
    for (int64_t i = r0; i < r1; ++i) {
        double xi[FPT];
        {
            const __amdgpu_buffer_rsrc_t rs = row_rsrc(X + i * f, f);  // columns >= f read 0
#pragma unroll
            for (int u = 0; u < FPT; ++u) {
                xi[u] = (double)row_at(rs, t + 256 * u);
                den[u] += xi[u] * xi[u];
            }
        }
        int64_t p0 = ip[i];
        const int64_t p1 = ip[i + 1];
        if (skip) {  // ascending row: the first entry with j >= i
            int64_t lo = p0, hi = p1;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (ix[mid] < i) lo = mid + 1; else hi = mid;
            }
            p0 = lo;
        }
        for (int64_t p = p0; p < p1; p += NE) {
            double cm[NE], ca[NE], cq[NE];
            float xjf[NE][FPT];
#pragma unroll
            for (int u = 0; u < NE; ++u) {
                const bool in = p + u < p1;
                const int j = in ? ix[p + u] : 0;
                const double vv = in ? v[p + u] : 0.0;
                const bool ok = in && !(sym && j < i);  // (j, i) covers j < i
                const bool g = ok && j != i && -vv > 0.0 && (g_mode == MN_G_TAUMODE || sym || j > i);
                cm[u] = ok ? ((j != i) ? mnum : 1.0) * vv : 0.0;
                ca[u] = g ? mg * -vv : 0.0;
                cq[u] = g ? mg * (vv * vv) : 0.0;
                // a skipped entry gets a zero-length resource: reads 0, no traffic
                const __amdgpu_buffer_rsrc_t rs = row_rsrc(X + (int64_t)j * f, ok ? f : 0);
#pragma unroll
                for (int w = 0; w < FPT; ++w) xjf[u][w] = row_at(rs, t + 256 * w);
            }
            __builtin_amdgcn_sched_barrier(0);  // the gathers issue before the folds
#pragma unroll
            for (int u = 0; u < NE; ++u)
#pragma unroll
                for (int w = 0; w < FPT; ++w) {
                    const double xj = (double)xjf[u][w];
                    num[w] = __builtin_fma(cm[u], xi[w] * xj, num[w]);
                    const double dd = xi[w] - xj;
                    const double d2 = dd * dd;
                    S[w] = __builtin_fma(ca[u], d2, S[w]);
                    Q[w] = __builtin_fma(cq[u], d2 * d2, Q[w]);
                }
        }
    }
    double *pb = part + (size_t)blockIdx.x * 4 * f;
#pragma unroll
    for (int u = 0; u < FPT; ++u) {
        const int c = t + 256 * u;
        if (c < f) {
            pb[c] = num[u];
            pb[f + c] = den[u];
            pb[2 * f + c] = S[u];
            pb[3 * f + c] = Q[u];
        }
    }
}

// First level of the fixed-order partial fold: segment y of the nb block
// partials (contiguous, ascending b) summed per signal, so the finish reads
// kSegs partials instead of nb (thousands) per signal on f threads.
constexpr int kSegs = 64;
__global__ __launch_bounds__(256) void k_energy_signals_fold(const double *__restrict__ part,
                                                             int nb, int f,
                                                             double *__restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= f) return;
    const int seg = blockIdx.y;
    const int b0 = (int)((int64_t)nb * seg / kSegs), b1 = (int)((int64_t)nb * (seg + 1) / kSegs);
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (int b = b0; b < b1; ++b) {
        const double *pb = part + (size_t)b * 4 * f;
        a0 += pb[c];
        a1 += pb[f + c];
        a2 += pb[2 * f + c];
        a3 += pb[3 * f + c];
    }
    double *o = out + (size_t)seg * 4 * f;
    o[c] = a0;
    o[f + c] = a1;
    o[2 * f + c] = a2;
    o[3 * f + c] = a3;
}

__global__ __launch_bounds__(256) void k_energy_signals_finish(const double *__restrict__ part,
                                                               int nb, int f,
                                                               double *__restrict__ E,
                                                               double *__restrict__ G) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= f) return;
    double num = 0.0, den = 0.0, S = 0.0, Q = 0.0;
    for (int b = 0; b < nb; ++b) {  // fixed order: deterministic
        const double *pb = part + (size_t)b * 4 * f;
        num += pb[c];
        den += pb[f + c];
        S += pb[2 * f + c];
        Q += pb[3 * f + c];
    }
    if (E) E[c] = den > 1e-12 ? fmax(num / den, 0.0) : 0.0;
    if (G) {
        double g = 0.0;
        if (S > 1e-12) {
            g = Q / (S * S);
            g = g < 0.0 ? 0.0 : (g > 1.0 ? 1.0 : g);
        }
        G[c] = g;
    }
}

}  // namespace energy

// LDS-bank-conflict-free entry lists for the f32 stage of k_energy_rows3
// (float2 per column: ds_read_b64 serves lanes 0-31 and 32-63 as two groups;
// column slot s sits on bank pair s mod 32).  A group of 32 entries whose
// x_i slots are distinct mod 32 and whose x_j slots are distinct mod 32
// gathers conflict-free: a matching in the bipartite multigraph of (slot(i)
// mod 32, slot(j) mod 32).  Edge-colouring it with max-degree colours
// (Konig; alternating-path recolouring) gives the groups; the column order
// (slot) is chosen first to balance both degree sides over the 32 classes.
// Each list is padded to whole E2_CH chunks with zero-slot, zero-weight
// entries (exact no-ops); the summation order changes (O(u) of the terms).
struct ConflictFree {
    std::vector<uint32_t> eij;  // (slot(i) | slot(j) << 16), list A then B
    std::vector<double> ev;
    std::vector<int32_t> perm;  // column -> stage slot
    int64_t na = 0, nb = 0;     // padded lengths
};
static ConflictFree conflict_free_lists(const std::vector<uint32_t> &e, const std::vector<double> &v,
                                        int64_t na, int f, int M, int chunk) {
    ConflictFree out;
    const int64_t ne = (int64_t)e.size();
    const int fpad = (f + 3) & ~3;
    // column order: columns by total degree, each to the class with the least
    // max(side-i load, side-j load) that still has room
    std::vector<int64_t> dgi(f, 0), dgj(f, 0);
    for (int64_t q = 0; q < ne; ++q) {
        dgi[e[q] & 0xFFFFu]++;
        dgj[e[q] >> 16]++;
    }
    std::vector<int> cols(f);
    for (int c = 0; c < f; ++c) cols[c] = c;
    std::stable_sort(cols.begin(), cols.end(),
                     [&](int a, int b) { return dgi[a] + dgj[a] > dgi[b] + dgj[b]; });
    const int cap = (f + M - 1) / M;
    std::vector<int64_t> li(M, 0), lj(M, 0);
    std::vector<int> used(M, 0);
    out.perm.assign(f, 0);
    for (int c : cols) {
        int best = -1;
        int64_t bv = 0;
        for (int k = 0; k < M; ++k) {
            if (used[k] >= cap || k + M * used[k] >= fpad) continue;
            const int64_t val = std::max(li[k] + dgi[c], lj[k] + dgj[c]);
            if (best < 0 || val < bv) { best = k; bv = val; }
        }
        out.perm[c] = best + M * used[best];
        used[best]++;
        li[best] += dgi[c];
        lj[best] += dgj[c];
    }
    const uint32_t zpair = (uint32_t)fpad | ((uint32_t)fpad << 16);
    auto colour = [&](int64_t q0, int64_t q1) -> int64_t {
        const int64_t m = q1 - q0;
        if (m == 0) return 0;
        std::vector<int> da(M, 0), db(M, 0);
        std::vector<int> ea(m), eb(m);
        for (int64_t q = 0; q < m; ++q) {
            ea[q] = out.perm[e[q0 + q] & 0xFFFFu] % M;
            eb[q] = out.perm[e[q0 + q] >> 16] % M;
            da[ea[q]]++;
            db[eb[q]]++;
        }
        int D = 0;
        for (int k = 0; k < M; ++k) D = std::max(D, std::max(da[k], db[k]));
        // at[side][vertex][colour] = edge or -1
        std::vector<int> atA((size_t)M * D, -1), atB((size_t)M * D, -1), col(m, -1);
        auto free_at = [&](std::vector<int> &at, int x) {
            for (int c = 0; c < D; ++c)
                if (at[(size_t)x * D + c] < 0) return c;
            return -1;
        };
        for (int64_t q = 0; q < m; ++q) {
            const int a = ea[q], b = eb[q];
            const int ca = free_at(atA, a), cb = free_at(atB, b);
            if (atB[(size_t)b * D + ca] >= 0) {
                // flip the (ca, cb) alternating path from b: afterwards ca is
                // free at b (the path cannot end at a in a bipartite graph)
                std::vector<int> path;
                int x = b;
                bool sideB = true;
                int c = ca;
                for (;;) {
                    const int ed = sideB ? atB[(size_t)x * D + c] : atA[(size_t)x * D + c];
                    if (ed < 0) break;
                    path.push_back(ed);
                    x = sideB ? ea[ed] : eb[ed];
                    sideB = !sideB;
                    c = c == ca ? cb : ca;
                }
                for (int ed : path) {
                    atA[(size_t)ea[ed] * D + col[ed]] = -1;
                    atB[(size_t)eb[ed] * D + col[ed]] = -1;
                }
                for (int ed : path) {
                    col[ed] = col[ed] == ca ? cb : ca;
                    atA[(size_t)ea[ed] * D + col[ed]] = ed;
                    atB[(size_t)eb[ed] * D + col[ed]] = ed;
                }
            }
            col[q] = ca;
            atA[(size_t)a * D + ca] = (int)q;
            atB[(size_t)b * D + ca] = (int)q;
        }
        // groups of M slots: colour classes, zero entries in the gaps; whole chunks
        const int64_t len = ((int64_t)D * M + chunk - 1) / chunk * chunk;
        const size_t base = out.eij.size();
        out.eij.resize(base + len, zpair);
        out.ev.resize(base + len, 0.0);
        std::vector<int> fill(D, 0);
        for (int64_t q = 0; q < m; ++q) {
            const size_t slotq = base + (size_t)col[q] * M + fill[col[q]]++;
            const uint32_t ij = e[q0 + q];
            out.eij[slotq] = (uint32_t)out.perm[ij & 0xFFFFu] | ((uint32_t)out.perm[ij >> 16] << 16);
            out.ev[slotq] = v[q0 + q];
        }
        return len;
    };
    out.na = colour(0, na);
    out.nb = colour(na, ne);
    return out;
}

static thread_local mn_energy_stats t_energy_stats{};

static int energy_impl(const mn_csr *L, const float *X, int64_t n, int32_t f,
                       const mn_energy_opts *opts, double *E, double *G, double *lam) {
    using namespace energy;
    clear_error();
    t_energy_stats = mn_energy_stats{};
    MN_REQUIRE(L && opts && X, MN_EINVAL, "mn_energy_rows: NULL argument");
    MN_REQUIRE(f >= 1 && f <= FMAX && n >= 0, MN_EINVAL,
               "mn_energy_rows: f=%d outside [1,%d]", f, FMAX);
    MN_REQUIRE(L->n_rows == f && L->n_cols == f, MN_EINVAL,
               "mn_energy_rows: Laplacian must be f x f (feature space), got %lld x %lld",
               (long long)L->n_rows, (long long)L->n_cols);
    MN_REQUIRE(opts->g_mode == MN_G_TAUMODE || opts->g_mode == MN_G_ENERGYMAPS ||
                   opts->g_mode == MN_G_SPECTRAL,
               MN_EINVAL, "mn_energy_rows: unknown g_mode");
    MN_REQUIRE(L->value_type == MN_F64 || (L->value_type == MN_F32 && opts->g_mode == MN_G_SPECTRAL),
               MN_ENOTSUP,
               "mn_energy_rows: Laplacian values must be f64 (legacy GraphLaplacian); f32 only "
               "for MN_G_SPECTRAL (Stage C output)");
    MN_REQUIRE(opts->tau_mode >= MN_TAU_FIXED && opts->tau_mode <= MN_TAU_PERCENTILE, MN_EINVAL,
               "mn_energy_rows: unknown tau_mode");
    hipStream_t s = (hipStream_t)opts->stream;
    if (n == 0) return MN_OK;
    const int64_t nnz = L->nnz;
    const bool spec = opts->g_mode == MN_G_SPECTRAL;
    const Vals vals{L->values, L->value_type == MN_F32 ? 1 : 0};
    char *g = (char *)scratch(kSlotGeneric0, (size_t)nnz * 12 + (size_t)f * 8 +
                                                 (size_t)(2 * f + 1) * 8 + (size_t)f * 8 + 256);
    if (spec) {  // E and the raw row energies are needed for the global pass
        double *sc = (double *)scratch(kSlotNorms2, (size_t)n * 16 + 8 * SUM_BLOCKS + 64);
        MN_REQUIRE(sc, MN_ENOMEM, "mn_energy_rows: scratch allocation failed");
        if (!E) E = sc;
        if (!G) G = sc + n;
    }
    MN_REQUIRE(g, MN_ENOMEM, "mn_energy_rows: scratch allocation failed");
    uint32_t *eij = (uint32_t *)g;
    int32_t *cnt = (int32_t *)(eij + nnz);
    double *ev = (double *)(((uintptr_t)(cnt + 2 * f) + 15) & ~(uintptr_t)15);
    int64_t *off = (int64_t *)(ev + nnz);
    double *dg = (double *)(off + 2 * f);
    int *flag = (int *)(dg + f);

    Timer tm;
    tm.start(opts->timing != 0, s);
    MN_HIP_TRY(hipMemsetAsync(flag, 0, 16, s));
    unsigned long long *ubal = (unsigned long long *)(flag + 2);
    const unsigned fb = (unsigned)((f + 255) / 256);
    if (L->nnz > 0)
        hipLaunchKernelGGL(k_check_sym, dim3(check_sym_grid(f)), dim3(256), 0, s,
                           L->indptr, L->indices, vals, f, flag, ubal);
    int hflag[4] = {0, 0, 0, 0};
    MN_HIP_TRY(hipMemcpyAsync(hflag, flag, 16, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(!(hflag[0] & 2), MN_EINVAL, "mn_energy_rows: Laplacian column index out of range");
    const int sym = ((hflag[0] & 1) || hflag[2] != 0 || hflag[3] != 0) ? 0 : 1;
    // k_energy_rows2 (default for f <= 1024; MN_ENERGY_V1=1: the round-2
    // kernels) takes the diagonal apart from the entry lists
    const char *v1e = knob("MN_ENERGY_V1");
    const int nr = (f + 63) / 64;
    int split = (nr <= 16 && !(v1e && *v1e == '1')) ? 1 : 0;
    int64_t na = 0, ne = 0;
    std::vector<int32_t> hc(2 * (size_t)f);
    std::vector<int64_t> ho(2 * (size_t)f);
    for (int attempt = 0; attempt < 2; ++attempt) {
    hipLaunchKernelGGL(k_count_entries, dim3(fb), dim3(256), 0, s, L->indptr, L->indices, vals,
                       f, sym, opts->g_mode, split, cnt);
    // tiny scan on the host side of the stream (f <= 4096): list A, then B
    MN_HIP_TRY(hipMemcpyAsync(hc.data(), cnt, 8 * (size_t)f, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    int64_t acc = 0;
    for (int i = 0; i < 2 * f; ++i) {
        ho[i] = acc;
        acc += hc[i];
    }
    na = ho[f];
    ne = acc;
    if (split && e2_lds_bytes(na, ne - na, f, E2_MIN_WAVES) > LDS_BUDGET) {
        split = 0;  // lists too long for the v2 LDS plan: rebuild them whole
        continue;
    }
    break;
    }
    MN_HIP_TRY(hipMemcpyAsync(off, ho.data(), 16 * (size_t)f, hipMemcpyHostToDevice, s));
    // K3 v3 (one pass over X, the list-A identity) for a symmetric L whose
    // lists fit its LDS plan; else k_row_tau + k_energy_rows2
    int64_t naP3 = (na + E2_CH - 1) / E2_CH * E2_CH;
    int64_t nbP3 = (ne - na + E2_CH - 1) / E2_CH * E2_CH;
    // default 2: the float2 stage at 16 waves a block (C3 median 2.31-2.48
    // ms vs 2.84-2.92 for the double2 stage at 8 waves, fixed tau 1.42 vs
    // 1.49: profiles/r04/r04_energy_ab.log).  Tuning build: MN_ENERGY_V3 = 0
    // the two-kernel path, 1 the double2 stage, 3 the float2 stage with the
    // host-ordered bank-conflict-free lists (slower: fixed 1.74 ms — the
    // kernel is VALU-bound, 17 VALU a lane per entry pair, not LDS-bound)
    const char *v3e = knob("MN_ENERGY_V3");
    const int v3k = (v3e && *v3e) ? atoi(v3e) : 2;
    const bool s64 = v3k == 1;
    const bool v3 = split && sym && nr <= 16 && v3k != 0 &&
                    e3_lds_bytes(naP3 + nbP3, f, s64 ? E3<true>::WAVES : E3<false>::WAVES,
                                 s64 ? E3<true>::XB : E3<false>::XB) <= LDS_BUDGET;
    hipLaunchKernelGGL(k_fill_entries, dim3(fb), dim3(256), 0, s, L->indptr, L->indices, vals, f,
                       sym, opts->g_mode, split, off, eij, ev, dg, v3 ? 1 : 0);
    // v3k 3: the f32 stage with LDS-bank-conflict-free entry lists (host
    // order, conflict_free_lists) in a bank-balanced column order
    const int32_t *perm3 = nullptr;
    const uint32_t *eij3 = eij;
    const double *ev3 = ev;
    int64_t naO = na, nbO = ne - na;
    if (v3 && v3k == 3) {
        std::vector<uint32_t> he((size_t)ne);
        std::vector<double> hv((size_t)ne);
        if (ne > 0) {
            MN_HIP_TRY(hipMemcpyAsync(he.data(), eij, 4 * (size_t)ne, hipMemcpyDeviceToHost, s));
            MN_HIP_TRY(hipMemcpyAsync(hv.data(), ev, 8 * (size_t)ne, hipMemcpyDeviceToHost, s));
            MN_HIP_TRY(hipStreamSynchronize(s));
        }
        ConflictFree cf = conflict_free_lists(he, hv, na, f, 32, E2_CH);
        const size_t nbytes = cf.eij.size() * 12 + (size_t)f * 4 + 256;
        char *cb = (char *)scratch(kSlotGeneric1, nbytes);
        MN_REQUIRE(cb, MN_ENOMEM, "mn_energy_rows: list scratch allocation failed");
        double *dv = (double *)cb;
        uint32_t *de = (uint32_t *)(cb + cf.eij.size() * 8);
        int32_t *dp = (int32_t *)(cb + ((cf.eij.size() * 12 + 15) & ~(size_t)15));
        MN_HIP_TRY(hipMemcpyAsync(dv, cf.ev.data(), 8 * cf.ev.size(), hipMemcpyHostToDevice, s));
        MN_HIP_TRY(hipMemcpyAsync(de, cf.eij.data(), 4 * cf.eij.size(), hipMemcpyHostToDevice, s));
        MN_HIP_TRY(hipMemcpyAsync(dp, cf.perm.data(), 4 * (size_t)f, hipMemcpyHostToDevice, s));
        if (e3_lds_bytes(cf.na + cf.nb, f, E3<false>::WAVES, E3<false>::XB) <= LDS_BUDGET) {
            perm3 = dp;
            eij3 = de;
            ev3 = dv;
            naO = naP3 = cf.na;
            nbO = nbP3 = cf.nb;
        }
    }
    int pct_rank = 0;
    if (opts->tau_mode == MN_TAU_PERCENTILE) {
        double pp = opts->tau_param;
        pp = pp != pp ? pp : (pp < 0.0 ? 0.0 : (pp > 1.0 ? 1.0 : pp));
        const double fi = std::round((double)(f - 1) * pp);  // f64::round
        pct_rank = (fi != fi || fi < 0) ? 0 : (int)std::min<double>(fi, f - 1);
    }
    // multiplicities of list A: num (2 for the upper-triangle list), dispersion
    // (taumode counts each undirected edge twice, energymaps once)
    const double mA_num = sym ? 2.0 : 1.0;
    const double mA_g = (sym && opts->g_mode != MN_G_ENERGYMAPS) ? 2.0 : 1.0;
    tm.mark();
    if (v3) {
        const int nw3 = s64 ? E3<true>::WAVES : E3<false>::WAVES;
        const size_t sh3 = e3_lds_bytes(naP3 + nbP3, f, nw3, s64 ? E3<true>::XB : E3<false>::XB);
        int dev = 0, ncu = 256;
        MN_HIP_TRY(hipGetDevice(&dev));
        MN_HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        const int64_t npass3 = (n + 1) / 2;
        const int64_t blocks3 = std::min<int64_t>((npass3 + nw3 - 1) / nw3, ncu);
        // tuning build: MN_ENERGY_SEL = 0 skips the histogram select (A/B)
        const int sel3 = knob_int("MN_ENERGY_SEL", 1);
#define MN_E3(NRV, S6)                                                                          \
    do {                                                                                        \
        MN_HIP_TRY(hipFuncSetAttribute((const void *)k_energy_rows3<NRV, S6>,                   \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh3));  \
        hipLaunchKernelGGL((k_energy_rows3<NRV, S6>), dim3((unsigned)blocks3), dim3(64 * nw3),  \
                           sh3, s, X, n, f, naO, naP3, nbO, nbP3, eij3, ev3, dg, mA_g,          \
                           opts->g_mode, opts->tau_mode, opts->tau_param, pct_rank, E, G, lam,  \
                           perm3, sel3);                                                        \
    } while (0)
#define MN_E3S(NRV) do { if (s64) MN_E3(NRV, true); else MN_E3(NRV, false); } while (0)
        if (nr <= 4) MN_E3S(4);
        else if (nr <= 8) MN_E3S(8);
        else if (nr <= 12) MN_E3S(12);
        else MN_E3S(16);
#undef MN_E3S
#undef MN_E3
        MN_KCHECK(s, "k_energy_rows3");
    } else if (split) {
        const int64_t naP = (na + E2_CH - 1) / E2_CH * E2_CH;
        const int64_t nbP = (ne - na + E2_CH - 1) / E2_CH * E2_CH;
        const char *tke = knob("MN_ENERGY_TAU");  // 1: the select inside the entry-loop kernel
        const bool tk = tke && *tke == '1';
        const size_t fixed = e2_lds_bytes(na, ne - na, f, 0);
        const size_t wbytes = e2_lds_bytes(na, ne - na, f, 1, tk) - fixed;
        const int nw2 = (int)std::min<size_t>(16, (LDS_BUDGET - fixed) / wbytes);
        const size_t sh2 = fixed + (size_t)nw2 * wbytes;
        const int64_t npass2 = (n + 1) / 2;
        const int64_t blocks2 = std::min<int64_t>((npass2 + nw2 - 1) / nw2, 1024);
        double *tau_d = nullptr;
        if (!tk && opts->g_mode == MN_G_TAUMODE &&
            (opts->tau_mode == MN_TAU_MEDIAN || opts->tau_mode == MN_TAU_PERCENTILE)) {
            tau_d = (double *)scratch(kSlotGeneric1, (size_t)n * 8 + 64);
            MN_REQUIRE(tau_d, MN_ENOMEM, "mn_energy_rows: tau scratch allocation failed");
            // one resident wave set, no second round: blocks = occupancy x CUs
            int dev = 0, ncu = 256;
            MN_HIP_TRY(hipGetDevice(&dev));
            MN_HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
#define MN_TAU(NRV)                                                                             \
    do {                                                                                        \
        int occ = 1;                                                                            \
        MN_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_row_tau<NRV>, 256, 0));   \
        const unsigned tb = (unsigned)std::min<int64_t>((n + 3) / 4, (int64_t)std::max(occ, 1) * ncu); \
        hipLaunchKernelGGL((k_row_tau<NRV>), dim3(tb), dim3(256), 0, s, X, n, f, opts->tau_mode, \
                           opts->tau_param, pct_rank, tau_d);                                   \
    } while (0)
            if (nr <= 4) MN_TAU(4);
            else if (nr <= 8) MN_TAU(8);
            else if (nr <= 12) MN_TAU(12);
            else MN_TAU(16);
#undef MN_TAU
            MN_KCHECK(s, "k_row_tau");
        }
#define MN_E2T(NRV, TKV)                                                                        \
    do {                                                                                        \
        MN_HIP_TRY(hipFuncSetAttribute((const void *)k_energy_rows2<NRV, TKV>,                  \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh2));  \
        hipLaunchKernelGGL((k_energy_rows2<NRV, TKV>), dim3((unsigned)blocks2), dim3(64 * nw2),  \
                           sh2, s, X, n, f, na, naP, ne - na, nbP, eij, ev, dg, mA_num, mA_g,    \
                           opts->g_mode, opts->tau_mode, opts->tau_param, pct_rank, tau_d, E, G, \
                           lam);                                                                \
    } while (0)
#define MN_E2(NRV)                                                                              \
    do {                                                                                        \
        if (tk) MN_E2T(NRV, true); else MN_E2T(NRV, false);                                     \
    } while (0)
        if (nr <= 4) MN_E2(4);
        else if (nr <= 8) MN_E2(8);
        else if (nr <= 12) MN_E2(12);
        else MN_E2(16);
#undef MN_E2
#undef MN_E2T
        MN_KCHECK(s, "k_energy_rows2");
    } else {
    const int fpad = (f + 3) & ~3;
    const size_t ebytes = (((size_t)ne * 12) + 15) & ~(size_t)15;
    const int in_lds = ebytes <= EDGE_LDS_MAX ? 1 : 0;
    // rows per wave pass: MN_ENERGY_ROWS (2 or 4; 4 halves the entry-list
    // reads per row, 16-B gathers, half the waves); tau select MN_TAU_SEL
    const char *rwe = knob("MN_ENERGY_ROWS");
    const int rows = (rwe && *rwe == '4' && nr <= 16) ? 4 : 2;
    const char *sle = knob("MN_TAU_SEL");
    // (MN_ENERGY_PROBE: timing-probe bits 16 / 32, see k_energy_rows)
    const char *epe = knob("MN_ENERGY_PROBE");
    const int sel = ((sle && *sle == '1') ? 1 : 0) | ((epe && *epe) ? (atoi(epe) & 48) : 0);
    const size_t per_wave = (size_t)rows * fpad * 4 + 256 * 4;
    const size_t avail = LDS_BUDGET - (in_lds ? ebytes : 0);
    const int wmax = nr <= 16 ? 16 : 4;  // = launch bounds / 64
    const int nw = (int)std::min<size_t>((size_t)wmax, avail / per_wave);
    MN_REQUIRE(nw >= 1, MN_ENOTSUP, "mn_energy_rows: f=%d does not fit the LDS plan", f);
    const size_t shmem = (in_lds ? ebytes : 0) + (size_t)nw * per_wave;
    const int64_t npass = (n + rows - 1) / rows;
    const int64_t blocks = std::min<int64_t>((npass + nw - 1) / nw, 1024);
    // register-resident entry lists (k_energy_rows_reg): the lists fit 48
    // slots a lane (list A padded to whole slots), rows of <= 1024 features
    const int64_t slots = (na + 63) / 64 + (ne - na + 63) / 64;
    const char *rge = knob("MN_ENERGY_REG");  // 1: register lists (A/B; slower so far)
    const bool reg = slots <= 48 && nr <= 16 && (rge && *rge == '1');
    if (reg) {
        const int nwr = slots <= 16 ? 8 : 4;  // = launch bounds / 64
        const size_t shr = (size_t)nwr * f * 16 + (size_t)nwr * 256 * 4;
        const int64_t blocks_r = std::min<int64_t>((npass + nwr - 1) / nwr, 1024);
#define MN_ERR(NRV, NEV)                                                                        \
    do {                                                                                        \
        MN_HIP_TRY(hipFuncSetAttribute((const void *)k_energy_rows_reg<NRV, NEV>,               \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shr));  \
        hipLaunchKernelGGL((k_energy_rows_reg<NRV, NEV>), dim3((unsigned)blocks_r),             \
                           dim3(64 * nwr), shr, s, X, n, f, na, ne, eij, ev, mA_num, mA_g,       \
                           opts->g_mode, opts->tau_mode, opts->tau_param, pct_rank, E, G, lam); \
    } while (0)
        if (nr <= 4) {
            if (slots <= 16) MN_ERR(4, 16); else if (slots <= 32) MN_ERR(4, 32); else MN_ERR(4, 48);
        } else if (nr <= 8) {
            if (slots <= 16) MN_ERR(8, 16); else if (slots <= 32) MN_ERR(8, 32); else MN_ERR(8, 48);
        } else if (nr <= 12) {
            if (slots <= 16) MN_ERR(12, 16); else if (slots <= 32) MN_ERR(12, 32); else MN_ERR(12, 48);
        } else {
            if (slots <= 16) MN_ERR(16, 16); else if (slots <= 32) MN_ERR(16, 32); else MN_ERR(16, 48);
        }
#undef MN_ERR
    }
#define MN_ER2(NRV, RW)                                                                         \
    do {                                                                                        \
        MN_HIP_TRY(hipFuncSetAttribute((const void *)k_energy_rows<NRV, RW>,                    \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem)); \
        hipLaunchKernelGGL((k_energy_rows<NRV, RW>), dim3((unsigned)blocks), dim3(64 * nw),     \
                           shmem, s, X, n, f, na, ne, in_lds, eij, ev, mA_num, mA_g,             \
                           opts->g_mode, opts->tau_mode, opts->tau_param, pct_rank, E, G, lam,  \
                           sel);                                                                \
    } while (0)
#define MN_ER(NRV)                                                                              \
    do {                                                                                        \
        if (rows == 4 && NRV <= 16) MN_ER2(NRV, 4);                                             \
        else MN_ER2(NRV, 2);                                                                    \
    } while (0)
    if (reg) {
    } else if (nr <= 4) MN_ER(4);
    else if (nr <= 8) MN_ER(8);
    else if (nr <= 12) MN_ER(12);
    else if (nr <= 16) MN_ER(16);
    else if (nr <= 32) MN_ER(32);
    else MN_ER(64);  // f <= 4096
#undef MN_ER
#undef MN_ER2
    MN_KCHECK(s, "k_energy_rows");
    }
    if (spec) {
        double *part = (double *)scratch(kSlotNorms2, (size_t)n * 16 + 8 * SUM_BLOCKS + 64) + 2 * n;
        hipLaunchKernelGGL(k_sum_partials, dim3(SUM_BLOCKS), dim3(256), 0, s, G, n, part);
        hipLaunchKernelGGL(k_spectral_finish,
                           dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                           s, part, n, E, G, lam);
        MN_KCHECK(s, "k_spectral_finish");
    }
    tm.mark();
    MN_HIP_TRY(hipStreamSynchronize(s));
    t_energy_stats.entries = ne;
    t_energy_stats.symmetric = sym;
    t_energy_stats.ms_rows = tm.ms(1, 2);
    t_energy_stats.ms_total = tm.ms(0, 2);
    return MN_OK;
}

static int energy_signals_impl(const mn_csr *L, const float *X, int64_t n, int32_t f,
                               int32_t g_mode, double *E, double *G, void *stream) {
    using namespace energy;
    clear_error();
    MN_REQUIRE(L && X, MN_EINVAL, "mn_energy_signals: NULL argument");
    MN_REQUIRE(n >= 1 && f >= 1 && f <= FMAX, MN_EINVAL, "mn_energy_signals: bad sizes");
    MN_REQUIRE(L->n_rows == n && L->n_cols == n && L->value_type == MN_F64, MN_EINVAL,
               "mn_energy_signals: L must be the n x n f64 item Laplacian");
    MN_REQUIRE(g_mode == MN_G_TAUMODE || g_mode == MN_G_ENERGYMAPS, MN_EINVAL,
               "mn_energy_signals: g_mode must be MN_G_TAUMODE or MN_G_ENERGYMAPS");
    hipStream_t s = (hipStream_t)stream;
    int *flag = (int *)scratch(kSlotFlags, 64);
    const int64_t nb = std::min<int64_t>(n, 16384);
    const int64_t rpb = (n + nb - 1) / nb;
    const int64_t nbu = (n + rpb - 1) / rpb;
    double *part = (double *)scratch(kSlotGeneric0, sizeof(double) * (size_t)nbu * 4 * f + 64);
    MN_REQUIRE(flag && part, MN_ENOMEM, "mn_energy_signals: scratch allocation failed");
    MN_HIP_TRY(hipMemsetAsync(flag, 0, 16, s));
    if (L->nnz > 0)
        hipLaunchKernelGGL(k_check_sym, dim3(check_sym_grid(n)), dim3(256), 0, s,
                           L->indptr, L->indices, Vals{L->values, 0}, (int)n, flag,
                           (unsigned long long *)(flag + 2));
    int hflag4[4] = {0, 0, 0, 0};
    MN_HIP_TRY(hipMemcpyAsync(hflag4, flag, 16, hipMemcpyDeviceToHost, s));
    const int hflag = hflag4[0] | ((hflag4[2] != 0 || hflag4[3] != 0) ? 1 : 0);
    MN_HIP_TRY(hipStreamSynchronize(s));
    MN_REQUIRE(!(hflag & 2), MN_EINVAL, "mn_energy_signals: Laplacian column index out of range");
    const int sym = (hflag & 1) ? 0 : 1;
    const int skip = sym && !(hflag4[0] & 4);  // symmetric, ascending rows
    const int fpt = (f + 255) / 256;
    const char *nee = knob("MN_SIG_NE");  // tuning build: entries per gather batch (2 / 4 / 8)
    const int ne = (nee && *nee) ? atoi(nee) : 4;
#define MN_ES(FP)                                                                               \
    do {                                                                                        \
        if (ne == 2)                                                                            \
            hipLaunchKernelGGL((k_energy_signals<FP, 2>), dim3((unsigned)nbu), dim3(256), 0, s, X, \
                               n, f, L->indptr, L->indices, (const double *)L->values, sym, skip, \
                               g_mode, rpb, part);                                              \
        else if (ne != 8)                                                                       \
            hipLaunchKernelGGL((k_energy_signals<FP, 4>), dim3((unsigned)nbu), dim3(256), 0, s, X, \
                               n, f, L->indptr, L->indices, (const double *)L->values, sym, skip, \
                               g_mode, rpb, part);                                              \
        else                                                                                    \
            hipLaunchKernelGGL((k_energy_signals<FP, 8>), dim3((unsigned)nbu), dim3(256), 0, s, X, \
                               n, f, L->indptr, L->indices, (const double *)L->values, sym, skip, \
                               g_mode, rpb, part);                                              \
    } while (0)
    if (fpt <= 1) MN_ES(1); else if (fpt <= 2) MN_ES(2); else if (fpt <= 3) MN_ES(3);
    else if (fpt <= 4) MN_ES(4); else if (fpt <= 8) MN_ES(8); else MN_ES(16);
#undef MN_ES
    MN_KCHECK(s, "k_energy_signals");
    double *part2 = (double *)scratch(kSlotGeneric1, sizeof(double) * (size_t)kSegs * 4 * f);
    MN_REQUIRE(part2, MN_ENOMEM, "mn_energy_signals: scratch allocation failed");
    hipLaunchKernelGGL(k_energy_signals_fold, dim3((unsigned)((f + 255) / 256), kSegs), dim3(256),
                       0, s, part, (int)nbu, f, part2);
    MN_KCHECK(s, "k_energy_signals_fold");
    hipLaunchKernelGGL(k_energy_signals_finish, dim3((unsigned)((f + 255) / 256)), dim3(256), 0, s,
                       part2, kSegs, f, E, G);
    MN_KCHECK(s, "k_energy_signals_finish");
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

static int diffuse_impl(const mn_csr *L, const void *X, int32_t x_is_f64, int64_t n, int32_t f,
                        double eta, int32_t steps, int matvec, double *out, void *stream) {
    using namespace energy;
    clear_error();
    MN_REQUIRE(L && X && out, MN_EINVAL, "mn_diffuse_rows: NULL argument");
    MN_REQUIRE(n >= 0 && f >= 1 && steps >= 0, MN_EINVAL, "mn_diffuse_rows: bad sizes");
    MN_REQUIRE(L->n_rows == f && L->n_cols == f && L->value_type == MN_F64, MN_EINVAL,
               "mn_diffuse_rows: L must be the f x f f64 GraphLaplacian CSR");
    MN_REQUIRE(x_is_f64 || (const void *)out != X, MN_EINVAL,
               "mn_diffuse_rows: an f32 input cannot alias the f64 output");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return MN_OK;
    const int64_t nnz = L->nnz;
    // feature rows by length (descending, stable): the lanes of one sweep fold
    // rows of about equal length (per-row order unchanged: bit-exact)
    std::vector<int64_t> hip_(f + 1);
    MN_HIP_TRY(hipMemcpyAsync(hip_.data(), L->indptr, 8 * ((size_t)f + 1), hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    std::vector<int32_t> hperm(f);
    for (int i = 0; i < f; ++i) hperm[i] = i;
    std::stable_sort(hperm.begin(), hperm.end(), [&](int a, int b) {
        return hip_[a + 1] - hip_[a] > hip_[b + 1] - hip_[b];
    });
    int32_t *perm = (int32_t *)scratch(kSlotGeneric2, (size_t)f * 4 + 64);
    MN_REQUIRE(perm, MN_ENOMEM, "mn_diffuse_rows: scratch allocation failed");
    MN_HIP_TRY(hipMemcpyAsync(perm, hperm.data(), 4 * (size_t)f, hipMemcpyHostToDevice, s));
    // round 4 fast path (f <= 1024): L interleaved by sweep (k_diffuse_rows2)
    {
        const int nsw = (f + 63) / 64;
        // sweeps per group: all of them for f <= 768 (12 independent folds a
        // step), else 4; tuning build: MN_DIFFUSE_G in {2, 4, 6, 12}
        // folds per group DF_G x entries per iteration DF_T at C3 (4 steps):
        // (2, 1) 9.5 ms, (2, 2) 10.0, (4, 1) 10.1, (4, 2) 10.5, (2, 4) 11.2,
        // (6, 1) 11.3, (1, 2) 11.7, (1, 4) 12.9, (12, 1) 15.4; the round-3
        // kernel 14.8 (profiles/r04/r04_diffusion_ab.log) — padding to the
        // group's longest row outweighs more independent folds; tuning build:
        // MN_DIFFUSE_GT = "G,T" with G in {1, 2, 4}, T in {1, 2, 4}
        const char *dge = knob("MN_DIFFUSE_GT");
        int DF_G = 2, DF_T = 1;
        if (dge && *dge) sscanf(dge, "%d,%d", &DF_G, &DF_T);
        if (DF_G != 1 && DF_G != 2 && DF_G != 4) DF_G = 2;
        if (DF_T != 1 && DF_T != 2 && DF_T != 4) DF_T = 1;
        const int ngr = (nsw + DF_G - 1) / DF_G;
        std::vector<int32_t> sw(2 * (size_t)ngr);
        int64_t S = 0;  // in steps of DF_G x 64 slots
        for (int G = 0; G < ngr; ++G) {
            int64_t mx = 0;
            for (int q = 64 * DF_G * G; q < std::min(f, 64 * DF_G * (G + 1)); ++q) {
                const int i = hperm[q];
                mx = std::max<int64_t>(mx, hip_[i + 1] - hip_[i]);
            }
            mx = (mx + DF_T - 1) / DF_T * DF_T;
            sw[2 * G] = (int32_t)S;
            sw[2 * G + 1] = (int32_t)mx;
            S += mx;
        }
        S *= DF_G;  // in steps of 64 slots
        const size_t lb2 = ((size_t)S * 64 * 12 + 15) & ~(size_t)15;
        const size_t pw2 = (size_t)2 * (f + 1) * 8;
        const char *dfe = knob("MN_DIFFUSE_V1");  // tuning build: 1 = the round-3 kernel (A/B)
        const char *d3e = knob("MN_DIFFUSE_V3");  // tuning build: 0 = the round-4 rows2 layout
        const int E3 = DF_G * DF_T;
        if (f <= 64 * DF_SW && lb2 + pw2 <= LDS_BUDGET && S * 64 < INT_MAX && !(dfe && *dfe == '1') &&
            !(d3e && *d3e == '0') && (E3 == 2 || E3 == 4 || E3 == 8)) {
            // k_diffuse_rows3 layout: iteration it of group G (sw in iterations)
            std::vector<int32_t> sw3(2 * (size_t)ngr);
            int64_t nit = 0;
            for (int G = 0; G < ngr; ++G) {
                sw3[2 * G] = (int32_t)nit;
                sw3[2 * G + 1] = sw[2 * G + 1] / DF_T;
                nit += sw[2 * G + 1] / DF_T;
            }
            const size_t slots = (size_t)nit * 64 * E3;
            std::vector<int32_t> hix((size_t)nnz);
            std::vector<double> hv((size_t)nnz);
            if (nnz > 0) {
                MN_HIP_TRY(hipMemcpyAsync(hix.data(), L->indices, 4 * (size_t)nnz, hipMemcpyDeviceToHost, s));
                MN_HIP_TRY(hipMemcpyAsync(hv.data(), L->values, 8 * (size_t)nnz, hipMemcpyDeviceToHost, s));
                MN_HIP_TRY(hipStreamSynchronize(s));
            }
            std::vector<double> iv(slots, 0.0);
            std::vector<int32_t> ic(slots, f);  // pads: the zero slot
            for (int g = 0; g < nsw; ++g)
                for (int l = 0; l < 64 && 64 * g + l < f; ++l) {
                    const int i = hperm[64 * g + l];
                    const int G = g / DF_G, u = g % DF_G;
                    for (int64_t p = hip_[i]; p < hip_[i + 1]; ++p) {
                        const int64_t t = p - hip_[i];
                        const int64_t it = sw3[2 * G] + t / DF_T;
                        const int k = (int)(t % DF_T) * DF_G + u;
                        const size_t qv = (((size_t)it * (E3 / 2) + k / 2) * 64 + l) * 2 + k % 2;
                        const size_t qc = E3 == 2 ? ((size_t)it * 64 + l) * 2 + k
                                                  : (((size_t)it * (E3 / 4) + k / 4) * 64 + l) * 4 + k % 4;
                        const int c = hix[p];
                        MN_REQUIRE(c >= 0 && c < f, MN_EINVAL, "mn_diffuse_rows: column index out of range");
                        iv[qv] = hv[p];
                        ic[qc] = c;
                    }
                }
            char *gb = (char *)scratch(kSlotGeneric3, slots * 12 + sw3.size() * 4 + 256);
            MN_REQUIRE(gb, MN_ENOMEM, "mn_diffuse_rows: scratch allocation failed");
            double *div = (double *)gb;
            int32_t *dic = (int32_t *)(gb + slots * 8);
            int32_t *dsw = (int32_t *)(gb + ((slots * 12 + 15) & ~(size_t)15));
            MN_HIP_TRY(hipMemcpyAsync(div, iv.data(), slots * 8, hipMemcpyHostToDevice, s));
            MN_HIP_TRY(hipMemcpyAsync(dic, ic.data(), slots * 4, hipMemcpyHostToDevice, s));
            MN_HIP_TRY(hipMemcpyAsync(dsw, sw3.data(), sw3.size() * 4, hipMemcpyHostToDevice, s));
            const int nw2 = (int)std::min<size_t>(8, (LDS_BUDGET - lb2) / pw2);
            const size_t sh2 = lb2 + (size_t)nw2 * pw2;
            const int64_t blocks2 = std::min<int64_t>((n + nw2 - 1) / nw2, 2048);
            auto kf = x_is_f64 ? k_diffuse_rows3<true, 2, 1> : k_diffuse_rows3<false, 2, 1>;
#define MN_DFK(G, T) \
    if (DF_G == G && DF_T == T) kf = x_is_f64 ? k_diffuse_rows3<true, G, T> : k_diffuse_rows3<false, G, T>
            MN_DFK(1, 2); MN_DFK(1, 4); MN_DFK(2, 2); MN_DFK(2, 4); MN_DFK(4, 1); MN_DFK(4, 2);
#undef MN_DFK
            MN_HIP_TRY(hipFuncSetAttribute((const void *)kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)sh2));
            hipLaunchKernelGGL(kf, dim3((unsigned)blocks2), dim3(64 * nw2), sh2, s, X, n, f, div, dic,
                               (int64_t)slots, dsw, perm, eta, steps, matvec, out);
            MN_KCHECK(s, "k_diffuse_rows3");
            MN_HIP_TRY(hipStreamSynchronize(s));
            return MN_OK;
        }
        if (f <= 64 * DF_SW && lb2 + pw2 <= LDS_BUDGET && S * 64 < INT_MAX && !(dfe && *dfe == '1')) {
            std::vector<int32_t> hix((size_t)nnz);
            std::vector<double> hv((size_t)nnz);
            if (nnz > 0) {
                MN_HIP_TRY(hipMemcpyAsync(hix.data(), L->indices, 4 * (size_t)nnz, hipMemcpyDeviceToHost, s));
                MN_HIP_TRY(hipMemcpyAsync(hv.data(), L->values, 8 * (size_t)nnz, hipMemcpyDeviceToHost, s));
                MN_HIP_TRY(hipStreamSynchronize(s));
            }
            const size_t slots = (size_t)S * 64;
            std::vector<double> iv(slots, 0.0);
            std::vector<int32_t> ic(slots, f);  // pads: the zero slot
            for (int g = 0; g < nsw; ++g)
                for (int l = 0; l < 64 && 64 * g + l < f; ++l) {
                    const int i = hperm[64 * g + l];
                    const int G = g / DF_G, u = g % DF_G;
                    for (int64_t p = hip_[i]; p < hip_[i + 1]; ++p) {
                        const size_t q = ((size_t)(sw[2 * G] + (p - hip_[i])) * DF_G + u) * 64 + l;
                        const int c = hix[p];
                        MN_REQUIRE(c >= 0 && c < f, MN_EINVAL, "mn_diffuse_rows: column index out of range");
                        iv[q] = hv[p];
                        ic[q] = c;
                    }
                }
            char *gb = (char *)scratch(kSlotGeneric3, slots * 12 + sw.size() * 4 + 256);
            MN_REQUIRE(gb, MN_ENOMEM, "mn_diffuse_rows: scratch allocation failed");
            double *div = (double *)gb;
            int32_t *dic = (int32_t *)(gb + slots * 8);
            int32_t *dsw = (int32_t *)(gb + ((slots * 12 + 15) & ~(size_t)15));
            MN_HIP_TRY(hipMemcpyAsync(div, iv.data(), slots * 8, hipMemcpyHostToDevice, s));
            MN_HIP_TRY(hipMemcpyAsync(dic, ic.data(), slots * 4, hipMemcpyHostToDevice, s));
            MN_HIP_TRY(hipMemcpyAsync(dsw, sw.data(), sw.size() * 4, hipMemcpyHostToDevice, s));
            const int nw2 = (int)std::min<size_t>(8, (LDS_BUDGET - lb2) / pw2);
            const size_t sh2 = lb2 + (size_t)nw2 * pw2;
            const int64_t blocks2 = std::min<int64_t>((n + nw2 - 1) / nw2, 2048);
            auto kf = x_is_f64 ? k_diffuse_rows2<true, 2, 1> : k_diffuse_rows2<false, 2, 1>;
#define MN_DFK(G, T) \
    if (DF_G == G && DF_T == T) kf = x_is_f64 ? k_diffuse_rows2<true, G, T> : k_diffuse_rows2<false, G, T>
            MN_DFK(1, 1); MN_DFK(1, 2); MN_DFK(1, 4); MN_DFK(2, 2); MN_DFK(2, 4);
            MN_DFK(4, 1); MN_DFK(4, 2); MN_DFK(4, 4);
#undef MN_DFK
            MN_HIP_TRY(hipFuncSetAttribute((const void *)kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)sh2));
            hipLaunchKernelGGL(kf, dim3((unsigned)blocks2), dim3(64 * nw2), sh2, s, X, n, f, div, dic,
                               (int64_t)slots, dsw, perm, eta, steps, matvec, out);
            MN_KCHECK(s, "k_diffuse_rows2");
            MN_HIP_TRY(hipStreamSynchronize(s));
            return MN_OK;
        }
    }
    const size_t lbytes = ((size_t)nnz * 12 + (size_t)(2 * f + 1) * 4 + 15) & ~(size_t)15;
    const size_t per_wave = (size_t)2 * f * 8;
    const int l_in_lds = lbytes + per_wave <= LDS_BUDGET ? 1 : 0;
    const size_t avail = LDS_BUDGET - (l_in_lds ? lbytes : 0);
    const int nw = (int)std::min<size_t>(8, avail / per_wave);
    MN_REQUIRE(nw >= 1, MN_ENOTSUP, "mn_diffuse_rows: f=%d too large for the LDS plan", f);
    const size_t shmem = (l_in_lds ? lbytes : 0) + (size_t)nw * per_wave;
    const int64_t blocks = std::min<int64_t>((n + nw - 1) / nw, 2048);
    if (x_is_f64) {
        MN_HIP_TRY(hipFuncSetAttribute((const void *)k_diffuse_rows<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
        hipLaunchKernelGGL(k_diffuse_rows<true>, dim3((unsigned)blocks), dim3(64 * nw), shmem, s,
                           X, n, f, L->indptr, L->indices, (const double *)L->values, nnz, l_in_lds,
                           perm, eta, steps, matvec, out);
    } else {
        MN_HIP_TRY(hipFuncSetAttribute((const void *)k_diffuse_rows<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
        hipLaunchKernelGGL(k_diffuse_rows<false>, dim3((unsigned)blocks), dim3(64 * nw), shmem, s,
                           X, n, f, L->indptr, L->indices, (const double *)L->values, nnz, l_in_lds,
                           perm, eta, steps, matvec, out);
    }
    MN_KCHECK(s, "k_diffuse_rows");
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

}  // namespace mn

extern "C" {

int mn_diffuse_rows(const mn_csr *L, const void *X, int32_t x_is_f64, int64_t n, int32_t f,
                    double eta, int32_t steps, double *X_out, void *stream) {
    return mn::diffuse_impl(L, X, x_is_f64, n, f, eta, steps, 0, X_out, stream);
}

int mn_energy_signals(const mn_csr *L, const float *X, int64_t n, int32_t f, int32_t g_mode,
                      double *E, double *G, void *stream) {
    return mn::energy_signals_impl(L, X, n, f, g_mode, E, G, stream);
}

int mn_laplacian_matvec_rows(const mn_csr *L, const void *X, int32_t x_is_f64, int64_t n,
                             int32_t f, double *Y, void *stream) {
    return mn::diffuse_impl(L, X, x_is_f64, n, f, 0.0, 1, 1, Y, stream);
}

int mn_energy_rows(const mn_csr *L, const float *X, int64_t n, int32_t f,
                   const mn_energy_opts *opts, double *E, double *G, double *lambda) {
    return mn::energy_impl(L, X, n, f, opts, E, G, lambda);
}

int mn_normalise_lambdas(double *lambda, int64_t n, double *out_min_max_range_host,
                         void *stream) {
    mn::clear_error();
    MN_REQUIRE(lambda || n == 0, MN_EINVAL, "mn_normalise_lambdas: NULL lambda");
    hipStream_t s = (hipStream_t)stream;
    unsigned long long *mm = (unsigned long long *)mn::scratch(mn::kSlotFlags, 64);
    MN_REQUIRE(mm, MN_ENOMEM, "mn_normalise_lambdas: scratch allocation failed");
    double *o3 = (double *)(mm + 2);
    unsigned long long init[2] = {~0ull, 0ull};
    MN_HIP_TRY(hipMemcpyAsync(mm, init, 16, hipMemcpyHostToDevice, s));
    if (n > 0) {
        const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
        hipLaunchKernelGGL(mn::energy::k_minmax, dim3((unsigned)blocks), dim3(256), 0, s, lambda, n,
                           mm);
    }
    hipLaunchKernelGGL(mn::energy::k_normalise, dim3((unsigned)std::max<int64_t>(1, (n + 255) / 256)),
                       dim3(256), 0, s, lambda, n, mm, o3);
    MN_HIP_TRY(hipGetLastError());
    if (out_min_max_range_host)
        MN_HIP_TRY(hipMemcpyAsync(out_min_max_range_host, o3, 24, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

int mn_energy_last_stats(mn_energy_stats *out) {
    if (!out) return MN_EINVAL;
    *out = mn::t_energy_stats;
    return MN_OK;
}

}  // extern "C"
