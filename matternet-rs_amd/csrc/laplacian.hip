// laplacian.hip — K2: kNN rows -> symmetric weighted graph -> Laplacian (CSR).
//
// Reference semantics:
//   UNION / unnormalised (legacy, f64) — src_legacy/laplacian.rs:245-294
//     (weight 1/(1+(dist/sigma)^p) for dist <= eps, kept if > 1e-12),
//     :297-348 (_symmetrise_adjancency: every directed edge also inserted
//     reversed, self loops dropped, rows sorted by column), :351-419
//     (_build_sparse_laplacian: L_ii = sum_j w_ij summed sequentially in
//     ascending j from -0.0 and stored for EVERY row, L_ij = -w_ij).
//   MAX / Stage C (f32) — surfface-core/src/laplacian.rs:312-394 (undirected
//     key with the max weight, w <= thr dropped, degrees in f32, optional
//     L_sym = I - D^-1/2 W D^-1/2) and :209-219 (dense -> CSR keeps |v|>1e-9).
//
// GPU design: an O(E) counting-sort CSR build, no global sort, every pass
// coalesced (one thread per kNN slot, one wave per graph row):
//   1. k_lap_slots      per slot: weight kernel + validity, in-degree atomics
//   2. scan             row segment = k forward slots + in-degree reverse slots
//   3. k_lap_scatter    forward slot r -> segment position r (an invalid slot
//                       holds a sentinel column), reverse entries by atomic
//                       fill (their order is fixed by step 4); the weight is
//                       recomputed rather than staged through HBM
//   4. row sort+dedupe  (col asc, w desc), a unique col keeps the max weight;
//                       one wave per row (<= 512 entries, bitonic in
//                       registers, sized 64/128/256/512 per row) fused with the
//                       row's degree: a sequential ascending-column fold (the
//                       reference's order on the legacy path) over the kept
//                       entries, lane values read in order by v_readlane; one
//                       1024-thread block per row <= 8192 (bitonic in LDS); hub
//                       rows: a block-wide bitonic network in HBM + LDS chunks
//                       (no host round trip: nnz is the call's one read-back)
//   5. (MAX) kept count per row (needs every degree), one wave per row
//   6. scan + CSR write, one wave per row, diagonal at its sorted position.
#include <algorithm>
#include <climits>
#include <vector>

#include "common.hpp"
#include "glibc_f64.hpp"
#include "scan.hpp"

namespace mn {
namespace lap {

struct Params {
    int kernel;     // MN_W_GIVEN / MN_W_RATIONAL
    int sym;        // MN_SYM_UNION / MN_SYM_MAX
    int normalize;  // MAX only
    double eps, sigma, p, thr;
};

constexpr int WAVE_CAP = 512;   // general (col, w) wave sort
constexpr int BLOCK_CAP = 16384;  // rows sorted in one block's LDS (packed 8-B keys)
constexpr int EMPTY = INT_MAX;  // sentinel column of an invalid forward slot
constexpr uint64_t SENT = ~0ull;  // sentinel packed key (column << 32 | entry)

// (d / sigma)^p as the reference's f64::powf = glibc pow (glibc_f64.hpp),
// for every p (pow(x, 2) need not round like x * x)
__device__ __forceinline__ double pw(double x, double p) { return glibc::pow_glibc(x, p); }

// Slot s = i*k + r of the kNN rows: neighbour j and edge weight w; false if
// the slot carries no edge (empty, self loop, filtered).  laplacian.rs:245-260
// (rational kernel), surfface-core/src/laplacian.rs:324 (MAX threshold).
__device__ __forceinline__ bool slot_edge(const int32_t *__restrict__ nbr,
                                          const void *__restrict__ val, int val_f64, int64_t n,
                                          int64_t i, int64_t s, const Params &P, int32_t &j,
                                          double &w, bool &bad) {
    j = nbr[s];
    const double x = val_f64 ? ((const double *)val)[s] : (double)((const float *)val)[s];
    bad = j >= n;
    bool valid = j >= 0 && (int64_t)j != i && !bad;
    w = x;
    if (valid && P.kernel == MN_W_RATIONAL) {
        valid = x <= P.eps;  // laplacian.rs:252 (NaN fails)
        w = 1.0 / (1.0 + pw(x / P.sigma, P.p));
        valid = valid && (w > 1e-12);
    }
    if (valid && P.sym == MN_SYM_MAX) valid = w > P.thr;
    return valid;
}

__global__ __launch_bounds__(256) void k_lap_slots(const int32_t *__restrict__ nbr,
                                                   const void *__restrict__ val, int val_f64,
                                                   int64_t n, int k, Params P,
                                                   int32_t *__restrict__ indeg,
                                                   int *__restrict__ bad) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n * k) return;
    int32_t j;
    double w;
    bool b;
    if (slot_edge(nbr, val, val_f64, n, s / k, s, P, j, w, b)) atomicAdd(&indeg[j], 1);
    if (b) atomicOr(bad, 1);
}

__global__ void k_seg_len(const int32_t *__restrict__ indeg, int64_t n, int k,
                          int32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = k + indeg[i];
}

__global__ __launch_bounds__(256) void k_lap_scatter(const int32_t *__restrict__ nbr,
                                                     const void *__restrict__ val, int val_f64,
                                                     int64_t n, int k, Params P,
                                                     const int64_t *__restrict__ offs,
                                                     int32_t *__restrict__ fill,
                                                     int32_t *__restrict__ col,
                                                     double *__restrict__ wt) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n * k) return;
    const int64_t i = s / k;
    const int r = (int)(s - i * k);
    int32_t j;
    double w;
    bool b;
    const bool valid = slot_edge(nbr, val, val_f64, n, i, s, P, j, w, b);
    const int64_t f = offs[i] + r;
    col[f] = valid ? j : EMPTY;
    wt[f] = w;
    if (valid) {
        const int64_t q = offs[j] + k + atomicAdd(&fill[j], 1);
        col[q] = (int32_t)i;
        wt[q] = w;
    }
}

// (col asc, w desc): the first entry of each column run carries the max weight
__device__ __forceinline__ bool cw_less(int ca, double wa, int cb, double wb) {
    return ca < cb || (ca == cb && wa > wb);
}

__device__ __forceinline__ double readlane_f64(double x, int l) {
    const long long u = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xFFFFFFFFll), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Sort, dedupe and fold one row of m <= 64*NR entries held by one wave.
// Source (cs, ws at o) and destination (col, wt at od) may differ: the
// bucket kernel sorts rows staged in LDS into their global segments.
template <int NR>
__device__ __forceinline__ void row_sort_fold(int64_t i, int64_t o, int m, int sym,
                                              const int32_t *cs, const double *ws, int64_t od,
                                              int32_t *__restrict__ col, double *__restrict__ wt,
                                              int32_t *__restrict__ uniq,
                                              int32_t *__restrict__ kept,
                                              double *__restrict__ deg64,
                                              float *__restrict__ deg32) {
    const int lane = threadIdx.x & 63;
    int c[NR];
    double w[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        c[r] = e < m ? cs[o + e] : EMPTY;
        w[r] = e < m ? ws[o + e] : 0.0;
    }
#pragma unroll
    for (int kk = 2; kk <= 64 * NR; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int pr = r ^ (j >> 6);
                    if (pr > r) {
                        const int e = lane + 64 * r;
                        const bool asc = (e & kk) == 0;
                        const bool sw = asc ? cw_less(c[pr], w[pr], c[r], w[r])
                                            : cw_less(c[r], w[r], c[pr], w[pr]);
                        if (sw) {
                            int tc = c[r]; c[r] = c[pr]; c[pr] = tc;
                            double tw = w[r]; w[r] = w[pr]; w[pr] = tw;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int e = lane + 64 * r;
                    const int pc = __shfl_xor(c[r], j);
                    const double pwv = __shfl_xor(w[r], j);
                    const bool asc = (e & kk) == 0;
                    const bool lower = (e & j) == 0;
                    const bool take = (asc == lower) ? cw_less(pc, pwv, c[r], w[r])
                                                     : cw_less(c[r], w[r], pc, pwv);
                    if (take) { c[r] = pc; w[r] = pwv; }
                }
            }
        }
    }
    // dedupe: keep e if it holds a column (not the sentinel) that differs from
    // its predecessor's; kept entries are compacted in place and folded in
    // ascending column order (lane values read one by one: the chain of adds
    // is the reference's sequential sum)
    int base = 0;
    double s64 = -0.0;  // laplacian.rs:367 s.iter().map(w).sum() in ascending j
    float s32 = 0.0f;   // surfface-core/src/laplacian.rs:331-340 (order: ascending column)
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        int prev = __shfl_up(c[r], 1);
        const int last_prev = (r > 0) ? __shfl(c[r > 0 ? r - 1 : 0], 63) : INT_MIN;
        if (lane == 0) prev = (r == 0) ? INT_MIN : last_prev;
        const bool keep = e < m && c[r] != EMPTY && c[r] != prev;
        uint64_t mk = __ballot(keep);
        if (keep) {
            const int pos = base + (int)__popcll(mk & ((1ull << lane) - 1ull));
            col[od + pos] = c[r];
            wt[od + pos] = w[r];
        }
        base += (int)__popcll(mk);
        if (sym == MN_SYM_UNION) {
            while (mk) {
                const int l = __builtin_ctzll(mk);
                mk &= mk - 1;
                s64 = s64 + readlane_f64(w[r], l);
            }
        } else {
            while (mk) {
                const int l = __builtin_ctzll(mk);
                mk &= mk - 1;
                s32 = s32 + (float)readlane_f64(w[r], l);
            }
        }
    }
    if (lane == 0) {
        uniq[i] = base;
        if (sym == MN_SYM_UNION) {
            deg64[i] = s64;
            kept[i] = base + 1;  // + the diagonal, stored for every row
        } else {
            deg32[i] = s32;
        }
    }
}

// one wave per row; rows with more than WAVE_CAP entries are listed for the
// block kernel
// Packed-key row (the default for rows of <= 64 NR entries): sort keys
// (column << 32 | entry index e) in registers — one 64-bit compare per
// exchange, the weights stay where they are — then each column run's first
// entry is kept with the run's largest weight (the (col asc, w desc) order of
// row_sort_fold), gathered through wf(e) for the kept entries and their run
// partners only; then the ascending-column degree fold.  keyf(e), e < m: the
// key of entry e (SENT for an empty slot).  Every gather is issued before the
// first store, so the destination may be the source segment.  Returns false
// (nothing written) for a run of 3 or more equal columns (duplicate ids in one
// kNN row): the caller then runs row_sort_fold.
// FOLD false (the bucket kernel): no degree fold here — the kept weights also
// go to lw[0 .. u) (LDS, ascending column) and *u_out = u, for the bucket's
// lane-per-row fold.
template <int NR, bool FOLD = true, class KeyF, class WF>
__device__ __forceinline__ bool packed_row(KeyF keyf, WF wf, int m, int64_t i, int64_t od, int sym,
                                           int32_t *__restrict__ col, double *__restrict__ wt,
                                           int32_t *__restrict__ uniq, int32_t *__restrict__ kept,
                                           double *__restrict__ deg64,
                                           float *__restrict__ deg32, double *lw = nullptr,
                                           int *u_out = nullptr) {
    const int lane = threadIdx.x & 63;
    uint64_t x[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        x[r] = e < m ? keyf(e) : SENT;
    }
#pragma unroll
    for (int q = 2; q <= 64 * NR; q <<= 1) {
#pragma unroll
        for (int j = q >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int pr = r ^ (j >> 6);
                    if (pr > r) {
                        const bool asc = ((lane + 64 * r) & q) == 0;
                        if (asc ? x[pr] < x[r] : x[r] < x[pr]) {
                            const uint64_t t = x[r]; x[r] = x[pr]; x[pr] = t;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int e = lane + 64 * r;
                    const uint64_t p = (uint64_t)__shfl_xor((long long)x[r], j);
                    const bool asc = (e & q) == 0, lower = (e & j) == 0;
                    if ((asc == lower) ? p < x[r] : x[r] < p) x[r] = p;
                }
            }
        }
    }
    auto colof = [](uint64_t v) { return v == SENT ? EMPTY : (int)(v >> 32); };
    // neighbours in sorted order: previous column, next key, next-but-one column
    bool run3 = false;
    uint64_t xn[NR];
    int cp[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int c = colof(x[r]);
        int up = __shfl_up(c, 1);
        const int prevlast = __shfl(colof(x[r > 0 ? r - 1 : 0]), 63);
        if (lane == 0) up = r == 0 ? INT_MIN : prevlast;
        cp[r] = up;
        uint64_t dn = (uint64_t)__shfl_down((long long)x[r], 1);
        const uint64_t nx0 = (uint64_t)__shfl((long long)x[r + 1 < NR ? r + 1 : r], 0);
        if (lane == 63) dn = r + 1 < NR ? nx0 : SENT;
        xn[r] = dn;
        int dn2 = __shfl_down(c, 2);
        const int n0 = colof(nx0), n1 = __shfl(colof(x[r + 1 < NR ? r + 1 : r]), 1);
        if (lane >= 62) dn2 = r + 1 < NR ? (lane == 62 ? n0 : n1) : EMPTY;
        run3 |= c != EMPTY && c == dn2;
    }
    if (__any(run3)) return false;
    double w[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int c = colof(x[r]);
        const bool keep = c != EMPTY && c != cp[r];
        w[r] = 0.0;
        if (keep) {
            w[r] = wf((uint32_t)x[r]);
            if (colof(xn[r]) == c) {
                const double wp = wf((uint32_t)xn[r]);
                if (wp > w[r]) w[r] = wp;
            }
        }
    }
    int base = 0;
    double s64 = -0.0;  // laplacian.rs:367 s.iter().map(w).sum() in ascending j
    float s32 = 0.0f;   // surfface-core/src/laplacian.rs:331-340 (order: ascending column)
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int c = colof(x[r]);
        const bool keep = c != EMPTY && c != cp[r];
        uint64_t mk = __ballot(keep);
        if (keep) {
            const int pos = base + (int)__popcll(mk & ((1ull << lane) - 1ull));
            col[od + pos] = c;
            wt[od + pos] = w[r];
            if constexpr (!FOLD) lw[pos] = w[r];
        }
        base += (int)__popcll(mk);
        if constexpr (FOLD) {
            if (sym == MN_SYM_UNION) {
                while (mk) {
                    const int l = __builtin_ctzll(mk);
                    mk &= mk - 1;
                    s64 = s64 + readlane_f64(w[r], l);
                }
            } else {
                while (mk) {
                    const int l = __builtin_ctzll(mk);
                    mk &= mk - 1;
                    s32 = s32 + (float)readlane_f64(w[r], l);
                }
            }
        }
    }
    if constexpr (!FOLD) {
        *u_out = base;
        return true;
    }
    if (lane == 0) {
        uniq[i] = base;
        if (sym == MN_SYM_UNION) {
            deg64[i] = s64;
            kept[i] = base + 1;
        } else {
            deg32[i] = s32;
        }
    }
    return true;
}

// 1: done; 0: a run of >= 3 equal columns (general path); -1: too long
template <int NRMAX, class KeyF, class WF, typename... A>
__device__ __forceinline__ int packed_row_any(KeyF keyf, WF wf, int m, A... a) {
    if (m <= 64) return packed_row<1>(keyf, wf, m, a...) ? 1 : 0;
    if (m <= 128) return packed_row<2>(keyf, wf, m, a...) ? 1 : 0;
    if (m <= 256) return packed_row<4>(keyf, wf, m, a...) ? 1 : 0;
    if constexpr (NRMAX >= 8)
        if (m <= 512) return packed_row<8>(keyf, wf, m, a...) ? 1 : 0;
    if constexpr (NRMAX >= 16)
        if (m <= 1024) return packed_row<16>(keyf, wf, m, a...) ? 1 : 0;
    return -1;
}

// 32-bit keys (column << 8 | the entry's index in its row) for rows of <= 256
// entries when every column < 2^24 - 1: one shuffle and one 32-bit compare
// per exchange instead of two and a 64-bit one.  The bucket kernel's form
// (no fold: the kept weights to lw[0 .. u), *u_out = u); keyf(e) the key of
// entry e (SENT32 for an empty slot), wf(e) its weight.  false: a run of >= 3
// equal columns (the caller's general path).
constexpr uint32_t SENT32 = ~0u;
template <int NR, class KeyF, class WF>
__device__ __forceinline__ bool packed_row32(KeyF keyf, WF wf, int m, int64_t od,
                                             int32_t *__restrict__ col, double *__restrict__ wt,
                                             double *lw, int *u_out) {
    const int lane = threadIdx.x & 63;
    uint32_t x[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        x[r] = e < m ? keyf(e) : SENT32;
    }
#pragma unroll
    for (int q = 2; q <= 64 * NR; q <<= 1) {
#pragma unroll
        for (int j = q >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int pr = r ^ (j >> 6);
                    if (pr > r) {
                        const bool asc = ((lane + 64 * r) & q) == 0;
                        if (asc ? x[pr] < x[r] : x[r] < x[pr]) {
                            const uint32_t t = x[r]; x[r] = x[pr]; x[pr] = t;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int e = lane + 64 * r;
                    const uint32_t p = (uint32_t)__shfl_xor((int)x[r], j);
                    const bool asc = (e & q) == 0, lower = (e & j) == 0;
                    if ((asc == lower) ? p < x[r] : x[r] < p) x[r] = p;
                }
            }
        }
    }
    auto colof = [](uint32_t v) { return v == SENT32 ? EMPTY : (int)(v >> 8); };
    bool run3 = false;
    uint32_t xn[NR];
    int cp[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int c = colof(x[r]);
        int up = __shfl_up(c, 1);
        const int prevlast = __shfl(colof(x[r > 0 ? r - 1 : 0]), 63);
        if (lane == 0) up = r == 0 ? INT_MIN : prevlast;
        cp[r] = up;
        uint32_t dn = (uint32_t)__shfl_down((int)x[r], 1);
        const uint32_t nx0 = (uint32_t)__shfl((int)x[r + 1 < NR ? r + 1 : r], 0);
        if (lane == 63) dn = r + 1 < NR ? nx0 : SENT32;
        xn[r] = dn;
        int dn2 = __shfl_down(c, 2);
        const int n0 = colof(nx0), n1 = __shfl(colof(x[r + 1 < NR ? r + 1 : r]), 1);
        if (lane >= 62) dn2 = r + 1 < NR ? (lane == 62 ? n0 : n1) : EMPTY;
        run3 |= c != EMPTY && c == dn2;
    }
    if (__any(run3)) return false;
    double w[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int c = colof(x[r]);
        const bool keep = c != EMPTY && c != cp[r];
        w[r] = 0.0;
        if (keep) {
            w[r] = wf((int)(x[r] & 255u));
            if (colof(xn[r]) == c) {
                const double wp = wf((int)(xn[r] & 255u));
                if (wp > w[r]) w[r] = wp;
            }
        }
    }
    int base = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int c = colof(x[r]);
        const bool keep = c != EMPTY && c != cp[r];
        const uint64_t mk = __ballot(keep);
        if (keep) {
            const int pos = base + (int)__popcll(mk & ((1ull << lane) - 1ull));
            col[od + pos] = c;
            wt[od + pos] = w[r];
            lw[pos] = w[r];
        }
        base += (int)__popcll(mk);
    }
    *u_out = base;
    return true;
}

// the bucket kernel's form: no fold (FOLD false), *u_out = kept entries
template <class KeyF, class WF, typename... A>
__device__ __forceinline__ int packed_row_nofold(KeyF keyf, WF wf, int m, A... a) {
    if (m <= 64) return packed_row<1, false>(keyf, wf, m, a...) ? 1 : 0;
    if (m <= 128) return packed_row<2, false>(keyf, wf, m, a...) ? 1 : 0;
    if (m <= 256) return packed_row<4, false>(keyf, wf, m, a...) ? 1 : 0;
    return -1;
}

template <typename... A>
__device__ __forceinline__ bool row_sort_fold_any(int64_t i, int64_t o, int m, int sym,
                                                  const int32_t *cs, const double *ws, int64_t od,
                                                  A... a) {
    if (m <= 64) row_sort_fold<1>(i, o, m, sym, cs, ws, od, a...);
    else if (m <= 128) row_sort_fold<2>(i, o, m, sym, cs, ws, od, a...);
    else if (m <= 256) row_sort_fold<4>(i, o, m, sym, cs, ws, od, a...);
    else if (m <= WAVE_CAP) row_sort_fold<8>(i, o, m, sym, cs, ws, od, a...);
    else return false;
    return true;
}

// list == NULL: row i = the wave's index; else rows list[0 .. *list_n).
// NRMAX 4 (the full pass / the bucket kernel's leftovers): rows of <= 256
// entries, longer ones (and rows with duplicate ids) to next_list; NRMAX 16
// (that list): rows of <= 1024 entries (duplicate ids: the general (col, w)
// sort up to WAVE_CAP), longer ones to next_list (the block kernel).
template <int NRMAX>
__global__ __launch_bounds__(256) void k_row_sort_wave(const int64_t *__restrict__ offs,
                                                       int64_t n, int sym,
                                                       int32_t *__restrict__ col,
                                                       double *__restrict__ wt,
                                                       int32_t *__restrict__ uniq,
                                                       int32_t *__restrict__ kept,
                                                       double *__restrict__ deg64,
                                                       float *__restrict__ deg32,
                                                       int32_t *__restrict__ next_list,
                                                       int *__restrict__ next_count,
                                                       const int32_t *__restrict__ list,
                                                       const int *__restrict__ list_n) {
    const int lane = threadIdx.x & 63;
    const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nrows = list ? (int64_t)*list_n : n;
    for (int64_t x = wv; x < nrows; x += nw) {
        const int64_t i = list ? (int64_t)list[x] : x;
        const int64_t o = offs[i];
        const int m = (int)(offs[i + 1] - o);
        auto keyf = [&](int e) {
            const int c = col[o + e];
            return c == EMPTY ? SENT : (((uint64_t)(uint32_t)c << 32) | (uint32_t)e);
        };
        auto wf = [&](uint32_t e) { return wt[o + e]; };
        const int rc = packed_row_any<NRMAX>(keyf, wf, m, i, o, sym, col, wt, uniq, kept, deg64,
                                             deg32);
        if (rc == 1) continue;
        if constexpr (NRMAX >= 16) {
            if (rc == 0 && row_sort_fold_any(i, o, m, sym, col, wt, o, col, wt, uniq, kept, deg64,
                                             deg32))
                continue;
        }
        if (lane == 0) next_list[atomicAdd(next_count, 1)] = (int32_t)i;
    }
}

// one 1024-thread block per row of 1024 < m <= BLOCK_CAP entries (the rows
// the wave kernels pass on): packed (column << 32 | entry) keys bitonic-sorted
// in LDS, weights gathered only for the kept entries (the first of each
// column run takes the run's largest weight, as (col asc, w desc) would),
// every gather before the first store (the row is compacted in place), then
// the kept weights in LDS for wave 0's ascending-column fold.
struct alignas(16) BigSmem {
    uint64_t key[BLOCK_CAP];  // reused as the kept weights (double) for the fold
    int wsum[16];
};

__global__ __launch_bounds__(1024) void k_row_sort_block(const int64_t *__restrict__ offs,
                                                         const int32_t *__restrict__ big_list,
                                                         const int *__restrict__ big_count,
                                                         int sym, int32_t *__restrict__ col,
                                                         double *__restrict__ wt,
                                                         int32_t *__restrict__ uniq,
                                                         int32_t *__restrict__ kept,
                                                         double *__restrict__ deg64,
                                                         float *__restrict__ deg32,
                                                         int32_t *__restrict__ huge_list,
                                                         int *__restrict__ huge_count) {
    constexpr int NQ = BLOCK_CAP / 1024;  // elements per thread
    __shared__ BigSmem sm;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int nb = *big_count;
    auto colof = [](uint64_t v) { return v == SENT ? EMPTY : (int)(v >> 32); };
    for (int b = blockIdx.x; b < nb; b += gridDim.x) {
        const int64_t i = big_list[b];
        const int64_t o = offs[i];
        const int m = (int)(offs[i + 1] - o);
        if (m > BLOCK_CAP) {
            if (t == 0) huge_list[atomicAdd(huge_count, 1)] = (int32_t)i;
            continue;
        }
        int P = 1;
        while (P < m) P <<= 1;
        for (int e = t; e < P; e += 1024) {
            const int c = e < m ? col[o + e] : EMPTY;
            sm.key[e] = c == EMPTY ? SENT : (((uint64_t)(uint32_t)c << 32) | (uint32_t)e);
        }
        __syncthreads();
        for (int kk = 2; kk <= P; kk <<= 1)
            for (int j = kk >> 1; j > 0; j >>= 1) {
                for (int e = t; e < P; e += 1024) {
                    const int pe = e ^ j;
                    if (pe > e) {
                        const uint64_t a = sm.key[e], c = sm.key[pe];
                        if (((e & kk) == 0) ? c < a : a < c) {
                            sm.key[e] = c;
                            sm.key[pe] = a;
                        }
                    }
                }
                __syncthreads();
            }
        // dedupe: element e = 1024 q + t; kept entries' weights in registers,
        // their positions from a block scan per chunk
        int pr[NQ];
        double wr[NQ];
        int base = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = 1024 * q + t;
            pr[q] = -1;
            wr[q] = 0.0;
            if (1024 * q >= m) continue;  // block-uniform
            const uint64_t x = e < m ? sm.key[e] : SENT;
            const int c = colof(x);
            const int cprev = (e > 0 && e < m) ? colof(sm.key[e - 1]) : INT_MIN;
            const bool keep = e < m && c != EMPTY && c != cprev;
            if (keep) {
                double w = wt[o + (uint32_t)x];
                for (int f = e + 1; f < m; ++f) {  // the column run (2 long at most in practice)
                    const uint64_t y = sm.key[f];
                    if (colof(y) != c) break;
                    const double wp = wt[o + (uint32_t)y];
                    if (wp > w) w = wp;
                }
                wr[q] = w;
            }
            const uint64_t mk = __ballot(keep);
            if (lane == 0) sm.wsum[wv] = (int)__popcll(mk);
            __syncthreads();
            int before = 0, tot = 0;
            for (int z = 0; z < 16; ++z) {
                if (z < wv) before += sm.wsum[z];
                tot += sm.wsum[z];
            }
            if (keep) pr[q] = base + before + (int)__popcll(mk & ((1ull << lane) - 1ull));
            base += tot;
            __syncthreads();
        }
        // every gather from wt happened above: compact the row in place (the
        // columns re-read from the keys), then stage the kept weights for the
        // fold over the dead keys
#pragma unroll
        for (int q = 0; q < NQ; ++q)
            if (pr[q] >= 0) {
                col[o + pr[q]] = colof(sm.key[1024 * q + t]);
                wt[o + pr[q]] = wr[q];
            }
        __syncthreads();
        double *kw = reinterpret_cast<double *>(sm.key);
#pragma unroll
        for (int q = 0; q < NQ; ++q)
            if (pr[q] >= 0) kw[pr[q]] = wr[q];
        __syncthreads();
        if (t < 64) {  // ascending-column fold: 64 weights a step, chained via v_readlane
            double s64 = -0.0;
            float s32 = 0.0f;
            for (int c0 = 0; c0 < base; c0 += 64) {
                const double v = c0 + lane < base ? kw[c0 + lane] : 0.0;
                const int cnt = min(64, base - c0);
                if (sym == MN_SYM_UNION)
                    for (int l = 0; l < cnt; ++l) s64 = s64 + readlane_f64(v, l);
                else
                    for (int l = 0; l < cnt; ++l) s32 = s32 + (float)readlane_f64(v, l);
            }
            if (lane == 0) {
                uniq[i] = base;
                if (sym == MN_SYM_UNION) {
                    deg64[i] = s64;
                    kept[i] = base + 1;
                } else {
                    deg32[i] = s32;
                }
            }
        }
        __syncthreads();
    }
}

// hub rows (m > BLOCK_CAP): one 1024-thread block per row, sorted in place in
// HBM by a bitonic network that keeps every sequence ascending (the first
// step of each merge compares e with e ^ (kk - 1)), so positions >= m act as
// +inf and are never touched; every step with partner distance < CH runs on
// LDS-resident chunks of CH entries.  Between steps that exchange data through
// HBM the block waits for its stores and invalidates its L1 (agent acquire).
constexpr int CH = 8192;  // hub rows: LDS chunk of the HBM bitonic network

__device__ __forceinline__ void hub_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// the kept entries' count and degree: one wave, coalesced 64-entry chunks;
// the ascending-column fold reads the lanes in order
__device__ __forceinline__ void hub_fold(int64_t i, int64_t o, int u, int sym,
                                         const double *__restrict__ wt, double (&cb)[2][64],
                                         int32_t *__restrict__ uniq, int32_t *__restrict__ kept,
                                         double *__restrict__ deg64, float *__restrict__ deg32) {
    constexpr int PF = 8;  // 64-entry chunks in flight ahead of the fold
    const int lane = threadIdx.x & 63;
    const int nch = (u + 63) / 64;
    double ring[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) ring[q] = (64 * q + lane < u) ? wt[o + 64 * q + lane] : 0.0;
    double s64 = -0.0;
    float s32 = 0.0f;
    for (int c0 = 0; c0 < nch; c0 += PF) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int c = c0 + q;
            if (c >= nch) break;
            const double w = ring[q];
            const int nx = 64 * (c + PF) + lane;
            ring[q] = nx < u ? wt[o + nx] : 0.0;
            const int m = min(64, u - 64 * c);
            if (sym == MN_SYM_UNION && m == 64) {  // full chunk: LDS broadcast chain
                cb[c & 1][lane] = w;
                __builtin_amdgcn_wave_barrier();
                s64 = lds_chain_f64<64>(s64, cb[c & 1]);
                __builtin_amdgcn_wave_barrier();
            } else {
                for (int l = 0; l < m; ++l) {
                    const double v = readlane_f64(w, l);
                    if (sym == MN_SYM_UNION) s64 = s64 + v;
                    else s32 = s32 + (float)v;
                }
            }
        }
    }
    if (lane == 0) {
        uniq[i] = u;
        if (sym == MN_SYM_UNION) {
            deg64[i] = s64;
            kept[i] = u + 1;
        } else {
            deg32[i] = s32;
        }
    }
}

struct alignas(16) HubSmem {
    double w[CH];
    int c[CH];
    int wsum[16];
    int carry;
    double cb[2][64];
};

__global__ __launch_bounds__(1024) void k_row_sort_hub(const int64_t *__restrict__ offs,
                                                       const int32_t *__restrict__ huge_list,
                                                       const int *__restrict__ huge_count,
                                                       int sym, int32_t *__restrict__ col,
                                                       double *__restrict__ wt,
                                                       int32_t *__restrict__ uniq,
                                                       int32_t *__restrict__ kept,
                                                       double *__restrict__ deg64,
                                                       float *__restrict__ deg32) {
    __shared__ HubSmem sm;
    const int t = threadIdx.x;
    const int nh = *huge_count;
    for (int h = blockIdx.x; h < nh; h += gridDim.x) {
        const int64_t i = huge_list[h];
        const int64_t o = offs[i];
        const int m = (int)(offs[i + 1] - o);
        int32_t *C = col + o;
        double *W = wt + o;
        int P = CH;
        while (P < m) P <<= 1;
        // one chunk through LDS: steps kk (or the half-cleaners below jmax when
        // full == false) of the network
        auto chunk_pass = [&](int base, bool full, int jmax) {
            for (int e = t; e < CH; e += blockDim.x) {
                const int g = base + e;
                sm.c[e] = g < m ? C[g] : EMPTY;
                sm.w[e] = g < m ? W[g] : 0.0;
            }
            __syncthreads();
            for (int kk = full ? 2 : 2 * CH; kk <= (full ? CH : 2 * CH); kk <<= 1) {
                const int j0 = full ? kk >> 1 : jmax;
                for (int j = j0; j > 0; j >>= 1) {
                    const bool flip = full && j == (kk >> 1);
                    for (int q = t; q < CH / 2; q += blockDim.x) {
                        const int e = ((q & ~(j - 1)) << 1) | (q & (j - 1));  // bit j clear
                        const int pe = flip ? (e ^ (2 * j - 1)) : (e | j);
                        if (base + pe < m && cw_less(sm.c[pe], sm.w[pe], sm.c[e], sm.w[e])) {
                            int tc = sm.c[e]; sm.c[e] = sm.c[pe]; sm.c[pe] = tc;
                            double tw = sm.w[e]; sm.w[e] = sm.w[pe]; sm.w[pe] = tw;
                        }
                    }
                    __syncthreads();
                }
            }
            for (int e = t; e < CH; e += blockDim.x) {
                const int g = base + e;
                if (g < m) {
                    C[g] = sm.c[e];
                    W[g] = sm.w[e];
                }
            }
        };
        for (int base = 0; base < m; base += CH) {  // sorted CH-runs
            chunk_pass(base, true, 0);
            __syncthreads();
        }
        hub_sync();
        for (int kk = 2 * CH; kk <= P; kk <<= 1) {
            for (int j = kk >> 1; j >= CH; j >>= 1) {  // steps across chunks, in HBM
                const bool flip = j == (kk >> 1);
                for (int q = t; q < P / 2; q += blockDim.x) {
                    const int e = ((q & ~(j - 1)) << 1) | (q & (j - 1));
                    const int pe = flip ? (e ^ (2 * j - 1)) : (e | j);
                    if (pe < m) {
                        const int ce = C[e], cp = C[pe];
                        const double we = W[e], wp = W[pe];
                        if (cw_less(cp, wp, ce, we)) {
                            C[e] = cp; W[e] = wp;
                            C[pe] = ce; W[pe] = we;
                        }
                    }
                }
                hub_sync();
            }
            for (int base = 0; base < m; base += CH) {  // the remaining steps per chunk
                chunk_pass(base, false, CH >> 1);
                __syncthreads();
            }
            hub_sync();
        }
        // dedupe (the first of each column run carries the max weight) and
        // compact in place: every chunk is read before any of it is written,
        // and a write lands at or before its source
        int nk = 0;
        if (t == 0) sm.carry = INT_MIN;
        __syncthreads();
        for (int c0 = 0; c0 < m; c0 += 1024) {
            const int e = c0 + t;
            const int ce = e < m ? C[e] : EMPTY;
            const double we = e < m ? W[e] : 0.0;
            const int prev = t == 0 ? sm.carry : (e - 1 < m ? C[e - 1] : EMPTY);
            const bool keep = e < m && ce != EMPTY && ce != prev;
            const uint64_t mk = __ballot(keep);
            const int lane = t & 63, wv = t >> 6;
            if (lane == 0) sm.wsum[wv] = (int)__popcll(mk);
            __syncthreads();
            int before = 0, tot = 0;
            for (int q = 0; q < 16; ++q) {
                if (q < wv) before += sm.wsum[q];
                tot += sm.wsum[q];
            }
            if (t == 1023) sm.carry = ce;
            hub_sync();  // every load of this chunk precedes its writes
            if (keep) {
                const int pos = nk + before + (int)__popcll(mk & ((1ull << lane) - 1ull));
                C[pos] = ce;
                W[pos] = we;
            }
            nk += tot;
            hub_sync();
        }
        if (t < 64) hub_fold(i, o, nk, sym, wt, sm.cb, uniq, kept, deg64, deg32);
        __syncthreads();
    }
}

// ---- bucketed assembly (default) -------------------------------------------
// The transpose of the kNN rows without global atomics: destination rows are
// grouped in buckets of BR rows; every reverse entry (j <- i) is written once
// into its bucket's contiguous region (runs per (slot block, bucket) placed
// by a 2-D count/scan, ranks inside a slot block from LDS atomics), then one
// block per bucket stages its rows' forward slots + reverse entries in LDS
// (counting sort by row), sorts / dedupes / folds each row there and writes
// the rows' kept entries to their segments.  Rows longer than WAVE_CAP, and
// every row of a bucket that does not fit the LDS stage (hub rows), go to the
// global-memory kernels above.
constexpr int BSH = 6, BR = 1 << BSH;  // rows per bucket
constexpr int ACH = 65536;             // slots per counting block
constexpr int ANT = 1024;
constexpr int NBMAX = 16384;           // buckets (LDS counters of the slot blocks)

__global__ __launch_bounds__(ANT) void k_lap_bhist(const int32_t *__restrict__ nbr,
                                                   const void *__restrict__ val, int val_f64,
                                                   int64_t n, int k, Params P, int NB,
                                                   int32_t *__restrict__ cnt,
                                                   int *__restrict__ bad) {
    __shared__ int h[NBMAX];
    const int b = blockIdx.x, t = threadIdx.x;
    for (int q = t; q < NB; q += ANT) h[q] = 0;
    __syncthreads();
    const int64_t s0 = (int64_t)b * ACH, s1 = min(n * k, s0 + ACH);
    bool anybad = false;
    for (int64_t sl = s0 + t; sl < s1; sl += ANT) {
        int32_t j;
        double w;
        bool bd;
        if (slot_edge(nbr, val, val_f64, n, sl / k, sl, P, j, w, bd)) atomicAdd(&h[j >> BSH], 1);
        anybad |= bd;
    }
    if (anybad) atomicOr(bad, 1);
    __syncthreads();
    for (int q = t; q < NB; q += ANT) cnt[(int64_t)b * NB + q] = h[q];
}

// per bucket: exclusive prefix over the slot blocks (in place) and the
// total; one wave per bucket, 64 slot blocks per step
__global__ __launch_bounds__(256) void k_lap_bscan(int32_t *__restrict__ cnt, int nA, int NB,
                                                   int32_t *__restrict__ tot) {
    const int q = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    if (q >= NB) return;
    int carry = 0;
    for (int b0 = 0; b0 < nA; b0 += 64) {
        const int b = b0 + lane;
        const int v = b < nA ? cnt[(int64_t)b * NB + q] : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (b < nA) cnt[(int64_t)b * NB + q] = carry + x - v;
        carry += __shfl(x, 63);
    }
    if (lane == 0) tot[q] = carry;
}

// reverse entry record: source row, destination row within its bucket, weight
__global__ __launch_bounds__(ANT) void k_lap_bscatter(const int32_t *__restrict__ nbr,
                                                      const void *__restrict__ val, int val_f64,
                                                      int64_t n, int k, Params P, int NB,
                                                      const int32_t *__restrict__ off,
                                                      const int64_t *__restrict__ bstart,
                                                      int4 *__restrict__ rec) {
    __shared__ int pos[NBMAX];
    const int b = blockIdx.x, t = threadIdx.x;
    for (int q = t; q < NB; q += ANT) pos[q] = (int)bstart[q] + off[(int64_t)b * NB + q];
    __syncthreads();
    const int64_t s0 = (int64_t)b * ACH, s1 = min(n * k, s0 + ACH);
    for (int64_t sl = s0 + t; sl < s1; sl += ANT) {
        int32_t j;
        double w;
        bool bd;
        const int64_t i = sl / k;
        if (slot_edge(nbr, val, val_f64, n, i, sl, P, j, w, bd)) {
            const int p = atomicAdd(&pos[j >> BSH], 1);
            const long long wb = __double_as_longlong(w);
            rec[p] = make_int4((int)i, j & (BR - 1), (int)(wb & 0xFFFFFFFFll), (int)(wb >> 32));
        }
    }
}

// Bucket stage: packed sort keys (column << 32 | entry index) — the weights
// stay where they are (forward: recomputed from the slot, reverse: the
// record) and are gathered only for the kept entries, so a bucket is 8 B per
// entry of LDS and two buckets share a CU.  Entry index e < BR k: forward
// slot e of the bucket; else reverse record e0 + e - BR k.
constexpr int BT = 1024;       // threads per bucket block (16 waves, 4 rows each)
constexpr int BKEYS = 8192;    // LDS-staged entries per bucket

// Round 4: the weights sit in LDS beside the keys (key payload = the stage
// position, wt[position]), so a row's sort / dedupe / fold never waits on a
// global gather (round 3 re-read the forward slot or the reverse record per
// kept entry: k_lap_bucket was latency-bound, SQ wait_any 0.55-0.79); 128 KB
// a bucket, one 16-wave block per CU.
struct alignas(16) BucketSmem {
    uint64_t key[BKEYS];
    double w[BKEYS];
    int rlen[BR];
    int roff[BR + 1];
    int rfill[BR];
    int nbig;
    int big[BR];
    int ukept[BR];  // kept entries of a row sorted here (-1: sorted elsewhere)
};

// one block per bucket of BR rows; offs (the rows' segment starts, int64) is
// written here: segment = k forward slots + the reverse entries, bucket
// regions in bucket order.  Kept entries go to the segment starts (the
// layout k_write_csr reads).
__global__ __launch_bounds__(BT) void k_lap_bucket(
    const int32_t *__restrict__ nbr, const void *__restrict__ val, int val_f64, int64_t n, int k,
    Params P, const int64_t *__restrict__ bstart, const int4 *__restrict__ rec,
    int64_t *__restrict__ offs, int32_t *__restrict__ col, double *__restrict__ wt,
    int32_t *__restrict__ uniq, int32_t *__restrict__ kept, double *__restrict__ deg64,
    float *__restrict__ deg32, int32_t *__restrict__ wave_list, int *__restrict__ wave_count,
    int32_t *__restrict__ mid_list, int *__restrict__ mid_count) {
    __shared__ BucketSmem sm;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const bool k32 = n < (1 << 24) - 1;  // 32-bit row keys (column << 8 | entry)
    const int64_t row0 = (int64_t)blockIdx.x * BR;
    const int nr = (int)min((int64_t)BR, n - row0);
    const int64_t e0 = bstart[blockIdx.x], e1 = bstart[blockIdx.x + 1];
    const int64_t gbase = row0 * k + e0;
    if (t < BR) {
        sm.rlen[t] = 0;
        sm.rfill[t] = 0;
    }
    if (t == 0) sm.nbig = 0;
    __syncthreads();
    for (int64_t e = e0 + t; e < e1; e += BT) atomicAdd(&sm.rlen[rec[e].y], 1);
    __syncthreads();
    if (t < 64) {  // exclusive scan of the BR = 64 segment lengths
        const int a = lane < nr ? k + sm.rlen[lane] : 0;
        int x = a;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        sm.roff[lane] = x - a;
        if (lane == 63) sm.roff[BR] = x;
        if (lane < nr) offs[row0 + lane] = gbase + x - a;
        if (lane == 63 && row0 + nr == n) offs[n] = gbase + x;
    }
    __syncthreads();
    const int m = sm.roff[BR];
    const bool staged = m <= BKEYS;
    for (int e = t; e < nr * k; e += BT) {
        const int r = e / k, q = e - r * k;
        const int64_t i = row0 + r, sl = i * k + q;
        int32_t j;
        double w;
        bool bd;
        const bool ok = slot_edge(nbr, val, val_f64, n, i, sl, P, j, w, bd);
        const int p = sm.roff[r] + q;
        if (staged) {
            sm.key[p] = ok ? (((uint64_t)(uint32_t)j << 32) | (uint32_t)p) : SENT;
            sm.w[p] = w;
        } else {
            col[gbase + p] = ok ? j : EMPTY;
            wt[gbase + p] = w;
        }
    }
    for (int64_t e = e0 + t; e < e1; e += BT) {
        const int4 rc = rec[e];
        const int p = sm.roff[rc.y] + k + atomicAdd(&sm.rfill[rc.y], 1);
        if (staged) {
            sm.key[p] = ((uint64_t)(uint32_t)rc.x << 32) | (uint32_t)p;
            sm.w[p] = __longlong_as_double(((long long)rc.w << 32) | (long long)(unsigned)rc.z);
        } else {
            col[gbase + p] = rc.x;
            wt[gbase + p] = __longlong_as_double(((long long)rc.w << 32) |
                                                 (long long)(unsigned)rc.z);
        }
    }
    __syncthreads();
    auto raw_out = [&](int r) {  // the row's raw segment for the general path
        const int o = sm.roff[r], mr = sm.roff[r + 1] - o;
        for (int e = lane; e < mr; e += 64) {
            const uint64_t x = sm.key[o + e];
            col[gbase + o + e] = x == SENT ? EMPTY : (int)(x >> 32);
            wt[gbase + o + e] = x == SENT ? 0.0 : sm.w[(uint32_t)x];
        }
    };
    for (int r = wv; r < nr; r += BT / 64) {
        const int64_t i = row0 + r;
        const int o = sm.roff[r], mr = sm.roff[r + 1] - o;
        if (!staged) {  // sorted from global memory by the list kernels
            if (lane == 0) {
                sm.ukept[r] = -1;
                if (mr <= 256) wave_list[atomicAdd(wave_count, 1)] = (int32_t)i;
                else mid_list[atomicAdd(mid_count, 1)] = (int32_t)i;
            }
            continue;
        }
        auto keyf = [&](int e) { return sm.key[o + e]; };
        auto wf = [&](uint32_t e) { return sm.w[e]; };
        // the kept weights go back into the row's own stage region (every
        // gather of the row is issued before its first store), ascending
        int u = 0;
        int rc;
        if (k32 && mr <= 256) {
            auto key32 = [&](int e) {
                const uint64_t kk = sm.key[o + e];
                return kk == SENT ? SENT32 : (((uint32_t)(kk >> 32) << 8) | (uint32_t)e);
            };
            auto w32 = [&](int e) { return sm.w[o + e]; };
            bool ok;
            if (mr <= 64) ok = packed_row32<1>(key32, w32, mr, gbase + o, col, wt, &sm.w[o], &u);
            else if (mr <= 128) ok = packed_row32<2>(key32, w32, mr, gbase + o, col, wt, &sm.w[o], &u);
            else ok = packed_row32<4>(key32, w32, mr, gbase + o, col, wt, &sm.w[o], &u);
            rc = ok ? 1 : 0;
        } else {
            rc = packed_row_nofold(keyf, wf, mr, i, gbase + o, P.sym, col, wt, uniq, kept, deg64,
                                   deg32, &sm.w[o], &u);
        }
        if (rc != 1) {  // longer rows / duplicate ids: the wave kernel <16> from global
            raw_out(r);
            if (lane == 0) mid_list[atomicAdd(mid_count, 1)] = (int32_t)i;
        }
        if (lane == 0) sm.ukept[r] = rc == 1 ? u : -1;
    }
    __syncthreads();
    // the degrees: one lane per row, the row's kept weights in ascending
    // column order (the reference's sequential sum), all rows of the bucket
    // at once instead of one lane read at a time per row
    if (t < nr && staged) {
        const int u = sm.ukept[t];
        if (u >= 0) {
            const int64_t i = row0 + t;
            const double *wr = &sm.w[sm.roff[t]];
            uniq[i] = u;
            if (P.sym == MN_SYM_UNION) {
                double s64 = -0.0;  // laplacian.rs:367 s.iter().map(w).sum() in ascending j
                for (int e = 0; e < u; ++e) s64 = s64 + wr[e];
                deg64[i] = s64;
                kept[i] = u + 1;
            } else {
                float s32 = 0.0f;  // surfface-core/src/laplacian.rs:331-340
                for (int e = 0; e < u; ++e) s32 = s32 + (float)wr[e];
                deg32[i] = s32;
            }
        }
    }
}

// ---- MAX: kept counts; CSR write ------------------------------------------

__device__ __forceinline__ float max_offdiag(float w, float di, float dj, int normalize) {
    return normalize ? -w / sqrt_rn_f32(di * dj) : -w;
}

// does the MAX entry (i, j) survive (surfface-core/src/laplacian.rs:355-394, 215)
__device__ __forceinline__ bool max_entry(const Params &P, float di, float dj, double w,
                                          float &v) {
    const float thr = (float)P.thr;
    if (P.normalize && (di <= thr || dj <= thr)) return false;
    v = max_offdiag((float)w, di, dj, P.normalize);
    return fabsf(v) > 1e-9f;
}

__device__ __forceinline__ bool max_has_diag(const Params &P, float di) {
    return di > (float)P.thr && fabsf(P.normalize ? 1.0f : di) > 1e-9f;
}

__global__ __launch_bounds__(256) void k_kept_max(const int64_t *__restrict__ offs,
                                                  const int32_t *__restrict__ col,
                                                  const double *__restrict__ wt,
                                                  const int32_t *__restrict__ uniq, int64_t n,
                                                  Params P, const float *__restrict__ deg32,
                                                  int32_t *__restrict__ kept) {
    const int lane = threadIdx.x & 63;
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i >= n) return;
    const int64_t o = offs[i];
    const int u = uniq[i];
    const float di = deg32[i];
    int c = 0;
    for (int e0 = 0; e0 < u; e0 += 64) {
        const int e = e0 + lane;
        float v = 0.f;
        const bool keep = e < u && max_entry(P, di, deg32[col[o + e]], wt[o + e], v);
        c += (int)__popcll(__ballot(keep));
    }
    if (lane == 0) kept[i] = c + (max_has_diag(P, di) ? 1 : 0);
}

// one wave per row: the row's entries (ascending columns) and its diagonal
__global__ __launch_bounds__(256) void k_write_csr(const int64_t *__restrict__ offs,
                                                   const int32_t *__restrict__ col,
                                                   const double *__restrict__ wt,
                                                   const int32_t *__restrict__ uniq, int64_t n,
                                                   Params P, const double *__restrict__ deg64,
                                                   const float *__restrict__ deg32,
                                                   const int64_t *__restrict__ indptr,
                                                   int64_t cap, int32_t *__restrict__ out_col,
                                                   double *__restrict__ out_v64,
                                                   float *__restrict__ out_v32) {
    const int lane = threadIdx.x & 63;
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i >= n) return;
    // a caller-owned output that is too small gets nothing (MN_ECAP on return)
    if (indptr[n] > cap) return;
    const int64_t o = offs[i];
    const int u = uniq[i];
    const int64_t q0 = indptr[i];
    const uint64_t below = (1ull << lane) - 1ull;
    if (P.sym == MN_SYM_UNION) {
        int nlt = 0;  // entries left of the diagonal
        for (int e0 = 0; e0 < u; e0 += 64) {
            const int e = e0 + lane;
            const bool ok = e < u;
            const int j = ok ? col[o + e] : 0;
            nlt += (int)__popcll(__ballot(ok && j < i));
            if (ok) {
                const int64_t q = q0 + e + (j > i ? 1 : 0);
                out_col[q] = j;
                out_v64[q] = -wt[o + e];
            }
        }
        if (lane == 0) {
            out_col[q0 + nlt] = (int32_t)i;
            out_v64[q0 + nlt] = deg64[i];
        }
        return;
    }
    const float di = deg32[i];
    const bool has_diag = max_has_diag(P, di);
    int base = 0, nlt = 0;
    for (int e0 = 0; e0 < u; e0 += 64) {
        const int e = e0 + lane;
        float v = 0.f;
        int j = 0;
        bool keep = false;
        if (e < u) {
            j = col[o + e];
            keep = max_entry(P, di, deg32[j], wt[o + e], v);
        }
        const uint64_t mk = __ballot(keep);
        nlt += (int)__popcll(__ballot(keep && j < i));
        if (keep) {
            const int64_t q =
                q0 + base + (int)__popcll(mk & below) + ((has_diag && j > i) ? 1 : 0);
            out_col[q] = j;
            out_v32[q] = v;
        }
        base += (int)__popcll(mk);
    }
    if (lane == 0 && has_diag) {
        out_col[q0 + nlt] = (int32_t)i;
        out_v32[q0 + nlt] = P.normalize ? 1.0f : di;
    }
}

inline unsigned grid_for(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

}  // namespace lap

static thread_local mn_lap_stats t_lap_stats{};

static int laplacian_impl(const int32_t *nbr, const void *val, int32_t val_f64, int64_t n,
                          int32_t k, const mn_lap_opts *opts, mn_csr *out, void *degrees_out) {
    using namespace lap;
    clear_error();
    t_lap_stats = mn_lap_stats{};
    MN_REQUIRE(opts && out, MN_EINVAL, "mn_laplacian_from_knn: NULL opts/out");
    const mn_csr given = *out;
    const bool caller = given.caller_owned == 1;
    *out = mn_csr{};
    if (caller) {
        MN_REQUIRE(given.indptr && given.indices && given.values && given.nnz >= 0, MN_EINVAL,
                   "mn_laplacian_from_knn: caller-owned output needs indptr/indices/values");
        const int want = opts->symmetrise == MN_SYM_UNION ? MN_F64 : MN_F32;
        MN_REQUIRE(given.value_type == want, MN_EINVAL,
                   "mn_laplacian_from_knn: caller-owned values must be %s",
                   want == MN_F64 ? "f64 (UNION)" : "f32 (MAX)");
    }
    MN_REQUIRE(n >= 1 && k >= 0 && (k == 0 || (nbr && val)), MN_EINVAL,
               "mn_laplacian_from_knn: bad shape n=%lld k=%d", (long long)n, k);
    MN_REQUIRE(n < INT_MAX, MN_EINVAL, "mn_laplacian_from_knn: n must fit int32");
    MN_REQUIRE(opts->weight_kernel == MN_W_GIVEN || opts->weight_kernel == MN_W_RATIONAL,
               MN_EINVAL, "mn_laplacian_from_knn: unknown weight_kernel");
    MN_REQUIRE(opts->symmetrise == MN_SYM_UNION || opts->symmetrise == MN_SYM_MAX, MN_EINVAL,
               "mn_laplacian_from_knn: unknown symmetrise mode");
    MN_REQUIRE(!(opts->symmetrise == MN_SYM_UNION && opts->normalize), MN_ENOTSUP,
               "mn_laplacian_from_knn: the legacy UNION Laplacian is unnormalised (D - W)");
    if (opts->weight_kernel == MN_W_RATIONAL)
        MN_REQUIRE(opts->sigma > 0.0, MN_EINVAL, "mn_laplacian_from_knn: sigma must be > 0");
    Params P{opts->weight_kernel, opts->symmetrise, opts->normalize ? 1 : 0, opts->eps,
             opts->sigma, opts->p, opts->weight_threshold};
    hipStream_t s = (hipStream_t)opts->stream;
    const int64_t nk = n * (int64_t)k;

    // scratch: per-row ints + offsets; row segments (k + in-degree per row)
    char *g1 = (char *)scratch(kSlotGeneric1, (size_t)n * 4 * 5 + (size_t)(n + 1) * 8 + 64 +
                                               ((size_t)n / scan::SB + 2) * 8);
    char *g2 = (char *)scratch(kSlotGeneric2, (size_t)(2 * nk + 1) * 12 + 64);
    int *flags = (int *)scratch(kSlotFlags, 64);
    int32_t *lists = (int32_t *)scratch(kSlotGeneric3, (size_t)n * 12 + 64);
    MN_REQUIRE(g1 && g2 && flags && lists, MN_ENOMEM,
               "mn_laplacian_from_knn: scratch allocation failed");
    int32_t *indeg = (int32_t *)g1;
    int32_t *seg = indeg + n;
    int32_t *fill = seg + n;
    int32_t *uniq = fill + n;
    int32_t *kept = uniq + n;
    int64_t *offs = (int64_t *)(((uintptr_t)(kept + n) + 15) & ~(uintptr_t)15);
    int64_t *part = offs + (n + 1);
    const int64_t E2 = 2 * nk;
    int32_t *col = (int32_t *)g2;
    double *wt = (double *)(g2 + (((size_t)E2 * 4 + 15) & ~(size_t)15));
    int32_t *big_list = lists, *huge_list = lists + n, *mid_list = lists + 2 * n;
    // degrees (into degrees_out when given, else scratch)
    void *degbuf = degrees_out;
    if (!degbuf) {
        degbuf = scratch(kSlotNorms2, (size_t)n * 8);
        MN_REQUIRE(degbuf, MN_ENOMEM, "mn_laplacian_from_knn: scratch allocation failed");
    }
    double *deg64 = P.sym == MN_SYM_UNION ? (double *)degbuf : nullptr;
    float *deg32 = P.sym == MN_SYM_UNION ? nullptr : (float *)degbuf;

    // bucketed assembly (the atomic counting-sort path for shapes outside its
    // limits; tuning build: MN_LAP_V1=1 forces it, A/B)
    const int64_t NB = (n + BR - 1) / BR;
    const int64_t nA = (nk + ACH - 1) / ACH;
    const char *v1e = knob("MN_LAP_V1");
    const bool v2 = k > 0 && NB <= NBMAX && nk < INT_MAX && !(v1e && *v1e == '1');
    char *g0 = nullptr;
    if (v2) {
        g0 = (char *)scratch(kSlotGeneric0, (size_t)nk * 16 + (size_t)nA * NB * 4 +
                                                (size_t)NB * 4 + (size_t)(NB + 1) * 8 + 1024);
        MN_REQUIRE(g0, MN_ENOMEM, "mn_laplacian_from_knn: scratch allocation failed");
    }

    Timer tm;
    tm.start(true, s);
    MN_HIP_TRY(hipMemsetAsync(indeg, 0, (size_t)n * 4 * 5, s));
    MN_HIP_TRY(hipMemsetAsync(flags, 0, 32, s));  // [1] big [2] hub [3] wave [4] mid lists
    if (v2) {
        int4 *rec = (int4 *)g0;
        int32_t *cnt = (int32_t *)(g0 + (size_t)nk * 16);
        int32_t *tot = cnt + (size_t)nA * NB;
        int64_t *bstart = (int64_t *)(((uintptr_t)(tot + NB) + 15) & ~(uintptr_t)15);
        int32_t *wave_list = huge_list;  // reused: the hub list is filled after the wave pass
        hipLaunchKernelGGL(k_lap_bhist, dim3((unsigned)nA), dim3(ANT), 0, s, nbr, val, val_f64, n,
                           k, P, (int)NB, cnt, flags);
        hipLaunchKernelGGL(k_lap_bscan, dim3(grid_for(NB * 64)), dim3(256), 0, s, cnt, (int)nA,
                           (int)NB, tot);
        MN_HIP_TRY(scan::exclusive_scan(tot, NB, bstart, part, s));
        hipLaunchKernelGGL(k_lap_bscatter, dim3((unsigned)nA), dim3(ANT), 0, s, nbr, val, val_f64,
                           n, k, P, (int)NB, cnt, bstart, rec);
        hipLaunchKernelGGL(k_lap_bucket, dim3((unsigned)NB), dim3(BT), 0, s, nbr, val, val_f64, n,
                           k, P, bstart, rec, offs, col, wt, uniq, kept, deg64, deg32, wave_list,
                           flags + 3, mid_list, flags + 4);
        MN_KCHECK(s, "k_lap_bucket");
        // rows of buckets too large for the LDS stage (hub buckets)
        hipLaunchKernelGGL(k_row_sort_wave<4>, dim3(256), dim3(256), 0, s, offs, n, P.sym, col, wt,
                           uniq, kept, deg64, deg32, mid_list, flags + 4, wave_list, flags + 3);
    } else {
        if (k > 0)
            hipLaunchKernelGGL(k_lap_slots, dim3(grid_for(nk)), dim3(256), 0, s, nbr, val, val_f64,
                               n, k, P, indeg, flags);
        hipLaunchKernelGGL(k_seg_len, dim3(grid_for(n)), dim3(256), 0, s, indeg, n, k, seg);
        MN_HIP_TRY(scan::exclusive_scan(seg, n, offs, part, s));
        if (k > 0)
            hipLaunchKernelGGL(k_lap_scatter, dim3(grid_for(nk)), dim3(256), 0, s, nbr, val,
                               val_f64, n, k, P, offs, fill, col, wt);
        hipLaunchKernelGGL(k_row_sort_wave<4>, dim3(grid_for(n * 64)), dim3(256), 0, s, offs, n,
                           P.sym, col, wt, uniq, kept, deg64, deg32, mid_list, flags + 4,
                           (const int32_t *)nullptr, (const int *)nullptr);
    }
    // rows of 257..1024 entries (one wave, 16 keys a lane), then longer ones
    hipLaunchKernelGGL(k_row_sort_wave<16>, dim3(1024), dim3(256), 0, s, offs, n, P.sym, col, wt,
                       uniq, kept, deg64, deg32, big_list, flags + 1, mid_list, flags + 4);
    hipLaunchKernelGGL(k_row_sort_block, dim3(256), dim3(1024), 0, s, offs, big_list, flags + 1,
                       P.sym, col, wt, uniq, kept, deg64, deg32, huge_list, flags + 2);
    hipLaunchKernelGGL(k_row_sort_hub, dim3(64), dim3(1024), 0, s, offs, huge_list, flags + 2,
                       P.sym, col, wt, uniq, kept, deg64, deg32);
    MN_KCHECK(s, "k_row_sort");
    if (P.sym == MN_SYM_MAX)
        hipLaunchKernelGGL(k_kept_max, dim3(grid_for(n * 64)), dim3(256), 0, s, offs, col, wt,
                           uniq, n, P, deg32, kept);
    // outputs sized on the device side: a library-owned CSR gets the bound
    // n + 2 n k (every row: its diagonal + at most k forward and all reverse
    // slots), a caller-owned one is checked against its capacity inside
    // k_write_csr, so nnz is read back once, with the final synchronisation
    const size_t vsz = P.sym == MN_SYM_UNION ? 8 : 4;
    const int64_t cap = caller ? given.nnz : n + 2 * nk;
    int64_t *indptr = caller ? given.indptr : nullptr;
    int32_t *ocol = caller ? given.indices : nullptr;
    void *oval = caller ? given.values : nullptr;
    if (!caller && (hipMalloc(&indptr, sizeof(int64_t) * (n + 1)) != hipSuccess ||
                    hipMalloc(&ocol, sizeof(int32_t) * std::max<int64_t>(cap, 1)) != hipSuccess ||
                    hipMalloc(&oval, vsz * std::max<int64_t>(cap, 1)) != hipSuccess)) {
        (void)hipFree(indptr); (void)hipFree(ocol); (void)hipFree(oval);
        set_error("mn_laplacian_from_knn: output allocation (%lld entries) failed", (long long)cap);
        return MN_ENOMEM;
    }
    MN_HIP_TRY(scan::exclusive_scan(kept, n, indptr, part, s));
    hipLaunchKernelGGL(k_write_csr, dim3(grid_for(n * 64)), dim3(256), 0, s, offs, col, wt, uniq,
                       n, P, deg64, deg32, indptr, cap, ocol, (double *)oval, (float *)oval);
    MN_HIP_TRY(hipGetLastError());
    tm.mark();
    int64_t nnz = 0;
    int hf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    MN_HIP_TRY(hipMemcpyAsync(&nnz, indptr + n, 8, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipMemcpyAsync(hf, flags, 32, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    t_lap_stats.big_rows = hf[4];  // rows past the one-wave 256-entry sort
    t_lap_stats.hub_rows = hf[2];
    if (hf[0] != 0) {  // out-of-range neighbour ids were skipped everywhere; outputs void
        if (!caller) { (void)hipFree(indptr); (void)hipFree(ocol); (void)hipFree(oval); }
        set_error("mn_laplacian_from_knn: neighbour index >= n");
        return MN_EINVAL;
    }
    if (nnz > cap) {  // caller-owned only (the library bound always holds)
        out->nnz = nnz;
        set_error("mn_laplacian_from_knn: output capacity %lld < nnz %lld", (long long)cap,
                  (long long)nnz);
        return MN_ECAP;
    }
    t_lap_stats.ms_total = tm.ms(0, 1);
    t_lap_stats.nnz = nnz;
    out->n_rows = n;
    out->n_cols = n;
    out->nnz = nnz;
    out->indptr = indptr;
    out->indices = ocol;
    out->values = oval;
    out->value_type = P.sym == MN_SYM_UNION ? MN_F64 : MN_F32;
    out->caller_owned = caller ? 1 : 0;
    return MN_OK;
}

}  // namespace mn

extern "C" {

int mn_laplacian_from_knn(const int32_t *nbr_idx, const void *nbr_val, int32_t val_is_f64,
                          int64_t n, int32_t k, const mn_lap_opts *opts, mn_csr *out,
                          void *degrees_out) {
    return mn::laplacian_impl(nbr_idx, nbr_val, val_is_f64, n, k, opts, out, degrees_out);
}

int mn_csr_free(mn_csr *m) {
    if (!m) return MN_OK;
    if (m->caller_owned) {  // not ours to free
        *m = mn_csr{};
        return MN_OK;
    }
    if (m->indptr) (void)hipFree(m->indptr);
    if (m->indices) (void)hipFree(m->indices);
    if (m->values) (void)hipFree(m->values);
    *m = mn_csr{};
    return MN_OK;
}

int mn_lap_last_stats(mn_lap_stats *out) {
    if (!out) return MN_EINVAL;
    *out = mn::t_lap_stats;
    return MN_OK;
}

}  // extern "C"
