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
#include <algorithm>
#include <climits>

#include "common.hpp"

namespace mn {
namespace kb16 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256;           // queries per block (8 waves x 32 rows)
constexpr int BN = 128;           // corpus rows per tile (4 column blocks of 32)
constexpr int BK = 32;            // bf16 features per LDS stage (2 x 16-deep MFMA steps)
constexpr int LDK = BK;           // 64-B rows, 16-B chunks XOR-swizzled by (row >> 2) & 3
constexpr int NWAVES = 8;         // two waves per SIMD: one's epilogue/DMA overlaps the other's MFMAs
constexpr int WR = BM / NWAVES;   // rows per wave (one 32-row MFMA block)
constexpr int RM = WR / 32;
constexpr int NT = 64 * NWAVES;
constexpr int NCT = BN / 32;
constexpr int QCAP = 40;
constexpr int QPRE = QCAP - 32;   // merge before a 32-column block if cnt > QPRE
constexpr int NSTAGE = 3;         // LDS-DMA ring depth (two stages in flight)
constexpr int LMAX = 128 - QCAP;  // L + QCAP <= 128
constexpr int KMAX = 64;

struct alignas(16) Smem {
    uint16_t A[NSTAGE][BM][LDK];
    uint16_t B[NSTAGE][BN][LDK];
    float qd[BM][QCAP];
    int qi[BM][QCAP];
    float cinv[2][BN];
    float qinv[BM];
    float tau[BM];
    int cnt[BM];
    int lsz[BM];
    int ovf[BM];
};

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
                acc = acc + a * a;
                acc = acc + b * b;
            }
        }
    } else {
        for (; t < d; ++t) {
            const double a = bf2d(p[t]);
            bad |= !isfinite(a);
            acc = acc + a * a;
        }
    }
    const double nv = __builtin_sqrt(acc);
    nrm[i] = nv;
    inv[i] = nv > 0.0 ? (float)(1.0 / nv) : 0.f;
    if (bad) atomicOr(nonfinite, 1);
}

// ---- candidate generation -----------------------------------------------------
__device__ __forceinline__ void merge_row(Smem &sm, int row, int L, float *__restrict__ ld,
                                          int *__restrict__ li) {
    const int lane = threadIdx.x & 63;
    const int s = sm.lsz[row], c = sm.cnt[row];
    float d[2];
    int ix[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        if (e < s) { d[r] = ld[e]; ix[r] = li[e]; }
        else if (e < s + c) { d[r] = sm.qd[row][e - s]; ix[r] = sm.qi[row][e - s]; }
        else { d[r] = __builtin_inff(); ix[r] = INT_MAX; }
    }
    wave_bitonic_sort<2>(d, ix);
    const int ns = min(L, s + c);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        if (e < ns) { ld[e] = d[r]; li[e] = ix[r]; }
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

__device__ const uint4 g_zero16[1] = {{0u, 0u, 0u, 0u}};
#ifdef MN_BF16_DEBUG
__device__ float g_dbg_keys[256 * 256];
#endif

// physical 16-B chunk of logical chunk c in LDS row r (conflict-free b128 reads
// for 32 consecutive rows; LDS-DMA writes lane-linearly, so the permutation is
// applied to the per-lane SOURCE address and again on the read)
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 2) & 3); }

// One LDS-DMA piece: 16 rows x 64 B (= 64 lanes x 16 B) of a [rows][d] bf16
// matrix, rows row0.., features k0..k0+31, into a lane-linear LDS image.
// Rows past nrows re-read row 0 (masked later); features past d read zeros.
__device__ __forceinline__ void dma_piece(const uint16_t *__restrict__ X, int64_t row0,
                                          int64_t nrows, int d, int k0, uint16_t *lds_piece,
                                          int lane) {
    const int r = lane >> 2, pc = lane & 3;
    const int c = pc ^ ((r >> 2) & 3);  // rows of a piece start at a multiple of 16
    const int64_t row = row0 + r;
    const int k = k0 + 8 * c;
    const void *src = (row < nrows && k < d) ? (const void *)(X + row * (int64_t)d + k)
                                             : (const void *)g_zero16;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_piece, 16, 0, 0);
}

struct EpiCtx {
    int dx, qlim, clim, gc0, par, S, sl, L;
    int64_t q0;
    float *list_d;
    int *list_i;
};

// One 32x32 accumulator block (rows 32M.. of the wave, columns 32T.. of the
// tile): merge rows whose queue could overflow (a block adds <= 32 entries per
// row), then filter key < tau and append survivors to the per-row LDS queues.
// `lane` is passed in opaque (see the call site).
template <int M, int T>
__device__ __forceinline__ void epilogue_block(Smem &sm, const EpiCtx &ec, const f32x16 &v,
                                               int lane, int w) {
    const int h = lane >> 5, cl = lane & 31;
    {
        const int c = lane < WR ? sm.cnt[WR * w + lane] : 0;
        uint64_t need = __ballot(c > QPRE);
        while (need) {
            const int rr = __builtin_ctzll(need);
            need &= need - 1;
            const int row = WR * w + rr;
            const int64_t base = ((ec.q0 + row) * ec.S + ec.sl) * (int64_t)ec.L;
            merge_row(sm, row, ec.L, ec.list_d + base, ec.list_i + base);
        }
    }
    const int colr = 32 * T + cl;
    const bool colok = colr < ec.clim;
    const float ci = sm.cinv[ec.par][colr];
    const int gcol = ec.gc0 + colr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int lrow = WR * w + 32 * M + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float qi = sm.qinv[lrow];
        const bool valid = colok && lrow < ec.qlim && (lrow - colr) != ec.dx;
        // n_q n_c near the reference's denom > 1e-12 switch: the approximation
        // cannot tell cos from 0, so the pair becomes a forced candidate (key
        // below every real key) and the exact re-rank decides.  Exactly-zero
        // norms give key = -0 = exact.
        const float key = (qi * ci > 5e11f) ? -2.f : -(v[r] * qi) * ci;  // -cos~
#ifdef MN_BF16_DEBUG
        if (blockIdx.x == 0 && ec.gc0 == 0) g_dbg_keys[lrow * 256 + colr] = key;
#endif
        const bool bad = valid && !(__builtin_fabsf(key) <= 2.f);
        const bool pass = valid && !bad && key < sm.tau[lrow];
        if (__builtin_expect(__ballot(bad) != 0, 0)) {
            if (bad) sm.ovf[lrow] = 1;
            __builtin_amdgcn_wave_barrier();
        }
        const uint64_t pm = __ballot(pass);
        if (pm) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const uint32_t mh = (uint32_t)(pm >> (32 * hh));
                if (!mh) continue;
                const int row = WR * w + 32 * M + (r & 3) + 8 * (r >> 2) + 4 * hh;
                const int c = sm.cnt[row];
                if (h == hh && pass) {
                    const int pos = c + __popc(mh & ((1u << cl) - 1u));
                    sm.qd[row][pos] = key;
                    sm.qi[row][pos] = gcol;
                }
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) sm.cnt[row] = c + __popc(mh);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

// Grid: one block per (query block, corpus slice), 1-D.  Consecutive blocks
// land on different XCDs, so the linear id is remapped (bijectively) such that
// the blocks one XCD runs together share query panels and corpus tiles in its
// L2: all S slices of a query block are adjacent in the remapped order.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__global__ __launch_bounds__(NT) void k_gram_bf16(
    const uint16_t *__restrict__ Q, int64_t nq, const uint16_t *__restrict__ C, int64_t nc, int d,
    int64_t q_off, int64_t c_off, int excl, const float *__restrict__ qinv,
    const float *__restrict__ cinv, int L, int S, int64_t chunk, float *__restrict__ list_d,
    int *__restrict__ list_i, int *__restrict__ out_lsz, float *__restrict__ out_tau) {
    __shared__ Smem sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR row math
    const int h = lane >> 5, cl = lane & 31;
    const int wg = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int64_t q0 = (int64_t)(wg / S) * BM;
    const int sl = wg % S;
    const int64_t cbeg = (int64_t)sl * chunk, cend = min(nc, cbeg + chunk);
    for (int r = tid; r < BM; r += NT) {
        sm.qinv[r] = (q0 + r < nq) ? qinv[q0 + r] : 0.f;
        sm.tau[r] = __builtin_inff();
        sm.cnt[r] = 0;
        sm.lsz[r] = 0;
        sm.ovf[r] = 0;
    }
    __syncthreads();
    const int nk = (d + BK - 1) / BK;
    // staging per stage: A = 16 pieces, B = 8 pieces (16 rows x 64 B each);
    // wave w issues A pieces 2w, 2w+1 and B piece w
    static_assert(BM / 16 == 2 * NWAVES && BN / 16 == NWAVES, "staging split");
    constexpr int kPiecesPerWave = 3;
    auto stage = [&](int buf, int64_t c0, int kt) {
        const int k0 = kt * BK;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int pc = 2 * w + u;
            dma_piece(Q, q0 + 16 * pc, nq, d, k0, &sm.A[buf][16 * pc][0], lane);
        }
        dma_piece(C, c0 + 16 * w, cend, d, k0, &sm.B[buf][16 * w][0], lane);
    };
    // Stage ring over the whole sweep: global stage g = tile * nk + kt lives in
    // buffer g % NSTAGE; two stages are in flight while one is consumed.  Each
    // wave issues kPiecesPerWave LDS-DMA pieces per stage, so "stage g landed" is
    // vmcnt(kPiecesPerWave * stages issued after g).
    int64_t ic0 = cbeg;  // next stage to issue: tile base, k-step, ring slot
    int ikt = 0, ibuf = 0;
    auto issue = [&]() {
        if (ic0 < cend) {
            stage(ibuf, ic0, ikt);
            ibuf = ibuf == NSTAGE - 1 ? 0 : ibuf + 1;
            if (++ikt == nk) { ikt = 0; ic0 += BN; }
        }
    };
    issue();
    issue();
    int cur = 0;
    int par = 0;
    for (int64_t c0 = cbeg; c0 < cend; c0 += BN, par ^= 1) {
        if (tid < BN) sm.cinv[par][tid] = (c0 + tid < cend) ? cinv[c0 + tid] : 0.f;
        f32x16 acc[RM][NCT];
#pragma unroll
        for (int m = 0; m < RM; ++m)
#pragma unroll
            for (int t = 0; t < NCT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[m][t][r] = 0.f;
        for (int kt = 0; kt < nk; ++kt, cur = cur == NSTAGE - 1 ? 0 : cur + 1) {
            // this stage landed (one stage may stay in flight behind it) ...
            if (ic0 < cend) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kPiecesPerWave) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // ... and is visible to all waves, which are all done with the
            // previous stage's buffer: the next issue overwrites it
            __builtin_amdgcn_s_barrier();
            issue();
#pragma unroll
            for (int ks = 0; ks < BK / 16; ++ks) {
                bf16x8 a[RM], b[NCT];
#pragma unroll
                for (int m = 0; m < RM; ++m) {
                    const int ar = WR * w + 32 * m + cl;
                    a[m] = *reinterpret_cast<const bf16x8 *>(&sm.A[cur][ar][8 * swz(ar, 2 * ks + h)]);
                }
#pragma unroll
                for (int t = 0; t < NCT; ++t) {
                    const int br = 32 * t + cl;
                    b[t] = *reinterpret_cast<const bf16x8 *>(&sm.B[cur][br][8 * swz(br, 2 * ks + h)]);
                }
#pragma unroll
                for (int t = 0; t < NCT; ++t)
#pragma unroll
                    for (int m = 0; m < RM; ++m)
                        acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m], b[t], acc[m][t], 0, 0, 0);
            }
        }
        __syncthreads();  // cinv[par] written by other waves
        // ---- epilogue: key = -cos~, filter, queue, merge (64 rows per wave) ----
        // global ids equal  <=>  lrow - col_in_tile == (c_off + c0) - (q_off + q0)
        const int64_t dl = (c_off + c0) - (q_off + q0);
        EpiCtx ec;
        ec.dx = (excl && dl > -2 * BM && dl < 2 * BM) ? (int)dl : INT_MIN / 2;
        ec.qlim = (int)min<int64_t>(BM, nq - q0);
        ec.clim = (int)min<int64_t>(BN, cend - c0);
        ec.gc0 = (int)(c_off + c0);
        ec.par = par;
        ec.q0 = q0;
        ec.S = S;
        ec.sl = sl;
        ec.L = L;
        ec.list_d = list_d;
        ec.list_i = list_i;
        // lane id re-materialised per block: keeps the compiler from hoisting
        // every epilogue address out of the tile loop (register pressure)
#define MN_EPI(M, T)                                                                       \
    {                                                                                      \
        int lo = lane, wo = w;                                                             \
        asm volatile("" : "+v"(lo), "+s"(wo));                                             \
        epilogue_block<M, T>(sm, ec, acc[M][T], lo, wo);                                   \
    }
        MN_EPI(0, 0) MN_EPI(0, 1) MN_EPI(0, 2) MN_EPI(0, 3)
#undef MN_EPI
        // the epilogue's list stores must not satisfy the next counted vmcnt
        // ahead of an older LDS-DMA piece: drain them here (once per tile)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (int rr = 0; rr < WR; ++rr) {
        const int row = WR * w + rr;
        if (sm.cnt[row] > 0) {
            const int64_t base = ((q0 + row) * S + sl) * (int64_t)L;
            merge_row(sm, row, L, list_d + base, list_i + base);
        }
    }
    {
        const int row = WR * w + lane;
        const int64_t q = q0 + row;
        if (q < nq) {
            out_lsz[q * S + sl] = sm.lsz[row];
            out_tau[q * S + sl] = sm.ovf[row] ? -__builtin_inff() : sm.tau[row];
        }
    }
}

// ---- exact re-rank / certification / filter --------------------------------------
__device__ __forceinline__ double exact_dot(const uint16_t *__restrict__ a,
                                            const uint16_t *__restrict__ b, int d) {
    double acc = -0.0;
    if ((d & 7) == 0) {
        for (int t = 0; t < d; t += 8) {
            const uint4 va = *reinterpret_cast<const uint4 *>(a + t);
            const uint4 vb = *reinterpret_cast<const uint4 *>(b + t);
            const uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = acc + bf2d((uint16_t)(wa[u] & 0xFFFFu)) * bf2d((uint16_t)(wb[u] & 0xFFFFu));
                acc = acc + bf2d((uint16_t)(wa[u] >> 16)) * bf2d((uint16_t)(wb[u] >> 16));
            }
        }
    } else {
        for (int t = 0; t < d; ++t) acc = acc + bf2d(a[t]) * bf2d(b[t]);
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
    const double pw = p == 2.0 ? x * x : (p == 1.0 ? x : pow(x, p));
    return 1.0 / (1.0 + pw);
}

template <int NR>
__global__ __launch_bounds__(256) void k_cos_rerank(
    const uint16_t *__restrict__ Q, int64_t nq, const uint16_t *__restrict__ C, int d,
    int64_t c_off, const double *__restrict__ qn, const double *__restrict__ cn, int S, int L,
    const int *__restrict__ list_i, const int *__restrict__ lsz, const float *__restrict__ ltau,
    int topk, int64_t nvalid_max, double delta, double eps, double sigma, double p,
    int32_t *__restrict__ out_idx, double *__restrict__ out_dist, double *__restrict__ out_w,
    int *__restrict__ fb_count, int *__restrict__ fb_list) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    double dd[NR];
    int ix[NR];
    int M = 0;
    float T = __builtin_inff();
    bool forced = false;
    for (int s = 0; s < S; ++s) {
        const int sz = lsz[q * S + s];
        const float ts = ltau[q * S + s];
        forced |= (ts == -__builtin_inff());
        if (sz >= L) T = fminf(T, ts);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int e = lane + 64 * r;
            if (s == 0) ix[r] = -1;
            if (e >= M && e < M + sz) ix[r] = list_i[(q * S + s) * (int64_t)L + (e - M)];
        }
        M += sz;
    }
    const uint16_t *qrow = Q + q * (int64_t)d;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if (ix[r] >= 0) {
            const int64_t c = (int64_t)ix[r] - c_off;
            dd[r] = cos_dist(exact_dot(qrow, C + c * d, d), qn[q], cn[c]);
        } else {
            dd[r] = __builtin_inf();
            ix[r] = INT_MAX;
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

}  // namespace kb16

static thread_local mn_knn_stats t_bf16_stats{};

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
    const int margin = o->margin > 0 ? o->margin : 16;
    const int L = o->topk + margin;
    MN_REQUIRE(L <= LMAX, MN_ENOTSUP, "mn_knn_cos_bf16: topk+margin=%d exceeds %d", L, LMAX);
    MN_REQUIRE(q_off + nq <= INT_MAX && c_off + nc <= INT_MAX, MN_EINVAL,
               "mn_knn_cos_bf16: ids must fit int32");
    hipStream_t s = (hipStream_t)o->stream;
    t_bf16_stats.n_queries = nq;
    if (nq == 0) return MN_OK;
    const bool same = (Q == C) && nq == nc && q_off == c_off;
    const int excl = 1;
    const int64_t blocks_q = (nq + BM - 1) / BM;
    int64_t S = 1;
    if (blocks_q < 512) S = (512 + blocks_q - 1) / blocks_q;
    S = std::min<int64_t>(S, 256 / L);
    S = std::min<int64_t>(S, std::max<int64_t>(1, (nc + BN - 1) / BN));
    S = std::max<int64_t>(S, 1);
    int64_t chunk = (nc + S - 1) / S;
    chunk = std::max<int64_t>(BN, ((chunk + BN - 1) / BN) * BN);
    S = std::max<int64_t>(1, (nc + chunk - 1) / chunk);
    const int SL = (int)(S * L);
    const int NR = SL <= 64 ? 1 : (SL <= 128 ? 2 : 4);
    t_bf16_stats.slices = (int)S;
    t_bf16_stats.list_len = L;

    char *g = (char *)scratch(kSlotNorms, (size_t)(nq + nc) * 12 + 256);
    const size_t nlist = (size_t)nq * S * L;
    char *lists = (char *)scratch(kSlotLists, nlist * 8 + 64);
    char *meta = (char *)scratch(kSlotListMeta, (size_t)nq * S * 8 + 64);
    int *fb_list = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nq + 64);
    int *flags = (int *)scratch(kSlotFlags, 64);
    MN_REQUIRE(g && lists && meta && fb_list && flags, MN_ENOMEM,
               "mn_knn_cos_bf16: scratch allocation failed");
    double *qn = (double *)g;
    double *cn = same ? qn : qn + nq;
    float *qinv = (float *)(qn + nq + (same ? 0 : nc));
    float *cinv = same ? qinv : qinv + nq;
    float *list_d = (float *)lists;
    int *list_i = (int *)(lists + nlist * 4);
    int *lsz = (int *)meta;
    float *ltau = (float *)(meta + (size_t)nq * S * 4);

    const bool misaligned = ((uintptr_t)Q & 15) || ((uintptr_t)C & 15);
    if ((d & 7) || misaligned) {
        // exact: appended zero features add +0 to every norm and dot
        const int d8 = (d + 7) & ~7;
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
    if (nc > 0) {
        hipLaunchKernelGGL(k_gram_bf16, dim3((unsigned)(blocks_q * S)), dim3(NT), 0, s, Q, nq,
                           C, nc, d, q_off, c_off, excl, qinv, cinv, L, (int)S, chunk, list_d,
                           list_i, lsz, ltau);
    } else {
        MN_HIP_TRY(hipMemsetAsync(lsz, 0, sizeof(int) * (size_t)nq * S, s));
    }
    MN_KCHECK(s, "k_gram_bf16");
    tm.mark();
    const double delta = 2.0 * ((double)d + 12.0) * 0x1p-24;
    const int64_t nvalid = same ? nc - 1 : nc;  // qc callers: exclusion inside the shard
    const dim3 rg((unsigned)((nq + 3) / 4));
#define MN_RR(NRV)                                                                              \
    hipLaunchKernelGGL(k_cos_rerank<NRV>, rg, dim3(256), 0, s, Q, nq, C, d, c_off, qn, cn,       \
                       (int)S, L, list_i, lsz, ltau, o->topk, std::max<int64_t>(nvalid, 0),     \
                       delta, o->eps, o->sigma, o->p, out_idx, out_dist, out_w, flags + 2,     \
                       fb_list)
    if (NR == 1) MN_RR(1); else if (NR == 2) MN_RR(2); else MN_RR(4);
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
