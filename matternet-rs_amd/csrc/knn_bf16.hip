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
#include <cmath>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "common.hpp"

namespace mn {
namespace kb16 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256;           // queries per block (8 waves x 32 rows)
constexpr int BN = 128;           // corpus rows per tile (4 column blocks of 32)
constexpr int BK = 64;            // bf16 features per stage (4 x 16-deep MFMA steps)
constexpr int DALIGN = 4 * BK;    // d is padded (exactly, with zeros) to a multiple of this
constexpr int NWAVES = 8;         // two waves per SIMD: one's epilogue/DMA overlaps the other's MFMAs
constexpr int WR = BM / NWAVES;   // rows per wave (one 32-row MFMA block)
constexpr int NT = 64 * NWAVES;
constexpr int NCT = BN / 32;
constexpr int QCAP = 40;          // queued keys per row between threshold updates
constexpr int QPRE = QCAP - 32;   // update before a 32-column block if cnt > QPRE
constexpr int NSLOT = 3;          // corpus-tile LDS-DMA ring (two stages in flight)
constexpr int LMAX = 64;          // L = topk + margin <= LMAX
constexpr int KMAX = 64;

// Query rows never touch LDS: each wave owns its 32 rows and loads their A
// fragments straight into registers.  Only the corpus tile, shared by all 8
// waves, is staged: B[slot][row][64 bf16] (128-B rows, 16-B chunks swizzled).
// Candidate bookkeeping is split: every surviving (key, id) goes straight to a
// per-(row, slice) buffer in HBM (write-only during the sweep); LDS keeps only
// keys — the row's L smallest so far (lk, sorted) and the keys queued since the
// last threshold update (qk) — so a threshold update never reads HBM.
struct alignas(16) Smem {
    uint16_t B[NSLOT][BN][BK];
    float lk[BM][LMAX];
    float qk[BM][QCAP];
    float cinv[2][BN];
    float qinv[BM];
    float tau[BM];
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

// ---- candidate generation -----------------------------------------------------
// Threshold update for row `row`: merge its c queued keys into its sorted
// L smallest keys (LDS only), tau = the L-th smallest once L keys were seen.
__device__ __forceinline__ void update_row(Smem &sm, int row, int c, int L) {
    const int lane = threadIdx.x & 63;
    const int s = sm.lsz[row];
    float k[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        k[r] = e < s ? sm.lk[row][e] : (e < s + c ? sm.qk[row][e - s] : __builtin_inff());
    }
    wave_sort_f32<2>(k);
    const int ns = min(L, s + c);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        if (e < ns) sm.lk[row][e] = k[r];
    }
    const float tl = wave_elem_f32<2>(k, L - 1);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        sm.lsz[row] = ns;
        sm.tau[row] = (ns == L) ? tl : __builtin_inff();
    }
    __builtin_amdgcn_wave_barrier();
}

#ifdef MN_BF16_DEBUG
__device__ float g_dbg_keys[256 * 256];
#endif

// k order inside a stage: MFMA step j, lane half h covers features
// 32h + 8j .. +7 (the dot is order-free; the Gram is only a candidate filter,
// its error bound does not depend on the order).  A lane's A fragments for the
// four steps are then one contiguous 64-B run of its row.
//
// B image: logical 16-B chunk c (= 4h + j) of tile row r sits at physical
// chunk c ^ ((r >> 1) & 7): conflict-free ds_read_b128 for 32 consecutive rows.
__device__ __forceinline__ int bswz(int r, int c) { return c ^ ((r >> 1) & 7); }

// One LDS-DMA piece: 8 tile rows x 128 B (= 64 lanes x 16 B) of the corpus
// stage, lane-linear in LDS, permutation applied on the SOURCE address.  Rows
// past the slice end re-read its last row (masked in the epilogue).
__device__ __forceinline__ void dma_b_piece(const uint16_t *__restrict__ C, int64_t c0,
                                            int64_t cend, int d, int k0, int piece,
                                            uint16_t *lds_piece, int lane) {
    const int r = 8 * piece + (lane >> 3);
    const int c = bswz(r, lane & 7);
    const int64_t row = min(c0 + r, cend - 1);
    const uint16_t *src = C + row * (int64_t)d + k0 + 8 * c;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_piece, 16, 0, 0);
}

struct EpiCtx {
    int dx, qlim, clim, gc0, par, L, cap;
    int64_t q0, S, sl;
    uint2 *buf;  // [q][S][cap] (key bits, id)
};

// Per-lane epilogue state, register resident: the wave's 32 rows are lane
// (h, r) -> row (r & 3) + 8 (r >> 2) + 4 h of the MFMA C layout, so each lane
// keeps qinv and the threshold of its 16 rows; lane l < 32 keeps the queue
// count and the HBM buffer count of row l.  Thresholds only change in
// updates, after which they are re-read: the common path has no LDS round trip.
struct RowRegs {
    float qi[16];
    float tau[16];
    int cnt;   // keys queued in LDS since the last update
    int gcnt;  // (key, id) pairs written to the row's HBM buffer
};

__device__ __forceinline__ void load_row_vals(const float *src, int base, int h, float (&v)[16]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4 *>(src + base + 8 * q + 4 * h);
        v[4 * q + 0] = x.x;
        v[4 * q + 1] = x.y;
        v[4 * q + 2] = x.z;
        v[4 * q + 3] = x.w;
    }
}

// One 32x32 accumulator block (the wave's 32 rows, columns 32T.. of the
// tile): update rows whose queue could overflow (a block adds <= 32 keys per
// row), then filter key < tau; survivors go to the row's HBM buffer and their
// keys to its LDS queue.  `lane` is passed in opaque (see the call site).
template <int T, int PROBE>
__device__ __forceinline__ void epilogue_block(Smem &sm, const EpiCtx &ec, const f32x16 &v,
                                               int lane, int w, RowRegs &rg) {
    const int h = lane >> 5, cl = lane & 31;
    const int base = WR * w;
    {
        uint64_t need = __ballot(lane < WR && rg.cnt > QPRE);
        if (need) {
            while (need) {
                const int rr = __builtin_ctzll(need);
                need &= need - 1;
                const int c = __builtin_amdgcn_readlane(rg.cnt, rr);
                if (PROBE != 3) update_row(sm, base + rr, c, ec.L);
                if (lane == rr) rg.cnt = 0;
            }
            load_row_vals(sm.tau, base, h, rg.tau);
        }
    }
    const int colr = 32 * T + cl;
    const bool colok = colr < ec.clim;
    const float ci = sm.cinv[ec.par][colr];
    const int gcol = ec.gc0 + colr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int lrow = base + rl;
        const float qi = rg.qi[r];
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
        const bool pass = valid && !bad && key < rg.tau[r] && PROBE == 0;
        if (__builtin_expect(__ballot(bad) != 0, 0)) {
            if (bad) sm.ovf[lrow] = 1;
        }
        const uint64_t pm = __ballot(pass);
        if (pm) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const uint32_t mh = (uint32_t)(pm >> (32 * hh));
                if (!mh) continue;
                const int rowl = (r & 3) + 8 * (r >> 2) + 4 * hh;
                const int c = __builtin_amdgcn_readlane(rg.cnt, rowl);
                const int gc = __builtin_amdgcn_readlane(rg.gcnt, rowl);
                if (h == hh && pass) {
                    const int rank = __popc(mh & ((1u << cl) - 1u));
                    sm.qk[base + rowl][c + rank] = key;
                    const int pos = gc + rank;
                    if (pos < ec.cap)
                        ec.buf[((ec.q0 + base + rowl) * ec.S + ec.sl) * (int64_t)ec.cap + pos] =
                            make_uint2(__float_as_uint(key), (uint32_t)gcol);
                }
                if (lane == rowl) {
                    rg.cnt = c + __popc(mh);
                    rg.gcnt = gc + __popc(mh);
                }
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

template <int PROBE>
__global__ __launch_bounds__(NT) void k_gram_bf16(
    const uint16_t *__restrict__ Q, int64_t nq, const uint16_t *__restrict__ C, int64_t nc, int d,
    int64_t q_off, int64_t c_off, int excl, const float *__restrict__ qinv,
    const float *__restrict__ cinv, int L, int S, int64_t chunk, int cap, uint2 *__restrict__ buf,
    int *__restrict__ out_cnt, float *__restrict__ out_tau) {
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
        sm.lsz[r] = 0;
        sm.ovf[r] = 0;
    }
    __syncthreads();
    const int nk = d / BK;  // a multiple of 4 (d is a multiple of DALIGN)
    // this lane's query row (clamped: rows past nq are masked in the epilogue)
    const uint16_t *arow = Q + min(q0 + WR * w + cl, nq - 1) * (int64_t)d + 32 * h;
    // Sweep = ntiles * nk stages; stage g: corpus tile g / nk, k-block g % nk.
    // Stage g's A fragments (4 loads into one of 4 register sets) are issued
    // three stages ahead, its B pieces (2 LDS-DMA into ring slot g % NSLOT) two
    // stages ahead (the slot consumed one step earlier).  Issue order is
    // ... A(g+2) B(g) | A(g+3) barrier B(g+1) ..., so when step g waits, the VM
    // ops issued after B(g) are A(g+2), B(g+1), A(g+3): vmcnt(10) in steady
    // state (fewer near the end of the sweep).
    const int64_t gtot = (int64_t)((cend - cbeg + BN - 1) / BN) * nk;
    int64_t bc0 = cbeg;  // next corpus stage to DMA
    int bkt = 0, bslot = 0;
    auto issue_b = [&]() {
        if (bc0 < cend) {
            dma_b_piece(C, bc0, cend, d, bkt * BK, 2 * w, &sm.B[bslot][16 * w][0], lane);
            dma_b_piece(C, bc0, cend, d, bkt * BK, 2 * w + 1, &sm.B[bslot][16 * w + 8][0], lane);
            bslot = bslot == NSLOT - 1 ? 0 : bslot + 1;
            if (++bkt == nk) { bkt = 0; bc0 += BN; }
        }
    };
    bf16x8 a0[4], a1[4], a2[4], a3[4];
    // A loads are issued from asm so that hipcc does not track them: with an
    // LDS-DMA in flight it would otherwise wait vmcnt(0) at their first use and
    // drain the whole prefetch pipeline every stage.  The counted waits below
    // cover them; `claim_a` then marks the registers as produced at that point.
    auto load_a = [&](bf16x8 (&av)[4], int kt) {
        const uint16_t *p = arow + kt * BK;
        asm volatile("global_load_dwordx4 %0, %4, off\n\t"
                     "global_load_dwordx4 %1, %4, off offset:16\n\t"
                     "global_load_dwordx4 %2, %4, off offset:32\n\t"
                     "global_load_dwordx4 %3, %4, off offset:48"
                     : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3])
                     : "v"(p)
                     : "memory");
    };
    auto claim_a = [&](bf16x8 (&av)[4]) {
        asm volatile("" : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]));
    };
    static_assert(NSLOT == 3, "B is issued two stages ahead into a 3-slot ring");
    if (gtot > 0) load_a(a0, 0);
    if (gtot > 1) load_a(a1, 1 % nk);
    issue_b();  // B(0)
    if (gtot > 2) load_a(a2, 2 % nk);
    issue_b();  // B(1)
    RowRegs rg;
    load_row_vals(sm.qinv, WR * w, h, rg.qi);
#pragma unroll
    for (int r = 0; r < 16; ++r) rg.tau[r] = __builtin_inff();
    rg.cnt = 0;
    rg.gcnt = 0;
    int64_t g = 0;
    int cur = 0;  // LDS slot of the stage being consumed
    int par = 0;
    for (int64_t c0 = cbeg; c0 < cend; c0 += BN, par ^= 1) {
        if (tid < BN) sm.cinv[par][tid] = (c0 + tid < cend) ? cinv[c0 + tid] : 0.f;
        f32x16 acc[NCT];
#pragma unroll
        for (int t = 0; t < NCT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
        auto step = [&](bf16x8 (&ac)[4], bf16x8 (&an)[4], int kt) {
            if (g + 3 < gtot) load_a(an, kt + 3 < nk ? kt + 3 : kt + 3 - nk);
            const int64_t rem = gtot - 1 - g;
            if (rem >= 3) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
            else if (rem == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if (rem == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            claim_a(ac);
            __builtin_amdgcn_s_barrier();  // stage landed for all; slot of g-1 free
            issue_b();      // B(g+2)
            // B fragments one MFMA step ahead: 4 ds_read_b128 in flight behind
            // each group of 4 MFMAs (the scheduler would otherwise serialise
            // read -> wait -> MFMA and expose the LDS latency every MFMA)
            bf16x8 b[2][NCT];
#pragma unroll
            for (int t = 0; t < NCT; ++t) {
                const int br = 32 * t + cl;
                b[0][t] = *reinterpret_cast<const bf16x8 *>(&sm.B[cur][br][8 * bswz(br, 4 * h)]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j < 3) {
#pragma unroll
                    for (int t = 0; t < NCT; ++t) {
                        const int br = 32 * t + cl;
                        b[(j + 1) & 1][t] = *reinterpret_cast<const bf16x8 *>(
                            &sm.B[cur][br][8 * bswz(br, 4 * h + j + 1)]);
                    }
                }
#pragma unroll
                for (int t = 0; t < NCT; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[j], b[j & 1][t], acc[t], 0, 0, 0);
            }
            // issue pattern: 4 reads, then per step {4 reads, 4 MFMAs}, last 4 MFMAs
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            cur = cur == NSLOT - 1 ? 0 : cur + 1;
            ++g;
        };
        for (int kt = 0; kt < nk; kt += 4) {
            step(a0, a3, kt);
            step(a1, a0, kt + 1);
            step(a2, a1, kt + 2);
            step(a3, a2, kt + 3);
        }
        __syncthreads();  // cinv[par] written by other waves
        if constexpr (PROBE == 1) {
            // timing probe (MN_BF16_PROBE=noepi): K loop only, results discarded
            float sacc = 0.f;
#pragma unroll
            for (int t = 0; t < NCT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) sacc += acc[t][r];
            if (sacc == 12345.678f) sm.ovf[0] = 1;
            continue;
        }
        // ---- epilogue: key = -cos~, filter, queue, merge (32 rows per wave) ----
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
        ec.cap = cap;
        ec.buf = buf;
        // lane id re-materialised per block: keeps the compiler from hoisting
        // every epilogue address out of the tile loop (register pressure)
#define MN_EPI(M, T)                                                                       \
    {                                                                                      \
        int lo = lane, wo = w;                                                             \
        asm volatile("" : "+v"(lo), "+s"(wo));                                             \
        epilogue_block<T, PROBE>(sm, ec, acc[T], lo, wo, rg);                                     \
    }
        MN_EPI(0, 0) MN_EPI(0, 1) MN_EPI(0, 2) MN_EPI(0, 3)
#undef MN_EPI
        // the epilogue's list stores must not satisfy the next counted vmcnt
        // ahead of an older load: drain them here (once per tile)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (int rr = 0; rr < WR; ++rr) {
        const int c = __builtin_amdgcn_readlane(rg.cnt, rr);
        if (c > 0) update_row(sm, WR * w + rr, c, L);
    }
    if (lane < WR) {
        const int row = WR * w + lane;
        const int64_t q = q0 + row;
        if (q < nq) {
            // buffer overflow or unusable keys: the row is rescanned exactly
            const bool forced = sm.ovf[row] || rg.gcnt > cap;
            out_cnt[q * S + sl] = min(rg.gcnt, cap);
            out_tau[q * S + sl] = forced ? -__builtin_inff() : sm.tau[row];
        }
    }
}

// ---- exact re-rank / certification / filter --------------------------------------
// The reference's `acc + a * b` in f64: a bf16 x bf16 product is exact in f64
// (8 + 8 significant bits), so one fused multiply-add rounds identically.
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
                acc = __builtin_fma(bf2d((uint16_t)(wa[u] & 0xFFFFu)),
                                    bf2d((uint16_t)(wb[u] & 0xFFFFu)), acc);
                acc = __builtin_fma(bf2d((uint16_t)(wa[u] >> 16)), bf2d((uint16_t)(wb[u] >> 16)),
                                    acc);
            }
        }
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
    const double pw = p == 2.0 ? x * x : (p == 1.0 ? x : pow(x, p));
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

static int getenv_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
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
    const int64_t blocks_q = (nq + BM - 1) / BM;
    // corpus slices: enough blocks to fill the chip, and at least kMinSlices
    // so the co-scheduled slices of one query block share its query panel in
    // the XCD's L2 (each block re-reads it once per corpus tile)
    const int64_t kMinSlices = (int64_t)getenv_int("MN_BF16_MIN_SLICES", 2);
    int64_t S = std::max<int64_t>(kMinSlices, (512 + blocks_q - 1) / blocks_q);
    S = std::min<int64_t>(S, 256 / L);
    S = std::min<int64_t>(S, std::max<int64_t>(1, (nc + BN - 1) / BN));
    S = std::max<int64_t>(S, 1);
    int64_t chunk = (nc + S - 1) / S;
    chunk = std::max<int64_t>(BN, ((chunk + BN - 1) / BN) * BN);
    S = std::max<int64_t>(1, (nc + chunk - 1) / chunk);
    // candidates re-ranked per query: S slices x (L + ties); room for 2x
    const int SL = (int)(S * L);
    const int NR = SL <= 32 ? 1 : (SL <= 64 ? 2 : (SL <= 128 ? 4 : 8));
    t_bf16_stats.slices = (int)S;
    t_bf16_stats.list_len = L;
    // HBM candidate buffer per (query, slice): a sweep over m columns keeping
    // the L best writes about L (1 + ln(m / L)) pairs (plus queue lag); cap is
    // 1.5x that plus slack, rows that overflow are rescanned exactly
    const double expect = L * (1.0 + std::log(std::max(1.0, (double)chunk / L)));
    int cap = (int)((1.5 * expect + 2 * QCAP + 64 + 63) / 64) * 64;
    cap = (int)std::min<int64_t>(cap, std::max<int64_t>(64, (chunk + 63) / 64 * 64));

    char *g = (char *)scratch(kSlotNorms, (size_t)(nq + nc) * 12 + 256);
    uint2 *cbuf = (uint2 *)scratch(kSlotLists, (size_t)nq * S * cap * sizeof(uint2) + 64);
    char *meta = (char *)scratch(kSlotListMeta, (size_t)nq * S * 8 + 64);
    int *fb_list = (int *)scratch(kSlotFallback, sizeof(int) * (size_t)nq + 64);
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
    if (nc > 0) {
        const char *probe = getenv("MN_BF16_PROBE");
        auto kern = !probe ? k_gram_bf16<0>
                    : !strcmp(probe, "noepi") ? k_gram_bf16<1>
                    : !strcmp(probe, "filteronly") ? k_gram_bf16<2>
                    : !strcmp(probe, "nomerge") ? k_gram_bf16<3> : k_gram_bf16<0>;
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
