// gram_bf16.hpp — candidate generation on v_mfma_f32_32x32x16_bf16, shared by
// the two kNN paths that feed it bf16 operands:
//
//   GM_COS  (knn_bf16.hip, C5)  rows are the bf16 items themselves; key =
//           -cos~ = -(dot~ * inv|q|) * inv|c| (one MFMA per 16 features).
//   GM_L2   (knn_f32.hip, C2/C4) rows are f32 vectors split exactly-ish into
//           two bf16 terms x = hi + lo + e (|e| <= 2^-16|x|), stored per 32-feature
//           group as [hi 32 | lo 32]; the dot is hi.hi + hi.lo + lo.hi (three MFMAs
//           per 16 features, products exact in f32, f32 accumulate) and
//           key = d~ = |q|^2 + |c|^2 - 2 dot~.  The dropped lo.lo term and the
//           split residuals are <= 3 2^-16 sum|q_t c_t|, inside the certification
//           bound of the exact re-rank (knn_f32.hip) — outputs stay bit-exact.
//
// Both are approximate FILTERS only: every row is re-ranked with the
// reference arithmetic and certified (or rescanned) afterwards.
//
// Structure (one block = 256 queries x one corpus slice, 8 waves x 32 rows):
//   * query fragments go straight from HBM/L2 into registers (asm loads, three
//     stages ahead), the 128-row corpus tile is staged by LDS-DMA into a 3-slot
//     ring (two stages in flight) shared by the 8 waves;
//   * per 32x32 accumulator block the epilogue filters key < tau(row) (the
//     row's L-th best key so far); survivors go straight to a per-(row, slice)
//     HBM buffer (write-only during the sweep) and their keys to an LDS queue;
//     a queue that could overflow is merged into the row's sorted L best keys
//     (LDS only) and tau drops.
#pragma once
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>

#include "common.hpp"

namespace mn {
namespace kb16 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// GM_L2H: L2 key on the single-bf16 rows (hi = bf16(x) only, one MFMA per 16
// features, the GM_COS row layout) — the sample phase of the two-phase L2
// generator (knn_f32.hip), certified with the residual-norm bound there.
enum GramMode { GM_COS = 0, GM_L2 = 1, GM_L2H = 2 };

constexpr int BM = 256;           // queries per block (8 waves x 32 rows)
constexpr int BN = 128;           // corpus rows per tile (4 column blocks of 32)
constexpr int BK = 64;            // bf16 elements per stage (128-B rows)
constexpr int DALIGN = 4 * BK;    // row length (bf16 elements) is padded to a multiple of this
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
// LDS keeps only keys — the row's L smallest so far (lk, sorted) and the keys
// queued since the last threshold update (qk) — so an update never reads HBM.
struct alignas(16) Smem {
    uint16_t B[NSLOT][BN][BK];
    float lk[BM][LMAX];
    float qk[BM][QCAP];
    float caux[2][BN];  // GM_COS: 1/|c|   GM_L2/GM_L2H: |c|^2
    float qaux[BM];     // GM_COS: 1/|q|   GM_L2/GM_L2H: |q|^2
    float tau[BM];
    int lsz[BM];
    int ovf[BM];
};

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

// B image: logical 16-B chunk c of tile row r sits at physical chunk
// c ^ ((r >> 1) & 7): any fixed logical chunk read by 32 consecutive rows is a
// conflict-free ds_read_b128 (each 16-lane group covers all 16 (r&1, p) banks).
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
// keeps the aux value and the threshold of its 16 rows; lane l < 32 keeps the
// queue count and the HBM buffer count of row l.  Thresholds only change in
// updates, after which they are re-read: the common path has no LDS round trip.
struct RowRegs {
    float qa[16];
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
template <int MODE, int T, int PROBE>
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
    const float ca = sm.caux[ec.par][colr];
    const int gcol = ec.gc0 + colr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int lrow = base + rl;
        const float qa = rg.qa[r];
        const bool valid = colok && lrow < ec.qlim && (lrow - colr) != ec.dx;
        float key;
        bool bad;
        if constexpr (MODE == GM_COS) {
            // n_q n_c near the reference's denom > 1e-12 switch: the
            // approximation cannot tell cos from 0, so the pair becomes a forced
            // candidate (key below every real key) and the exact re-rank
            // decides.  Exactly-zero norms give key = -0 = exact.
            key = (qa * ca > 5e11f) ? -2.f : -(v[r] * qa) * ca;  // -cos~
            bad = valid && !(__builtin_fabsf(key) <= 2.f);
        } else {
            // d~ = |q|^2 + |c|^2 - 2 dot~; NaN / +inf (overflow, or a split
            // term that rounded to inf) voids the threshold argument for the
            // row: it is rescanned exactly
            key = __builtin_fmaf(-2.f, v[r], qa + ca);
            bad = valid && !(key < __builtin_inff());
        }
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

// Q [nq][d], C [nc][d] bf16 (d = elements per row, a multiple of DALIGN; for
// GM_L2 the split layout, 2 elements per feature).  qaux/caux per row: see
// Smem.  Outputs per (query, slice): out_cnt = pairs written to buf (capped),
// out_tau = the slice's L-th best key (+inf if never filled, -inf if the row
// must be rescanned exactly).
template <int MODE, int PROBE>
__global__ __launch_bounds__(NT) void k_gram_bf16(
    const uint16_t *__restrict__ Q, int64_t nq, const uint16_t *__restrict__ C, int64_t nc, int d,
    int64_t q_off, int64_t c_off, int excl, const float *__restrict__ qaux,
    const float *__restrict__ caux, int L, int S, int64_t chunk, int cap, uint2 *__restrict__ buf,
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
        sm.qaux[r] = (q0 + r < nq) ? qaux[q0 + r] : 0.f;
        sm.tau[r] = __builtin_inff();
        sm.lsz[r] = 0;
        sm.ovf[r] = 0;
    }
    __syncthreads();
    const int nk = d / BK;  // a multiple of 4 (d is a multiple of DALIGN)
    // this lane's query row (clamped: rows past nq are masked in the epilogue).
    // GM_COS / GM_L2H: step j, lane half h covers elements 32h + 8j .. +7 of the stage
    // (the dot is order-free), so a lane's four fragments are one 64-B run.
    // GM_L2: stage = features 32s..32s+31 as [hi 32 | lo 32]; step j covers
    // features 16j + 8h .. +7: fragments hi(j=0), hi(j=1), lo(j=0), lo(j=1) =
    // 16-B chunks h, 2+h, 4+h, 6+h.
    const uint16_t *arow =
        Q + min(q0 + WR * w + cl, nq - 1) * (int64_t)d + (MODE != GM_L2 ? 32 * h : 8 * h);
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
        if constexpr (MODE != GM_L2)
            asm volatile("global_load_dwordx4 %0, %4, off\n\t"
                         "global_load_dwordx4 %1, %4, off offset:16\n\t"
                         "global_load_dwordx4 %2, %4, off offset:32\n\t"
                         "global_load_dwordx4 %3, %4, off offset:48"
                         : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3])
                         : "v"(p)
                         : "memory");
        else
            asm volatile("global_load_dwordx4 %0, %4, off\n\t"
                         "global_load_dwordx4 %1, %4, off offset:32\n\t"
                         "global_load_dwordx4 %2, %4, off offset:64\n\t"
                         "global_load_dwordx4 %3, %4, off offset:96"
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
    load_row_vals(sm.qaux, WR * w, h, rg.qa);
#pragma unroll
    for (int r = 0; r < 16; ++r) rg.tau[r] = __builtin_inff();
    rg.cnt = 0;
    rg.gcnt = 0;
    int64_t g = 0;
    int cur = 0;  // LDS slot of the stage being consumed
    int par = 0;
    for (int64_t c0 = cbeg; c0 < cend; c0 += BN, par ^= 1) {
        if (tid < BN) sm.caux[par][tid] = (c0 + tid < cend) ? caux[c0 + tid] : 0.f;
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
            if constexpr (MODE != GM_L2) {
                // B fragments one MFMA step ahead: 4 ds_read_b128 in flight
                // behind each group of 4 MFMAs (the scheduler would otherwise
                // serialise read -> wait -> MFMA and expose the LDS latency)
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
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[j], b[j & 1][t], acc[t],
                                                                         0, 0, 0);
                }
                // issue pattern: 4 reads, then per step {4 reads, 4 MFMAs}, last 4 MFMAs
                __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            } else {
                // two 16-feature steps x 4 column blocks = 8 (step, block)
                // pairs, each hi.hi, hi.lo, lo.hi; the pair's two fragments are
                // read one pair ahead (16 VGPRs of B in flight)
                bf16x8 bh[2], bl[2];
                auto rd = [&](int pi, int slot) {
                    const int j = pi >> 2, br = 32 * (pi & 3) + cl;
                    bh[slot] = *reinterpret_cast<const bf16x8 *>(
                        &sm.B[cur][br][8 * bswz(br, 2 * j + h)]);
                    bl[slot] = *reinterpret_cast<const bf16x8 *>(
                        &sm.B[cur][br][8 * bswz(br, 4 + 2 * j + h)]);
                };
                rd(0, 0);
#pragma unroll
                for (int pi = 0; pi < 2 * NCT; ++pi) {
                    if (pi + 1 < 2 * NCT) rd(pi + 1, (pi + 1) & 1);
                    const int j = pi >> 2, t = pi & 3, sb = pi & 1;
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[j], bh[sb], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[j], bl[sb], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[2 + j], bh[sb], acc[t], 0,
                                                                     0, 0);
                }
                // issue pattern: 2 reads, then per pair {2 reads (next), 3 MFMAs}
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
                for (int pi = 0; pi < 2 * NCT - 1; ++pi) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
            }
            cur = cur == NSLOT - 1 ? 0 : cur + 1;
            ++g;
        };
        for (int kt = 0; kt < nk; kt += 4) {
            step(a0, a3, kt);
            step(a1, a0, kt + 1);
            step(a2, a1, kt + 2);
            step(a3, a2, kt + 3);
        }
        __syncthreads();  // caux[par] written by other waves
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
        // ---- epilogue: key, filter, queue, merge (32 rows per wave) ----
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
#define MN_EPI(T)                                                                          \
    {                                                                                      \
        int lo = lane, wo = w;                                                             \
        asm volatile("" : "+v"(lo), "+s"(wo));                                             \
        epilogue_block<MODE, T, PROBE>(sm, ec, acc[T], lo, wo, rg);                        \
    }
        MN_EPI(0) MN_EPI(1) MN_EPI(2) MN_EPI(3)
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

// Corpus slicing + candidate-buffer sizing shared by the drivers.
struct GramPlan {
    int64_t S, chunk;
    int cap, NR;
};

// max_slices > 0 caps S (the two-phase generators' sample pass: their
// threshold is the L-th best of the WHOLE sample only with one slice; with S
// slices it is the best of S per-slice L-th bests, about S x more candidates)
inline GramPlan plan_gram(int64_t nq, int64_t nc, int L, int64_t min_slices,
                          int64_t max_slices = 0) {
    GramPlan p;
    const int64_t blocks_q = (nq + BM - 1) / BM;
    // corpus slices: enough blocks to fill the chip, and at least min_slices
    // so the co-scheduled slices of one query block share its query panel in
    // the XCD's L2 (each block re-reads it once per corpus tile)
    int64_t S = std::max<int64_t>(min_slices, (512 + blocks_q - 1) / blocks_q);
    // S * L bounds the re-rank width (8 registers x 64 lanes); 256 leaves room
    // for 2x (ties, queue lag); MN_GRAM_MAX_SL overrides it (experiments)
    const char *msl = knob("MN_GRAM_MAX_SL");
    const int64_t max_sl = (msl && *msl) ? std::min(480, std::max(64, atoi(msl))) : 256;
    S = std::min<int64_t>(S, std::max<int64_t>(1, max_sl / L));
    S = std::min<int64_t>(S, std::max<int64_t>(1, (nc + BN - 1) / BN));
    if (max_slices > 0) S = std::min(S, max_slices);
    S = std::max<int64_t>(S, 1);
    int64_t chunk = (nc + S - 1) / S;
    chunk = std::max<int64_t>(BN, ((chunk + BN - 1) / BN) * BN);
    S = std::max<int64_t>(1, (nc + chunk - 1) / chunk);
    p.S = S;
    p.chunk = chunk;
    // candidates re-ranked per query: S slices x (L + ties); room for 2x
    const int SL = (int)(S * L);
    p.NR = SL <= 32 ? 1 : (SL <= 64 ? 2 : (SL <= 128 ? 4 : 8));
    // HBM candidate buffer per (query, slice): a sweep over m columns keeping
    // the L best writes about L (1 + ln(m / L)) pairs (plus queue lag); cap is
    // 1.5x that plus slack, rows that overflow are rescanned exactly
    const double expect = L * (1.0 + std::log(std::max(1.0, (double)chunk / L)));
    int cap = (int)((1.5 * expect + 2 * QCAP + 64 + 63) / 64) * 64;
    cap = (int)std::min<int64_t>(cap, std::max<int64_t>(64, (chunk + 63) / 64 * 64));
    p.cap = cap;
    return p;
}

}  // namespace kb16
}  // namespace mn
