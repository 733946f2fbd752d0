// gram_sweep2.hpp — phase 2 of the two-phase L2 candidate generator
// (MN_KNN_BF16X1), second generation: the same contract as gram_sweep.hpp
// (fixed per-query threshold folded into the accumulator, a pair is a
// candidate iff acc = tq(q) - hc(c) + qh.ch > 0, buffered per (query, slice)),
// re-scheduled for gfx950's MFMA pipe:
//
//  * v_mfma_f32_16x16x32_bf16 (the chip holds a higher clock on this shape
//    than on 32x32x16 for the same FLOPs: MI355X_MICROARCH.md 'DVFS give-back'
//    item 7), 256-query x 256-row block tile, each wave 64 queries x 128 rows
//    = 4 x 8 fragments, 128 accumulator VGPRs.
//  * Ping-pong: the two waves that share a SIMD (w and w+4) run one barrier
//    window apart.  In every window one of them issues its 32 MFMAs (one
//    32-deep k-step) while the other reads the next k-step's 12 fragments
//    from LDS and issues its LDS-DMA pieces, so the MFMA pipe never waits on
//    LDS latency or on the barrier itself.
//  * 4-slot LDS ring of 32-deep k-steps (both operands, 32 KB per slot), each
//    k-step issued 3 ahead by LDS-DMA (`buffer_load_dwordx4 ... lds`): a k-step
//    is read 6 windows after its DMA was issued; counted `vmcnt(8)` (never 0
//    in the loop), raw `s_barrier`.
//  * One KB32 row is 64 B (4 chunks of 16 B); a 16x16x32 fragment read is 16
//    rows x 4 chunks.  Chunk c of row r sits at c ^ (((r >> 3) & 1) << 1):
//    every ds_read_b128 lane group covers all 16 slots of a 256-B bank row
//    (conflict-free); the DMA writes lane-linear and the swizzle is applied to
//    its source address.
//  * The next tile's |c|^2/2 values come in by waves 0-3's dword loads issued
//    4 k-steps before the tile ends (older than the counted window, so the
//    regular waits retire it) and are written to LDS 2 k-steps before use.
//  * The per-tile epilogue (max3 tree + ballot over the 128 accumulators, the
//    rare candidate staging, the next tile's accumulator init) runs in the
//    wave's READ window, beside its partner's MFMAs.
#pragma once
#include <algorithm>
#include <array>
#include <climits>
#include <type_traits>
#include <vector>

#include "common.hpp"

namespace mn {
namespace ksw2 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int BQ = 256;      // queries per block
constexpr int BC = 256;      // corpus rows per tile
constexpr int KB = 32;       // bf16 per k-step (one KB32 block)
constexpr int NWAVES = 8;
constexpr int NT = 64 * NWAVES;
constexpr int NSLOT = 4;     // LDS ring of k-steps
constexpr int WQF = 4;       // 16-query fragments per wave
constexpr int WCF = 8;       // 16-row corpus fragments per wave
constexpr int SCAP = 224;    // staged candidates per wave
constexpr uint32_t kSkip = 0xffffffffu;  // a reserved staging slot left empty

// the LDS-DMA ring is its own LDS object: the compiler's wait insertion then
// knows the DMA never writes the per-tile arrays below (one shared object made
// it drain every DMA in flight before each tile's accumulator init)
struct alignas(16) Ring {
    uint16_t C[NSLOT][BC][KB];   // corpus k-step, 16 KB per slot
    uint16_t Q[NSLOT][BQ][KB];   // query k-step, 16 KB per slot
};
struct alignas(16) Smem {
    float hc[2][BC];             // |c|^2 / 2 of a tile (+inf past the slice end)
    float tc[2][BC];             // SW_SYM: tau0 of a tile's rows (off-diagonal keys)
    union {
        int qcnt[BQ];            // candidates written per query of the block
        float ta[BQ];            // SW_SYM: -|q|^2 / 2 (off-diagonal tiles)
    };
    float t0[BQ];                // tau0 of the block's queries
    float tq[BQ];                // (tau0 - |q|^2) / 2 of the block's queries
    float sq[BQ];                // F16: the queries' scales 2^e
    float sc[2][BC];             // F16: a tile's rows' scales 2^e
    int scnt[NWAVES];            // staged entries per wave
    uint2 stk[NWAVES][SCAP];     // staged candidates per wave: (key bits, global id)
    uint32_t stp[NWAVES][SCAP];  //   and (query in block | buffer position << 8)
};
static_assert(sizeof(Smem) + sizeof(Ring) <= 163840, "LDS budget");

__device__ __forceinline__ int swz(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }

// byte address of an LDS object (for inline-asm ds_* operands)
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// vmcnt waits with an immediate count
#define MN_VMCNT(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

// Qk [nkb][nq][32], Ck [nkb][nc][32] (KB32 bf16).  Corpus rows [c_begin, nc)
// in S slices of `chunk` rows (a multiple of BC).  tq / tau0 [nq], hc [nc].
// Per (query, slice): buf[(q*S + s)*cap + i] = (key bits, global corpus id),
// cnt[q*S + s] = entries (-1: overflow).  PROBE = 1: K loop only (timing);
// diagnostics (results invalid): PROBE = 2 also without the in-loop LDS-DMA
// issue, PROBE = 3 also without the fragment reads, PROBE = 4 with the DMA
// issued but never waited for.
// MODE = SW_COS (C5, knn_bf16.hip): hc holds -|c| and tq = t(q) |q| (t the
// cosine threshold): acc0 = tq * hc, so acc = q.c - t |q||c| and a pair is a
// candidate iff q.c / (|q||c|) > t; rows past the slice end are padded with
// NaN (never positive); key = -acc / |c| (the re-rank maps it back to cos).
// A tile's epilogue (candidate check + next accumulator init) runs in the
// wave's read window (fusing the init into the first MFMA window, or one
// ballot per 2 or 4 fragments before the per-fragment ones, measured equal
// within noise at C2).
enum SweepMode { SW_L2 = 0, SW_COS = 1, SW_SYM = 2, SW_COS_SYM = 3 };

// SW_COS_SYM (the C5 self item graph, X both operands, rows in DESCENDING
// cosine-threshold order t): SW_SYM's block table and per-row buffers with
// SW_COS's product-form accumulator.  Diagonal tile: acc0 = tq(q) hc(c) with
// tq = t(q)|q|, hc = -|c| (the row's own test, key = -acc / |c|, as SW_COS).
// Off-diagonal tile (J > I, so t(c) <= t(q)): acc0 = ta(q) hoff(c) with ta =
// |q|, hoff = -t(c)|c|: acc > 0 iff cos~ > t(c), the column's test; its key
// -acc / |q| (the re-rank maps key / |c| - t(c) = -cos~); row q's own key
// k_q = (-acc + hoff(c) ta(q)) / |c| + tq(q) (= -acc_q / |c|, acc_q = acc +
// (t(c) - t(q)) |q||c|), buffered when k_q < 0.  tau0 carries |c| per
// position (sm.tc).

// SW_SYM (self kNN, X both operands, rows in ascending-tau0 order): the
// sweep covers each unordered pair once.  Block b takes row block I = tab[b].x
// against the tab[b].z column tiles J = tab[b].y + t tab[b].w (t = 0, 1, ..),
// every J >= I (sym_block_table).  The
// diagonal tile (J == I, only ever a block's first tile) runs as SW_L2: acc0 =
// tq(q) - hc(c), a pair is row q's candidate iff acc > 0, key = tau0(q) -
// 2 acc.  An off-diagonal tile (J > I, so tau0(c) >= tau0(q): sorted order)
// folds the COLUMN's threshold: acc0 = aoff(q) - hoff(c) with aoff = -|q|^2/2,
// hoff = (|c|^2 - tau0(c)) / 2, so acc > 0 iff key = tau0(c) - 2 acc < tau0(c),
// the test of row c; row q's own test key < tau0(q) <= tau0(c) implies it and
// is checked only on those hits.  Both rows' candidates go to per-ROW
// buffers buf[row][cap] through global counters cnt[row] (returned atomics at
// the flush of the per-wave LDS staging area; counts past cap mean overflow).
struct SymArgs {
    const int4 *tab;     // per block: (I, Jfirst, tiles, tile stride) in 256-row blocks
    const float *aoff;   // [n] off-diagonal fold, row side
    const float *hoff;   // [n] off-diagonal fold, column side
    const float *scale;  // F16: [n] 2^e of each row's fp16 copy (x 2^e, per-row e)
};
// F16 (fp16 operands with per-row exponents, knn_f32.hip k_prep_f16r /
// k_sym_pos): the folds carry the per-pair certification bound and are
// scaled by the row's own 2^e, so acc0 = A(q) s_c + B(c) s_q (diagonal: A = tq,
// B = hc; off-diagonal: A = aoff, B = hoff) and a hit's key is
// Teff - 2 acc / (s_q s_c) (tau0 carries Teff); padding folds are -inf.

// TM (tile-major layout): element (row r, feature e) of Qk / Ck at
// ((r / 256) pst + e / 32) * 8192 + (r % 256) * 32 + e % 32 (pst >= nkb: the
// panel stride in k-steps, padded so panels do not alias), rows padded to a
// multiple of 256 (allocated; never candidates): a block's k-steps are then
// consecutive 16-KB pieces of one contiguous 256-row panel instead of pieces
// n * 64 B apart (one page per k-step and operand), and c_begin / chunk must
// be multiples of BC.
// F16: the operands are fp16 copies of x 2^e (one v_mfma_f32_16x16x32_f16 per
// 32 features: the same rate as bf16, 11 significant bits instead of 8, so the
// residual-norm bound is ~8x tighter); SW_SYM only.
// V (schedule variant, tuning A/B): 0 = each wave issues its LDS-DMA pieces
// at the start of its read window; 1 = interleaved with its MFMAs (one piece
// after every 8), so the read window holds only the fragment reads; 2 = in
// the read window AFTER the fragment reads (the reads go to the LDS pipe
// while the DMA issue waits on the CU's shared texture-address unit); 3 = two
// pieces after the reads, two between the MFMA rows.
// Default 14 (placement 2, builtin DMA, plain fragment reads): C2 same
// process 752.6 ms vs 754.4 (asm reads), 763.1 (asm DMA + reads), 766.3 (asm
// DMA), round 4's build 757.8; placement 0 / 1 / 3 774 / 827 / 777 (with the
// asm forms; profiles/r05/r05_ab_*.log).  The asm forms keep the compiler
// from draining the DMA before LDS accesses, but cost more than they save.
template <int PROBE, int MODE = SW_L2, bool TM = false, bool F16 = false, int V = 14>
__global__ __launch_bounds__(NT) void k_gram_sweep2(
    const uint16_t *__restrict__ Qk, int64_t nq, const uint16_t *__restrict__ Ck, int64_t nc,
    int nkb, int64_t q_off, int64_t c_off, int excl, const float *__restrict__ tq,
    const float *__restrict__ tau0, const float *__restrict__ hc, int64_t c_begin, int S,
    int64_t chunk, int cap, uint2 *__restrict__ buf, int *__restrict__ cnt, int pst = 0,
    SymArgs sym = SymArgs{}) {
    // PROBE 5 / 6 (tuning build, results invalid): every block's rows read
    // from panel 0 and its column tiles from panel 1 (L2-resident), with /
    // without the epilogue — the kernel's own ceiling without fabric traffic
    constexpr bool L2RES = PROBE == 5 || PROBE == 6;
    // V bits: 0..1 the DMA placement; 4: the LDS-DMA through the compiler
    // builtin instead of inline asm; 8: the fragment reads as plain loads
    constexpr int VP = V & 3;
    constexpr bool ASM_DMA = !(V & 4), ASM_READ = !(V & 8);
    constexpr bool EPI = PROBE == 0 || PROBE == 5;
    constexpr bool SYM = MODE == SW_SYM || MODE == SW_COS_SYM;
    constexpr bool COSM = MODE == SW_COS || MODE == SW_COS_SYM;  // product-form acc0, NaN pads
    __shared__ Ring rg;
    __shared__ Smem sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wq = w & 3, wc = w >> 2;  // wc: ping-pong group (0 leads by one window)
    const int fr = lane & 15, fk = lane >> 4;
    const int v = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    // (32-bit row / step counters: nq * 32, nc * 32 < 2^31 is checked by the driver)
    // Tiles start at cbeg, cbeg + cstr, ... (ntile of them); rows >= cend are
    // padding (the slice end; SW_SYM: the corpus end)
    int q0, sl, cbeg, cend, cstr, ntile;
    if constexpr (SYM) {
        const int4 e = sym.tab[v];
        q0 = e.x * BQ;
        sl = 0;
        cbeg = e.y * BC;
        cend = (int)nc;
        ntile = e.z;
        cstr = e.w * BC;
    } else {
        q0 = (v / S) * BQ;
        sl = v % S;
        cbeg = (int)(c_begin + (int64_t)sl * chunk);
        cend = (int)min(nc, (int64_t)cbeg + chunk);
        ntile = cend > cbeg ? (cend - cbeg + BC - 1) / BC : 0;
        cstr = BC;
    }
    const int gtot = ntile * nkb;
    // padding rows never qualify: acc0 = -inf (COS: NaN, as -inf * -|c| = +inf;
    // F16 adds the column fold: -inf)
    const float pad = COSM ? __builtin_nanf("") : (F16 ? -__builtin_inff() : __builtin_inff());
    const bool diag0 = SYM && cbeg == q0;  // SW_SYM: the first tile is the diagonal one

    if (tid < NWAVES) sm.scnt[tid] = 0;
    if (tid < BQ) {
        // padded queries never qualify (COS: NaN, as -inf * -|c| would be +inf)
        sm.tq[tid] = q0 + tid < nq ? tq[q0 + tid] : (COSM ? pad : -__builtin_inff());
        sm.t0[tid] = q0 + tid < nq ? tau0[q0 + tid] : 0.f;
        if constexpr (SYM) sm.ta[tid] = q0 + tid < nq ? sym.aoff[q0 + tid] : (COSM ? pad : -__builtin_inff());
        else sm.qcnt[tid] = 0;
        if constexpr (F16) sm.sq[tid] = q0 + tid < nq ? sym.scale[q0 + tid] : 1.f;
    }
    if (ntile > 0 && tid < BC) {
        const int c = cbeg + tid;
        if constexpr (SYM) {
            sm.hc[0][tid] = (c < cend) ? (diag0 ? hc[c] : sym.hoff[c]) : pad;
            sm.tc[0][tid] = (c < cend) ? tau0[c] : pad;
            if constexpr (F16) sm.sc[0][tid] = (c < cend) ? sym.scale[c] : 1.f;
        } else {
            sm.hc[0][tid] = (c < cend) ? hc[c] : pad;
        }
    }

    // ---- LDS-DMA issue state: the next k-step gi to stage (tile row bt0,
    // k-block bkb).  Each wave stages rows [32w, 32w+32) of both operands:
    // two 16-row pieces each, lane l -> row +(l>>2), physical chunk l&3.
    int bt0 = cbeg, bti = 0;  // tile start row / index being staged
    int bkb = 0, bslot = 0;
    const int prow0 = 32 * w + (lane >> 2), prow1 = prow0 + 16;
    const int pch = 8 * ((lane & 3) ^ (((lane >> 5) & 1) << 1));  // source chunk (swizzle)
    const int qo0 = TM ? prow0 * KB + pch : min(q0 + prow0, (int)nq - 1) * KB + pch;
    const int qo1 = TM ? prow1 * KB + pch : min(q0 + prow1, (int)nq - 1) * KB + pch;
    const int co0 = TM ? prow0 * KB + pch : min(bt0 + prow0, cend - 1) * KB + pch;
    const int co1 = TM ? prow1 * KB + pch : min(bt0 + prow1, cend - 1) * KB + pch;
    const int64_t panel = (int64_t)pst * BC * KB;  // TM: elements between 256-row panels
    const uint16_t *const qpan = TM ? Qk + (int64_t)(L2RES ? 0 : q0 / BQ) * panel : Qk;
    auto cpan = [&](int row0) {
        return TM ? Ck + (int64_t)(L2RES ? 1 : row0 / BC) * panel : Ck;
    };
    const uint16_t *cbk = cpan(bt0), *qbk = qpan;
    const int cstep = TM ? BC * KB : (int)nc * KB, qstep = TM ? BQ * KB : (int)nq * KB;
    // LDS-DMA through buffer descriptors: one k-block region ([n][32] bf16,
    // 64-B rows) per descriptor, rebuilt from wave-uniform values per k-step
    // (SALU only); the per-lane 32-bit byte offsets (co*/qo* x 2) are fixed per
    // tile, so a piece costs no VALU address arithmetic and no VGPR reuse
    // hazard (the flat-address form serialised the four pieces on one
    // 64-bit address register)
    const int qb0 = 2 * qo0, qb1 = 2 * qo1;
    int cb0 = 2 * co0, cb1 = 2 * co1;
    // (nc * 32, nq * 32 < 2^31 is checked by the driver: the byte counts fit 32 bits)
    const int cbytes = TM ? BC * KB * 2 : (int)(uint32_t)(nc * 64);
    const int qbytes = TM ? BQ * KB * 2 : (int)(uint32_t)(nq * 64);
    // LDS-DMA as inline asm (M0 = the LDS destination, one wait state before
    // the load): the compiler does not track these, so it never drains them
    // before the epilogue's LDS accesses (it cannot tell that those do not
    // alias the ring); the ring protocol's counted waits order them instead
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    auto rsrc = [&](const uint16_t *base, int bytes) {
        const uint64_t a = (uint64_t)(uintptr_t)base;
        u32x4 r;
        r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
        r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
        r.z = (uint32_t)bytes;
        r.w = 0x00020000u;
        return r;
    };
    auto dma = [&](const u32x4 &rs, int voff, uint16_t *lds) {
        if constexpr (ASM_DMA) {
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
                         :
                         : "s"(__builtin_amdgcn_readfirstlane(lds_addr(lds))), "v"(voff), "s"(rs)
                         : "memory", "m0");
        } else {
            const uint64_t a = ((uint64_t)rs.y << 32) | rs.x;
            const __amdgpu_buffer_rsrc_t r =
                __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)a, (short)0, (int)rs.z, (int)rs.w);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)lds,
                                                     16, voff, 0, 0, 0);
        }
    };
    // piece i (0, 1: the corpus tile's rows 32w.. / 32w+16..; 2, 3: the
    // query panel's) of the next k-step to stage; advance() moves on
    auto piece = [&](int i) {
        if (i < 2) dma(rsrc(cbk, cbytes), i ? cb1 : cb0, &rg.C[bslot][32 * w + 16 * i][0]);
        else dma(rsrc(qbk, qbytes), i == 3 ? qb1 : qb0, &rg.Q[bslot][32 * w + 16 * (i - 2)][0]);
    };
    auto advance = [&]() {
        {
            bslot = (bslot + 1) & (NSLOT - 1);
            cbk += cstep;
            qbk += qstep;
            if (++bkb == nkb) {
                bkb = 0;
                bt0 += cstr;
                ++bti;
                cbk = cpan(bt0);
                qbk = qpan;
                if constexpr (!TM) {
                    cb0 = 2 * (min(bt0 + prow0, cend - 1) * KB + pch);
                    cb1 = 2 * (min(bt0 + prow1, cend - 1) * KB + pch);
                }
            }
        }
    };
    auto issue = [&]() {
        if (bti < ntile) {
            const u32x4 rc = rsrc(cbk, cbytes);
            const u32x4 rq = rsrc(qbk, qbytes);
            dma(rc, cb0, &rg.C[bslot][32 * w][0]);
            dma(rc, cb1, &rg.C[bslot][32 * w + 16][0]);
            dma(rq, qb0, &rg.Q[bslot][32 * w][0]);
            dma(rq, qb1, &rg.Q[bslot][32 * w + 16][0]);
            advance();
        }
    };

    typedef typename std::conditional<F16, f16x8, bf16x8>::type frag_t;
    f32x4 acc[WQF][WCF];
    frag_t fq[WQF], fc[WCF];
    auto init_acc = [&](int par, bool diag) {
        float tql[WQF];  // this lane's queries, one per 16-query fragment
        const float *qa = (SYM && !diag) ? sm.ta : sm.tq;
#pragma unroll
        for (int f = 0; f < WQF; ++f) tql[f] = qa[64 * wq + 16 * f + fr];
        float sql[WQF];
        if constexpr (F16) {
#pragma unroll
            for (int f = 0; f < WQF; ++f) sql[f] = sm.sq[64 * wq + 16 * f + fr];
        }
#pragma unroll
        for (int g = 0; g < WCF; ++g) {
            const float4 x =
                *reinterpret_cast<const float4 *>(&sm.hc[par][128 * wc + 16 * g + 4 * fk]);
            float4 sc4 = make_float4(1.f, 1.f, 1.f, 1.f);
            if constexpr (F16)
                sc4 = *reinterpret_cast<const float4 *>(&sm.sc[par][128 * wc + 16 * g + 4 * fk]);
#pragma unroll
            for (int f = 0; f < WQF; ++f) {
                // (hipcc packs these into v_pk_add_f32 / v_pk_mul_f32 pairs)
                if constexpr (F16) {
                    // A(q) s_c + B(c) s_q: both products exact (powers of 2),
                    // one rounding
                    acc[f][g][0] = __builtin_fmaf(tql[f], sc4.x, x.x * sql[f]);
                    acc[f][g][1] = __builtin_fmaf(tql[f], sc4.y, x.y * sql[f]);
                    acc[f][g][2] = __builtin_fmaf(tql[f], sc4.z, x.z * sql[f]);
                    acc[f][g][3] = __builtin_fmaf(tql[f], sc4.w, x.w * sql[f]);
                } else if constexpr (COSM) {
                    acc[f][g][0] = tql[f] * x.x;
                    acc[f][g][1] = tql[f] * x.y;
                    acc[f][g][2] = tql[f] * x.z;
                    acc[f][g][3] = tql[f] * x.w;
                } else {
                    acc[f][g][0] = tql[f] - x.x;
                    acc[f][g][1] = tql[f] - x.y;
                    acc[f][g][2] = tql[f] - x.z;
                    acc[f][g][3] = tql[f] - x.w;
                }
            }
        }
    };
    // fragment reads as inline asm: the compiler cannot see that the ring
    // protocol (counted vmcnt + barrier) already orders them after the
    // LDS-DMA, and would drain every DMA in flight before them
    const int chs0 = 8 * swz(fr, fk);
    const uint32_t qrd = lds_addr(&rg.Q[0][64 * wq + fr][chs0]);
    const uint32_t crd = lds_addr(&rg.C[0][128 * wc + fr][chs0]);
    auto read_frags = [&](int slot) {
        if constexpr (!ASM_READ) {
            const int chs = 8 * swz(fr, fk);
#pragma unroll
            for (int f = 0; f < WQF; ++f)
                fq[f] = *reinterpret_cast<const frag_t *>(&rg.Q[slot][64 * wq + 16 * f + fr][chs]);
#pragma unroll
            for (int g = 0; g < WCF; ++g)
                fc[g] = *reinterpret_cast<const frag_t *>(&rg.C[slot][128 * wc + 16 * g + fr][chs]);
            return;
        }
        const uint32_t qa = qrd + (uint32_t)slot * (BQ * KB * 2), ca = crd + (uint32_t)slot * (BC * KB * 2);
        asm volatile("ds_read_b128 %0, %1" : "=v"(fq[0]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(fq[1]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(fq[2]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(fq[3]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1" : "=v"(fc[0]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(fc[1]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(fc[2]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(fc[3]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(fc[4]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:5120" : "=v"(fc[5]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(fc[6]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:7168" : "=v"(fc[7]) : "v"(ca));
    };
    static_assert(WQF == 4 && WCF == 8, "read_frags: 4 query and 8 corpus fragments");
    auto mfma_row = [&](int f) {
#pragma unroll
        for (int g = 0; g < WCF; ++g)
            if constexpr (F16)
                acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fc[g], fq[f], acc[f][g], 0, 0, 0);
            else
                acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[g], fq[f], acc[f][g], 0, 0, 0);
    };
    auto mfmas = [&]() {
#pragma unroll
        for (int f = 0; f < WQF; ++f) mfma_row(f);
    };
    // V = 1: the next k-step's four pieces between the MFMA rows; V = 3: the
    // last two (the query panel's) after rows 1 and 3
    auto mfmas_dma = [&]() {
        const bool go = bti < ntile;
#pragma unroll
        for (int f = 0; f < WQF; ++f) {
            mfma_row(f);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (VP == 1) {
                if (go) piece(f);
            } else {
                if (go && (f & 1)) piece(2 + (f >> 1));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (go) advance();
    };

    bool dirty = false;  // candidate stores issued since the last counted wait
    // Stores complete out of order with the DMA loads on the VM counter, so a
    // counted wait after a store is not trusted: candidates are staged in LDS
    // (a per-wave area, slots from an LDS counter) and written out in batches
    // when the area fills; only then is the next wait a full drain.
    auto flush = [&]() {
        const int n = min(sm.scnt[w], SCAP);
        for (int e = lane; e < n; e += 64) {
            const uint32_t pq = sm.stp[w][e];
            if constexpr (SYM) {  // pq = the row; its slot from the row's counter
                const int pos = atomicAdd(&cnt[pq], 1);
                if (pos < cap) buf[(int64_t)pq * cap + pos] = sm.stk[w][e];
            } else if (pq != kSkip) {
                const int ql = (int)(pq & 255u), pos = (int)(pq >> 8);
                buf[((int64_t)(q0 + ql) * S + sl) * cap + pos] = sm.stk[w][e];
            }
        }
        sm.scnt[w] = 0;
        dirty = true;
    };
    // SW_SYM: one candidate (row, id, key) into the wave's staging area
    auto emit_sym = [&](uint32_t row, uint32_t id, float key) {
        const uint2 kv = make_uint2(__float_as_uint(key), id);
        const int e = atomicAdd(&sm.scnt[w], 1);
        if (e < SCAP) {
            sm.stk[w][e] = kv;
            sm.stp[w][e] = row;
        } else {  // area full: straight out (rare)
            const int pos = atomicAdd(&cnt[row], 1);
            if (pos < cap) buf[(int64_t)row * cap + pos] = kv;
            dirty = true;
        }
    };
    // candidates of the tile starting at corpus row ct0: positive accumulators.
    // Per 16 x 16 fragment one prefilter (the max of the four accumulators'
    // bit patterns as signed integers: positive iff some float is > 0 or a
    // +NaN, which the exact test below drops) and one ballot (wave-uniform
    // branch); the staging body runs only for fragments where some lane has
    // a candidate (a few per wave and tile at the C2 threshold).
    auto check_block = [&](int f, int g, int ct0, int hpar, bool diag) {
        const f32x4 a = acc[f][g];
        const int mi = max(max(__float_as_int(a[0]), __float_as_int(a[1])),
                           max(__float_as_int(a[2]), __float_as_int(a[3])));
        if (__builtin_expect(__ballot(mi > 0) == 0, 1)) return;
        const int ql = 64 * wq + 16 * f + fr;
        const int qgl = (int)q_off + q0 + ql;  // (global ids fit int32: the outputs are int32)
        const int c = (int)c_off + ct0 + 128 * wc + 16 * g + 4 * fk;  // id of register 0
        unsigned pm = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) pm |= a[r] > 0.f ? (1u << r) : 0u;
        if (excl && (unsigned)(qgl - c) < 4u) pm &= ~(1u << (qgl - c));
        if constexpr (SYM) {
            if constexpr (MODE == SW_COS_SYM) {
                const float tql = sm.tq[ql], tal = sm.ta[ql];
                while (pm) {
                    const int r = __builtin_ctz(pm);
                    pm &= pm - 1;
                    const int cl = 128 * wc + 16 * g + 4 * fk + r;
                    const float hcl = sm.hc[hpar][cl];
                    if (diag) {  // row q's test (SW_COS): key = -acc / |c|
                        emit_sym((uint32_t)qgl, (uint32_t)(c + r), a[r] / hcl);
                    } else {     // row c's test; row q's on these hits
                        emit_sym((uint32_t)(c + r), (uint32_t)qgl, -a[r] / tal);
                        const float kq = (hcl * tal - a[r]) / sm.tc[hpar][cl] + tql;
                        if (kq < 0.f) emit_sym((uint32_t)qgl, (uint32_t)(c + r), kq);
                    }
                }
                return;
            }
            const float t0l = sm.t0[ql];
            // F16: 2 acc / (s_q s_c) as the two divisions by powers of 2 round
            // it — two ldexp (correctly rounded) instead of two divisions
            const int eq = F16 ? 1 - __builtin_amdgcn_frexp_expf(sm.sq[ql]) : 0;
            while (pm) {
                const int r = __builtin_ctz(pm);
                pm &= pm - 1;
                const int cl = 128 * wc + 16 * g + 4 * fk + r;
                float a2 = a[r];
                if constexpr (F16) {
                    a2 = __builtin_ldexpf(a2, eq);
                    a2 = __builtin_ldexpf(a2, 1 - __builtin_amdgcn_frexp_expf(sm.sc[hpar][cl]));
                }
                a2 *= 2.f;
                if (diag) {  // row q's test, as SW_L2
                    emit_sym((uint32_t)qgl, (uint32_t)(c + r), t0l - a2);
                } else {     // row c's test (acc > 0); row q's only on these hits
                    const float key = sm.tc[hpar][cl] - a2;
                    emit_sym((uint32_t)(c + r), (uint32_t)qgl, key);
                    if (key < t0l) emit_sym((uint32_t)qgl, (uint32_t)(c + r), key);
                }
            }
            return;
        }
        if (pm != 0) {
            const int mine = __popc(pm);
            int pos = atomicAdd(&sm.qcnt[ql], mine);
            int e = atomicAdd(&sm.scnt[w], mine);
            const float t0l = sm.t0[ql];
            while (pm) {
                const int r = __builtin_ctz(pm);
                pm &= pm - 1;
                float key;
                if constexpr (MODE == SW_COS)  // hc = -|c|: key = -acc / |c|
                    key = a[r] / sm.hc[hpar][128 * wc + 16 * g + 4 * fk + r];
                else
                    key = t0l - 2.f * a[r];
                const uint2 kv = make_uint2(__float_as_uint(key), (uint32_t)(c + r));
                if (pos < cap) {
                    if (e < SCAP) {
                        sm.stk[w][e] = kv;
                        sm.stp[w][e] = (uint32_t)ql | ((uint32_t)pos << 8);
                    } else {  // area full: straight out (rare)
                        buf[((int64_t)(q0 + ql) * S + sl) * cap + pos] = kv;
                        dirty = true;
                    }
                } else if (e < SCAP) {
                    // past the row's cap (an overflow): the slot was reserved
                    // with the others; mark it empty, or the flush would write
                    // whatever an earlier entry (or another block) left there
                    sm.stp[w][e] = kSkip;
                }
                ++e;
                ++pos;
            }
        }
    };
    // candidates of the tile starting at corpus row ct0: positive accumulators
    // (hpar: the hc parity of that tile)
    auto check = [&](int ct0, int hpar, bool diag) {
        if constexpr (EPI) {
#pragma unroll
            for (int f = 0; f < WQF; ++f)
#pragma unroll
                for (int g = 0; g < WCF; ++g) check_block(f, g, ct0, hpar, diag);
            // wave-uniform: spill the area once it is 3/4 full (or overran)
            if (sm.scnt[w] >= SCAP * 3 / 4) flush();
        } else {
            float sum = 0.f;
#pragma unroll
            for (int f = 0; f < WQF; ++f)
#pragma unroll
                for (int g = 0; g < WCF; ++g) sum += acc[f][g][0];
            if (sum == 12345.678f) sm.qcnt[0] = 1;
        }
    };
    // ---- prologue: k-steps 0, 1, 2 in flight; k-step 0 landed everywhere
    issue();
    issue();
    issue();
    if (gtot > 2) MN_VMCNT(8);
    else if (gtot == 2) MN_VMCNT(4);
    else MN_VMCNT(0);
    __syncthreads();  // also publishes sm.hc[0], qcnt, t0
    if (gtot > 0) init_acc(0, diag0);
    if (wc == 1) __builtin_amdgcn_s_barrier();  // the trailing group starts one window late

    int c0 = cbeg, ti = 0;  // first corpus row / index of the current tile
    int kb = 0, par = 0;
    float hcn = 0.f, tcn = 0.f, scn = 1.f;  // next tile's hc (SW_SYM tau0, F16 scale), waves 0-3
    for (int g = 0; g < gtot; ++g) {
        // ================= READ window of k-step g =================
        const bool more = ti + 1 < ntile;
        if (wc == 0 && kb == nkb - 4 && more) {
            // the next tile's |c|^2 / 2: waves 0-3 load one value per lane
            // (asm loads: the compiler's own waits would drain the DMA queue);
            // older than the DMA issued just below, so the counted waits
            // retire them.  SW_SYM: the next tile is off-diagonal: hoff, tau0
            const int cn = min(c0 + cstr + 64 * wq + lane, (int)nc - 1);
            const float *p = SYM ? sym.hoff + cn : hc + cn;
            asm volatile("global_load_dword %0, %1, off" : "=v"(hcn) : "v"(p) : "memory");
            if constexpr (SYM) {
                const float *pt = tau0 + cn;
                asm volatile("global_load_dword %0, %1, off" : "=v"(tcn) : "v"(pt) : "memory");
            }
            if constexpr (F16) {
                const float *ps = sym.scale + cn;
                asm volatile("global_load_dword %0, %1, off" : "=v"(scn) : "v"(ps) : "memory");
            }
        }
        if constexpr (VP == 0 && (PROBE < 2 || PROBE >= 4)) issue();  // k-step g + 3
        if (kb == 0 && g > 0) {
            // the previous tile's candidates, then this tile's accumulator
            // init (before the fragment reads: the fragments are dead here)
            check(c0 - cstr, par ^ 1, diag0 && ti == 1);
            init_acc(par, false);
        }
        if constexpr (PROBE < 3 || PROBE >= 4) read_frags((int)(g & (NSLOT - 1)));
        if constexpr (PROBE < 2 || PROBE >= 4) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (VP == 2) issue();  // k-step g + 3, behind the reads
            if constexpr (VP == 3)
                if (bti < ntile) {
                    piece(0);
                    piece(1);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (kb == nkb - 2 && more && wc == 0) {
            // written 2 k-steps (>= 2 barriers) before init_acc reads it
            const int cb = c0 + cstr + 64 * wq + lane;
            sm.hc[par ^ 1][64 * wq + lane] = cb < cend ? hcn : pad;
            if constexpr (SYM) sm.tc[par ^ 1][64 * wq + lane] = cb < cend ? tcn : pad;
            if constexpr (F16) sm.sc[par ^ 1][64 * wq + lane] = cb < cend ? scn : 1.f;
        }
        // the fragments are defined here (tied operands), not at the asm reads
        if constexpr (ASM_READ)
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fq[0]), "+v"(fq[1]), "+v"(fq[2]), "+v"(fq[3]), "+v"(fc[0]),
                           "+v"(fc[1]), "+v"(fc[2]), "+v"(fc[3]), "+v"(fc[4]), "+v"(fc[5]),
                           "+v"(fc[6]), "+v"(fc[7])
                         :
                         : "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (PROBE != 4 && wc == 1) {
            // trailing group: k-step g+1 landed for the window after this one
            // (V = 1: k-step g+3 is not issued yet)
            const int rem = gtot - 1 - g;
            if (dirty) MN_VMCNT(0);
            else if ((VP == 0 || VP == 2) && rem >= 3) MN_VMCNT(8);
            else if (VP == 3 && rem >= 3) MN_VMCNT(6);  // k-step g+3: 2 of 4 pieces
            else if (rem >= 2) MN_VMCNT(4);
            else MN_VMCNT(0);
            dirty = false;
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ================= MFMA window of k-step g =================
        __builtin_amdgcn_s_setprio(1);
        if constexpr ((VP == 1 || VP == 3) && (PROBE < 2 || PROBE >= 4)) mfmas_dma();  // k-step g + 3
        else mfmas();
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (PROBE != 4 && wc == 0) {
            const int rem = gtot - 1 - g;
            if (dirty) MN_VMCNT(0);
            else if (rem >= 3) MN_VMCNT(8);
            else if (rem == 2) MN_VMCNT(4);
            else MN_VMCNT(0);
            dirty = false;
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (++kb == nkb) {
            kb = 0;
            c0 += cstr;
            ++ti;
            par ^= 1;
        }
    }
    if (wc == 0) __builtin_amdgcn_s_barrier();  // match the trailing group's extra window
    if (gtot > 0) check(c0 - cstr, par ^ 1, diag0 && ti == 1);
    if (sm.scnt[w] > 0) flush();
    if constexpr (SYM) return;  // the per-row counters are final
    __syncthreads();
    if (tid < BQ && q0 + tid < nq) {
        const int c = sm.qcnt[tid];
        cnt[(int64_t)(q0 + tid) * S + sl] = c > cap ? -1 : c;
    }
}

#undef MN_VMCNT

// Slicing + buffer sizing of the query-major sweep: nc2 = corpus rows of the
// sweep, expect = expected candidates per query.
struct SweepPlan {
    int64_t S, chunk;
    int cap;
};

inline SweepPlan plan_sweep(int64_t nq, int64_t nc2, double expect) {
    SweepPlan p;
    const int64_t nqb = (nq + BQ - 1) / BQ;
    int64_t S = std::max<int64_t>(8, (2048 + nqb - 1) / nqb);
    const char *es = knob("MN_SWEEP_S");  // tuning build: corpus slices
    if (es && *es) S = std::max(1, atoi(es));
    S = std::min<int64_t>(S, std::max<int64_t>(1, nc2 / (4 * BC)));
    S = std::max<int64_t>(S, 1);
    int64_t chunk = (nc2 + S - 1) / S;
    chunk = std::max<int64_t>(BC, (chunk + BC - 1) / BC * BC);
    S = std::max<int64_t>(1, (nc2 + chunk - 1) / chunk);
    p.S = S;
    p.chunk = chunk;
    const double per = expect / (double)S;
    const int cap = (int)((2.5 * per + 64.0 + 15.0) / 16.0) * 16;
    p.cap = std::max(cap, 64);
    return p;
}

// SW_SYM / SW_COS_SYM block table: entries (I, Jfirst, tiles, stride) = row
// block I against column tiles Jfirst + t stride, all J >= I.
//   order 1: ranges of TPB consecutive tiles aligned to a TPB grid, ordered by
//     range then row, so the co-resident blocks of an XCD stream the same
//     column tiles while their row panels come from the Infinity Cache;
//   order 0: ranges from the diagonal, the longest first;
//   order 2 (XCD groups): the 32 co-resident blocks of an XCD form a 4 x 8
//     group — row blocks I0..I0+3 x column phases c = 0..7 over a range of
//     8 TPB8 tiles (block (r, c) takes J = J0 + c + 8 t) — so in every tile
//     step the group reads 4 row panels (each shared by 8 blocks) and 8 column
//     tiles (each shared by 4) instead of 32 row panels and one column tile:
//     2.75x fewer panel reads beyond L2.  The diagonal tiles run as one-tile
//     blocks.  Groups are dealt to the XCDs so that concurrent groups on
//     different XCDs share a column range (one Infinity-Cache fill); each
//     XCD's list is padded with empty entries to a common length (the
//     kernel's xcd_remap gives XCD x the contiguous range x L .. x L + L - 1).
//   sharded (sym_block_table_share): the order-2 table of an N-row problem
//     split over `world` ranks (row-sharded build, shard.hip): the groups in
//     time order are dealt in rounds of 8 (one per XCD), each round to the
//     least-loaded rank so far, and diagonal tile I to rank (I / 8) % world, so every tile
//     runs on exactly one rank, each rank's share keeps the XCD-group
//     structure, and the full groups (equal tile counts) spread evenly.
//     world = 1 is order 2.
//   group shape gr x 32/gr (row blocks x column phases): 4 x 8 by default;
//   C2's knn_x1 uses 2 x 16 (d = 768: 754 vs 759-760 ms same process, 8 x 4
//   767-769, 16 x 2 785, 1 x 32 755-782 — profiles/r04/r04_gr_ab*.log); C5's
//   d = 3072 takes 8 x 4 since round 6 (sweep3: 2510-2524 vs 2630-2652 ms for
//   4 x 8 — profiles/r06/r06_c5_gr_scan*.log); tuning build: MN_SYM_GR
constexpr int kShareGR = 8;  // the sharded (C4) table's group rows (knn_f32.hip shard_share)
inline std::vector<int4> sym_block_table_share(int nbk, int TPB, int rank, int world, int gr = 4) {
    const int gre = knob_int("MN_SYM_GR", gr);
    const int GR = (gre == 1 || gre == 2 || gre == 8 || gre == 16) ? gre : 4, GC = 32 / GR;
    constexpr int NX = 8;
    const int T8 = std::max(1, TPB / GC);  // tiles per block
    const int W = GC * T8;                 // column range of a group
    // groups in time order: column range outer (shared across XCDs), row band
    // inner; the full groups (every block T8 tiles: they finish together, so
    // the next group starts in step) first, then the ragged ones near the
    // diagonal; group g goes to XCD g % 8
    std::vector<std::vector<int4>> full, part;
    std::vector<int> jfull, jpart;  // each group's column range (index)
    for (int J0 = 0; J0 < nbk; J0 += W) {
        for (int I0 = 0; I0 < nbk && I0 < J0 + W - 1; I0 += GR) {
            std::vector<int4> grp;
            bool all = true;
            for (int r = 0; r < GR; ++r)
                for (int c = 0; c < GC; ++c) {
                    const int I = I0 + r;
                    if (I >= nbk) { all = false; continue; }
                    // J = J0 + c + GC t with I < J < min(nbk, J0 + W)
                    const int Jend = std::min(nbk, J0 + W);
                    const int t0 = (J0 + c <= I) ? (I - (J0 + c)) / GC + 1 : 0;
                    const int Jf = J0 + c + GC * t0;
                    if (Jf >= Jend) { all = false; continue; }
                    const int cnt = (Jend - 1 - Jf) / GC + 1;
                    all = all && cnt == T8;
                    grp.push_back(make_int4(I, Jf, cnt, GC));
                }
            if (!grp.empty()) {
                (all ? full : part).push_back(grp);
                (all ? jfull : jpart).push_back(J0 / W);
            }
        }
    }
    std::vector<const std::vector<int4> *> all;
    std::vector<int> jr;
    for (auto *list : {&full, &part})
        for (auto &grp : *list) all.push_back(&grp);
    jr.insert(jr.end(), jfull.begin(), jfull.end());
    jr.insert(jr.end(), jpart.begin(), jpart.end());
    // rounds of NX groups in time order, each to the least-loaded rank so far
    // (the ragged groups near the diagonal vary in size); ties go to the first
    // rank counted from the round's column-range index, so that the same row
    // bands do not land on the same rank in every column range (the rows are
    // in threshold order, and the low-threshold rows of dense regions carry
    // more candidates: round 6 measured rank 0 at 1.18x the mean share when
    // it took rows 0-31 of every range)
    std::vector<long> load((size_t)world, 0);
    std::vector<std::vector<int4>> xl(NX);
    for (size_t g0 = 0; g0 < all.size(); g0 += NX) {
        long t = 0;
        for (size_t g = g0; g < std::min(all.size(), g0 + NX); ++g)
            for (const int4 &e : *all[g]) t += e.z;
        const int rot = jr[g0] % world;
        int dst = rot;
        for (int k = 1; k < world; ++k) {
            const int r = (rot + k) % world;
            if (load[(size_t)r] < load[(size_t)dst]) dst = r;
        }
        load[(size_t)dst] += t;
        if (dst != rank) continue;
        for (size_t g = g0; g < std::min(all.size(), g0 + NX); ++g)
            xl[g % NX].insert(xl[g % NX].end(), all[g]->begin(), all[g]->end());
    }
    // the diagonal tiles: one-tile blocks, spread over the XCDs
    for (int I = 0; I < nbk; ++I)
        if ((I / NX) % world == rank) xl[I % NX].push_back(make_int4(I, I, 1, 1));
    size_t L = 0;
    for (auto &x : xl) L = std::max(L, x.size());
    std::vector<int4> tab;
    tab.reserve(L * NX);
    for (auto &x : xl) {
        tab.insert(tab.end(), x.begin(), x.end());
        tab.insert(tab.end(), L - x.size(), make_int4(0, 0, 0, 1));
    }
    return tab;
}

inline std::vector<int4> sym_block_table(int nbk, int TPB, int order, int gr = 4) {
    if (order == 2) return sym_block_table_share(nbk, TPB, 0, 1, gr);
    std::vector<int4> tab;
    tab.reserve((size_t)nbk * ((size_t)nbk / TPB + 2) / 2 + 16);
    if (order == 1) {
        std::vector<int> key;
        for (int I = 0; I < nbk; ++I)
            for (int J0 = I; J0 < nbk;) {
                const int J1 = std::min((J0 / TPB + 1) * TPB, nbk);
                tab.push_back(make_int4(I, J0, J1 - J0, 1));
                key.push_back(J0 / TPB);
                J0 = J1;
            }
        std::vector<size_t> ord(tab.size());
        for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
            return key[a] != key[b] ? key[a] < key[b] : tab[a].x < tab[b].x;
        });
        std::vector<int4> out(tab.size());
        for (size_t i = 0; i < ord.size(); ++i) out[i] = tab[ord[i]];
        return out;
    }
    for (int I = 0; I < nbk; ++I)
        for (int J0 = I; J0 < nbk; J0 += TPB)
            tab.push_back(make_int4(I, J0, std::min(J0 + TPB, nbk) - J0, 1));
    std::stable_sort(tab.begin(), tab.end(), [](const int4 &a, const int4 &b) { return a.z > b.z; });
    return tab;
}

// The block table is a pure function of (nbk, TPB, order, group shape,
// rank, world): built once per thread and shape (the build is ~17 ms of host
// time at C2, during which the device idles) and uploaded into kSlotSymTab
// only when that slot does not already hold it.  Returns the table; *dtab the
// device copy (nullptr on an allocation failure).
inline const std::vector<int4> &sym_table_device(int nbk, int TPB, int order, int gr, int rank,
                                                 int world, hipStream_t s, int4 **dtab) {
    struct Entry {
        std::array<int, 6> key;
        std::vector<int4> tab;
    };
    thread_local std::vector<Entry> cache;
    struct Up {  // the last upload: its slot, key and stream (another stream re-uploads,
        int dev = -1;          // so no kernel can read the table ahead of its copy)
        void *p = nullptr;
        hipStream_t s = nullptr;
        std::array<int, 6> key{};
        bool valid = false;
    };
    thread_local Up last;
    // (the tuning knob MN_SYM_GR overrides the group shape inside the
    // builder: part of the key, so same-process A/Bs rebuild)
    const std::array<int, 6> key{nbk, TPB, order, knob_int("MN_SYM_GR", gr) * 64 + gr, rank, world};
    const std::vector<int4> *tp = nullptr;
    for (const Entry &e : cache)
        if (e.key == key) tp = &e.tab;
    if (!tp) {
        if (cache.size() >= 8) cache.erase(cache.begin());
        std::vector<int4> t = (order == 2 || world > 1) ? sym_block_table_share(nbk, TPB, rank, world, gr)
                                                        : sym_block_table(nbk, TPB, order, gr);
        cache.push_back(Entry{key, std::move(t)});
        tp = &cache.back().tab;
    }
    *dtab = (int4 *)scratch(kSlotSymTab, tp->size() * sizeof(int4) + 64);
    int dev = -1;
    (void)hipGetDevice(&dev);
    if (!*dtab) return *tp;
    if (!(last.valid && last.p == (void *)*dtab && last.key == key && last.dev == dev && last.s == s)) {
        if (hipMemcpyAsync(*dtab, tp->data(), tp->size() * sizeof(int4), hipMemcpyHostToDevice, s) !=
            hipSuccess) {
            last.valid = false;
            *dtab = nullptr;
            return *tp;
        }
        last = Up{dev, (void *)*dtab, s, key, true};
    }
    return *tp;
}

}  // namespace ksw2
}  // namespace mn
