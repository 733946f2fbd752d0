// gram_sweep.hpp — phase 2 of the two-phase L2 candidate generator (knn_f32.hip,
// MN_KNN_BF16X1): a plain bf16 Gram sweep with a FIXED per-query threshold.
//
// Phase 1 (gram_bf16.hpp GM_L2H on a corpus sample) gives every query a
// threshold tau0(q) — an L1-th best key of the sample, so a few hundred corpus
// rows beat it.  Phase 2 then needs no per-query top-L state at all: a pair
// (q, c) is a candidate iff its approximate key d~ = |q|^2 + |c|^2 - 2 dot~ is
// below tau0(q).  That test is folded into the accumulator itself:
//
//     acc0(q, c) = tq(q) - hc(c),   tq = (tau0 - |q|^2) / 2,   hc = |c|^2 / 2
//     acc        = acc0 + sum_t qh_t ch_t       (v_mfma_f32_32x32x16_bf16)
//     candidate  <=>  acc > 0                   (key = tau0 - 2 acc)
//
// so the per-tile epilogue is one max3 tree per 32x32 block and a branch that
// is almost never taken.  With no list state in LDS, all of it stages operands:
// a 256-query x 256-corpus block tile (the largest the register file holds at
// two waves per SIMD: 8 waves x 64 queries x 128 corpus rows, 128 accumulator
// VGPRs each) with a 4-slot LDS-DMA ring of 32-feature stages.
//
// Operand layout "KB32" (built by k_prep_x1): [dp/32][n][32] bf16, so one
// stage of 256 rows is one contiguous 16 KB run (fully coalesced DMA; one
// piece = 16 rows x 64 B, lane-linear in LDS, the swizzle applied on the
// source address).  LDS rows are 64 B, 16-B chunks swizzled c ^ ((r >> 2) & 3):
// every ds_read_b128 of a 32-row MFMA fragment is conflict-free.
//
// MFMA roles: A = corpus fragment (M = corpus rows), B = query fragment
// (N = queries), so lane l owns query column l & 31 and its 16 accumulator
// registers are 16 corpus candidates of that query (rows 8(r>>2) + 4h + (r&3)).
// Candidates go to a per-(query, slice) HBM buffer; the four lanes that hold a
// query (h = 0, 1 in the two waves of its corpus halves) take positions from
// one LDS counter per query.
#pragma once
#include <cstdlib>
#include <climits>

#include "common.hpp"

namespace mn {
namespace ksw {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BQ = 256;        // queries per block
constexpr int BC = 256;        // corpus rows per tile
constexpr int KB = 32;         // bf16 elements per stage (one KB32 block)
constexpr int NWAVES = 8;
constexpr int NT = 64 * NWAVES;
constexpr int NSLOT = 4;       // LDS ring: stage g+3 is issued while g is consumed
constexpr int WQB = 2;         // 32-query MFMA blocks per wave
constexpr int WCB = 4;         // 32-row corpus MFMA blocks per wave
constexpr int SCAP = 256;      // staged candidates per wave (flushed to HBM when full)

struct alignas(16) SwSmem {
    uint16_t C[NSLOT][BC][KB];  // corpus stage, 16 KB per slot
    uint16_t Q[NSLOT][BQ][KB];  // query stage, 16 KB per slot
    float hc[2][BC];            // |c|^2 / 2 of a tile (+inf past the slice end)
    int qcnt[BQ];               // candidates written per query of the block
    float t0[BQ];               // tau0 of the block's queries (keys of staged entries)
    uint2 stk[NWAVES][SCAP];    // staged candidates per wave: (key bits, global id)
    uint32_t stp[NWAVES][SCAP]; //   and (query in block | buffer position << 8)
};

__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 2) & 3); }

// Bijective block remap: the blocks one XCD runs together get consecutive
// virtual ids, i.e. (query block, slice) pairs that share query panels and
// corpus stages in that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Qk [nkb][nq][32], Ck [nkb][nc][32] (KB32 bf16).  Corpus rows [c_begin, nc)
// in S slices of `chunk` rows (a multiple of BC).  tq / tau0 [nq], hc [nc].
// Per (query, slice): buf[(q*S + s)*cap + i] = (key bits, global corpus id),
// cnt[q*S + s] = entries (-1: overflow).
template <int PROBE>
__global__ __launch_bounds__(NT, 2) void k_gram_sweep(
    const uint16_t *__restrict__ Qk, int64_t nq, const uint16_t *__restrict__ Ck, int64_t nc,
    int nkb, int64_t q_off, int64_t c_off, int excl, const float *__restrict__ tq,
    const float *__restrict__ tau0, const float *__restrict__ hc, int64_t c_begin, int S,
    int64_t chunk, int cap, uint2 *__restrict__ buf, int *__restrict__ cnt) {
    __shared__ SwSmem sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wq = w & 3, wc = w >> 2;  // SIMD partners (w, w+4) share queries
    const int h = lane >> 5, cl = lane & 31;
    const int v = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int64_t q0 = (int64_t)(v / S) * BQ;
    const int sl = v % S;
    const int64_t cbeg = c_begin + (int64_t)sl * chunk;
    const int64_t cend = min(nc, cbeg + chunk);
    const int64_t ntile = cend > cbeg ? (cend - cbeg + BC - 1) / BC : 0;
    const int64_t gtot = ntile * nkb;

    // this lane's queries (one per 32-query block): (tau0 - |q|^2) / 2
    float tql[WQB];
#pragma unroll
    for (int b = 0; b < WQB; ++b) {
        const int64_t q = q0 + 64 * wq + 32 * b + cl;
        tql[b] = q < nq ? tq[q] : -__builtin_inff();
    }
    if (tid < BQ) {
        sm.qcnt[tid] = 0;
        sm.t0[tid] = q0 + tid < nq ? tau0[q0 + tid] : 0.f;
    }
    if (ntile > 0 && tid < BC) {
        const int64_t c = cbeg + tid;
        sm.hc[0][tid] = (c < cend) ? hc[c] : __builtin_inff();
    }

    // DMA issue state: next stage to stage (tile bt0, k-block bkb) into bslot.
    // Per-lane source offsets (elements within a KB32 block) are fixed for the
    // query pieces and change per tile for the corpus pieces (row clamp).
    int64_t bt0 = cbeg;
    int bkb = 0, bslot = 0;
    const int prow0 = 32 * w + (lane >> 2), prow1 = prow0 + 16;
    const int pch0 = 8 * swz(prow0, lane & 3), pch1 = 8 * swz(prow1, lane & 3);
    // (32-bit: n * 32 < 2^31 is checked by the driver)
    const int qo0 = (int)(min(q0 + prow0, nq - 1) * KB + pch0);
    const int qo1 = (int)(min(q0 + prow1, nq - 1) * KB + pch1);
    int co0 = (int)(min(bt0 + prow0, cend - 1) * KB + pch0);
    int co1 = (int)(min(bt0 + prow1, cend - 1) * KB + pch1);
    const uint16_t *cbk = Ck, *qbk = Qk;  // current k-block bases
    const int64_t cstep = nc * KB, qstep = nq * KB;
    auto dma = [&](const uint16_t *src, uint16_t *lds) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
    };
    auto issue = [&]() {
        if (bt0 < cend) {
            dma(cbk + co0, &sm.C[bslot][32 * w][0]);
            dma(cbk + co1, &sm.C[bslot][32 * w + 16][0]);
            dma(qbk + qo0, &sm.Q[bslot][32 * w][0]);
            dma(qbk + qo1, &sm.Q[bslot][32 * w + 16][0]);
            bslot = bslot == NSLOT - 1 ? 0 : bslot + 1;
            cbk += cstep;
            qbk += qstep;
            if (++bkb == nkb) {
                bkb = 0;
                bt0 += BC;
                cbk = Ck;
                qbk = Qk;
                co0 = (int)(min(bt0 + prow0, cend - 1) * KB + pch0);
                co1 = (int)(min(bt0 + prow1, cend - 1) * KB + pch1);
            }
        }
    };
    issue();  // stage 0
    issue();  // stage 1
    issue();  // stage 2

    f32x16 acc[WQB][WCB];
    // acc0 = tq(q) - hc(c) for the tile whose hc sits in sm.hc[par]
    auto init_acc = [&](int par) {
#pragma unroll
        for (int cb = 0; cb < WCB; ++cb) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 x = *reinterpret_cast<const float4 *>(
                    &sm.hc[par][128 * wc + 32 * cb + 8 * g + 4 * h]);
#pragma unroll
                for (int b = 0; b < WQB; ++b) {
                    acc[b][cb][4 * g + 0] = tql[b] - x.x;
                    acc[b][cb][4 * g + 1] = tql[b] - x.y;
                    acc[b][cb][4 * g + 2] = tql[b] - x.z;
                    acc[b][cb][4 * g + 3] = tql[b] - x.w;
                }
            }
        }
    };
    // fragment registers: F[0] / F[1] hold k-steps 0 / 1 of a stage
    bf16x8 fq[2][WQB], fc[2][WCB];
    auto read_frags = [&](int slot, int j, bf16x8 (&q)[WQB], bf16x8 (&c)[WCB]) {
        const int ch = 2 * j + h;
#pragma unroll
        for (int b = 0; b < WQB; ++b) {
            const int r = 64 * wq + 32 * b + cl;
            q[b] = *reinterpret_cast<const bf16x8 *>(&sm.Q[slot][r][8 * swz(r, ch)]);
        }
#pragma unroll
        for (int cb = 0; cb < WCB; ++cb) {
            const int r = 128 * wc + 32 * cb + cl;
            c[cb] = *reinterpret_cast<const bf16x8 *>(&sm.C[slot][r][8 * swz(r, ch)]);
        }
    };
    auto mfmas = [&](const bf16x8 (&q)[WQB], const bf16x8 (&c)[WCB]) {
#pragma unroll
        for (int b = 0; b < WQB; ++b)
#pragma unroll
            for (int cb = 0; cb < WCB; ++cb)
                acc[b][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c[cb], q[b], acc[b][cb], 0, 0, 0);
    };

    // prologue: stage 0 landed for every wave (stages 1, 2 still in flight)
    if (gtot > 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (gtot == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // also publishes sm.hc[0]
    if (gtot > 0) {
        init_acc(0);
        read_frags(0, 0, fq[0], fc[0]);
    }
    int cur = 0, par = 0;
    int64_t c0 = cbeg;
    int kb = 0;
    float hc_next = 0.f;  // next tile's hc, staged in a register (see below)
    bool dirty = false;   // candidate stores were issued since the last wait
    int scnt = 0;         // entries in this wave's staging area
    // staged candidates -> HBM (rare: the area holds SCAP entries).  Stores
    // complete out of order with loads, so the next counted wait drains.
    auto flush = [&]() {
        for (int e = lane; e < scnt; e += 64) {
            const uint2 v = sm.stk[w][e];
            const uint32_t pq = sm.stp[w][e];
            const int pos = (int)(pq >> 8), ql = (int)(pq & 255u);
            if (pos < cap) buf[((q0 + ql) * S + sl) * (int64_t)cap + pos] = v;
        }
        scnt = 0;
        dirty = true;
    };
    for (int64_t g = 0; g < gtot; ++g) {
        // k-step 1 of stage g
        read_frags(cur, 1, fq[1], fc[1]);
        mfmas(fq[0], fc[0]);
        // stage g+1 landed (stage g+2's 4 pieces may stay in flight); the
        // barrier also frees the slot of stage g-1 for stage g+3.  Stores
        // complete out of order with loads, so after candidate stores the
        // count is not trusted: drain once.
        const int64_t rem = gtot - 1 - g;
        if (rem >= 2 && !dirty) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        dirty = false;
        __builtin_amdgcn_s_barrier();
        // the next tile's hc: loaded at k-block 0 (older than stage g+3, so the
        // counted wait of k-block 1 covers it), written at k-block 1, read by
        // init_acc after k-block nkb-1 (>= 2 barriers later; nkb >= 4)
        // (an asm load: the compiler would otherwise drain vmcnt to 0 twice
        // per tile around it)
        const bool more = c0 + BC < cend;
        if (kb == 0 && more && tid < BC) {
            const float *p = hc + min(c0 + BC + tid, cend - 1);
            asm volatile("global_load_dword %0, %1, off" : "=v"(hc_next) : "v"(p) : "memory");
        }
        if (kb == 1 && more && tid < BC)
            sm.hc[par ^ 1][tid] = c0 + BC + tid < cend ? hc_next : __builtin_inff();
        issue();  // stage g+3
        const int nxt = cur == NSLOT - 1 ? 0 : cur + 1;
        // unconditional (the last step reads a stale slot, unused): a
        // conditional read would make the compiler wait lgkmcnt(0) below
        read_frags(nxt, 0, fq[0], fc[0]);
        mfmas(fq[1], fc[1]);
        cur = nxt;
        if (++kb < nkb) continue;
        // ---- tile done: candidates are the positive accumulators ----
        kb = 0;
        if constexpr (PROBE == 0) {
            const int64_t cg0 = c_off + c0 + 128 * wc;
#pragma unroll
            for (int b = 0; b < WQB; ++b) {
#pragma unroll
                for (int cb = 0; cb < WCB; ++cb) {
                    const f32x16 &a = acc[b][cb];
                    float m = fmaxf(fmaxf(a[0], a[1]), a[2]);
#pragma unroll
                    for (int r = 3; r < 15; r += 2) m = fmaxf(fmaxf(m, a[r]), a[r + 1]);
                    m = fmaxf(m, a[15]);
                    if (__builtin_expect(__ballot(m > 0.f) == 0, 1)) continue;
                    // rare: stage this lane's positive entries in LDS
                    unsigned pm = 0;
#pragma unroll
                    for (int r = 0; r < 16; ++r) pm |= a[r] > 0.f ? (1u << r) : 0u;
                    // the self pair can only sit in a block whose query and
                    // corpus id ranges overlap (wave-uniform test)
                    const int64_t qlo = q_off + q0 + 64 * wq + 32 * b;
                    const int64_t clo = cg0 + 32 * cb;
                    if (excl && qlo < clo + 32 && clo < qlo + 32) {
                        const int64_t qgl = qlo + cl;
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            if (clo + 8 * (r >> 2) + 4 * h + (r & 3) == qgl) pm &= ~(1u << r);
                    }
                    const int mine = __popc(pm);
                    // wave prefix sum of the counts (inclusive)
                    int pre = mine;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int t = __shfl_up(pre, o);
                        if (lane >= o) pre += t;
                    }
                    const int total = __shfl(pre, 63);
                    if (scnt + total > SCAP) flush();
                    const int ql = 64 * wq + 32 * b + cl;
                    if (total > SCAP) {
                        // a burst beyond the staging area: the threshold is far
                        // too loose for these queries, which overflow (exact scan)
                        if (mine) atomicMax(&sm.qcnt[ql], cap + 1);
                        continue;
                    }
                    const float t0l = sm.t0[ql];
                    int pos = mine ? atomicAdd(&sm.qcnt[ql], mine) : 0;
                    // (positions past cap are staged as cap: skipped by flush)
                    int e = scnt + pre - mine;
                    while (pm) {
                        const int r = __builtin_ctz(pm);
                        pm &= pm - 1;
                        sm.stk[w][e] = make_uint2(__float_as_uint(t0l - 2.f * a[r]),
                                                  (uint32_t)(clo + 8 * (r >> 2) + 4 * h + (r & 3)));
                        sm.stp[w][e] = (uint32_t)ql | ((uint32_t)min(pos, cap) << 8);
                        ++e;
                        ++pos;
                    }
                    scnt += total;
                }
            }
        } else {
            // timing probe: K loop only (results discarded)
            float s = 0.f;
#pragma unroll
            for (int b = 0; b < WQB; ++b)
#pragma unroll
                for (int cb = 0; cb < WCB; ++cb) s += acc[b][cb][0];
            if (s == 12345.678f) sm.qcnt[0] = 1;
        }
        c0 += BC;
        par ^= 1;
        if (c0 < cend) init_acc(par);  // sm.hc[par] was written during this tile
    }
    if (scnt > 0) flush();
    __syncthreads();
    if (tid < BQ && q0 + tid < nq) {
        const int c = sm.qcnt[tid];
        cnt[(q0 + tid) * S + sl] = c > cap ? -1 : c;
    }
}

// Slicing + buffer sizing of the sweep.
struct SweepPlan {
    int64_t S, chunk;
    int cap;
};

// nc2 = corpus rows of phase 2; expect = expected candidates per query.
inline SweepPlan plan_sweep(int64_t nq, int64_t nc2, double expect) {
    SweepPlan p;
    const int64_t nqb = (nq + BQ - 1) / BQ;
    int64_t S = std::max<int64_t>(8, (2048 + nqb - 1) / nqb);
    const char *es = getenv("MN_SWEEP_S");  // experiments: corpus slices
    if (es && *es) S = std::max(1, atoi(es));
    S = std::min<int64_t>(S, std::max<int64_t>(1, nc2 / (4 * BC)));
    S = std::max<int64_t>(S, 1);
    int64_t chunk = (nc2 + S - 1) / S;
    chunk = std::max<int64_t>(BC, (chunk + BC - 1) / BC * BC);
    S = std::max<int64_t>(1, (nc2 + chunk - 1) / chunk);
    p.S = S;
    p.chunk = chunk;
    const double per = expect / (double)S;
    int cap = (int)((2.5 * per + 64.0 + 15.0) / 16.0) * 16;
    p.cap = std::max(cap, 64);
    return p;
}

}  // namespace ksw
}  // namespace mn
