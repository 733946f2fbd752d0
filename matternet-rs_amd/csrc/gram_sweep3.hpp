// gram_sweep3.hpp — the symmetric sweeps (SW_SYM: C2's self L2 kNN on fp16
// x 2^e operands; SW_COS_SYM: C5's bf16 cosine item graph) re-scheduled for
// instruction issue.  Same contract, block table, LDS layout, ring protocol
// and ping-pong as gram_sweep2.hpp's k_gram_sweep2<0, SW_SYM / SW_COS_SYM,
// TM>; the outputs are identical bit for bit.  The query-major modes SW_L2 /
// SW_COS run the phase-1 sample sweeps of C2 and C5 (per-(row, slice)
// buffers through global counters).  What changed (round 6):
//
//  * The read window's SALU.  sweep2 rebuilt two buffer descriptors per
//    k-step, walked a branch tree per window to pick vmcnt(8 / 4 / 0) and a
//    'dirty' flag, and advanced 64-bit pointers: ~70 SALU per k-step and wave
//    (2.2 per MFMA, SQ_INSTS_SALU in profiles/r05_legs), all of it issued by
//    the reading wave inside the window its partner's 32 MFMAs must cover.
//    Here the panel descriptors are built once per tile, the k-block advances
//    in `soffset`, every k-step issues exactly four LDS-DMA pieces (past the
//    block's last k-step the last one is re-staged into the slot nobody reads
//    any more), so the in-loop wait is always vmcnt(8), and a flush of the
//    candidate staging area drains its own stores (vmcnt(0), rare) instead of
//    marking the next wait.
//  * The tile epilogue's code size.  sweep2 inlined the candidate-emission
//    body once per fragment (32 copies, 91 KB of code for the kernel against
//    a 64 KB instruction cache shared by two CUs), so every rare hit jumped
//    into cold code.  Here the per-fragment prefilter only sets a bit of a
//    wave-uniform 32-bit mask; the hits are then picked out one at a time
//    (a switch copies that fragment's four accumulators) into ONE emission
//    body.
#pragma once
#include "gram_sweep2.hpp"

namespace mn {
namespace ksw2 {

// AHEAD (tuning A/B): the LDS-DMA runs AHEAD k-steps ahead of the reads.
// 3: a k-step's fragment reads complete (lgkmcnt(0)) before the barrier that
// ends its read window — the DMA issued in the next window re-fills that slot.
// 2: the slot re-filled next is two k-steps old, so the reads may complete
// across the barrier: the wait moves to the head of the MFMA window and the
// read window holds only the issue of the reads and of the DMA.
// sweep3's LDS beside the ring: sweep2's per-tile arrays, and per wave a
// staging area of RAW hits — one entry per lane and fragment with a candidate:
// (query position | diag << 31, position of the fragment's register 0 | the
// candidate registers << 28) and the four accumulators.  The keys, the second
// direction and the per-row slots are worked out when the area is flushed,
// for 64 entries at a time, so a hit costs the tile epilogue two LDS stores.
constexpr int RCAP = 112;  // raw entries per wave
struct alignas(16) Smem3 {
    float hc[2][BC];   // a tile's column folds (diagonal: hc, else hoff; +pad)
    float tc[2][BC];   // a tile's tau0 (Teff; COS: |c|)
    float ta[BQ];      // the queries' off-diagonal folds
    float t0[BQ];      // the queries' tau0
    float tq[BQ];      // the queries' diagonal folds
    float sq[BQ];      // F16: the queries' scales
    float sc[2][BC];   // F16: a tile's scales
    uint2 rid[NWAVES][RCAP];
    f32x4 racc[NWAVES][RCAP];
};
static_assert(sizeof(Smem3) + sizeof(Ring) <= 163840, "LDS budget");

// PH (tuning A/B): windows per k-step and group.  1: one read window (12
// fragment reads, 4 DMA pieces) and one MFMA window (32 MFMAs); 2: two of
// each (8 reads + the corpus tile's 2 pieces | 16 MFMAs, then 4 reads + the
// query panel's 2 pieces | 16 MFMAs) — half the burst per window.
// EMI (tuning A/B): 0 = the fragments' hit mask, then a switch picks each
// hit fragment into one staging body; 1 = the (small) staging body inline
// per fragment behind its ballot.
template <int PROBE, int MODE, int AHEAD = 3, int PH = 1, int EMI = 0>
__global__ __launch_bounds__(NT) void k_gram_sweep3(
    const uint16_t *__restrict__ Qk, int64_t nq, const uint16_t *__restrict__ Ck, int64_t nc,
    int nkb, int64_t q_off, int64_t c_off, int excl, const float *__restrict__ tq,
    const float *__restrict__ tau0, const float *__restrict__ hc, int64_t c_begin, int S,
    int64_t chunk, int cap, uint2 *__restrict__ buf, int *__restrict__ cnt, int pst, SymArgs sym) {
    // QM (round 6): the query-major sweeps SW_L2 / SW_COS (the phase-1 sample
    // sweeps of C2 and C5): block v takes query panel v / S against slice
    // v % S ([c_begin + sl chunk, + chunk)), bf16 operands, the row's own
    // test only; candidates go to buf[(q S + sl) cap + pos] through global
    // counters cnt[q S + sl] (a count past cap = overflow; the callers'
    // selects read it as a full buffer)
    constexpr bool QM = MODE == SW_L2 || MODE == SW_COS;
    constexpr bool F16 = MODE == SW_SYM;     // fp16 x 2^e operands, per-row scales
    constexpr bool COSM = MODE == SW_COS_SYM || MODE == SW_COS;
    static_assert(!(QM && EMI == 1), "k_gram_sweep3: EMI 1 marks symmetric rows only");
    // PROBE (tuning build, results invalid): 1 = K loop only (no check, no
    // init), 2 = init only, 3 = init + prefilter (no emission)
    // 4 / 5 / 6 = K loop only and also without the in-loop LDS-DMA issue /
    // the in-loop barriers / the fragment reads (timing only)
    constexpr bool EPI = PROBE == 0 || PROBE == 3;
    constexpr bool INIT = PROBE == 0 || PROBE == 2 || PROBE == 3;
    constexpr bool NODMA = PROBE == 4, NOBAR = PROBE == 5, NOREAD = PROBE == 6;
    __shared__ Ring rg;
    __shared__ Smem3 sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wq = w & 3, wc = w >> 2;
    const int fr = lane & 15, fk = lane >> 4;
    const int v = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    int q0, sl = 0, cbeg, cend, ntile, cstr;
    if constexpr (QM) {
        q0 = (v / S) * BQ;
        sl = v % S;
        cbeg = (int)(c_begin + (int64_t)sl * chunk);
        cend = (int)min(nc, (int64_t)cbeg + chunk);
        ntile = cend > cbeg ? (cend - cbeg + BC - 1) / BC : 0;
        cstr = BC;
    } else {
        const int4 te = sym.tab[v];
        q0 = te.x * BQ;
        cbeg = te.y * BC;
        cend = (int)nc;
        ntile = te.z;
        cstr = te.w * BC;
    }
    // padding columns never qualify: COS NaN, SW_L2 +inf (acc0 = tq - inf),
    // SW_SYM -inf (the fold is added)
    const float pad = COSM ? __builtin_nanf("") : (QM ? __builtin_inff() : -__builtin_inff());
    const bool diag0 = !QM && cbeg == q0;
    if (ntile == 0) return;  // the per-XCD padding entries of the table (block-uniform)

    if (tid < BQ) {
        sm.tq[tid] = q0 + tid < nq ? tq[q0 + tid] : (COSM ? pad : -__builtin_inff());
        sm.t0[tid] = q0 + tid < nq ? tau0[q0 + tid] : 0.f;
        if constexpr (!QM) sm.ta[tid] = q0 + tid < nq ? sym.aoff[q0 + tid] : (COSM ? pad : -__builtin_inff());
        if constexpr (F16) sm.sq[tid] = q0 + tid < nq ? sym.scale[q0 + tid] : 1.f;
    }
    if (ntile > 0 && tid < BC) {
        const int c = cbeg + tid;
        sm.hc[0][tid] = (c < cend) ? ((QM || diag0) ? hc[c] : sym.hoff[c]) : pad;
        if constexpr (!QM) sm.tc[0][tid] = (c < cend) ? tau0[c] : pad;
        if constexpr (F16) sm.sc[0][tid] = (c < cend) ? sym.scale[c] : 1.f;
    }

    // ---- LDS-DMA: wave w stages rows [32w, 32w + 32) of the corpus tile and
    // of the query panel, two 16-row pieces each; lane l -> row + (l >> 2),
    // physical chunk l & 3 (the read swizzle applied to the source).  Both
    // operands are tile-major panels: a k-step is the 16-KB piece at
    // soffset = kb * 16384 of a panel, the per-lane offsets never change.
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const int prow0 = 32 * w + (lane >> 2);
    const int pch = 8 * ((lane & 3) ^ (((lane >> 5) & 1) << 1));
    const int vo0 = 2 * (prow0 * KB + pch), vo1 = vo0 + 2 * 16 * KB;
    const int64_t panel = (int64_t)pst * BC * KB;  // elements between 256-row panels
    const int pbytes = pst * BC * KB * 2;           // one panel (descriptor range)
    auto rsrc = [&](const uint16_t *base) __attribute__((always_inline)) {
        const uint64_t a = (uint64_t)(uintptr_t)base;
        u32x4 r;
        r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
        r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
        r.z = (uint32_t)pbytes;
        r.w = 0x00020000u;
        return r;
    };
    auto dma = [&](const u32x4 &rs, int soff, int voff, uint32_t lds) __attribute__((always_inline)) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :
                     : "s"(lds), "v"(voff), "s"(rs), "s"(soff)
                     : "memory", "m0");
    };
    const u32x4 rq = rsrc(Qk + (int64_t)(q0 / BQ) * panel);  // the block's query panel
    u32x4 rc = rsrc(Ck + (int64_t)(cbeg / BC) * panel);       // the staged step's corpus tile
    int dt = 0, dsoff = 0;                                     // staged step: tile, k-block bytes
    uint32_t dsl = 0;                                          // its ring slot (bytes)
    const uint32_t ldsC = __builtin_amdgcn_readfirstlane(lds_addr(&rg.C[0][32 * w][0]));
    const uint32_t ldsQ = __builtin_amdgcn_readfirstlane(lds_addr(&rg.Q[0][32 * w][0]));
    const int kend = nkb * (KB * BC * 2);
    // stage the next k-step (four pieces, always: past the block's last
    // k-step the last one again, into the slot nobody reads any more)
    auto issue_c = [&]() __attribute__((always_inline)) {
        dma(rc, dsoff, vo0, ldsC + dsl);
        dma(rc, dsoff, vo1, ldsC + dsl + 1024);
    };
    auto issue_q = [&]() __attribute__((always_inline)) {  // then the next step
        dma(rq, dsoff, vo0, ldsQ + dsl);
        dma(rq, dsoff, vo1, ldsQ + dsl + 1024);
        dsl = (dsl + (uint32_t)(BC * KB * 2)) & (uint32_t)(NSLOT * BC * KB * 2 - 1);
        dsoff += KB * BC * 2;
        if (dsoff == kend) {
            if (dt + 1 < ntile) {
                ++dt;
                dsoff = 0;
                rc = rsrc(Ck + (int64_t)((cbeg + dt * cstr) / BC) * panel);
            } else {
                dsoff -= KB * BC * 2;
            }
        }
    };
    auto issue = [&]() __attribute__((always_inline)) {
        issue_c();
        issue_q();
    };

    typedef typename std::conditional<F16, f16x8, bf16x8>::type frag_t;
    f32x4 acc[WQF][WCF];
    frag_t fq[WQF], fc[WCF];
    auto init_acc = [&](int par, bool diag) __attribute__((always_inline)) {
        float tql[WQF];
        const float *qa = (QM || diag) ? sm.tq : sm.ta;
#pragma unroll
        for (int f = 0; f < WQF; ++f) tql[f] = qa[64 * wq + 16 * f + fr];
        float sql[WQF];
        if constexpr (F16) {
#pragma unroll
            for (int f = 0; f < WQF; ++f) sql[f] = sm.sq[64 * wq + 16 * f + fr];
        }
#pragma unroll
        for (int g = 0; g < WCF; ++g) {
            const float4 x = *reinterpret_cast<const float4 *>(&sm.hc[par][128 * wc + 16 * g + 4 * fk]);
            float4 sc4 = make_float4(1.f, 1.f, 1.f, 1.f);
            if constexpr (F16)
                sc4 = *reinterpret_cast<const float4 *>(&sm.sc[par][128 * wc + 16 * g + 4 * fk]);
#pragma unroll
            for (int f = 0; f < WQF; ++f) {
                if constexpr (F16) {
                    acc[f][g][0] = __builtin_fmaf(tql[f], sc4.x, x.x * sql[f]);
                    acc[f][g][1] = __builtin_fmaf(tql[f], sc4.y, x.y * sql[f]);
                    acc[f][g][2] = __builtin_fmaf(tql[f], sc4.z, x.z * sql[f]);
                    acc[f][g][3] = __builtin_fmaf(tql[f], sc4.w, x.w * sql[f]);
                } else if constexpr (COSM) {
                    acc[f][g][0] = tql[f] * x.x;
                    acc[f][g][1] = tql[f] * x.y;
                    acc[f][g][2] = tql[f] * x.z;
                    acc[f][g][3] = tql[f] * x.w;
                } else {  // SW_L2: acc0 = tq(q) - hc(c)
                    acc[f][g][0] = tql[f] - x.x;
                    acc[f][g][1] = tql[f] - x.y;
                    acc[f][g][2] = tql[f] - x.z;
                    acc[f][g][3] = tql[f] - x.w;
                }
            }
        }
    };
    const int chs0 = 8 * swz(fr, fk);
    const uint32_t qrd = lds_addr(&rg.Q[0][64 * wq + fr][chs0]);
    const uint32_t crd = lds_addr(&rg.C[0][128 * wc + fr][chs0]);
    auto read_frags_h0 = [&](uint32_t so) __attribute__((always_inline)) {
        const uint32_t qa = qrd + so, ca = crd + so;
        asm volatile("ds_read_b128 %0, %1" : "=v"(fq[0]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(fq[1]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(fq[2]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(fq[3]) : "v"(qa));
        asm volatile("ds_read_b128 %0, %1" : "=v"(fc[0]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(fc[1]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(fc[2]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(fc[3]) : "v"(ca));
    };
    auto read_frags_h1 = [&](uint32_t so) __attribute__((always_inline)) {
        const uint32_t ca = crd + so;
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(fc[4]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:5120" : "=v"(fc[5]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(fc[6]) : "v"(ca));
        asm volatile("ds_read_b128 %0, %1 offset:7168" : "=v"(fc[7]) : "v"(ca));
    };
    auto read_frags = [&](uint32_t so) __attribute__((always_inline)) {
        const uint32_t qa = qrd + so, ca = crd + so;
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
    auto mfmas = [&](int g0, int g1) __attribute__((always_inline)) {
#pragma unroll
        for (int f = 0; f < WQF; ++f)
#pragma unroll
            for (int g = g0; g < g1; ++g)
                if constexpr (F16)
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fc[g], fq[f], acc[f][g], 0, 0, 0);
                else
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[g], fq[f], acc[f][g], 0, 0, 0);
    };

    // ---- candidates.  expand(): one raw hit (query position q, diag, the
    // position c of register 0, candidate registers pm, accumulators a4) ->
    // its candidates (row, key, id) appended to the per-row buffers through
    // the per-row counters: every slot atomic first, then the entries (one
    // round trip).  Keys exactly as sweep2 forms them.
    // build(): the up to 8 candidates of one raw hit into rw / kv / go
    auto build = [&](bool valid, uint32_t qw, uint32_t cw, const f32x4 a4, uint32_t (&rw)[8],
                     uint2 (&kv)[8], bool (&go)[8]) __attribute__((always_inline)) {
        const int q = (int)(qw & 0x7fffffffu), c = (int)(cw & 0x0fffffffu);
        const bool dg = (qw >> 31) != 0u;
        const unsigned pm = valid ? (cw >> 28) : 0u;
        const int ql = q - (int)q_off - q0;
        float colv[4], cols[4];
        if constexpr (QM) {  // the row's own test: one candidate per register
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool h = (pm >> r) & 1u;
                float key;
                if constexpr (COSM) {  // hc = -|c|: key = -acc / |c|
                    const int cc = min(c + r - (int)c_off, (int)nc - 1);
                    key = a4[r] / (h ? hc[cc] : 1.f);
                } else {
                    key = sm.t0[ql] - 2.f * a4[r];
                }
                go[2 * r] = h;
                rw[2 * r] = h ? (uint32_t)(ql + q0) * (uint32_t)S + (uint32_t)sl : 0u;
                kv[2 * r] = make_uint2(__float_as_uint(key), (uint32_t)(c + r));
                go[2 * r + 1] = false;
                rw[2 * r + 1] = 0u;
                kv[2 * r + 1] = make_uint2(0u, 0u);
            }
            return;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // the columns' values (global: the tile may be gone)
            const int cc = min(c + r - (int)c_off, (int)nc - 1);
            colv[r] = ((pm >> r) & 1u) ? (COSM ? (dg ? hc[cc] : sym.hoff[cc]) : tau0[cc]) : 0.f;
            cols[r] = ((pm >> r) & 1u) ? (COSM ? tau0[cc] : sym.scale[cc]) : 1.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const bool h = (pm >> r) & 1u;
            const uint32_t cr = (uint32_t)(c + r);
            if constexpr (COSM) {
                if (dg) {  // row q's test: key = -acc / |c| (hc = -|c|)
                    go[2 * r] = h;
                    rw[2 * r] = (uint32_t)q;
                    kv[2 * r] = make_uint2(__float_as_uint(a4[r] / colv[r]), cr);
                    go[2 * r + 1] = false;
                } else {   // row c's test; row q's on these hits
                    const float tal = sm.ta[ql];
                    go[2 * r] = h;
                    rw[2 * r] = cr;
                    kv[2 * r] = make_uint2(__float_as_uint(-a4[r] / tal), (uint32_t)q);
                    const float kq = (colv[r] * tal - a4[r]) / cols[r] + sm.tq[ql];
                    go[2 * r + 1] = h && kq < 0.f;
                    rw[2 * r + 1] = (uint32_t)q;
                    kv[2 * r + 1] = make_uint2(__float_as_uint(kq), cr);
                }
            } else {
                const float t0l = sm.t0[ql];
                float a2 = __builtin_ldexpf(a4[r], 1 - __builtin_amdgcn_frexp_expf(sm.sq[ql]));
                a2 = __builtin_ldexpf(a2, 1 - __builtin_amdgcn_frexp_expf(cols[r]));
                a2 *= 2.f;
                if (dg) {  // row q's test
                    go[2 * r] = h;
                    rw[2 * r] = (uint32_t)q;
                    kv[2 * r] = make_uint2(__float_as_uint(t0l - a2), cr);
                    go[2 * r + 1] = false;
                } else {   // row c's test (acc > 0); row q's only on these hits
                    const float key = colv[r] - a2;
                    go[2 * r] = h;
                    rw[2 * r] = cr;
                    kv[2 * r] = make_uint2(__float_as_uint(key), (uint32_t)q);
                    go[2 * r + 1] = h && key < t0l;
                    rw[2 * r + 1] = (uint32_t)q;
                    kv[2 * r + 1] = make_uint2(__float_as_uint(key), cr);
                }
            }
            rw[2 * r + 1] = go[2 * r + 1] ? rw[2 * r + 1] : 0u;
            rw[2 * r] = go[2 * r] ? rw[2 * r] : 0u;
        }
    };
    auto expand = [&](bool valid, uint32_t qw, uint32_t cw, const f32x4 a4) __attribute__((always_inline)) {
        uint32_t rw[8];
        uint2 kv[8];
        bool go[8];
        int pos[8];
        build(valid, qw, cw, a4, rw, kv, go);
#pragma unroll
        for (int j = 0; j < 8; ++j) pos[j] = go[j] ? atomicAdd(&cnt[rw[j]], 1) : cap;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (pos[j] < cap) buf[(int64_t)rw[j] * cap + pos[j]] = kv[j];
    };
    int ns = 0;  // raw entries staged by this wave (wave-uniform)
    static_assert(RCAP <= 128, "flush: two raw entries per lane");
    auto flush = [&]() __attribute__((always_inline)) {
        const int n = min(ns, RCAP);
        // both entries of the lane built first, then all 16 slot atomics, then
        // the entries: one round trip per flush
        uint32_t rw[2][8];
        uint2 kv[2][8];
        bool go[2][8];
        int pos[2][8];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int e = lane + 64 * j;
            const bool ok = e < n;
            const int ee = ok ? e : 0;
            build(ok, sm.rid[w][ee].x, sm.rid[w][ee].y, sm.racc[w][ee], rw[j], kv[j], go[j]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i) pos[j][i] = go[j][i] ? atomicAdd(&cnt[rw[j][i]], 1) : cap;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (pos[j][i] < cap) buf[(int64_t)rw[j][i] * cap + pos[j][i]] = kv[j][i];
        ns = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no store left for the counted waits
    };
    // one fragment's hits (a = its accumulators, f / g its position): the
    // lanes with a candidate register stage one raw entry each, slots from
    // the wave's prefix count (mbcnt over the ballot)
    auto emit_frag = [&](const f32x4 a, int f, int g, int ct0, bool diag) __attribute__((always_inline)) {
        const int ql = 64 * wq + 16 * f + fr;
        const int qgl = (int)q_off + q0 + ql;
        const int c = (int)c_off + ct0 + 128 * wc + 16 * g + 4 * fk;  // id of register 0
        unsigned pm = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) pm |= a[r] > 0.f ? (1u << r) : 0u;
        if (excl && (unsigned)(qgl - c) < 4u) pm &= ~(1u << (qgl - c));
        const bool h = pm != 0u;
        const uint64_t b = __ballot(h);
        if (b == 0) return;
        const int e = ns + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        ns += __builtin_popcountll(b);
        const uint32_t qw = (uint32_t)qgl | (diag ? 0x80000000u : 0u), cw = (uint32_t)c | (pm << 28);
        if (h && e < RCAP) {
            sm.rid[w][e] = make_uint2(qw, cw);
            sm.racc[w][e] = a;
        }
        if (ns > RCAP) {  // area full (rare)
            if constexpr (EMI == 1) {
                // (the body is inlined per fragment: no expansion here) the
                // rows those entries would feed are marked overflowed, so
                // they take the exact path
                if (h && e >= RCAP) {
                    atomicMax(&cnt[qgl - (int)q_off], cap + 1);
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if ((pm >> r) & 1u) atomicMax(&cnt[c + r - (int)c_off], cap + 1);
                }
            } else {  // those lanes' entries straight out
                expand(h && e >= RCAP, qw, cw, a);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    };
    // the tile starting at corpus row ct0: a wave-uniform mask of the
    // fragments where some lane holds a positive accumulator (the maximum of
    // its four as signed integers: positive iff a float > 0 or a +NaN, which
    // the exact test drops), then each such fragment through the one body
    auto check = [&](int ct0, int hpar, bool diag) __attribute__((always_inline)) {
        if constexpr (EPI) {
            uint32_t fm = 0;
#pragma unroll
            for (int f = 0; f < WQF; ++f)
#pragma unroll
                for (int g = 0; g < WCF; ++g) {
                    const f32x4 a = acc[f][g];
                    const int mi = max(max(__float_as_int(a[0]), __float_as_int(a[1])),
                                       max(__float_as_int(a[2]), __float_as_int(a[3])));
                    if constexpr (EMI == 1) {
                        if (__builtin_expect(__ballot(mi > 0) != 0, 0)) emit_frag(a, f, g, ct0, diag);
                    } else {
                        fm |= __ballot(mi > 0) != 0 ? (1u << (8 * f + g)) : 0u;
                    }
                }
            if constexpr (PROBE == 3) {  // keep the mask live; never a staged entry
                if (fm == 0x12345u) sm.ta[0] = 0.f;
                fm = 0;
            }
            while (__builtin_expect(fm != 0, 0)) {
                const int i = __builtin_ctz(fm);
                fm &= fm - 1;
                f32x4 a;
                switch (i) {
// (a distinct asm per case: the cases' copies must not be merged into one
// load through a computed index, which would move acc to scratch)
#define MN_PICK(F, G) \
    case 8 * F + G: asm volatile("; pick " #F #G : "=v"(a) : "0"(acc[F][G])); break;
#define MN_PICK8(F) MN_PICK(F, 0) MN_PICK(F, 1) MN_PICK(F, 2) MN_PICK(F, 3) \
                    MN_PICK(F, 4) MN_PICK(F, 5) MN_PICK(F, 6) MN_PICK(F, 7)
                    MN_PICK8(0) MN_PICK8(1) MN_PICK8(2) MN_PICK8(3)
                    default: a = acc[0][0]; break;
#undef MN_PICK8
#undef MN_PICK
                }
                emit_frag(a, i >> 3, i & 7, ct0, diag);
            }
            if (ns >= RCAP * 3 / 4) flush();
        } else {
            float s = 0.f;
#pragma unroll
            for (int f = 0; f < WQF; ++f)
#pragma unroll
                for (int g = 0; g < WCF; ++g) s += acc[f][g][0];
            if (s == 12345.678f) sm.ta[0] = 0.f;  // keep acc live (results invalid anyway)
        }
    };

    static_assert(AHEAD == 2 || AHEAD == 3, "k_gram_sweep3: AHEAD 2 or 3");
    // the wait that retires k-step + 1 while the later AHEAD - 1 are in flight
    auto vm_wait = [&]() __attribute__((always_inline)) {
        if constexpr (AHEAD == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    };
    auto lgkm_wait_h0 = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(fq[0]), "+v"(fq[1]), "+v"(fq[2]), "+v"(fq[3]), "+v"(fc[0]),
                       "+v"(fc[1]), "+v"(fc[2]), "+v"(fc[3])
                     :
                     : "memory");
    };
    auto lgkm_wait_h1 = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fc[4]), "+v"(fc[5]), "+v"(fc[6]), "+v"(fc[7]) : : "memory");
    };
    auto lgkm_wait = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(fq[0]), "+v"(fq[1]), "+v"(fq[2]), "+v"(fq[3]), "+v"(fc[0]),
                       "+v"(fc[1]), "+v"(fc[2]), "+v"(fc[3]), "+v"(fc[4]), "+v"(fc[5]),
                       "+v"(fc[6]), "+v"(fc[7])
                     :
                     : "memory");
    };
    // ---- prologue: k-steps 0 .. AHEAD-1 in flight; k-step 0 landed everywhere
    issue();
    issue();
    if constexpr (AHEAD == 3) issue();
    vm_wait();
    __syncthreads();  // also publishes sm.hc[0], t0, tq
    init_acc(0, diag0);
    if (wc == 1 && !NOBAR) __builtin_amdgcn_s_barrier();  // the trailing group starts one window late

    uint32_t so = 0;  // ring slot of the current k-step (bytes)
    int par = 0;
    float hcn = 0.f, tcn = 0.f, scn = 1.f;  // next tile's folds (waves 0-3)
    // the k-steps of a tile that carry extra work, as one compare each (the
    // conditions folded per tile: ~45 -> ~30 SALU a k-step and wave)
    const bool lead = wc == 0, trail = wc == 1;
    for (int ti = 0; ti < ntile; ++ti) {
        const int c0 = cbeg + ti * cstr;
        const bool more = ti + 1 < ntile;
        const int k_chk = ti > 0 ? 0 : -1;                    // the previous tile's epilogue
        const int k_ld = (more && lead) ? nkb - 4 : -1;        // the next tile's fold loads
        const int k_st = (more && lead) ? nkb - 2 : -1;        //   and their stores
        for (int kb = 0; kb < nkb; ++kb) {
            // ================= READ window =================
            if (kb == k_ld) {
                // the next tile's off-diagonal folds: one value per lane, asm
                // loads older than the DMA issued below (the counted waits
                // retire them 2 k-steps before the store)
                const int cn = min(c0 + cstr + 64 * wq + lane, (int)nc - 1);
                asm volatile("global_load_dword %0, %1, off" : "=v"(hcn) : "v"((QM ? hc : sym.hoff) + cn) : "memory");
                if constexpr (!QM)
                    asm volatile("global_load_dword %0, %1, off" : "=v"(tcn) : "v"(tau0 + cn) : "memory");
                if constexpr (F16)
                    asm volatile("global_load_dword %0, %1, off" : "=v"(scn) : "v"(sym.scale + cn) : "memory");
            }
            if (kb == k_chk) {
                check(c0 - cstr, par ^ 1, diag0 && ti == 1);
                if constexpr (INIT) init_acc(par, false);
            }
            if constexpr (PH == 2) {
                static_assert(PH != 2 || AHEAD == 2, "PH 2 takes AHEAD 2");
                read_frags_h0(so);
                __builtin_amdgcn_sched_barrier(0);
                issue_c();  // k-step + 2: the corpus tile's pieces
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                lgkm_wait_h0();
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(1);
                mfmas(0, WCF / 2);
                __builtin_amdgcn_s_setprio(0);
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                read_frags_h1(so);
                __builtin_amdgcn_sched_barrier(0);
                issue_q();  // k-step + 2: the query panel's pieces
                __builtin_amdgcn_sched_barrier(0);
                if (kb == nkb - 2 && more && wc == 0) {
                    const int cb = c0 + cstr + 64 * wq + lane;
                    sm.hc[par ^ 1][64 * wq + lane] = cb < cend ? hcn : pad;
                    sm.tc[par ^ 1][64 * wq + lane] = cb < cend ? tcn : pad;
                    if constexpr (F16) sm.sc[par ^ 1][64 * wq + lane] = cb < cend ? scn : 1.f;
                }
                if (wc == 1) vm_wait();
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                lgkm_wait_h1();
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(1);
                mfmas(WCF / 2, WCF);
                __builtin_amdgcn_s_setprio(0);
                __builtin_amdgcn_sched_barrier(0);
                if (wc == 0) vm_wait();
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                so = (so + (uint32_t)(BC * KB * 2)) & (uint32_t)(NSLOT * BC * KB * 2 - 1);
                continue;
            }
            if constexpr (!NOREAD) read_frags(so);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!NODMA) issue();  // k-step + AHEAD, behind the reads
            __builtin_amdgcn_sched_barrier(0);
            if (kb == k_st) {
                const int cb = c0 + cstr + 64 * wq + lane;
                sm.hc[par ^ 1][64 * wq + lane] = cb < cend ? hcn : pad;
                sm.tc[par ^ 1][64 * wq + lane] = cb < cend ? tcn : pad;
                if constexpr (F16) sm.sc[par ^ 1][64 * wq + lane] = cb < cend ? scn : 1.f;
            }
            if constexpr (AHEAD == 3 && !NOREAD) lgkm_wait();
            // trailing group: its k-step + 1 landed before the barrier
            if (trail && !NODMA) vm_wait();
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!NOBAR) __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            // ================= MFMA window =================
            if constexpr (AHEAD == 2 && !NOREAD) {
                lgkm_wait();
                __builtin_amdgcn_sched_barrier(0);
            }
            __builtin_amdgcn_s_setprio(1);
            mfmas(0, WCF);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            if (lead && !NODMA) vm_wait();
            if constexpr (!NOBAR) __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            so = (so + (uint32_t)(BC * KB * 2)) & (uint32_t)(NSLOT * BC * KB * 2 - 1);
        }
        par ^= 1;
    }
    if (wc == 0 && !NOBAR) __builtin_amdgcn_s_barrier();  // match the trailing group's extra window
    if (ntile > 0) check(cbeg + (ntile - 1) * cstr, par ^ 1, diag0 && ntile == 1);
    if (ns > 0) flush();
    // the re-staged pieces past the last k-step land before the LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace ksw2
}  // namespace mn
