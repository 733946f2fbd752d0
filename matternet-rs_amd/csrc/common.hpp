// common.hpp — shared plumbing for the matternet HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "matternet_hip.h"

namespace mn {

// Thread-local error text behind mn_last_error().
void set_error(const char *fmt, ...);
void clear_error();

// MN_DEBUG_SYNC=1: synchronise after every launch so a fault names its kernel.
bool debug_sync();

// Tuning knobs (A/B experiments, timing probes whose outputs are invalid):
// read from the environment ONLY in the tuning build (-DMN_TUNING,
// libmatternet_hip_tuning.so, loaded by scripts/ on request).  The release
// library ignores every MN_* variable except the diagnostics MN_DEBUG_SYNC
// and MN_X1_DEBUG, which never change an output.
#ifdef MN_TUNING
inline const char *knob(const char *name) { return getenv(name); }
#else
inline const char *knob(const char *) { return nullptr; }
#endif
// integer knob with a default (the release build: always the default)
inline int knob_int(const char *name, int dflt) {
    const char *e = knob(name);
    return (e && *e) ? atoi(e) : dflt;
}

// Grow-only device scratch, one set of slots per (thread, device).  Growing
// frees the old block (hipFree synchronises), so never call it while kernels
// that use that slot are in flight on another stream of this thread.
void *scratch(int slot, size_t bytes);

enum ScratchSlot {
    kSlotNorms = 0,
    kSlotNorms2,
    kSlotFlags,
    kSlotLists,
    kSlotListMeta,
    kSlotFallback,
    kSlotGeneric0,
    kSlotGeneric1,
    kSlotGeneric2,
    kSlotGeneric3,
    kSlotX1QR,     // MN_KNN_BF16X1: query rows, bf16 row-major (phase 1)
    kSlotX1QK,     //                query rows, bf16 KB32 (phase 2)
    kSlotX1CR,     //                corpus rows, bf16 row-major
    kSlotX1CK,     //                corpus rows, bf16 KB32
    kSlotX1Aux,    //                per-row norms / thresholds / bounds
    kSlotX1Buf2,   //                phase-2 candidate buffer
    kSlotX1Meta2,  //                phase-2 counts
    kSlotX1Esc,    //                escalated rows (gathered queries, lists)
    kSlotPerm,     // corpus visiting order (+ permuted norms / sample rows)
    kSlotL2List,   // MN_L2: the extended L2^2 list before the root order
    kSlotSymOrd,   // MN_KNN_BF16X1 symmetric sweep: tau0 order + per-position arrays
    kSlotSymTab,   //                block table
    kSlotSortTmp,  // radix-sort temporary storage
    kNumSlots
};

// The calling thread's non-blocking side stream on the current device
// (library-owned, created on first use) for work that runs concurrently with
// the caller's stream; nullptr on failure.
hipStream_t side_stream();
// Make `waiter` wait for all work issued so far on `on`.
hipError_t stream_wait(hipStream_t waiter, hipStream_t on);

// Per-call HIP-event timer (active only when requested).
struct Timer {
    bool on = false;
    hipStream_t s = nullptr;
    hipEvent_t ev[8] = {};
    int n = 0;
    void start(bool enable, hipStream_t stream);
    void mark();               // records the next event
    float ms(int a, int b);    // elapsed between marks a and b (after sync)
    ~Timer();
};

}  // namespace mn

#define MN_HIP_TRY(expr)                                                        \
    do {                                                                        \
        hipError_t _e = (expr);                                                 \
        if (_e != hipSuccess) {                                                 \
            mn::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),\
                          __FILE__, __LINE__);                                  \
            return MN_EHIP;                                                     \
        }                                                                       \
    } while (0)

#define MN_KCHECK(stream, name)                                                 \
    do {                                                                        \
        MN_HIP_TRY(hipGetLastError());                                          \
        if (mn::debug_sync()) {                                                 \
            hipError_t _e = hipStreamSynchronize(stream);                       \
            if (_e != hipSuccess) {                                             \
                mn::set_error("%s: %s (%s:%d)", name, hipGetErrorString(_e),    \
                              __FILE__, __LINE__);                              \
                return MN_EHIP;                                                 \
            }                                                                   \
        }                                                                       \
    } while (0)

#define MN_REQUIRE(cond, code, ...)                                             \
    do {                                                                        \
        if (!(cond)) {                                                          \
            mn::set_error(__VA_ARGS__);                                         \
            return (code);                                                      \
        }                                                                       \
    } while (0)

// ---- device helpers ------------------------------------------------------

namespace mn {

// (dist, idx) lexicographic total order used by every selection in the path:
// the reference's stable sort by distance over ascending j (mst.rs:344).
__device__ __forceinline__ bool key_less(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
}
__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

// Bitonic sort of 64*NR (key, idx) pairs held one per lane per register:
// element e = lane + 64*r.  Ascending by (key, idx).  Whole wave must call.
template <int NR, typename T>
__device__ __forceinline__ void wave_bitonic_sort(T (&d)[NR], int (&ix)[NR]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 2; k <= 64 * NR; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int pr = r ^ (j >> 6);
                    if (pr > r) {
                        const int e = lane + 64 * r;
                        const bool asc = (e & k) == 0;
                        const bool sw = asc ? key_less(d[pr], ix[pr], d[r], ix[r])
                                            : key_less(d[r], ix[r], d[pr], ix[pr]);
                        if (sw) {
                            T td = d[r]; d[r] = d[pr]; d[pr] = td;
                            int ti = ix[r]; ix[r] = ix[pr]; ix[pr] = ti;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int e = lane + 64 * r;
                    const T pd = __shfl_xor(d[r], j);
                    const int pi = __shfl_xor(ix[r], j);
                    const bool asc = (e & k) == 0;
                    const bool lower = (e & j) == 0;
                    const bool keep_min = (asc == lower);
                    const bool take = keep_min ? key_less(pd, pi, d[r], ix[r])
                                               : key_less(d[r], ix[r], pd, pi);
                    if (take) { d[r] = pd; ix[r] = pi; }
                }
            }
        }
    }
}

// Correctly rounded f32 square root.  On gfx950 / ROCm 7.2 both sqrtf() and
// __fsqrt_rn() are NOT correctly rounded (measured: 1-ulp misses, e.g.
// sqrt(0x3da6a80c)); the f64 square root rounded to f32 is (53 >= 2*24+2, so
// the double rounding is innocuous) and matches Rust's IEEE f32::sqrt.
// Maxima of non-negative float bit patterns over a loop: keep them in
// registers and issue ONE atomic per wave at the end (a per-row atomicMax on
// one address serialises a whole launch at the memory-side atomic unit).
__device__ __forceinline__ void wave_atomic_umax(unsigned *p, unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o));
    if ((threadIdx.x & 63) == 0 && v != 0u) atomicMax(p, v);
}

__device__ __forceinline__ float sqrt_rn_f32(float x) { return (float)__builtin_sqrt((double)x); }

// Ordered fold acc = (((acc + b[0]) + b[1]) + ...) over N values in LDS that
// every lane reads as broadcasts (same address: conflict-free).  The loads
// go out in register batches of 32 values, the next batch issued before the
// current batch's adds, so the chain waits on the add latency only.
template <int N>
__device__ __forceinline__ double lds_chain_f64(double acc, const double *b) {
    static_assert(N % 64 == 0, "chain length must be a multiple of 64");
    constexpr int NB = N / 32;  // batches of 16 double2
    const double2 *b2 = reinterpret_cast<const double2 *>(b);
    double2 v[2][16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[0][q] = b2[q];
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
    for (int bt = 0; bt < NB; ++bt) {
        // the next batch's 16 reads go out before this batch's 32 adds (the
        // scheduler would otherwise interleave them and expose the LDS
        // latency on the chain)
        if (bt + 1 < NB) {
#pragma unroll
            for (int q = 0; q < 16; ++q) v[(bt + 1) & 1][q] = b2[16 * (bt + 1) + q];
            __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            acc = acc + v[bt & 1][q].x;
            acc = acc + v[bt & 1][q].y;
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 32, 0);
    }
    return acc;
}
template <int N>
__device__ __forceinline__ float lds_chain_f32(float acc, const float *b) {
    static_assert(N % 128 == 0, "chain length must be a multiple of 128");
    constexpr int NB = N / 32;  // batches of 8 float4
    const float4 *b4 = reinterpret_cast<const float4 *>(b);
    float4 v[2][8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[0][q] = b4[q];
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int bt = 0; bt < NB; ++bt) {
        if (bt + 1 < NB) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[(bt + 1) & 1][q] = b4[8 * (bt + 1) + q];
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            acc = acc + v[bt & 1][q].x;
            acc = acc + v[bt & 1][q].y;
            acc = acc + v[bt & 1][q].z;
            acc = acc + v[bt & 1][q].w;
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 32, 0);
    }
    return acc;
}

// Read element `pos` of a register-distributed array (wave-uniform pos).
template <int NR, typename T>
__device__ __forceinline__ T wave_elem(const T (&d)[NR], int pos) {
    const int r = pos >> 6, l = pos & 63;
    T v = d[0];
#pragma unroll
    for (int q = 1; q < NR; ++q) if (q == r) v = d[q];
    return __shfl(v, l);
}

// Store a wave's sorted (key, idx) list (element e = lane + 64 r) as the k
// entries out[0..k): the first keff, then (-1, +inf) padding.  k <= 64 NR.
template <int NR, typename T>
__device__ __forceinline__ void wave_store_list(const T (&d)[NR], const int (&ix)[NR], int k,
                                                int keff, int32_t *__restrict__ oi,
                                                T *__restrict__ od) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = lane + 64 * r;
        if (e < k) {
            const bool ok = e < keff;
            oi[e] = ok ? ix[r] : -1;
            od[e] = ok ? d[r] : (T)__builtin_inf();
        }
    }
}

// Keys-only ascending bitonic sort of 64*NR floats (element e = lane + 64*r),
// min/max exchanges (no tie-break needed).  NaN-free inputs.  Whole wave.
template <int NR>
__device__ __forceinline__ void wave_sort_f32(float (&d)[NR]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 2; k <= 64 * NR; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int pr = r ^ (j >> 6);
                    if (pr > r) {
                        const bool asc = ((lane + 64 * r) & k) == 0;
                        const float lo = fminf(d[r], d[pr]), hi = fmaxf(d[r], d[pr]);
                        d[r] = asc ? lo : hi;
                        d[pr] = asc ? hi : lo;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int e = lane + 64 * r;
                    const float pd = __shfl_xor(d[r], j);
                    const bool keep_min = (((e & k) == 0) == ((e & j) == 0));
                    d[r] = keep_min ? fminf(d[r], pd) : fmaxf(d[r], pd);
                }
            }
        }
    }
}

template <int NR>
__device__ __forceinline__ float wave_elem_f32(const float (&d)[NR], int pos) {
    return wave_elem<NR, float>(d, pos);
}

}  // namespace mn
