// glibc_f32.hpp — the platform libm's logf / expf restated on the device, so
// the kernels' f32 ln / exp are bit-identical to the reference's.
//
// Rust's f32::ln / f32::exp lower to calls of the C library's logf / expf;
// on Linux that is glibc (>= 2.28), whose single-precision log / exp are the
// table + polynomial algorithms of ARM's optimized-routines (sysdeps/ieee754/
// flt-32/e_logf.c, e_expf.c; data e_logf_data.c, e_exp2f_data.c: a 16-entry
// {1/c, log c} table + a degree-4 log1p polynomial, and a 32-entry 2^(i/32)
// table + a degree-3 polynomial, all evaluated in double and rounded once).
// The constants below are those tables.  On x86-64 with FMA (every server CPU
// the reference would run on) glibc dispatches to the variant compiled with
// -mfma: in expf that fuses x * InvLn2N into both the rounding shift and the
// reduced argument; the fused forms are written out here.  Verification:
// oracle/glibc_check.c compares these restatements with the host glibc for
// EVERY f32 input (logf: all 2^31 non-negative + the negative/NaN paths;
// expf: all 2^32 inputs) — 0 mismatches (tests/test_oracle.py runs a strided
// subset on every CPU test run; scripts/glibc_tables.py re-derives the
// tables from the host libm).  Pure double arithmetic (v_fma_f64 is IEEE),
// no f32 denormal flushing (the library's kernels keep denorm mode 3).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mn {
namespace glibc {

__device__ __constant__ static const double kLogT[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
constexpr double kLogA0 = -0x1.00ea348b88334p-2, kLogA1 = 0x1.5575b0be00b6ap-2,
                 kLogA2 = -0x1.ffffef20a4123p-2;
constexpr double kLn2 = 0x1.62e42fefa39efp-1;

__device__ __constant__ static const uint64_t kExpT[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51,
    0x3fef72b83c7d517b, 0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1,
    0x3fef06fe0a31b715, 0x3feef1a7373aa9cb, 0x3feedea64c123422, 0x3feece086061892d,
    0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429, 0x3feea47eb03a5585,
    0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d,
    0x3feee89f995ad3ad, 0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069,
    0x3fef5818dcfba487, 0x3fef7c97337b9b5f, 0x3fefa4afa2a490da, 0x3fefd0765b6e4540};
constexpr double kExpC0 = 0x1.c6af84b912394p-20, kExpC1 = 0x1.ebfce50fac4f3p-13,
                 kExpC2 = 0x1.62e42ff0c52d6p-6;
constexpr double kInvLn2N = 0x1.71547652b82fep+5, kShift = 0x1.8p+52;

// glibc logf (e_logf.c): x = 2^k z, z in [OFF, 2 OFF); log x = log1p(z/c - 1)
// + log c + k ln2 with c the centre of z's 1/16 subinterval
__device__ __forceinline__ float logf(float x) {
    uint32_t ix = __float_as_uint(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2u == 0u) return -__builtin_inff();            // log(+-0) = -inf
        if (ix == 0x7f800000u) return x;                        // log(inf) = inf
        if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u) return __builtin_nanf("");
        // subnormal: the bits of x * 0x1p23f (exact), by integer ops
        const int sh = __clz(ix) - 8;
        ix = (((uint32_t)(24 - sh)) << 23) | ((ix << sh) & 0x7fffffu);
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16u);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = kLogT[i][0], logc = kLogT[i][1];
    const double z = (double)__uint_as_float(iz);
    const double r = __builtin_fma(z, invc, -1.0);
    const double y0 = __builtin_fma((double)k, kLn2, logc);
    const double r2 = r * r;
    double y = __builtin_fma(kLogA1, r, kLogA2);
    y = __builtin_fma(kLogA0, r2, y);
    y = __builtin_fma(y, r2, y0 + r);
    return (float)y;
}

// glibc expf (e_expf.c, the -mfma variant): x N / ln2 = k + r, exp x =
// 2^(k/N) 2^(r/N), N = 32
__device__ __forceinline__ float expf(float x) {
    const double xd = (double)x;
    const uint32_t abstop = (__float_as_uint(x) >> 20) & 0x7ffu;
    if (abstop >= 0x42bu) {  // |x| >= 88 or NaN
        if (__float_as_uint(x) == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8u) return x + x;
        if (x > 0x1.62e42ep6f) return __builtin_inff();
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    double kd = __builtin_fma(kInvLn2N, xd, kShift);
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd -= kShift;
    const double r = __builtin_fma(kInvLn2N, xd, -kd);
    uint64_t t = kExpT[ki % 32u];
    t += ki << 47;
    const double s = __longlong_as_double((long long)t);
    const double z = __builtin_fma(kExpC0, r, kExpC1);
    const double r2 = r * r;
    double y = __builtin_fma(kExpC2, r, 1.0);
    y = __builtin_fma(z, r2, y);
    y = y * s;
    return (float)y;
}

}  // namespace glibc
}  // namespace mn
