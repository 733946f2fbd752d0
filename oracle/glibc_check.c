/* glibc_check.c — TEST INFRASTRUCTURE (checker only; the product never links
 * this).  Two things the GPU kernels' f32 ln / exp parity rests on:
 *
 *  1. or_libm_f32: the HOST glibc logf / expf — what the reference's f32::ln /
 *     f32::exp call (Rust lowers them to libm calls; surfface-core/src/
 *     distance.rs:102, 283-289) — over an array or a range of bit patterns,
 *     so tests compare the device restatement (mn_libm_f32) with it.
 *  2. or_glibc_restated_check: a host copy of the restatement in
 *     matternet-rs_amd/csrc/glibc_f32.hpp (same tables, same operations)
 *     against the host glibc over every `stride`-th f32 bit pattern; the
 *     tables were read out of the host libm (scripts/glibc_tables.py) and a
 *     stride-1 run over all 2^32 inputs gives 0 mismatches for both.
 *
 * Algorithms: glibc >= 2.28 sysdeps/ieee754/flt-32/e_logf.c / e_expf.c (ARM
 * optimized-routines), x86-64 FMA dispatch variant. */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

#define OR_EINVAL (-1)

static const double LT[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
static const double LA0 = -0x1.00ea348b88334p-2, LA1 = 0x1.5575b0be00b6ap-2,
                    LA2 = -0x1.ffffef20a4123p-2, LN2 = 0x1.62e42fefa39efp-1;
static const uint64_t ET[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51,
    0x3fef72b83c7d517b, 0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1,
    0x3fef06fe0a31b715, 0x3feef1a7373aa9cb, 0x3feedea64c123422, 0x3feece086061892d,
    0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429, 0x3feea47eb03a5585,
    0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d,
    0x3feee89f995ad3ad, 0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069,
    0x3fef5818dcfba487, 0x3fef7c97337b9b5f, 0x3fefa4afa2a490da, 0x3fefd0765b6e4540};
static const double EC0 = 0x1.c6af84b912394p-20, EC1 = 0x1.ebfce50fac4f3p-13,
                    EC2 = 0x1.62e42ff0c52d6p-6, INVLN2N = 0x1.71547652b82fep+5,
                    SHIFT = 0x1.8p+52;

static inline uint32_t asu(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static inline float asf(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static inline uint64_t asu64(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double asd(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

static float r_logf(float x) {
    uint32_t ix = asu(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2u == 0u) return -INFINITY;
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u) return NAN;
        int sh = __builtin_clz(ix) - 8;
        ix = (((uint32_t)(24 - sh)) << 23) | ((ix << sh) & 0x7fffffu);
        ix -= 23u << 23;
    }
    uint32_t tmp = ix - 0x3f330000u;
    int i = (int)((tmp >> 19) % 16u);
    int k = (int32_t)tmp >> 23;
    uint32_t iz = ix - (tmp & 0xff800000u);
    double z = (double)asf(iz);
    double r = fma(z, LT[i][0], -1.0);
    double y0 = fma((double)k, LN2, LT[i][1]);
    double r2 = r * r;
    double y = fma(LA1, r, LA2);
    y = fma(LA0, r2, y);
    y = fma(y, r2, y0 + r);
    return (float)y;
}

static float r_expf(float x) {
    double xd = (double)x;
    uint32_t abstop = (asu(x) >> 20) & 0x7ffu;
    if (abstop >= 0x42bu) {
        if (asu(x) == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8u) return x + x;
        if (x > 0x1.62e42ep6f) return INFINITY;
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    double kd = fma(INVLN2N, xd, SHIFT);
    uint64_t ki = asu64(kd);
    kd -= SHIFT;
    double r = fma(INVLN2N, xd, -kd);
    uint64_t t = ET[ki % 32u] + (ki << 47);
    double s = asd(t);
    double z = fma(EC0, r, EC1);
    double r2 = r * r;
    double y = fma(EC2, r, 1.0);
    y = fma(z, r2, y);
    return (float)(y * s);
}

static inline int same_f32(float a, float b) {
    return asu(a) == asu(b) || (a != a && b != b);
}

int or_libm_f32(const float *x, int64_t n, uint32_t bits0, int fn, float *out, int nthreads) {
    if (!out || n < 0 || (fn != 0 && fn != 1)) return OR_EINVAL;
    (void)nthreads;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const float v = x ? x[i] : asf(bits0 + (uint32_t)i);
        out[i] = fn == 0 ? logf(v) : expf(v);
    }
    return 0;
}

int64_t or_libm_mismatch(uint32_t bits0, int64_t n, int fn, const float *got) {
    int64_t bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
    for (int64_t i = 0; i < n; ++i) {
        const float v = asf(bits0 + (uint32_t)i);
        const float ref = fn == 0 ? logf(v) : expf(v);
        bad += !same_f32(ref, got[i]);
    }
    return bad;
}

int64_t or_glibc_restated_check(int fn, int64_t stride) {
    if (stride < 1) stride = 1;
    int64_t bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
    for (int64_t u = 0; u < 0x100000000ll; u += stride) {
        const float v = asf((uint32_t)u);
        const float ref = fn == 0 ? logf(v) : expf(v);
        const float got = fn == 0 ? r_logf(v) : r_expf(v);
        bad += !same_f32(ref, got);
    }
    return bad;
}

/* the restatement's tables, for the CPU test that matches them against the
 * device header and the host libm bytes: 0 = log {invc, logc} x16 + A0 A1 A2
 * LN2 (36 doubles), 1 = exp table bits x32 (as doubles' bit patterns) + C0 C1 C2
 * INVLN2N SHIFT (37 values) */
int or_glibc_tables(int which, uint64_t *out) {
    if (!out) return OR_EINVAL;
    if (which == 0) {
        for (int i = 0; i < 16; ++i) { out[2 * i] = asu64(LT[i][0]); out[2 * i + 1] = asu64(LT[i][1]); }
        out[32] = asu64(LA0); out[33] = asu64(LA1); out[34] = asu64(LA2); out[35] = asu64(LN2);
        return 36;
    }
    for (int i = 0; i < 32; ++i) out[i] = ET[i];
    out[32] = asu64(EC0); out[33] = asu64(EC1); out[34] = asu64(EC2); out[35] = asu64(INVLN2N);
    out[36] = asu64(SHIFT);
    return 37;
}

/* the host glibc pow elementwise (what Rust's f64::powf calls): the checker
 * for the device restatement (glibc_f64.hpp; numpy's power may dispatch to a
 * vector math library instead of libm on AVX-512 hosts) */
int or_pow_f64(const double *x, const double *y, int64_t n, double *out) {
    if (!x || !y || !out || n < 0) return OR_EINVAL;
    for (int64_t i = 0; i < n; ++i) out[i] = pow(x[i], y[i]);
    return 0;
}
