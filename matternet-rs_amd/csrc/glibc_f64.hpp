// glibc_f64.hpp — the platform libm's f64 pow restated (device and host), so
// the kernels' weights (d / sigma)^p are bit-identical to the reference's.
//
// Rust's f64::powf lowers to the C library's pow (src_legacy/laplacian.rs:256
// `(distance / sigma).powf(p)`, sorted_index.rs:65 `2.0_f64.powf(p)`); on
// Linux that is glibc (>= 2.28), whose pow is ARM optimized-routines'
// algorithm (sysdeps/ieee754/dbl-64/e_pow.c):
//   log(x) in double-double: x = 2^k z, z / c - 1 = r exactly (a 128-entry
//     {1/c, log c, log c tail} table), k ln2 + log c + r + A[0] r^2 with the
//     error terms carried in lo, and r^3 times a degree-5 polynomial;
//   y log(x) = ehi + elo (one fma for the product's error);
//   exp(ehi + elo) = 2^(k/128) (table: scale bits and a tail) (1 + tmp), tmp a
//     degree-5 polynomial of the reduced argument, scale + scale tmp;
//   special cases: x or y zero / inf / nan, x < 0 (y integer: the sign), |y|
//     tiny or huge, subnormal x, results that overflow / underflow
//     (specialcase: the 2^k scaling split so the last rounding is the only
//     one).
// On x86-64 with FMA (every server CPU the reference would run on) glibc
// dispatches to the variant compiled with -mfma, where __FP_FAST_FMA selects
// the fma forms and GCC contracts a * b + c with a single-use product into
// fma; those fused forms are written out here.  The tables are the host
// libm's own (glibc_f64_tables.hpp, scripts/glibc_pow_tables.py).
// Verification: tests/native/pow_check.cpp compares this header (host build)
// with the host pow over random and structured (x, p) — 0 mismatches
// (tests/test_oracle.py) — and the GPU test compares the device build.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "glibc_f64_tables.hpp"

namespace mn {
namespace glibc {

__host__ __device__ inline uint64_t d2u(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
__host__ __device__ inline double u2d(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}
__host__ __device__ inline uint32_t top12(double x) { return (uint32_t)(d2u(x) >> 52); }

__host__ __device__ inline double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

__host__ __device__ inline void pow_log_entry(int i, double &invc, double &logc, double &logct) {
#ifdef __HIP_DEVICE_COMPILE__
    invc = kPowT[i][0];
    logc = kPowT[i][1];
    logct = kPowT[i][2];
#else
    invc = kPowTHost[i][0];
    logc = kPowTHost[i][1];
    logct = kPowTHost[i][2];
#endif
}
__host__ __device__ inline uint64_t exp_entry(int i) {
#ifdef __HIP_DEVICE_COMPILE__
    return kPowExpT[i];
#else
    return kPowExpTHost[i];
#endif
}

// log(x) = hi + tail for the bits ix of a positive normal (or normalised) x
__host__ __device__ inline double pow_log_inline(uint64_t ix, double *tail) {
    constexpr uint64_t OFF = 0x3fe6955500000000ull;
    const uint64_t tmp = ix - OFF;
    const int i = (int)((tmp >> (52 - 7)) % 128);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const double z = u2d(iz);
    const double kd = (double)k;
    double invc, logc, logctail;
    pow_log_entry(i, invc, logc, logctail);
    const double r = fma_(z, invc, -1.0);
    // k Ln2 + log(c) + r
    const double t1 = fma_(kd, kPowLn2hi, logc);
    const double t2 = t1 + r;
    const double lo1 = fma_(kd, kPowLn2lo, logctail);
    const double lo2 = t1 - t2 + r;
    const double ar = kPowA[0] * r;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double hi = t2 + ar2;
    const double lo3 = fma_(ar, r, -ar2);
    const double lo4 = t2 - hi + ar2;
    // p = log1p(r) - r - A[0] r^2 (the product ar3 * q fused into the sum)
    const double q = fma_(ar2, fma_(ar2, fma_(r, kPowA[6], kPowA[5]), fma_(r, kPowA[4], kPowA[3])),
                          fma_(r, kPowA[2], kPowA[1]));
    const double lo = fma_(ar3, q, lo1 + lo2 + lo3 + lo4);
    const double y = hi + lo;
    *tail = hi - y + lo;
    return y;
}

// results past the normal range: scale 2^k split so that the final rounding
// is the only one (e_exp.c specialcase)
__host__ __device__ inline double pow_specialcase(double tmp, uint64_t sbits, uint64_t ki) {
    if ((ki & 0x80000000ull) == 0) {
        // k > 0: the exponent of scale might have overflowed by <= 460
        sbits -= 1009ull << 52;
        const double scale = u2d(sbits);
        return 0x1p1009 * fma_(scale, tmp, scale);
    }
    // k < 0: avoid the double rounding of a subnormal result
    // (scale * tmp has two uses here: GCC keeps the product, no fma)
    sbits += 1022ull << 52;
    const double scale = u2d(sbits);
    const double st = scale * tmp;
    double y = scale + st;
    if ((y < 0 ? -y : y) < 1.0) {
        const double one = y < 0 ? -1.0 : 1.0;
        const double lo = scale - y + st;
        const double hi = one + y;
        const double lo2 = one - hi + y + lo;
        y = (hi + lo2) - one;
        if (y == 0) y = u2d(sbits & 0x8000000000000000ull);  // -0 / +0
    }
    return 0x1p-1022 * y;
}

__host__ __device__ inline double pow_exp_inline(double x, double xtail, uint32_t sign_bias) {
    uint32_t abstop = top12(x) & 0x7ff;
    if (abstop - top12(0x1p-54) >= top12(512.0) - top12(0x1p-54)) {
        if (abstop - top12(0x1p-54) >= 0x80000000u) {
            // tiny x: 1 (rounded as 1 + x)
            const double one = 1.0 + x;
            return sign_bias ? -one : one;
        }
        if (abstop >= top12(1024.0)) {
            const double huge = 0x1p769, tiny = 0x1p-767;
            if (d2u(x) >> 63) return sign_bias ? -tiny * tiny : tiny * tiny;  // underflow
            return sign_bias ? -huge * huge : huge * huge;                   // overflow
        }
        abstop = 0;  // large |x|: specialcase below
    }
    // exp(x) = 2^(k/N) exp(r), x = ln2/N k + r
    double kd = fma_(kPowExpInvLn2N, x, kPowExpShift);
    const uint64_t ki = d2u(kd);
    kd -= kPowExpShift;
    double r = fma_(kd, kPowExpNegLn2loN, fma_(kd, kPowExpNegLn2hiN, x));
    r += xtail;
    const uint64_t idx = 2 * (ki % 128);
    const uint64_t top = (ki + sign_bias) << (52 - 7);
    const double tl = u2d(exp_entry((int)idx));
    const uint64_t sbits = exp_entry((int)idx + 1) + top;
    const double r2 = r * r;
    const double tmp = fma_(r2 * r2, fma_(r, kPowExpC5, kPowExpC4), fma_(r2, fma_(r, kPowExpC3, kPowExpC2), tl + r));
    if (abstop == 0) return pow_specialcase(tmp, sbits, ki);
    const double scale = u2d(sbits);
    return fma_(scale, tmp, scale);
}

// 0: not an integer, 1: odd integer, 2: even integer (bits of y)
__host__ __device__ inline int pow_checkint(uint64_t iy) {
    const int e = (int)(iy >> 52 & 0x7ff);
    if (e < 0x3ff) return 0;
    if (e > 0x3ff + 52) return 2;
    if (iy & ((1ull << (0x3ff + 52 - e)) - 1)) return 0;
    if (iy & (1ull << (0x3ff + 52 - e))) return 1;
    return 2;
}

__host__ __device__ inline bool pow_zeroinfnan(uint64_t i) { return 2 * i - 1 >= 2 * d2u(__builtin_inf()) - 1; }

// glibc pow (x86-64 FMA variant), restated
__host__ __device__ inline double pow_glibc(double x, double y) {
    uint32_t sign_bias = 0;
    uint64_t ix = d2u(x), iy = d2u(y);
    uint32_t topx = top12(x), topy = top12(y);
    if (topx - 0x001 >= 0x7ff - 0x001 || (topy & 0x7ff) - 0x3be >= 0x43e - 0x3be) {
        if (pow_zeroinfnan(iy)) {
            if (2 * iy == 0) return 1.0;
            if (ix == d2u(1.0)) return 1.0;
            if (2 * ix > 2 * d2u(__builtin_inf()) || 2 * iy > 2 * d2u(__builtin_inf())) return x + y;
            if (2 * ix == 2 * d2u(1.0)) return 1.0;
            if ((2 * ix < 2 * d2u(1.0)) == !(iy >> 63)) return 0.0;  // |x| < 1 && y == inf or |x| > 1 && y == -inf
            return y * y;
        }
        if (pow_zeroinfnan(ix)) {
            double x2 = x * x;
            if (ix >> 63 && pow_checkint(iy) == 1) x2 = -x2;
            return (iy >> 63) ? 1 / x2 : x2;
        }
        // x and y are non-zero finite
        if (ix >> 63) {
            const int yint = pow_checkint(iy);
            if (yint == 0) return __builtin_nan("");  // (x - x) / (x - x): invalid
            if (yint == 1) sign_bias = 0x800 << 7;
            ix &= 0x7fffffffffffffffull;
            topx &= 0x7ff;
        }
        if ((topy & 0x7ff) - 0x3be >= 0x43e - 0x3be) {
            // |y| < 2^-65 or |y| >= 2^63 (and x finite nonzero)
            if (ix == d2u(1.0)) return 1.0;
            if ((topy & 0x7ff) < 0x3be) return ix > d2u(1.0) ? 1.0 + y : 1.0 - y;  // |y| tiny
            const double huge = 0x1p769, tiny = 0x1p-767;
            return (ix > d2u(1.0)) == (topy < 0x800) ? huge * huge : tiny * tiny;
        }
        if (topx == 0) {
            // subnormal x: normalise so the exponent becomes negative
            ix = d2u(u2d(ix) * 0x1p52);
            ix &= 0x7fffffffffffffffull;
            ix -= 52ull << 52;
        }
    }
    double lo;
    const double hi = pow_log_inline(ix, &lo);
    const double ehi = y * hi;
    const double elo = fma_(y, lo, fma_(y, hi, -ehi));
    return pow_exp_inline(ehi, elo, sign_bias);
}

}  // namespace glibc
}  // namespace mn
