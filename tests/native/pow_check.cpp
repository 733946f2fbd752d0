// Host check of the restated glibc pow (matternet-rs_amd/csrc/glibc_f64.hpp)
// against the host libm's pow: random (x, y) over wide ranges, the weight
// kernel's (d / sigma)^p with p in {0.5, 2, 3, 2.7, random}, and special
// values.  Built with g++ (no HIP): tests/test_oracle.py.
#define __host__
#define __device__
#define __constant__
#include "glibc_f64.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

static uint64_t bits(double v) { uint64_t u; memcpy(&u, &v, 8); return u; }

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 g(1234);
    long bad = 0, tot = 0;
    auto check = [&](double x, double y) {
        const double a = mn::glibc::pow_glibc(x, y), b = std::pow(x, y);
        ++tot;
        if (bits(a) != bits(b) && !(std::isnan(a) && std::isnan(b))) {
            if (bad < 10) printf("mismatch x=%a y=%a got %a want %a\n", x, y, a, b);
            ++bad;
        }
    };
    std::uniform_real_distribution<double> u01(0.0, 1.0);
    const double ps[] = {0.5, 2.0, 3.0, 2.7, 1.5, 0.25, 7.0, -1.0, -2.5};
    for (long i = 0; i < n; ++i) {
        // weights: distance / sigma in [0, 4) and a wide random range
        const double x1 = 4.0 * u01(g);
        const double x2 = std::ldexp(u01(g) + 0.5, (int)(g() % 200) - 100);
        for (double p : ps) { check(x1, p); }
        check(x2, ps[i % 9]);
        // random bit patterns of positive x, y in a moderate range
        const double x3 = std::ldexp(u01(g) + 0.5, (int)(g() % 2000) - 1000);
        const double y3 = (u01(g) - 0.5) * std::ldexp(1.0, (int)(g() % 20) - 6);
        check(x3, y3);
        // subnormal / negative x with integer y
        const double x4 = std::ldexp(u01(g), -1060);
        check(x4, 0.5 + (double)(i % 7));
        check(-x1, (double)(i % 5) - 2.0);
        // results near and below the normal range, and near overflow
        check(0.5 * (1.0 + u01(g)), 1000.0 + 80.0 * u01(g));
        check(2.0 * (1.0 + u01(g)), 1000.0 + 30.0 * u01(g));
        check(0.5 + 0.5 * u01(g), -(1000.0 + 30.0 * u01(g)));
    }
    const double sp[] = {0.0, -0.0, 1.0, -1.0, INFINITY, -INFINITY, NAN, 0x1p-1074, 0x1p1023, 2.0, 0.5};
    for (double x : sp)
        for (double y : sp) check(x, y);
    printf("pow checks %ld mismatches %ld\n", tot, bad);
    return bad != 0;
}
