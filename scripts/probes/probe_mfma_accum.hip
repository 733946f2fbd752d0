// Probe: accumulation error of v_mfma_f32_16x16x32_{bf16,f16} chains against
// the exact sum, to sanity-check the certification bound of the K1 sweep
// (|acc - exact| <= 2 (dp + 33) u (|acc0| + sum |a_k b_k|),
// i.e. <= 2u per addition in any order, products exact).
// For every output element: ratio = |got - exact| / (u * (|c0| + sum|a b|)).
//   hipcc --offload-arch=gfx950 -O3 probe_mfma_accum.hip -o probe_mfma_accum
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// one wave per case: A [16][K], B [K][16] (K = 32 nk), C0 [16][16]
template <bool F16>
__global__ void k_chain(const uint16_t *A, const uint16_t *B, const float *C0, int nk,
                        float *out) {
    const int lane = threadIdx.x, cs = blockIdx.x;
    const int K = 32 * nk;
    const uint16_t *a = A + (size_t)cs * 16 * K, *b = B + (size_t)cs * K * 16;
    f32x4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = C0[(size_t)cs * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)];
    for (int t = 0; t < nk; ++t) {
        uint16_t fa[8], fb[8];
        for (int e = 0; e < 8; ++e) {
            const int k = 32 * t + 8 * (lane >> 4) + e;
            fa[e] = a[(lane & 15) * K + k];
            fb[e] = b[k * 16 + (lane & 15)];
        }
        if constexpr (F16) {
            f16x8 x, y;
            __builtin_memcpy(&x, fa, 16);
            __builtin_memcpy(&y, fb, 16);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, acc, 0, 0, 0);
        } else {
            bf16x8 x, y;
            __builtin_memcpy(&x, fa, 16);
            __builtin_memcpy(&y, fb, 16);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc, 0, 0, 0);
        }
    }
    for (int r = 0; r < 4; ++r) out[(size_t)cs * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[r];
}

static uint16_t to_bits(double v, bool f16) {
    if (f16) { _Float16 h = (_Float16)v; uint16_t u; std::memcpy(&u, &h, 2); return u; }
    float f = (float)v; uint32_t u; std::memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
static double from_bits(uint16_t u, bool f16) {
    if (f16) { _Float16 h; std::memcpy(&h, &u, 2); return (double)h; }
    uint32_t w = (uint32_t)u << 16; float f; std::memcpy(&f, &w, 4); return f;
}

int main() {
    const int cases = 512;
    std::mt19937_64 rng(42);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(-1.0, 1.0);
    for (int f16 = 0; f16 < 2; ++f16)
        for (int nk : {1, 24, 96})
            for (int mode = 0; mode < 4; ++mode) {
                // mode 0: uniform, c0 = 0; 1: uniform, large c0 cancelling the
                // dot (the sweep's acc0); 2: products of mixed magnitudes;
                // 3: all products positive, large c0 of the opposite sign
                const int K = 32 * nk;
                std::vector<uint16_t> A((size_t)cases * 16 * K), B((size_t)cases * K * 16);
                std::vector<float> C0((size_t)cases * 256), out((size_t)cases * 256);
                const double sc = f16 ? 1024.0 : 1.0;
                for (size_t i = 0; i < A.size(); ++i) {
                    double v = mode == 2 ? ud(rng) * std::pow(2.0, (double)(rng() % 12) - 6) : ud(rng);
                    if (mode == 3) v = std::fabs(v);
                    A[i] = to_bits(v * sc, f16);
                }
                for (size_t i = 0; i < B.size(); ++i) {
                    double v = mode == 2 ? ud(rng) * std::pow(2.0, (double)(rng() % 12) - 6) : ud(rng);
                    if (mode == 3) v = std::fabs(v);
                    B[i] = to_bits(v * sc, f16);
                }
                std::vector<double> ex((size_t)cases * 256), mag((size_t)cases * 256);
                for (int c = 0; c < cases; ++c)
                    for (int i = 0; i < 16; ++i)
                        for (int j = 0; j < 16; ++j) {
                            double s = 0, m = 0;
                            for (int k = 0; k < K; ++k) {
                                const double p = from_bits(A[((size_t)c * 16 + i) * K + k], f16) *
                                                 from_bits(B[((size_t)c * K + k) * 16 + j], f16);
                                s += p;  // exact enough: checked against a long-double pass below
                                m += std::fabs(p);
                            }
                            double c0 = 0.0;
                            if (mode == 1) c0 = (double)(float)(-s + nd(rng) * 0.01 * std::sqrt(m));
                            if (mode == 3) c0 = (double)(float)(-s);
                            C0[(size_t)c * 256 + i * 16 + j] = (float)c0;
                            long double se = c0;
                            for (int k = 0; k < K; ++k)
                                se += (long double)from_bits(A[((size_t)c * 16 + i) * K + k], f16) *
                                      (long double)from_bits(B[((size_t)c * K + k) * 16 + j], f16);
                            ex[(size_t)c * 256 + i * 16 + j] = (double)se;
                            mag[(size_t)c * 256 + i * 16 + j] = std::fabs(c0) + m;
                        }
                uint16_t *dA, *dB; float *dC, *dO;
                hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
                hipMalloc(&dC, C0.size() * 4); hipMalloc(&dO, out.size() * 4);
                hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
                hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
                hipMemcpy(dC, C0.data(), C0.size() * 4, hipMemcpyHostToDevice);
                if (f16) hipLaunchKernelGGL(k_chain<true>, dim3(cases), dim3(64), 0, 0, dA, dB, dC, nk, dO);
                else hipLaunchKernelGGL(k_chain<false>, dim3(cases), dim3(64), 0, 0, dA, dB, dC, nk, dO);
                hipMemcpy(out.data(), dO, out.size() * 4, hipMemcpyDeviceToHost);
                double worst = 0, mean = 0;
                for (size_t e = 0; e < out.size(); ++e) {
                    const double r = std::fabs((double)out[e] - ex[e]) / (std::ldexp(1.0, -24) * mag[e]);
                    worst = std::max(worst, r);
                    mean += r;
                }
                printf("%s nk=%3d (K=%4d) mode=%d: max |err| / (u sum|terms|) = %.3f  mean %.4f"
                       "  [bound 2 (K + 33) = %d]\n", f16 ? "f16 " : "bf16", nk, K, mode, worst,
                       mean / out.size(), 2 * (K + 33));
                hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dO);
            }
    return 0;
}
