// Probe: sustained bf16 MFMA rate on random register operands (no memory
// traffic) — the practical ceiling under load (DVFS) for the Gram kernels.
//   hipcc --offload-arch=gfx950 -O3 probe_mfma_peak.hip -o probe_mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int SHAPE>
__global__ __launch_bounds__(512) void k_peak(int iters, float *out, unsigned seed) {
    const int lane = threadIdx.x;
    bf16x8 a[4], b[4];
    unsigned z = seed ^ (lane * 2654435761u) ^ (blockIdx.x * 40503u);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) {
            z = z * 1664525u + 1013904223u;
            a[i][j] = (__bf16)((float)(z >> 8) * 0x1p-24f - 0.5f);
            z = z * 1664525u + 1013904223u;
            b[i][j] = (__bf16)((float)(z >> 8) * 0x1p-24f - 0.5f);
        }
    float s = 0.f;
    if constexpr (SHAPE == 0) {
        f32x16 acc[8];
        for (int t = 0; t < 8; ++t) for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[j], b[(j + t) & 3], acc[t], 0, 0, 0);
        }
        for (int t = 0; t < 8; ++t) for (int r = 0; r < 16; ++r) s += acc[t][r];
    } else {
        f32x4 acc[32];
        for (int t = 0; t < 32; ++t) for (int r = 0; r < 4; ++r) acc[t][r] = 0.f;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int t = 0; t < 32; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j + (t & 1) * 2], b[(j + t) & 3], acc[t], 0, 0, 0);
        }
        for (int t = 0; t < 32; ++t) for (int r = 0; r < 4; ++r) s += acc[t][r];
    }
    if (s == 1.2345f) out[0] = s;
}

int main() {
    float *out;
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 2, iters = 20000;
    for (int shape = 0; shape < 2; ++shape) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            if (shape == 0) hipLaunchKernelGGL(k_peak<0>, dim3(blocks), dim3(512), 0, 0, iters, out, 7u + rep);
            else hipLaunchKernelGGL(k_peak<1>, dim3(blocks), dim3(512), 0, 0, iters, out, 7u + rep);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // per wave per iter: 32 MFMAs of 32768 flops (32x32x16) or 64 of 16384 (16x16x32)
            const double fl = (double)blocks * 8 * iters * 32 * 32768.0;
            printf("shape %s rep %d: %.3f ms  %.1f TFLOP/s\n", shape ? "16x16x32" : "32x32x16", rep, ms,
                   fl / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
