// What paces the ordered f64 chains of knn_cos.hip (k_cos_exact_*,
// k_col_norms)?  One wave per CU (or four), no global traffic:
//   mode 0: dependent adds on register operands (the add latency floor)
//   mode 1: lds_chain_f64<256> over a resident LDS buffer (broadcast reads)
//   mode 2: mode 1 + the product phase (16 cvt/mul pairs + 8 ds_write_b128 a
//           lane per 256-element chunk, operands in registers)
// Prints shader cycles per chain element (s_memtime) and wall ms for 1M
// elements.   hipcc --offload-arch=gfx950 -O3 -I../../matternet-rs_amd/csrc probe_lds_chain.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "common.hpp"

using mn::lds_chain_f64;
constexpr int CH = 256, CHP = CH + 2;

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(double *out, long long *cyc, int nchunks) {
    __shared__ __attribute__((aligned(16))) double buf[4][2][4][CHP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, gl = lane & 15;
    for (int t = lane; t < 2 * 4 * CHP; t += 64) (&buf[w][0][0][0])[t] = 1e-3 * (t + 1);
    float ra[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) ra[u] = 1e-2f * (lane + u + 1);
    __syncthreads();
    double acc = -0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (MODE == 0) {
        double v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = 1e-3 * (lane + i + 1);
        for (int c = 0; c < nchunks; ++c) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int i = 0; i < 32; ++i) acc = acc + v[i];
        }
    } else {
        for (int c = 0; c < nchunks; ++c) {
            double *bb = buf[w][c & 1][g];
            if constexpr (MODE == 2) {
#pragma unroll
                for (int u = 0; u < 16; u += 2)
                    *reinterpret_cast<double2 *>(bb + 16 * gl + u) =
                        make_double2((double)ra[u] * (double)ra[u], (double)ra[u + 1] * (double)ra[u + 1]);
#pragma unroll
                for (int u = 0; u < 16; ++u) ra[u] = ra[u] * 1.0000001f;
            }
            __builtin_amdgcn_wave_barrier();
            acc = lds_chain_f64<CH>(acc, bb);
            __builtin_amdgcn_wave_barrier();
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double *out; long long *cyc;
    hipMalloc(&out, 256 * 256 * 8); hipMalloc(&cyc, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int nchunks = 1000000 / CH;
    for (int mode = 0; mode < 3; ++mode)
        for (int waves = 1; waves <= 4; waves *= 4)
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                auto k = mode == 0 ? k_probe<0> : (mode == 1 ? k_probe<1> : k_probe<2>);
                hipLaunchKernelGGL(k, dim3(256), dim3(64 * waves), 0, 0, out, cyc, nchunks);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
                printf("mode %d waves/CU %d: %.2f cycles/element, %.3f ms for 1M elements\n", mode, waves,
                       (double)c / (nchunks * (double)CH), ms);
            }
    return 0;
}
