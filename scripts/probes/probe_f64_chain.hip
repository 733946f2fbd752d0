// Dependent f64 add chain latency on gfx950: one wave, N adds whose operands
// sit in registers (a) or come from LDS broadcasts 32 ahead (b, the
// lds_chain_f64 pattern of knn_cos.hip).  Prints cycles per add (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_reg(double *out, long long *cyc, int reps) {
    double v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = 1e-3 * (threadIdx.x + i + 1);
    double acc = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int i = 0; i < 32; ++i) acc = acc + v[i];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_fma(double *out, long long *cyc, int reps) {
    double v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = 1e-3 * (threadIdx.x + i + 1);
    double acc = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int i = 0; i < 32; ++i) acc = __builtin_fma(v[i], v[i], acc);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double *out; long long *cyc;
    hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
    const int reps = 1 << 14;
    for (int k = 0; k < 2; ++k) {
        for (int it = 0; it < 3; ++it) {
            if (k == 0) hipLaunchKernelGGL(k_reg, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            else hipLaunchKernelGGL(k_fma, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            hipDeviceSynchronize();
            long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("%s: %.2f cycles per dependent op (s_memtime ticks)\n", k ? "fma_f64" : "add_f64",
                   (double)c / (reps * 32.0));
        }
    }
    return 0;
}
