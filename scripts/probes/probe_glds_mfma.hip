// Probe: (1) global_load_lds_dwordx4 LDS placement, (2) 32x32x16 bf16 MFMA layouts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ void k_glds(const uint32_t *g, uint32_t *out) {
    __shared__ uint32_t s[64 * 4 * 2];
    for (int i = threadIdx.x; i < 512; i += 64) s[i] = 0xFFFFFFFFu;
    __syncthreads();
    const uint32_t *src = g + 4 * (63 - threadIdx.x);   // lane l loads record 63-l
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)(s + 256), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) out[i] = s[i];
}

__global__ void k_mfma(const uint16_t *A, const uint16_t *B, float *D) {
    // A [32][16] row-major, B [32 cols][16 k] (col-major k), D [32][32]
    const int l = threadIdx.x;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        uint16_t av = A[(l & 31) * 16 + 8 * (l >> 5) + j];
        uint16_t bv = B[(l & 31) * 16 + 8 * (l >> 5) + j];
        a[j] = __builtin_bit_cast(__bf16, av);
        b[j] = __builtin_bit_cast(__bf16, bv);
    }
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
        D[row * 32 + col] = c[r];
    }
}

static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
static float bf2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }

int main() {
    std::vector<uint32_t> h(256);
    for (int i = 0; i < 256; ++i) h[i] = i;
    uint32_t *dg, *dout;
    hipMalloc(&dg, 1024); hipMalloc(&dout, 2048);
    hipMemcpy(dg, h.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_glds, dim3(1), dim3(64), 0, 0, dg, dout);
    std::vector<uint32_t> o(512);
    hipMemcpy(o.data(), dout, 2048, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int i = 0; i < 256; ++i) if (o[i] != 0xFFFFFFFFu) ok = 0;
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 4; ++j)
        if (o[256 + 4 * l + j] != (uint32_t)(4 * (63 - l) + j)) ok = 0;
    printf("glds lane-linear placement: %s\n", ok ? "OK" : "MISMATCH");
    if (!ok) { for (int i = 256; i < 288; ++i) printf("%u ", o[i]); printf("\n"); }

    std::vector<uint16_t> A(32 * 16), B(32 * 16);
    for (int i = 0; i < 32; ++i) for (int k = 0; k < 16; ++k) {
        A[i * 16 + k] = f2bf((float)((i * 7 + k * 3) % 11 - 5));
        B[i * 16 + k] = f2bf((float)((i * 5 + k * 2) % 13 - 6));
    }
    uint16_t *dA, *dB; float *dD;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 4096);
    hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    std::vector<float> D(1024);
    hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
        float s = 0; for (int k = 0; k < 16; ++k) s += bf2f(A[i * 16 + k]) * bf2f(B[j * 16 + k]);
        if (s != D[i * 32 + j]) ++bad;
    }
    printf("mfma 32x32x16 layout: %s (%d bad)\n", bad ? "MISMATCH" : "OK", bad);
    return 0;
}
