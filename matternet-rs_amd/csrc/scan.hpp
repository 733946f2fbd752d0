// scan.hpp — device-wide exclusive prefix sum (int32/int64 counts -> int64
// offsets), hand-written: block partials -> single-block carry scan -> add.
#pragma once
#include "common.hpp"

namespace mn {
namespace scan {
namespace {  // internal linkage: this header is included by several TUs

constexpr int SB = 1024;  // elements per block (256 threads x 4)

template <typename T>
__device__ __forceinline__ int64_t block_exclusive(int64_t v, int64_t *sh, int64_t &total) {
    // 256-thread block scan of one value per thread (wave64 shuffles + LDS)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int64_t base = 0;
    for (int i = 0; i < w; ++i) base += sh[i];
    total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return base + x - v;
}

template <typename T>
__global__ __launch_bounds__(256) void k_partials(const T *__restrict__ in, int64_t n,
                                                  int64_t *__restrict__ part) {
    __shared__ int64_t sh[4];
    const int64_t b0 = (int64_t)blockIdx.x * SB;
    int64_t s = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = b0 + threadIdx.x * 4 + r;
        if (i < n) s += (int64_t)in[i];
    }
    int64_t tot;
    block_exclusive<T>(s, sh, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// single block: exclusive scan of the partials with a running carry
__global__ __launch_bounds__(256) void k_scan_partials(int64_t *__restrict__ part, int64_t np,
                                                       int64_t *__restrict__ total_out) {
    __shared__ int64_t sh[4];
    int64_t carry = 0;
    for (int64_t c0 = 0; c0 < np; c0 += 256) {
        const int64_t i = c0 + threadIdx.x;
        const int64_t v = i < np ? part[i] : 0;
        int64_t tot;
        const int64_t ex = block_exclusive<int64_t>(v, sh, tot);
        if (i < np) part[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

template <typename T>
__global__ __launch_bounds__(256) void k_apply(const T *__restrict__ in, int64_t n,
                                               const int64_t *__restrict__ part,
                                               int64_t *__restrict__ out) {
    __shared__ int64_t sh[4];
    const int64_t b0 = (int64_t)blockIdx.x * SB;
    int64_t v[4];
    int64_t s = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = b0 + threadIdx.x * 4 + r;
        v[r] = i < n ? (int64_t)in[i] : 0;
        s += v[r];
    }
    int64_t tot;
    int64_t ex = block_exclusive<T>(s, sh, tot) + part[blockIdx.x];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = b0 + threadIdx.x * 4 + r;
        if (i < n) out[i] = ex;
        ex += v[r];
    }
}

// out[0..n) = exclusive scan of in; out[n] = total (out must hold n+1).
// `part` scratch must hold ceil(n/SB)+1 int64.
template <typename T>
inline hipError_t exclusive_scan(const T *in, int64_t n, int64_t *out, int64_t *part,
                                 hipStream_t s) {
    const int64_t nb = (n + SB - 1) / SB;
    if (nb > 0) {
        hipLaunchKernelGGL(k_partials<T>, dim3((unsigned)nb), dim3(256), 0, s, in, n, part);
    }
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(256), 0, s, part, nb, out + n);
    if (nb > 0) {
        hipLaunchKernelGGL(k_apply<T>, dim3((unsigned)nb), dim3(256), 0, s, in, n, part, out);
    }
    return hipGetLastError();
}

}  // namespace
}  // namespace scan
}  // namespace mn
