// runtime.hip — error state, device scratch, memory plumbing and the
// synthetic-input generator of the C ABI (include/matternet_hip.h).
#include <mutex>
#include <string>
#include <unordered_map>

#include <cstdlib>

#include "common.hpp"
#include "glibc_f32.hpp"
#include "glibc_f64.hpp"

namespace mn {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
void clear_error() { g_err.clear(); }

bool debug_sync() {
    static const bool on = [] {
        const char *e = getenv("MN_DEBUG_SYNC");
        return e && e[0] && e[0] != '0';
    }();
    return on;
}

namespace {
struct Block { void *p = nullptr; size_t bytes = 0; };
struct DevScratch { Block slot[kNumSlots]; };
struct ThreadScratch {
    std::unordered_map<int, DevScratch> per_dev;
    ~ThreadScratch() {
        for (auto &kv : per_dev)
            for (auto &b : kv.second.slot)
                if (b.p) (void)hipFree(b.p);
    }
};
thread_local ThreadScratch t_scratch;
}  // namespace

void *scratch(int slot, size_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    Block &b = t_scratch.per_dev[dev].slot[slot];
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return b.p;
    if (b.p) { (void)hipFree(b.p); b.p = nullptr; b.bytes = 0; }
    size_t want = bytes + bytes / 8;  // headroom against creeping growth
    if (hipMalloc(&b.p, want) != hipSuccess) {
        b.p = nullptr;
        return nullptr;
    }
    b.bytes = want;
    return b.p;
}

namespace {
struct ThreadStreams {
    std::unordered_map<int, hipStream_t> side;
    std::unordered_map<int, hipEvent_t> ev;
    ~ThreadStreams() {
        for (auto &kv : side) (void)hipStreamDestroy(kv.second);
        for (auto &kv : ev) (void)hipEventDestroy(kv.second);
    }
};
thread_local ThreadStreams t_streams;
}  // namespace

hipStream_t side_stream() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    auto it = t_streams.side.find(dev);
    if (it != t_streams.side.end()) return it->second;
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
    t_streams.side[dev] = st;
    return st;
}

hipError_t stream_wait(hipStream_t waiter, hipStream_t on) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    hipEvent_t &ev = t_streams.ev[dev];
    if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipEventRecord(ev, on)) != hipSuccess) return e;
    return hipStreamWaitEvent(waiter, ev, 0);
}

void Timer::start(bool enable, hipStream_t stream) {
    on = enable;
    s = stream;
    n = 0;
    if (!on) return;
    for (auto &e : ev)
        if (!e) (void)hipEventCreate(&e);
    mark();
}
void Timer::mark() {
    if (!on || n >= 8) return;
    (void)hipEventRecord(ev[n++], s);
}
float Timer::ms(int a, int b) {
    if (!on || a >= n || b >= n) return 0.f;
    (void)hipEventSynchronize(ev[b]);
    float t = 0.f;
    (void)hipEventElapsedTime(&t, ev[a], ev[b]);
    return t;
}
Timer::~Timer() {
    for (auto &e : ev)
        if (e) (void)hipEventDestroy(e);
}

// splitmix64 counter generator; identical to tests/datagen.py
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_fill_uniform_f32(float *__restrict__ X, int64_t total, int32_t d,
                                   uint64_t seed, int64_t row0) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
        const int64_t r = e / d, c = e - r * d;
        const uint64_t ctr = (uint64_t)((row0 + r) * (int64_t)d + c) ^ seed;
        const double u = (double)(splitmix64(ctr) >> 40) * 0x1p-24;
        X[e] = (float)(2.0 * u - 1.0);
    }
}

}  // namespace mn

namespace mn {
__global__ __launch_bounds__(256) void k_libm_pow_f64(const double *__restrict__ x,
                                                      const double *__restrict__ y, int64_t n,
                                                      double *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        out[i] = glibc::pow_glibc(x[i], y[i]);
}

__global__ __launch_bounds__(256) void k_libm_f32(const float *__restrict__ x, int64_t n,
                                                  uint32_t bits0, int fn, float *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float v = x ? x[i] : __uint_as_float(bits0 + (uint32_t)i);
        out[i] = fn == 0 ? glibc::logf(v) : glibc::expf(v);
    }
}
}  // namespace mn

extern "C" {

int mn_version(void) { return 100; }

const char *mn_last_error(void) { return mn::g_err.c_str(); }

int mn_device_alloc(size_t bytes, void **out) {
    MN_REQUIRE(out != nullptr, MN_EINVAL, "mn_device_alloc: out is NULL");
    if (hipMalloc(out, bytes ? bytes : 16) != hipSuccess) {
        mn::set_error("mn_device_alloc: hipMalloc(%zu) failed", bytes);
        return MN_ENOMEM;
    }
    return MN_OK;
}

int mn_device_free(void *p) {
    if (p) MN_HIP_TRY(hipFree(p));
    return MN_OK;
}

int mn_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    MN_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

int mn_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    MN_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

int mn_memcpy_d2d(void *dst, const void *src, size_t bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    MN_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

int mn_stream_synchronize(void *stream) {
    MN_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return MN_OK;
}

int mn_fill_uniform_f32(float *X, int64_t n, int32_t d, uint64_t seed, int64_t row0,
                        void *stream) {
    MN_REQUIRE(X && n >= 0 && d >= 1 && row0 >= 0, MN_EINVAL, "mn_fill_uniform_f32: bad args");
    const int64_t total = n * (int64_t)d;
    if (total == 0) return MN_OK;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mn::k_fill_uniform_f32, dim3((unsigned)blocks), dim3(256), 0, s, X, total,
                       d, seed, row0);
    MN_HIP_TRY(hipGetLastError());
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

// The library's f32 ln / exp (glibc_f32.hpp) on device arrays: fn 0 = logf,
// 1 = expf; x == NULL evaluates the consecutive bit patterns bits0 + i.
int mn_libm_f32(const float *x, int64_t n, uint32_t bits0, int32_t fn, float *out,
                void *stream) {
    MN_REQUIRE(out && n >= 0 && (fn == 0 || fn == 1), MN_EINVAL, "mn_libm_f32: bad args");
    if (n == 0) return MN_OK;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mn::k_libm_f32, dim3((unsigned)blocks), dim3(256), 0, s, x, n, bits0, fn,
                       out);
    MN_HIP_TRY(hipGetLastError());
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

// The library's f64 pow (glibc_f64.hpp) on device arrays: out[i] = pow(x[i], y[i]).
int mn_libm_pow_f64(const double *x, const double *y, int64_t n, double *out, void *stream) {
    MN_REQUIRE(x && y && out && n >= 0, MN_EINVAL, "mn_libm_pow_f64: bad args");
    if (n == 0) return MN_OK;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mn::k_libm_pow_f64, dim3((unsigned)blocks), dim3(256), 0, s, x, y, n, out);
    MN_HIP_TRY(hipGetLastError());
    MN_HIP_TRY(hipStreamSynchronize(s));
    return MN_OK;
}

}  // extern "C"
