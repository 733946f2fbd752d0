// Probe: k_gram_bf16 keys + lists for block (0,0) vs a host f64 computation.
#define MN_BF16_DEBUG 1
#include "../../matternet-rs_amd/csrc/knn_bf16.hip"
#include <cstring>
#include <cmath>
#include <vector>
#include <algorithm>
using namespace mn::kb16;
static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
static double bf2(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
    const int n = 257, d = 32, L = 21;
    std::vector<uint16_t> X(n * d);
    uint64_t z = 12345;
    for (auto &v : X) { z = z * 6364136223846793005ull + 1442695040888963407ull; v = f2bf((float)((z >> 40) * 0x1p-24) * 2.f - 1.f); }
    std::vector<double> nr(n); std::vector<float> inv(n);
    for (int i = 0; i < n; ++i) { double a = 0; for (int k = 0; k < d; ++k) a += bf2(X[i*d+k]) * bf2(X[i*d+k]); nr[i] = sqrt(a); inv[i] = (float)(1.0 / nr[i]); }
    uint16_t *dX; float *dinv, *ld; int *li, *lsz; float *tau;
    hipMalloc(&dX, X.size() * 2); hipMalloc(&dinv, n * 4); hipMalloc(&ld, n * L * 4); hipMalloc(&li, n * L * 4);
    hipMalloc(&lsz, n * 4); hipMalloc(&tau, n * 4);
    hipMemcpy(dX, X.data(), X.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dinv, inv.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_gram_bf16, dim3(2, 1), dim3(NT), 0, 0, dX, (int64_t)n, dX, (int64_t)n, d, (int64_t)0, (int64_t)0, 1,
                       dinv, dinv, L, 1, (int64_t)512, ld, li, lsz, tau);
    hipError_t e = hipDeviceSynchronize();
    printf("sync: %s\n", hipGetErrorString(e));
    std::vector<float> keys(256 * 256);
    hipMemcpyFromSymbol(keys.data(), HIP_SYMBOL(g_dbg_keys), keys.size() * 4);
    int bad = 0; double maxerr = 0;
    for (int i = 0; i < 256; ++i) for (int j = 0; j < 128; ++j) {
        if (i == j) continue;
        double dot = 0; for (int k = 0; k < d; ++k) dot += bf2(X[i*d+k]) * bf2(X[j*d+k]);
        double ref = -dot / (nr[i] * nr[j]);
        double er = fabs(ref - keys[i * 256 + j]);
        maxerr = std::max(maxerr, er);
        if (er > 1e-3) { if (bad < 8) printf("key mismatch i=%d j=%d ref=%f got=%f\n", i, j, ref, keys[i*BN+j]); ++bad; }
    }
    printf("keys: %d bad, max err %g\n", bad, maxerr);
    std::vector<float> hld(n * L); std::vector<int> hli(n * L), hsz(n); std::vector<float> ht(n);
    hipMemcpy(hld.data(), ld, n * L * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hli.data(), li, n * L * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hsz.data(), lsz, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(ht.data(), tau, n * 4, hipMemcpyDeviceToHost);
    for (int q : {0, 1, 2, 100, 256}) {
        std::vector<std::pair<double,int>> v;
        for (int j = 0; j < n; ++j) if (j != q) { double dot = 0; for (int k = 0; k < d; ++k) dot += bf2(X[q*d+k]) * bf2(X[j*d+k]); v.push_back({-dot/(nr[q]*nr[j]), j}); }
        std::sort(v.begin(), v.end());
        printf("row %d lsz %d tau %f\n  gpu:", q, hsz[q], ht[q]);
        for (int e2 = 0; e2 < std::min(hsz[q], 8); ++e2) printf(" %d(%.4f)", hli[q*L+e2], hld[q*L+e2]);
        printf("\n  ref:");
        for (int e2 = 0; e2 < 8; ++e2) printf(" %d(%.4f)", v[e2].second, v[e2].first);
        printf("\n");
    }
    return 0;
}
