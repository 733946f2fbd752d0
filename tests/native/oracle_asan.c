/* The oracle's C restatement under ASan / UBSan (tests/test_sanitizers.py):
 * every entry point on small random inputs and on the edge shapes the parity
 * tests use (one row, k beyond n - 1, empty rows, NaN lambdas).  Exit 0 and
 * no sanitizer report = clean. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static uint64_t st = 88172645463325252ull;
static double urand(void) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) / 9007199254740992.0;
}

static int check_knn(int64_t n, int d, int k) {
    float *X = malloc(sizeof(float) * n * d);
    for (int64_t i = 0; i < n * d; ++i) X[i] = (float)(2 * urand() - 1);
    int32_t *idx = malloc(sizeof(int32_t) * n * k), *idx2 = malloc(sizeof(int32_t) * n * k);
    float *dist = malloc(sizeof(float) * n * k), *dist2 = malloc(sizeof(float) * n * k);
    int rc = or_knn_l2sq_f32(X, n, d, k, 0, n, 0, 2, idx, dist);
    rc |= or_knn_l2sq_f32(X, n, d, k, 0, n, 1, 2, idx2, dist2);
    if (memcmp(idx, idx2, sizeof(int32_t) * n * k)) rc |= 1;
    int64_t *rows = malloc(sizeof(int64_t) * n);
    for (int64_t i = 0; i < n; ++i) rows[i] = n - 1 - i;
    rc |= or_knn_l2sq_rows_f32(X, n, d, k, rows, n, 2, idx2, dist2);
    rc |= or_knn_l2sq_qc_f32(X, n, rows, X, n, d, 0, k, 1, 2, idx2, dist2);
    double *cd = malloc(sizeof(double) * n * k), *cw = malloc(sizeof(double) * n * k);
    rc |= or_knn_cos_f64(X, n, d, k, 1.0, 1.0, 2.0, 0, n, 2, idx2, cd, cw);
    double *Xd = malloc(sizeof(double) * n * d);
    for (int64_t i = 0; i < n * d; ++i) Xd[i] = X[i];
    rc |= or_knn_cos_f64d(Xd, n, d, k, 1.0, 1.0, 2.7, 0, n, 2, idx2, cd, cw);
    rc |= or_knn_l2_f64(Xd, n, Xd, n, d, rows, k, 1, 2, idx2, cd);
    /* Laplacian (UNION) from the kNN rows, then energy / diffusion over it */
    double *w = malloc(sizeof(double) * n * k);
    for (int64_t i = 0; i < n * k; ++i) w[i] = dist[i] == INFINITY ? 0.0 : 1.0 / (1.0 + dist[i]);
    int64_t cap = 2 * n * k + n, nnz = 0;
    int64_t *ip = malloc(sizeof(int64_t) * (n + 1));
    int32_t *ix = malloc(sizeof(int32_t) * cap);
    double *iv = malloc(sizeof(double) * cap);
    rc |= or_laplacian_union(n, k, idx, w, cap, ip, ix, iv, &nnz);
    double *out = malloc(sizeof(double) * n * d);
    if (n == d) {
        double E[64], G[64], L[64];
        rc |= or_energy_rows(X, n, d, ip, ix, iv, OR_G_TAUMODE, OR_TAU_MEDIAN, 0.0, 2, E, G, L);
        rc |= or_energy_rows_faithful(X, n, d, ip, ix, iv, OR_TAU_MEDIAN, 0.0, 2, E, G, L);
        rc |= or_diffuse_rows(Xd, n, d, ip, ix, iv, 0.1, 3, 0, out);
    }
    int64_t *oip = malloc(sizeof(int64_t) * (n + 1));
    int32_t *oix = malloc(sizeof(int32_t) * (nnz + 1));
    double *ow = malloc(sizeof(double) * (nnz + 1));
    rc |= or_sfgrass(n, ip, ix, iv, 0.5, oip, oix, ow);
    free(X); free(idx); free(idx2); free(dist); free(dist2); free(rows); free(cd); free(cw);
    free(Xd); free(w); free(ip); free(ix); free(iv); free(out); free(oip); free(oix); free(ow);
    return rc < 0 ? rc : 0;
}

int main(void) {
    int rc = 0;
    rc |= check_knn(300, 16, 10);
    rc |= check_knn(1, 4, 3);     /* one row: every slot padded */
    rc |= check_knn(5, 7, 9);     /* k beyond n - 1 */
    rc |= check_knn(48, 48, 4);   /* square: the energy / diffusion paths */
    /* sorted index + lookups with NaN and signed zeros */
    double lam[12] = {0.5, 0.125, NAN, 0.875, -0.0, 0.0, 0.5, 1e-300, 3.0, NAN, 0.25, 0.5};
    int64_t order[12], oi[12];
    double keys[12], ok[12], sd = 0;
    rc |= or_sorted_index(lam, 12, order, keys, &sd);
    if (or_range_bylambda(keys, order, 12, sd, 0.5, 12, 1.0, oi, ok) < -1) rc |= 1;
    if (or_k_nearest_by_lambda(keys, order, 12, sd, 0.3, 5, 1.0, 0, 0.0, 1.7, 10.0, oi, ok) < -1)
        rc |= 1;
    double nl[6] = {0.3, 0.1, 0.9, 0.9, 0.0, 0.5}, mn, mx, rg;
    rc |= or_normalise_lambdas(nl, 6, &mn, &mx, &rg);
    double x[7] = {3, 1, 2, 5, 4, 0, -1};
    for (int m = 0; m < 4; ++m) (void)or_select_tau(x, 7, m, 0.9);
    /* Stage C and MST candidates on a few centroids */
    float means[8 * 6], vars[8 * 6];
    for (int i = 0; i < 48; ++i) { means[i] = (float)urand(); vars[i] = (float)(0.1 + urand()); }
    int32_t bi[6 * 3], mv[8 * 3];
    float bw[6 * 3], md[8 * 3], mc[8 * 3];
    rc |= or_bc_knn(means, vars, 8, 6, 3, 1e-6f, 1e-3f, bi, bw);
    for (int metric = 0; metric < 3; ++metric)
        for (int tw = 0; tw < 5; ++tw)
            rc |= or_mst_candidates(means, vars, 8, 6, 3, metric, tw, NULL, mv, md, mc);
    int32_t ci[8];
    float cdd[8];
    rc |= or_nearest_centroid(means, 8, vars, 8, 6, ci, cdd);
    printf("oracle sanitizer run rc %d\n", rc);
    return rc != 0;
}
