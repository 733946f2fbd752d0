/*
 * oracle.c — CPU restatement of the surfface hot path (TEST INFRASTRUCTURE).
 * See oracle.h for the contract, provenance and the per-function reference
 * citations.  Compiled with -ffp-contract=off -fno-fast-math so every
 * expression rounds exactly as the (non-contracting) Rust reference does.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_EINVAL (-1)
#define OR_ENOMEM (-2)
#define OR_ENONFINITE (-3)
#define OR_ECAP (-4)

static void set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

/* ------------------------------------------------------------------------ */
/* K1 — A.1 L2^2                                                             */
/* ------------------------------------------------------------------------ */

/* surfface-core/src/distance.rs:206-213: zip().map((a-b).powi(2)).sum() */
static inline float fold_l2sq_f32(const float *a, const float *b, int32_t d) {
    float acc = -0.0f; /* Rust >= 1.83 float Sum starts at -0.0 */
    for (int32_t t = 0; t < d; ++t) {
        float diff = a[t] - b[t];
        float sq = diff * diff; /* powi(2) lowers to one multiply */
        acc = acc + sq;
    }
    return acc;
}

typedef struct { float d; int32_t j; } cand_f32;

/* (dist, j) total order == stable sort by dist over ascending-j input. */
static inline int lt_f32(float da, int32_t ja, float db, int32_t jb) {
    return da < db || (da == db && ja < jb);
}

static int cmp_cand_f32(const void *pa, const void *pb) {
    const cand_f32 *a = (const cand_f32 *)pa, *b = (const cand_f32 *)pb;
    if (lt_f32(a->d, a->j, b->d, b->j)) return -1;
    if (lt_f32(b->d, b->j, a->d, a->j)) return 1;
    return 0;
}

/* bounded max-heap of the k best (dist, j) */
static void heap_sift_down(cand_f32 *h, int32_t n, int32_t i) {
    for (;;) {
        int32_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < n && lt_f32(h[m].d, h[m].j, h[l].d, h[l].j)) m = l;
        if (r < n && lt_f32(h[m].d, h[m].j, h[r].d, h[r].j)) m = r;
        if (m == i) return;
        cand_f32 t = h[i]; h[i] = h[m]; h[m] = t; i = m;
    }
}
static void heap_sift_up(cand_f32 *h, int32_t i) {
    while (i > 0) {
        int32_t p = (i - 1) / 2;
        if (!lt_f32(h[p].d, h[p].j, h[i].d, h[i].j)) return;
        cand_f32 t = h[i]; h[i] = h[p]; h[p] = t; i = p;
    }
}

static int knn_l2sq_core(const float *X, int64_t n, int32_t d, int32_t k,
                         int64_t q_begin, int64_t q_end, const int64_t *rows, int mode,
                         int nthreads, int32_t *out_idx, float *out_dist);

int or_knn_l2sq_f32(const float *X, int64_t n, int32_t d, int32_t k,
                    int64_t q_begin, int64_t q_end, int mode, int nthreads,
                    int32_t *out_idx, float *out_dist) {
    if (!X || !out_idx || !out_dist || n < 1 || d < 1 || k < 1 || q_begin < 0 ||
        q_end > n || q_begin > q_end)
        return OR_EINVAL;
    return knn_l2sq_core(X, n, d, k, q_begin, q_end, NULL, mode, nthreads, out_idx, out_dist);
}

int or_knn_l2sq_rows_f32(const float *X, int64_t n, int32_t d, int32_t k,
                         const int64_t *rows, int64_t nrows, int nthreads,
                         int32_t *out_idx, float *out_dist) {
    if (!X || !rows || !out_idx || !out_dist || n < 1 || d < 1 || k < 1 || nrows < 0)
        return OR_EINVAL;
    for (int64_t t = 0; t < nrows; ++t) if (rows[t] < 0 || rows[t] >= n) return OR_EINVAL;
    return knn_l2sq_core(X, n, d, k, 0, nrows, rows, 1, nthreads, out_idx, out_dist);
}

static int knn_l2sq_core(const float *X, int64_t n, int32_t d, int32_t k,
                         int64_t q_begin, int64_t q_end, const int64_t *rows, int mode,
                         int nthreads, int32_t *out_idx, float *out_dist) {
    const int64_t keff64 = (n - 1) < (int64_t)k ? (n - 1) : (int64_t)k;
    const int32_t keff = (int32_t)keff64;
    int err = 0;
    set_threads(nthreads);
#pragma omp parallel
    {
        cand_f32 *buf = NULL;
        if (mode == 0) buf = (cand_f32 *)malloc(sizeof(cand_f32) * (size_t)(n > 1 ? n - 1 : 1));
        else buf = (cand_f32 *)malloc(sizeof(cand_f32) * (size_t)(keff > 0 ? keff : 1));
        if (!buf) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 1) /* rows cost ~n d each: one per chunk */
        for (int64_t qq = q_begin; qq < q_end; ++qq) {
            if (!buf) continue;
            const int64_t i = rows ? rows[qq] : qq;
            const float *xi = X + i * (int64_t)d;
            int32_t *oi = out_idx + (qq - q_begin) * (int64_t)k;
            float *od = out_dist + (qq - q_begin) * (int64_t)k;
            int bad = 0;
            int32_t cnt = 0;
            for (int64_t j = 0; j < n; ++j) {
                if (j == i) continue;
                float dist = fold_l2sq_f32(xi, X + j * (int64_t)d, d);
                if (dist != dist) { bad = 1; break; }
                if (mode == 0) {
                    buf[cnt].d = dist; buf[cnt].j = (int32_t)j; ++cnt;
                } else if (cnt < keff) {
                    buf[cnt].d = dist; buf[cnt].j = (int32_t)j;
                    heap_sift_up(buf, cnt); ++cnt;
                } else if (keff > 0 && lt_f32(dist, (int32_t)j, buf[0].d, buf[0].j)) {
                    buf[0].d = dist; buf[0].j = (int32_t)j;
                    heap_sift_down(buf, cnt, 0);
                }
            }
            if (bad) {
#pragma omp atomic write
                err = OR_ENONFINITE;
                continue;
            }
            qsort(buf, (size_t)cnt, sizeof(cand_f32), cmp_cand_f32);
            for (int32_t r = 0; r < k; ++r) {
                if (r < keff) { oi[r] = buf[r].j; od[r] = buf[r].d; }
                else { oi[r] = -1; od[r] = INFINITY; }
            }
        }
        free(buf);
    }
    return err;
}

/* A.1 in the per-shard form of the row-sharded build: query
 * rows Q[t] (global ids q_ids[t]) against a corpus shard C (global ids c_off +
 * j); the pair whose global ids are equal is skipped when excl.  Output ids
 * are global; (dist, id) order; restated-efficient heap (mode 1).  The
 * reference's mst.rs:330-360 over the shard's rows. */
int or_knn_l2sq_qc_f32(const float *Q, int64_t nq, const int64_t *q_ids, const float *C,
                       int64_t nc, int32_t d, int64_t c_off, int32_t k, int excl, int nthreads,
                       int32_t *out_idx, float *out_dist) {
    if (!Q || !C || !q_ids || !out_idx || !out_dist || nq < 0 || nc < 1 || d < 1 || k < 1)
        return OR_EINVAL;
    int err = 0;
    set_threads(nthreads);
#pragma omp parallel
    {
        cand_f32 *buf = (cand_f32 *)malloc(sizeof(cand_f32) * (size_t)k);
        if (!buf) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 1)
        for (int64_t t = 0; t < nq; ++t) {
            if (!buf) continue;
            const float *xq = Q + t * (int64_t)d;
            int32_t cnt = 0;
            int bad = 0;
            for (int64_t j = 0; j < nc; ++j) {
                const int64_t g = c_off + j;
                if (excl && g == q_ids[t]) continue;
                const float dist = fold_l2sq_f32(xq, C + j * (int64_t)d, d);
                if (dist != dist) { bad = 1; break; }
                if (cnt < k) {
                    buf[cnt].d = dist; buf[cnt].j = (int32_t)g;
                    heap_sift_up(buf, cnt); ++cnt;
                } else if (lt_f32(dist, (int32_t)g, buf[0].d, buf[0].j)) {
                    buf[0].d = dist; buf[0].j = (int32_t)g;
                    heap_sift_down(buf, cnt, 0);
                }
            }
            if (bad) {
#pragma omp atomic write
                err = OR_ENONFINITE;
                continue;
            }
            qsort(buf, (size_t)cnt, sizeof(cand_f32), cmp_cand_f32);
            for (int32_t r = 0; r < k; ++r) {
                out_idx[t * k + r] = r < cnt ? buf[r].j : -1;
                out_dist[t * k + r] = r < cnt ? buf[r].d : INFINITY;
            }
        }
        free(buf);
    }
    return err;
}

/* ------------------------------------------------------------------------ */
/* K1 — A.1c rectified cosine, f64                                           */
/* ------------------------------------------------------------------------ */

typedef struct { double d; double w; int32_t j; } cand_f64;

static inline int lt_f64(double da, int32_t ja, double db, int32_t jb) {
    return da < db || (da == db && ja < jb);
}
static int cmp_cand_f64(const void *pa, const void *pb) {
    const cand_f64 *a = (const cand_f64 *)pa, *b = (const cand_f64 *)pb;
    if (lt_f64(a->d, a->j, b->d, b->j)) return -1;
    if (lt_f64(b->d, b->j, a->d, a->j)) return 1;
    return 0;
}
static void heap64_down(cand_f64 *h, int32_t n, int32_t i) {
    for (;;) {
        int32_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < n && lt_f64(h[m].d, h[m].j, h[l].d, h[l].j)) m = l;
        if (r < n && lt_f64(h[m].d, h[m].j, h[r].d, h[r].j)) m = r;
        if (m == i) return;
        cand_f64 t = h[i]; h[i] = h[m]; h[m] = t; i = m;
    }
}
static void heap64_up(cand_f64 *h, int32_t i) {
    while (i > 0) {
        int32_t p = (i - 1) / 2;
        if (!lt_f64(h[p].d, h[p].j, h[i].d, h[i].j)) return;
        cand_f64 t = h[i]; h[i] = h[p]; h[p] = t; i = p;
    }
}

/* test_helpers.rs:80-83: (item.iter().map(|&x| x * x).sum::<f64>()).sqrt() */
static inline double norm_f64(const float *a, int32_t d) {
    double acc = -0.0;
    for (int32_t t = 0; t < d; ++t) {
        double x = (double)a[t];
        acc = acc + x * x;
    }
    return sqrt(acc);
}

int or_knn_cos_f64(const float *X, int64_t n, int32_t d, int32_t topk,
                   double eps, double sigma, double p,
                   int64_t q_begin, int64_t q_end, int nthreads,
                   int32_t *out_idx, double *out_dist, double *out_w) {
    if (!X || !out_idx || !out_dist || n < 1 || d < 1 || topk < 1 || q_begin < 0 ||
        q_end > n || q_begin > q_end)
        return OR_EINVAL;
    double *norms = (double *)malloc(sizeof(double) * (size_t)n);
    if (!norms) return OR_ENOMEM;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) norms[i] = norm_f64(X + i * (int64_t)d, d);

#pragma omp parallel
    {
        cand_f64 *buf = (cand_f64 *)malloc(sizeof(cand_f64) * (size_t)topk);
        if (!buf) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = q_begin; i < q_end; ++i) {
            if (!buf) continue;
            const float *xi = X + i * (int64_t)d;
            int32_t cnt = 0;
            int bad = 0;
            for (int64_t j = 0; j < n; ++j) {
                if (j == i) continue;
                double denom = norms[i] * norms[j];
                double cs;
                if (denom > 1e-12) {
                    const float *xj = X + j * (int64_t)d;
                    double dot = -0.0;
                    for (int32_t t = 0; t < d; ++t) dot = dot + (double)xi[t] * (double)xj[t];
                    cs = dot / denom;
                    if (cs != cs) { bad = 1; break; }
                    cs = cs < -1.0 ? -1.0 : (cs > 1.0 ? 1.0 : cs);
                } else {
                    cs = 0.0;
                }
                double dist = 1.0 - (cs > 0.0 ? cs : 0.0);
                if (!(dist <= eps)) continue;
                double nd = dist / sigma;
                double wgt = 1.0 / (1.0 + pow(nd, p)); /* f64::powf = glibc pow, every p */
                if (!(wgt > 1e-12)) continue;
                if (cnt < topk) {
                    buf[cnt].d = dist; buf[cnt].w = wgt; buf[cnt].j = (int32_t)j;
                    heap64_up(buf, cnt); ++cnt;
                } else if (lt_f64(dist, (int32_t)j, buf[0].d, buf[0].j)) {
                    buf[0].d = dist; buf[0].w = wgt; buf[0].j = (int32_t)j;
                    heap64_down(buf, cnt, 0);
                }
            }
            if (bad) {
#pragma omp atomic write
                err = OR_ENONFINITE;
                continue;
            }
            qsort(buf, (size_t)cnt, sizeof(cand_f64), cmp_cand_f64);
            int32_t *oi = out_idx + (i - q_begin) * (int64_t)topk;
            double *od = out_dist + (i - q_begin) * (int64_t)topk;
            double *ow = out_w ? out_w + (i - q_begin) * (int64_t)topk : NULL;
            for (int32_t r = 0; r < topk; ++r) {
                if (r < cnt) { oi[r] = buf[r].j; od[r] = buf[r].d; if (ow) ow[r] = buf[r].w; }
                else { oi[r] = -1; od[r] = INFINITY; if (ow) ow[r] = 0.0; }
            }
        }
        free(buf);
    }
    free(norms);
    return err;
}

/* A.1c on f64 rows (the legacy DenseMatrix<f64> items): the same arithmetic
 * with the reference's rounded f64 products (test_helpers.rs:77-126). */
static double norm_f64d(const double *x, int32_t d) {
    double s = -0.0;
    for (int32_t t = 0; t < d; ++t) s = s + x[t] * x[t];
    return sqrt(s);
}

int or_knn_cos_f64d(const double *X, int64_t n, int32_t d, int32_t topk,
                   double eps, double sigma, double p,
                   int64_t q_begin, int64_t q_end, int nthreads,
                   int32_t *out_idx, double *out_dist, double *out_w) {
    if (!X || !out_idx || !out_dist || n < 1 || d < 1 || topk < 1 || q_begin < 0 ||
        q_end > n || q_begin > q_end)
        return OR_EINVAL;
    double *norms = (double *)malloc(sizeof(double) * (size_t)n);
    if (!norms) return OR_ENOMEM;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) norms[i] = norm_f64d(X + i * (int64_t)d, d);

#pragma omp parallel
    {
        cand_f64 *buf = (cand_f64 *)malloc(sizeof(cand_f64) * (size_t)topk);
        if (!buf) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = q_begin; i < q_end; ++i) {
            if (!buf) continue;
            const double *xi = X + i * (int64_t)d;
            int32_t cnt = 0;
            int bad = 0;
            for (int64_t j = 0; j < n; ++j) {
                if (j == i) continue;
                double denom = norms[i] * norms[j];
                double cs;
                if (denom > 1e-12) {
                    const double *xj = X + j * (int64_t)d;
                    double dot = -0.0;
                    for (int32_t t = 0; t < d; ++t) dot = dot + (double)xi[t] * (double)xj[t];
                    cs = dot / denom;
                    if (cs != cs) { bad = 1; break; }
                    cs = cs < -1.0 ? -1.0 : (cs > 1.0 ? 1.0 : cs);
                } else {
                    cs = 0.0;
                }
                double dist = 1.0 - (cs > 0.0 ? cs : 0.0);
                if (!(dist <= eps)) continue;
                double nd = dist / sigma;
                double wgt = 1.0 / (1.0 + pow(nd, p)); /* f64::powf = glibc pow, every p */
                if (!(wgt > 1e-12)) continue;
                if (cnt < topk) {
                    buf[cnt].d = dist; buf[cnt].w = wgt; buf[cnt].j = (int32_t)j;
                    heap64_up(buf, cnt); ++cnt;
                } else if (lt_f64(dist, (int32_t)j, buf[0].d, buf[0].j)) {
                    buf[0].d = dist; buf[0].w = wgt; buf[0].j = (int32_t)j;
                    heap64_down(buf, cnt, 0);
                }
            }
            if (bad) {
#pragma omp atomic write
                err = OR_ENONFINITE;
                continue;
            }
            qsort(buf, (size_t)cnt, sizeof(cand_f64), cmp_cand_f64);
            int32_t *oi = out_idx + (i - q_begin) * (int64_t)topk;
            double *od = out_dist + (i - q_begin) * (int64_t)topk;
            double *ow = out_w ? out_w + (i - q_begin) * (int64_t)topk : NULL;
            for (int32_t r = 0; r < topk; ++r) {
                if (r < cnt) { oi[r] = buf[r].j; od[r] = buf[r].d; if (ow) ow[r] = buf[r].w; }
                else { oi[r] = -1; od[r] = INFINITY; if (ow) ow[r] = 0.0; }
            }
        }
        free(buf);
    }
    free(norms);
    return err;
}


/* A.1c on bf16 rows (config 5), explicit query rows: the same arithmetic as
 * or_knn_cos_f64 on the exactly widened values (bf16 -> f32 is a 16-bit
 * shift).  Used for full-size parity samples without a 4x host copy. */
static inline double bf16_to_f64(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return (double)f;
}

int or_knn_cos_bf16_rows(const uint16_t *X, int64_t n, int32_t d, int32_t topk,
                         double eps, double sigma, double p,
                         const int64_t *rows, int64_t nrows, int nthreads,
                         int32_t *out_idx, double *out_dist, double *out_w) {
    if (!X || !rows || !out_idx || !out_dist || n < 1 || d < 1 || topk < 1 || nrows < 0)
        return OR_EINVAL;
    for (int64_t r = 0; r < nrows; ++r)
        if (rows[r] < 0 || rows[r] >= n) return OR_EINVAL;
    double *norms = (double *)malloc(sizeof(double) * (size_t)n);
    if (!norms) return OR_ENOMEM;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const uint16_t *x = X + i * (int64_t)d;
        double acc = -0.0;
        for (int32_t t = 0; t < d; ++t) {
            const double v = bf16_to_f64(x[t]);
            acc = acc + v * v;
        }
        norms[i] = sqrt(acc);
    }
#pragma omp parallel
    {
        cand_f64 *buf = (cand_f64 *)malloc(sizeof(cand_f64) * (size_t)topk);
        double *xi = (double *)malloc(sizeof(double) * (size_t)d);
        if (!buf || !xi) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 1)
        for (int64_t r = 0; r < nrows; ++r) {
            if (!buf || !xi) continue;
            const int64_t i = rows[r];
            for (int32_t t = 0; t < d; ++t) xi[t] = bf16_to_f64(X[i * (int64_t)d + t]);
            int32_t cnt = 0;
            for (int64_t j = 0; j < n; ++j) {
                if (j == i) continue;
                double denom = norms[i] * norms[j];
                double cs;
                if (denom > 1e-12) {
                    const uint16_t *xj = X + j * (int64_t)d;
                    double dot = -0.0;
                    for (int32_t t = 0; t < d; ++t) dot = dot + xi[t] * bf16_to_f64(xj[t]);
                    cs = dot / denom;
                    cs = cs < -1.0 ? -1.0 : (cs > 1.0 ? 1.0 : cs);
                } else {
                    cs = 0.0;
                }
                double dist = 1.0 - (cs > 0.0 ? cs : 0.0);
                if (!(dist <= eps)) continue;
                double nd = dist / sigma;
                double wgt = 1.0 / (1.0 + pow(nd, p)); /* f64::powf = glibc pow, every p */
                if (!(wgt > 1e-12)) continue;
                if (cnt < topk) {
                    buf[cnt].d = dist; buf[cnt].w = wgt; buf[cnt].j = (int32_t)j;
                    heap64_up(buf, cnt); ++cnt;
                } else if (lt_f64(dist, (int32_t)j, buf[0].d, buf[0].j)) {
                    buf[0].d = dist; buf[0].w = wgt; buf[0].j = (int32_t)j;
                    heap64_down(buf, cnt, 0);
                }
            }
            qsort(buf, (size_t)cnt, sizeof(cand_f64), cmp_cand_f64);
            int32_t *oi = out_idx + r * (int64_t)topk;
            double *od = out_dist + r * (int64_t)topk;
            double *ow = out_w ? out_w + r * (int64_t)topk : NULL;
            for (int32_t q = 0; q < topk; ++q) {
                if (q < cnt) { oi[q] = buf[q].j; od[q] = buf[q].d; if (ow) ow[q] = buf[q].w; }
                else { oi[q] = -1; od[q] = INFINITY; if (ow) ow[q] = 0.0; }
            }
        }
        free(buf);
        free(xi);
    }
    free(norms);
    return err;
}

/* ------------------------------------------------------------------------ */
/* K2 — A.2 UNION / unnormalised                                             */
/* ------------------------------------------------------------------------ */

typedef struct { int64_t key; double w; } edge64;  /* key = i*n + j */

static int cmp_edge64(const void *pa, const void *pb) {
    const edge64 *a = (const edge64 *)pa, *b = (const edge64 *)pb;
    if (a->key < b->key) return -1;
    if (a->key > b->key) return 1;
    /* equal keys: larger weight first so the dedup keeps the max */
    if (a->w > b->w) return -1;
    if (a->w < b->w) return 1;
    return 0;
}

int or_laplacian_union(int64_t n, int32_t k, const int32_t *nbr_idx,
                       const double *nbr_w, int64_t cap, int64_t *indptr,
                       int32_t *indices, double *values, int64_t *nnz_out) {
    if (n < 1 || k < 0 || !indptr || !nnz_out) return OR_EINVAL;
    int64_t m = 0;
    edge64 *e = (edge64 *)malloc(sizeof(edge64) * (size_t)(2 * n * (int64_t)k + 1));
    if (!e) return OR_ENOMEM;
    for (int64_t i = 0; i < n; ++i)
        for (int32_t r = 0; r < k; ++r) {
            int32_t j = nbr_idx[i * k + r];
            if (j < 0 || j == i) continue; /* laplacian.rs:331 src != dst */
            if (j >= n) { free(e); return OR_EINVAL; }
            double w = nbr_w[i * k + r];
            e[m].key = i * n + j; e[m].w = w; ++m;
            e[m].key = (int64_t)j * n + i; e[m].w = w; ++m;
        }
    qsort(e, (size_t)m, sizeof(edge64), cmp_edge64);
    int64_t u = 0;
    for (int64_t t = 0; t < m; ++t)
        if (u == 0 || e[t].key != e[u - 1].key) e[u++] = e[t];
    int64_t nnz = u + n; /* + one diagonal per row */
    *nnz_out = nnz;
    if (nnz > cap || !indices || !values) { free(e); return nnz > cap ? OR_ECAP : OR_EINVAL; }
    int64_t pos = 0, t = 0;
    for (int64_t i = 0; i < n; ++i) {
        indptr[i] = pos;
        int64_t t0 = t;
        double deg = -0.0; /* laplacian.rs:367 s.iter().map(w).sum() */
        while (t < u && e[t].key / n == i) { deg = deg + e[t].w; ++t; }
        int diag_done = 0;
        for (int64_t s = t0; s < t; ++s) {
            int32_t j = (int32_t)(e[s].key % n);
            if (!diag_done && j > i) {
                indices[pos] = (int32_t)i; values[pos] = deg; ++pos; diag_done = 1;
            }
            indices[pos] = j; values[pos] = -e[s].w; ++pos;
        }
        if (!diag_done) { indices[pos] = (int32_t)i; values[pos] = deg; ++pos; }
    }
    indptr[n] = pos;
    free(e);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* K2 — A.2 MAX / Stage C (f32)                                              */
/* ------------------------------------------------------------------------ */

typedef struct { int64_t key; float w; } edge32;
static int cmp_edge32(const void *pa, const void *pb) {
    const edge32 *a = (const edge32 *)pa, *b = (const edge32 *)pb;
    if (a->key < b->key) return -1;
    if (a->key > b->key) return 1;
    if (a->w > b->w) return -1;
    if (a->w < b->w) return 1;
    return 0;
}
typedef struct { int64_t key; float v; } ent32;
static int cmp_ent32(const void *pa, const void *pb) {
    const ent32 *a = (const ent32 *)pa, *b = (const ent32 *)pb;
    return a->key < b->key ? -1 : (a->key > b->key ? 1 : 0);
}

int or_laplacian_max(int64_t n, int64_t n_edges, const int32_t *src,
                     const int32_t *dst, const float *w, float thr,
                     int normalize, int64_t cap, int64_t *indptr,
                     int32_t *indices, float *values, int64_t *nnz_out,
                     float *degrees, int64_t *nnz_ref_out) {
    if (n < 1 || n_edges < 0 || !indptr || !nnz_out || !degrees) return OR_EINVAL;
    edge32 *e = (edge32 *)malloc(sizeof(edge32) * (size_t)(n_edges + 1));
    if (!e) return OR_ENOMEM;
    int64_t m = 0;
    for (int64_t t = 0; t < n_edges; ++t) {
        int32_t i = src[t], j = dst[t];
        if (i < 0 || j < 0) continue;
        if (i == j || !(w[t] > thr)) continue; /* laplacian.rs:324 */
        int32_t a = i < j ? i : j, b = i < j ? j : i;
        e[m].key = (int64_t)a * n + b; e[m].w = w[t]; ++m;
    }
    qsort(e, (size_t)m, sizeof(edge32), cmp_edge32);
    int64_t u = 0;
    for (int64_t t = 0; t < m; ++t)
        if (u == 0 || e[t].key != e[u - 1].key) e[u++] = e[t];
    for (int64_t i = 0; i < n; ++i) degrees[i] = 0.0f;
    for (int64_t t = 0; t < u; ++t) {
        int64_t a = e[t].key / n, b = e[t].key % n;
        degrees[a] += e[t].w;
        degrees[b] += e[t].w;
    }
    ent32 *ent = (ent32 *)malloc(sizeof(ent32) * (size_t)(2 * u + n + 1));
    if (!ent) { free(e); return OR_ENOMEM; }
    int64_t q = 0, nnz_ref = 0;
    for (int64_t i = 0; i < n; ++i)
        if (degrees[i] > thr) {
            ent[q].key = i * n + i; ent[q].v = normalize ? 1.0f : degrees[i]; ++q; ++nnz_ref;
        }
    for (int64_t t = 0; t < u; ++t) {
        int64_t a = e[t].key / n, b = e[t].key % n;
        float v;
        if (normalize) {
            float di = degrees[a], dj = degrees[b];
            if (di <= thr || dj <= thr) continue;
            v = -e[t].w / sqrtf(di * dj);
        } else {
            v = -e[t].w;
        }
        ent[q].key = a * n + b; ent[q].v = v; ++q;
        ent[q].key = b * n + a; ent[q].v = v; ++q;
        nnz_ref += 2;
    }
    qsort(ent, (size_t)q, sizeof(ent32), cmp_ent32);
    int64_t nnz = 0;
    for (int64_t t = 0; t < q; ++t) if (fabsf(ent[t].v) > 1e-9f) ++nnz;
    *nnz_out = nnz;
    if (nnz_ref_out) *nnz_ref_out = nnz_ref;
    if (nnz > cap || !indices || !values) { free(e); free(ent); return nnz > cap ? OR_ECAP : OR_EINVAL; }
    int64_t pos = 0, t = 0;
    for (int64_t i = 0; i < n; ++i) {
        indptr[i] = pos;
        while (t < q && ent[t].key / n == i) {
            if (fabsf(ent[t].v) > 1e-9f) { indices[pos] = (int32_t)(ent[t].key % n); values[pos] = ent[t].v; ++pos; }
            ++t;
        }
    }
    indptr[n] = pos;
    free(e); free(ent);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* K3 — energy                                                              */
/* ------------------------------------------------------------------------ */

static int cmp_double(const void *pa, const void *pb) {
    double a = *(const double *)pa, b = *(const double *)pb;
    return a < b ? -1 : (a > b ? 1 : 0);
}

double or_select_tau(const double *x, int64_t n, int mode, double param) {
    const double FLOOR = 1e-10; /* taumode.rs:25 */
    if (mode == OR_TAU_FIXED) return (isfinite(param) && param > 0.0) ? param : FLOOR;
    if (mode == OR_TAU_MEAN) {
        double s = 0.0; int64_t c = 0; /* fold((0.0, 0)) */
        for (int64_t i = 0; i < n; ++i) if (isfinite(x[i])) { s = s + x[i]; ++c; }
        if (c == 0) return FLOOR;
        double m = s / (double)c;
        return m > FLOOR ? m : FLOOR;
    }
    double *v = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    if (!v) return FLOOR;
    int64_t c = 0;
    for (int64_t i = 0; i < n; ++i) if (isfinite(x[i])) v[c++] = x[i];
    if (c == 0) { free(v); return FLOOR; }
    qsort(v, (size_t)c, sizeof(double), cmp_double);
    double r;
    if (mode == OR_TAU_PERCENTILE) {
        double pp = param < 0.0 ? 0.0 : (param > 1.0 ? 1.0 : param);
        if (param != param) pp = param; /* f64::clamp keeps NaN */
        double fidx = round((double)(c - 1) * pp); /* f64::round: half away from zero */
        int64_t idx = (fidx != fidx || fidx < 0) ? 0 : (int64_t)fidx; /* `as usize` saturates, NaN -> 0 */
        if (idx >= c) idx = c - 1; /* unreachable for pp in [0,1] */
        r = v[idx];
    } else if (c % 2 == 1) {
        r = v[c / 2];
    } else {
        r = 0.5 * (v[c / 2 - 1] + v[c / 2]);
    }
    free(v);
    return r > FLOOR ? r : FLOOR; /* f64::max */
}

static inline double fmax0(double a) { return a > 0.0 ? a : 0.0; }
static inline double clamp01(double a) { return a < 0.0 ? 0.0 : (a > 1.0 ? 1.0 : a); }

int or_energy_rows(const float *X, int64_t n_rows, int32_t f,
                   const int64_t *indptr, const int32_t *indices,
                   const double *values, int g_mode, int tau_mode,
                   double tau_param, int nthreads, double *E, double *G,
                   double *lambda) {
    if (!X || n_rows < 0 || f < 1 || !indptr || !indices || !values) return OR_EINVAL;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel
    {
        double *x = (double *)malloc(sizeof(double) * (size_t)f);
        if (!x) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 64)
        for (int64_t r = 0; r < n_rows; ++r) {
            if (!x) continue;
            const float *xr = X + r * (int64_t)f;
            for (int32_t t = 0; t < f; ++t) x[t] = (double)xr[t];
            double e_raw = 0.0, g_raw = 0.0, lam = 0.0;
            if (g_mode == OR_G_TAUMODE) {
                int zero = 1; /* taumode.rs:268-274 */
                for (int32_t t = 0; t < f; ++t) if (!(fabs(x[t]) <= 1e-10)) { zero = 0; break; }
                if (!zero) {
                    /* rayleigh, taumode.rs:340-354 */
                    double num = 0.0;
                    for (int32_t i = 0; i < f; ++i) {
                        double xi = x[i], rs = -0.0;
                        for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p)
                            rs = rs + (xi * values[p]) * x[indices[p]];
                        num = num + rs;
                    }
                    double den = -0.0;
                    for (int32_t t = 0; t < f; ++t) den = den + x[t] * x[t];
                    e_raw = den > 1e-12 ? fmax0(num / den) : 0.0;
                    /* dispersion, taumode.rs:366-408 (CSR order == (i,j) loop order) */
                    double s = 0.0;
                    for (int32_t i = 0; i < f; ++i)
                        for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) {
                            int32_t j = indices[p];
                            if (j == i) continue;
                            double wv = fmax0(-values[p]);
                            if (wv > 0.0) { double dd = x[i] - x[j]; s += wv * dd * dd; }
                        }
                    if (s <= 1e-12) g_raw = 0.0;
                    else {
                        double g = 0.0;
                        for (int32_t i = 0; i < f; ++i)
                            for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) {
                                int32_t j = indices[p];
                                if (j == i) continue;
                                double wv = fmax0(-values[p]);
                                if (wv > 0.0) {
                                    double dd = x[i] - x[j];
                                    double c = wv * dd * dd;
                                    double sh = c / s;
                                    g += sh * sh;
                                }
                            }
                        g_raw = clamp01(g);
                    }
                    double tau = or_select_tau(x, f, tau_mode, tau_param);
                    double eb = e_raw / (e_raw + tau);
                    lam = tau * eb + (1.0 - tau) * clamp01(g_raw);
                }
            } else {
                /* energymaps.rs:961-1037 */
                double num = -0.0, den = -0.0;
                for (int32_t i = 0; i < f; ++i) {
                    double lx = 0.0; /* graph.rs:485 let mut sum = 0.0 */
                    for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) lx += values[p] * x[indices[p]];
                    num = num + x[i] * lx;
                }
                for (int32_t t = 0; t < f; ++t) den = den + x[t] * x[t];
                e_raw = den > 1e-12 ? fmax0(num / den) : 0.0;
                double s = -0.0;
                for (int32_t i = 0; i < f; ++i) {
                    double loc = 0.0;
                    for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) {
                        int32_t j = indices[p];
                        if (j <= i) continue;
                        double wv = fmax0(-values[p]);
                        if (wv > 0.0) { double dd = x[i] - x[j]; loc += wv * dd * dd; }
                    }
                    s = s + loc;
                }
                if (s > 1e-12) {
                    double g = -0.0;
                    for (int32_t i = 0; i < f; ++i) {
                        double loc = 0.0;
                        for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) {
                            int32_t j = indices[p];
                            if (j <= i) continue;
                            double wv = fmax0(-values[p]);
                            if (wv > 0.0) {
                                double dd = x[i] - x[j];
                                double c = wv * dd * dd;
                                double sh = c / s;
                                loc += sh * sh;
                            }
                        }
                        g = g + loc;
                    }
                    g_raw = clamp01(g);
                } else {
                    g_raw = 0.0;
                }
                lam = e_raw;
            }
            if (E) E[r] = e_raw;
            if (G) G[r] = g_raw;
            if (lambda) lambda[r] = lam;
        }
        free(x);
    }
    return err;
}

int or_normalise_lambdas(double *lam, int64_t n, double *min_out,
                         double *max_out, double *range_out) {
    if (!lam || n < 0) return OR_EINVAL;
    double mn = INFINITY, mx = 0.0;
    for (int64_t i = 0; i < n; ++i) mn = fmin(mn, lam[i]); /* f64::min ignores NaN */
    for (int64_t i = 0; i < n; ++i) mx = fmax(mx, lam[i]);
    double range = fmax(mx - mn, 1e-9);
    for (int64_t i = 0; i < n; ++i) lam[i] = (lam[i] - mn) / range;
    if (min_out) *min_out = mn;
    if (max_out) *max_out = mx;
    if (range_out) *range_out = range;
    return 0;
}

int or_spectral_lambdas_f32(const float *X, int64_t n, int32_t f,
                            const int64_t *indptr, const int32_t *indices,
                            const float *values, float *out) {
    if (!X || !out || n < 0 || f < 1) return OR_EINVAL;
    float *deg = (float *)calloc((size_t)f, sizeof(float));
    float *rows = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    if (!deg || !rows) { free(deg); free(rows); return OR_ENOMEM; }
    for (int32_t i = 0; i < f; ++i)
        for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) {
            float wv = -values[p]; if (wv > 0.0f) deg[i] += wv;
        }
    float total = 0.0f;
    for (int64_t r = 0; r < n; ++r) {
        const float *x = X + r * (int64_t)f;
        float num = 0.0f, den = 0.0f, row = 0.0f;
        for (int32_t i = 0; i < f; ++i) {
            float lx = 0.0f, wx = 0.0f, wx2 = 0.0f;
            for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) {
                float xv = x[indices[p]];
                lx += values[p] * xv;
                float wv = -values[p]; if (wv < 0.0f) wv = 0.0f;
                wx += wv * xv; wx2 += wv * (xv * xv);
            }
            num += x[i] * lx;
            den += x[i] * x[i];
            float ee = deg[i] * (x[i] * x[i]) - x[i] * wx * 2.0f + wx2;
            row += ee > 0.0f ? ee : 0.0f;
        }
        float R = num / (den + 1e-9f);
        R = R < -1e6f ? -1e6f : (R > 1e6f ? 1e6f : R);
        out[r] = R;
        rows[r] = row;
        total += row;
    }
    for (int64_t r = 0; r < n; ++r) {
        float D = rows[r] / (total + 1e-12f);
        D = D < 0.0f ? 0.0f : (D > 1.0f ? 1.0f : D);
        out[r] += D;
    }
    free(deg); free(rows);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* K4 — sorted index                                                         */
/* ------------------------------------------------------------------------ */

typedef struct { double lam; int64_t idx; char id[24]; } skey;

/* ordered_float::OrderedFloat Ord: NaN == NaN, NaN > everything; -0 == +0 */
static int cmp_ordered_float(double a, double b) {
    int an = a != a, bn = b != b;
    if (an || bn) return an && bn ? 0 : (an ? 1 : -1);
    return a < b ? -1 : (a > b ? 1 : 0);
}
static int cmp_skey(const void *pa, const void *pb) {
    const skey *a = (const skey *)pa, *b = (const skey *)pb;
    int c = cmp_ordered_float(a->lam, b->lam);
    if (c) return c;
    c = strcmp(a->id, b->id); /* String Ord == byte-wise lexicographic */
    return c;
}

int or_sorted_index(const double *lam, int64_t n, int64_t *order_out,
                    double *key_out, double *std_out) {
    if (!lam || n < 0 || !order_out) return OR_EINVAL;
    if (std_out) {
        /* laplacian.rs:421-448 */
        if (n == 0) *std_out = NAN;
        else {
            double s = -0.0;
            for (int64_t i = 0; i < n; ++i) s = s + lam[i];
            float mean = (float)s / (float)n;
            float var = -0.0f;
            for (int64_t i = 0; i < n; ++i) { float df = mean - (float)lam[i]; var = var + df * df; }
            var = var / (float)n;
            *std_out = (double)sqrtf(var);
        }
    }
    skey *k = (skey *)malloc(sizeof(skey) * (size_t)(n > 0 ? n : 1));
    if (!k) return OR_ENOMEM;
    for (int64_t i = 0; i < n; ++i) {
        k[i].lam = lam[i]; k[i].idx = i;
        /* decimal string of usize */
        char tmp[24]; int len = 0; uint64_t v = (uint64_t)i;
        do { tmp[len++] = (char)('0' + v % 10); v /= 10; } while (v);
        for (int t = 0; t < len; ++t) k[i].id[t] = tmp[len - 1 - t];
        k[i].id[len] = 0;
    }
    qsort(k, (size_t)n, sizeof(skey), cmp_skey);
    /* bucket key = first-inserted (lowest idx) lambda of each equal class */
    int64_t start = 0;
    while (start < n) {
        int64_t end = start + 1;
        while (end < n && cmp_ordered_float(k[end].lam, k[start].lam) == 0) ++end;
        int64_t first = k[start].idx;
        for (int64_t t = start; t < end; ++t) if (k[t].idx < first) first = k[t].idx;
        for (int64_t t = start; t < end; ++t) {
            order_out[t] = k[t].idx;
            if (key_out) key_out[t] = lam[first];
        }
        start = end;
    }
    free(k);
    return 0;
}

/* sorted_index.rs:64-80: BTreeMap::range(OrderedFloat(lo)..=OrderedFloat(hi)) */
int64_t or_range_bylambda(const double *keys, const int64_t *order, int64_t n, double std_dev,
                          double lq, int64_t k, double p, int64_t *out_idx, double *out_key) {
    /* 2.0_f64.powf(p): LLVM rewrites llvm.pow(2.0, p) to exp2(p) in an
       optimised build (LibCallSimplifier::replacePowWithExp) */
    double band = std_dev / exp2(p);
    double lo = lq - band, hi = lq + band;
    if (cmp_ordered_float(lo, hi) > 0) return -1; /* range start > end: panic */
    int64_t cnt = 0;
    for (int64_t r = 0; r < n && cnt < k; ++r)
        if (cmp_ordered_float(keys[r], lo) >= 0 && cmp_ordered_float(keys[r], hi) <= 0) {
            out_idx[cnt] = order[r];
            out_key[cnt] = keys[r];
            ++cnt;
        }
    return cnt;
}

typedef struct { double d; int64_t rank; } nkey;
static int cmp_nkey(const void *pa, const void *pb) {
    const nkey *a = (const nkey *)pa, *b = (const nkey *)pb;
    if (a->d < b->d) return -1;
    if (a->d > b->d) return 1;
    return a->rank < b->rank ? -1 : (a->rank > b->rank ? 1 : 0);
}

/* sorted_index.rs:85-140 */
int64_t or_k_nearest_by_lambda(const double *keys, const int64_t *order, int64_t n,
                               double std_dev, double lq, int64_t k, double lambda_p,
                               int has_base_delta, double base_delta, double growth,
                               double max_multiplier, int64_t *out_idx, double *out_key) {
    if (k == 0 || n == 0) return 0;
    double delta = fabs(has_base_delta ? base_delta : fmax(std_dev * lambda_p, 1e-9));
    if (!(isfinite(growth) && growth > 1.0)) growth = 1.7;
    double max_delta = fmin(delta * fmax(max_multiplier, 1.0), 1.0);
    int64_t r0 = 0, r1 = 0;
    for (;;) {
        double lo = fmax(lq - delta, 0.0), hi = fmin(lq + delta, 1.0); /* f64::max / min */
        if (cmp_ordered_float(lo, hi) > 0) return -1;
        r0 = n; r1 = 0;
        int64_t c = 0;
        for (int64_t r = 0; r < n; ++r)
            if (cmp_ordered_float(keys[r], lo) >= 0 && cmp_ordered_float(keys[r], hi) <= 0) {
                if (c == 0) r0 = r;
                r1 = r + 1;
                ++c;
            }
        if (c == 0) r0 = r1 = 0;
        if (c >= k || delta >= max_delta) break;
        delta = fmin(delta * growth, max_delta);
    }
    int64_t m = r1 - r0;
    if (m <= 0) return 0;
    if (lq != lq && m >= 2) return -1; /* NaN distances: partial_cmp().unwrap() panics */
    nkey *c = (nkey *)malloc(sizeof(nkey) * (size_t)m);
    if (!c) return -2;
    for (int64_t r = r0; r < r1; ++r) { c[r - r0].d = fabs(keys[r] - lq); c[r - r0].rank = r; }
    qsort(c, (size_t)m, sizeof(nkey), cmp_nkey);
    int64_t cnt = m < k ? m : k;
    for (int64_t e = 0; e < cnt; ++e) {
        out_idx[e] = order[c[e].rank];
        out_key[e] = keys[c[e].rank];
    }
    free(c);
    return cnt;
}

int or_diffuse_rows(const double *X, int64_t n, int32_t f, const int64_t *indptr,
                    const int32_t *indices, const double *values, double eta, int32_t steps,
                    int matvec, double *out) {
    if (!X || !out || n < 0 || f < 1 || steps < 0) return OR_EINVAL;
    int err = 0;
#pragma omp parallel
    {
        double *x = (double *)malloc(sizeof(double) * (size_t)f);
        double *lx = (double *)malloc(sizeof(double) * (size_t)f);
        if (!x || !lx) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(static)
        for (int64_t r = 0; r < n; ++r) {
            if (!x || !lx) continue;
            memcpy(x, X + r * (int64_t)f, sizeof(double) * (size_t)f);
            int ns = matvec ? 1 : steps;
            for (int st = 0; st < ns; ++st) {
                for (int32_t i = 0; i < f; ++i) { /* multiply_vector */
                    double sum = 0.0;
                    for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p)
                        sum += values[p] * x[indices[p]];
                    lx[i] = sum;
                }
                for (int32_t i = 0; i < f; ++i) x[i] = matvec ? lx[i] : x[i] - eta * lx[i];
            }
            memcpy(out + r * (int64_t)f, x, sizeof(double) * (size_t)f);
        }
        free(x);
        free(lx);
    }
    return err;
}

/* ---- MST candidate graph (mst.rs:312-412, distance.rs:78-108) ---------- */

float or_bhattacharyya_distance(const float *mean_i, const float *var_i, const float *mean_j,
                                const float *var_j, int64_t f) {
    const float eps = 1e-10f; /* distance.rs:87 */
    float distance = 0.0f;
    for (int64_t k = 0; k < f; ++k) {
        float sigma_i = fmaxf(var_i[k], eps); /* f32::max: NaN -> the other */
        float sigma_j = fmaxf(var_j[k], eps);
        float sigma_sum = sigma_i + sigma_j;
        float sigma_prod = sigma_i * sigma_j;
        float mean_diff = mean_i[k] - mean_j[k];
        float mahalanobis = 0.25f * (mean_diff * mean_diff) / sigma_sum;
        float log_term = 0.25f * logf(fmaxf(sigma_sum / (2.0f * sqrtf(sigma_prod)), eps));
        distance += mahalanobis + log_term;
    }
    return distance;
}

typedef struct { float d; int32_t j; } mstc;
static int cmp_mstc(const void *pa, const void *pb) { /* stable sort_by on ascending j */
    const mstc *a = (const mstc *)pa, *b = (const mstc *)pb;
    if (a->d < b->d) return -1;
    if (a->d > b->d) return 1;
    return a->j < b->j ? -1 : (a->j > b->j ? 1 : 0);
}

int or_mst_candidates(const float *means, const float *vars, int64_t c, int32_t f, int32_t k,
                      int metric, int tw, const float *thickness, int32_t *out_v,
                      float *out_dist, float *out_cost) {
    if (!means || !out_v || !out_dist || !out_cost || c < 2 || f < 1 || k < 1) return OR_EINVAL;
    if (metric < 0 || metric > 2 || tw < 0 || tw > 4) return OR_EINVAL;
    if ((metric == 0 || !thickness) && !vars) return OR_EINVAL;
    const int64_t kk = k < c - 1 ? k : c - 1; /* mst.rs:317 */
    float *th = (float *)malloc(sizeof(float) * (size_t)c);
    if (!th) return OR_ENOMEM;
    for (int64_t i = 0; i < c; ++i) {
        if (thickness) { th[i] = thickness[i]; continue; }
        float s = 0.0f; /* centroid.rs:107-109 (Burn's order unspecified) */
        for (int32_t t = 0; t < f; ++t) s += vars[i * f + t];
        th[i] = s / (float)f;
    }
    int err = 0;
#pragma omp parallel
    {
        mstc *sc = (mstc *)malloc(sizeof(mstc) * (size_t)c);
        if (!sc) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 4)
        for (int64_t i = 0; i < c; ++i) {
            if (!sc) continue;
            int64_t m = 0;
            for (int64_t j = 0; j < c; ++j) {
                if (j == i) continue;
                float d;
                if (metric == 0) {
                    d = or_bhattacharyya_distance(means + i * f, vars + i * f, means + j * f,
                                                  vars + j * f, f);
                } else {
                    float s = 0.0f; /* mst.rs:383-397 */
                    for (int32_t t = 0; t < f; ++t) {
                        float diff = means[i * f + t] - means[j * f + t];
                        s += diff * diff;
                    }
                    d = metric == 1 ? sqrtf(s) : s;
                }
                if (d != d) {
#pragma omp atomic write
                    err = OR_ENONFINITE;
                }
                sc[m].d = d;
                sc[m].j = (int32_t)j;
                ++m;
            }
            qsort(sc, (size_t)m, sizeof(mstc), cmp_mstc);
            for (int64_t r = 0; r < kk; ++r) {
                const float d = sc[r].d, ti = th[i], tj = th[sc[r].j];
                float cost;
                switch (tw) { /* mst.rs:400-412 */
                case 0: cost = d * ((ti + tj) / 2.0f); break;
                case 1: cost = d * fminf(ti, tj); break;
                case 2: cost = d * fmaxf(ti, tj); break;
                case 3: cost = d * sqrtf(ti * tj); break;
                default: cost = d; break;
                }
                out_v[i * kk + r] = sc[r].j;
                out_dist[i * kk + r] = d;
                out_cost[i * kk + r] = cost;
            }
        }
        free(sc);
    }
    free(th);
    return err;
}

int or_nearest_centroid(const float *batch, int64_t b, const float *cents, int64_t c, int32_t f,
                        int32_t *out_idx, float *out_dist) {
    if (!batch || !cents || !out_idx || !out_dist || b < 1 || c < 1 || f < 1) return OR_EINVAL;
    float *cn = (float *)malloc(sizeof(float) * (size_t)c);
    if (!cn) return OR_ENOMEM;
    for (int64_t j = 0; j < c; ++j) {
        float s = 0.0f;
        for (int32_t t = 0; t < f; ++t) s = s + cents[j * f + t] * cents[j * f + t];
        cn[j] = s;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < b; ++i) {
        const float *x = batch + i * f;
        float bn = 0.0f;
        for (int32_t t = 0; t < f; ++t) bn = bn + x[t] * x[t];
        float best = NAN, first = NAN;
        int32_t bj = -1;
        for (int64_t j = 0; j < c; ++j) {
            float dot = 0.0f;
            for (int32_t t = 0; t < f; ++t) dot = dot + x[t] * cents[j * f + t];
            const float dd = sqrtf((bn + cn[j]) - 2.0f * dot);
            if (j == 0) first = dd;
            if (dd == dd && (bj < 0 || dd < best)) { best = dd; bj = (int32_t)j; }
        }
        out_idx[i] = bj < 0 ? 0 : bj;
        out_dist[i] = bj < 0 ? first : best;
    }
    free(cn);
    return 0;
}

typedef struct { float w; int32_t j; } bcent;
static int cmp_bcent(const void *pa, const void *pb) {
    const bcent *a = (const bcent *)pa, *b = (const bcent *)pb;
    if (a->w > b->w) return -1;
    if (a->w < b->w) return 1;
    return a->j < b->j ? -1 : (a->j > b->j ? 1 : 0);
}

int or_bc_knn(const float *means, const float *vars, int64_t c, int32_t f, int32_t k,
              float reg, float thr, int32_t *out_idx, float *out_w) {
    if (!means || !vars || !out_idx || !out_w || c < 1 || f < 2 || k < 1) return OR_EINVAL;
    int err = 0;
#pragma omp parallel
    {
        bcent *sc = (bcent *)malloc(sizeof(bcent) * (size_t)f);
        if (!sc) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 4)
        for (int32_t i = 0; i < f; ++i) {
            if (!sc) continue;
            int32_t m = 0;
            for (int32_t j = 0; j < f; ++j) {
                if (j == i) continue;
                float db = 0.0f; /* distance.rs:271-286 */
                for (int64_t t = 0; t < c; ++t) {
                    float vi = fmaxf(vars[t * f + i], reg), vj = fmaxf(vars[t * f + j], reg);
                    float vs = vi + vj;
                    float d = means[t * f + i] - means[t * f + j];
                    float mean_term = (d * d) / (4.0f * vs);
                    float log_term = 0.5f * logf(vs / (2.0f * sqrtf(vi * vj)));
                    db += mean_term + log_term;
                }
                float w = expf(-db);
                w = w < 0.0f ? 0.0f : (w > 1.0f ? 1.0f : w);
                if (w > thr) { sc[m].w = w; sc[m].j = j; ++m; } /* laplacian.rs:282 */
            }
            qsort(sc, (size_t)m, sizeof(bcent), cmp_bcent);
            int32_t kk = k < f - 1 ? k : f - 1;
            for (int32_t r = 0; r < k; ++r) {
                int ok = r < kk && r < m;
                out_idx[(int64_t)i * k + r] = ok ? sc[r].j : -1;
                out_w[(int64_t)i * k + r] = ok ? sc[r].w : 0.0f;
            }
        }
        free(sc);
    }
    return err;
}

/* ------------------------------------------------------------------------ */
/* K5 — SF-GRASS                                                             */
/* ------------------------------------------------------------------------ */

typedef struct { double score; double w; int32_t j; int32_t pos; } sedge;
static int cmp_sedge(const void *pa, const void *pb) {
    const sedge *a = (const sedge *)pa, *b = (const sedge *)pb;
    /* b.2.partial_cmp(a.2).unwrap_or(Equal): descending; NaN compares Equal */
    if (a->score > b->score) return -1;
    if (a->score < b->score) return 1;
    return a->pos < b->pos ? -1 : (a->pos > b->pos ? 1 : 0);
}

int or_sfgrass(int64_t n, const int64_t *indptr, const int32_t *indices,
               const double *w, double ratio, int64_t *out_indptr,
               int32_t *out_indices, double *out_w) {
    if (n < 1 || !indptr || !out_indptr) return OR_EINVAL;
    int64_t orig = indptr[n] - indptr[0];
    double avg = (double)orig / (double)n;
    out_indptr[0] = 0;
    if (avg < 10.0) {
        for (int64_t i = 0; i < n; ++i) {
            int64_t o = out_indptr[i];
            for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p, ++o) {
                out_indices[o] = indices[p]; out_w[o] = w[p];
            }
            out_indptr[i + 1] = o;
        }
        return 0;
    }
    int64_t maxlen = 0;
    for (int64_t i = 0; i < n; ++i) if (indptr[i + 1] - indptr[i] > maxlen) maxlen = indptr[i + 1] - indptr[i];
    sedge *buf = (sedge *)malloc(sizeof(sedge) * (size_t)(maxlen + 1));
    if (!buf) return OR_ENOMEM;
    for (int64_t i = 0; i < n; ++i) {
        int64_t len = indptr[i + 1] - indptr[i];
        int64_t o = out_indptr[i];
        if (len > 0) {
            uint64_t di = (uint64_t)len;
            for (int64_t p = 0; p < len; ++p) {
                int32_t j = indices[indptr[i] + p];
                uint64_t dj = (uint64_t)(indptr[j + 1] - indptr[j]);
                buf[p].w = w[indptr[i] + p];
                buf[p].score = buf[p].w * sqrt((double)(di * dj));
                buf[p].j = j; buf[p].pos = (int32_t)p;
            }
            qsort(buf, (size_t)len, sizeof(sedge), cmp_sedge);
            int64_t keep = (int64_t)ceil((double)len * ratio);
            if (keep < 1) keep = 1;
            if (keep > len) keep = len;
            for (int64_t p = 0; p < keep; ++p, ++o) { out_indices[o] = buf[p].j; out_w[o] = buf[p].w; }
        }
        out_indptr[i + 1] = o;
    }
    free(buf);
    return 0;
}

/* ---- §8(f) rank 2: lambda-aware search (core.rs:1156-1193) ------------- */

typedef struct { double s; int64_t i; } sscore;
/* sort_by(|a, b| b.1.partial_cmp(&a.1)) over ascending i, stable: score
 * descending, equal scores (0.0 == -0.0 included) by ascending i. */
static int cmp_sscore(const void *pa, const void *pb) {
    const sscore *a = (const sscore *)pa, *b = (const sscore *)pb;
    if (a->s > b->s) return -1;
    if (a->s < b->s) return 1;
    return a->i < b->i ? -1 : (a->i > b->i ? 1 : 0);
}

/* ArrowItem::norm, core.rs:210-214: sequential f64 sum of x*x, sqrt */
static double item_norm(const double *a, int32_t f) {
    double s = -0.0; /* Rust >= 1.83 float Sum starts at -0.0 */
    for (int32_t t = 0; t < f; ++t) s = s + a[t] * a[t];
    return sqrt(s);
}

int or_search_lambda_aware(const double *X, int64_t n, int32_t f, const double *lambdas,
                           const double *Q, const double *lambda_q, int64_t nq, int64_t k,
                           double alpha, int nthreads, int64_t *out_idx, double *out_score,
                           int64_t *out_count) {
    if (n < 0 || f < 0 || nq < 0 || k < 0) return -1;
    set_threads(nthreads);
    double *xn = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    if (!xn) return -2;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) xn[i] = item_norm(X + (size_t)i * f, f);
    int rc = 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t q = 0; q < nq; ++q) {
        const double *qv = Q + (size_t)q * f;
        int64_t *oi = out_idx + (size_t)q * k;
        double *os = out_score + (size_t)q * k;
        for (int64_t r = 0; r < k; ++r) { oi[r] = -1; os[r] = NAN; }
        if (lambda_q[q] == 0.0) { out_count[q] = -1; continue; } /* core.rs:1169-1172 */
        sscore *sc = (sscore *)malloc(sizeof(sscore) * (size_t)(n > 0 ? n : 1));
        if (!sc) { rc = -2; continue; }
        const double qn = item_norm(qv, f);
        int nan = 0;
        for (int64_t i = 0; i < n; ++i) {
            const double *x = X + (size_t)i * f;
            const double denom = qn * xn[i];
            double cs = 0.0;
            if (denom > 0.0) {
                double dot = -0.0;
                for (int32_t t = 0; t < f; ++t) dot = dot + qv[t] * x[t];
                cs = dot / denom;
            }
            const double ld = fabs(lambda_q[q] - lambdas[i]);
            const double ls = 1.0 - fmin(ld, 1.0);
            const double s = alpha * cs + (1.0 - alpha) * ls;
            if (isnan(s)) nan = 1;
            sc[i].s = s;
            sc[i].i = i;
        }
        if (nan) { out_count[q] = -3; free(sc); continue; }
        qsort(sc, (size_t)n, sizeof(sscore), cmp_sscore);
        const int64_t c = k < n ? k : n;
        for (int64_t r = 0; r < c; ++r) { oi[r] = sc[r].i; os[r] = sc[r].s; }
        out_count[q] = c;
        free(sc);
    }
    free(xn);
    return rc;
}

/* ArrowSpace::search_lambda_aware_hybrid (core.rs:1196-1318), deterministic
 * restatement: lambda top-k by (score desc, i asc) (the reference's parallel
 * heap keeps an unspecified member of a tie class), every item with cosine >
 * 0.9999 (score = cosine), the best-cosine item (smallest i on ties; the
 * reference's rayon reduce picks an unspecified one); union with the first
 * insertion winning (high-semantic, then lambda top-k, then best cosine);
 * sorted by (score desc, i asc) (sort_unstable: ties unspecified), first k. */
int or_search_lambda_aware_hybrid(const double *X, int64_t n, int32_t f, const double *lambdas,
                                  const double *Q, const double *lambda_q, int64_t nq,
                                  int64_t k, double alpha, int nthreads, int64_t *out_idx,
                                  double *out_score, int64_t *out_count) {
    if (n < 0 || f < 0 || nq < 0 || k < 0) return -1;
    set_threads(nthreads);
    double *xn = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    if (!xn) return -2;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) xn[i] = item_norm(X + (size_t)i * f, f);
    int rc = 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t q = 0; q < nq; ++q) {
        const double *qv = Q + (size_t)q * f;
        int64_t *oi = out_idx + (size_t)q * k;
        double *os = out_score + (size_t)q * k;
        for (int64_t r = 0; r < k; ++r) { oi[r] = -1; os[r] = NAN; }
        out_count[q] = 0;
        if (k == 0) continue;
        sscore *sc = (sscore *)malloc(sizeof(sscore) * (size_t)(n > 0 ? n : 1));
        double *cosv = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
        sscore *u = (sscore *)malloc(sizeof(sscore) * (size_t)(n + k + 1));
        char *in = (char *)calloc((size_t)(n > 0 ? n : 1), 1);
        if (!sc || !cosv || !u || !in) { rc = -2; free(sc); free(cosv); free(u); free(in); continue; }
        const double qn = item_norm(qv, f);
        int nan = 0;
        int64_t best = -1;
        for (int64_t i = 0; i < n; ++i) {
            const double *x = X + (size_t)i * f;
            const double denom = qn * xn[i];
            double cs = 0.0;
            if (denom > 0.0) {
                double dot = -0.0;
                for (int32_t t = 0; t < f; ++t) dot = dot + qv[t] * x[t];
                cs = dot / denom;
            }
            cosv[i] = cs;
            const double ls = 1.0 - fmin(fabs(lambda_q[q] - lambdas[i]), 1.0);
            const double s = alpha * cs + (1.0 - alpha) * ls;
            if (isnan(s)) nan = 1;
            sc[i].s = s;
            sc[i].i = i;
            if (best < 0 || cs > cosv[best]) best = i;
        }
        if (nan) { out_count[q] = -3; free(sc); free(cosv); free(u); free(in); continue; }
        int64_t nu = 0;
        for (int64_t i = 0; i < n; ++i)
            if (cosv[i] > 0.9999) { u[nu].s = cosv[i]; u[nu].i = i; ++nu; in[i] = 1; }
        qsort(sc, (size_t)n, sizeof(sscore), cmp_sscore);
        for (int64_t r = 0; r < k && r < n; ++r)
            if (!in[sc[r].i]) { u[nu++] = sc[r]; in[sc[r].i] = 1; }
        if (best >= 0 && !in[best]) { u[nu].s = cosv[best]; u[nu].i = best; ++nu; }
        qsort(u, (size_t)nu, sizeof(sscore), cmp_sscore);
        const int64_t c = k < nu ? k : nu;
        for (int64_t r = 0; r < c; ++r) { oi[r] = u[r].i; os[r] = u[r].s; }
        out_count[q] = c;
        free(sc); free(cosv); free(u); free(in);
    }
    free(xn);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* K1 — f64 Euclidean call sites (topk_by_l2 / prepare_query_item / Two-NN) */
/* ------------------------------------------------------------------------ */

/* energymaps.rs:881-885 / core.rs:895-900 / clustering.rs:160-165:
 * zip().map((a-b)*(a-b)).sum::<f64>() — sequential, from -0.0 */
static inline double fold_l2sq_f64(const double *a, const double *b, int32_t d) {
    double acc = -0.0;
    for (int32_t t = 0; t < d; ++t) {
        double diff = a[t] - b[t];
        acc = acc + diff * diff;
    }
    return acc;
}

int or_knn_l2_f64(const double *Q, int64_t nq, const double *C, int64_t nc, int32_t d,
                  const int64_t *q_ids, int32_t k, int use_sqrt, int nthreads,
                  int32_t *out_idx, double *out_dist) {
    if (!Q || !C || !out_idx || !out_dist || nq < 0 || nc < 0 || d < 1 || k < 1)
        return OR_EINVAL;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t q = 0; q < nq; ++q) {
        /* sorted (d, j) list of the k best: insertion keeps the stable order */
        double *bd = (double *)malloc(sizeof(double) * (size_t)k);
        int32_t *bj = (int32_t *)malloc(sizeof(int32_t) * (size_t)k);
        int32_t cnt = 0;
        const double *qr = Q + q * (int64_t)d;
        for (int64_t j = 0; j < nc; ++j) {
            if (q_ids && q_ids[q] == j) continue;
            double v = fold_l2sq_f64(qr, C + j * (int64_t)d, d);
            if (use_sqrt) v = sqrt(v);
            if (v != v) {
#pragma omp atomic write
                err = OR_ENONFINITE;
                break;
            }
            if (cnt == k && !(v < bd[k - 1])) continue; /* later j loses ties */
            int32_t p = cnt < k ? cnt : k - 1;
            while (p > 0 && v < bd[p - 1]) {
                bd[p] = bd[p - 1];
                bj[p] = bj[p - 1];
                --p;
            }
            bd[p] = v;
            bj[p] = (int32_t)j;
            if (cnt < k) ++cnt;
        }
        for (int32_t r = 0; r < k; ++r) {
            out_idx[q * k + r] = r < cnt ? bj[r] : -1;
            out_dist[q * k + r] = r < cnt ? bd[r] : INFINITY;
        }
        free(bd);
        free(bj);
    }
    return err;
}

/* ------------------------------------------------------------------------ */
/* K3 faithful cost model (taumode.rs:366-408 with CsMat::get)               */
/* ------------------------------------------------------------------------ */

/* sprs CsMat::get(i, j) on a CSR matrix with sorted indices: binary search */
static inline double csr_get(const int64_t *indptr, const int32_t *indices, const double *values,
                             int32_t i, int32_t j) {
    int64_t lo = indptr[i], hi = indptr[i + 1];
    while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        if (indices[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    return (lo < indptr[i + 1] && indices[lo] == j) ? values[lo] : 0.0;
}

int or_energy_rows_faithful(const float *X, int64_t n_rows, int32_t f,
                            const int64_t *indptr, const int32_t *indices,
                            const double *values, int tau_mode, double tau_param,
                            int nthreads, double *E, double *G, double *lambda) {
    if (!X || n_rows < 0 || f < 1 || !indptr || !indices || !values) return OR_EINVAL;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel
    {
        double *x = (double *)malloc(sizeof(double) * (size_t)f);
        if (!x) {
#pragma omp atomic write
            err = OR_ENOMEM;
        }
#pragma omp for schedule(dynamic, 4)
        for (int64_t r = 0; r < n_rows; ++r) {
            if (!x) continue;
            const float *xr = X + r * (int64_t)f;
            for (int32_t t = 0; t < f; ++t) x[t] = (double)xr[t];
            double e_raw = 0.0, g_raw = 0.0, lam = 0.0;
            int zero = 1;
            for (int32_t t = 0; t < f; ++t) if (!(fabs(x[t]) <= 1e-10)) { zero = 0; break; }
            if (!zero) {
                double num = 0.0;
                for (int32_t i = 0; i < f; ++i) {
                    double xi = x[i], rs = -0.0;
                    for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p)
                        rs = rs + (xi * values[p]) * x[indices[p]];
                    num = num + rs;
                }
                double den = -0.0;
                for (int32_t t = 0; t < f; ++t) den = den + x[t] * x[t];
                e_raw = den > 1e-12 ? fmax0(num / den) : 0.0;
                double s = 0.0;
                for (int32_t i = 0; i < f; ++i)
                    for (int32_t j = 0; j < f; ++j) {
                        if (i == j) continue;
                        double wv = fmax0(-csr_get(indptr, indices, values, i, j));
                        if (wv > 0.0) { double dd = x[i] - x[j]; s += wv * dd * dd; }
                    }
                if (s <= 1e-12) g_raw = 0.0;
                else {
                    double g = 0.0;
                    for (int32_t i = 0; i < f; ++i)
                        for (int32_t j = 0; j < f; ++j) {
                            if (i == j) continue;
                            double wv = fmax0(-csr_get(indptr, indices, values, i, j));
                            if (wv > 0.0) {
                                double dd = x[i] - x[j];
                                double c = wv * dd * dd;
                                double sh = c / s;
                                g += sh * sh;
                            }
                        }
                    g_raw = clamp01(g);
                }
                double tau = or_select_tau(x, f, tau_mode, tau_param);
                double eb = e_raw / (e_raw + tau);
                lam = tau * eb + (1.0 - tau) * clamp01(g_raw);
            }
            if (E) E[r] = e_raw;
            if (G) G[r] = g_raw;
            if (lambda) lambda[r] = lam;
        }
        free(x);
    }
    return err;
}
