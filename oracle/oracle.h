/*
 * oracle.h — CPU restatement of the matternet-rs (crate `surfface`) hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may
 * load liboracle.so, and only as the checker (or the timed CPU baseline),
 * never as the thing measured or shipped.  The HIP library
 * (matternet-rs_amd/csrc, include/matternet_hip.h) never links or calls it.
 *
 * Provenance / pinning.  The reference is Rust; no Rust toolchain exists in
 * this image and the hot-path sources (src_legacy/) are not a compile target
 * of the reference workspace, so the reference cannot be built here
 * (SURVEY.md §8c).  The reference ships no golden vectors.  This restatement
 * is therefore pinned by (1) every known-answer test the reference's own test
 * suites hold for this path (tests/golden/reference_known_answers.json, each
 * case citing its reference test file:line), and (2) an independent
 * pure-Python restatement (tests/golden/make_golden.py) whose small-case
 * outputs are committed as fixtures.  Bit patterns beyond those fixtures are
 * pinned only by the arithmetic contracts transcribed from the reference
 * (SURVEY.md Appendix A), cited per function below.
 *
 * Build: oracle/Makefile (gcc -O3 -fno-fast-math -ffp-contract=off -fopenmp).
 * All functions return 0 on success, negative on error (-1 EINVAL,
 * -3 non-finite distance: the reference panics in partial_cmp().unwrap()).
 */
#ifndef MATTERNET_ORACLE_H
#define MATTERNET_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- K1: brute-force kNN ------------------------------------------------ */

/* A.1  L2^2 kNN over rows of X [n][d] f32 row-major.
 *   surfface-core/src/distance.rs:206-213 (squared_euclidean_distance_slice:
 *   sequential f32 fold of (a-b)^2, no FMA), surfface-core/src/mst.rs:330-360
 *   (build_candidate_graph: j != i, stable sort_by(partial_cmp) => ties by
 *   ascending j, truncate k = min(k, n-1)).
 * Query rows [q_begin, q_end) are computed; outputs are indexed by
 * (i - q_begin) * k.  Slots beyond min(k, n-1) get idx -1, dist +inf.
 * mode 0 = faithful (full stable sort of all n-1 candidates, as the
 * reference), mode 1 = restated-efficient (bounded max-heap on the same
 * (dist, j) total order; identical output).  nthreads <= 0 => OpenMP default.
 */
int or_knn_l2sq_f32(const float *X, int64_t n, int32_t d, int32_t k,
                    int64_t q_begin, int64_t q_end, int mode, int nthreads,
                    int32_t *out_idx, float *out_dist);

/* A.1 on an explicit list of query rows (rows[t] in [0,n)): output row t is
 * the kNN of X[rows[t]] over all of X (self excluded).  Used for sampled
 * parity checks and the sampled CPU baseline. */
int or_knn_l2sq_rows_f32(const float *X, int64_t n, int32_t d, int32_t k,
                         const int64_t *rows, int64_t nrows, int nthreads,
                         int32_t *out_idx, float *out_dist);

/* A.1 per-shard form: queries Q [nq][d] with global ids
 * q_ids[nq] against corpus C [nc][d] with global ids c_off + j; the equal-id
 * pair skipped when excl; output ids global, (dist, id) order. */
int or_knn_l2sq_qc_f32(const float *Q, int64_t nq, const int64_t *q_ids, const float *C,
                       int64_t nc, int32_t d, int64_t c_off, int32_t k, int excl, int nthreads,
                       int32_t *out_idx, float *out_dist);

/* A.1c rectified-cosine kNN, f64 arithmetic on exactly-widened f32 inputs.
 *   src_legacy/tests/test_helpers.rs:77-126 (build_adjacency_matrix):
 *   norms sqrt(sum x*x) sequential f64; dot sequential f64;
 *   cos = denom > 1e-12 ? clamp(dot/denom,-1,1) : 0; dist = 1 - max(cos,0);
 *   keep dist <= eps and w = 1/(1+(dist/sigma)^p) > 1e-12;
 *   sort by (dist asc, j asc); truncate topk.
 * out_w may be NULL.  Unused slots: idx -1, dist +inf, w 0.
 */
int or_knn_cos_f64(const float *X, int64_t n, int32_t d, int32_t topk,
                   double eps, double sigma, double p,
                   int64_t q_begin, int64_t q_end, int nthreads,
                   int32_t *out_idx, double *out_dist, double *out_w);
/* The same over f64 rows (products rounded in f64 like the reference's). */
int or_knn_cos_f64d(const double *X, int64_t n, int32_t d, int32_t topk,
                    double eps, double sigma, double p,
                    int64_t q_begin, int64_t q_end, int nthreads,
                    int32_t *out_idx, double *out_dist, double *out_w);

/* A.1c on bf16 rows (bf16 bits, row-major [n][d]) for explicit query rows
 * (config 5 parity samples); outputs [nrows][topk]. */
int or_knn_cos_bf16_rows(const uint16_t *X, int64_t n, int32_t d, int32_t topk,
                         double eps, double sigma, double p,
                         const int64_t *rows, int64_t nrows, int nthreads,
                         int32_t *out_idx, double *out_dist, double *out_w);

/* f64 Euclidean kNN, the reference's three f64 call sites (exact folds):
 *  - topk_by_l2 (src_legacy/energymaps.rs:875-892): d = sum (a-b)*(a-b),
 *    f64 sequential fold, j != i, stable sort_by(partial_cmp), truncate k;
 *  - prepare_query_item energy mode (src_legacy/core.rs:872-909): d =
 *    sqrt(sum (a-b).powi(2)), 1-NN with strict '<' (lowest index among ties);
 *  - estimate_intrinsic_dimension (src_legacy/clustering.rs:132-195): sqrt'd
 *    distances of sampled rows to all j != i, stable sort, d1 and d2.
 * Queries Q [nq][d], corpus C [nc][d] (f64, row-major); q_ids[q] (may be
 * NULL) = the corpus index excluded for query q.  use_sqrt: order and report
 * sqrt(d) (ties under the rounded root go to the smaller index, as the
 * reference's stable sort / strict '<' on the rooted values).  out_idx
 * [nq][k] (-1 padded), out_dist [nq][k] (+inf padded).  OR_ENONFINITE if a
 * distance is NaN (the reference's partial_cmp().unwrap() panics). */
int or_knn_l2_f64(const double *Q, int64_t nq, const double *C, int64_t nc, int32_t d,
                  const int64_t *q_ids, int32_t k, int use_sqrt, int nthreads,
                  int32_t *out_idx, double *out_dist);

/* ---- K2: Laplacian assembly --------------------------------------------- */

/* A.2 UNION / unnormalised (legacy).
 *   src_legacy/laplacian.rs:297-348 (_symmetrise_adjancency: every directed
 *   edge inserted as (i,j,w) and (j,i,w), self loops dropped, rows sorted by
 *   j) and :351-419 (_build_sparse_laplacian: L_ii = sum_j w_ij sequential
 *   f64 in ascending j starting from -0.0 (Rust >= 1.83 float Sum), stored
 *   for every i; L_ij = -w_ij; CSR sorted by (row, col)).
 * Input: directed neighbour rows nbr_idx/nbr_w [n][k] (idx < 0 = empty slot).
 * When both (i,j) and (j,i) exist with different weights the reference's
 * DashMap keeps whichever write lands last (nondeterministic); this contract
 * keeps the larger weight (identical for symmetric metrics).
 * Output CSR: indptr [n+1] int64, indices/values capacity `cap`.
 */
int or_laplacian_union(int64_t n, int32_t k, const int32_t *nbr_idx,
                       const double *nbr_w, int64_t cap, int64_t *indptr,
                       int32_t *indices, double *values, int64_t *nnz_out);

/* A.2 MAX / Stage C (f32).
 *   surfface-core/src/laplacian.rs:320-394 (build_laplacian_flat: undirected
 *   key (min,max) with max weight; drop i==j or w <= thr; degrees f32;
 *   normalize: L_ii = 1 iff d_i > thr, L_ij = -w/sqrt(d_i d_j) iff both
 *   > thr; else L_ii = d_i iff d_i > thr, L_ij = -w) and :209-219 (dense ->
 *   CSR keeps |v| > 1e-9).
 * Degree summation order in the reference is DashMap iteration order (not
 * reproducible); here: undirected edges in ascending (min,max) key order.
 * nnz_ref_out receives the reference's `nnz` counter (pre-filter count).
 */
int or_laplacian_max(int64_t n, int64_t n_edges, const int32_t *src,
                     const int32_t *dst, const float *w, float thr,
                     int normalize, int64_t cap, int64_t *indptr,
                     int32_t *indices, float *values, int64_t *nnz_out,
                     float *degrees, int64_t *nnz_ref_out);

/* ---- K3: energy row reductions ------------------------------------------ */

enum { OR_TAU_FIXED = 0, OR_TAU_MEDIAN = 1, OR_TAU_MEAN = 2, OR_TAU_PERCENTILE = 3 };
enum { OR_G_TAUMODE = 0, OR_G_ENERGYMAPS = 1 };

/* src_legacy/taumode.rs:29-70 (select_tau; TAU_FLOOR = 1e-10 at :25). */
double or_select_tau(const double *x, int64_t n, int mode, double param);

/* Per row x (f32 storage widened to f64) of X [n_rows][f] against CSR L
 * (f x f, f64 values):
 *  g_mode OR_G_TAUMODE: src_legacy/taumode.rs:261-408
 *    zero test all |x_t| <= 1e-10 => lambda 0 (:268-274, approx::relative_eq);
 *    E = rayleigh (:326-361) num = sum_i sum_{j in row i} (x_i*L_ij)*x_j,
 *        den = sum x^2, E = den > 1e-12 ? max(num/den, 0) : 0
 *        (reference sums with rayon par_bridge: order nondeterministic; here
 *        rows ascending, entries ascending);
 *    G over ordered pairs i != j with w = max(-L_ij,0) > 0 (:366-408);
 *    tau = select_tau(x); lambda = tau*E/(E+tau) + (1-tau)*clamp(G,0,1).
 *  g_mode OR_G_ENERGYMAPS: src_legacy/energymaps.rs:923-1045
 *    E = max(x.(Lx)/x.x, 0) with (Lx)_i = sum_j L_ij x_j (graph.rs:464-501);
 *    G over j > i only; lambda = E (tau unused, G reported separately).
 * E, G, lambda: [n_rows] (any may be NULL).
 */
int or_energy_rows(const float *X, int64_t n_rows, int32_t f,
                   const int64_t *indptr, const int32_t *indices,
                   const double *values, int g_mode, int tau_mode,
                   double tau_param, int nthreads, double *E, double *G,
                   double *lambda);

/* The same TAUMODE rows computed as the reference writes them (the FAITHFUL
 * CPU baseline of BASELINE.md): compute_item_dispersion's two passes over all
 * F^2 ordered pairs with a CsMat::get (binary search of row i) per pair
 * (src_legacy/taumode.rs:366-408); Rayleigh by CSR rows (:340-354).  Values
 * equal or_energy_rows(G_TAUMODE) (zero pairs add +0.0); only the cost
 * differs. */
int or_energy_rows_faithful(const float *X, int64_t n_rows, int32_t f,
                            const int64_t *indptr, const int32_t *indices,
                            const double *values, int tau_mode, double tau_param,
                            int nthreads, double *E, double *G, double *lambda);

/* src_legacy/core.rs:1341-1354 normalise_lambdas: min = fold(+inf,min),
 * max = fold(0.0,max), range = max(max-min,1e-9), x' = (x-min)/range. */
int or_normalise_lambdas(double *lam, int64_t n, double *min_out,
                         double *max_out, double *range_out);

/* surfface-core/src/spectral/mod.rs:69-181 (compute_lambdas_gpu, f32):
 * R = clamp(num/(den+1e-9), -1e6, 1e6); W = max(0,-L); deg = W.1;
 * row = sum_f max(0, deg_f x_f^2 - 2 x_f (Wx)_f + (Wx^2)_f);
 * D = clamp(row / (sum rows + 1e-12), 0, 1); lambda = R + D.
 * (Burn matmul summation order is backend-defined: tolerance only.) */
int or_spectral_lambdas_f32(const float *X, int64_t n, int32_t f,
                            const int64_t *indptr, const int32_t *indices,
                            const float *values, float *out);

/* ---- K4: sorted lambda index -------------------------------------------- */

/* src_legacy/sorted_index.rs:22-54: ascending OrderedFloat(lambda) (all NaN
 * equal and greatest, -0.0 == +0.0), ties by decimal-string id compared as
 * bytes ("10" < "2").  order_out[r] = idx at rank r; key_out[r] = the
 * bucket key (first-inserted lambda of the equal class).  std_out (may be
 * NULL) = laplacian.rs:421-448 std_deviation (f32 arithmetic). */
int or_sorted_index(const double *lam, int64_t n, int64_t *order_out,
                    double *key_out, double *std_out);

/* src_legacy/sorted_index.rs:64-80 range_bylambda and :85-140
 * k_nearest_by_lambda over a built index (keys/order as or_sorted_index
 * returns them: the BTreeMap flattened in key order), one query lambda.
 * Writes up to k (idx, key) pairs, returns the count, or -1 where the
 * reference panics (range start > end; NaN distance compare).
 * k_nearest: candidates = every item in the final window, sorted stably by
 * |key - lq| (the reference's sort_unstable leaves tie order unspecified;
 * the contract is index order), truncated to k. */
int64_t or_range_bylambda(const double *keys, const int64_t *order, int64_t n, double std_dev,
                          double lq, int64_t k, double p, int64_t *out_idx, double *out_key);
int64_t or_k_nearest_by_lambda(const double *keys, const int64_t *order, int64_t n,
                               double std_dev, double lq, int64_t k, double lambda_p,
                               int has_base_delta, double base_delta, double growth,
                               double max_multiplier, int64_t *out_idx, double *out_key);

/* src_legacy/energymaps.rs:518-546 (diffusion: steps x [x <- x - eta L x])
 * and graph.rs:464-501 (multiply_vector: y = L x, CSR row fold from +0.0 in
 * stored order), per row of X [n][f] (f64).  matvec != 0: out = L x. */
int or_diffuse_rows(const double *X, int64_t n, int32_t f, const int64_t *indptr,
                    const int32_t *indices, const double *values, double eta, int32_t steps,
                    int matvec, double *out);

/* surfface-core/src/laplacian.rs:254-298 compute_bhattacharyya_weights with
 * distance.rs:260-290 bhattacharyya_coefficient (f32, host libm logf/expf,
 * as the Rust reference links them): means/vars [c][f] (feature columns are
 * the nodes), per node the k' = min(k, f-1) largest BC > thr over j != i,
 * (BC desc, j asc).  out_idx/out_w [f][k] (-1 / 0 padded). */
int or_bc_knn(const float *means, const float *vars, int64_t c, int32_t f, int32_t k,
              float reg, float thr, int32_t *out_idx, float *out_w);

/* surfface-core/src/distance.rs:78-108 bhattacharyya_distance_diagonal (f32,
 * sequential fold, host libm logf / IEEE sqrtf as the Rust reference links). */
float or_bhattacharyya_distance(const float *mean_i, const float *var_i, const float *mean_j,
                                const float *var_j, int64_t f);

/* surfface-core/src/mst.rs:312-412 build_candidate_graph + compute_distance +
 * compute_edge_cost: nodes = the c rows of means/vars [c][f]; metric 0 =
 * Bhattacharyya, 1 = Euclidean (sqrtf of the f32 fold), 2 = SquaredEuclidean;
 * per node i every j != i, stable sort by distance (j ascending on ties),
 * truncated to k' = min(k, c-1); cost = distance * phi(t_i, t_j) with tw
 * 0 Mean, 1 Min, 2 Max, 3 GeometricMean, 4 None (cost = distance);
 * thickness [c] (host) or NULL = sequential f32 mean of the variance row.
 * out_v / out_dist / out_cost [c][k'].  OR_ENONFINITE on a NaN distance. */
int or_mst_candidates(const float *means, const float *vars, int64_t c, int32_t f, int32_t k,
                      int metric, int tw, const float *thickness, int32_t *out_v,
                      float *out_dist, float *out_cost);

/* surfface-pipeline/src/stages/clustering.rs:42-63 batch nearest centroid,
 * in the fixed order of mn_nearest_centroid_f32 (Burn's is backend-defined:
 * parity-unpinned): sequential f32 |x|^2, |c|^2 and x.c folds,
 * sqrtf((bx + bc) - 2 dot), first index of the minimum, NaN never wins
 * (an all-NaN row: index 0 and its NaN). */
int or_nearest_centroid(const float *batch, int64_t b, const float *cents, int64_t c, int32_t f,
                        int32_t *out_idx, float *out_dist);

/* ---- K5: SF-GRASS ------------------------------------------------------- */

/* src_legacy/sparsification.rs:32-113: avg = sum len / n; avg < 10 => copy;
 * score = w * sqrt((deg_i*deg_j) as f64), sort desc (ties: ascending
 * position in the input row — the reference's sort_unstable leaves ties
 * unspecified), keep min(max(ceil(len*ratio),1),len), kept edges returned in
 * score order. */
int or_sfgrass(int64_t n, const int64_t *indptr, const int32_t *indices,
               const double *w, double ratio, int64_t *out_indptr,
               int32_t *out_indices, double *out_w);

/* ---- §8(f) rank 2: lambda-aware search ---------------------------------- */

/* ArrowSpace::search_lambda_aware (src_legacy/core.rs:1156-1193) for nq
 * queries over the n item rows of X (f64, row-major, the exactly widened
 * f32 data): score = alpha*cos + (1-alpha)*(1 - min(|lq - l_i|, 1))
 * (ArrowItem::lambda_similarity core.rs:162-179, lambda_component_similarity
 * :141-144); cos = dot/(norm(q)*norm(x_i)) if the product > 0 else 0
 * (cosine_similarity :233-244, norm :210-214, dot :196-205: sequential
 * non-contracted f64 folds).  Results sorted by score descending with a
 * stable sort over ascending i (sort_by is stable), truncated to k.
 * out_idx/out_score [nq][k], -1 / NaN padded when k > n.  out_count[q] =
 * min(k, n), or -1 where the reference asserts lambda_q != 0, -3 on a NaN
 * score (partial_cmp().unwrap() panics). */
int or_search_lambda_aware(const double *X, int64_t n, int32_t f, const double *lambdas,
                           const double *Q, const double *lambda_q, int64_t nq, int64_t k,
                           double alpha, int nthreads, int64_t *out_idx, double *out_score,
                           int64_t *out_count);

/* ArrowSpace::search_lambda_aware_hybrid (core.rs:1196-1318), deterministic
 * restatement (tie policy in oracle.c); no lambda != 0 assert (the reference
 * has none here). */
int or_search_lambda_aware_hybrid(const double *X, int64_t n, int32_t f, const double *lambdas,
                                  const double *Q, const double *lambda_q, int64_t nq,
                                  int64_t k, double alpha, int nthreads, int64_t *out_idx,
                                  double *out_score, int64_t *out_count);

/* glibc_check.c: the host glibc logf / expf (what the reference's f32::ln /
 * f32::exp call) and a host copy of the device restatement (csrc/glibc_f32.hpp). */
int or_libm_f32(const float *x, int64_t n, uint32_t bits0, int fn, float *out, int nthreads);
/* the host glibc pow elementwise: out[i] = pow(x[i], y[i]) (the reference's f64::powf) */
int or_pow_f64(const double *x, const double *y, int64_t n, double *out);
int64_t or_libm_mismatch(uint32_t bits0, int64_t n, int fn, const float *got);
int64_t or_glibc_restated_check(int fn, int64_t stride);
int or_glibc_tables(int which, uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif
