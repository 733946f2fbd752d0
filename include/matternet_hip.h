/*
 * matternet_hip.h — C ABI of the MI355X-native (gfx950) surfface hot path.
 *
 * The reference (tuned-org-uk/matternet-rs, crate `surfface`) has no FFI of its
 * own (surfface-py/src/main.rs:1-3 is a hello-world; no extern "C" anywhere).
 * Its de-facto operator API for this path is the set of Rust functions listed
 * in SURVEY.md §8(b); each entry point below names the reference function it
 * replaces (file:line).  INTEGRATION.md shows the `extern "C"` block a Rust
 * `matternet-hip-sys` crate would declare to bind exactly these symbols.
 *
 * Conventions
 *  - Plain C: pointers + sizes, no torch / HIP types in signatures
 *    (`stream` is an opaque hipStream_t, NULL = the legacy default stream).
 *  - Array arguments are DEVICE pointers (HBM) unless a comment says "host".
 *    mn_device_alloc/mn_memcpy_* are provided for callers without a HIP
 *    runtime of their own.
 *  - Every call is synchronous with respect to its stream on return (so the
 *    error code is final) and reentrant across threads; per-thread error text
 *    via mn_last_error().
 *  - Return value: MN_OK (0) or a negative MN_E* code.  The reference panics
 *    (assert!/partial_cmp().unwrap()) where these return errors.
 *  - Indices are int32 (graphs up to 2^31-1 nodes), CSR row pointers int64.
 */
#ifndef MATTERNET_HIP_H
#define MATTERNET_HIP_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MN_OK 0
#define MN_EINVAL (-1)     /* bad argument (reference: assert!/panic)          */
#define MN_ENOMEM (-2)     /* device allocation failed                          */
#define MN_ENONFINITE (-3) /* NaN/inf input (reference: partial_cmp().unwrap()) */
#define MN_ECAP (-4)       /* output capacity too small (nnz_out holds need)   */
#define MN_EHIP (-5)       /* HIP runtime error                                 */
#define MN_ENOTSUP (-6)    /* unsupported parameter combination                 */
#define MN_ECOMM (-7)      /* a collective failed or missed its deadline; the
                              RCCL communicator was aborted (mn_rccl_set_timeout) */

/* ---------------------------------------------------------------------- */
/* Library / memory plumbing                                              */
/* ---------------------------------------------------------------------- */
int mn_version(void);                 /* 100*major + minor                  */
const char *mn_last_error(void);      /* thread-local, valid until next call */
int mn_device_alloc(size_t bytes, void **out);
int mn_device_free(void *p);
int mn_memcpy_h2d(void *dst_dev, const void *src_host, size_t bytes, void *stream);
int mn_memcpy_d2h(void *dst_host, const void *src_dev, size_t bytes, void *stream);
int mn_memcpy_d2d(void *dst_dev, const void *src_dev, size_t bytes, void *stream);
int mn_stream_synchronize(void *stream);

/* Synthetic input generator, identical to tests/datagen.py:
 * X[r][c] = 2*((splitmix64(seed ^ ((row0+r)*d + c)) >> 40) * 2^-24) - 1. */
int mn_fill_uniform_f32(float *X, int64_t n, int32_t d, uint64_t seed,
                        int64_t row0, void *stream);

/* The library's f32 ln / exp on device arrays (fn 0 = logf, 1 = expf): the
 * platform glibc's logf / expf restated on the device, which the reference's
 * f32::ln / f32::exp call (distance.rs:102, 283-289) — used by the
 * Bhattacharyya kernels; exported so callers and tests can check them.  x ==
 * NULL evaluates the consecutive f32 bit patterns bits0 + i (i < n). */
int mn_libm_f32(const float *x, int64_t n, uint32_t bits0, int32_t fn, float *out, void *stream);
/* The library's f64 pow on device arrays, out[i] = pow(x[i], y[i]): glibc's
 * pow restated (the reference's f64::powf: the rational kernel's
 * (d / sigma)^p, src_legacy/laplacian.rs:256; sorted_index.rs:65). */
int mn_libm_pow_f64(const double *x, const double *y, int64_t n, double *out, void *stream);

/* ---------------------------------------------------------------------- */
/* K1 — brute-force kNN (Gram on MFMA + LDS top-k + exact re-rank)        */
/* ---------------------------------------------------------------------- */
enum mn_metric {
    MN_L2SQ = 0,     /* surfface-core/src/distance.rs:206-213 (f32 fold)     */
    MN_COS_RECT = 1, /* src_legacy/tests/test_helpers.rs:77-126 (f64)        */
    MN_L2 = 2        /* distance.rs:195-203: sqrt of the L2SQ fold (f32)     */
};

typedef struct mn_knn_opts {
    int32_t k;            /* neighbours per row; rows get min(k, n-1) (mst.rs:317) */
    int32_t metric;       /* enum mn_metric                                        */
    int32_t exclude_self; /* 1 = the reference behaviour (mst.rs:336 j != i)       */
    int32_t margin;       /* candidate margin m (list length L = k + m); 0 => 16   */
    int32_t timing;       /* 1 = record per-kernel HIP-event times in mn_knn_stats */
    int32_t algo;         /* enum mn_knn_algo: candidate generator (results are
                             identical; only speed differs)                       */
    void *stream;         /* hipStream_t or NULL                                   */
} mn_knn_opts;

enum mn_knn_algo {
    MN_KNN_AUTO = 0,   /* BF16X1 for large corpora (>= 2^17 rows), else BF16X3 when
                          k + margin <= 64, else F32                                */
    MN_KNN_F32 = 1,    /* v_mfma_f32_16x16x4_f32 Gram (exact f32 products)          */
    MN_KNN_BF16X3 = 2, /* f32 rows split into bf16 hi + lo; hi.hi + hi.lo + lo.hi on
                          v_mfma_f32_32x32x16_bf16 (16x the rate per instruction)   */
    MN_KNN_BF16X1 = 3  /* two-phase single-bf16 filter: a corpus sample sets each
                          query's threshold, then one fixed-threshold bf16 Gram sweep
                          (one MFMA per 16 features); certified by a residual-norm
                          bound, uncertified rows rescanned exactly                  */
};

typedef struct mn_knn_stats {
    int64_t n_queries;
    int64_t n_uncertified;  /* rows no certificate settled (resolved by a batched
                               split-generator pass or the exact scan)        */
    int32_t slices;         /* corpus split factor used                         */
    int32_t list_len;       /* L = k + margin                                   */
    float ms_norms, ms_gram, ms_rerank, ms_fallback, ms_total; /* timing == 1   */
    int32_t algo;           /* candidate generator used (enum mn_knn_algo)      */
    /* MN_KNN_BF16X1 only (else 0): ms_gram = ms_sample + ms_sweep             */
    float ms_sample;        /* phase 1: sample Gram (thresholds)                */
    float ms_sweep;         /* phase 2: fixed-threshold sweep (the hot kernel)  */
    int64_t sample_rows;    /* corpus rows in the phase-1 sample                */
    int64_t n_candidates;   /* buffered (query, row) pairs re-ranked            */
    int32_t sweep_slices;
    int32_t sweep_cap;      /* buffer entries per (query, slice)                */
    int64_t n_escalated;    /* rows the bf16x1 bound could not certify, refilled
                               by the bf16x3 sweep at their own threshold      */
    float ms_escalate;
    int32_t n_root_rescan;  /* MN_L2: rows rescanned for the root order (k_l2_order) */
} mn_knn_stats;

/* Self kNN over the rows of X [n][d] f32 (device, row-major): replaces
 * MSTStage::build_candidate_graph's kNN (surfface-core/src/mst.rs:312-363,
 * DistanceMetric::SquaredEuclidean, or Euclidean with metric MN_L2: the
 * correctly rounded f32 sqrt of the same fold, distance.rs:195-203).  The f64
 * topk_by_l2 (energymaps.rs:875-892) is mn_knn_l2_f64 below; the cosine
 * graphs are mn_knn_cos_columns_f32 / mn_knn_cos_bf16.  Output row i:
 * out_idx[i*k + r], out_dist[i*k + r] in (dist asc, idx asc) order —
 * bit-identical to the reference's sequential f32 fold and stable sort.
 * Slots beyond min(k, n-1): idx -1, dist +inf.  metric MN_L2SQ or MN_L2.
 * 1 <= k <= 512: k <= 64 through the candidate generators (opts->algo); k > 64
 * (the reference takes any k) through the exact split scan of every row
 * (each 1024-row corpus part's best k, merged; d <= ~2300). */
int mn_knn_f32(const float *X, int64_t n, int32_t d, const mn_knn_opts *opts,
               int32_t *out_idx, float *out_dist);

/* Queries Q [nq][d] against a corpus C [nc][d] (both device).  Global ids:
 * query i is q_offset+i, corpus row j is c_offset+j; out_idx holds global
 * corpus ids; exclude_self drops pairs with equal global id.  This is the
 * per-shard primitive of the row-sharded multi-GPU build:
 * the result is the EXACT per-shard top-k, so merging shards with
 * mn_knn_merge is exact. */
int mn_knn_f32_qc(const float *Q, int64_t nq, const float *C, int64_t nc,
                  int32_t d, int64_t q_offset, int64_t c_offset,
                  const mn_knn_opts *opts, int32_t *out_idx, float *out_dist);

/* Merge `parts` exact per-shard lists per query (each [nq][k], device,
 * parts-major: part p row i at (p*nq + i)*k) into the global top-k by
 * (dist asc, idx asc).  idx < 0 entries are empty. */
int mn_knn_merge_f32(const int32_t *part_idx, const float *part_dist,
                     int32_t parts, int64_t nq, int32_t k, int32_t *out_idx,
                     float *out_dist, void *stream);

/* f64 Euclidean kNN with the reference's exact f64 folds, for its three f64
 * call sites: topk_by_l2 (src_legacy/energymaps.rs:875-892: d = sum
 * (a-b)*(a-b), stable sort, use_sqrt = 0), prepare_query_item's energy-mode
 * nearest sub-centroid (src_legacy/core.rs:872-909: sqrt'd distance, 1-NN
 * with strict '<' = k 1, use_sqrt 1) and estimate_intrinsic_dimension's
 * Two-NN distances (src_legacy/clustering.rs:132-195: k 2, use_sqrt 1).
 * Q [nq][d], C [nc][d] (device; f64, or f32 widened exactly when
 * x_is_f64 == 0); q_ids [nq] (device, may be NULL): the corpus index each
 * query excludes (the reference's j != i).  out_idx [nq][k] int32 (-1 pad),
 * out_dist [nq][k] f64 (+inf pad), in (dist, idx) order = the reference's
 * stable sort truncated to k.  Bit-exact.  k <= 64, nq <= 2097120 per call.
 * MN_ENONFINITE on a NaN distance (the reference's partial_cmp().unwrap()). */
int mn_knn_l2_f64(const void *Q, int64_t nq, const void *C, int64_t nc, int32_t d,
                  int32_t x_is_f64, const int64_t *q_ids, int32_t k, int32_t use_sqrt,
                  int32_t *out_idx, double *out_dist, void *stream);

/* Row-sharded multi-GPU build (SURVEY.md §8(b) mn_knn_sharded_f32, §8(e)) on
 * a caller-owned RCCL communicator (an ncclComm_t, passed as void*; one rank
 * per GPU, rank r holding rows [r n_local, (r+1) n_local) of X).  The shards
 * are all-gathered.  Symmetric form (self kNN, MN_L2SQ, algo AUTO / BF16X1,
 * world > 1): each rank computes its rows' sweep thresholds against a global
 * sample, the thresholds are all-gathered, every rank sweeps its share of the
 * node-wide symmetric tile table (each unordered tile pair once) and
 * re-ranks all rows' admitted candidates, the partial lists go to the rows'
 * owners (grouped ncclSend/ncclRecv), which merge and certify them.  Per-shard
 * form (otherwise): exact per-shard top-k of all N queries against the
 * resident shard (mn_knn_f32_qc, chunks of query_chunk rows; <= 0: 2^21),
 * the exchange, mn_knn_merge_f32.  out_idx / out_dist [n_local][k]: the
 * rank's rows of the global graph, global ids, bit-identical to a single-GPU
 * mn_knn_f32 of X.  opts as mn_knn_f32 (opts->stream is used for every
 * operation; timing 1: mn_knn_last_stats has ms_norms = the all-gathers,
 * ms_sample = stage A, ms_sweep = stage B (the per-shard form: its query
 * passes), ms_rerank = the exchange, ms_fallback = stage C (the merge),
 * ms_total = the call).  Collective: every rank calls it with the same
 * n_local, d and opts.  <= 16 ranks.  Failure detection: a status agreement
 * precedes every collective phase (a rank whose stage failed returns its own
 * code, the others MN_EHIP "another rank failed"), and every collective is
 * waited for by polling the stream and ncclCommGetAsyncError against the
 * mn_rccl_set_timeout deadline: an RCCL error or a peer that never arrives
 * ends the call with MN_ECOMM at that deadline: the communicator is aborted
 * (destroying it afterwards is a no-op; later calls on it return MN_EINVAL)
 * and the call's buffers are freed off the calling thread once the stream
 * has drained (mn_shard_quiesce). */
int mn_knn_sharded_f32(const float *X_shard, int64_t n_local, int32_t d, void *rccl_comm,
                       const mn_knn_opts *opts, int64_t query_chunk, int32_t *out_idx,
                       float *out_dist);
/* The same sharded build with `world` ranks on ONE device (tests and
 * single-GPU measurement of one rank's share): the driver of
 * mn_knn_sharded_f32 over a loopback transport — rank r on its own stream,
 * its stages run in turn, device copies for the all-gathers and the
 * exchange (the same buffer layout and offsets as over RCCL).  X_all
 * [n_tot][d] (device) holds the shards (rank r's at r n_tot / world; n_tot a
 * multiple of world <= 16).  Either form, chosen as mn_knn_sharded_f32
 * chooses it for world ranks.  out_idx / out_dist [n_tot][k]: the global
 * graph, bit-identical to mn_knn_f32.  rank_ms (host, may be NULL)
 * [world][3]: per rank the stage A (phase-1 thresholds), stage B (sweep share
 * + partial re-rank; per-shard form: the query passes) and stage C (merge +
 * certify + exact scan) milliseconds. */
int mn_knn_sharded_sim_f32(const float *X_all, int64_t n_tot, int32_t d, int32_t world,
                           const mn_knn_opts *opts, int32_t *out_idx, float *out_dist,
                           float *rank_ms);
/* The same sharded build with `world` ranks on ONE device, ONE HOST THREAD
 * PER RANK (replaces nothing in the reference: SURVEY.md §8(e) — the
 * reference has no distribution; this is the concurrency rehearsal of
 * mn_knn_sharded_f32): each thread drives its rank exactly as one RCCL process
 * does (nlocal 1, its own stream and scratch), the ranks' stages and
 * collectives run concurrently, and every collective is a rendezvous that
 * checks that all ranks issued the same collective (kind, sequence number,
 * name, byte size).  A divergent collective order, or a rank that left the
 * driver while others wait in a collective, ends every rank with MN_ECOMM
 * (message: which ranks, which collectives) where RCCL would hang; a rank
 * that never arrives, at the mn_rccl_set_timeout deadline.  Arguments,
 * outputs and rank_ms as mn_knn_sharded_sim_f32 (mn_knn_last_stats: maxima
 * of the ranks' times, sums of their counts). */
int mn_knn_sharded_threads_f32(const float *X_all, int64_t n_tot, int32_t d, int32_t world,
                               const mn_knn_opts *opts, int32_t *out_idx, float *out_dist,
                               float *rank_ms);
/* After a sharded call ended with MN_ECOMM its communicator is aborted and its
 * buffers are released by a background thread once the device work queued on
 * them has drained (the call itself returns at its deadline).  Waits up to
 * timeout_s for those releases; MN_ECOMM if some are still pending. */
int mn_shard_quiesce(double timeout_s);
/* Host only (no device work): rank `rank`'s share of the symmetric form's
 * node-wide tile table over nbk 256-row blocks — entries (I, Jfirst, tiles,
 * stride) = row block I against column blocks Jfirst + t stride, t < tiles
 * (J >= I; empty padding entries have tiles 0).  Over all ranks every tile
 * (I, J >= I) appears exactly once.  out4 [cap][4] (may be NULL: count only);
 * *n_out = entries; MN_ECAP when cap is too small. */
int mn_sym_share_table(int32_t nbk, int32_t rank, int32_t world, int32_t *out4, int64_t cap,
                       int64_t *n_out);
/* RCCL communicator helpers for callers without an RCCL binding of their own:
 * rank 0 creates the 128-byte id and distributes it; each rank then inits. */
int mn_rccl_unique_id(void *out_128_bytes);
int mn_rccl_comm_init(const void *unique_id_128_bytes, int32_t world, int32_t rank,
                      void **comm_out);
int mn_rccl_comm_destroy(void *comm);
/* Process-wide deadline (seconds, default 600) for one collective of
 * mn_knn_sharded_f32, including the wait for the slowest peer's stage. */
int mn_rccl_set_timeout(double seconds);

/* Statistics of the calling thread's last mn_knn_* call. */
int mn_knn_last_stats(mn_knn_stats *out);


/* Stage C feature kNN by Bhattacharyya coefficient: replaces
 * LaplacianStage::compute_bhattacharyya_weights (surfface-core/src/
 * laplacian.rs:254-298) with bhattacharyya_coefficient (distance.rs:260-290).
 * Nodes = the f feature columns of means / vars [c][f] (f32, device; the
 * CentroidState [C, F] tensors).  Per node the k' = min(k, f-1) largest
 * BC > weight_thr over j != i, ordered (BC desc, j asc; the reference's
 * sort_unstable leaves ties unspecified): out_idx [f][k] (int32, -1 pad),
 * out_w [f][k] (f32, 0 pad) — the directed edges the Stage C Laplacian
 * (mn_laplacian_from_knn, MN_SYM_MAX) symmetrises.  f32 arithmetic and fold
 * order as the reference; ln / exp are glibc's logf / expf restated
 * (mn_libm_f32): bit-exact.  2 <= f <= 4096, k >= 1.  MN_ENONFINITE on NaN
 * coefficients (the reference panics). */
int mn_bc_knn_f32(const float *means, const float *vars, int64_t c, int32_t f, int32_t k,
                  float var_reg, float weight_thr, int32_t *out_idx, float *out_w, void *stream);

/* Clustering stage, batch nearest centroid (surfface-pipeline/src/stages/
 * clustering.rs:42-63): per item of batch [b][f] the nearest of the c
 * centroids [c][f] (device, f32) by sqrt((|x|^2 + |c|^2) - 2 x.c), out_idx /
 * out_dist [b] (first index of the minimum; NaN distances never win).  The
 * reference's Burn reductions have a backend-defined order (parity-unpinned):
 * here sequential f32 folds over the features, correctly rounded sqrt —
 * bit-exact against the oracle's restatement of that order.  The incremental
 * centroid creation (:65-88) stays on the host, as in the reference. */
int mn_nearest_centroid_f32(const float *batch, int64_t b, const float *centroids, int64_t c,
                            int32_t f, int32_t *out_idx, float *out_dist, void *stream);

enum mn_mst_metric {
    MN_MST_BHATTACHARYYA = 0,
    MN_MST_EUCLIDEAN = 1,
    MN_MST_SQEUCLIDEAN = 2
};
enum mn_thickness_weight { /* mst.rs:58-74 ThicknessWeight */
    MN_TW_MEAN = 0,    /* (t_i + t_j) / 2 */
    MN_TW_MIN = 1,
    MN_TW_MAX = 2,
    MN_TW_GEOMEAN = 3, /* sqrt(t_i * t_j) */
    MN_TW_NONE = 4
};
/* MST stage candidate graph (surfface-core/src/mst.rs:312-363
 * MSTStage::build_candidate_graph + compute_distance :366-397 +
 * compute_edge_cost :400-412).  Nodes are the C centroid ROWS of means /
 * vars [C][F] (device, f32).  Per node i, the k = min(k_neighbors, C-1)
 * nearest j != i by (distance asc, j asc) — the reference's stable sort —
 * as edges out_v / out_dist / out_cost [C][k] (u = i implicit), cost =
 * distance * phi(t_i, t_j) (MN_TW_NONE: cost = distance).  thickness [C]
 * (device) or NULL = the mean variance per row (centroid.rs:107-109;
 * sequential f32 sum / F — Burn's summation order is backend-defined, so
 * that default is parity-unpinned); out_thickness [C] optional.
 * MN_MST_BHATTACHARYYA (the default metric, mst.rs:77-84) folds
 * bhattacharyya_distance_diagonal (distance.rs:78-108) in feature order with
 * the reference's f32 operations (sqrt correctly rounded; ln = glibc's logf
 * restated, mn_libm_f32): bit-exact; C <= 65536, k <= 512.  MN_MST_EUCLIDEAN /
 * MN_MST_SQEUCLIDEAN run mn_knn_f32 (bit-exact).  MN_ENONFINITE on a NaN
 * distance (the reference's partial_cmp().unwrap()). */
int mn_mst_candidate_graph_f32(const float *means, const float *vars, int64_t c, int32_t f,
                               int32_t k_neighbors, int32_t metric, int32_t thickness_weight,
                               const float *thickness, float *out_thickness, int32_t *out_v,
                               float *out_dist, float *out_cost, void *stream);


/* ---------------------------------------------------------------------- */
/* K2 — Laplacian assembly from kNN rows (CSR)                            */
/* ---------------------------------------------------------------------- */
enum mn_value_type { MN_F32 = 0, MN_F64 = 1 };
enum mn_weight_kernel {
    MN_W_GIVEN = 0,    /* nbr_val already holds edge weights                    */
    MN_W_RATIONAL = 1  /* w = 1/(1+(dist/sigma)^p), dist <= eps, w > 1e-12
                          (src_legacy/laplacian.rs:245-260)                      */
};
enum mn_symmetrise {
    MN_SYM_UNION = 0,  /* legacy: union of directed edges, L = D - W, f64 values
                          (src_legacy/laplacian.rs:297-419)                      */
    MN_SYM_MAX = 1     /* Stage C: undirected max weight, optional L_sym, f32
                          (surfface-core/src/laplacian.rs:312-394, 209-219)      */
};

typedef struct mn_lap_opts {
    int32_t weight_kernel;   /* enum mn_weight_kernel                            */
    int32_t symmetrise;      /* enum mn_symmetrise                               */
    int32_t normalize;       /* MAX only: 1 = I - D^-1/2 W D^-1/2, 0 = D - W     */
    int32_t reserved0;
    double eps;              /* MN_W_RATIONAL: keep dist <= eps                  */
    double sigma;            /* MN_W_RATIONAL: kernel scale (> 0)                */
    double p;                /* MN_W_RATIONAL: kernel exponent                   */
    double weight_threshold; /* MAX: drop w <= thr (LaplacianConfig 1e-9)        */
    void *stream;
} mn_lap_opts;

/* CSR matrix.  As an output: library-allocated device buffers (release with
 * mn_csr_free), or, when caller_owned == 1 on entry, the caller's device
 * buffers indptr [n_rows + 1], indices / values [nnz = capacity] of the
 * mode's value_type; a capacity that is too small returns MN_ECAP with nnz =
 * the entries needed.  n(2k + 1) entries always suffice for kNN rows. */
typedef struct mn_csr {
    int64_t n_rows, n_cols, nnz;
    int64_t *indptr;   /* [n_rows + 1] */
    int32_t *indices;  /* [nnz], ascending within a row */
    void *values;      /* [nnz] of value_type */
    int32_t value_type;
    int32_t caller_owned;
} mn_csr;

typedef struct mn_lap_stats {
    int64_t nnz;
    int64_t big_rows;  /* rows sorted by the wider kernels (> 256 entries)     */
    int64_t hub_rows;  /* rows resolved by the dense column map (> 8192)       */
    float ms_total;
    float reserved0;
} mn_lap_stats;

/* Directed kNN rows (nbr_idx [n][k], -1 = empty; nbr_val [n][k] distances for
 * MN_W_RATIONAL or weights for MN_W_GIVEN, f64 if val_is_f64 else f32) ->
 * symmetric Laplacian CSR.  Replaces _symmetrise_adjancency +
 * _build_sparse_laplacian (src_legacy/laplacian.rs:297-419; UNION: values
 * and structure bit-identical) and LaplacianStage::build_laplacian_flat + the
 * dense->CSR pass (surfface-core/src/laplacian.rs:312-394, 209-219; MAX:
 * structure identical, values within f32 tolerance because the reference
 * sums degrees in DashMap order).  degrees_out (device, may be NULL): [n]
 * f64 (UNION) or f32 (MAX). */
int mn_laplacian_from_knn(const int32_t *nbr_idx, const void *nbr_val, int32_t val_is_f64,
                          int64_t n, int32_t k, const mn_lap_opts *opts, mn_csr *out,
                          void *degrees_out);
int mn_csr_free(mn_csr *m);
int mn_lap_last_stats(mn_lap_stats *out);


/* ---------------------------------------------------------------------- */
/* K3 — energy row reductions (Rayleigh E, dispersion G, taumode lambda)  */
/* ---------------------------------------------------------------------- */
enum mn_g_mode {
    MN_G_TAUMODE = 0,    /* ordered pairs, lambda = tau*E/(E+tau)+(1-tau)G
                            (src_legacy/taumode.rs:261-408)                      */
    MN_G_ENERGYMAPS = 1, /* j > i pairs, lambda = E (energymaps.rs:923-1045)     */
    MN_G_SPECTRAL = 2    /* Stage D device lambdas (surfface-core/src/spectral/
                            mod.rs:69-181): E = clamp(num/(den+1e-9), +-1e6),
                            G = D = clamp(row/(sum_rows row + 1e-12), 0, 1) with
                            row = sum_f max(0, sum_j w_fj (x_f - x_j)^2),
                            lambda = E + D; f32 or f64 Laplacian values        */
};
enum mn_tau_mode { MN_TAU_FIXED = 0, MN_TAU_MEDIAN = 1, MN_TAU_MEAN = 2, MN_TAU_PERCENTILE = 3 };

typedef struct mn_energy_opts {
    int32_t g_mode;     /* enum mn_g_mode                                        */
    int32_t tau_mode;   /* enum mn_tau_mode (TauMode, taumode.rs:17-23; default Median) */
    double tau_param;   /* Fixed(t) / Percentile(p) parameter                    */
    int32_t timing;
    int32_t reserved0;
    void *stream;
} mn_energy_opts;

typedef struct mn_energy_stats {
    int64_t entries;    /* Laplacian entries streamed per row                   */
    int32_t symmetric;  /* 1: upper-triangle list with multiplicity 2           */
    int32_t reserved0;
    float ms_rows, ms_total;
} mn_energy_stats;

/* Items X [n][f] (f32, device) against the f x f feature Laplacian L (CSR,
 * f64 values, device; e.g. from mn_laplacian_from_knn UNION): writes E, G,
 * lambda [n] (f64, device, any may be NULL).  Replaces
 * TauMode::compute_taumode_lambdas_parallel's per-item work
 * (src_legacy/taumode.rs:117-250, 261-408) and node_energy_and_dispersion
 * (src_legacy/energymaps.rs:923-1045).  Tolerance 1e-9 relative (the
 * reference sums in rayon order).  MN_G_SPECTRAL replaces compute_lambdas_gpu
 * / compute_tau_mode_gpu (surfface-core/src/spectral/mod.rs:158-181,
 * bridge.rs:27-69) and also takes the Stage C f32 Laplacian (MN_SYM_MAX
 * output); the reference computes in f32 (Burn matmuls), this in f64:
 * tolerance 1e-4 relative.  f <= 4096. */
int mn_energy_rows(const mn_csr *L, const float *X, int64_t n, int32_t f,
                   const mn_energy_opts *opts, double *E, double *G, double *lambda);

/* In place: src_legacy/core.rs:1341-1354 normalise_lambdas (min fold +inf,
 * max fold 0.0, range floor 1e-9).  out_min_max_range_host (host, 3 doubles,
 * may be NULL). */
int mn_normalise_lambdas(double *lambda, int64_t n, double *out_min_max_range_host,
                         void *stream);
int mn_energy_last_stats(mn_energy_stats *out);

/* Item-graph orientation: node_energy_and_dispersion
 * applied to the F feature SIGNALS (columns of X [n][f], length n, f32,
 * device) against the n x n item Laplacian L (f64 CSR, e.g. the C3 item
 * graph from mn_laplacian_from_knn UNION) (src_legacy/energymaps.rs:923-1045
 * with x = X^T): E[f] = max(0, s^T L s / s^T s) (den > 1e-12), G[f] =
 * clamp(sum (e/S)^2, 0, 1) over ordered pairs (MN_G_TAUMODE) or j > i
 * (MN_G_ENERGYMAPS).  E, G [f] f64 device (may be NULL).  Tolerance 1e-9
 * relative (the reference sums in rayon order).  f <= 4096. */
int mn_energy_signals(const mn_csr *L, const float *X, int64_t n, int32_t f, int32_t g_mode,
                      double *E, double *G, void *stream);

/* EnergyMaps diffusion pre-pass (src_legacy/energymaps.rs:518-546): `steps`
 * times every row x (length f) becomes x - eta * (L x), where (L x)_i is the
 * CSR row fold sum += L[i,p] * x[col[p]] from +0.0 in stored order
 * (GraphLaplacian::multiply_vector, src_legacy/graph.rs:464-501).  X [n][f]
 * f32 or f64 (x_is_f64, device), X_out [n][f] f64 (device; may alias X when
 * it is f64), L the f x f f64 CSR.  Bit-exact (f64, no contraction). */
int mn_diffuse_rows(const mn_csr *L, const void *X, int32_t x_is_f64, int64_t n, int32_t f,
                    double eta, int32_t steps, double *X_out, void *stream);
/* Y = L x per row (GraphLaplacian::multiply_vector), same conventions. */
int mn_laplacian_matvec_rows(const mn_csr *L, const void *X, int32_t x_is_f64, int64_t n,
                             int32_t f, double *Y, void *stream);


/* ---------------------------------------------------------------------- */
/* K4 — lambda-sorted index                                               */
/* ---------------------------------------------------------------------- */
/* SortedLambdas::build_from + to_vec (src_legacy/sorted_index.rs:22-54):
 * order_out[r] (device, int64) = item index at rank r, ascending
 * OrderedFloat(lambda) (NaN greatest, -0.0 == +0.0) with ties ordered by the
 * DECIMAL STRING of the index ("10" < "2"); key_out[r] (device, may be NULL)
 * = the bucket key (lambda of the smallest index in the equal class);
 * std_out_host (host, may be NULL) = std_deviation (laplacian.rs:421-448),
 * bit-exact (sequential fold on one device thread).  Order bit-exact given
 * identical lambdas. */
int mn_sorted_index(const double *lambda, int64_t n, int64_t *order_out, double *key_out,
                    double *std_out_host, void *stream);


/* Lambda-aware lookups on a built index (keys / order = mn_sorted_index
 * outputs, device, n items), batched over nq query lambdas (device).  Per
 * query t: out_idx [t][k] item indices (int64, -1 padded), out_lambda [t][k]
 * their bucket keys (f64), out_count [t] = entries written, or -1 where the
 * reference panics (BTreeMap::range with start > end; partial_cmp().unwrap()
 * on NaN distances).  Bit-exact. */

/* SortedLambdas::range_bylambda (src_legacy/sorted_index.rs:64-80): band =
 * std_dev / 2^p; the items whose key lies in [lq - band, lq + band]
 * (OrderedFloat order) in index order, the first k. */
int mn_sorted_range_bylambda(const double *keys, const int64_t *order, int64_t n,
                             double std_dev, const double *lambda_q, int64_t nq, int32_t k,
                             double p, int64_t *out_idx, double *out_lambda, int32_t *out_count,
                             void *stream);

/* SortedLambdas::k_nearest_by_lambda (src_legacy/sorted_index.rs:85-140):
 * window [max(lq - delta, 0), min(lq + delta, 1)] from delta = |base_delta|
 * (has_base_delta) or max(std_dev * lambda_p, 1e-9), grown by `growth` (> 1
 * and finite, else 1.7) up to min(delta * max(max_multiplier, 1), 1) until it
 * holds k items; then the k smallest |lambda - lq|.  The reference sorts
 * unstably (tie order unspecified): ties here keep index order. */
int mn_sorted_k_nearest_by_lambda(const double *keys, const int64_t *order, int64_t n,
                                  double std_dev, const double *lambda_q, int64_t nq, int32_t k,
                                  double lambda_p, int32_t has_base_delta, double base_delta,
                                  double growth, double max_multiplier, int64_t *out_idx,
                                  double *out_lambda, int32_t *out_count, void *stream);

/* ArrowSpace::search_lambda_aware (src_legacy/core.rs:1156-1193), batched over
 * nq queries: Q [nq][f] f64 query rows, lambda_q [nq] their (prepared) lambdas,
 * over the n item rows of X [n][f] (f32, the exactly widened values the
 * reference's f64 ArrowSpace.data holds, or f64 when x_is_f64) with item
 * lambdas [n] (f64); all device pointers.  score = alpha*cos(q, x_i) +
 * (1 - alpha)*(1 - min(|lq - l_i|, 1)) (ArrowItem::lambda_similarity,
 * core.rs:141-179; cos = dot/(norm*norm), 0 when that product is not > 0,
 * :196-244: sequential non-contracted f64 folds).  out_idx / out_score
 * [nq][k] (device): the reference's stable sort by score descending (ties by
 * ascending i) truncated to k, padded with (-1, NaN) when k > n.  Bit-exact.
 * MN_EINVAL when some lambda_q == 0.0 (the reference's assert_ne!, :1169),
 * MN_ENONFINITE on a NaN score (its partial_cmp().unwrap() panics),
 * MN_ENOTSUP for k > 256. */
int mn_search_lambda_aware(const void *X, int32_t x_is_f64, int64_t n, int32_t f,
                           const double *lambdas, const double *Q, const double *lambda_q,
                           int64_t nq, int32_t k, double alpha, int64_t *out_idx,
                           double *out_score, void *stream);

/* ArrowSpace::search_lambda_aware_hybrid (src_legacy/core.rs:1196-1318), same
 * arguments: the union of the lambda-score top k, every item with cosine >
 * 0.9999 (scored by its cosine) and the best-cosine item (first insertion
 * wins: high-semantic, lambda top k, best cosine), sorted by score descending,
 * first k (-1 / NaN padded).  The reference's parallel heap, reduce and
 * sort_unstable leave tie order unspecified: here every tie goes to the
 * smaller index.  No lambda != 0 check (the reference has none here).
 * MN_ENOTSUP for k > 255. */
int mn_search_lambda_aware_hybrid(const void *X, int32_t x_is_f64, int64_t n, int32_t f,
                                  const double *lambdas, const double *Q,
                                  const double *lambda_q, int64_t nq, int32_t k, double alpha,
                                  int64_t *out_idx, double *out_score, void *stream);


/* ---------------------------------------------------------------------- */
/* K5 — sparsification of directed neighbour rows                         */
/* ---------------------------------------------------------------------- */
enum mn_sparsify_mode {
    MN_SPARSIFY_SFGRASS = 0, /* SfGrassSparsifier::sparsify_graph
                                (src_legacy/sparsification.rs:32-113)            */
    MN_SPARSIFY_INLINE = 1   /* _build_adjacency inline pruning
                                (src_legacy/laplacian.rs:216-282)                */
};
/* Rows nbr_idx/nbr_w [n][k] (device; idx -1 = empty, k <= 64) -> out rows
 * [n][k]: kept entries first in descending score w*sqrt(deg_i*deg_j) (ties by
 * input position), the rest -1 / 0.0.  When the average degree does not
 * enable pruning the rows are copied (compacted, slot order).  ratio: SF-GRASS
 * target ratio (SfGrassSparsifier::new() = 0.5; with_target_ratio clamps to
 * [0.1, 1]).  degrees [n] (device, may be NULL): deg_i for the scores and the
 * average-degree switch; NULL = the row lengths (SF-GRASS).  The inline
 * pruning passes the eps-valid neighbour counts, taken BEFORE the weight
 * filter (laplacian.rs:219-229).  applied_host (host, may be NULL) = 1 if
 * pruning ran.  Bit-exact. */
int mn_sparsify_rows(const int32_t *nbr_idx, const double *nbr_w, int64_t n, int32_t k,
                     double ratio, int32_t mode, const int32_t *degrees, int32_t *out_idx,
                     double *out_w, int32_t *applied_host, void *stream);

/* SfGrassSparsifier::sparsify_graph (src_legacy/sparsification.rs:32-101) on
 * CSR rows of ANY length (the reference's &[Vec<(usize, f64)>]; e.g. a
 * symmetrised adjacency with hub rows): `in` (device CSR, f64 values, indptr
 * from 0) -> `out` (library-allocated, release with mn_csr_free, or the
 * caller's buffers when out->caller_owned == 1; too small: MN_ECAP with
 * out->nnz = the need).  n_nodes: the reference's n_nodes argument (the
 * average-degree divisor; <= 0: in->n_rows).  avg = nnz / n_nodes < 10: the
 * rows unchanged; else per row keep min(max(ceil(len ratio), 1), len) entries
 * by descending w * sqrt((deg_i deg_j) as f64), deg = row lengths, in score
 * order (ties by input position = ascending j for a column-sorted CSR; the
 * reference's sort_unstable leaves them unspecified).  applied_host (host,
 * may be NULL) = 1 if pruning ran.  Bit-exact. */
int mn_sparsify_sfgrass(const mn_csr *in, int64_t n_nodes, double ratio, mn_csr *out,
                        int32_t *applied_host, void *stream);


/* ---------------------------------------------------------------------- */
/* K1 (cosine) — rectified-cosine kNN                                     */
/* ---------------------------------------------------------------------- */
typedef struct mn_cos_opts {
    int32_t topk;       /* neighbours kept per node (GraphParams.topk)            */
    int32_t margin;     /* candidate margin (0 => 16)                              */
    double eps;         /* keep dist <= eps                                        */
    double sigma;       /* weight 1/(1+(dist/sigma)^p)                              */
    double p;
    int32_t timing;
    int32_t reserved0;
    void *stream;
} mn_cos_opts;

/* Feature graph: nodes are the f COLUMNS of X [n_rows][f] (f32, device), each
 * with an n_rows-long profile — GraphFactory::build_laplacian_matrix_from_k_cluster
 * builds its Laplacian on the transposed data (src_legacy/graph.rs:214-228).
 * Distances/weights/order are the brute-force spec of the legacy adjacency
 * (src_legacy/tests/test_helpers.rs:77-126): f64 sequential norms and dots,
 * rectified cosine distance, eps/weight filter, (dist, j) order, topk.
 * Outputs [f][topk] (device): idx (-1 empty), dist (f64), w (f64, may be
 * NULL).  Bit-exact.  2 <= f <= 4096, topk <= 64. */
int mn_knn_cos_columns_f32(const float *X, int64_t n_rows, int32_t f, const mn_cos_opts *opts,
                           int32_t *out_idx, double *out_dist, double *out_w);
/* Same over an f64 X [n_rows][f] (the legacy DenseMatrix<f64> path:
 * build_laplacian_matrix on arbitrary f64 items, src_legacy/laplacian.rs:
 * 122-201, and the "Laplacian of Laplacian" signals graph built on the
 * densified F x F Laplacian, graph.rs:257-313).  Products are the reference's
 * rounded f64 products, folded in the same order: bit-exact. */
int mn_knn_cos_columns_f64(const double *X, int64_t n_rows, int32_t f, const mn_cos_opts *opts,
                           int32_t *out_idx, double *out_dist, double *out_w);
/* GraphParams.normalise pre-pass of build_laplacian_matrix
 * (src_legacy/laplacian.rs:143-150: smartcore StandardScaler over the columns
 * of the items matrix).  smartcore is not in the reference tree, so this is
 * parity-unpinned: mean and population std by sequential f64 folds, out =
 * (x - mean) / std, std == 0 -> x - mean.  X, out [n_rows][n_cols] f64. */
int mn_standardize_columns_f64(const double *X, int64_t n_rows, int32_t n_cols, double *out,
                               void *stream);
int mn_cos_last_stats(mn_knn_stats *out);

/* C5 item graph (config 5): rectified-cosine kNN over the ROWS of a bf16
 * matrix X [n][d] (raw bf16 bits, device).  Semantics are those of the legacy
 * adjacency builder (src_legacy/laplacian.rs:245-290 _build_adjacency /
 * src_legacy/tests/test_helpers.rs:77-126) evaluated on the exactly widened
 * values: f64 sequential norms and dots, dist = 1 - max(cos, 0) with cos = 0
 * when norm_i*norm_j <= 1e-12, keep dist <= eps and w = 1/(1+(dist/sigma)^p)
 * > 1e-12, order (dist, j), truncate topk.  Outputs [n][topk] (device): idx
 * (-1 empty), dist (f64), w (f64, may be NULL).  Bit-exact.  topk <= 64.
 * Candidates come from v_mfma_f32_32x32x16_bf16; every row is certified or
 * rescanned exactly (n_uncertified in mn_bf16_last_stats). */
int mn_knn_cos_bf16(const uint16_t *X, int64_t n, int32_t d, const mn_cos_opts *opts,
                    int32_t *out_idx, double *out_dist, double *out_w);
/* Row shard form: queries Q [nq][d] with global ids q_offset.., corpus C
 * [nc][d] with global ids c_offset..; the row whose global id equals the
 * query's is skipped; returned ids are global. */
int mn_knn_cos_bf16_qc(const uint16_t *Q, int64_t nq, const uint16_t *C, int64_t nc, int32_t d,
                       int64_t q_offset, int64_t c_offset, const mn_cos_opts *opts,
                       int32_t *out_idx, double *out_dist, double *out_w);
int mn_bf16_last_stats(mn_knn_stats *out);

#ifdef __cplusplus
}
#endif
#endif /* MATTERNET_HIP_H */
