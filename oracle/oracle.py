"""ctypes binding of liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline.  The
product (matternet-rs_amd/, include/matternet_hip.h) never touches it.
See oracle.h for the reference citations of every function.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

TAU_FIXED, TAU_MEDIAN, TAU_MEAN, TAU_PERCENTILE = 0, 1, 2, 3
G_TAUMODE, G_ENERGYMAPS = 0, 1


def build() -> str:
    """Compile liboracle.so in place (gcc); returns its path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liboracle.so")


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        src = os.path.join(_HERE, "oracle.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            build()
        _LIB = C.CDLL(path)
        _declare(_LIB)
    return _LIB


P = C.c_void_p
I64 = C.c_int64
I32 = C.c_int32
D = C.c_double
F = C.c_float


def _declare(L):
    L.or_knn_l2sq_f32.argtypes = [P, I64, I32, I32, I64, I64, C.c_int, C.c_int, P, P]
    L.or_knn_l2sq_rows_f32.argtypes = [P, I64, I32, I32, P, I64, C.c_int, P, P]
    L.or_libm_f32.argtypes = [P, I64, C.c_uint32, C.c_int, P, C.c_int]
    L.or_pow_f64.argtypes = [P, P, I64, P]
    L.or_libm_mismatch.argtypes = [C.c_uint32, I64, C.c_int, P]
    L.or_libm_mismatch.restype = I64
    L.or_glibc_restated_check.argtypes = [C.c_int, I64]
    L.or_glibc_restated_check.restype = I64
    L.or_glibc_tables.argtypes = [C.c_int, P]
    L.or_knn_l2sq_qc_f32.argtypes = [P, I64, P, P, I64, I32, I64, I32, C.c_int, C.c_int, P, P]
    L.or_knn_l2_f64.argtypes = [P, I64, P, I64, I32, P, I32, C.c_int, C.c_int, P, P]
    L.or_knn_cos_f64.argtypes = [P, I64, I32, I32, D, D, D, I64, I64, C.c_int, P, P, P]
    L.or_knn_cos_f64d.argtypes = [P, I64, I32, I32, D, D, D, I64, I64, C.c_int, P, P, P]
    L.or_knn_cos_bf16_rows.argtypes = [P, I64, I32, I32, D, D, D, P, I64, C.c_int, P, P, P]
    L.or_laplacian_union.argtypes = [I64, I32, P, P, I64, P, P, P, P]
    L.or_laplacian_max.argtypes = [I64, I64, P, P, P, F, C.c_int, I64, P, P, P, P, P, P]
    L.or_select_tau.argtypes = [P, I64, C.c_int, D]
    L.or_select_tau.restype = D
    L.or_energy_rows.argtypes = [P, I64, I32, P, P, P, C.c_int, C.c_int, D, C.c_int, P, P, P]
    L.or_energy_rows_faithful.argtypes = [P, I64, I32, P, P, P, C.c_int, D, C.c_int, P, P, P]
    L.or_normalise_lambdas.argtypes = [P, I64, P, P, P]
    L.or_spectral_lambdas_f32.argtypes = [P, I64, I32, P, P, P, P]
    L.or_sorted_index.argtypes = [P, I64, P, P, P]
    L.or_bc_knn.argtypes = [P, P, I64, I32, I32, C.c_float, C.c_float, P, P]
    L.or_bhattacharyya_distance.argtypes = [P, P, P, P, I64]
    L.or_bhattacharyya_distance.restype = C.c_float
    L.or_nearest_centroid.argtypes = [P, I64, P, I64, I32, P, P]
    L.or_mst_candidates.argtypes = [P, P, I64, I32, I32, C.c_int, C.c_int, P, P, P, P]
    L.or_diffuse_rows.argtypes = [P, I64, I32, P, P, P, C.c_double, I32, C.c_int, P]
    L.or_range_bylambda.argtypes = [P, P, I64, C.c_double, C.c_double, I64, C.c_double, P, P]
    L.or_range_bylambda.restype = I64
    L.or_k_nearest_by_lambda.argtypes = [P, P, I64, C.c_double, C.c_double, I64, C.c_double,
                                         C.c_int, C.c_double, C.c_double, C.c_double, P, P]
    L.or_k_nearest_by_lambda.restype = I64
    L.or_sfgrass.argtypes = [I64, P, P, P, D, P, P, P]
    L.or_search_lambda_aware.argtypes = [P, I64, I32, P, P, P, I64, I64, D, C.c_int, P, P, P]
    L.or_search_lambda_aware_hybrid.argtypes = [P, I64, I32, P, P, P, I64, I64, D, C.c_int, P, P,
                                                P]


def _p(a):
    return a.ctypes.data_as(P) if a is not None else None


def _check(rc, name):
    if rc != 0:
        raise RuntimeError(f"oracle {name} failed with code {rc}")


def knn_l2sq(X, k, q_begin=0, q_end=None, mode=1, nthreads=0):
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, d = X.shape
    q_end = n if q_end is None else q_end
    m = q_end - q_begin
    idx = np.empty((m, k), np.int32)
    dist = np.empty((m, k), np.float32)
    _check(lib().or_knn_l2sq_f32(_p(X), n, d, k, q_begin, q_end, mode, nthreads, _p(idx), _p(dist)),
           "knn_l2sq")
    return idx, dist


def knn_l2sq_rows(X, k, rows, nthreads=0):
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, d = X.shape
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    idx = np.empty((len(rows), k), np.int32)
    dist = np.empty((len(rows), k), np.float32)
    _check(lib().or_knn_l2sq_rows_f32(_p(X), n, d, k, _p(rows), len(rows), nthreads, _p(idx),
                                      _p(dist)), "knn_l2sq_rows")
    return idx, dist


def knn_l2sq_qc(Q, q_ids, Cm, c_off, k, excl=True, nthreads=0):
    """Per-shard L2^2 kNN (or_knn_l2sq_qc_f32): queries with global ids against
    a corpus shard whose rows have global ids c_off + j."""
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    Cm = np.ascontiguousarray(Cm, dtype=np.float32)
    q_ids = np.ascontiguousarray(q_ids, dtype=np.int64)
    nq, d = Q.shape
    idx = np.empty((nq, k), np.int32)
    dist = np.empty((nq, k), np.float32)
    _check(lib().or_knn_l2sq_qc_f32(_p(Q), nq, _p(q_ids), _p(Cm), Cm.shape[0], d, c_off, k,
                                    int(excl), nthreads, _p(idx), _p(dist)), "knn_l2sq_qc")
    return idx, dist


def knn_l2_f64(Q, Cm, k, q_ids=None, use_sqrt=False, nthreads=0):
    """f64 Euclidean kNN of the rows of Q against C (oracle.h or_knn_l2_f64)."""
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    Cm = np.ascontiguousarray(Cm, dtype=np.float64)
    nq, d = Q.shape
    ids = None if q_ids is None else np.ascontiguousarray(q_ids, dtype=np.int64)
    idx = np.empty((nq, k), np.int32)
    dist = np.empty((nq, k), np.float64)
    _check(lib().or_knn_l2_f64(_p(Q), nq, _p(Cm), Cm.shape[0], d, _p(ids), k,
                               1 if use_sqrt else 0, nthreads, _p(idx), _p(dist)), "knn_l2_f64")
    return idx, dist


def knn_cos(X, topk, eps=1.0, sigma=1.0, p=2.0, q_begin=0, q_end=None, nthreads=0):
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, d = X.shape
    q_end = n if q_end is None else q_end
    m = q_end - q_begin
    idx = np.empty((m, topk), np.int32)
    dist = np.empty((m, topk), np.float64)
    w = np.empty((m, topk), np.float64)
    _check(lib().or_knn_cos_f64(_p(X), n, d, topk, eps, sigma, p, q_begin, q_end, nthreads,
                                _p(idx), _p(dist), _p(w)), "knn_cos")
    return idx, dist, w


def knn_cos_f64(X, topk, eps=1.0, sigma=1.0, p=2.0, nthreads=0):
    """A.1c over f64 rows (nodes = rows)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    idx = np.empty((n, topk), np.int32)
    dist = np.empty((n, topk), np.float64)
    w = np.empty((n, topk), np.float64)
    _check(lib().or_knn_cos_f64d(_p(X), n, d, topk, eps, sigma, p, 0, n, nthreads,
                                 _p(idx), _p(dist), _p(w)), "knn_cos_f64")
    return idx, dist, w


def knn_cos_bf16_rows(Xbits, topk, rows, eps=1.0, sigma=1.0, p=2.0, nthreads=0):
    """A.1c on bf16 rows given as uint16 bits [n, d], for explicit query rows."""
    Xbits = np.ascontiguousarray(Xbits, dtype=np.uint16)
    n, d = Xbits.shape
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    m = rows.shape[0]
    idx = np.empty((m, topk), np.int32)
    dist = np.empty((m, topk), np.float64)
    w = np.empty((m, topk), np.float64)
    _check(lib().or_knn_cos_bf16_rows(_p(Xbits), n, d, topk, eps, sigma, p, _p(rows), m,
                                      nthreads, _p(idx), _p(dist), _p(w)), "knn_cos_bf16_rows")
    return idx, dist, w


def laplacian_union(nbr_idx, nbr_w):
    nbr_idx = np.ascontiguousarray(nbr_idx, dtype=np.int32)
    nbr_w = np.ascontiguousarray(nbr_w, dtype=np.float64)
    n, k = nbr_idx.shape
    cap = 2 * n * k + n
    indptr = np.empty(n + 1, np.int64)
    indices = np.empty(cap, np.int32)
    values = np.empty(cap, np.float64)
    nnz = np.zeros(1, np.int64)
    _check(lib().or_laplacian_union(n, k, _p(nbr_idx), _p(nbr_w), cap, _p(indptr), _p(indices),
                                    _p(values), _p(nnz)), "laplacian_union")
    nz = int(nnz[0])
    return indptr, indices[:nz].copy(), values[:nz].copy()


def laplacian_max(n, src, dst, w, thr=1e-9, normalize=True):
    src = np.ascontiguousarray(src, dtype=np.int32)
    dst = np.ascontiguousarray(dst, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float32)
    m = len(src)
    cap = 2 * m + n
    indptr = np.empty(n + 1, np.int64)
    indices = np.empty(cap, np.int32)
    values = np.empty(cap, np.float32)
    nnz = np.zeros(1, np.int64)
    deg = np.empty(n, np.float32)
    nnz_ref = np.zeros(1, np.int64)
    _check(lib().or_laplacian_max(n, m, _p(src), _p(dst), _p(w), thr, int(normalize), cap,
                                  _p(indptr), _p(indices), _p(values), _p(nnz), _p(deg),
                                  _p(nnz_ref)), "laplacian_max")
    nz = int(nnz[0])
    return indptr, indices[:nz].copy(), values[:nz].copy(), deg, int(nnz_ref[0])


def select_tau(x, mode, param=0.0):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return float(lib().or_select_tau(_p(x), len(x), mode, param))


def energy_rows(X, indptr, indices, values, g_mode=G_TAUMODE, tau_mode=TAU_MEDIAN,
                tau_param=0.0, nthreads=0):
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, f = X.shape
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    values = np.ascontiguousarray(values, dtype=np.float64)
    E = np.empty(n, np.float64)
    G = np.empty(n, np.float64)
    lam = np.empty(n, np.float64)
    _check(lib().or_energy_rows(_p(X), n, f, _p(indptr), _p(indices), _p(values), g_mode,
                                tau_mode, tau_param, nthreads, _p(E), _p(G), _p(lam)),
           "energy_rows")
    return E, G, lam


def energy_rows_faithful(X, indptr, indices, values, tau_mode=TAU_MEDIAN, tau_param=0.0,
                         nthreads=0):
    """TAUMODE rows with the reference's F^2 CsMat::get dispersion (cost model
    of the faithful CPU baseline); values equal energy_rows(G_TAUMODE)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, f = X.shape
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    values = np.ascontiguousarray(values, dtype=np.float64)
    E = np.empty(n); G = np.empty(n); lam = np.empty(n)
    _check(lib().or_energy_rows_faithful(_p(X), n, f, _p(indptr), _p(indices), _p(values),
                                         tau_mode, tau_param, nthreads, _p(E), _p(G), _p(lam)),
           "energy_rows_faithful")
    return E, G, lam


def normalise_lambdas(lam):
    lam = np.array(lam, dtype=np.float64, copy=True)
    mn, mx, rg = np.zeros(1), np.zeros(1), np.zeros(1)
    _check(lib().or_normalise_lambdas(_p(lam), len(lam), _p(mn), _p(mx), _p(rg)), "normalise")
    return lam, float(mn[0]), float(mx[0]), float(rg[0])


def spectral_lambdas(X, indptr, indices, values):
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, f = X.shape
    out = np.empty(n, np.float32)
    _check(lib().or_spectral_lambdas_f32(
        _p(X), n, f, _p(np.ascontiguousarray(indptr, np.int64)),
        _p(np.ascontiguousarray(indices, np.int32)), _p(np.ascontiguousarray(values, np.float32)),
        _p(out)), "spectral")
    return out


def sorted_index(lam):
    lam = np.ascontiguousarray(lam, dtype=np.float64)
    n = len(lam)
    order = np.empty(n, np.int64)
    keys = np.empty(n, np.float64)
    std = np.zeros(1)
    _check(lib().or_sorted_index(_p(lam), n, _p(order), _p(keys), _p(std)), "sorted_index")
    return order, keys, float(std[0])


def bc_knn(means, variances, k, reg=1e-6, thr=1e-9):
    """compute_bhattacharyya_weights (surfface-core/src/laplacian.rs:254-298):
    means/variances [C, F] -> (idx [F, k] int32, w [F, k] f32)."""
    means = np.ascontiguousarray(means, np.float32)
    variances = np.ascontiguousarray(variances, np.float32)
    c, f = means.shape
    idx = np.empty((f, k), np.int32)
    w = np.empty((f, k), np.float32)
    _check(lib().or_bc_knn(_p(means), _p(variances), c, f, k, reg, thr, _p(idx), _p(w)), "bc_knn")
    return idx, w


def bhattacharyya_distance(mean_i, var_i, mean_j, var_j):
    """distance.rs:78-108 bhattacharyya_distance_diagonal (f32)."""
    a = [np.ascontiguousarray(v, np.float32) for v in (mean_i, var_i, mean_j, var_j)]
    return np.float32(lib().or_bhattacharyya_distance(*[_p(v) for v in a], a[0].shape[0]))


MST_BHATTACHARYYA, MST_EUCLIDEAN, MST_SQEUCLIDEAN = 0, 1, 2
TW_MEAN, TW_MIN, TW_MAX, TW_GEOMEAN, TW_NONE = 0, 1, 2, 3, 4


def mst_candidates(means, variances, k, metric=MST_BHATTACHARYYA, tw=TW_MEAN, thickness=None):
    """MSTStage::build_candidate_graph (mst.rs:312-412): (v, dist, cost) [c, k']."""
    means = np.ascontiguousarray(means, np.float32)
    c, f = means.shape
    variances = None if variances is None else np.ascontiguousarray(variances, np.float32)
    th = None if thickness is None else np.ascontiguousarray(thickness, np.float32)
    kk = min(k, c - 1)
    v = np.empty((c, kk), np.int32)
    d = np.empty((c, kk), np.float32)
    cost = np.empty((c, kk), np.float32)
    _check(lib().or_mst_candidates(_p(means), None if variances is None else _p(variances), c, f,
                                   k, metric, tw, None if th is None else _p(th), _p(v), _p(d),
                                   _p(cost)), "mst_candidates")
    return v, d, cost


def nearest_centroid(batch, cents):
    """stages/clustering.rs:42-63 batch nearest centroid (fixed-order restatement)."""
    batch = np.ascontiguousarray(batch, np.float32)
    cents = np.ascontiguousarray(cents, np.float32)
    b, f = batch.shape
    idx = np.empty(b, np.int32)
    dist = np.empty(b, np.float32)
    _check(lib().or_nearest_centroid(_p(batch), b, _p(cents), cents.shape[0], f, _p(idx),
                                     _p(dist)), "nearest_centroid")
    return idx, dist


def diffuse_rows(X, indptr, indices, values, eta=0.1, steps=4, matvec=False):
    """energymaps.rs:518-546 diffusion (or graph.rs:464-501 L x) per row, f64."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, f = X.shape
    out = np.empty_like(X)
    _check(lib().or_diffuse_rows(_p(X), n, f, _p(np.ascontiguousarray(indptr, np.int64)),
                                 _p(np.ascontiguousarray(indices, np.int32)),
                                 _p(np.ascontiguousarray(values, np.float64)), eta, steps,
                                 1 if matvec else 0, _p(out)), "diffuse")
    return out


def range_bylambda(keys, order, std_dev, lq, k, p):
    """sorted_index.rs:64-80 for one query; None where the reference panics."""
    oi, ok = np.empty(max(k, 1), np.int64), np.empty(max(k, 1), np.float64)
    c = lib().or_range_bylambda(_p(np.ascontiguousarray(keys, np.float64)),
                                _p(np.ascontiguousarray(order, np.int64)), len(keys), std_dev,
                                lq, k, p, _p(oi), _p(ok))
    return None if c < 0 else (oi[:c], ok[:c])


def k_nearest_by_lambda(keys, order, std_dev, lq, k, lambda_p, base_delta=None, growth=1.7,
                        max_multiplier=10.0):
    """sorted_index.rs:85-140 for one query; None where the reference panics."""
    oi, ok = np.empty(max(k, 1), np.int64), np.empty(max(k, 1), np.float64)
    c = lib().or_k_nearest_by_lambda(_p(np.ascontiguousarray(keys, np.float64)),
                                     _p(np.ascontiguousarray(order, np.int64)), len(keys),
                                     std_dev, lq, k, lambda_p, 0 if base_delta is None else 1,
                                     0.0 if base_delta is None else base_delta, growth,
                                     max_multiplier, _p(oi), _p(ok))
    if c == -2:
        raise MemoryError("or_k_nearest_by_lambda")
    return None if c < 0 else (oi[:c], ok[:c])


def sfgrass(indptr, indices, w, ratio=0.5):
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float64)
    n = len(indptr) - 1
    cap = max(int(indptr[-1]), 1)
    oi = np.empty(n + 1, np.int64)
    oj = np.empty(cap, np.int32)
    ow = np.empty(cap, np.float64)
    _check(lib().or_sfgrass(n, _p(indptr), _p(indices), _p(w), ratio, _p(oi), _p(oj), _p(ow)),
           "sfgrass")
    nz = int(oi[-1])
    return oi, oj[:nz].copy(), ow[:nz].copy()


def search_lambda_aware(X, lambdas, Q, lambda_q, k, alpha, nthreads=0, hybrid=False):
    """core.rs:1156-1193 for every query row of Q: (idx [nq,k], score [nq,k],
    count [nq]); count -1 where the reference asserts lambda != 0, -3 on NaN."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    lam = np.ascontiguousarray(lambdas, dtype=np.float64)
    lq = np.ascontiguousarray(lambda_q, dtype=np.float64)
    n, f = X.shape
    nq = Q.shape[0]
    oi = np.empty((nq, max(k, 1)), np.int64)
    os_ = np.empty((nq, max(k, 1)), np.float64)
    oc = np.empty(nq, np.int64)
    fn = lib().or_search_lambda_aware_hybrid if hybrid else lib().or_search_lambda_aware
    _check(fn(_p(X), n, f, _p(lam), _p(Q), _p(lq), nq, k, alpha, nthreads, _p(oi), _p(os_),
              _p(oc)), "search_lambda_aware")
    return oi[:, :k], os_[:, :k], oc


# ---- glibc logf / expf (glibc_check.c) -------------------------------------
def libm_f32(x=None, n=None, bits0=0, fn=0):
    """The HOST glibc logf (fn 0) / expf (fn 1) of x, or of the bit patterns
    bits0 .. bits0 + n - 1."""
    if x is not None:
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = len(x)
    out = np.empty(n, np.float32)
    _check(lib().or_libm_f32(None if x is None else _p(x), n, bits0, fn, _p(out), 0), "libm_f32")
    return out


def libm_mismatch(bits0, got, fn):
    """How many of got[i] differ from the host glibc value at bit pattern
    bits0 + i (NaN matches NaN)."""
    got = np.ascontiguousarray(got, dtype=np.float32)
    return int(lib().or_libm_mismatch(bits0, len(got), fn, _p(got)))


def glibc_restated_check(fn, stride):
    """Mismatches of the host copy of the device restatement vs host glibc
    over every stride-th f32 bit pattern."""
    return int(lib().or_glibc_restated_check(fn, stride))


def glibc_tables(which):
    out = np.zeros(40, np.uint64)
    m = lib().or_glibc_tables(which, _p(out))
    return out[:m]


def glibc_tables_from_libm(path=None):
    """Re-derive the restatement's tables from the host libm's bytes: the
    logf table is the 16 {1/c, log c} pairs right before ln2 (followed by the
    3 polynomial coefficients, e_logf_data.c layout); the expf data is the 32
    table words + shift_scaled + poly[3] + shift + invln2_scaled +
    poly_scaled[3] (e_exp2f_data.c layout) around invln2_scaled = 32/ln2."""
    import ctypes.util
    import struct
    path = path or "/lib/x86_64-linux-gnu/libm.so.6"
    data = open(path, "rb").read()
    ln2 = struct.pack("<d", float.fromhex("0x1.62e42fefa39efp-1"))
    log = None
    p = data.find(ln2)
    while p >= 0:
        if p >= 256:
            tab = np.frombuffer(data[p - 256:p], dtype="<f8").reshape(16, 2)
            if np.all((tab[:, 0] > 0.6) & (tab[:, 0] < 1.6)) and \
                    np.allclose(tab[:, 1], -np.log(tab[:, 0]), atol=1e-6):
                poly = np.frombuffer(data[p + 8:p + 32], dtype="<u8")
                log = np.concatenate([tab.reshape(-1).view(np.uint64), poly[[0, 1, 2]],
                                      np.frombuffer(ln2, dtype="<u8")])
                break
        p = data.find(ln2, p + 1)
    inv = struct.pack("<d", float.fromhex("0x1.71547652b82fep+5"))
    q = data.find(inv)
    base = q - 256 - 8 - 24 - 8
    tab = np.frombuffer(data[base:base + 256], dtype="<u8")
    rest = np.frombuffer(data[base + 256:base + 256 + 72], dtype="<u8")
    # rest: shift_scaled, poly[3], shift, invln2_scaled, poly_scaled[3]
    exp = np.concatenate([tab, rest[[6, 7, 8]], rest[[5]], rest[[4]]])
    return log, exp


def pow_f64(x, y):
    """The host glibc pow elementwise (or_pow_f64): the reference's f64::powf."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(np.broadcast_to(np.asarray(y, np.float64), x.shape), dtype=np.float64)
    out = np.empty_like(x)
    _check(lib().or_pow_f64(_p(x), _p(y), x.size, _p(out)), "pow_f64")
    return out
