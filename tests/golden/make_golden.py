"""Generate the committed golden fixtures (run: python tests/golden/make_golden.py).

Two kinds of data are written here:

1. reference_known_answers.json — the known-answer cases the reference's own
   test suites assert for this path, transcribed as data (inputs + expected
   outputs), each citing the reference test file:line.  The reference ships no
   golden vectors and cannot be built here (no Rust toolchain), so these are
   what pins the oracle to the reference.

2. golden_small.npz — small input/output vectors produced by an independent
   pure-Python restatement of the reference arithmetic (scalar loops on numpy
   float32/float64 scalars so every operation rounds exactly like the Rust
   code).  It is written independently of oracle/oracle.c, so agreement of the
   two is a cross-check of both.  Only small sizes (pure-Python speed).

Reference citations for the restatement are inline.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import datagen  # noqa: E402

f32 = np.float32
f64 = np.float64


# --------------------------------------------------------------------------
# Pure-Python restatement
# --------------------------------------------------------------------------

def py_l2sq(a, b):
    """surfface-core/src/distance.rs:206-213 (sequential f32 fold, no FMA)."""
    acc = f32(-0.0)
    for t in range(len(a)):
        diff = f32(f32(a[t]) - f32(b[t]))
        acc = f32(acc + f32(diff * diff))
    return acc


def py_knn_l2sq(X, k):
    """surfface-core/src/mst.rs:330-360 build_candidate_graph (stable sort)."""
    n = X.shape[0]
    keff = min(k, n - 1)
    idx = np.full((n, k), -1, np.int32)
    dist = np.full((n, k), np.inf, np.float32)
    for i in range(n):
        cand = [(j, py_l2sq(X[i], X[j])) for j in range(n) if j != i]
        cand.sort(key=lambda t: t[1])  # Python sort is stable == Rust sort_by
        for r in range(keff):
            idx[i, r], dist[i, r] = cand[r][0], cand[r][1]
    return idx, dist


def py_knn_cos(X, topk, eps, sigma, p):
    """src_legacy/tests/test_helpers.rs:77-126 build_adjacency_matrix (f64)."""
    n, d = X.shape
    norms = []
    for i in range(n):
        acc = f64(-0.0)
        for t in range(d):
            x = f64(X[i, t])
            acc = f64(acc + f64(x * x))
        norms.append(f64(math.sqrt(acc)))
    idx = np.full((n, topk), -1, np.int32)
    dist = np.full((n, topk), np.inf, np.float64)
    wts = np.zeros((n, topk), np.float64)
    for i in range(n):
        cands = []
        for j in range(n):
            if i == j:
                continue
            denom = f64(norms[i] * norms[j])
            if denom > 1e-12:
                dot = f64(-0.0)
                for t in range(d):
                    dot = f64(dot + f64(f64(X[i, t]) * f64(X[j, t])))
                cs = f64(dot / denom)
                cs = min(max(cs, -1.0), 1.0)
            else:
                cs = f64(0.0)
            distance = f64(1.0 - max(cs, 0.0))
            if distance <= eps:
                nd = f64(distance / sigma)
                w = f64(1.0 / f64(1.0 + f64(nd ** p)))
                if w > 1e-12:
                    cands.append((j, distance, w))
        cands.sort(key=lambda t: (t[1], t[0]))
        for r, (j, dd, w) in enumerate(cands[:topk]):
            idx[i, r], dist[i, r], wts[i, r] = j, dd, w
    return idx, dist, wts


def py_laplacian_union(nbr_idx, nbr_w):
    """src_legacy/laplacian.rs:297-419 (union symmetrise, D - W, CSR)."""
    n, k = nbr_idx.shape
    edges = {}
    for i in range(n):
        for r in range(k):
            j = int(nbr_idx[i, r])
            if j < 0 or j == i:
                continue
            w = float(nbr_w[i, r])
            for key in ((i, j), (j, i)):
                edges[key] = max(edges.get(key, -np.inf), w)
    indptr, indices, values = [0], [], []
    for i in range(n):
        row = sorted((j, w) for (a, j), w in edges.items() if a == i)
        deg = f64(-0.0)
        for _, w in row:
            deg = f64(deg + f64(w))
        ent = [(j, -w) for j, w in row] + [(i, deg)]
        ent.sort(key=lambda t: t[0])
        for j, v in ent:
            indices.append(j)
            values.append(v)
        indptr.append(len(indices))
    return (np.array(indptr, np.int64), np.array(indices, np.int32),
            np.array(values, np.float64))


def py_select_tau(x, mode, param=0.0):
    """src_legacy/taumode.rs:29-70."""
    FLOOR = 1e-10
    if mode == "fixed":
        return param if (math.isfinite(param) and param > 0.0) else FLOOR
    v = [float(t) for t in x if math.isfinite(t)]
    if mode == "mean":
        if not v:
            return FLOOR
        s = 0.0
        for t in v:
            s += t
        return max(s / len(v), FLOOR)
    if not v:
        return FLOOR
    v.sort()
    if mode == "percentile":
        pp = min(max(param, 0.0), 1.0)
        i = int(math.floor((len(v) - 1) * pp + 0.5))  # f64::round, pp >= 0
        return max(v[i], FLOOR)
    mid = v[len(v) // 2] if len(v) % 2 == 1 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])
    return max(mid, FLOOR)


def py_energy_taumode(x, indptr, indices, values, tau_mode="median", tau_param=0.0):
    """src_legacy/taumode.rs:261-408 (one item)."""
    f = len(x)
    x = [f64(t) for t in x]
    if all(abs(t) <= 1e-10 for t in x):
        return 0.0, 0.0, 0.0
    num = f64(-0.0)
    for i in range(f):
        rs = f64(-0.0)
        for p in range(indptr[i], indptr[i + 1]):
            rs = f64(rs + f64(f64(x[i] * values[p]) * x[indices[p]]))
        num = f64(num + rs)
    den = f64(-0.0)
    for t in x:
        den = f64(den + f64(t * t))
    E = max(float(num / den), 0.0) if den > 1e-12 else 0.0
    dense = {}
    for i in range(f):
        for p in range(indptr[i], indptr[i + 1]):
            dense[(i, int(indices[p]))] = f64(values[p])
    s = f64(0.0)
    for i in range(f):
        for j in range(f):
            if i != j:
                w = max(-dense.get((i, j), 0.0), 0.0)
                if w > 0.0:
                    dd = f64(x[i] - x[j])
                    s = f64(s + f64(f64(w * dd) * dd))
    if s <= 1e-12:
        G = 0.0
    else:
        g = f64(0.0)
        for i in range(f):
            for j in range(f):
                if i != j:
                    w = max(-dense.get((i, j), 0.0), 0.0)
                    if w > 0.0:
                        dd = f64(x[i] - x[j])
                        c = f64(f64(w * dd) * dd)
                        sh = f64(c / s)
                        g = f64(g + f64(sh * sh))
        G = min(max(float(g), 0.0), 1.0)
    tau = py_select_tau(x, tau_mode, tau_param)
    eb = E / (E + tau)
    lam = tau * eb + (1.0 - tau) * min(max(G, 0.0), 1.0)
    return E, G, lam


def py_sorted_index(lam):
    """src_legacy/sorted_index.rs:22-54 (OrderedFloat, then string id)."""
    def key(i):
        v = lam[i]
        if v != v:
            return (1, 0.0, str(i))
        return (0, v + 0.0, str(i))  # -0.0 == +0.0
    return np.array(sorted(range(len(lam)), key=key), np.int64)


def py_sfgrass(rows, ratio=0.5):
    """src_legacy/sparsification.rs:32-113 (ties kept in input order)."""
    n = len(rows)
    total = sum(len(r) for r in rows)
    if total / n < 10.0:
        return [list(r) for r in rows]
    deg = [len(r) for r in rows]
    out = []
    for i, r in enumerate(rows):
        if not r:
            out.append([])
            continue
        sc = [(w * math.sqrt(float(deg[i] * deg[j])), pos, j, w) for pos, (j, w) in enumerate(r)]
        sc.sort(key=lambda t: (-t[0], t[1]))
        keep = min(max(int(math.ceil(len(r) * ratio)), 1), len(r))
        out.append([(j, w) for _, _, j, w in sc[:keep]])
    return out


# --------------------------------------------------------------------------
# Known answers from the reference's own tests
# --------------------------------------------------------------------------

def known_answers():
    nan, inf = "nan", "inf"
    return {
        "_about": "Known-answer cases asserted by the reference's own tests, transcribed as data. "
                  "Values 'nan'/'inf'/'-inf' are strings. Each case cites the reference test.",
        "select_tau": [
            {"cite": "src_legacy/tests/test_taumode.rs:17", "x": [0.1, 0.5, 1.0], "mode": "fixed", "param": 0.3, "expect": 0.3},
            {"cite": "src_legacy/tests/test_taumode.rs:20-23", "x": [0.1, 0.5, 1.0], "mode": "fixed", "param": -0.1, "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:24-27", "x": [0.1, 0.5, 1.0], "mode": "fixed", "param": 0.0, "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:28-31", "x": [0.1, 0.5, 1.0], "mode": "fixed", "param": nan, "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:32-35", "x": [0.1, 0.5, 1.0], "mode": "fixed", "param": inf, "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:43-45", "x": [1.0, 2.0, 3.0], "mode": "mean", "expect": 2.0, "tol": 1e-12},
            {"cite": "src_legacy/tests/test_taumode.rs:48-53", "x": [1.0, nan, 3.0, inf, 2.0], "mode": "mean", "expect": 2.0, "tol": 1e-12},
            {"cite": "src_legacy/tests/test_taumode.rs:56-57", "x": [nan, inf, "-inf"], "mode": "mean", "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:60-61", "x": [], "mode": "mean", "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:69-70", "x": [3.0, 1.0, 2.0], "mode": "median", "expect": 2.0},
            {"cite": "src_legacy/tests/test_taumode.rs:73-75", "x": [1.0, 2.0, 3.0, 4.0], "mode": "median", "expect": 2.5, "tol": 1e-12},
            {"cite": "src_legacy/tests/test_taumode.rs:78-79", "x": [5.0], "mode": "median", "expect": 5.0},
            {"cite": "src_legacy/tests/test_taumode.rs:82-83", "x": [nan, 1.0, 3.0, inf, 2.0], "mode": "median", "expect": 2.0},
            {"cite": "src_legacy/tests/test_taumode.rs:86-90", "x": [nan, inf], "mode": "median", "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:93-94", "x": [], "mode": "median", "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:104-107", "x": [1, 2, 3, 4, 5], "mode": "percentile", "param": 0.0, "expect": 1.0},
            {"cite": "src_legacy/tests/test_taumode.rs:110-113", "x": [1, 2, 3, 4, 5], "mode": "percentile", "param": 1.0, "expect": 5.0},
            {"cite": "src_legacy/tests/test_taumode.rs:116-119", "x": [1, 2, 3, 4, 5], "mode": "percentile", "param": 0.5, "expect": 3.0},
            {"cite": "src_legacy/tests/test_taumode.rs:122-125", "x": [1, 2, 3, 4, 5], "mode": "percentile", "param": -0.1, "expect": 1.0},
            {"cite": "src_legacy/tests/test_taumode.rs:126-129", "x": [1, 2, 3, 4, 5], "mode": "percentile", "param": 1.5, "expect": 5.0},
            {"cite": "src_legacy/tests/test_taumode.rs:133-137", "x": [], "mode": "percentile", "param": 0.5, "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:145-150", "x": [2e-10], "mode": "mean", "expect": 2e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:153-154", "x": [5e-11], "mode": "mean", "expect": 1e-10},
            {"cite": "src_legacy/tests/test_taumode.rs:157-158", "x": [0.0], "mode": "mean", "expect": 1e-10},
        ],
        "l2sq_distance": [
            {"cite": "surfface-core/src/tests/test_distance.rs:236-251", "a": [1, 2, 3], "b": [4, 5, 6], "expect": 27.0, "tol": 1e-5},
            {"cite": "surfface-core/src/tests/test_distance.rs:218-233,254-263", "a": [0, 0], "b": [3, 4], "expect_sqrt": 5.0, "tol": 1e-5},
        ],
        "cosine": [
            {"cite": "surfface-core/src/tests/test_distance.rs:266-281", "a": [1, 1], "b": [2, 2], "expect_cos": 1.0, "tol": 1e-5},
            {"cite": "surfface-core/src/tests/test_distance.rs:284-299", "a": [1, 0], "b": [0, 1], "expect_cos": 0.0, "tol": 1e-5},
            {"cite": "surfface-core/src/tests/test_distance.rs:302-317", "a": [1, 0], "b": [0, 1], "expect_dist": 1.0, "tol": 1e-5},
        ],
        "knn_line": {
            "cite": "surfface-core/src/tests/test_mst.rs:15-22 (5 centroids on a line); kNN tie rule mst.rs:344 stable sort_by",
            "X": [[0, 0], [1, 0], [2, 0], [3, 0], [4, 0]],
            "k": 2,
            "expect_idx": [[1, 2], [0, 2], [1, 3], [2, 4], [3, 2]],
            "expect_dist": [[1, 4], [1, 1], [1, 1], [1, 1], [1, 4]],
        },
        "rayleigh": [
            {"cite": "surfface-core/src/tests/test_spectral.rs:102-122", "L_dense": [[1, -1], [-1, 1]], "x": [[1, 1]], "expect_E": [0.0], "tol": 1e-5},
            {"cite": "surfface-core/src/tests/test_spectral.rs:187-251 (chain 0-1-2)",
             "L_dense": [[1, -1, 0], [-1, 2, -1], [0, -1, 1]], "x": [[1, 1, 1], [1, 0, -1]],
             "expect_E": [0.0, 1.0], "expect_lambda0_zero": True, "expect_lambda1_gt_lambda0": True, "tol": 1e-5,
             "note": "the test asserts lambda0 ~ 0 and lambda1 > lambda0; E1 = x.Lx/x.x = 2/2 = 1 is derived "
                     "(the test's inline comment claiming x^T L x = 0 miscomputes L.x)"},
        ],
        "dispersion_constant_rows": {
            "cite": "surfface-core/src/tests/test_spectral.rs:124-144",
            "L_dense": [[1, -0.5], [-0.5, 1]], "x": [[1, 1], [1, 1]], "expect_G": [0.0, 0.0], "tol": 1e-5},
        "laplacian_d_minus_a": {
            "cite": "src_legacy/tests/test_laplacian.rs:655-721 (test_with_adjacency_output)",
            "items": [[1.0, 0.0], [0.9, 0.1], [0.0, 1.0]],
            "params": {"eps": 0.5, "topk": 1, "p": 1.0, "sigma": 0.2},
            "check": "L_ii == sum_j A_ij and L_ij == -A_ij within 1e-10; adjacency diagonal zero",
        },
        "sfgrass_basic": {
            "cite": "src_legacy/tests/test_sparsification.rs:5-16",
            "rows": [[[1, 1.0], [2, 0.5]], [[0, 1.0], [2, 0.8]], [[0, 0.5], [1, 0.8]]],
            "check": "3 rows, none empty (avg degree < 10 => unchanged)",
        },
        "sfgrass_larger": {
            "cite": "src_legacy/tests/test_sparsification.rs:19-39",
            "n": 50, "rule": "edge (i,j) iff i != j and (i+j) % 3 == 0, w = 1/(1+|i-j|)",
            "check": "50 rows, fewer edges than the input",
        },
        "sorted_index_ascending": {
            "cite": "src_legacy/storage/test_load_from_storage.rs:243-267; sorted_index.rs:22-28 (ties by string id)",
            "lambda": [0.5, 0.1, 0.5, 0.3, 0.1, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.1],
            "expect_order": [1, 11, 4, 3, 0, 10, 2, 5, 6, 7, 8, 9],
        },
        "normalise_lambdas": {
            "cite": "src_legacy/core.rs:1341-1354",
            "lambda": [-1.0, -3.0, -2.0],
            "expect": [2.0 / 3.0, 0.0, 1.0 / 3.0],
            "note": "max fold starts at 0.0 => max=0, min=-3, range=3",
        },
    }


def main():
    ka = known_answers()
    with open(os.path.join(HERE, "reference_known_answers.json"), "w") as fh:
        json.dump(ka, fh, indent=1)

    out = {}
    # K1 L2^2: uniform, clustered-with-duplicates, and integer grid (many exact ties)
    Xu = datagen.uniform(40, 8, seed=42)
    out["l2_uniform_X"] = Xu
    out["l2_uniform_idx"], out["l2_uniform_dist"] = py_knn_l2sq(Xu, 5)
    Xc = datagen.clustered(36, 6, seed=7, blobs=3, dup_frac=0.1, zero_frac=0.06)
    out["l2_clustered_X"] = Xc
    out["l2_clustered_idx"], out["l2_clustered_dist"] = py_knn_l2sq(Xc, 7)
    g = np.array([[a, b] for a in range(5) for b in range(5)], np.float32)
    out["l2_grid_X"] = g
    out["l2_grid_idx"], out["l2_grid_dist"] = py_knn_l2sq(g, 6)
    # K1 cosine (production-style parameters eps=1, sigma=1, p=2)
    Xk = datagen.uniform(30, 6, seed=11)
    out["cos_X"] = Xk
    ci, cd, cw = py_knn_cos(Xk, 4, eps=1.0, sigma=1.0, p=2.0)
    out["cos_idx"], out["cos_dist"], out["cos_w"] = ci, cd, cw
    # K2 union Laplacian from the cosine kNN
    out["lapu_indptr"], out["lapu_indices"], out["lapu_values"] = py_laplacian_union(ci, cw)
    # K3 taumode energy on the cosine-kNN feature graph (f = 30 nodes) for 12 items
    Xe = datagen.uniform(12, 30, seed=5)
    Xe[3] = 0.0  # zero-vector path
    out["energy_X"] = Xe
    ip, ix, iv = out["lapu_indptr"], out["lapu_indices"], out["lapu_values"]
    res = [py_energy_taumode(Xe[r], ip, ix, iv) for r in range(Xe.shape[0])]
    out["energy_E"] = np.array([r[0] for r in res])
    out["energy_G"] = np.array([r[1] for r in res])
    out["energy_lambda"] = np.array([r[2] for r in res])
    # K4 sorted index with ties, -0.0, NaN and multi-digit ids
    lam = np.array([0.5, 0.1, 0.5, np.nan, -0.0, 0.0, 0.3, 0.1, 0.5, np.nan, 0.3, 0.5, 0.1], np.float64)
    out["sort_lambda"] = lam
    out["sort_order"] = py_sorted_index(lam)
    # K5 SF-GRASS on the reference's "larger" test graph
    n = 50
    rows = [[(j, 1.0 / (1.0 + abs(i - j))) for j in range(n) if i != j and (i + j) % 3 == 0]
            for i in range(n)]
    sp = py_sfgrass(rows, 0.5)
    out["sf_in_indptr"] = np.cumsum([0] + [len(r) for r in rows]).astype(np.int64)
    out["sf_in_indices"] = np.array([j for r in rows for j, _ in r], np.int32)
    out["sf_in_w"] = np.array([w for r in rows for _, w in r], np.float64)
    out["sf_out_indptr"] = np.cumsum([0] + [len(r) for r in sp]).astype(np.int64)
    out["sf_out_indices"] = np.array([j for r in sp for j, _ in r], np.int32)
    out["sf_out_w"] = np.array([w for r in sp for _, w in r], np.float64)
    np.savez_compressed(os.path.join(HERE, "golden_small.npz"), **out)
    print("wrote", sorted(out))


if __name__ == "__main__":
    main()
