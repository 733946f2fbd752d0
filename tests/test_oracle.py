"""Pin the CPU oracle (oracle/liboracle.so) before trusting it.

* against every known-answer case the reference's own tests assert
  (tests/golden/reference_known_answers.json, each citing its test file:line);
* against the independent pure-Python restatement's fixtures
  (tests/golden/golden_small.npz, made by tests/golden/make_golden.py).
Bit-exact for integer/index outputs and for the sequential-fold distances;
1e-12 relative for the f64 energy scalars (same summation order).
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

import datagen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HERE = os.path.dirname(os.path.abspath(__file__))
KA = json.load(open(os.path.join(HERE, "golden", "reference_known_answers.json")))
GS = np.load(os.path.join(HERE, "golden", "golden_small.npz"))


def _num(v):
    if isinstance(v, str):
        return {"nan": math.nan, "inf": math.inf, "-inf": -math.inf}[v]
    return float(v)


MODES = {"fixed": O.TAU_FIXED, "median": O.TAU_MEDIAN, "mean": O.TAU_MEAN,
         "percentile": O.TAU_PERCENTILE}


@pytest.mark.parametrize("case", KA["select_tau"], ids=lambda c: c["cite"])
def test_select_tau_known_answers(case):
    x = np.array([_num(v) for v in case["x"]], np.float64)
    got = O.select_tau(x, MODES[case["mode"]], _num(case.get("param", 0.0)))
    tol = case.get("tol", 0.0)
    assert abs(got - case["expect"]) <= tol, (got, case)


def test_l2sq_known_answers():
    c = KA["l2sq_distance"]
    X = np.array([c[0]["a"], c[0]["b"]], np.float32)
    _, dist = O.knn_l2sq(X, 1)
    assert abs(dist[0, 0] - c[0]["expect"]) <= c[0]["tol"]
    X = np.array([c[1]["a"], c[1]["b"]], np.float32)
    _, dist = O.knn_l2sq(X, 1)
    assert abs(math.sqrt(dist[0, 0]) - c[1]["expect_sqrt"]) <= c[1]["tol"]


def test_cosine_known_answers():
    for c in KA["cosine"]:
        X = np.array([c["a"], c["b"]], np.float32)
        _, dist, _ = O.knn_cos(X, 1, eps=1.0, sigma=1.0, p=2.0)
        if "expect_cos" in c:
            assert abs((1.0 - dist[0, 0]) - c["expect_cos"]) <= c["tol"]
        else:
            assert abs(dist[0, 0] - c["expect_dist"]) <= c["tol"]


def test_knn_line_tie_rule():
    c = KA["knn_line"]
    idx, dist = O.knn_l2sq(np.array(c["X"], np.float32), c["k"])
    assert idx.tolist() == c["expect_idx"]
    assert dist.tolist() == c["expect_dist"]


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("name,k", [("l2_uniform", 5), ("l2_clustered", 7), ("l2_grid", 6)])
def test_knn_l2sq_vs_python_restatement(name, k, mode):
    idx, dist = O.knn_l2sq(GS[name + "_X"], k, mode=mode)
    np.testing.assert_array_equal(idx, GS[name + "_idx"])
    np.testing.assert_array_equal(dist.view(np.uint32), GS[name + "_dist"].view(np.uint32))


def test_knn_l2sq_query_range_and_small_n():
    X = GS["l2_uniform_X"]
    i_all, d_all = O.knn_l2sq(X, 5)
    i_sub, d_sub = O.knn_l2sq(X, 5, q_begin=7, q_end=19)
    np.testing.assert_array_equal(i_sub, i_all[7:19])
    # k > n-1: reference truncates to min(k, n-1)
    idx, dist = O.knn_l2sq(X[:3], 5)
    assert (idx[:, 2:] == -1).all() and np.isinf(dist[:, 2:]).all()


def test_knn_l2sq_nonfinite_is_error():
    X = np.array([[0, 0], [np.nan, 1], [1, 1]], np.float32)
    with pytest.raises(RuntimeError):
        O.knn_l2sq(X, 1)


def test_knn_cos_vs_python_restatement():
    idx, dist, w = O.knn_cos(GS["cos_X"], 4, eps=1.0, sigma=1.0, p=2.0)
    np.testing.assert_array_equal(idx, GS["cos_idx"])
    np.testing.assert_array_equal(dist, GS["cos_dist"])
    np.testing.assert_array_equal(w, GS["cos_w"])


def test_laplacian_union_vs_python_restatement():
    ip, ix, iv = O.laplacian_union(GS["cos_idx"], GS["cos_w"])
    np.testing.assert_array_equal(ip, GS["lapu_indptr"])
    np.testing.assert_array_equal(ix, GS["lapu_indices"])
    np.testing.assert_array_equal(iv, GS["lapu_values"])


def test_laplacian_d_minus_a_known_answer():
    c = KA["laplacian_d_minus_a"]
    X = np.array(c["items"], np.float32)
    p = c["params"]
    idx, dist, w = O.knn_cos(X, p["topk"], eps=p["eps"], sigma=p["sigma"], p=p["p"])
    ip, ix, iv = O.laplacian_union(idx, w)
    n = X.shape[0]
    L = np.zeros((n, n))
    for i in range(n):
        L[i, ix[ip[i]:ip[i + 1]]] = iv[ip[i]:ip[i + 1]]
    A = -L.copy()
    np.fill_diagonal(A, 0.0)
    assert np.all(np.diag(A) == 0)
    for i in range(n):
        assert abs(L[i, i] - A[i].sum()) < 1e-10
    assert np.allclose(L, L.T, atol=1e-10)


def test_energy_taumode_vs_python_restatement():
    E, G, lam = O.energy_rows(GS["energy_X"], GS["lapu_indptr"], GS["lapu_indices"],
                              GS["lapu_values"], O.G_TAUMODE, O.TAU_MEDIAN)
    np.testing.assert_allclose(E, GS["energy_E"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(G, GS["energy_G"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(lam, GS["energy_lambda"], rtol=1e-12, atol=1e-15)
    assert lam[3] == 0.0  # zero-vector path (taumode.rs:268-274)


def _csr(Ld):
    Ld = np.array(Ld, np.float64)
    ip, ix, iv = [0], [], []
    for i in range(Ld.shape[0]):
        for j in range(Ld.shape[1]):
            if Ld[i, j] != 0:
                ix.append(j)
                iv.append(Ld[i, j])
        ip.append(len(ix))
    return np.array(ip, np.int64), np.array(ix, np.int32), np.array(iv)


@pytest.mark.parametrize("case", KA["rayleigh"], ids=lambda c: c["cite"])
def test_rayleigh_known_answers(case):
    ip, ix, iv = _csr(case["L_dense"])
    X = np.array(case["x"], np.float32)
    E, G, lam = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, O.TAU_MEDIAN)
    assert np.all(np.abs(E - np.array(case["expect_E"])) < case["tol"])
    spec = O.spectral_lambdas(X, ip, ix, iv.astype(np.float32))
    if case.get("expect_lambda0_zero"):
        assert abs(spec[0]) < case["tol"]
    if case.get("expect_lambda1_gt_lambda0"):
        assert spec[1] > spec[0]


def test_dispersion_constant_rows_known_answer():
    c = KA["dispersion_constant_rows"]
    ip, ix, iv = _csr(c["L_dense"])
    X = np.array(c["x"], np.float32)
    E, G, _ = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, O.TAU_MEDIAN)
    assert np.all(np.abs(G) < c["tol"])
    # spectral lambda = R + D; the reference asserts the Dirichlet part D == 0
    spec = O.spectral_lambdas(X, ip, ix, iv.astype(np.float32))
    assert np.all(np.abs(spec - E) < c["tol"])


def test_energymaps_dispersion_is_twice_taumode_shares_relation():
    # upper-triangle G uses half the pairs; on a symmetric L the
    # ordered-pair total S is 2x the upper total, each share halves => G_tau = G_em / 2.
    X = GS["energy_X"]
    args = (GS["lapu_indptr"], GS["lapu_indices"], GS["lapu_values"])
    _, Gt, _ = O.energy_rows(X, *args, O.G_TAUMODE, O.TAU_MEDIAN)
    _, Ge, _ = O.energy_rows(X, *args, O.G_ENERGYMAPS, O.TAU_MEDIAN)
    nz = Gt > 0
    np.testing.assert_allclose(Ge[nz], 2.0 * Gt[nz], rtol=1e-9)


def test_sorted_index_known_answer_and_restatement():
    c = KA["sorted_index_ascending"]
    order, keys, std = O.sorted_index(np.array(c["lambda"]))
    assert order.tolist() == c["expect_order"]
    order, keys, _ = O.sorted_index(GS["sort_lambda"])
    np.testing.assert_array_equal(order, GS["sort_order"])


def test_normalise_known_answer():
    c = KA["normalise_lambdas"]
    lam, mn, mx, rg = O.normalise_lambdas(c["lambda"])
    np.testing.assert_allclose(lam, c["expect"], rtol=0, atol=1e-15)
    assert mx == 0.0 and mn == -3.0


def test_sfgrass_known_answers_and_restatement():
    c = KA["sfgrass_basic"]
    rows = c["rows"]
    ip = np.cumsum([0] + [len(r) for r in rows])
    ix = np.array([j for r in rows for j, _ in r])
    w = np.array([x for r in rows for _, x in r])
    oi, oj, ow = O.sfgrass(ip, ix, w)
    assert len(oi) - 1 == 3 and all(oi[i + 1] > oi[i] for i in range(3))
    oi, oj, ow = O.sfgrass(GS["sf_in_indptr"], GS["sf_in_indices"], GS["sf_in_w"])
    np.testing.assert_array_equal(oi, GS["sf_out_indptr"])
    np.testing.assert_array_equal(oj, GS["sf_out_indices"])
    np.testing.assert_array_equal(ow, GS["sf_out_w"])
    assert oi[-1] < GS["sf_in_indptr"][-1]


def test_laplacian_max_properties():
    X = GS["l2_uniform_X"]
    idx, dist = O.knn_l2sq(X, 5)
    n, k = idx.shape
    w = (1.0 / (1.0 + dist)).astype(np.float32)
    src = np.repeat(np.arange(n), k)
    ip, ix, iv, deg, nnz_ref = O.laplacian_max(n, src, idx.ravel(), w.ravel(), normalize=True)
    L = np.zeros((n, n))
    for i in range(n):
        L[i, ix[ip[i]:ip[i + 1]]] = iv[ip[i]:ip[i + 1]]
    assert np.allclose(L, L.T)
    assert np.allclose(np.diag(L), 1.0)
    assert (L - np.diag(np.diag(L)) <= 0).all()
    # null space: L D^{1/2} 1 = 0 (surfface-core tests/test_laplacian.rs invariants)
    assert np.abs(L @ np.sqrt(deg.astype(np.float64))).max() < 1e-5
    ip, ix, iv, deg, _ = O.laplacian_max(n, src, idx.ravel(), w.ravel(), normalize=False)
    L = np.zeros((n, n))
    for i in range(n):
        L[i, ix[ip[i]:ip[i + 1]]] = iv[ip[i]:ip[i + 1]]
    assert np.abs(L.sum(axis=1)).max() < 1e-4


def test_knn_rows_variant_matches_full():
    X = GS["l2_clustered_X"]
    i_all, d_all = O.knn_l2sq(X, 7)
    rows = np.array([5, 0, 35, 17, 17])
    i_r, d_r = O.knn_l2sq_rows(X, 7, rows)
    np.testing.assert_array_equal(i_r, i_all[rows])
    np.testing.assert_array_equal(d_r, d_all[rows])


def test_knn_cos_bf16_rows_matches_widened_f32():
    """The bf16-row oracle (config 5 parity samples) is the f32 oracle on the
    exactly widened values, row for row, bit for bit."""
    X = datagen.uniform(600, 40, seed=3)
    X[5] = 0.0
    X[9] = X[10]
    bits = datagen.to_bf16_bits(X)
    Xf = datagen.bf16_bits_to_f32(bits)
    full = O.knn_cos(Xf, 7, eps=0.9, sigma=0.5)
    rows = np.array([0, 5, 9, 17, 599])
    part = O.knn_cos_bf16_rows(bits, 7, rows, eps=0.9, sigma=0.5)
    for a, b in zip(full, part):
        np.testing.assert_array_equal(a[rows].view(np.uint8), b.view(np.uint8))


def test_lambda_lookups_known_answers():
    """sorted_index.rs:64-140 on a hand-checked 6-item index (binary-exact
    lambdas): keys in OrderedFloat order with string-id ties; range band =
    std / 2^p (std = 0.2357 here); k_nearest grows its window x1.7 from
    base_delta and ranks by |lambda - lq| (ties: index order)."""
    lam = np.array([0.5, 0.125, 0.5, 0.875, 0.25, 0.5])
    order, keys, std = O.sorted_index(lam)
    assert order.tolist() == [1, 4, 0, 2, 5, 3] and abs(std - 0.23570226) < 1e-7
    idx, key = O.range_bylambda(keys, order, std, 0.5, 3, 0.0)      # [0.264, 0.736]
    assert idx.tolist() == [0, 2, 5] and key.tolist() == [0.5, 0.5, 0.5]
    idx, _ = O.range_bylambda(keys, order, std, 0.5, 3, -1.0)       # [0.029, 0.971]
    assert idx.tolist() == [1, 4, 0]
    r = O.range_bylambda(keys, order, std, float("nan"), 3, 0.0)   # lo = hi = NaN bucket
    assert r is not None and len(r[0]) == 0
    # windows around 0.3: 0.05 -> 0.085 -> 0.1445 -> 0.24565 holds 5 >= 3 items
    idx, key = O.k_nearest_by_lambda(keys, order, std, 0.3, 3, 1.0, base_delta=0.05)
    assert idx.tolist() == [4, 1, 0] and key.tolist() == [0.25, 0.125, 0.5]
    # 0.25 and 0.5 are both exactly 0.125 from 0.375: index (rank) order
    idx, _ = O.k_nearest_by_lambda(keys, order, std, 0.375, 2, 1.0, base_delta=0.2)
    assert idx.tolist() == [4, 0]
    # window lo > hi (lq far above 1): the reference panics in BTreeMap::range
    assert O.k_nearest_by_lambda(keys, order, std, 5.0, 2, 1.0, base_delta=0.1) is None


def _py_search(X, lam, q, lq, k, alpha):
    """Pure-Python restatement of core.rs:1156-1193 (sequential folds)."""
    def norm(a):
        s = -0.0
        for v in a:
            s = s + v * v
        return math.sqrt(s)
    qn = norm(q)
    out = []
    for i, x in enumerate(X):
        denom = qn * norm(x)
        cs = 0.0
        if denom > 0.0:
            d = -0.0
            for a, b in zip(q, x):
                d = d + a * b
            cs = d / denom
        ls = 1.0 - min(abs(lq - lam[i]), 1.0)
        out.append((i, alpha * cs + (1.0 - alpha) * ls))
    out.sort(key=lambda t: -t[1])  # stable: ties keep ascending i
    return out[:k]


def test_search_lambda_aware_known_answers_and_restatement():
    # ArrowItem::lambda_similarity doctest (core.rs:155-160): a=[1,0] l=.5,
    # b=[1,0] l=.6, alpha=.7 -> .7*1 + .3*(1-.1) = 0.97 (within [0,1])
    X = np.array([[1.0, 0.0]])
    oi, osc, oc = O.search_lambda_aware(X, np.array([0.6]), np.array([[1.0, 0.0]]),
                                        np.array([0.5]), 1, 0.7)
    assert oc[0] == 1 and oi[0, 0] == 0
    assert osc[0, 0] == 0.7 * 1.0 + (1.0 - 0.7) * (1.0 - min(abs(0.5 - 0.6), 1.0))
    # cosine_similarity doctest (core.rs:226-231): orthogonal -> 0; zero vector -> 0
    X = np.array([[0.0, 1.0], [0.0, 0.0], [3.0, 0.0]])
    oi, osc, oc = O.search_lambda_aware(X, np.array([0.5, 0.5, 0.5]), np.array([[1.0, 0.0]]),
                                        np.array([0.5]), 5, 1.0)
    assert oc[0] == 3 and list(oi[0, :3]) == [2, 0, 1] and oi[0, 3] == -1
    assert list(osc[0, :3]) == [1.0, 0.0, 0.0]
    # lambda 0.0 -> the reference's assert_ne! (count -1)
    _, _, oc = O.search_lambda_aware(X, np.zeros(3), np.array([[1.0, 0.0]]), np.array([0.0]),
                                     2, 0.5)
    assert oc[0] == -1
    rng = np.random.default_rng(3)
    X = rng.uniform(-1, 1, (200, 9)).astype(np.float32).astype(np.float64)
    X[17] = X[3]                        # duplicate rows -> exact score ties
    lam = rng.uniform(0, 1, 200)
    lam[17] = lam[3]
    Q = rng.uniform(-1, 1, (4, 9))
    lq = rng.uniform(0.01, 1, 4)
    for alpha in (0.7, 0.1, 1.3):
        oi, osc, oc = O.search_lambda_aware(X, lam, Q, lq, 25, alpha)
        for t in range(4):
            ref = _py_search(X.tolist(), lam.tolist(), Q[t].tolist(), lq[t], 25, alpha)
            assert oc[t] == 25
            assert [i for i, _ in ref] == oi[t].tolist()
            assert [s for _, s in ref] == osc[t].tolist()


def test_search_hybrid_oracle_vs_python():
    # core.rs:1196-1318 restated with its tie policy (ties -> smaller index)
    rng = np.random.default_rng(8)
    X = rng.uniform(-1, 1, (150, 6)).astype(np.float32).astype(np.float64)
    X[40] = X[7] * 2.0                       # cosine 1 with row 7 (high-semantic)
    lam = rng.uniform(0, 1, 150)
    Q = np.stack([X[7], rng.uniform(-1, 1, 6)])
    lq = np.array([0.3, 0.6])
    for alpha in (0.7, 0.0):
        oi, osc, oc = O.search_lambda_aware(X, lam, Q, lq, 12, alpha, hybrid=True)
        for t in range(2):
            ref = _py_search(X.tolist(), lam.tolist(), Q[t].tolist(), lq[t], 12, alpha)
            full = _py_search(X.tolist(), lam.tolist(), Q[t].tolist(), lq[t], 150, 1.0)
            cosv = dict(full)
            u = {i: c for i, c in cosv.items() if c > 0.9999}
            for i, s in ref:
                u.setdefault(i, s)
            best = min(cosv, key=lambda i: (-cosv[i], i))
            u.setdefault(best, cosv[best])
            exp = sorted(u.items(), key=lambda p: (-p[1], p[0]))[:12]
            assert oc[t] == len(exp)
            assert [i for i, _ in exp] == oi[t, :oc[t]].tolist()
            assert [s for _, s in exp] == osc[t, :oc[t]].tolist()


def test_energy_rows_faithful_equals_csr_restatement():
    """The faithful (F^2 CsMat::get) TAUMODE rows equal the CSR-iterating
    restatement bit for bit (absent pairs add +0.0)."""
    rng = np.random.default_rng(3)
    f = 40
    X = rng.standard_normal((300, f)).astype(np.float32)
    X[7] = 0.0
    idx, _, w = O.knn_cos(X.T.copy(), 4, eps=1.0, sigma=1.0, p=2.0)
    ip, ix, iv = O.laplacian_union(idx, np.where(idx >= 0, w, 0.0))
    e1, g1, l1 = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, O.TAU_MEDIAN)
    e2, g2, l2 = O.energy_rows_faithful(X, ip, ix, iv, O.TAU_MEDIAN)
    for a, b in ((e1, e2), (g1, g2), (l1, l2)):
        np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64))


# ---- MST candidate graph (mst.rs:312-412, distance.rs:78-108) -------------

def _bd_python(mi, vi, mj, vj):
    """Independent scalar restatement of bhattacharyya_distance_diagonal
    (distance.rs:78-108) in numpy float32 (math.log of the f32 value, rounded
    to f32: correctly rounded ln)."""
    f32 = np.float32
    eps = f32(1e-10)
    dist = f32(0.0)
    for k in range(len(mi)):
        si = max(f32(vi[k]), eps)
        sj = max(f32(vj[k]), eps)
        ss = f32(si + sj)
        sp = f32(si * sj)
        md = f32(f32(mi[k]) - f32(mj[k]))
        mahal = f32(f32(f32(0.25) * f32(md * md)) / ss)
        r = max(f32(ss / f32(f32(2.0) * np.sqrt(sp))), eps)
        lt = f32(f32(0.25) * f32(math.log(float(r))))
        dist = f32(dist + f32(mahal + lt))
    return dist


def test_bhattacharyya_distance_known_answers():
    """test_distance.rs:9-60: identical distributions -> 0 (asserted < 1e-5),
    different means / variances -> > 0; the exact values follow from the
    formula: means 0 vs 1 at var 1 -> 2 x 0.125; var 0.5 vs 2 -> 2 x ln(1.25)/4."""
    z = O.bhattacharyya_distance([1, 2, 3], [0.5] * 3, [1, 2, 3], [0.5] * 3)
    assert z == np.float32(0.0)
    assert O.bhattacharyya_distance([0, 0], [1, 1], [1, 1], [1, 1]) == np.float32(0.25)
    dv = O.bhattacharyya_distance([0, 0], [0.5, 0.5], [0, 0], [2.0, 2.0])
    t = np.float32(np.float32(0.25) * np.float32(math.log(1.25)))
    assert dv == np.float32(t + t) and dv > 0
    # test_bhattacharyya_slice_vs_tensor (test_distance.rs:62-88): the slice
    # value agrees with the tensor formula (f64 here) within 1e-4
    mi, mj, vi, vj = [1.0, 2.0, 3.0], [1.5, 2.5, 3.5], [0.5] * 3, [0.6] * 3
    # tensor form (distance.rs:28-61): 0.25 md^2/ss + 0.25 ln(ss / (2 sqrt(sp)))
    ref = sum(0.25 * (a - b) ** 2 / (x + y) + 0.25 * math.log((x + y) / (2 * math.sqrt(x * y)))
              for a, b, x, y in zip(mi, mj, vi, vj))
    s = O.bhattacharyya_distance(mi, vi, mj, vj)
    assert abs(float(s) - ref) < 1e-4


def test_bhattacharyya_oracle_vs_python_restatement():
    rng = np.random.default_rng(5)
    for f in (1, 7, 33):
        for _ in range(40):
            mi, mj = rng.normal(size=f).astype(np.float32), rng.normal(size=f).astype(np.float32)
            vi = np.abs(rng.normal(size=f)).astype(np.float32)
            vj = np.abs(rng.normal(size=f)).astype(np.float32)
            vi[rng.random(f) < 0.1] = 0.0  # floored to 1e-10
            a = O.bhattacharyya_distance(mi, vi, mj, vj)
            b = _bd_python(mi, vi, mj, vj)
            # glibc logf vs correctly rounded ln: equal but for rare ulp terms
            assert abs(float(a) - float(b)) <= 4e-6 * max(1.0, abs(float(b)))


def test_mst_candidates_oracle_semantics():
    """mst.rs:312-412 on a small case: stable (dist, j) order, k = min(k, C-1),
    thickness = mean variance (test_thickness_weight_functions' centroids:
    equal means, per-row constant variances), every ThicknessWeight."""
    means = np.ones((4, 3), np.float32)
    var = np.repeat(np.array([[0.5], [1.0], [0.2], [0.8]], np.float32), 3, axis=1)
    th = var.mean(axis=1).astype(np.float32)
    for tw in range(5):
        v, d, cost = O.mst_candidates(means, var, 3, O.MST_BHATTACHARYYA, tw)
        assert v.shape == (4, 3)
        for i in range(4):
            dd = [(_bd_python(means[i], var[i], means[j], var[j]), j) for j in range(4) if j != i]
            dd.sort(key=lambda t: (t[0], t[1]))
            assert list(v[i]) == [j for _, j in dd]
            for r, (dv, j) in enumerate(dd):
                assert abs(float(d[i, r]) - float(dv)) <= 1e-6
                ti, tj = th[i], th[j]
                phi = [np.float32((ti + tj) / np.float32(2)), min(ti, tj), max(ti, tj),
                       np.sqrt(np.float32(ti * tj)), None][tw]
                want = d[i, r] if phi is None else np.float32(d[i, r] * phi)
                assert cost[i, r] == want
    # duplicates tie at distance 0 -> j ascending; k > C-1 truncates
    m2 = np.zeros((5, 2), np.float32)
    v2, d2, _ = O.mst_candidates(m2, np.ones((5, 2), np.float32), 10, O.MST_BHATTACHARYYA, 4)
    assert v2.shape == (5, 4) and (d2 == 0).all()
    assert [list(r) for r in v2] == [[j for j in range(5) if j != i] for i in range(5)]
    # L2 metrics agree with the kNN oracle
    X = datagen.uniform(300, 12, seed=3)
    v3, d3, c3 = O.mst_candidates(X, None, 7, O.MST_SQEUCLIDEAN, 4,
                                  thickness=np.ones(300, np.float32))
    ridx, rdist = O.knn_l2sq(X, 7)
    assert np.array_equal(v3, ridx) and np.array_equal(d3.view(np.uint32), rdist.view(np.uint32))
    v4, d4, _ = O.mst_candidates(X, None, 7, O.MST_EUCLIDEAN, 4,
                                 thickness=np.ones(300, np.float32))
    assert np.array_equal(v4, ridx)
    assert np.array_equal(d4.view(np.uint32), np.sqrt(rdist).view(np.uint32))


def test_nearest_centroid_oracle_known_answers():
    """stages/clustering.rs:42-63 on exact small integers: d = sqrt(|x|^2 +
    |c|^2 - 2 x.c); ties take the first centroid."""
    cents = np.array([[0, 0], [3, 4], [0, 0]], np.float32)
    batch = np.array([[0, 0], [3, 4], [1, 0], [6, 8]], np.float32)
    idx, dist = O.nearest_centroid(batch, cents)
    assert idx.tolist() == [0, 1, 0, 1]
    assert dist.tolist() == [0.0, 0.0, 1.0, 5.0]


def test_glibc_logf_expf_restatement():
    """The kernels' f32 ln / exp (csrc/glibc_f32.hpp) restate the platform
    glibc logf / expf the reference's f32::ln / f32::exp call.  CPU checks:
    (1) the restatement's tables are the bytes of the host libm's
    e_logf_data / e_exp2f_data (re-derived from the binary), (2) the device
    header holds the same literals, (3) the host copy of the algorithm equals
    the host glibc on every 61st f32 bit pattern (a stride-1 run over all
    2^32 inputs: 0 mismatches; the device code is checked exhaustively by
    tests/test_libm_gpu.py)."""
    import re
    import struct
    lg, ex = O.glibc_tables_from_libm()
    assert lg is not None
    np.testing.assert_array_equal(lg, O.glibc_tables(0))
    np.testing.assert_array_equal(ex, O.glibc_tables(1))
    hdr = open(os.path.join(ROOT, "matternet-rs_amd", "csrc", "glibc_f32.hpp")).read()
    body = hdr[hdr.index("kLogT"):hdr.index("// glibc logf")]
    lits = re.findall(r"-?0x[0-9a-f]+\.?[0-9a-f]*p[+-]\d+|0x[0-9a-f]{16}", body)
    vals = []
    for t in lits:
        if "p" in t:
            vals.append(struct.unpack("<Q", struct.pack("<d", float.fromhex(t)))[0])
        else:
            vals.append(int(t, 16))
    # header order: log table (32), A0 A1 A2, Ln2, exp table (32), C0 C1 C2, InvLn2N, Shift
    np.testing.assert_array_equal(np.array(vals[:36], np.uint64), O.glibc_tables(0))
    np.testing.assert_array_equal(np.array(vals[36:], np.uint64), O.glibc_tables(1))
    assert O.glibc_restated_check(0, 61) == 0
    assert O.glibc_restated_check(1, 61) == 0


def test_glibc_pow_restatement_host():
    """The kernels' f64 pow (csrc/glibc_f64.hpp: glibc's pow restated with the
    host libm's own tables) against the host pow: random and structured (x, p)
    — the weight kernel's (d / sigma)^p for p in {0.5, 2, 3, 2.7, ...}, wide x
    and y, subnormal / overflowing results, negative x with integer y, the
    special values — bit for bit (tests/native/pow_check.cpp, built with g++)."""
    import shutil
    import subprocess
    import tempfile
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not installed")
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "pow_check")
        subprocess.run([gxx, "-O2", "-std=c++17", "-mfma", "-ffp-contract=off",
                        "-I", os.path.join(ROOT, "tests", "native", "stub"),
                        "-I", os.path.join(ROOT, "matternet-rs_amd", "csrc"),
                        os.path.join(ROOT, "tests", "native", "pow_check.cpp"), "-o", exe],
                       check=True, capture_output=True)
        r = subprocess.run([exe, "1000000"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr



# a query whose band edge reaches the key 0.75 under exp2(p) but not under
# glibc pow(2, p) (the two differ in ~0.1 % of fractional p), index [0.25, 0.75]
EXP2_EDGE = {"lam": [0.25, 0.75], "p": 0.8158310053062214, "lq": 0.6079797068751175}


def test_range_band_uses_exp2_like_an_optimised_reference_build():
    """sorted_index.rs:65 `std / 2.0_f64.powf(p)`: LLVM's library-call
    simplifier rewrites llvm.pow(2.0, p) to exp2(p) in an optimised build
    (replacePowWithExp; no fast-math flag needed), so the band is
    std / exp2(p).  At this query only that band reaches the 0.75 key."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    for fn in (libm.exp2, libm.pow):
        fn.restype = ctypes.c_double
    libm.exp2.argtypes = [ctypes.c_double]
    libm.pow.argtypes = [ctypes.c_double, ctypes.c_double]
    e = EXP2_EDGE
    order, keys, std = O.sorted_index(np.array(e["lam"]))
    assert std == 0.25
    assert e["lq"] + std / libm.exp2(e["p"]) >= 0.75 > e["lq"] + std / libm.pow(2.0, e["p"])
    idx, key = O.range_bylambda(keys, order, std, e["lq"], 4, e["p"])
    assert idx.tolist() == [1] and key.tolist() == [0.75]
