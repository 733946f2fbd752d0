"""Legacy GraphParams-driven Laplacian build on the GPU (surfface_hip.graph)
vs the oracle pipeline on the same inputs:

  oracle: or_knn_cos_f64 / _f64d (rows = nodes, test_helpers.rs:77-126 brute
  force, topk nearest other nodes) -> inline sparsification restated here
  (laplacian.rs:216-282) -> or_laplacian_union (laplacian.rs:297-419).

Bit-exact CSR (structure and f64 values) for f32 and f64 items, for the
"Laplacian of Laplacian" signals graph (graph.rs:257-313), and through
EigenMaps.compute_taumode (lambdas within 1e-9 relative, like K3)."""
import math

import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _inline(idx, w, deg=None):
    """laplacian.rs:216-282 on the eps-filtered rows: deg = the eps-valid
    neighbour counts (default: the row lengths, equal when no weight is
    filtered), sparsify iff avg > 10, rows with len > 2 keep max(len/2, 1) by
    w * sqrt(deg_i deg_j) desc (ties: input position)."""
    n, k = idx.shape
    if deg is None:
        deg = (idx >= 0).sum(1)
    if not deg.sum() / n > 10.0:
        return idx, w
    oi = np.full_like(idx, -1)
    ow = np.zeros_like(w)
    for i in range(n):
        row = [(int(idx[i, r]), float(w[i, r]), r) for r in range(k) if idx[i, r] >= 0]
        if len(row) > 2:
            sc = sorted(((wt * math.sqrt(float(deg[i] * deg[j])), p, j, wt) for j, wt, p in row),
                        key=lambda t: (-t[0], t[1]))
            row = [(j, wt, p) for _, p, j, wt in sc[:max(len(row) // 2, 1)]]
        for r, (j, wt, _) in enumerate(row):
            oi[i, r] = j
            ow[i, r] = wt
    return oi, ow


def _oracle_graph(items, topk, eps, sigma, p):
    items = np.asarray(items)
    knn = O.knn_cos_f64 if items.dtype == np.float64 else O.knn_cos
    idx, _, w = knn(items, topk, eps, sigma, p)
    # laplacian.rs:219-229: degrees count the eps-valid neighbours before the
    # weight filter (:255-258): the same query with a weight that never drops
    i2, _, _ = knn(items, topk, eps, 1.0, 1.0)
    oi, ow = _inline(idx, w, (i2 >= 0).sum(1))
    return O.laplacian_union(oi, ow)


def _csr_equal(L, ref, rtol=0.0):
    ip, ix, iv = L.to_numpy()
    rip, rix, riv = ref
    np.testing.assert_array_equal(ip, rip)
    np.testing.assert_array_equal(ix, rix)
    if rtol == 0.0:
        np.testing.assert_array_equal(iv.view(np.uint64), riv.view(np.uint64))
    else:
        np.testing.assert_allclose(iv, riv, rtol=rtol, atol=0.0)


@pytest.mark.parametrize("topk,eps", [(3, 1.0), (16, 1.0), (6, 0.3)])
def test_k_cluster_f32_centroids(topk, eps):
    """GraphFactory::build_laplacian_matrix_from_k_cluster (graph.rs:193-249):
    X x F centroids -> the F x F feature Laplacian (nodes = feature columns)."""
    import surfface_hip as S
    C = datagen.clustered(400, 96, seed=topk, blobs=5, dup_frac=0.02, zero_frac=0.0)
    gl = S.GraphFactory.build_laplacian_matrix_from_k_cluster(
        torch.from_numpy(C).cuda(), eps, 6, topk, 2.0, None, False, False, 10_000)
    assert gl.nnodes == 10_000 and gl.shape == (96, 96)
    _csr_equal(gl.matrix, _oracle_graph(C.T.copy(), topk, eps, 1.0, 2.0))


def test_f64_items_and_sigma_p():
    """build_laplacian_matrix on f64 items not representable in f32, with an
    explicit sigma and p (laplacian.rs:256): the device pow is glibc's
    restated (glibc_f64.hpp), so p = 1.5 and p = 2 (the default) are both
    bit-exact against the oracle's host pow."""
    import surfface_hip as S
    rng = np.random.default_rng(4)
    T = rng.normal(size=(70, 500)) + 0.3  # rows = nodes
    params = S.GraphParams(eps=0.9, k=6, topk=12, p=1.5, sigma=0.4)
    gl = S.build_laplacian_matrix(torch.from_numpy(T).cuda(), params)
    assert gl.nnodes == 500  # laplacian.rs:129,165-168: n = the column count of `transposed`
    _csr_equal(gl.matrix, _oracle_graph(T, 12, 0.9, 0.4, 1.5))  # glibc pow restated: bit-exact
    params2 = S.GraphParams(eps=0.9, k=6, topk=12, p=2.0, sigma=0.4)
    gl2 = S.build_laplacian_matrix(torch.from_numpy(T).cuda(), params2)
    _csr_equal(gl2.matrix, _oracle_graph(T, 12, 0.9, 0.4, 2.0))


def test_inline_degree_counts_eps_valid_before_the_weight_filter():
    """laplacian.rs:219-229 counts a node's neighbours with dist <= eps, before
    the weight > 1e-12 filter of :255-258.  sigma = 1e-7, p = 2 drops every
    edge with d >= 0.1: 7 groups of 10 near-identical nodes keep 9 weighted
    edges each (row length 9, avg < 10) while every node has 16 eps-valid
    neighbours (avg 16 > 10), so the reference prunes and a row-length
    degree rule would not."""
    import surfface_hip as S
    rng = np.random.default_rng(12)
    base = rng.normal(size=(7, 400))
    T = np.repeat(base, 10, axis=0) + 0.02 * rng.normal(size=(70, 400))
    params = S.GraphParams(eps=1.0, k=6, topk=16, p=2.0, sigma=1e-7)
    gl = S.build_laplacian_matrix(torch.from_numpy(T).cuda(), params)
    ref = _oracle_graph(T, 16, 1.0, 1e-7, 2.0)
    _csr_equal(gl.matrix, ref)
    # pruned: 4 = max(9 // 2, 1) kept per row before symmetrisation, so fewer
    # than the 9 + 1 entries per row of the unpruned groups
    assert gl.matrix.nnz < 70 * 10
    idx, _, w = O.knn_cos_f64(T, 16, 1.0, 1e-7, 2.0)
    assert ((idx >= 0).sum(1) == 9).all()


def test_spectral_signals_laplacian_of_laplacian():
    """build_spectral_laplacian (graph.rs:257-313) on the densified F x F
    Laplacian, then EigenMaps.compute_taumode prefers the signals
    (taumode.rs:138-145)."""
    import surfface_hip as S
    C = datagen.clustered(300, 64, seed=2, blobs=4, dup_frac=0.0, zero_frac=0.0)
    b = S.BuilderParams(lambda_eps=1.0, lambda_k=12, lambda_topk=8, prebuilt_spectral=True)
    res = S.EigenMaps.eigenmaps(b, torch.from_numpy(C).cuda(), 5000)
    ref_L = _oracle_graph(C.T.copy(), 8, 1.0, 1.0, 2.0)
    _csr_equal(res.gl.matrix, ref_L)
    dense = np.zeros((64, 64))
    for i in range(64):
        dense[i, ref_L[1][ref_L[0][i]:ref_L[0][i + 1]]] = ref_L[2][ref_L[0][i]:ref_L[0][i + 1]]
    ref_sig = _oracle_graph(dense, 8, 1.0, 1.0, 2.0)
    _csr_equal(res.signals, ref_sig)
    items = datagen.uniform(2000, 64, seed=9)
    lam = S.EigenMaps.compute_taumode(torch.from_numpy(items).cuda(), res, S.TauMode.Median)
    _, _, rl = O.energy_rows(items, *ref_sig, O.G_TAUMODE, O.TAU_MEDIAN)
    rn, _, _, _ = O.normalise_lambdas(rl)
    np.testing.assert_allclose(lam.cpu().numpy(), rn, rtol=1e-9, atol=1e-12)


def test_eigenmaps_without_signals_uses_the_laplacian():
    import surfface_hip as S
    C = datagen.clustered(200, 48, seed=5, blobs=3, dup_frac=0.0, zero_frac=0.0)
    b = S.BuilderParams(lambda_eps=1.0, lambda_k=4).define_result_k()
    assert b.lambda_topk == 3
    assert S.BuilderParams(lambda_k=7).define_result_k().lambda_topk == 4
    assert S.BuilderParams(lambda_k=12, lambda_topk=9).define_result_k().lambda_topk == 9
    res = S.EigenMaps.eigenmaps(b, torch.from_numpy(C).cuda(), 1000)
    assert res.signals is None
    items = datagen.uniform(500, 48, seed=1)
    lam = S.EigenMaps.compute_taumode(torch.from_numpy(items).cuda(), res)
    ref = _oracle_graph(C.T.copy(), 3, 1.0, 1.0, 2.0)
    _, _, rl = O.energy_rows(items, *ref, O.G_TAUMODE, O.TAU_MEDIAN)
    rn, _, _, _ = O.normalise_lambdas(rl)
    np.testing.assert_allclose(lam.cpu().numpy(), rn, rtol=1e-9, atol=1e-12)


def test_sparsity_check_panics():
    """graph.rs:230-238: sparsity > 0.95 with sparsity_check -> panic."""
    import surfface_hip as S
    C = datagen.uniform(100, 64, seed=3)
    with pytest.raises(S.SparsityError):
        S.GraphFactory.build_laplacian_matrix_from_k_cluster(
            torch.from_numpy(C).cuda(), 1e-6, 6, 3, 2.0, None, False, True, 100)
    gl = S.GraphFactory.build_laplacian_matrix_from_k_cluster(
        torch.from_numpy(C).cuda(), 1e-6, 6, 3, 2.0, None, False, False, 100)
    assert S.GraphLaplacian.sparsity(gl.matrix) > 0.95


def test_normalise_standardizes_then_builds():
    """normalise = true (laplacian.rs:143-150): the StandardScaler pass
    (smartcore absent: parity-unpinned; checked against numpy's population
    statistics to 1e-12) followed by the same graph build, bit-exact given the
    standardised items."""
    import surfface_hip as S
    rng = np.random.default_rng(6)
    T = rng.normal(size=(50, 300)) * 3.0 + 1.0
    params = S.GraphParams(eps=1.0, k=6, topk=5, normalise=True)
    gl = S.build_laplacian_matrix(torch.from_numpy(T).cuda(), params)
    Z = gl.init_data.cpu().numpy()
    want = (T - T.mean(axis=0)) / T.std(axis=0)
    np.testing.assert_allclose(Z, want, rtol=1e-12, atol=1e-12)
    _csr_equal(gl.matrix, _oracle_graph(Z, 5, 1.0, 1.0, 2.0))


def test_shape_assert():
    import surfface_hip as S
    with pytest.raises(ValueError):
        S.build_laplacian_matrix(torch.zeros((1, 5), device="cuda"), S.GraphParams())
