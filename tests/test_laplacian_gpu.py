"""K2 parity on the GPU: HIP Laplacian assembly (C ABI) vs the CPU oracle.

UNION / legacy (f64): CSR structure AND values bit-exact (the reference's
degree is a sequential ascending-column sum, reproduced exactly).
MAX / Stage C (f32): structure exact; values and degrees within 1e-5
relative (the reference sums degrees in DashMap iteration order).
"""
import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GS = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                        "golden_small.npz"))


def lap(idx, val, **kw):
    import surfface_hip as S
    m, deg = S.build_laplacian_from_knn(torch.from_numpy(np.ascontiguousarray(idx)).cuda(),
                                        torch.from_numpy(np.ascontiguousarray(val)).cuda(), **kw)
    return m.to_numpy() + (deg.cpu().numpy(),)


def host_pow(x, p):
    """The reference's f64::powf = the host glibc pow (oracle or_pow_f64: numpy's
    power may use a vector math library, or sqrt / square for scalar exponents)."""
    return O.pow_f64(x, p)


def rational_weights(dist, eps, sigma, p):
    d = dist.astype(np.float64)
    w = 1.0 / (1.0 + host_pow(d / sigma, p))
    valid = (d <= eps) & (w > 1e-12)
    return np.where(valid, w, 0.0), valid


def test_union_golden_cosine_graph():
    ip, ix, iv, deg = lap(GS["cos_idx"], GS["cos_w"], weight_kernel="given")
    np.testing.assert_array_equal(ip, GS["lapu_indptr"])
    np.testing.assert_array_equal(ix, GS["lapu_indices"])
    np.testing.assert_array_equal(iv.view(np.uint64), GS["lapu_values"].view(np.uint64))


@pytest.mark.parametrize("n,d,k", [(5000, 32, 10), (20000, 64, 32)])
def test_union_from_l2_knn_rational_kernel(n, d, k):
    X = datagen.uniform(n, d, seed=3)
    idx, dist = O.knn_l2sq(X, k)
    eps, sigma = 1e30, 4.0
    ip, ix, iv, deg = lap(idx, dist, weight_kernel="rational", eps=eps, sigma=sigma, p=2.0)
    w, valid = rational_weights(dist, eps, sigma, 2.0)
    ridx = np.where(valid, idx, -1).astype(np.int32)
    rip, rix, riv = O.laplacian_union(ridx, w)
    np.testing.assert_array_equal(ip, rip)
    np.testing.assert_array_equal(ix, rix)
    np.testing.assert_array_equal(iv.view(np.uint64), riv.view(np.uint64))
    # degrees == diagonal, rows sum to zero (reference invariant)
    diag = np.array([iv[ip[i]:ip[i + 1]][ix[ip[i]:ip[i + 1]] == i][0] for i in range(0, n, 97)])
    np.testing.assert_array_equal(diag, deg[::97])


def test_union_eps_filter_and_hub_rows():
    import surfface_hip as S
    n, k = 12000, 4
    rng = np.random.default_rng(0)
    idx = rng.integers(0, n, size=(n, k)).astype(np.int32)
    idx[:, 0] = 0        # node 0 is everybody's neighbour: in-degree ~ n (one block's LDS sort)
    idx[:700, 1] = 1     # node 1: in-degree ~ 500 valid (the 16-keys-a-lane wave sort)
    idx[5, 2] = 5        # self loop dropped
    idx[7, 3] = -1       # empty slot
    dist = rng.uniform(0, 2.0, size=(n, k)).astype(np.float64)
    ip, ix, iv, deg = lap(idx, dist, weight_kernel="rational", eps=1.5, sigma=0.7, p=3.0)
    st = S.laplacian.last_stats()
    # rows past the one-wave sort (> 256 entries); hub rows (> 16384: the HBM
    # network) are covered by test_large_hub_rows_device_sort
    assert st["big_rows"] >= 2
    d = dist
    w = 1.0 / (1.0 + host_pow(d / 0.7, 3.0))
    valid = (d <= 1.5) & (w > 1e-12) & (idx >= 0)
    rip, rix, riv = O.laplacian_union(np.where(valid, idx, -1).astype(np.int32), w)
    np.testing.assert_array_equal(ip, rip)
    np.testing.assert_array_equal(ix, rix)
    # the device pow is glibc's restated (glibc_f64.hpp): bit-exact
    np.testing.assert_array_equal(iv.view(np.uint64), riv.view(np.uint64))


@pytest.mark.parametrize("p", [0.5, 3.0, 2.7, 1.0, 2.0])
def test_rational_kernel_exponents_bit_exact(p):
    """laplacian.rs:256 `1 / (1 + (d / sigma).powf(p))` for p in {0.5, 3, 2.7}
    (and the shortcut-prone 1, 2): the weights and the assembled Laplacian bit
    for bit against the oracle with the host glibc pow."""
    n, k = 20000, 16
    rng = np.random.default_rng(int(p * 10))
    idx = rng.integers(0, n, size=(n, k)).astype(np.int32)
    dist = rng.uniform(0, 3.0, size=(n, k)).astype(np.float64)
    ip, ix, iv, deg = lap(idx, dist, weight_kernel="rational", eps=2.5, sigma=0.9, p=p)
    w, valid = rational_weights(dist, 2.5, 0.9, p)
    valid &= idx != np.arange(n)[:, None]
    rip, rix, riv = O.laplacian_union(np.where(valid, idx, -1).astype(np.int32), w)
    np.testing.assert_array_equal(ip, rip)
    np.testing.assert_array_equal(ix, rix)
    np.testing.assert_array_equal(iv.view(np.uint64), riv.view(np.uint64))


@pytest.mark.parametrize("sym", ["union", "max"])
def test_large_hub_rows_device_sort(sym):
    """Hub rows far beyond one LDS chunk (P = 65536: global flip + half-cleaner
    steps and chunk passes) with duplicate columns (max weight kept)."""
    import surfface_hip as S
    n, k = 50000, 4
    rng = np.random.default_rng(11)
    idx = rng.integers(0, n, size=(n, k)).astype(np.int32)
    idx[:, 0] = 0                       # node 0: in-degree n -> m ~ 50k
    idx[: n // 2, 1] = 3                # node 3: ~25k
    idx[::3, 2] = idx[::3, 3]           # duplicate columns within rows
    w = rng.uniform(0.01, 1.0, size=(n, k)).astype(np.float64 if sym == "union" else np.float32)
    if sym == "union":
        ip, ix, iv, deg = lap(idx, w, weight_kernel="given")
        rip, rix, riv = O.laplacian_union(idx, w.astype(np.float64))
        np.testing.assert_array_equal(ip, rip)
        np.testing.assert_array_equal(ix, rix)
        np.testing.assert_array_equal(iv.view(np.uint64), riv.view(np.uint64))
    else:
        ip, ix, iv, deg = lap(idx, w, weight_kernel="given", symmetrise="max",
                              weight_threshold=1e-9)
        src = np.repeat(np.arange(n), k)
        rip, rix, riv, rdeg, _ = O.laplacian_max(n, src, idx.ravel(), w.ravel(), thr=1e-9,
                                                 normalize=False)
        np.testing.assert_array_equal(ip, rip)
        np.testing.assert_array_equal(ix, rix)
        np.testing.assert_allclose(iv, riv, rtol=1e-5, atol=1e-7)
    assert S.laplacian.last_stats()["hub_rows"] >= 2


@pytest.mark.parametrize("normalize", [True, False])
def test_max_variant_vs_oracle(normalize):
    X = datagen.clustered(3000, 24, seed=7, blobs=6)
    idx, dist = O.knn_l2sq(X, 15)
    w = (1.0 / (1.0 + dist.astype(np.float64))).astype(np.float32)
    w[::17, 3] = 1e-10   # below the weight threshold: dropped
    ip, ix, iv, deg = lap(idx, w, weight_kernel="given", symmetrise="max", normalize=normalize,
                          weight_threshold=1e-9)
    n, k = idx.shape
    src = np.repeat(np.arange(n), k)
    rip, rix, riv, rdeg, _ = O.laplacian_max(n, src, idx.ravel(), w.ravel(), thr=1e-9,
                                             normalize=normalize)
    np.testing.assert_array_equal(ip, rip)
    np.testing.assert_array_equal(ix, rix)
    np.testing.assert_allclose(iv, riv, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(deg, rdeg, rtol=1e-5)


@pytest.mark.parametrize("normalize", [True, False])
def test_stage_nnz_counts_before_the_filter(normalize):
    """LaplacianOutput.nnz is the reference's counter taken while the dense L
    is written (surfface-core/src/laplacian.rs:344-391), BEFORE the |v| > 1e-9
    filter of the CSR conversion (:215); sparsity = 1 - nnz/F^2 in f32 (:187).
    Normalized mode: tiny weights (> thr) on high-degree nodes give
    |w / sqrt(d_i d_j)| <= 1e-9, dropped from the CSR but counted."""
    import surfface_hip as S
    X = datagen.uniform(600, 16, seed=3)
    idx, dist = O.knn_l2sq(X, 15)
    w = (1.0 / (1.0 + dist.astype(np.float64))).astype(np.float32) * np.float32(8.0)
    w[::5, 7] = np.float32(2e-9)     # > thr, but |v| <= 1e-9 once normalized
    w[::23, 2] = np.float32(5e-10)   # <= thr: not an edge at all
    out = S.laplacian_stage_from_edges(torch.from_numpy(idx).cuda(), torch.from_numpy(w).cuda(),
                                       S.LaplacianConfig(k_neighbors=15, normalize=normalize))
    n, k = idx.shape
    src = np.repeat(np.arange(n), k)
    rip, rix, riv, rdeg, nnz_ref = O.laplacian_max(n, src, idx.ravel(), w.ravel(), thr=1e-9,
                                                   normalize=normalize)
    assert out.nnz == nnz_ref
    if normalize:
        assert out.nnz > out.matrix.nnz  # filtered entries still counted
    sp = np.float32(1.0) - np.float32(np.float32(nnz_ref) / np.float32(n * n))
    assert np.float32(out.sparsity) == sp


def test_laplacian_stage_output_properties():
    import surfface_hip as S
    X = datagen.uniform(800, 16, seed=2)
    idx, dist = O.knn_l2sq(X, 15)
    w = torch.from_numpy((1.0 / (1.0 + dist)).astype(np.float32)).cuda()
    out = S.laplacian_stage_from_edges(torch.from_numpy(idx).cuda(), w,
                                       S.LaplacianConfig(k_neighbors=15))
    L = out.matrix.to_dense().astype(np.float64)
    assert np.allclose(L, L.T, atol=1e-6)
    assert np.allclose(np.diag(L), 1.0)
    off = L - np.diag(np.diag(L))
    assert (off <= 0).all()
    assert out.nnz <= 800 * (2 * 15 + 1)
    # null space L D^{1/2} 1 = 0 (surfface-core tests/test_laplacian.rs invariant)
    assert np.abs(L @ np.sqrt(out.degrees.cpu().numpy().astype(np.float64))).max() < 1e-4


def test_library_owned_output_and_capacity_error():
    """The C ABI's two output modes: library-allocated CSR (mn_csr_free) and
    caller-owned buffers; a too-small caller capacity is MN_ECAP with nnz =
    the entries needed."""
    import ctypes as C
    import surfface_hip as S
    from surfface_hip import _lib
    from surfface_hip._torch import ptr
    X = datagen.uniform(3000, 16, seed=2)
    idx, dist = O.knn_l2sq(X, 8)
    ref = S.build_laplacian_from_knn(torch.from_numpy(idx).cuda(), torch.from_numpy(dist).cuda(),
                                     eps=1e30, sigma=2.0)[0].to_numpy()
    L = _lib.lib()
    di, dd = torch.from_numpy(idx).cuda(), torch.from_numpy(dist).cuda()
    o = _lib.LapOpts(weight_kernel=_lib.MN_W_RATIONAL, symmetrise=_lib.MN_SYM_UNION, normalize=0,
                     reserved0=0, eps=1e30, sigma=2.0, p=2.0, weight_threshold=1e-9, stream=None)
    csr = _lib.Csr()
    _lib.check(L.mn_laplacian_from_knn(ptr(di), ptr(dd), 0, 3000, 8, C.byref(o), C.byref(csr),
                                       None))
    assert csr.caller_owned == 0 and csr.nnz == len(ref[1])
    ip = torch.empty(3001, dtype=torch.int64, device="cuda")
    ix = torch.empty(csr.nnz, dtype=torch.int32, device="cuda")
    iv = torch.empty(csr.nnz, dtype=torch.float64, device="cuda")
    for dst, src, nb in ((ip, csr.indptr, 8 * 3001), (ix, csr.indices, 4 * csr.nnz),
                         (iv, csr.values, 8 * csr.nnz)):
        _lib.check(L.mn_memcpy_d2d(ptr(dst), src, nb, None))
    _lib.check(L.mn_csr_free(C.byref(csr)))
    np.testing.assert_array_equal(ip.cpu().numpy(), ref[0])
    np.testing.assert_array_equal(ix.cpu().numpy(), ref[1])
    np.testing.assert_array_equal(iv.cpu().numpy().view(np.uint64), ref[2].view(np.uint64))
    small = _lib.Csr(n_rows=3000, n_cols=3000, nnz=100, indptr=ptr(ip).value,
                     indices=ptr(ix).value, values=ptr(iv).value, value_type=_lib.MN_F64,
                     caller_owned=1)
    rc = L.mn_laplacian_from_knn(ptr(di), ptr(dd), 0, 3000, 8, C.byref(o), C.byref(small), None)
    assert rc == -4 and small.nnz == len(ref[1])


def _centroids(c, f, seed, group=5):
    """[C, F] centroid means / variances in the spirit of the surfface-core
    tests' centroids_from_gaussian_blobs (test_laplacian.rs:257-275): feature
    columns come in groups of near-identical profiles (so Bhattacharyya
    coefficients span (0, 1] and the top-k are meaningful), U(0.05, 0.3)
    variances, some below the variance floor."""
    rng = np.random.default_rng(seed)
    base = rng.uniform(-1, 1, size=(c, (f + group - 1) // group))
    means = (base[:, np.arange(f) // group] + rng.normal(0, 0.05, size=(c, f))).astype(np.float32)
    var = rng.uniform(0.05, 0.3, size=(c, f)).astype(np.float32)
    var[:, ::17] = 0.0  # below the variance floor: max(var, reg)
    return means, var


@pytest.mark.parametrize("c,f,k", [(64, 200, 15), (300, 129, 8), (7, 70, 69)])
def test_bhattacharyya_stage_c_knn_vs_oracle(c, f, k):
    """compute_bhattacharyya_weights (laplacian.rs:254-298): neighbour lists
    and weights bit-exact (the device ln / exp are glibc's logf / expf
    restated, csrc/glibc_f32.hpp; ties by ascending j)."""
    import surfface_hip as S
    means, var = _centroids(c, f, seed=c + f)
    cfg = S.LaplacianConfig(k_neighbors=k)
    gi, gw = S.compute_bhattacharyya_weights(torch.from_numpy(means).cuda(),
                                             torch.from_numpy(var).cuda(), cfg)
    gi, gw = gi.cpu().numpy(), gw.cpu().numpy()
    ri, rw = O.bc_knn(means, var, k)
    assert (ri >= 0).mean() > 0.2  # a real neighbourhood, not an empty graph
    np.testing.assert_array_equal(gi, ri)
    np.testing.assert_array_equal(gw.view(np.uint32), rw.view(np.uint32))


def test_laplacian_stage_execute_end_to_end():
    """LaplacianStage::execute (laplacian.rs:135-228) on the GPU: BC kNN ->
    MAX symmetrisation -> L_sym; invariants of surfface-core tests/test_laplacian.rs
    (symmetric, unit diagonal, off-diagonals <= 0, nnz <= F(2k+1))."""
    import surfface_hip as S
    means, var = _centroids(96, 150, seed=5)
    out = S.LaplacianStage(S.LaplacianConfig(k_neighbors=10)).execute(
        torch.from_numpy(means).cuda(), torch.from_numpy(var).cuda())
    L = out.matrix.to_dense().astype(np.float64)
    assert np.allclose(L, L.T, atol=1e-6)
    deg = out.degrees.cpu().numpy()
    # unit diagonal where the node has edges (L_ii = 1 iff d_i > thr, laplacian.rs:355-365);
    # the floored-variance features (every 17th) are isolated
    assert np.allclose(np.diag(L)[deg > 1e-9], 1.0) and (np.diag(L)[deg <= 1e-9] == 0).all()
    assert (deg[::17] <= 1e-9).all() and (deg > 1e-9).mean() > 0.9
    assert (L - np.diag(np.diag(L)) <= 0).all()
    assert out.nnz <= 150 * (2 * 10 + 1)
    ri, rw = O.bc_knn(means, var, 10)
    src = np.repeat(np.arange(150), 10)
    rip, rix, riv, rdeg, _ = O.laplacian_max(150, src, ri.ravel(), rw.ravel(), thr=1e-9,
                                              normalize=True)
    ip, ix, iv = out.matrix.to_numpy()
    np.testing.assert_allclose(L, _dense(rip, rix, riv, 150), rtol=1e-4, atol=1e-6)


def _dense(ip, ix, iv, n):
    M = np.zeros((n, n))
    for i in range(n):
        M[i, ix[ip[i]:ip[i + 1]]] = iv[ip[i]:ip[i + 1]]
    return M
