"""§8(f) rank 2 parity on the GPU: batched search_lambda_aware (C ABI) vs the
CPU oracle restatement of src_legacy/core.rs:1156-1193.

Contract: bit-exact indices AND scores (same sequential non-contracted f64
folds; order = stable sort by score descending, ties by ascending index).
"""
import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def hip_search(X, lam, Q, lq, k, alpha):
    import surfface_hip as S
    oi, osc = S.search_lambda_aware(torch.from_numpy(X).cuda(), torch.from_numpy(lam).cuda(),
                                    torch.from_numpy(Q).cuda(), torch.from_numpy(lq).cuda(), k,
                                    alpha)
    return oi.cpu().numpy(), osc.cpu().numpy()


def case(n, f, nq, seed, dup=False, zero=False):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-1, 1, (n, f)).astype(np.float32)
    lam = rng.uniform(0, 1, n)
    if dup and n > 8:
        X[n // 2] = X[1]
        lam[n // 2] = lam[1]
        lam[5] = lam[3]
        X[5] = X[3]
    if zero and n > 4:
        X[2] = 0.0
    Q = rng.uniform(-1, 1, (nq, f))
    lq = rng.uniform(0.01, 1, nq)
    return X, lam, Q, lq


def check(X, lam, Q, lq, k, alpha):
    oi, osc = hip_search(X, lam, Q, lq, k, alpha)
    ri, rs, rc = O.search_lambda_aware(X.astype(np.float64), lam, Q, lq, k, alpha)
    assert (rc == min(k, X.shape[0])).all()
    np.testing.assert_array_equal(oi, ri)
    np.testing.assert_array_equal(osc.view(np.uint64), rs.view(np.uint64))


@pytest.mark.parametrize("n,f,nq,k", [(1, 3, 1, 1), (5, 7, 2, 10), (255, 33, 3, 8),
                                      (256, 64, 16, 32), (257, 64, 17, 256),
                                      (5000, 100, 20, 10), (70_001, 48, 5, 64)])
@pytest.mark.parametrize("alpha", [0.7, 0.0, 1.3])
def test_search_vs_oracle(n, f, nq, k, alpha):
    check(*case(n, f, nq, n + nq, dup=True, zero=True), k, alpha)


def test_search_f64_items():
    X, lam, Q, lq = case(3000, 40, 4, 11, dup=True)
    X64 = X.astype(np.float64) + 1e-9  # not representable in f32
    import surfface_hip as S
    oi, osc = S.search_lambda_aware(torch.from_numpy(X64).cuda(), torch.from_numpy(lam).cuda(),
                                    torch.from_numpy(Q).cuda(), torch.from_numpy(lq).cuda(), 12,
                                    0.6)
    ri, rs, _ = O.search_lambda_aware(X64, lam, Q, lq, 12, 0.6)
    np.testing.assert_array_equal(oi.cpu().numpy(), ri)
    np.testing.assert_array_equal(osc.cpu().numpy().view(np.uint64), rs.view(np.uint64))


def test_search_all_ties_index_order():
    # identical items and lambdas: every score ties -> ascending index
    X = np.ones((1000, 8), np.float32)
    lam = np.full(1000, 0.25)
    Q = np.ones((2, 8))
    oi, osc = hip_search(X, lam, Q, np.array([0.5, 0.75]), 40, 0.5)
    np.testing.assert_array_equal(oi, np.tile(np.arange(40), (2, 1)))


def test_single_query_list_and_errors():
    import surfface_hip as S
    X, lam, Q, lq = case(100, 6, 1, 5)
    res = S.search_lambda_aware(torch.from_numpy(X).cuda(), torch.from_numpy(lam).cuda(),
                                torch.from_numpy(Q[0]).cuda(), float(lq[0]), 3, 0.7)
    ri, rs, _ = O.search_lambda_aware(X.astype(np.float64), lam, Q, lq, 3, 0.7)
    assert res == list(zip(ri[0].tolist(), rs[0].tolist()))
    with pytest.raises(S.MnError) as e:   # core.rs:1169 assert_ne!(lambda, 0.0)
        S.search_lambda_aware(torch.from_numpy(X).cuda(), torch.from_numpy(lam).cuda(),
                              torch.from_numpy(Q).cuda(), 0.0, 3, 0.7)
    assert e.value.code == S._lib.MN_EINVAL
    Xn = X.copy()
    Xn[7, 2] = np.nan   # norm NaN -> `denom > 0.0` false -> cos 0 (core.rs:234-241): no panic
    check(Xn, lam, Q, lq, 10, 0.7)
    Xn[7, 2] = np.inf   # inf/inf = NaN score: partial_cmp().unwrap() panics
    with pytest.raises(S.MnError) as e:
        S.search_lambda_aware(torch.from_numpy(Xn).cuda(), torch.from_numpy(lam).cuda(),
                              torch.from_numpy(Q).cuda(), torch.from_numpy(lq).cuda(), 3, 0.7)
    assert e.value.code == S._lib.MN_ENONFINITE
    _, _, rc = O.search_lambda_aware(Xn.astype(np.float64), lam, Q, lq, 3, 0.7)
    assert rc[0] == -3
    with pytest.raises(S.MnError):
        S.search_lambda_aware(torch.from_numpy(X).cuda(), torch.from_numpy(lam).cuda(),
                              torch.from_numpy(Q).cuda(), torch.from_numpy(lq).cuda(), 257, 0.7)


def test_search_large_c3_shape_sampled():
    # 262144 x 768 items (C3 feature width): 3 queries checked against the oracle
    X = datagen.uniform(262_144, 768, seed=42)
    rng = np.random.default_rng(9)
    lam = rng.uniform(0, 1, X.shape[0])
    Q = X[[5, 100_000, 262_143]].astype(np.float64)
    lq = lam[[5, 100_000, 262_143]]
    check(X, lam, Q, lq, 32, 0.7)


def test_end_to_end_query_path_vs_oracle():
    """build lambdas (taumode, normalised) -> prepare query lambdas -> search:
    query lambdas within the energy pass tolerance (1e-9 rel), then the
    search bit-exact given those lambdas (core.rs:864-933, 1156-1193)."""
    import surfface_hip as S
    from test_energy_gpu import csr_dev, feature_laplacian
    ip, ix, iv = feature_laplacian(f=64, profile=800, topk=4, seed=3)
    X = datagen.uniform(4000, 64, seed=5)
    Lf = csr_dev(ip, ix, iv)
    lam, st = S.compute_taumode_lambdas(torch.from_numpy(X).cuda(), Lf)
    rng = np.random.default_rng(4)
    Qf = (X[[0, 17, 3999]] + rng.uniform(-0.05, 0.05, (3, 64))).astype(np.float32)
    lq = S.prepare_query_lambdas(torch.from_numpy(Qf).cuda(), Lf, min_lambdas=st["min"],
                                 range_lambdas=st["range"])
    _, _, rl = O.energy_rows(Qf, ip, ix, iv, O.G_TAUMODE, O.TAU_MEDIAN)
    rq = np.clip((rl - st["min"]) / st["range"], 0.0, 1.0)
    np.testing.assert_allclose(lq.cpu().numpy(), rq, rtol=1e-9, atol=1e-12)
    oi, osc = S.search_lambda_aware(torch.from_numpy(X).cuda(), lam,
                                    torch.from_numpy(Qf.astype(np.float64)).cuda(), lq, 10, 0.7)
    ri, rs, rc = O.search_lambda_aware(X.astype(np.float64), lam.cpu().numpy(),
                                       Qf.astype(np.float64), lq.cpu().numpy(), 10, 0.7)
    np.testing.assert_array_equal(oi.cpu().numpy(), ri)
    np.testing.assert_array_equal(osc.cpu().numpy().view(np.uint64), rs.view(np.uint64))
    with pytest.raises(ValueError):    # zero query: raw lambda 0 -> the reference panics
        S.prepare_query_lambdas(torch.zeros((1, 64), device="cuda"), Lf)


def check_hybrid(X, lam, Q, lq, k, alpha):
    import surfface_hip as S
    oi, osc = S.search_lambda_aware_hybrid(torch.from_numpy(X).cuda(),
                                           torch.from_numpy(lam).cuda(),
                                           torch.from_numpy(Q).cuda(),
                                           torch.from_numpy(lq).cuda(), k, alpha)
    ri, rs, rc = O.search_lambda_aware(X.astype(np.float64), lam, Q, lq, k, alpha, hybrid=True)
    np.testing.assert_array_equal(oi.cpu().numpy(), ri)
    np.testing.assert_array_equal(osc.cpu().numpy().view(np.uint64), rs.view(np.uint64))
    return ri, rc


@pytest.mark.parametrize("n,f,k", [(1, 3, 1), (7, 5, 10), (300, 33, 8), (5000, 64, 32),
                                   (70_001, 48, 255)])
@pytest.mark.parametrize("alpha", [0.7, 0.0, 1.0])
def test_hybrid_vs_oracle(n, f, k, alpha):
    X, lam, Q, lq = case(n, f, 5, n + 3, dup=True, zero=True)
    # high-semantic matches: queries that are (scaled) item rows, + scaled copies
    if n > 20:
        X[n - 1] = X[4] * 3.0
        X[n - 2] = X[4] * 0.5
        Q[0] = X[4]
        Q[1] = X[n // 3]
    ri, rc = check_hybrid(X, lam, Q, lq, k, alpha)
    assert (rc >= 1).all()


def test_hybrid_k_limit():
    import surfface_hip as S
    X, lam, Q, lq = case(100, 6, 1, 5)
    with pytest.raises(S.MnError) as e:
        S.search_lambda_aware_hybrid(torch.from_numpy(X).cuda(), torch.from_numpy(lam).cuda(),
                                     torch.from_numpy(Q).cuda(), torch.from_numpy(lq).cuda(),
                                     256, 0.7)
    assert e.value.code == S._lib.MN_ENOTSUP


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_hybrid_many_high_semantic_items_small_k(k):
    """More than k items with cosine > 0.9999 (scaled copies of the query):
    every such item keeps its COSINE as score (core.rs:1289-1299), including
    one that reaches the union only through the lambda top k (advisor r1)."""
    rng = np.random.default_rng(40 + k)
    n, f = 2000, 16
    X, lam, Q, lq = case(n, f, 3, 77)
    scales = rng.uniform(0.2, 5.0, size=40).astype(np.float32)
    rows = rng.choice(n, 40, replace=False)
    X[rows] = (Q[0].astype(np.float32)[None, :] * scales[:, None]).astype(np.float32)
    Q[0] = X[rows[0]].astype(np.float64)
    # lambdas: the copies' lambdas near lq[0] beat every other item's lambda score
    lam[rows] = lq[0] + rng.uniform(-1e-3, 1e-3, size=40)
    for alpha in (0.7, 0.2):
        check_hybrid(X, lam, Q, lq, k, alpha)
