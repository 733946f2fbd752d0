"""f64 Euclidean kNN call sites (mn_knn_l2_f64) vs the oracle, bit-exact.

References: topk_by_l2 (src_legacy/energymaps.rs:875-892), prepare_query_item
energy mode (src_legacy/core.rs:872-909), estimate_intrinsic_dimension
(src_legacy/clustering.rs:132-195).
"""
import math

import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _eq(idx, dist, ridx, rdist):
    np.testing.assert_array_equal(idx, ridx)
    np.testing.assert_array_equal(dist.view(np.uint64), rdist.view(np.uint64))


@pytest.mark.parametrize("n,d,k", [(3000, 37, 10), (700, 768, 32), (300, 5, 64)])
def test_topk_by_l2_all_rows_vs_oracle(n, d, k):
    import surfface_hip as S
    X = np.random.default_rng(n).standard_normal((n, d))
    ids = np.arange(n)
    idx, dist = S.knn_l2_f64(torch.from_numpy(X).cuda(), torch.from_numpy(X).cuda(), k,
                             q_ids=ids)
    ridx, rdist = O.knn_l2_f64(X, X, k, q_ids=ids)
    _eq(idx.cpu().numpy(), dist.cpu().numpy(), ridx, rdist)


def test_ties_under_sqrt_go_to_the_lower_index():
    """Integer grid: many exactly equal distances; under sqrt more collide."""
    import surfface_hip as S
    rng = np.random.default_rng(5)
    X = rng.integers(-3, 4, size=(2500, 6)).astype(np.float64)
    for use_sqrt in (False, True):
        idx, dist = S.knn_l2_f64(torch.from_numpy(X).cuda(), torch.from_numpy(X).cuda(), 7,
                                 q_ids=np.arange(2500), use_sqrt=use_sqrt)
        ridx, rdist = O.knn_l2_f64(X, X, 7, q_ids=np.arange(2500), use_sqrt=use_sqrt)
        _eq(idx.cpu().numpy(), dist.cpu().numpy(), ridx, rdist)


def test_f32_input_is_widened_exactly():
    import surfface_hip as S
    X = datagen.uniform(4000, 48, seed=3)
    idx, dist = S.knn_l2_f64(torch.from_numpy(X).cuda(), torch.from_numpy(X).cuda(), 5,
                             q_ids=np.arange(4000))
    ridx, rdist = O.knn_l2_f64(X.astype(np.float64), X.astype(np.float64), 5,
                               q_ids=np.arange(4000))
    _eq(idx.cpu().numpy(), dist.cpu().numpy(), ridx, rdist)


def test_topk_by_l2_single_row_and_rows():
    import surfface_hip as S
    X = np.random.default_rng(1).standard_normal((900, 20))
    ridx, _ = O.knn_l2_f64(X[[17, 4, 800]], X, 6, q_ids=[17, 4, 800])
    assert S.topk_by_l2(X, 17, 6) == ridx[0].tolist()
    np.testing.assert_array_equal(S.topk_by_l2_rows(X, [17, 4, 800], 6).cpu().numpy(), ridx)


def test_prepare_query_items_energy_mode():
    """1-NN by sqrt'd distance with strict '<'; duplicated sub-centroids make
    the lowest index win."""
    import surfface_hip as S
    rng = np.random.default_rng(2)
    sc = rng.standard_normal((777, 32))
    sc[500] = sc[12]          # exact duplicate: 12 must win
    lam = rng.random(777)
    Q = np.vstack([rng.standard_normal((1000, 32)), sc[[12, 3]] + 0.0])
    got = S.prepare_query_items_energy(torch.from_numpy(Q).cuda(), torch.from_numpy(sc).cuda(),
                                       torch.from_numpy(lam).cuda()).cpu().numpy()
    ridx, _ = O.knn_l2_f64(Q, sc, 1, use_sqrt=True)
    np.testing.assert_array_equal(got.view(np.uint64), lam[ridx[:, 0]].view(np.uint64))
    assert ridx[-2, 0] == 12


def _two_nn_restated(X, f, sample):
    """clustering.rs:132-195 with the oracle's distances (sequential Sum)."""
    ids = np.asarray(sample)
    _, dist = O.knn_l2_f64(X[ids], X, 2, q_ids=ids, use_sqrt=True)
    ratios = [r[1] / r[0] for r in dist if r[0] > 1e-12]
    acc = -0.0
    for r in ratios:
        acc = acc + r
    m = acc / len(ratios)
    ident = 1.0 / math.log(m) if m > 1.001 else float(f)
    r = math.floor(ident)
    r = r + 1 if ident - r >= 0.5 else r
    return max(1, min(f, int(r)))


def test_two_nn_intrinsic_dimension_sampled_rows():
    import surfface_hip as S
    n, f = 120_000, 24
    rng = np.random.default_rng(11)
    latent = rng.standard_normal((n, 5))
    X = latent @ rng.standard_normal((5, f))  # intrinsic dimension 5
    sample = rng.permutation(n)[:500]
    got = S.estimate_intrinsic_dimension(torch.from_numpy(X).cuda(), f, sample)
    assert got == _two_nn_restated(X, f, sample)
    assert 3 <= got <= 7
