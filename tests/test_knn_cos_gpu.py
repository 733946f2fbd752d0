"""K1 (cosine feature graph) parity on the GPU vs the oracle.

Contract: indices, distances (f64) and weights bit-exact vs the reference's
sequential-f64 rectified-cosine semantics (test_helpers.rs:77-126).
"""
import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def hip_cols(X, topk, **kw):
    import surfface_hip as S
    i, d, w, st = S.knn_cos_columns(torch.from_numpy(np.ascontiguousarray(X)).cuda(), topk, **kw)
    return i.cpu().numpy(), d.cpu().numpy(), w.cpu().numpy(), st


def ref_cols(X, topk, q=None, **kw):
    XT = np.ascontiguousarray(X.T)
    if q is None:
        return O.knn_cos(XT, topk, **kw)
    return O.knn_cos(XT, topk, q_begin=q[0], q_end=q[1], **kw)


def exact(a, b):
    for x, y in zip(a, b):
        np.testing.assert_array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


@pytest.mark.parametrize("n,f,topk", [(1500, 768, 4), (20000, 256, 8), (300, 70, 10)])
def test_feature_graph_uniform(n, f, topk):
    X = datagen.uniform(n, f, seed=9)
    i, d, w, st = hip_cols(X, topk)
    exact((i, d, w), ref_cols(X, topk))


def test_feature_graph_eps_sigma_p_filters_and_zero_columns():
    X = datagen.clustered(4000, 150, seed=3, blobs=5)
    X[:, 7] = 0.0   # zero column: cos = 0 -> dist 1 to everything
    X[:, 9] = X[:, 11]  # duplicate columns: distance 0
    kw = dict(eps=0.9, sigma=0.3, p=3.0)
    i, d, w, st = hip_cols(X, 6, **kw)
    ri, rd, rw = ref_cols(X, 6, **kw)
    np.testing.assert_array_equal(i, ri)
    np.testing.assert_array_equal(d, rd)
    # the device pow is glibc's restated (glibc_f64.hpp): weights bit-exact
    np.testing.assert_array_equal(w.view(np.uint64), rw.view(np.uint64))


def test_ties_force_exact_fallback():
    X = np.zeros((500, 60), np.float32)
    X[:, :30] = datagen.uniform(500, 1, seed=2)  # 30 identical columns: ties beyond k+margin
    X[:, 30:] = datagen.uniform(500, 30, seed=3)
    i, d, w, st = hip_cols(X, 5)
    exact((i, d, w), ref_cols(X, 5))
    assert st["n_uncertified"] >= 30


def test_long_profiles_sampled_nodes():
    n, f = 200_000, 768
    X = datagen.uniform(n, f, seed=42)
    i, d, w, st = hip_cols(X, 4)
    ri, rd, rw = ref_cols(X, 4, q=(100, 108))
    exact((i[100:108], d[100:108], w[100:108]), (ri, rd, rw))
    assert st["n_uncertified"] == 0


@pytest.mark.parametrize("topk", [65, 150, 300])
def test_feature_graph_topk_beyond_64(topk):
    """graph.rs topk is any usize: topk > 64 takes the exact all-pairs path
    (every node's f - 1 exact distances, sorted, filtered, padded past f - 1)
    — bit-exact vs the oracle, including topk > f - 1 (300 > 199)."""
    X = datagen.clustered(3000, 200, seed=9, blobs=7)
    kw = dict(eps=0.95, sigma=0.5, p=2.7)
    i, d, w, st = hip_cols(X, topk, **kw)
    ri, rd, rw = ref_cols(X, topk, **kw)
    np.testing.assert_array_equal(i, ri)
    np.testing.assert_array_equal(d.view(np.uint64), rd.view(np.uint64))
    np.testing.assert_array_equal(w.view(np.uint64), rw.view(np.uint64))


def test_norms_from_the_exact_pass_tiny_columns_and_the_1e12_cut():
    """Round 5: the exact norms come with the exact pass and the selection
    uses sqrt(G_ii).  Columns scaled so that n_i n_j straddles the
    reference's 1e-12 cut (norms ~1e-6), tiny and huge columns side by side,
    a zero column and a NaN column: bit-exact vs the oracle, and the same
    graph as the round-4 order (exact norms first, MN_COS_NORMS_SIDE=1)."""
    import os
    import surfface_hip as S
    X = datagen.uniform(3000, 96, seed=21)
    nrm = np.sqrt((X.astype(np.float64) ** 2).sum(0))
    for c, target in ((3, 1e-6), (4, 1e-6 * (1 + 1e-12)), (5, 0.999999e-6), (6, 1.0000001e-6),
                      (7, 1e-9), (8, 1e6)):
        X[:, c] = (X[:, c] * (target / nrm[c])).astype(np.float32)
    X[:, 10] = 0.0
    kw = dict(eps=1.0, sigma=1.0, p=2.0)
    i, d, w, st = hip_cols(X, 4, **kw)
    exact((i, d, w), ref_cols(X, 4, **kw))
    Xn = X.copy()
    Xn[17, 12] = np.nan  # non-finite data: that column's node and its partners fall back
    i2, d2, w2, _ = hip_cols(Xn, 4, **kw)
    exact((i2, d2, w2), ref_cols(Xn, 4, **kw))
    with S._lib.use_tuning():
        os.environ["MN_COS_NORMS_SIDE"] = "1"
        try:
            i3, d3, w3, _ = hip_cols(X, 4, **kw)
        finally:
            os.environ.pop("MN_COS_NORMS_SIDE", None)
    exact((i, d, w), (i3, d3, w3))


@pytest.mark.parametrize("case", ["uniform", "tiny_columns"])
def test_f32_gram_tuning_path_bit_exact(case):
    """Tuning build, MN_COS_GRAM=1: the f32-MFMA Gram with the f64 fold and
    its wider certification band (and, for columns whose max |x| leaves
    [2^-20, 2^40], the device range check sending G back to f64 MFMA): the
    graph stays bit-exact vs the oracle."""
    import os
    import surfface_hip as S
    X = datagen.uniform(6000, 200, seed=23)
    if case == "tiny_columns":
        X[:, 5] *= np.float32(1e-9)  # max |x| below 2^-20: the f64 Gram runs
        X[:, 6] = 0.0
    kw = dict(eps=1.0, sigma=1.0, p=2.0)
    with S._lib.use_tuning():
        os.environ["MN_COS_GRAM"] = "1"
        try:
            i, d, w, st = hip_cols(X, 4, **kw)
        finally:
            os.environ.pop("MN_COS_GRAM", None)
    exact((i, d, w), ref_cols(X, 4, **kw))
