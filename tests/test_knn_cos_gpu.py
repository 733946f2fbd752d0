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
