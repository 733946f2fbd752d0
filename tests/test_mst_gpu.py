"""MST stage candidate graph on the GPU (mn_mst_candidate_graph_f32) vs the
oracle restatement of surfface-core/src/mst.rs:312-412 (+ distance.rs:78-108).

Bhattacharyya: the kernel's ln is glibc's logf restated on the device
(csrc/glibc_f32.hpp, checked on every f32 input by tests/test_libm_gpu.py),
the oracle calls the host glibc, everything else is the reference's f32
arithmetic in its order: indices, distances and costs bit-exact, including
on constructed sub-ulp near-ties.  The L2 metrics run the K1 kNN (bit-exact)."""
import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _inputs(c, f, seed, small_var_frac=0.05, dups=0):
    rng = np.random.default_rng(seed)
    means = rng.normal(size=(c, f)).astype(np.float32)
    var = (rng.random((c, f)) * 2.0).astype(np.float32)
    var[rng.random((c, f)) < small_var_frac] = np.float32(1e-12)  # below the 1e-10 floor
    for t in range(dups):
        means[c - 1 - t] = means[t]
        var[c - 1 - t] = var[t]
    return means, var


def _gpu(means, var, k, metric, tw, thickness=None):
    import surfface_hip as S
    e = S.build_candidate_graph(torch.from_numpy(means).cuda(),
                                None if var is None else torch.from_numpy(var).cuda(), k,
                                S.DistanceMetric(metric), S.ThicknessWeight(tw),
                                thickness=None if thickness is None else torch.from_numpy(thickness).cuda())
    kk = min(k, len(means) - 1)
    return (e.v.cpu().numpy().reshape(-1, kk), e.distance.cpu().numpy().reshape(-1, kk),
            e.cost.cpu().numpy().reshape(-1, kk), e)


def _check(means, var, k, tw=O.TW_MEAN):
    v, d, cost, e = _gpu(means, var, k, O.MST_BHATTACHARYYA, tw)
    rv, rd, rc = O.mst_candidates(means, var, k, O.MST_BHATTACHARYYA, tw)
    np.testing.assert_array_equal(v, rv)
    np.testing.assert_array_equal(d.view(np.uint32), rd.view(np.uint32))
    np.testing.assert_array_equal(cost.view(np.uint32), rc.view(np.uint32))
    return e


def test_bhattacharyya_sub_ulp_near_ties():
    """399 copies of one centroid whose means and variances are
    perturbed by a few ulps: every distance from row 0 is tiny and the order
    of the near-equal ones is decided by the last bits of the ln terms (and
    ties by j).  Bit-exact indices and distances."""
    rng = np.random.default_rng(17)
    c, f = 400, 16
    base_m = rng.normal(size=f).astype(np.float32)
    base_v = (rng.random(f) + 0.5).astype(np.float32)
    means = np.repeat(base_m[None], c, 0)
    var = np.repeat(base_v[None], c, 0)
    steps = rng.integers(-3, 4, size=(c - 1, f)).astype(np.int32)
    var[1:] = (var[1:].view(np.int32) + steps).view(np.float32)
    msteps = rng.integers(-1, 2, size=(c - 1, f)).astype(np.int32) * (rng.random((c - 1, f)) < 0.2)
    means[1:] = (means[1:].view(np.int32) + msteps.astype(np.int32)).view(np.float32)
    e = _check(means, var, 24)
    _check(means, var, 300)


@pytest.mark.parametrize("c,f,k", [(2, 3, 8), (37, 5, 8), (700, 48, 16), (1500, 20, 200)])
def test_bhattacharyya_graph_vs_oracle(c, f, k):
    means, var = _inputs(c, f, seed=c + f)
    _check(means, var, k)


def test_bhattacharyya_multi_pass_selection_and_ties():
    """C > 1024 (several selection passes with a carried prefix) and
    duplicated centroids (distance exactly 0: ties resolved by ascending j)."""
    means, var = _inputs(3000, 12, seed=9, dups=40)
    e = _check(means, var, 8)
    v = e.v.cpu().numpy().reshape(-1, 8)
    d = e.distance.cpu().numpy().reshape(-1, 8)
    for t in range(40):  # row t's nearest is its twin at distance 0
        assert d[t, 0] == 0.0 and v[t, 0] == 3000 - 1 - t


@pytest.mark.parametrize("tw", [0, 1, 2, 3, 4])
def test_thickness_weights(tw):
    means, var = _inputs(300, 9, seed=31)
    _check(means, var, 6, tw=tw)


def test_reference_thickness_case():
    """test_mst.rs:274-327 test_thickness_weight_functions' centroid state:
    equal means, variance rows 0.5 / 1.0 / 0.2 / 0.8, k = 3."""
    means = np.ones((4, 3), np.float32)
    var = np.repeat(np.array([[0.5], [1.0], [0.2], [0.8]], np.float32), 3, axis=1)
    for tw in range(5):
        e = _check(means, var, 3, tw=tw)
        th = e.thickness.cpu().numpy()
        np.testing.assert_array_equal(th, np.array([0.5, 1.0, 0.2, 0.8], np.float32))
        assert (e.cost.cpu().numpy() > 0).all()


@pytest.mark.parametrize("metric", [1, 2])
def test_l2_metrics_bit_exact(metric):
    X = datagen.clustered(2000, 24, seed=4, blobs=6, dup_frac=0.01, zero_frac=0.002)
    th = np.linspace(0.1, 2.0, 2000).astype(np.float32)
    for tw in (0, 3, 4):
        v, d, cost, _ = _gpu(X, None, 10, metric, tw, thickness=th)
        rv, rd, rc = O.mst_candidates(X, None, 10, metric, tw, thickness=th)
        np.testing.assert_array_equal(v, rv)
        np.testing.assert_array_equal(d.view(np.uint32), rd.view(np.uint32))
        np.testing.assert_array_equal(cost.view(np.uint32), rc.view(np.uint32))


def test_nan_distance_is_error():
    import surfface_hip as S
    means, var = _inputs(50, 4, seed=1)
    means[7, 2] = np.nan
    with pytest.raises(S.MnError) as ei:
        _gpu(means, var, 4, O.MST_BHATTACHARYYA, O.TW_MEAN)
    assert ei.value.args[0] == -3 or "NaN" in str(ei.value)
