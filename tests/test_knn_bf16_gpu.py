"""K1/C5 (bf16 rectified-cosine item graph) parity on the GPU vs the oracle.

Contract: indices, distances (f64) and weights bit-exact vs the reference's
sequential-f64 rectified-cosine semantics (src_legacy/tests/test_helpers.rs:77-126,
src_legacy/laplacian.rs:245-290) on the exactly widened bf16 values.  The
oracle (or_knn_cos_f64) receives the same values as f32 (bf16 -> f32 is exact).
"""
import numpy as np
import pytest
import torch

import datagen
from surfface_hip import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def bf16_rows(X):
    """(bf16 bits as a cuda bfloat16 tensor, the same values as f32 numpy)."""
    bits = datagen.to_bf16_bits(np.ascontiguousarray(X, dtype=np.float32))
    t = torch.from_numpy(bits.view(np.int16)).cuda().view(torch.bfloat16)
    return t, datagen.bf16_bits_to_f32(bits)


def hip(Xt, topk, **kw):
    import surfface_hip as S
    i, d, w, st = S.knn_cos_bf16(Xt, topk, **kw)
    return i.cpu().numpy(), d.cpu().numpy(), w.cpu().numpy(), st


def exact(a, b):
    for x, y in zip(a, b):
        np.testing.assert_array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


@pytest.mark.parametrize("n,d,topk", [(3000, 256, 10), (700, 3072, 32), (1500, 100, 8),
                                      (2000, 64, 64), (257, 24, 5)])
def test_item_graph_uniform(n, d, topk):
    Xt, Xf = bf16_rows(datagen.uniform(n, d, seed=11))
    i, dd, w, st = hip(Xt, topk)
    exact((i, dd, w), O.knn_cos(Xf, topk))
    assert st["n_queries"] == n


def test_item_graph_clustered_dups_zero_rows_and_filters():
    X = datagen.clustered(5000, 96, seed=5, blobs=40, sigma=0.05, dup_frac=0.02, zero_frac=0.002)
    X[10] = -X[11]          # antipodal pair: cos -1 -> rectified dist 1
    Xt, Xf = bf16_rows(X)
    kw = dict(eps=0.6, sigma=0.25, p=2.0)
    exact(hip(Xt, 12, **kw)[:3], O.knn_cos(Xf, 12, **kw))


def test_item_graph_pow_weights():
    Xt, Xf = bf16_rows(datagen.clustered(3000, 128, seed=8, blobs=16))
    kw = dict(eps=0.95, sigma=0.4, p=3.0)
    i, d, w, _ = hip(Xt, 7, **kw)
    ri, rd, rw = O.knn_cos(Xf, 7, **kw)
    np.testing.assert_array_equal(i, ri)
    np.testing.assert_array_equal(d, rd)
    # the device pow is glibc's restated (glibc_f64.hpp): weights bit-exact
    np.testing.assert_array_equal(w.view(np.uint64), rw.view(np.uint64))


def test_ties_force_exact_fallback():
    X = datagen.uniform(1200, 48, seed=4)
    X[:100] = X[0]          # 100 identical rows: ties beyond topk + margin
    Xt, Xf = bf16_rows(X)
    i, d, w, st = hip(Xt, 8)
    exact((i, d, w), O.knn_cos(Xf, 8))
    assert st["n_uncertified"] >= 100


def test_tiny_norm_rows_are_exact():
    X = datagen.uniform(900, 32, seed=6)
    X[5] *= 1e-7            # norm^2 ~ 1e-13: denom = n_i n_j crosses the 1e-12 switch
    X[6] *= 3e-7
    X[7] = 0.0
    Xt, Xf = bf16_rows(X)
    exact(hip(Xt, 6)[:3], O.knn_cos(Xf, 6))


def test_few_rows():
    for n in (1, 2, 5):
        Xt, Xf = bf16_rows(datagen.uniform(n, 16, seed=n))
        exact(hip(Xt, 4)[:3], O.knn_cos(Xf, 4))


def test_query_shard_against_full_corpus():
    import surfface_hip as S
    Xt, Xf = bf16_rows(datagen.uniform(4000, 200, seed=21))
    a, b = 1000, 2300
    i, d, w, _ = S.knn_cos_bf16_qc(Xt[a:b].contiguous(), Xt, 9, q_offset=a, c_offset=0)
    ri, rd, rw = O.knn_cos(Xf, 9, q_begin=a, q_end=b)
    exact((i.cpu().numpy(), d.cpu().numpy(), w.cpu().numpy()), (ri, rd, rw))


def test_large_sampled_rows():
    """Size-independent check at a production-like shape: 120k x 768 bf16, every
    row certified or rescanned, sampled rows bit-exact vs the oracle."""
    n, d, k = 120_000, 768, 16
    Xt, Xf = bf16_rows(datagen.uniform(n, d, seed=77))
    i, dd, w, st = hip(Xt, k)
    rows = [0, 1, 4097, 65535, n - 1]
    for r in rows:
        ri, rd, rw = O.knn_cos(Xf, k, q_begin=r, q_end=r + 1)
        exact((i[r:r + 1], dd[r:r + 1], w[r:r + 1]), (ri, rd, rw))
    # uniform data: the candidate bound certifies every row
    assert st["n_uncertified"] == 0
    # every list is sorted by (dist, idx) and excludes self
    assert np.all(np.diff(dd, axis=1) >= 0)
    assert not np.any(i == np.arange(n)[:, None])


def test_errors():
    import surfface_hip as S
    Xt, _ = bf16_rows(datagen.uniform(100, 16, seed=1))
    with pytest.raises(S.MnError):
        S.knn_cos_bf16(Xt, 0)
    with pytest.raises(S.MnError):
        S.knn_cos_bf16(Xt, 65)
    bad = Xt.clone()
    bad[3, 3] = float("nan")
    with pytest.raises(S.MnError):
        S.knn_cos_bf16(bad, 4)


def test_two_phase_edge_rows_and_one_phase_agree(monkeypatch):
    """The two-phase generator (sample thresholds + SW_COS sweep, n >= 2048):
    zero rows, tiny norms, an antipodal pair, 150 identical rows (ties beyond
    any threshold -> uncertified -> exact scan) and clustered duplicates, all
    bit-exact vs the oracle and vs the one-phase generator (MN_BF16_X1=0)."""
    X = datagen.clustered(6000, 96, seed=13, blobs=30, sigma=0.05, dup_frac=0.02,
                          zero_frac=0.002)
    X[20] = -X[21]
    X[30] *= 1e-7
    X[40:190] = X[40]
    Xt, Xf = bf16_rows(X)
    kw = dict(eps=0.8, sigma=0.5, p=2.0)
    i, d, w, st = hip(Xt, 16, **kw)
    assert st["algo"] == 3 and st["sample_rows"] > 0  # MN_KNN_BF16X1
    assert st["n_uncertified"] >= 150
    exact((i, d, w), O.knn_cos(Xf, 16, **kw))
    with _lib.use_tuning():  # the alternative paths: tuning build knobs
        monkeypatch.setenv("MN_BF16_TM", "0")  # k-block-major sweep layout
        exact((i, d, w), hip(Xt, 16, **kw)[:3])
        monkeypatch.delenv("MN_BF16_TM")
        monkeypatch.setenv("MN_BF16_X1", "0")
        i1, d1, w1, st1 = hip(Xt, 16, **kw)
    assert st1["sample_rows"] == 0
    exact((i, d, w), (i1, d1, w1))


def test_phase1_sweep_matches_list_generator(monkeypatch):
    """Phase 1 by sweep (round 4b, knn_bf16.hip cos_sweep_phase1) vs the list
    generator (MN_BF16_P1_SWEEP=0), and with a pre-sample list of 2
    (MN_BF16_P1_L0) that leaves many rows to the fallback: bit-exact vs the
    oracle every time."""
    Xt, Xf = bf16_rows(datagen.clustered(12000, 96, seed=31, blobs=20, dup_frac=0.01,
                                         zero_frac=0.002))
    ref = O.knn_cos(Xf, 16)
    with _lib.use_tuning():
        for env in ({}, {"MN_BF16_P1_L0": "2"}, {"MN_BF16_P1_SWEEP": "0"}):
            for kk in ("MN_BF16_P1_L0", "MN_BF16_P1_SWEEP"):
                monkeypatch.delenv(kk, raising=False)
            for kk, vv in env.items():
                monkeypatch.setenv(kk, vv)
            i, dd, w, st = hip(Xt, 16)
            assert st["sample_rows"] > 0, (env, st)
            exact((i, dd, w), ref)


@pytest.mark.parametrize("n,d,topk", [(2048 + 1024, 768, 32), (9000, 40, 3), (4500, 3072, 64)])
def test_two_phase_shapes(n, d, topk):
    """two-phase at the smallest size it runs at, a d that is not a multiple
    of 32 (zero-padded KB32 k-blocks), and topk = 64 (L1 = 32)."""
    Xt, Xf = bf16_rows(datagen.uniform(n, d, seed=n))
    i, dd, w, st = hip(Xt, topk)
    assert st["sample_rows"] > 0
    exact((i, dd, w), O.knn_cos(Xf, topk))


@pytest.mark.parametrize("kind", ["near_1d", "projection"])
def test_two_phase_sorted_rows_stay_certified(kind):
    """Rows in an adversarial order (ADVICE r1 / VERDICT r2): near_1d is the
    ORIGINAL round-2 stress case (t v + 0.05 noise + 0.2, rows sorted by t),
    projection a normal cloud sorted by one projection.  Every row of the
    graph is bit-exact vs the oracle; the uncertified rows (resolved by the
    exact scan) and the fallback time are recorded, and the projection case
    keeps almost every row certified."""
    import json
    n, d = 20_000, 64
    X = datagen.sorted_rows(n, d, kind)
    Xt, Xf = bf16_rows(X)
    i, dd, w, st = hip(Xt, 10, timing=True)
    print(f"sorted-rows cosine {kind}", json.dumps(
        {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}))
    assert st["sample_rows"] > 0
    exact((i, dd, w), O.knn_cos(Xf, 10))
    if kind == "projection":
        assert st["n_uncertified"] <= n // 100, st


@pytest.mark.parametrize("kind", ["uniform", "clustered"])
def test_two_phase_symmetric_sweep_matches_query_major(kind, monkeypatch):
    """The self item graph's symmetric sweep (gram_sweep2.hpp SW_COS_SYM: rows
    in descending-threshold order, each unordered pair once, the column's
    test in the accumulator and the row's key from the same hit; the default)
    and the query-major SW_COS sweep (MN_BF16_SYM=0): both bit-exact vs the
    oracle, so identical to each other."""
    import json
    X = (datagen.uniform(12_000, 192, seed=17) if kind == "uniform"
         else datagen.clustered(12_000, 192, seed=18, blobs=16, dup_frac=0.01, zero_frac=0.002))
    Xt, Xf = bf16_rows(X)
    kw = dict(eps=0.9, sigma=0.7, p=2.0)
    i, d, w, st = hip(Xt, 24, timing=True, **kw)
    print(f"COS_SYM {kind}", json.dumps({k: (round(v, 2) if isinstance(v, float) else v)
                                         for k, v in st.items()}))
    assert st["sweep_slices"] == -1  # the symmetric sweep ran
    monkeypatch.setenv("MN_BF16_SYM", "0")
    with _lib.use_tuning():
        i0, d0, w0, st0 = hip(Xt, 24, **kw)
    assert st0["sweep_slices"] > 0
    ref = O.knn_cos(Xf, 24, **kw)
    exact((i, d, w), ref)
    exact((i0, d0, w0), ref)
