"""K1 parity on the GPU: HIP kNN (through the C ABI) vs the CPU oracle.

Contract: neighbour indices bit-exact and distances bit-exact
(the re-rank IS the reference's sequential f32 fold), ties by ascending index.
Every case runs with both candidate generators: the bf16-split MFMA Gram (the
default, algo "bf16x3") and the f32 MFMA Gram (algo "f32").
"""
import numpy as np
import pytest
import torch

import datagen
from surfface_hip import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GS = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                        "golden_small.npz"))


@pytest.fixture(params=["bf16x1", "bf16x3", "f32"])
def algo(request):
    return request.param


def hip_knn(X, k, **kw):
    import surfface_hip as S
    r = S.knn_l2sq(torch.from_numpy(np.ascontiguousarray(X)).cuda(), k, **kw)
    torch.cuda.synchronize()
    return r.idx.cpu().numpy(), r.dist.cpu().numpy(), r.stats


def assert_exact(idx, dist, ridx, rdist):
    np.testing.assert_array_equal(idx, ridx)
    np.testing.assert_array_equal(dist.view(np.uint32), rdist.view(np.uint32))


@pytest.mark.parametrize("name,k", [("l2_uniform", 5), ("l2_clustered", 7), ("l2_grid", 6)])
def test_golden_fixtures(name, k, algo):
    idx, dist, _ = hip_knn(GS[name + "_X"], k, algo=algo)
    assert_exact(idx, dist, GS[name + "_idx"], GS[name + "_dist"])


def test_config1_shape_10k_x_64_k10(algo):
    X = datagen.uniform(10_000, 64, seed=42)
    idx, dist, st = hip_knn(X, 10, algo=algo)
    ridx, rdist = O.knn_l2sq(X, 10)
    assert_exact(idx, dist, ridx, rdist)


@pytest.mark.parametrize("n,d,k", [(3000, 96, 32), (2500, 17, 10), (1000, 5, 3), (700, 768, 32)])
def test_clustered_duplicates_and_zero_rows(n, d, k, algo):
    X = datagen.clustered(n, d, seed=7, blobs=8, dup_frac=0.03, zero_frac=0.01)
    idx, dist, st = hip_knn(X, k, algo=algo)
    ridx, rdist = O.knn_l2sq(X, k)
    assert_exact(idx, dist, ridx, rdist)


def test_small_n_and_k_clamp(algo):
    X = datagen.uniform(5, 8, seed=3)
    idx, dist, _ = hip_knn(X, 10, algo=algo)
    ridx, rdist = O.knn_l2sq(X, 10)
    assert_exact(idx, dist, ridx, rdist)
    assert (idx[:, 4:] == -1).all()


def test_all_identical_rows_tie_by_index(algo):
    X = np.ones((300, 12), np.float32)
    idx, dist, st = hip_knn(X, 8, algo=algo)
    ridx, rdist = O.knn_l2sq(X, 8)
    assert_exact(idx, dist, ridx, rdist)
    assert st["n_uncertified"] == 300  # every row ties beyond L -> exact fallback path


def test_zero_rows_tie_beyond_candidate_list(algo):
    X = datagen.uniform(2000, 32, seed=4)
    X[::7] = 0.0  # 286 identical zero rows: ties far beyond k + margin
    idx, dist, st = hip_knn(X, 16, algo=algo)
    ridx, rdist = O.knn_l2sq(X, 16)
    assert_exact(idx, dist, ridx, rdist)
    assert st["n_uncertified"] >= 286


def test_huge_values_overflow_to_inf(algo):
    X = datagen.uniform(400, 8, seed=9)
    X[17] *= 3e19  # its distances overflow to +inf in the f32 fold
    idx, dist, st = hip_knn(X, 6, algo=algo)
    ridx, rdist = O.knn_l2sq(X, 6)
    assert_exact(idx, dist, ridx, rdist)


def test_nonfinite_input_is_an_error(algo):
    import surfface_hip as S
    X = datagen.uniform(100, 8, seed=1)
    X[5, 3] = np.nan
    with pytest.raises(S.MnError):
        hip_knn(X, 4, algo=algo)


def test_query_corpus_offsets_and_shard_merge(algo):
    import surfface_hip as S
    X = datagen.uniform(6000, 64, seed=5)
    Xd = torch.from_numpy(X).cuda()
    k = 16
    parts_i, parts_d = [], []
    bounds = [0, 1500, 3100, 6000]
    for a, b in zip(bounds[:-1], bounds[1:]):
        r = S.knn_l2sq_qc(Xd, Xd[a:b], k, q_offset=0, c_offset=a, algo=algo)
        parts_i.append(r.idx)
        parts_d.append(r.dist)
    idx, dist = S.merge_parts(torch.stack(parts_i), torch.stack(parts_d))
    ridx, rdist = O.knn_l2sq(X, k)
    assert_exact(idx.cpu().numpy(), dist.cpu().numpy(), ridx, rdist)


def test_large_n_sampled_rows_d768(algo):
    """200k x 768, k=32: full GPU run, oracle on a sample of 192 query rows."""
    n, d, k = 200_000, 768, 32
    X = datagen.uniform(n, d, seed=42)
    idx, dist, st = hip_knn(X, k, algo=algo)
    rows = np.random.default_rng(0).choice(n, 192, replace=False)
    ridx, rdist = O.knn_l2sq_rows(X, k, rows)
    assert_exact(idx[rows], dist[rows], ridx, rdist)
    # size-independent properties on every row
    assert (np.diff(dist, axis=1) >= 0).all()
    assert (idx != np.arange(n)[:, None]).all()
    # bf16x1: the n/32 x 8 sample leaves a few rows to the split exact scan
    assert st["n_uncertified"] <= 64


def test_tiny_values_flush_to_exact_path(algo):
    """Values near the f32 subnormal range: the split flushes subnormal parts,
    the certification's absolute slack then sends rows to the exact scan."""
    X = datagen.uniform(600, 24, seed=11) * np.float32(1e-30)
    X[::5] *= np.float32(1e-8)
    idx, dist, st = hip_knn(X, 8, algo=algo)
    ridx, rdist = O.knn_l2sq(X, 8)
    assert_exact(idx, dist, ridx, rdist)


def test_mixed_row_scales(algo):
    """Rows whose norms differ by many orders of magnitude (the bound scales
    with |q|^2 + max|c|^2)."""
    X = datagen.clustered(1500, 40, seed=13, blobs=6, dup_frac=0.02, zero_frac=0.0)
    scale = np.float32(10.0) ** np.random.default_rng(2).integers(-6, 7, size=(1500, 1))
    X = (X * scale.astype(np.float32)).astype(np.float32)
    idx, dist, st = hip_knn(X, 12, algo=algo)
    ridx, rdist = O.knn_l2sq(X, 12)
    assert_exact(idx, dist, ridx, rdist)


def test_bf16_range_overflow_in_split():
    """|x| beyond the bf16 range: the split's hi term rounds to inf, the row is
    flagged and rescanned exactly (f32 fold: those distances are +inf too)."""
    X = datagen.uniform(300, 16, seed=21)
    X[7, 3] = np.float32(3.3999e38)
    idx, dist, st = hip_knn(X, 5, algo="bf16x3")
    ridx, rdist = O.knn_l2sq(X, 5)
    assert_exact(idx, dist, ridx, rdist)


def test_k64_uses_f32_generator_in_auto():
    """k + margin > 64 exceeds the bf16 kernel's list width: auto picks f32,
    an explicit bf16x3 request is an error."""
    import surfface_hip as S
    X = datagen.uniform(500, 16, seed=1)
    idx, dist, _ = hip_knn(X, 60, algo="auto")
    ridx, rdist = O.knn_l2sq(X, 60)
    assert_exact(idx, dist, ridx, rdist)
    with pytest.raises(S.MnError):
        hip_knn(X, 60, algo="bf16x3")


@pytest.mark.parametrize("algo_e", ["bf16x1", "bf16x3", "f32"])
def test_euclidean_metric_sqrt_is_correctly_rounded(algo_e):
    """DistanceMetric::Euclidean (mst.rs:382-389, distance.rs:195-203): the
    library returns Rust's correctly rounded f32::sqrt of the L2^2 fold (gfx950
    sqrtf is not correctly rounded; numpy's float32 sqrt is IEEE)."""
    import surfface_hip as S
    X = datagen.clustered(4000, 40, seed=21, blobs=9, dup_frac=0.01, zero_frac=0.002)
    r = S.knn_l2sq(torch.from_numpy(X).cuda(), 12, euclidean=True, algo=algo_e)
    ridx, rdist = oracle_euclidean(X, 12)
    np.testing.assert_array_equal(r.idx.cpu().numpy(), ridx)
    np.testing.assert_array_equal(r.dist.cpu().numpy().view(np.uint32), rdist.view(np.uint32))
    # candidate-graph mirror (mst.rs:312-363) with the Euclidean metric
    e = S.build_candidate_graph(X, None, 12, S.DistanceMetric.Euclidean,
                                S.ThicknessWeight.NoWeight, thickness=np.ones(len(X), np.float32))
    np.testing.assert_array_equal(e.v.cpu().numpy(), ridx.reshape(-1))
    np.testing.assert_array_equal(e.distance.cpu().numpy().view(np.uint32),
                                  rdist.reshape(-1).view(np.uint32))
    np.testing.assert_array_equal(e.cost.cpu().numpy().view(np.uint32),
                                  e.distance.cpu().numpy().view(np.uint32))


def oracle_euclidean(X, k):
    """The reference's Euclidean candidate graph (mst.rs:330-360 with
    euclidean_distance_slice, distance.rs:195-203): the oracle's f32 fold,
    sqrtf, then the stable sort of the ROOTS (ties by index)."""
    v, d, _ = O.mst_candidates(X, None, k, O.MST_EUCLIDEAN, O.TW_NONE,
                               thickness=np.ones(len(X), np.float32))
    return v, d


def _root_tie_rows():
    """[0, 0, ...] and rows whose squared distances to it are 1.25 + 2^-23 and
    1.25: different f32 L2^2 values with the same correctly rounded root."""
    hi = np.float32(0.5) + np.float32(2.0 ** -23)
    assert np.float32(1.0) + hi * hi != np.float32(1.25)
    assert np.sqrt(np.float32(1.0) + hi * hi) == np.sqrt(np.float32(1.25))
    return np.array([1.0, hi], np.float32), np.array([1.0, 0.5], np.float32)


@pytest.mark.parametrize("algo_e", ["bf16x1", "bf16x3", "f32"])
def test_euclidean_root_ties_order_by_index(algo_e):
    """the reference sorts the ROOTED distances (stable, so equal
    roots go by index).  A larger L2^2 on a smaller index that shares its root
    with a smaller L2^2 must come first, and win the last kept slot.  Case 2:
    the equal-root run extends past the extended k + 8 list (the root-keyed
    exact rescan)."""
    import surfface_hip as S
    hi, lo = _root_tie_rows()
    far = np.stack([np.array([10.0 + j, 3.0], np.float32) for j in range(60)])
    X = np.concatenate([np.zeros((1, 2), np.float32), hi[None], lo[None], far])
    X = np.concatenate([X, np.zeros((len(X), 6), np.float32)], axis=1)  # d = 8
    for k in (1, 2, 5):
        r = S.knn_l2sq(torch.from_numpy(X).cuda(), k, euclidean=True, algo=algo_e)
        ridx, rdist = oracle_euclidean(X, k)
        assert ridx[0, 0] == 1  # the larger L2^2 on the smaller index
        np.testing.assert_array_equal(r.idx.cpu().numpy(), ridx)
        np.testing.assert_array_equal(r.dist.cpu().numpy().view(np.uint32), rdist.view(np.uint32))
    # 20 hi rows (ids 1..20) and 20 lo rows (ids 21..40): L2^2 order puts
    # every lo row first, the root order the hi rows
    X2 = np.concatenate([np.zeros((1, 2), np.float32), np.repeat(hi[None], 20, 0),
                         np.repeat(lo[None], 20, 0), far])
    X2 = np.concatenate([X2, np.zeros((len(X2), 6), np.float32)], axis=1)
    r = S.knn_l2sq(torch.from_numpy(X2).cuda(), 4, euclidean=True, algo=algo_e)
    ridx, rdist = oracle_euclidean(X2, 4)
    assert list(ridx[0]) == [1, 2, 3, 4]
    np.testing.assert_array_equal(r.idx.cpu().numpy(), ridx)
    np.testing.assert_array_equal(r.dist.cpu().numpy().view(np.uint32), rdist.view(np.uint32))
    assert r.stats["n_root_rescan"] >= 1


@pytest.mark.parametrize("kind", ["near_1d", "projection"])
def test_bf16x1_two_phase_sorted_rows(kind):
    """The headline L2 generator (bf16x1 two-phase) on rows in an adversarial
    order: every row bit-exact vs the oracle; uncertified rows and
    the fallback cost recorded."""
    import json
    n, d, k = 20_000, 64, 10
    X = datagen.sorted_rows(n, d, kind)
    idx, dist, st = hip_knn(X, k, algo="bf16x1", timing=True)
    print(f"sorted-rows L2 {kind}", json.dumps(
        {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in st.items()}))
    assert st["algo"] == 3 and st["sample_rows"] > 0
    ridx, rdist = O.knn_l2sq(X, k)
    assert_exact(idx, dist, ridx, rdist)


@pytest.mark.parametrize("kind", ["uniform", "clustered"])
def test_bf16x1_symmetric_sweep_matches_query_major(kind, monkeypatch):
    """The self-kNN sweep covers each unordered pair once (gram_sweep2.hpp
    SW_SYM: rows in ascending-threshold order, a tile's hits feed both rows'
    buffers, fp16 operands x 2^e with per-row e, the per-pair bound in the
    folds); the query-major sweep (MN_X1_SYM=0) covers every ordered pair.
    All bit-exact vs the oracle, so identical to each other."""
    import json
    n, d, k = 30_000, 96, 16
    X = (datagen.uniform(n, d, seed=8) if kind == "uniform"
         else datagen.clustered(n, d, seed=9, blobs=12, dup_frac=0.01, zero_frac=0.002))
    with _lib.use_tuning():  # the tuning build honours the knobs
        idx, dist, st = hip_knn(X, k, algo="bf16x1", timing=True)
        print(f"SYM {kind}", json.dumps({kk: (round(v, 2) if isinstance(v, float) else v)
                                         for kk, v in st.items()}))
        assert st["sweep_slices"] == -1  # the symmetric sweep ran
        monkeypatch.setenv("MN_X1_SYM", "0")
        idx0, dist0, st0 = hip_knn(X, k, algo="bf16x1", timing=True)
    assert st0["sweep_slices"] > 0
    ridx, rdist = O.knn_l2sq(X, k)
    assert_exact(idx, dist, ridx, rdist)
    assert_exact(idx0, dist0, ridx, rdist)


@pytest.mark.parametrize("kind", ["uniform", "clustered"])
def test_phase1_sweep_matches_list_generator(kind, monkeypatch):
    """Phase 1 by sweep (round 4b, knn_f32.hip sweep_phase1: pre-sample list
    generator -> threshold, SW_L2 sweep of the sample, exact L1-th key select,
    the list generator for the rows left short) vs the list generator over the
    whole sample (MN_P1_SWEEP=0): the same thresholds up to rounding, graphs
    bit-exact vs the oracle either way; a pre-sample list of 2 (MN_P1_L0)
    leaves many rows short and forces the fallback."""
    n, d, k = 40_000, 64, 16
    X = (datagen.uniform(n, d, seed=21) if kind == "uniform"
         else datagen.clustered(n, d, seed=22, blobs=16, dup_frac=0.01, zero_frac=0.002))
    ridx, rdist = O.knn_l2sq(X, k)
    with _lib.use_tuning():
        for env in ({}, {"MN_P1_L0": "2"}, {"MN_P1_SWEEP": "0"}):
            for kk in ("MN_P1_L0", "MN_P1_SWEEP"):
                monkeypatch.delenv(kk, raising=False)
            for kk, vv in env.items():
                monkeypatch.setenv(kk, vv)
            idx, dist, st = hip_knn(X, k, algo="bf16x1", timing=True)
            assert st["sweep_slices"] == -1 and st["sample_rows"] > 0, (env, st)
            assert_exact(idx, dist, ridx, rdist)


def test_uncertified_rows_batched_fallback():
    """Rows no certificate settles (all-zero rows: exact ties far beyond k)
    against a corpus >= 2^16 go through the batched split-generator pass
    (k + 1 with self, own id dropped) — bit-exact with the oracle."""
    n, d, k = 70000, 32, 32
    X = datagen.uniform(n, d, seed=11)
    zero = np.random.default_rng(2).choice(n, 300, replace=False)
    X[zero] = 0.0
    idx, dist, st = hip_knn(X, k, algo="bf16x1")
    rows = np.unique(np.concatenate([zero[:40], np.random.default_rng(3).choice(n, 40, replace=False)]))
    ridx, rdist = O.knn_l2sq_rows(X, k, rows)
    np.testing.assert_array_equal(idx[rows], ridx)
    np.testing.assert_array_equal(dist[rows].view(np.uint32), rdist.view(np.uint32))
    assert st["n_uncertified"] > 0, st


@pytest.mark.parametrize("split", ["100000", "0"], ids=["split_scan", "batched"])
def test_uncertified_rows_split_scan(split, monkeypatch):
    """Uncertified rows (all-zero rows: exact ties far beyond k, plus exact
    duplicate pairs) against a corpus >= 2^16: up to 256 of them go through
    the split exact scan (corpus parts in parallel, pruned by each row's exact
    upper bound of D_k, part lists merged by (dist, id)) — here every one of
    them (MN_FB_SPLIT raises the row limit); MN_FB_SPLIT=0 takes the batched
    split-generator pass.  Both bit-exact with the oracle."""
    import json
    n, d, k = 70000, 32, 32
    X = datagen.uniform(n, d, seed=11)
    zero = np.random.default_rng(2).choice(n, 300, replace=False)
    X[zero] = 0.0
    dup = np.setdiff1d(np.arange(1, 12), zero)
    X[dup + 20000] = X[dup]
    monkeypatch.setenv("MN_FB_SPLIT", split)
    with _lib.use_tuning():  # the tuning build honours MN_FB_SPLIT
        idx, dist, st = hip_knn(X, k, algo="bf16x1", timing=True)
    print(f"uncertified split={split}", json.dumps(
        {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in st.items()}))
    assert st["n_uncertified"] > 0, st
    rows = np.unique(np.concatenate([zero[:64], dup, dup + 20000,
                                     np.random.default_rng(6).choice(n, 24, replace=False)]))
    ridx, rdist = O.knn_l2sq_rows(X, k, rows)
    np.testing.assert_array_equal(idx[rows], ridx)
    np.testing.assert_array_equal(dist[rows].view(np.uint32), rdist.view(np.uint32))


def _euclid_rows_np(X, rows, k):
    """Reference Euclidean lists of `rows` (distance.rs:195-213 f32 fold from
    -0.0 in feature order, IEEE sqrt, stable sort of the roots, self
    excluded) — vectorised over corpus rows, sequential over features."""
    out_i, out_d = [], []
    for q in rows:
        acc = np.full(len(X), -0.0, np.float32)
        for t in range(X.shape[1]):
            df = (X[q, t] - X[:, t]).astype(np.float32)
            acc = (acc + df * df).astype(np.float32)
        r = np.sqrt(acc)
        r[q] = np.inf
        o = np.argsort(r, kind="stable")[:k]
        out_i.append(o.astype(np.int32))
        out_d.append(r[o])
    return np.stack(out_i), np.stack(out_d)


def test_euclidean_root_ties_rescan_large_corpus():
    """The root-keyed rescan (equal-root run past the extended list) against a
    corpus >= 2^16: the split scan with root keys."""
    import surfface_hip as S
    hi, lo = _root_tie_rows()
    far = (datagen.uniform(70000, 2, seed=13) + np.float32(20.0)).astype(np.float32)
    X = np.concatenate([np.zeros((1, 2), np.float32), np.repeat(hi[None], 20, 0),
                        np.repeat(lo[None], 20, 0), far])
    X = np.ascontiguousarray(np.concatenate([X, np.zeros((len(X), 6), np.float32)], axis=1))
    r = S.knn_l2sq(torch.from_numpy(X).cuda(), 4, euclidean=True, algo="bf16x1")
    rows = np.array([0, 1, 25, 100, 5000], np.int64)
    ridx, rdist = _euclid_rows_np(X, rows, 4)
    assert list(ridx[0]) == [1, 2, 3, 4]
    np.testing.assert_array_equal(r.idx.cpu().numpy()[rows], ridx)
    np.testing.assert_array_equal(r.dist.cpu().numpy()[rows].view(np.uint32), rdist.view(np.uint32))
    assert r.stats["n_root_rescan"] >= 1


def _wide_range_rows(case, n, d, seed):
    """data the fp16 symmetric sweep's single global
    exponent and corpus-maximum bounds handle worst.
      log_scales  every row scaled by 10^U(-6, 6): the largest rows set the
                  fp16 exponent, rows below ~1e-2 flush to all-zero fp16;
      tiny_mixed  10 % of the rows scaled by 1e-30 among O(1) rows (their
                  squared differences underflow: exact ties at 0);
      fp16_edge   O(1) rows plus rows at the fp16 range limit (65504 and
                  65520, which rounds to fp16 inf unscaled)."""
    rng = np.random.default_rng(seed)
    X = datagen.uniform(n, d, seed=seed)
    if case == "log_scales":
        X = (X * (10.0 ** rng.uniform(-6, 6, n))[:, None]).astype(np.float32)
    elif case == "tiny_mixed":
        rows = rng.choice(n, n // 10, replace=False)
        X[rows] *= np.float32(1e-30)
    else:
        X[123] *= np.float32(65504.0)
        X[4567, 7] = np.float32(65520.0)
        X[8901] = np.float32(65504.0)
    return np.ascontiguousarray(X)


@pytest.mark.parametrize("case", ["log_scales", "tiny_mixed", "fp16_edge"])
def test_symmetric_fp16_sweep_wide_dynamic_range(case):
    """The headline fp16 symmetric sweep (SW_SYM ran: sweep_slices == -1) on
    wide-dynamic-range rows at a size where it is selected: every row
    bit-exact vs the oracle; the rows the certification leaves to the
    refill / exact scan and the time they take are printed and bounded."""
    import json
    n, d, k = 40_000, 64, 16
    X = _wide_range_rows(case, n, d, seed={"log_scales": 31, "tiny_mixed": 32, "fp16_edge": 33}[case])
    idx, dist, st = hip_knn(X, k, algo="bf16x1", timing=True)
    print(f"wide-range {case}", json.dumps({kk: (round(v, 2) if isinstance(v, float) else v)
                                            for kk, v in st.items()}))
    assert st["sweep_slices"] == -1  # SW_SYM ran
    ridx, rdist = O.knn_l2sq(X, k)
    assert_exact(idx, dist, ridx, rdist)
    assert st["ms_total"] < 20_000, st
    # the certification cost, per case (profiles/r05: measured values):
    # log_scales certifies every row; fp16_edge leaves a handful; tiny_mixed
    # leaves ~all rows — its 1e-30 rows square to 0 in f32, so every tiny row
    # is at distance exactly |q|^2 from an O(1) row q and those 4000 exact ties
    # sit at the k-th distance of most rows (a strict certificate cannot
    # settle a tie at D_k): the refill and the exact scan resolve them
    if case == "log_scales":
        assert st["n_uncertified"] <= n // 1000 and st["ms_fallback"] < 50, st
    elif case == "fp16_edge":
        assert st["n_uncertified"] <= n // 100 and st["ms_fallback"] < 200, st
    else:
        assert st["n_escalated"] <= n and st["ms_escalate"] < 500, st
        assert st["ms_fallback"] < 2000, st


def test_symmetric_sweep_block_table_cache_across_shapes():
    """Round 6: the SW_SYM block table is built once per shape and thread and
    uploaded only when the device slot lacks it.  Interleaved shapes (n = 36k,
    40k, 36k again) and a repeated call must each use their own table: every
    row bit-exact vs the oracle, and the repeat identical to the first call."""
    d, k = 32, 8
    XA = datagen.uniform(36_000, d, seed=61)
    XB = datagen.uniform(40_000, d, seed=62)
    ia, da, sa = hip_knn(XA, k, algo="bf16x1", timing=True)
    ib, db, sb = hip_knn(XB, k, algo="bf16x1", timing=True)
    ia2, da2, _ = hip_knn(XA, k, algo="bf16x1", timing=True)
    assert sa["sweep_slices"] == -1 and sb["sweep_slices"] == -1  # SW_SYM ran
    for X, i, dd in ((XA, ia, da), (XB, ib, db)):
        ri, rd = O.knn_l2sq(X, k)
        assert_exact(i, dd, ri, rd)
    assert np.array_equal(ia, ia2) and np.array_equal(da.view(np.int32), da2.view(np.int32))


def test_split_scan_small_k_many_parts():
    """the split exact scan's final merge with k < 8 over
    more than 512 corpus parts (nc > 600K: 684 parts of 1024 rows) — the
    merge groups are capped at FMG / 8 parts.  Zero rows (exact ties at 0
    far beyond k) are the uncertified rows; bit-exact vs the oracle."""
    n, d, k = 700_000, 16, 3
    X = datagen.uniform(n, d, seed=17)
    zero = np.random.default_rng(4).choice(n, 200, replace=False)
    X[zero] = 0.0
    idx, dist, st = hip_knn(X, k, algo="bf16x1", timing=True)
    assert 0 < st["n_uncertified"] <= 4096, st  # the split scan's row range
    rows = np.unique(np.concatenate([zero[:48], np.random.default_rng(5).choice(n, 16, replace=False)]))
    ridx, rdist = O.knn_l2sq_rows(X, k, rows)
    np.testing.assert_array_equal(idx[rows], ridx)
    np.testing.assert_array_equal(dist[rows].view(np.uint32), rdist.view(np.uint32))


@pytest.mark.parametrize("algo_e", ["auto", "bf16x1"])
def test_euclidean_k64_extended_list(algo_e):
    """MN_L2 at k = 64 computes the L2^2 list k + 8 = 72
    long (two entries a lane), so a row is sent to the root-keyed rescan only
    when its equal-root run really reaches past the list: on random data
    (almost) none; sampled rows bit-exact vs the reference root order."""
    import surfface_hip as S
    n, d, k = 20_000, 32, 64
    X = datagen.uniform(n, d, seed=23)
    r = S.knn_l2sq(torch.from_numpy(X).cuda(), k, euclidean=True, algo=algo_e, timing=True)
    torch.cuda.synchronize()
    assert r.stats["n_root_rescan"] <= 16, r.stats
    rows = np.random.default_rng(7).choice(n, 24, replace=False)
    ridx, rdist = _euclid_rows_np(X, rows, k)
    np.testing.assert_array_equal(r.idx.cpu().numpy()[rows], ridx)
    np.testing.assert_array_equal(r.dist.cpu().numpy()[rows].view(np.uint32), rdist.view(np.uint32))


@pytest.mark.parametrize("k", [100, 512])
def test_large_k_exact_split_scan(k):
    """k beyond the generators' 64 (mst.rs:317 takes any k): every row through
    the exact split scan — bit-exact vs the oracle, self excluded, and the
    MN_L2 root order for k = 100 (ties of equal roots by index)."""
    import surfface_hip as S
    X = datagen.clustered(20000, 48, seed=31, blobs=12, dup_frac=0.01, zero_frac=0.002)
    r = S.knn_l2sq(torch.from_numpy(X).cuda(), k)
    ridx, rdist = O.knn_l2sq(X, k)
    np.testing.assert_array_equal(r.idx.cpu().numpy(), ridx)
    np.testing.assert_array_equal(r.dist.cpu().numpy().view(np.uint32), rdist.view(np.uint32))
    if k == 100:
        Xs = X[:3000].copy()
        r = S.knn_l2sq(torch.from_numpy(Xs).cuda(), 100, euclidean=True)
        ridx, rdist = oracle_euclidean(Xs, 100)
        np.testing.assert_array_equal(r.idx.cpu().numpy(), ridx)
        np.testing.assert_array_equal(r.dist.cpu().numpy().view(np.uint32), rdist.view(np.uint32))
