"""K4 parity on the GPU: HIP sorted index (C ABI) vs the CPU oracle.

Contract: order bit-exact given identical lambdas (ascending OrderedFloat,
ties by the decimal-string id); bucket keys and std_dev bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from surfface_hip import _lib

pytestmark = pytest.mark.gpu

GS = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                        "golden_small.npz"))


def hip_sort(lam):
    import surfface_hip as S
    sl = S.SortedLambdas().build_from(torch.from_numpy(np.ascontiguousarray(lam)).cuda())
    return sl.order.cpu().numpy(), sl.keys.cpu().numpy(), sl.std_dev


def check(lam):
    order, keys, sd = hip_sort(lam)
    ro, rk, rsd = O.sorted_index(lam)
    np.testing.assert_array_equal(order, ro)
    np.testing.assert_array_equal(keys.view(np.uint64), rk.view(np.uint64))
    if np.isfinite(rsd):
        assert np.float32(sd) == np.float32(rsd)  # sequential f32 fold reproduced


def test_golden_with_nan_and_signed_zero():
    order, keys, _ = hip_sort(GS["sort_lambda"])
    np.testing.assert_array_equal(order, GS["sort_order"])


@pytest.mark.parametrize("n", [1, 2, 10, 11, 2047, 2049, 100_003, 1_000_000])
def test_massive_ties_string_order(n):
    rng = np.random.default_rng(n)
    lam = rng.integers(0, 7, size=n).astype(np.float64) / 7.0  # ~n/7 per bucket
    check(lam)


def test_random_unique_and_special_values():
    rng = np.random.default_rng(5)
    lam = rng.normal(size=300_000)
    lam[::1000] = -0.0
    lam[5::1000] = 0.0
    lam[7::5000] = np.nan
    lam[9::7000] = np.inf
    lam[11::7000] = -np.inf
    check(lam)


def _lookup_case(lam, queries, k, p, lambda_p, base_delta, growth=1.7, mult=10.0):
    import surfface_hip as S
    sl = S.SortedLambdas().build_from(torch.from_numpy(np.ascontiguousarray(lam)).cuda())
    ro, rk, rsd = O.sorted_index(lam)
    q = torch.from_numpy(np.ascontiguousarray(queries, np.float64)).cuda()
    for kind in ("range", "nearest"):
        if kind == "range":
            oi, ol, oc = sl.range_bylambda(q, k, p)
        else:
            oi, ol, oc = sl.k_nearest_by_lambda(q, k, lambda_p, base_delta, growth, mult)
        oi, ol, oc = oi.cpu().numpy(), ol.cpu().numpy(), oc.cpu().numpy()
        for t, lq in enumerate(queries):
            ref = (O.range_bylambda(rk, ro, rsd, lq, k, p) if kind == "range" else
                   O.k_nearest_by_lambda(rk, ro, rsd, lq, k, lambda_p, base_delta, growth, mult))
            if ref is None:
                assert oc[t] == -1, (kind, t, lq)
                continue
            c = len(ref[0])
            assert oc[t] == c, (kind, t, lq, oc[t], c)
            np.testing.assert_array_equal(oi[t, :c], ref[0])
            np.testing.assert_array_equal(ol[t, :c].view(np.uint64), ref[1].view(np.uint64))


def test_lambda_lookups_vs_oracle_massive_ties():
    """range_bylambda / k_nearest_by_lambda (sorted_index.rs:64-140) batched on
    the GPU: 200k items in 9 lambda buckets (ties in string-id order)."""
    rng = np.random.default_rng(4)
    lam = rng.integers(0, 9, size=200_000).astype(np.float64) / 8.0
    qs = np.concatenate([rng.uniform(-0.1, 1.1, 60), [0.0, 0.5, 1.0, 0.0625, np.nan, 3.0, -2.0]])
    _lookup_case(lam, qs, 25, 1.0, 0.5, None)
    _lookup_case(lam, qs, 7, 3.0, 0.01, 0.001, growth=2.0, mult=50.0)


def test_lambda_lookups_vs_oracle_unique_and_edges():
    rng = np.random.default_rng(6)
    lam = rng.uniform(0.0, 1.0, 50_001)
    lam[::97] = 0.25  # equal distances on both sides of 0.3 / 0.2 queries
    lam[1::97] = 0.35
    qs = np.concatenate([rng.uniform(0, 1, 80), [0.3, 0.2, 0.25, 1.5, -0.5, np.nan]])
    _lookup_case(lam, qs, 40, 2.0, 0.001, None)
    _lookup_case(lam, qs, 1, 0.0, 1.0, 0.0)     # base_delta 0: one window
    _lookup_case(lam[:1], qs[:10], 3, 1.0, 0.5, None)  # a single item


def _std_both(lam, monkeypatch):
    """std_dev through the certified pass 1 (default) and through the forced
    sequential pass 1 (MN_STD_SEQ=1)."""
    _, _, sd = hip_sort(lam)
    monkeypatch.setenv("MN_STD_SEQ", "1")
    with _lib.use_tuning():  # the tuning build honours MN_STD_SEQ
        _, _, sd_seq = hip_sort(lam)
    monkeypatch.delenv("MN_STD_SEQ")
    return sd, sd_seq


def _midpoint_case(n, rng, offset_units):
    """multiples of 2^-30 in [0, 1) whose f64 sum is exact, the last value set
    so the sum lands on an f32 rounding midpoint (+ offset_units * 2^-30)."""
    lam = rng.integers(0, 2**30, size=n).astype(np.float64) * 2.0**-30
    head = float(np.sum(lam[:-1]))  # exact: every partial sum fits in 53 bits
    e = int(np.floor(np.log2(head + 1.0)))
    ulp = 2.0 ** (e - 23)
    target = np.ceil(head / ulp) * ulp + ulp / 2 + offset_units * 2.0**-30
    lam[-1] = target - head
    assert 0.0 <= lam[-1] and np.float64(head + lam[-1]) == target
    return lam


@pytest.mark.parametrize("case", ["tie2", "cancel", "mid_1m", "mid_plus_1m", "normal_1m",
                                  "huge_mixed"])
def test_std_pass1_certificate_matches_sequential(case, monkeypatch):
    """K4 std_dev: pass 1's f64 sum is certified from a double-double parallel
    sum plus the sequential-fold error bound (gamma_n * sum|x|); inputs whose
    bound straddles an f32 rounding boundary must fall back to the sequential
    fold.  Both paths bit-equal to the oracle's sequential restatement."""
    rng = np.random.default_rng(11)
    lam = {
        "tie2": lambda: np.array([1.0, 2.0**-24]),           # exact f32 tie -> even
        "cancel": lambda: np.array([1e16, 1.0, -1e16, 3.0]),  # fold 3, exact 4
        "mid_1m": lambda: _midpoint_case(1_000_000, rng, 0),
        "mid_plus_1m": lambda: _midpoint_case(1_000_000, rng, 1),
        "normal_1m": lambda: rng.normal(size=1_000_000),
        "huge_mixed": lambda: np.concatenate([rng.normal(size=50_000) * 1e15,
                                              rng.normal(size=50_000) * 1e-30]),
    }[case]()
    sd, sd_seq = _std_both(lam, monkeypatch)
    _, _, rsd = O.sorted_index(lam)
    assert np.float32(sd_seq) == np.float32(rsd)
    assert np.float32(sd) == np.float32(rsd)


def test_range_band_exp2_edge():
    """The band of range_bylambda is std / exp2(p) (an optimised reference
    build: LLVM rewrites pow(2.0, p) to exp2(p)); the edge case of
    tests/test_oracle.py, where pow(2, p) would exclude the key."""
    import surfface_hip as S
    from test_oracle import EXP2_EDGE as e
    sl = S.SortedLambdas().build_from(torch.tensor(e["lam"], dtype=torch.float64, device="cuda"))
    assert sl.std_dev == 0.25
    out = sl.range_bylambda(e["lq"], 4, e["p"])
    assert [i for i, _ in out] == [1] and [l for _, l in out] == [0.75]
