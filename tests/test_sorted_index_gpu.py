"""K4 parity on the GPU: HIP sorted index (C ABI) vs the CPU oracle.

Contract: order bit-exact given identical lambdas (ascending OrderedFloat,
ties by the decimal-string id); bucket keys and std_dev bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

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
