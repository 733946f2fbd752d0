"""K5 parity on the GPU: HIP sparsification (C ABI) vs the oracle / restatement.

Contract: kept edges and their order bit-exact; ties by input position (the
reference's sort_unstable leaves them unspecified).
"""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GS = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                        "golden_small.npz"))


def to_rows(ip, ix, w, k):
    n = len(ip) - 1
    idx = np.full((n, k), -1, np.int32)
    ww = np.zeros((n, k))
    for i in range(n):
        m = ip[i + 1] - ip[i]
        idx[i, :m] = ix[ip[i]:ip[i + 1]]
        ww[i, :m] = w[ip[i]:ip[i + 1]]
    return idx, ww


def to_csr(idx, w):
    ip, ix, iw = [0], [], []
    for i in range(idx.shape[0]):
        for r in range(idx.shape[1]):
            if idx[i, r] >= 0:
                ix.append(idx[i, r]); iw.append(w[i, r])
        ip.append(len(ix))
    return np.array(ip), np.array(ix, np.int32), np.array(iw)


def hip(idx, w, ratio=0.5, mode=0):
    import surfface_hip as S
    oi, ow, applied = S.sparsify_rows(torch.from_numpy(idx).cuda(), torch.from_numpy(w).cuda(),
                                      ratio, mode)
    return oi.cpu().numpy(), ow.cpu().numpy(), applied


def test_golden_reference_larger_graph():
    idx, w = to_rows(GS["sf_in_indptr"], GS["sf_in_indices"], GS["sf_in_w"], 64)
    oi, ow, applied = hip(idx, w)
    assert applied
    ip, ix, iw = to_csr(oi, ow)
    np.testing.assert_array_equal(ip, GS["sf_out_indptr"])
    np.testing.assert_array_equal(ix, GS["sf_out_indices"])
    np.testing.assert_array_equal(iw, GS["sf_out_w"])


@pytest.mark.parametrize("ratio", [0.5, 0.1, 0.37, 1.0])
def test_knn_rows_with_score_ties(ratio):
    rng = np.random.default_rng(3)
    n, k = 20000, 32
    idx = rng.integers(0, n, size=(n, k)).astype(np.int32)
    idx[rng.random((n, k)) < 0.2] = -1          # ragged rows
    w = np.round(rng.random((n, k)) * 8) / 8.0  # quantised weights: many score ties
    oi, ow, applied = hip(idx, w, ratio)
    rip, rix, riw = O.sfgrass(*to_csr(idx, w), ratio=ratio)
    ip, ix, iw = to_csr(oi, ow)
    np.testing.assert_array_equal(ip, rip)
    np.testing.assert_array_equal(ix, rix)
    np.testing.assert_array_equal(iw, riw)


def test_sparse_graph_passthrough():
    idx = np.array([[1, 2, -1], [0, -1, 2], [0, 1, -1]], np.int32)  # avg degree < 10
    w = np.array([[1.0, 0.5, 0], [1.0, 0, 0.8], [0.5, 0.8, 0]])
    oi, ow, applied = hip(idx, w)
    assert not applied
    assert oi.tolist() == [[1, 2, -1], [0, 2, -1], [0, 1, -1]]


def test_inline_mode_vs_restatement():
    """laplacian.rs:216-282: avg > 10 enables; rows with len > 2 keep len/2."""
    rng = np.random.default_rng(8)
    n, k = 5000, 24
    idx = rng.integers(0, n, size=(n, k)).astype(np.int32)
    idx[rng.random((n, k)) < 0.4] = -1
    w = rng.random((n, k))
    oi, ow, applied = hip(idx, w, mode=1)
    assert applied
    deg = (idx >= 0).sum(1)
    for i in range(0, n, 37):
        row = [(idx[i, r], w[i, r], p) for p, r in enumerate(np.nonzero(idx[i] >= 0)[0])]
        if len(row) > 2:
            sc = [(wt * math.sqrt(float(deg[i] * deg[j])), p, j, wt) for j, wt, p in row]
            sc.sort(key=lambda t: (-t[0], t[1]))
            keep = max(len(row) // 2, 1)
            exp = [t[2] for t in sc[:keep]]
        else:
            exp = [j for j, _, _ in row]
        got = [int(v) for v in oi[i] if v >= 0]
        assert got == exp, i


def _csr_hip(ip, ix, w, ratio=0.5, n_nodes=0):
    import surfface_hip as S
    n = len(ip) - 1
    A = S.CsrMatrix(torch.from_numpy(np.asarray(ip, np.int64)).cuda(),
                    torch.from_numpy(np.asarray(ix, np.int32)).cuda(),
                    torch.from_numpy(np.asarray(w, np.float64)).cuda(), (n, n))
    out, applied = S.sparsify_sfgrass_csr(A, ratio, n_nodes)
    oip, oix, oiw = out.to_numpy()
    return oip, oix, oiw, applied


@pytest.mark.parametrize("ratio", [0.5, 0.1, 0.37, 1.0])
def test_csr_rows_of_any_length_vs_oracle(ratio):
    """mn_sparsify_sfgrass: CSR rows of ANY length — empty,
    single, wave-sized, block-sized (LDS) and hub rows beyond the LDS image
    (global-scratch bitonic) — with quantised weights (score ties by input
    position), bit-exact vs or_sfgrass (sparsification.rs:32-101)."""
    rng = np.random.default_rng(11)
    n = 30_000
    lens = rng.integers(0, 40, size=n)
    lens[:5] = [0, 1, 2, 3, 0]
    lens[100:110] = rng.integers(65, 512, size=10)      # wave tiers
    lens[200:220] = rng.integers(513, 8192, size=20)    # LDS block sort
    lens[300] = 8192
    lens[301] = 8193                                    # first hub size
    lens[302] = 20_000
    lens[303] = 70_001                                  # > 2^16
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ix = rng.integers(0, n, size=int(ip[-1])).astype(np.int32)
    w = np.round(rng.random(int(ip[-1])) * 8) / 8.0
    oip, oix, oiw, applied = _csr_hip(ip, ix, w, ratio)
    assert applied
    rip, rix, riw = O.sfgrass(ip, ix, w, ratio)
    np.testing.assert_array_equal(oip, rip)
    np.testing.assert_array_equal(oix, rix)
    np.testing.assert_array_equal(oiw.view(np.uint64), riw.view(np.uint64))


def test_csr_sparse_graph_unchanged_and_n_nodes():
    """avg = edges / n_nodes < 10: the rows come back unchanged
    (sparsification.rs:41-53); the same rows with a smaller n_nodes divisor
    cross the switch."""
    rng = np.random.default_rng(2)
    n = 1000
    lens = rng.integers(0, 12, size=n)                   # avg ~5.5
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ix = rng.integers(0, n, size=int(ip[-1])).astype(np.int32)
    w = rng.random(int(ip[-1]))
    oip, oix, oiw, applied = _csr_hip(ip, ix, w)
    assert not applied
    np.testing.assert_array_equal(oip, ip)
    np.testing.assert_array_equal(oix, ix)
    np.testing.assert_array_equal(oiw, w)
    oip, oix, oiw, applied = _csr_hip(ip, ix, w, n_nodes=400)  # avg ~13.8
    assert applied
    assert oip[-1] < ip[-1]
