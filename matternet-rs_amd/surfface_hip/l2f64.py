"""f64 Euclidean kNN call sites of the reference, on mn_knn_l2_f64.

  * topk_by_l2                    src_legacy/energymaps.rs:875-892
  * prepare_query_item (energy)   src_legacy/core.rs:872-909
  * estimate_intrinsic_dimension  src_legacy/clustering.rs:132-195 (Two-NN)

The distance folds, their order and the tie rules are the reference's (see
include/matternet_hip.h); results are bit-exact.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from . import _lib
from ._torch import ptr, stream_handle, to_device, on_device

_MAX_NQ = 65535 * 32  # queries per library call


@on_device


def knn_l2_f64(Q, Cm, k: int, q_ids=None, use_sqrt: bool = False, stream=None):
    """Exact f64 Euclidean kNN of the rows of Q against Cm (device tensors, f64
    or f32 widened exactly).  q_ids [nq] (int64): the corpus row each query
    excludes.  Returns (idx [nq, k] int32 (-1 pad), dist [nq, k] f64)."""
    Q = to_device(Q)
    Cm = to_device(Cm)
    if Q.dtype != Cm.dtype or Q.dtype not in (torch.float32, torch.float64):
        raise TypeError("Q and C must both be float32 or both float64")
    if Q.dim() != 2 or Cm.dim() != 2 or Q.shape[1] != Cm.shape[1]:
        raise ValueError("Q [nq, d] and C [nc, d] must share d")
    nq, d = Q.shape
    ids = None if q_ids is None else to_device(np.asarray(q_ids, dtype=np.int64)
                                               if not isinstance(q_ids, torch.Tensor) else q_ids
                                               ).to(torch.int64).contiguous()
    idx = torch.empty((nq, k), dtype=torch.int32, device=Q.device)
    dist = torch.empty((nq, k), dtype=torch.float64, device=Q.device)
    f64 = 1 if Q.dtype == torch.float64 else 0
    for a in range(0, max(nq, 1), _MAX_NQ):
        b = min(nq, a + _MAX_NQ)
        if b <= a:
            break
        _lib.check(_lib.lib().mn_knn_l2_f64(
            C.c_void_p(Q[a:b].data_ptr()), b - a, ptr(Cm), Cm.shape[0], d, f64,
            None if ids is None else C.c_void_p(ids[a:b].data_ptr()), k, 1 if use_sqrt else 0,
            C.c_void_p(idx[a:b].data_ptr()), C.c_void_p(dist[a:b].data_ptr()),
            stream_handle(stream)))
    return idx, dist


def topk_by_l2(dm, i: int, k: int):
    """energymaps.rs:875-892: the k nearest rows of row i (j != i) by the f64
    squared-difference fold, stable order.  Returns a list of row indices."""
    X = to_device(dm)
    idx, _ = knn_l2_f64(X[i:i + 1], X, k, q_ids=[i])
    return [int(j) for j in idx[0].cpu().tolist() if j >= 0]


def topk_by_l2_rows(dm, rows, k: int):
    """Batched topk_by_l2 over several rows: idx [len(rows), k] (-1 pad)."""
    X = to_device(dm)
    r = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=X.device)
    idx, _ = knn_l2_f64(X.index_select(0, r), X, k, q_ids=r)
    return idx


def nearest_subcentroid(queries, subcentroids):
    """prepare_query_item's energy-mode scan (core.rs:883-900) for a batch of
    (already projected) queries: index and distance of the nearest
    sub-centroid by sqrt of the f64 fold, strict '<' (lowest index on ties)."""
    idx, dist = knn_l2_f64(queries, subcentroids, 1, use_sqrt=True)
    return idx[:, 0], dist[:, 0]


def prepare_query_items_energy(queries, subcentroids, subcentroid_lambdas):
    """core.rs:872-909 energy mode, batched: the lambda of each query's nearest
    sub-centroid.  The reference asserts finite queries (core.rs:866-869)."""
    Q = to_device(queries)
    if not bool(torch.isfinite(Q).all()):
        raise ValueError("query item has non-finite values")  # core.rs:866-869 assert!
    i, _ = nearest_subcentroid(Q, subcentroids)
    lam = to_device(subcentroid_lambdas).to(torch.float64)
    return lam.index_select(0, i.to(torch.int64))


def estimate_intrinsic_dimension(rows, f: int, sample_indices) -> int:
    """Two-NN (clustering.rs:132-195) given the reference's shuffled sample
    (its StdRng stream is the caller's): d1, d2 = the two smallest sqrt'd f64
    distances of each sampled row to every other row; ratios d2/d1 where
    d1 > 1e-12, summed in sample order (Rust's sequential f64 Sum)."""
    X = to_device(rows)
    n = X.shape[0]
    if n < 10:
        return min(f, 2)
    s = torch.as_tensor(np.asarray(sample_indices, dtype=np.int64), device=X.device)
    _, dist = knn_l2_f64(X.index_select(0, s), X, 2, q_ids=s, use_sqrt=True)
    d = dist.cpu().numpy()
    ratios = [float(r[1] / r[0]) for r in d if r[0] > 1e-12]
    if not ratios:
        return min(f, 3)
    acc = -0.0
    for r in ratios:
        acc = acc + r
    mean_ratio = acc / len(ratios)
    ident = 1.0 / math.log(mean_ratio) if mean_ratio > 1.001 else float(f)
    return max(1, min(f, _round_half_away(ident)))


def _round_half_away(x: float) -> int:
    """Rust f64::round (half away from zero), exact: x - floor(x) is exact."""
    a = abs(x)
    r = math.floor(a)
    if a - r >= 0.5:
        r += 1
    return int(math.copysign(r, x)) if r else 0
