"""§8(f) rank 2 — the lambda-aware query path through the HIP C ABI.

Mirror of ArrowSpace::search_lambda_aware (src_legacy/core.rs:1156-1193) and
ArrowSpace::normalise_query_lambda (core.rs:1361-1372), batched over query
rows: every query scores every item with ArrowItem::lambda_similarity
(core.rs:162-179) and keeps the reference's stable-sorted top k.  Bit-exact
(mn_search_lambda_aware).
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle, on_device


@on_device


def search_lambda_aware(X: torch.Tensor, lambdas: torch.Tensor, queries: torch.Tensor,
                        query_lambdas, k: int, alpha: float, stream=None, hybrid: bool = False):
    """X [n, f] (f32 — the exactly widened values of ArrowSpace.data — or f64),
    item lambdas [n] f64, queries [nq, f] (or [f]) f64, query_lambdas [nq] f64
    (or a float for one query).  Returns (idx int64 [nq, k], score f64 [nq, k]),
    (-1, NaN) padded when k > n; for a 1-D query, the reference's
    [(idx, score)] list.  Raises MnError(MN_EINVAL) where the reference's
    assert_ne!(lambda, 0.0) fires and MnError(MN_ENONFINITE) on a NaN score.
    hybrid=True: search_lambda_aware_hybrid (core.rs:1196-1318; ties to the
    smaller index where the reference leaves them unspecified)."""
    if X.dtype not in (torch.float32, torch.float64):
        raise TypeError("X must be float32 or float64")
    X = require_cuda(X, X.dtype, "X", 2)
    n, f = X.shape
    lam = require_cuda(lambdas, torch.float64, "lambdas", 1)
    if lam.numel() != n:
        raise ValueError(f"lambdas has {lam.numel()} entries for {n} items")
    single = queries.dim() == 1
    Q = require_cuda(queries.reshape(1, -1) if single else queries, torch.float64, "queries", 2)
    if Q.shape[1] != f:
        raise ValueError(f"items should be of the same length ({Q.shape[1]} vs {f})")
    nq = Q.shape[0]
    if isinstance(query_lambdas, torch.Tensor):
        lq = require_cuda(query_lambdas.reshape(-1), torch.float64, "query_lambdas", 1)
    else:
        lq = torch.full((nq,), float(query_lambdas), dtype=torch.float64, device=X.device)
    if lq.numel() != nq:
        raise ValueError("one lambda per query")
    oi = torch.empty((nq, max(k, 1)), dtype=torch.int64, device=X.device)
    osc = torch.empty((nq, max(k, 1)), dtype=torch.float64, device=X.device)
    fn = _lib.lib().mn_search_lambda_aware_hybrid if hybrid else _lib.lib().mn_search_lambda_aware
    _lib.check(fn(
        ptr(X), 1 if X.dtype == torch.float64 else 0, n, f, ptr(lam), ptr(Q), ptr(lq), nq, k,
        float(alpha), ptr(oi), ptr(osc), stream_handle(stream)))
    oi, osc = oi[:, :k], osc[:, :k]
    if single:
        ids, scs = oi[0].cpu().tolist(), osc[0].cpu().tolist()
        return [(i, v) for i, v in zip(ids, scs) if i >= 0]
    return oi, osc


def normalise_query_lambda(raw_lambda: float, min_lambdas: float, range_lambdas: float) -> float:
    """core.rs:1361-1372: (raw - min) / range clamped to [0, 1]."""
    v = (raw_lambda - min_lambdas) / range_lambdas
    return min(max(v, 0.0), 1.0)


_UNDECIDABLE = ("Check your eps parameter for the builder, every dataset has an optimal eps. "
                "Also, the query item may be out of context for the dataset (undecidable), "
                "despite all safeguards its lambda is 0.0")


def prepare_query_lambdas(queries: torch.Tensor, L_features, taumode=None, min_lambdas=None,
                          range_lambdas=None):
    """ArrowSpace::prepare_query_item, eigen mode without a projection
    (core.rs:912-933), batched: the synthetic lambda of every query row
    (TauMode::compute_synthetic_lambda, taumode.rs:261-320, tau =
    select_tau(query)) on the GPU energy pass (mn_energy_rows, MN_G_TAUMODE),
    then normalise_query_lambda when the index statistics are finite.
    queries: [nq, f] f32 (the exactly widened values the reference's f64
    query holds).  Raises ValueError where the reference panics (a raw lambda
    within 1e-12 of 0, approx::relative_eq!)."""
    from .energy import TauMode, energy_rows
    tm = TauMode.Median if taumode is None else taumode
    if not torch.isfinite(queries).all():
        raise ValueError("query item has non-finite values")  # core.rs:865-868
    _, _, lam = energy_rows(queries, L_features, _lib.MN_G_TAUMODE, tm)
    if bool((lam.abs() <= 1e-12).any()):
        raise ValueError(_UNDECIDABLE)
    if range_lambdas is not None and math.isfinite(range_lambdas):
        lam = ((lam - min_lambdas) / range_lambdas).clamp_(0.0, 1.0)
    return lam


@on_device


def search_lambda_aware_hybrid(X, lambdas, queries, query_lambdas, k: int, alpha: float,
                               stream=None):
    """ArrowSpace::search_lambda_aware_hybrid (core.rs:1196-1318), batched."""
    return search_lambda_aware(X, lambdas, queries, query_lambdas, k, alpha, stream, hybrid=True)
