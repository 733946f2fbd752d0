"""Legacy lambda-tau graph build under GraphParams semantics, composed from the
HIP C ABI (no host arithmetic on the data path):

  * build_laplacian_matrix        src_legacy/laplacian.rs:122-201 (+ _main_laplacian
                                  :177-198, _build_adjacency :205-294 with the
                                  production defaults: sigma = sigma.unwrap_or(1.0)
                                  (:256), eps-valid degrees (:219-229), inline
                                  sparsification iff avg degree > 10 (:231-282))
  * GraphLaplacian / sparsity     src_legacy/graph.rs:121-132, :626-632
  * GraphFactory.build_laplacian_matrix_from_k_cluster
                                  src_legacy/graph.rs:193-249 (sparsity_check panic
                                  :230-238 -> SparsityError)
  * GraphFactory.build_spectral_laplacian
                                  src_legacy/graph.rs:257-313 ("Laplacian of
                                  Laplacian" -> signals, which taumode prefers:
                                  taumode.rs:138-145)
  * EigenMaps.eigenmaps / compute_taumode
                                  src_legacy/eigenmaps.rs:133-227
  * BuilderParams.define_result_k surfface-pipeline/src/builder.rs:785-793

Kernels used: mn_knn_cos_columns_f32/_f64 (rectified-cosine kNN of the node
profiles, bit-exact), mn_sparsify_rows (MN_SPARSIFY_INLINE), mn_laplacian_from_knn
(UNION symmetrisation + L = D - W, f64, bit-exact), mn_standardize_columns_f64
(normalise = true; smartcore's StandardScaler is absent: parity-unpinned),
mn_energy_rows (taumode lambdas).

Two readings the reference leaves to smartcore's CosinePair (absent, parity
unpinned): query_row_top_k(i, topk + 1) is taken to return i itself first
(distance 0), so dropping it leaves the topk nearest other nodes — the
brute-force spec of test_helpers.rs:73-170 — and the degree of a node is its
count of eps-valid neighbours among those (the weight > 1e-12 filter of the
adjacency step only differs from it for sigma / p so extreme that a cosine
distance <= eps maps below 1e-12).
"""
from __future__ import annotations

import math

from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import _lib
from .energy import TauMode, compute_taumode_lambdas
from .knn import knn_cos_columns
from .laplacian import CsrMatrix, GraphParams, build_laplacian_from_knn
from .sparsification import sparsify_rows
from ._torch import ptr, stream_handle, on_device


class SparsityError(RuntimeError):
    """The reference's panic!("Resulting laplacian matrix is too sparse")."""


@dataclass
class GraphLaplacian:
    """src_legacy/graph.rs:121-132."""
    init_data: torch.Tensor       # the (optionally standardised) items, rows = nodes
    matrix: CsrMatrix             # n x n, f64
    nnodes: int                   # items of the ORIGINAL data (n_items) or n
    graph_params: GraphParams
    energy: bool = False

    @property
    def shape(self):
        return self.matrix.shape

    def nnz(self) -> int:
        return self.matrix.nnz

    @staticmethod
    def sparsity(matrix: CsrMatrix) -> float:
        """graph.rs:626-632: 1 - nnz / (rows * cols)."""
        r, c = matrix.shape
        return 1.0 - matrix.nnz / float(r * c)


@on_device
def standardize_columns(X: torch.Tensor, stream=None) -> torch.Tensor:
    """StandardScaler over the columns of X (f64 on the device)."""
    X = X.to(torch.float64).contiguous()
    out = torch.empty_like(X)
    n, m = X.shape
    _lib.check(_lib.lib().mn_standardize_columns_f64(ptr(X), n, m, ptr(out),
                                                      stream_handle(stream)))
    return out


def _cos_graph(items: torch.Tensor, params: GraphParams):
    """_build_adjacency (laplacian.rs:205-294) on the rows of `items`:
    (idx [n, topk] int32, w [n, topk] f64) after the inline pruning."""
    n = items.shape[0]
    sigma = params.sigma if params.sigma is not None else 1.0  # :256 unwrap_or(1.0)
    # the kernels take nodes as COLUMNS: X = items^T ([profile, nodes])
    X = items.t().contiguous()
    if X.dtype == torch.float64:
        idx, _, w = _knn_cos_columns_f64(X, params.topk, params.eps, sigma, params.p)
    else:
        idx, _, w, _ = knn_cos_columns(X.float(), params.topk, eps=params.eps, sigma=sigma,
                                       p=params.p)
    # degrees = the eps-valid neighbours among the topk nearest others
    # (:219-229), counted BEFORE the weight > 1e-12 filter (:255-258); sparsify
    # iff their average > 10, keep max(len/2, 1) of rows with len > 2 by
    # w * sqrt(deg_i deg_j) (:231-282).  The kernels' rows hold the entries
    # passing both filters, so where the weight filter can drop an eps-valid
    # entry the counts come from a second, weight-neutral query (sigma 1, p 1:
    # w = 1/(1 + d) >= 1/2); otherwise they are the row lengths.
    deg = None
    if _weight_can_drop(params.eps, sigma, params.p):
        if X.dtype == torch.float64:
            i2, _, _ = _knn_cos_columns_f64(X, params.topk, params.eps, 1.0, 1.0)
        else:
            i2, _, _, _ = knn_cos_columns(X.float(), params.topk, eps=params.eps, sigma=1.0, p=1.0)
        deg = (i2 >= 0).sum(dim=1, dtype=torch.int32)
    oi, ow, applied = sparsify_rows(idx, w, 0.5, _lib.MN_SPARSIFY_INLINE, degrees=deg)
    return oi, ow, applied, n


def _weight_can_drop(eps: float, sigma: float, p: float) -> bool:
    """Can w = 1/(1 + (d/sigma)^p) <= 1e-12 for an eps-valid rectified cosine
    distance d in [0, min(eps, 1)]?  w is monotone in d, so the ends decide."""
    dmax = min(eps, 1.0)
    if not dmax >= 0.0:
        return False

    def w(d):
        # the reference's f64 arithmetic (laplacian.rs:256 `(d / sigma).powf(p)`):
        # sigma = 0 or a negative base with a fractional p give inf / NaN, the
        # weight then fails the `> 1e-12` filter (no Python raise)
        with np.errstate(all="ignore"):
            base = np.float64(d) / np.float64(sigma)
            try:  # math.pow is the C library's pow (numpy may vectorise its own)
                t = np.float64(math.pow(float(base), float(p)))
            except (ValueError, OverflowError):
                t = np.power(base, np.float64(p))
            return np.float64(1.0) / (np.float64(1.0) + t)
    # NaN-safe: a NaN weight can drop (it fails the filter)
    return not (min(w(0.0), w(dmax)) > 1e-12) or bool(np.isnan(w(0.0)) or np.isnan(w(dmax)))


@on_device
def _knn_cos_columns_f64(X: torch.Tensor, topk: int, eps: float, sigma: float, p: float,
                         margin: int = 16, stream=None):
    n, f = X.shape
    idx = torch.empty((f, topk), dtype=torch.int32, device=X.device)
    dist = torch.empty((f, topk), dtype=torch.float64, device=X.device)
    w = torch.empty((f, topk), dtype=torch.float64, device=X.device)
    o = _lib.CosOpts(topk=topk, margin=margin, eps=eps, sigma=sigma, p=p, timing=0, reserved0=0,
                     stream=stream_handle(stream))
    _lib.check(_lib.lib().mn_knn_cos_columns_f64(ptr(X), n, f, _lib.C.byref(o), ptr(idx),
                                                 ptr(dist), ptr(w)))
    return idx, dist, w


def build_laplacian_matrix(transposed: torch.Tensor, params: GraphParams,
                           n_items: Optional[int] = None, energy: bool = False) -> GraphLaplacian:
    """src_legacy/laplacian.rs:122-201: the graph over the ROWS of `transposed`
    (the reference calls it with the centroids transposed, so the nodes are
    the features), each with its row as profile.  f32 or f64 on the device."""
    if transposed.dim() != 2:
        raise ValueError("transposed must be 2-D")
    d, n = transposed.shape
    if not (n >= 2 and d >= 2):
        raise ValueError(f"items should be at least of shape (2,2): ({d},{n})")
    items = standardize_columns(transposed) if params.normalise else transposed
    idx, w, _, _ = _cos_graph(items, params)
    L, _ = build_laplacian_from_knn(idx, w, weight_kernel="given", symmetrise="union")
    # laplacian.rs:129,165-168: nnodes = n_items, else n (the column count of
    # `transposed`, i.e. the profile length), not the node count d
    return GraphLaplacian(init_data=items, matrix=L,
                          nnodes=n_items if n_items is not None else n,
                          graph_params=params, energy=energy)


class GraphFactory:
    """src_legacy/graph.rs:184-313."""

    @staticmethod
    def build_laplacian_matrix_from_k_cluster(clustered: torch.Tensor, eps: float, k: int,
                                              topk: int, p: float,
                                              sigma_override: Optional[float], normalise: bool,
                                              sparsity_check: bool,
                                              n_items: int) -> GraphLaplacian:
        """X x F centroids -> the F x F feature Laplacian (graph.rs:193-249)."""
        if not clustered.shape[0] <= n_items:
            raise ValueError("assert!(clustered.shape().0 <= n_items) failed")
        gl = build_laplacian_matrix(clustered.t(), GraphParams(eps, k, topk, p, sigma_override,
                                                               normalise, sparsity_check),
                                    n_items, False)
        if sparsity_check:
            sp = GraphLaplacian.sparsity(gl.matrix)
            if sp > 0.95:
                raise SparsityError(f"Resulting laplacian matrix is too sparse {sp!r}")
        return gl

    @staticmethod
    def build_spectral_laplacian(gl: GraphLaplacian, n_items: int) -> CsrMatrix:
        """graph.rs:257-313: the graph over the rows of the densified
        Laplacian (the "Laplacian of Laplacian"), returned as the signals
        matrix."""
        ip, ix, iv = gl.matrix.indptr, gl.matrix.indices, gl.matrix.values
        n = gl.matrix.shape[0]
        dense = torch.zeros((n, n), dtype=torch.float64, device=iv.device)
        rows = torch.repeat_interleave(torch.arange(n, device=iv.device), ip[1:] - ip[:-1])
        dense[rows, ix.long()] = iv  # sparse_to_dense (graph.rs:316-330): a copy
        signals = build_laplacian_matrix(dense, gl.graph_params, n_items, False).matrix
        sp = GraphLaplacian.sparsity(signals)
        if sp > 0.95 and gl.graph_params.sparsity_check:
            raise SparsityError(f"Resulting spectral matrix is too sparse {sp!r}")
        return signals


@dataclass
class BuilderParams:
    """The lambda-graph fields of ArrowSpaceBuilder (surfface-pipeline/src/
    builder.rs:60-111 defaults)."""
    lambda_eps: float = 1e-3
    lambda_k: int = 6
    lambda_topk: int = 3
    lambda_p: float = 2.0
    lambda_sigma: Optional[float] = None
    normalise: bool = False
    sparsity_check: bool = False
    prebuilt_spectral: bool = False
    synthesis: TauMode = field(default_factory=lambda: TauMode.Median)

    def define_result_k(self) -> "BuilderParams":
        """builder.rs:785-793."""
        if self.lambda_k <= 5:
            self.lambda_topk = 3
        elif self.lambda_k < 10:
            self.lambda_topk = 4
        return self


@dataclass
class EigenMapsResult:
    gl: GraphLaplacian
    signals: Optional[CsrMatrix] = None
    lambdas: Optional[torch.Tensor] = None


class EigenMaps:
    """src_legacy/eigenmaps.rs:133-227 on device tensors."""

    @staticmethod
    def eigenmaps(builder: BuilderParams, centroids: torch.Tensor,
                  n_items: int) -> EigenMapsResult:
        gl = GraphFactory.build_laplacian_matrix_from_k_cluster(
            centroids, builder.lambda_eps, builder.lambda_k, builder.lambda_topk,
            builder.lambda_p, builder.lambda_sigma, builder.normalise, builder.sparsity_check,
            n_items)
        signals = GraphFactory.build_spectral_laplacian(gl, n_items) \
            if builder.prebuilt_spectral else None
        return EigenMapsResult(gl, signals)

    @staticmethod
    def compute_taumode(items: torch.Tensor, res: EigenMapsResult,
                        taumode: TauMode = TauMode.Median) -> torch.Tensor:
        """TauMode::compute_taumode_lambdas_parallel (taumode.rs:117-250): every
        item's F-vector against the signals graph if built, else the F x F
        Laplacian (taumode.rs:138-145); update_lambdas normalises
        (core.rs:1427-1442)."""
        graph = res.signals if res.signals is not None else res.gl.matrix
        lam, _ = compute_taumode_lambdas(items, graph, taumode, normalise=True)
        res.lambdas = lam
        return lam
