"""K2 — Laplacian assembly through the HIP C ABI (mn_laplacian_from_knn).

Host-side mirror of the reference types/entry points:
  * GraphParams            src_legacy/graph.rs:94-102
  * build_laplacian_from_knn  == _build_adjacency's weight step +
    _symmetrise_adjancency + _build_sparse_laplacian (src_legacy/laplacian.rs:
    245-419): UNION symmetrisation, L = D - W, f64 values (bit-identical)
  * LaplacianConfig / LaplacianOutput / laplacian_stage_from_edges
    surfface-core/src/laplacian.rs:49-99, 312-394: MAX symmetrisation,
    optional L_sym = I - D^-1/2 W D^-1/2, f32 values
  * compute_bhattacharyya_weights / LaplacianStage.execute
    surfface-core/src/laplacian.rs:135-298, distance.rs:260-290: the whole
    Stage C on the GPU (BC kNN of the feature columns -> MAX Laplacian)
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle, on_device


@dataclass
class GraphParams:
    """src_legacy/graph.rs:94-102 (builder defaults builder.rs:104-111)."""
    eps: float = 1e-3
    k: int = 6
    topk: int = 3
    p: float = 2.0
    sigma: Optional[float] = None
    normalise: bool = False
    sparsity_check: bool = False


@dataclass
class LaplacianConfig:
    """surfface-core/src/laplacian.rs:49-77."""
    k_neighbors: int = 15
    variance_regularizer: float = 1e-6
    normalize: bool = True
    weight_threshold: float = 1e-9


@dataclass
class CsrMatrix:
    """Device CSR (torch tensors): indptr int64 [n+1], indices int32, values."""
    indptr: torch.Tensor
    indices: torch.Tensor
    values: torch.Tensor
    shape: tuple

    @property
    def nnz(self) -> int:
        return int(self.indices.numel())

    def to_numpy(self):
        return (self.indptr.cpu().numpy(), self.indices.cpu().numpy(), self.values.cpu().numpy())

    def to_dense(self) -> np.ndarray:
        ip, ix, iv = self.to_numpy()
        out = np.zeros(self.shape, dtype=iv.dtype)
        for i in range(self.shape[0]):
            out[i, ix[ip[i]:ip[i + 1]]] = iv[ip[i]:ip[i + 1]]
        return out


@dataclass
class LaplacianOutput:
    """surfface-core/src/laplacian.rs:84-99."""
    matrix: CsrMatrix
    n_features: int
    nnz: int
    degrees: torch.Tensor
    sparsity: float


def last_stats() -> dict:
    st = _lib.LapStats()
    _lib.check(_lib.lib().mn_lap_last_stats(C.byref(st)))
    return st.as_dict()


def _adopt(csr: _lib.Csr, device) -> CsrMatrix:
    """Copy the library-owned CSR into torch tensors and free it."""
    L = _lib.lib()
    n, nnz = csr.n_rows, csr.nnz
    vdt = torch.float64 if csr.value_type == _lib.MN_F64 else torch.float32
    indptr = torch.empty(n + 1, dtype=torch.int64, device=device)
    indices = torch.empty(nnz, dtype=torch.int32, device=device)
    values = torch.empty(nnz, dtype=vdt, device=device)
    try:
        s = stream_handle()
        _lib.check(L.mn_memcpy_d2d(ptr(indptr), csr.indptr, 8 * (n + 1), s))
        if nnz:
            _lib.check(L.mn_memcpy_d2d(ptr(indices), csr.indices, 4 * nnz, s))
            _lib.check(L.mn_memcpy_d2d(ptr(values), csr.values, values.element_size() * nnz, s))
    finally:
        L.mn_csr_free(C.byref(csr))
    return CsrMatrix(indptr, indices, values, (n, n))


@on_device


def build_laplacian_from_knn(nbr_idx: torch.Tensor, nbr_val: torch.Tensor, *,
                             weight_kernel: str = "rational", symmetrise: str = "union",
                             normalize: bool = False, eps: float = 1.0, sigma: float = 1.0,
                             p: float = 2.0, weight_threshold: float = 1e-9, stream=None):
    """kNN rows -> (Laplacian CSR on device, degrees on device)."""
    nbr_idx = require_cuda(nbr_idx, torch.int32, "nbr_idx", 2)
    if nbr_val.dtype not in (torch.float32, torch.float64):
        raise TypeError("nbr_val must be float32 or float64")
    nbr_val = require_cuda(nbr_val, nbr_val.dtype, "nbr_val", 2)
    n, k = nbr_idx.shape
    wk = {"given": _lib.MN_W_GIVEN, "rational": _lib.MN_W_RATIONAL}[weight_kernel]
    sy = {"union": _lib.MN_SYM_UNION, "max": _lib.MN_SYM_MAX}[symmetrise]
    o = _lib.LapOpts(weight_kernel=wk, symmetrise=sy, normalize=1 if normalize else 0,
                     reserved0=0, eps=eps, sigma=sigma, p=p, weight_threshold=weight_threshold,
                     stream=stream_handle(stream))
    vdt = torch.float64 if sy == _lib.MN_SYM_UNION else torch.float32
    dev = nbr_idx.device
    deg = torch.empty(n, dtype=vdt, device=dev)
    # the library writes straight into torch-owned buffers sized for the
    # worst case (every row: k forward + k reverse entries + the diagonal)
    cap = n * (2 * k + 1)
    indptr = torch.empty(n + 1, dtype=torch.int64, device=dev)
    indices = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    values = torch.empty(max(cap, 1), dtype=vdt, device=dev)
    csr = _lib.Csr(n_rows=n, n_cols=n, nnz=cap, indptr=ptr(indptr).value,
                   indices=ptr(indices).value, values=ptr(values).value,
                   value_type=_lib.MN_F64 if sy == _lib.MN_SYM_UNION else _lib.MN_F32,
                   caller_owned=1)
    _lib.check(_lib.lib().mn_laplacian_from_knn(
        ptr(nbr_idx), ptr(nbr_val), 1 if nbr_val.dtype == torch.float64 else 0, n, k,
        C.byref(o), C.byref(csr), ptr(deg)))
    nnz = csr.nnz
    return CsrMatrix(indptr, indices[:nnz], values[:nnz], (n, n)), deg


def laplacian_stage_from_edges(nbr_idx: torch.Tensor, weights: torch.Tensor,
                               config: LaplacianConfig = LaplacianConfig()) -> LaplacianOutput:
    """LaplacianStage::execute steps 2-3 (surfface-core/src/laplacian.rs:179-227)
    given the top-k affinity rows (the Bhattacharyya scoring itself is §8(f))."""
    m, deg = build_laplacian_from_knn(nbr_idx, weights.float(), weight_kernel="given",
                                      symmetrise="max", normalize=config.normalize,
                                      weight_threshold=config.weight_threshold)
    f = nbr_idx.shape[0]
    nnz = _stage_c_nnz(nbr_idx, weights, deg, config)
    # laplacian.rs:187: `1.0 - (nnz as f32 / total as f32)`, all in f32
    sp = np.float32(1.0) - np.float32(np.float32(nnz) / np.float32(f * f))
    return LaplacianOutput(matrix=m, n_features=f, nnz=nnz, degrees=deg, sparsity=float(sp))


def _stage_c_nnz(nbr_idx: torch.Tensor, weights: torch.Tensor, deg: torch.Tensor,
                 config: LaplacianConfig) -> int:
    """The reference's nnz count (surfface-core/src/laplacian.rs:344-391): taken
    while the dense L is written, BEFORE the `|v| > 1e-9` filter of the CSR
    conversion (:215): the diagonal entries with d_i > thr plus 2 per
    undirected edge (key (min, max), i != j, w > thr), in normalized mode only
    the edges whose both degrees exceed thr."""
    thr = config.weight_threshold
    f = nbr_idx.shape[0]
    k = nbr_idx.shape[1]
    i = torch.arange(f, device=nbr_idx.device, dtype=torch.int64).repeat_interleave(k)
    j = nbr_idx.reshape(-1).to(torch.int64)
    w = weights.reshape(-1).float()
    keep = (j >= 0) & (j < f) & (i != j) & (w > thr)
    i, j = i[keep], j[keep]
    key = torch.unique(torch.minimum(i, j) * f + torch.maximum(i, j))
    a, b = key // f, key % f
    dg = deg.float()
    n_diag = int((dg > thr).sum().item())
    if config.normalize:
        n_edges = int(((dg[a] > thr) & (dg[b] > thr)).sum().item())
    else:
        n_edges = int(key.numel())
    return n_diag + 2 * n_edges


@on_device


def compute_bhattacharyya_weights(means: torch.Tensor, variances: torch.Tensor,
                                  config: LaplacianConfig = LaplacianConfig(), stream=None):
    """laplacian.rs:254-298: per feature node the k = min(k, F-1) largest
    Bhattacharyya coefficients > weight_threshold (BC desc, j asc).
    means/variances [C, F] (CentroidState layout) -> (idx [F, k] int32 (-1 pad),
    w [F, k] f32)."""
    means = require_cuda(means, torch.float32, "means", 2)
    variances = require_cuda(variances, torch.float32, "variances", 2)
    if means.shape != variances.shape:
        raise ValueError("means and variances must have the same [C, F] shape")
    c, f = means.shape
    k = config.k_neighbors
    idx = torch.empty((f, k), dtype=torch.int32, device=means.device)
    w = torch.empty((f, k), dtype=torch.float32, device=means.device)
    _lib.check(_lib.lib().mn_bc_knn_f32(ptr(means), ptr(variances), c, f, k,
                                        config.variance_regularizer, config.weight_threshold,
                                        ptr(idx), ptr(w), stream_handle(stream)))
    return idx, w


class LaplacianStage:
    """surfface-core/src/laplacian.rs:113-228 — Stage C, feature-space Laplacian."""

    def __init__(self, config: LaplacianConfig = LaplacianConfig()):
        self.config = config

    def execute(self, means: torch.Tensor, variances: torch.Tensor) -> LaplacianOutput:
        idx, w = compute_bhattacharyya_weights(means, variances, self.config)
        return laplacian_stage_from_edges(idx, w, self.config)
