"""K5 — sparsification through the HIP C ABI (mn_sparsify_rows).

Mirror of SfGrassSparsifier (src_legacy/sparsification.rs:14-113) and of the
inline pruning inside _build_adjacency (src_legacy/laplacian.rs:216-282).
Rows are directed neighbour lists [n][k] (idx -1 = empty).  Bit-exact; the
reference leaves score ties unspecified (sort_unstable): ties here keep the
input position order.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle, on_device


@on_device


def sparsify_rows(nbr_idx: torch.Tensor, nbr_w: torch.Tensor, ratio: float = 0.5,
                  mode: int = _lib.MN_SPARSIFY_SFGRASS, degrees: torch.Tensor = None,
                  stream=None):
    """Padded rows [n][k] (k <= 64).  degrees [n] int32 (None: the row lengths)
    feed the scores and the average-degree switch."""
    nbr_idx = require_cuda(nbr_idx, torch.int32, "nbr_idx", 2)
    nbr_w = require_cuda(nbr_w, torch.float64, "nbr_w", 2)
    n, k = nbr_idx.shape
    if degrees is not None:
        degrees = require_cuda(degrees, torch.int32, "degrees", 1)
        if degrees.shape[0] != n:
            raise ValueError("degrees must have one entry per row")
    oi = torch.empty_like(nbr_idx)
    ow = torch.empty_like(nbr_w)
    applied = C.c_int32(0)
    _lib.check(_lib.lib().mn_sparsify_rows(ptr(nbr_idx), ptr(nbr_w), n, k, ratio, mode,
                                           ptr(degrees) if degrees is not None else None,
                                           ptr(oi), ptr(ow), C.byref(applied),
                                           stream_handle(stream)))
    return oi, ow, bool(applied.value)


@on_device
def sparsify_sfgrass_csr(adj, ratio: float = 0.5, n_nodes: int = 0, stream=None):
    """SfGrassSparsifier::sparsify_graph (sparsification.rs:32-101) on CSR rows
    of any length: adj = CsrMatrix (f64 values) -> (CsrMatrix, applied)."""
    from .laplacian import CsrMatrix
    ip = require_cuda(adj.indptr, torch.int64, "indptr", 1)
    ix = require_cuda(adj.indices, torch.int32, "indices", 1)
    iv = require_cuda(adj.values, torch.float64, "values", 1)
    n = ip.shape[0] - 1
    src = _lib.Csr(n_rows=n, n_cols=adj.shape[1], nnz=ix.numel(), indptr=ptr(ip).value,
                   indices=ptr(ix).value if ix.numel() else None,
                   values=ptr(iv).value if iv.numel() else None, value_type=_lib.MN_F64,
                   caller_owned=1)
    # caller-owned output sized for the worst case (no pruning: nnz entries)
    cap = max(ix.numel(), 1)
    oip = torch.empty(n + 1, dtype=torch.int64, device=ip.device)
    oix = torch.empty(cap, dtype=torch.int32, device=ip.device)
    oiv = torch.empty(cap, dtype=torch.float64, device=ip.device)
    dst = _lib.Csr(n_rows=n, n_cols=adj.shape[1], nnz=cap, indptr=ptr(oip).value,
                   indices=ptr(oix).value, values=ptr(oiv).value, value_type=_lib.MN_F64,
                   caller_owned=1)
    applied = C.c_int32(0)
    _lib.check(_lib.lib().mn_sparsify_sfgrass(C.byref(src), n_nodes, ratio, C.byref(dst),
                                              C.byref(applied), stream_handle(stream)))
    nz = dst.nnz
    return CsrMatrix(oip, oix[:nz], oiv[:nz], tuple(adj.shape)), bool(applied.value)


class SfGrassSparsifier:
    """sparsification.rs:14-29: new() keeps 50%; with_target_ratio clamps to [0.1, 1]."""

    def __init__(self):
        self.target_ratio = 0.5

    def with_target_ratio(self, ratio: float) -> "SfGrassSparsifier":
        self.target_ratio = min(max(float(ratio), 0.1), 1.0)
        return self

    def sparsify_graph(self, nbr_idx, nbr_w=None, n_nodes: int = 0):
        """Padded rows (nbr_idx [n][k] int32, nbr_w [n][k] f64), or a CsrMatrix
        of rows of any length (nbr_w None) -> the same form, pruned."""
        if nbr_w is None:
            out, _ = sparsify_sfgrass_csr(nbr_idx, self.target_ratio, n_nodes)
            return out
        oi, ow, _ = sparsify_rows(nbr_idx, nbr_w, self.target_ratio, _lib.MN_SPARSIFY_SFGRASS)
        return oi, ow
