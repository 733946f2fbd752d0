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
                  mode: int = _lib.MN_SPARSIFY_SFGRASS, stream=None):
    nbr_idx = require_cuda(nbr_idx, torch.int32, "nbr_idx", 2)
    nbr_w = require_cuda(nbr_w, torch.float64, "nbr_w", 2)
    n, k = nbr_idx.shape
    oi = torch.empty_like(nbr_idx)
    ow = torch.empty_like(nbr_w)
    applied = C.c_int32(0)
    _lib.check(_lib.lib().mn_sparsify_rows(ptr(nbr_idx), ptr(nbr_w), n, k, ratio, mode, ptr(oi),
                                           ptr(ow), C.byref(applied), stream_handle(stream)))
    return oi, ow, bool(applied.value)


class SfGrassSparsifier:
    """sparsification.rs:14-29: new() keeps 50%; with_target_ratio clamps to [0.1, 1]."""

    def __init__(self):
        self.target_ratio = 0.5

    def with_target_ratio(self, ratio: float) -> "SfGrassSparsifier":
        self.target_ratio = min(max(float(ratio), 0.1), 1.0)
        return self

    def sparsify_graph(self, nbr_idx: torch.Tensor, nbr_w: torch.Tensor):
        oi, ow, _ = sparsify_rows(nbr_idx, nbr_w, self.target_ratio, _lib.MN_SPARSIFY_SFGRASS)
        return oi, ow
