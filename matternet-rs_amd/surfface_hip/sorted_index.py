"""K4 — lambda-sorted index through the HIP C ABI (mn_sorted_index).

Mirror of SortedLambdas (src_legacy/sorted_index.rs:8-54): build_from(),
to_vec(), std_dev.  Order: ascending OrderedFloat(lambda), ties by the
decimal-string id — bit-exact given identical lambdas.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle


class SortedLambdas:
    def __init__(self):
        self.order = None   # int64 [n] item index at each rank (device)
        self.keys = None    # f64 [n] bucket key at each rank (device)
        self.std_dev = 0.0

    def build_from(self, lambdas: torch.Tensor, stream=None) -> "SortedLambdas":
        lam = require_cuda(lambdas, torch.float64, "lambdas", 1)
        n = lam.numel()
        if n == 0:
            raise ValueError("Cannot compute proper standard deviations for lambdas "
                             "(sorted_index.rs:33-39 panics on empty input)")
        self.order = torch.empty(n, dtype=torch.int64, device=lam.device)
        self.keys = torch.empty(n, dtype=torch.float64, device=lam.device)
        sd = C.c_double(0.0)
        _lib.check(_lib.lib().mn_sorted_index(ptr(lam), n, ptr(self.order), ptr(self.keys),
                                              C.byref(sd), stream_handle(stream)))
        self.std_dev = sd.value
        return self

    def to_vec(self):
        """[(lambda, idx)] in index order (sorted_index.rs:46-54)."""
        return list(zip(self.keys.cpu().tolist(), self.order.cpu().tolist()))
