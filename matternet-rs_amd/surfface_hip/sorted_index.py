"""K4 — lambda-sorted index through the HIP C ABI (mn_sorted_index).

Mirror of SortedLambdas (src_legacy/sorted_index.rs:8-54): build_from(),
to_vec(), std_dev.  Order: ascending OrderedFloat(lambda), ties by the
decimal-string id — bit-exact given identical lambdas.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle, on_device


class SortedLambdas:
    def __init__(self):
        self.order = None   # int64 [n] item index at each rank (device)
        self.keys = None    # f64 [n] bucket key at each rank (device)
        self.std_dev = 0.0

    @on_device

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

    # ---- lambda-aware lookups (sorted_index.rs:64-140), batched on the GPU ----
    def _queries(self, lambda_q):
        if self.order is None:
            raise ValueError("build_from() first")
        scalar = not isinstance(lambda_q, torch.Tensor)
        q = torch.tensor([float(lambda_q)], dtype=torch.float64, device=self.order.device) \
            if scalar else require_cuda(lambda_q, torch.float64, "lambda_q", 1)
        return scalar, q

    def _outputs(self, nq, k):
        dev = self.order.device
        return (torch.empty((nq, max(k, 1)), dtype=torch.int64, device=dev),
                torch.empty((nq, max(k, 1)), dtype=torch.float64, device=dev),
                torch.empty(nq, dtype=torch.int32, device=dev))

    @on_device

    def range_bylambda(self, lambda_q, k: int, p: float):
        """Items with key in [lq - std/2^p, lq + std/2^p], index order, first k.
        Scalar query -> [(idx, lambda)]; tensor [nq] -> (idx [nq,k], lambda
        [nq,k], count [nq]) with count -1 where the reference panics."""
        scalar, q = self._queries(lambda_q)
        oi, ol, oc = self._outputs(q.numel(), k)
        _lib.check(_lib.lib().mn_sorted_range_bylambda(
            ptr(self.keys), ptr(self.order), self.order.numel(), self.std_dev, ptr(q), q.numel(),
            k, p, ptr(oi), ptr(ol), ptr(oc), stream_handle()))
        return self._result(scalar, oi, ol, oc, k, with_id=False)

    @on_device

    def k_nearest_by_lambda(self, lambda_q, k: int, lambda_p: float, base_delta=None,
                            growth: float = 1.7, max_multiplier: float = 10.0):
        """Expanding-window k nearest by |lambda - lq|; ties in index order.
        Scalar query -> [(idx, lambda, id)] as the reference; tensor [nq] ->
        (idx, lambda, count) tensors."""
        scalar, q = self._queries(lambda_q)
        oi, ol, oc = self._outputs(q.numel(), k)
        _lib.check(_lib.lib().mn_sorted_k_nearest_by_lambda(
            ptr(self.keys), ptr(self.order), self.order.numel(), self.std_dev, ptr(q), q.numel(),
            k, lambda_p, 0 if base_delta is None else 1,
            0.0 if base_delta is None else float(base_delta), growth, max_multiplier, ptr(oi),
            ptr(ol), ptr(oc), stream_handle()))
        return self._result(scalar, oi, ol, oc, k, with_id=True)

    @staticmethod
    def _result(scalar, oi, ol, oc, k, with_id):
        if not scalar:
            return oi[:, :k], ol[:, :k], oc
        c = int(oc[0].item())
        if c < 0:
            raise ValueError("the reference panics on this query (sorted_index.rs: BTreeMap::range "
                             "start > end, or NaN distances)")
        idx, lam = oi[0, :c].cpu().tolist(), ol[0, :c].cpu().tolist()
        return [(i, l, str(i)) if with_id else (i, l) for i, l in zip(idx, lam)]
