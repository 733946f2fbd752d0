"""Device-memory plumbing via PyTorch-ROCm (allocation and streams only)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch


def require_cuda(t: torch.Tensor, dtype, name: str, ndim: int | None = None) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise TypeError(f"{name} must be a torch tensor on a ROCm device")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D")
    return t.contiguous()


def ptr(t: torch.Tensor) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


def stream_handle(stream=None) -> C.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def to_device(a, device="cuda") -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(device).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _first_cuda(args, kwargs):
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor) and a.device.type == "cuda":
            return a.device
        for v in (getattr(a, "indptr", None), getattr(a, "keys", None)):
            if isinstance(v, torch.Tensor) and v.device.type == "cuda":
                return v.device
    return None


def on_device(fn):
    """Run a wrapper with its first device tensor's GPU current, so the
    library's launches, scratch and the default stream (the current stream of
    that device) all land on the device that holds the data."""
    import functools

    @functools.wraps(fn)
    def wrapped(*args, **kwargs):
        dev = _first_cuda(args, kwargs)
        if dev is None or dev.index is None or dev.index == torch.cuda.current_device():
            return fn(*args, **kwargs)
        with torch.cuda.device(dev):
            return fn(*args, **kwargs)
    return wrapped
