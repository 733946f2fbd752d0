"""K3 — energy row reductions through the HIP C ABI (mn_energy_rows).

Host-side mirror of:
  * TauMode (src_legacy/taumode.rs:17-23; default Median, core.rs:409)
  * TauMode::compute_taumode_lambdas_parallel + ArrowSpace::update_lambdas /
    normalise_lambdas (taumode.rs:117-250, core.rs:1341-1354, 1427-1454)
      -> compute_taumode_lambdas()
  * node_energy_and_dispersion (energymaps.rs:923-1045) -> node_energy_and_dispersion()
  * ArrowSpace::normalise_lambdas                       -> normalise_lambdas()
Values within 1e-9 relative of the reference (it sums in rayon order).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle
from .laplacian import CsrMatrix


@dataclass(frozen=True)
class TauMode:
    """Fixed(t) | Median | Mean | Percentile(p)."""
    kind: int
    param: float = 0.0

    @staticmethod
    def Fixed(t: float) -> "TauMode":
        return TauMode(_lib.MN_TAU_FIXED, float(t))

    @staticmethod
    def Percentile(p: float) -> "TauMode":
        return TauMode(_lib.MN_TAU_PERCENTILE, float(p))


TauMode.Median = TauMode(_lib.MN_TAU_MEDIAN)
TauMode.Mean = TauMode(_lib.MN_TAU_MEAN)

TAU_FLOOR = 1e-10


def _csr_struct(L: CsrMatrix) -> _lib.Csr:
    if L.values.dtype != torch.float64:
        raise TypeError("the feature Laplacian must hold f64 values (legacy GraphLaplacian)")
    return _lib.Csr(n_rows=L.shape[0], n_cols=L.shape[1], nnz=L.nnz, indptr=ptr(L.indptr).value,
                    indices=ptr(L.indices).value, values=ptr(L.values).value,
                    value_type=_lib.MN_F64, reserved0=0)


def last_stats() -> dict:
    st = _lib.EnergyStats()
    _lib.check(_lib.lib().mn_energy_last_stats(C.byref(st)))
    return st.as_dict()


def energy_rows(X: torch.Tensor, L: CsrMatrix, g_mode: int = _lib.MN_G_TAUMODE,
                taumode: TauMode = TauMode.Median, timing: bool = False, stream=None):
    """Raw per-row (E, G, lambda) as f64 device tensors."""
    X = require_cuda(X, torch.float32, "X", 2)
    n, f = X.shape
    E = torch.empty(n, dtype=torch.float64, device=X.device)
    G = torch.empty(n, dtype=torch.float64, device=X.device)
    lam = torch.empty(n, dtype=torch.float64, device=X.device)
    o = _lib.EnergyOpts(g_mode=g_mode, tau_mode=taumode.kind, tau_param=taumode.param,
                        timing=1 if timing else 0, reserved0=0, stream=stream_handle(stream))
    csr = _csr_struct(L)
    _lib.check(_lib.lib().mn_energy_rows(C.byref(csr), ptr(X), n, f, C.byref(o), ptr(E), ptr(G),
                                         ptr(lam)))
    return E, G, lam


def normalise_lambdas(lam: torch.Tensor, stream=None):
    """In place; returns (min, max, range) as floats (core.rs:1341-1354)."""
    lam = require_cuda(lam, torch.float64, "lambdas", 1)
    out = (C.c_double * 3)()
    _lib.check(_lib.lib().mn_normalise_lambdas(ptr(lam), lam.numel(), out, stream_handle(stream)))
    return lam, float(out[0]), float(out[1]), float(out[2])


def compute_taumode_lambdas(X: torch.Tensor, L: CsrMatrix, taumode: TauMode = TauMode.Median,
                            normalise: bool = True):
    """Synthetic lambdas of every item (taumode.rs:117-250 then update_lambdas)."""
    _, _, lam = energy_rows(X, L, _lib.MN_G_TAUMODE, taumode)
    stats = None
    if normalise:
        lam, mn, mx, rg = normalise_lambdas(lam)
        stats = {"min": mn, "max": mx, "range": rg}
    return lam, stats


def node_energy_and_dispersion(X: torch.Tensor, L: CsrMatrix):
    """(lambda = Rayleigh E, G over j > i) per row (energymaps.rs:923-1045)."""
    E, G, _ = energy_rows(X, L, _lib.MN_G_ENERGYMAPS)
    return E, G
