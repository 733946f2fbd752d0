"""K3 — energy row reductions through the HIP C ABI (mn_energy_rows).

Host-side mirror of:
  * TauMode (src_legacy/taumode.rs:17-23; default Median, core.rs:409)
  * TauMode::compute_taumode_lambdas_parallel + ArrowSpace::update_lambdas /
    normalise_lambdas (taumode.rs:117-250, core.rs:1341-1354, 1427-1454)
      -> compute_taumode_lambdas()
  * node_energy_and_dispersion (energymaps.rs:923-1045) -> node_energy_and_dispersion()
  * ArrowSpace::normalise_lambdas                       -> normalise_lambdas()
  * node_energy_and_dispersion on the item graph (X^T vs the n x n item
    Laplacian, SURVEY §8(d) orientation (ii))             -> signal_energy_and_dispersion()
  * EnergyMaps diffusion pre-pass (energymaps.rs:518-546)   -> diffuse_rows()
  * GraphLaplacian::multiply_vector (graph.rs:464-501)       -> laplacian_matvec_rows()
    (both bit-exact: f64 CSR row folds in stored order)
  * Stage D compute_lambdas_gpu / compute_tau_mode_gpu
    (surfface-core/src/spectral/mod.rs:158-181, bridge.rs:27-69)
      -> compute_lambdas_gpu() / compute_tau_mode_gpu()
Values within 1e-9 relative of the reference (it sums in rayon order); Stage D
within 1e-4 (the reference computes in f32 through Burn matmuls, this in f64).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle, on_device
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


def _csr_struct(L: CsrMatrix, allow_f32: bool = False) -> _lib.Csr:
    if L.values.dtype == torch.float32 and allow_f32:
        vt = _lib.MN_F32
    elif L.values.dtype == torch.float64:
        vt = _lib.MN_F64
    else:
        raise TypeError("the feature Laplacian must hold f64 values (legacy GraphLaplacian); "
                        "f32 (Stage C) only for the spectral lambdas")
    return _lib.Csr(n_rows=L.shape[0], n_cols=L.shape[1], nnz=L.nnz, indptr=ptr(L.indptr).value,
                    indices=ptr(L.indices).value, values=ptr(L.values).value,
                    value_type=vt, caller_owned=1)


def last_stats() -> dict:
    st = _lib.EnergyStats()
    _lib.check(_lib.lib().mn_energy_last_stats(C.byref(st)))
    return st.as_dict()


@on_device


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
    csr = _csr_struct(L, allow_f32=(g_mode == _lib.MN_G_SPECTRAL))
    _lib.check(_lib.lib().mn_energy_rows(C.byref(csr), ptr(X), n, f, C.byref(o), ptr(E), ptr(G),
                                         ptr(lam)))
    return E, G, lam


@on_device


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


def compute_lambdas_gpu(L: CsrMatrix, X: torch.Tensor):
    """Stage D device lambdas (spectral/mod.rs:158-181): per item the clamped
    Rayleigh quotient plus the globally normalised Dirichlet dispersion.
    Returns (lambda, rayleigh, dirichlet) as f64 device tensors."""
    R, D, lam = energy_rows(X, L, _lib.MN_G_SPECTRAL)
    return lam, R, D


def compute_tau_mode_gpu(laplacian, data: torch.Tensor, n_items: int = None,
                         n_features: int = None):
    """bridge.rs:27-69: Stage C output (LaplacianOutput or CsrMatrix, f32
    values) + the N x F item matrix -> f64 lambdas (no normalisation, as in
    the reference)."""
    L = getattr(laplacian, "matrix", laplacian)
    X = data if data.dim() == 2 else data.view(n_items, n_features)
    lam, _, _ = compute_lambdas_gpu(L, X)
    return lam


def _rows_in(X: torch.Tensor):
    if X.dtype not in (torch.float32, torch.float64):
        raise TypeError("X must be float32 or float64")
    X = require_cuda(X, X.dtype, "X", 2)
    return X, 1 if X.dtype == torch.float64 else 0


@on_device


def diffuse_rows(X: torch.Tensor, L: CsrMatrix, eta: float = 0.1, steps: int = 4,
                 out: torch.Tensor = None, stream=None) -> torch.Tensor:
    """`steps` x [x <- x - eta * L x] per row (EnergyParams defaults eta 0.1,
    steps 4, energymaps.rs:59-60); f64 result."""
    X, xf64 = _rows_in(X)
    n, f = X.shape
    out = torch.empty((n, f), dtype=torch.float64, device=X.device) if out is None else out
    csr = _csr_struct(L)
    _lib.check(_lib.lib().mn_diffuse_rows(C.byref(csr), ptr(X), xf64, n, f, eta, steps, ptr(out),
                                          stream_handle(stream)))
    return out


@on_device


def laplacian_matvec_rows(X: torch.Tensor, L: CsrMatrix, stream=None) -> torch.Tensor:
    """Y = L x per row (GraphLaplacian::multiply_vector); f64 result."""
    X, xf64 = _rows_in(X)
    n, f = X.shape
    Y = torch.empty((n, f), dtype=torch.float64, device=X.device)
    csr = _csr_struct(L)
    _lib.check(_lib.lib().mn_laplacian_matvec_rows(C.byref(csr), ptr(X), xf64, n, f, ptr(Y),
                                                   stream_handle(stream)))
    return Y


@on_device


def signal_energy_and_dispersion(X: torch.Tensor, L_items: CsrMatrix,
                                 g_mode: int = _lib.MN_G_ENERGYMAPS, stream=None):
    """node_energy_and_dispersion(X^T, L_items): the F feature signals (columns
    of X [n, F]) against the n x n item Laplacian -> (E [F], G [F]) f64."""
    X = require_cuda(X, torch.float32, "X", 2)
    n, f = X.shape
    E = torch.empty(f, dtype=torch.float64, device=X.device)
    G = torch.empty(f, dtype=torch.float64, device=X.device)
    csr = _csr_struct(L_items)
    _lib.check(_lib.lib().mn_energy_signals(C.byref(csr), ptr(X), n, f, g_mode, ptr(E), ptr(G),
                                            stream_handle(stream)))
    return E, G
