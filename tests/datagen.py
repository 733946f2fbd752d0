"""Seeded synthetic inputs shared by tests and bench.

uniform:   x[r, c] = 2 * ((splitmix64(seed ^ (r*d + c)) >> 40) * 2^-24) - 1
           (exact in f32, independent of sharding; the HIP library generates
           the identical stream on device via mn_fill_uniform_f32).
clustered: 64 Gaussian blobs (sigma 0.1) + ~1% exact duplicate rows +
           ~0.1% all-zero rows — the parity-stress distribution.
"""
from __future__ import annotations

import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(n: int, d: int, seed: int = 42, row0: int = 0) -> np.ndarray:
    r = np.arange(row0, row0 + n, dtype=np.uint64)[:, None]
    c = np.arange(d, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        ctr = (r * np.uint64(d) + c) ^ np.uint64(seed)
    u = (splitmix64(ctr) >> np.uint64(40)).astype(np.float64) * 2.0 ** -24
    return (2.0 * u - 1.0).astype(np.float32)


def clustered(n: int, d: int, seed: int = 7, blobs: int = 64, sigma: float = 0.1,
              dup_frac: float = 0.01, zero_frac: float = 0.001) -> np.ndarray:
    rng = np.random.default_rng(seed)
    centers = rng.uniform(-1.0, 1.0, size=(blobs, d)).astype(np.float32)
    lab = rng.integers(0, blobs, size=n)
    X = (centers[lab] + sigma * rng.standard_normal((n, d))).astype(np.float32)
    nd = max(1, int(round(n * dup_frac))) if dup_frac > 0 else 0
    if nd and n > 2:
        src = rng.integers(0, n, size=nd)
        dst = rng.integers(0, n, size=nd)
        X[dst] = X[src]
    nz = max(1, int(round(n * zero_frac))) if zero_frac > 0 else 0
    if nz and n > 2:
        X[rng.integers(0, n, size=nz)] = 0.0
    return np.ascontiguousarray(X)


def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """f32 -> bf16 round-to-nearest-even (finite inputs), returned as uint16."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << np.uint32(16)).view(np.float32)


def sorted_rows(n: int, d: int, kind: str, seed: int = 3) -> np.ndarray:
    """Adversarial row ORDERS for the two-phase generators: rows
    sorted so that the corpus order keeps improving every row's candidates.
      near_1d    — x = t v + 0.05 noise + 0.2 with t sorted (the original
                   stress case of the round-2 cosine test: almost every row's
                   neighbours are its index neighbours)
      projection — a normal cloud (+0.3) sorted by one random projection."""
    rng = np.random.default_rng(seed)
    if kind == "near_1d":
        t = np.sort(rng.uniform(-1.0, 1.0, n))
        v = rng.normal(size=d)
        return (np.outer(t, v) + 0.05 * rng.normal(size=(n, d)) + 0.2).astype(np.float32)
    if kind == "projection":
        X = rng.normal(size=(n, d)) + 0.3
        return X[np.argsort(X @ rng.normal(size=d))].astype(np.float32)
    raise ValueError(kind)
