"""Clustering stage mirror (surfface-pipeline/src/stages/clustering.rs:6-134).

The data-parallel step — every batch item's nearest current centroid by the
Gram-form distance sqrt(|x|^2 + |c|^2 - 2 x.c) (:42-63) — runs on the GPU
(mn_nearest_centroid_f32); the incremental centroid creation (:65-88) is the
reference's own host loop over the downloaded batch results, replayed here
in the same order (a centroid created inside a batch is not seen by the
rest of that batch, exactly as in the reference).  Parity of the distances
is pinned to the fixed-order restatement in the oracle (Burn's reduction
order is backend-defined).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle, on_device


@on_device
def nearest_centroid(batch: torch.Tensor, centroids: torch.Tensor, stream=None):
    """(idx [b] int32, dist [b] f32) of the nearest centroid per batch row."""
    batch = require_cuda(batch, torch.float32, "batch", 2)
    centroids = require_cuda(centroids, torch.float32, "centroids", 2)
    b, f = batch.shape
    if centroids.shape[1] != f:
        raise ValueError("batch and centroids must have the same feature dimension")
    idx = torch.empty(b, dtype=torch.int32, device=batch.device)
    dist = torch.empty(b, dtype=torch.float32, device=batch.device)
    _lib.check(_lib.lib().mn_nearest_centroid_f32(ptr(batch), b, ptr(centroids),
                                                  centroids.shape[0], f, ptr(idx), ptr(dist),
                                                  stream_handle(stream)))
    return idx, dist


@dataclass
class ClusteringOutput:
    """clustering.rs:12-16."""
    centroids: torch.Tensor    # [C, F] f32 (device)
    assignments: torch.Tensor  # [N] int64
    counts: torch.Tensor       # [C] int64


class ClusteringStage:
    """clustering.rs:6-10: target_centroids, radius (f32), batch_size."""

    def __init__(self, target_centroids: int, radius: float, batch_size: int):
        self.target_centroids = target_centroids
        self.radius = radius
        self.batch_size = batch_size

    def execute(self, data: torch.Tensor) -> ClusteringOutput:
        data = require_cuda(data, torch.float32, "data", 2)
        n, f = data.shape
        cents = [data[0:1]]              # first item is the first centroid (:27)
        cent_t = data[0:1].contiguous()
        assignments = []
        n_cent = 1
        rad = torch.tensor(self.radius, dtype=torch.float32).item()  # f32 compare (:75)
        for b0 in range(0, n, self.batch_size):
            b1 = min(b0 + self.batch_size, n)
            idx, dist = nearest_centroid(data[b0:b1].contiguous(), cent_t)
            idx_h = idx.cpu().tolist()
            dist_h = dist.cpu()
            added = []
            for i in range(b1 - b0):
                d = dist_h[i].item()
                if d < rad:
                    assignments.append(idx_h[i])
                elif n_cent < self.target_centroids:
                    added.append(b0 + i)
                    assignments.append(n_cent)
                    n_cent += 1
                else:
                    assignments.append(idx_h[i])
            if added:
                cents.append(data[added])
                cent_t = torch.cat(cents, 0).contiguous()
        a = torch.tensor(assignments, dtype=torch.int64)
        counts = torch.bincount(a, minlength=n_cent)  # compute_counts (:117-133)
        return ClusteringOutput(cent_t, a.to(data.device), counts.to(data.device))
