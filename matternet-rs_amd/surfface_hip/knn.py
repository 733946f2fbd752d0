"""K1 — brute-force kNN through the HIP C ABI (mn_knn_f32 / _qc / merge).

Host-side mirror of the reference's kNN entry points:
  * surfface-core/src/mst.rs:312-412  MSTStage::build_candidate_graph with
    compute_distance / compute_edge_cost (every DistanceMetric, every
    ThicknessWeight)  -> build_candidate_graph()
  * surfface-core/src/distance.rs:78-108 bhattacharyya_distance_diagonal,
    :195-213 squared/euclidean distance
L2 results are bit-identical to the reference's sequential f32 fold + stable
sort; Bhattacharyya distances are bit-identical but for rare ulp-level log
terms (mst.hip header).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from enum import IntEnum

import torch

from . import _lib
from ._torch import ptr, require_cuda, stream_handle, to_device, on_device


class DistanceMetric(IntEnum):
    """surfface-core/src/mst.rs:45-54 (values = enum mn_mst_metric)."""
    Bhattacharyya = 0
    Euclidean = 1
    SquaredEuclidean = 2


class ThicknessWeight(IntEnum):
    """surfface-core/src/mst.rs:58-74 (values = enum mn_thickness_weight)."""
    Mean = 0
    Min = 1
    Max = 2
    GeometricMean = 3
    NoWeight = 4  # ThicknessWeight::None


@dataclass
class MSTConfig:
    """surfface-core/src/mst.rs:26-40, defaults :77-84 (the candidate-graph
    fields; compute_trunk belongs to the out-of-scope MST/trunk stage)."""
    k_neighbors: int = 8
    distance_metric: DistanceMetric = DistanceMetric.Bhattacharyya
    thickness_weight: ThicknessWeight = ThicknessWeight.Mean
    compute_trunk: bool = True

    @staticmethod
    def high_dimensional() -> "MSTConfig":
        return MSTConfig(k_neighbors=16)

    @staticmethod
    def prototype() -> "MSTConfig":
        return MSTConfig(4, DistanceMetric.SquaredEuclidean, ThicknessWeight.NoWeight, False)


@dataclass
class CandidateEdges:
    """The reference's Vec<Edge> (mst.rs:110-119) as device columns, edge
    e = i * k + r for node i's r-th nearest (u ascending, then distance, then v)."""
    u: torch.Tensor            # [E] int64
    v: torch.Tensor            # [E] int64
    distance: torch.Tensor     # [E] f32
    thickness_u: torch.Tensor  # [E] f32
    thickness_v: torch.Tensor  # [E] f32
    cost: torch.Tensor         # [E] f32
    thickness: torch.Tensor    # [C] f32 per-node thickness used


@dataclass
class KnnResult:
    idx: torch.Tensor    # [n, k] int32 (global ids; -1 = empty slot)
    dist: torch.Tensor   # [n, k] float32 (+inf = empty slot)
    stats: dict


ALGOS = {"auto": _lib.MN_KNN_AUTO, "f32": _lib.MN_KNN_F32, "bf16x3": _lib.MN_KNN_BF16X3,
         "bf16x1": _lib.MN_KNN_BF16X1}


def _opts(k, margin, timing, stream, exclude_self=True, metric=_lib.MN_L2SQ, algo="auto"):
    return _lib.KnnOpts(k=k, metric=metric, exclude_self=1 if exclude_self else 0,
                        margin=margin, timing=1 if timing else 0, algo=ALGOS[algo],
                        stream=stream_handle(stream))


def last_stats() -> dict:
    st = _lib.KnnStats()
    _lib.check(_lib.lib().mn_knn_last_stats(C.byref(st)))
    return st.as_dict()


@on_device


def knn_l2sq(X: torch.Tensor, k: int, margin: int = 16, timing: bool = False,
             stream=None, out_idx=None, out_dist=None, algo: str = "auto",
             euclidean: bool = False) -> KnnResult:
    """Exact kNN of every row of X [n, d] (f32, on device) by squared L2
    (euclidean=True: DistanceMetric::Euclidean, the correctly rounded sqrt of
    the same fold, computed in the library).  algo picks the candidate
    generator ("auto": "bf16x1" for corpora >= 2^17 rows, else "bf16x3" when
    k + margin <= 64, else "f32"); the result is the same bit for bit."""
    X = require_cuda(X, torch.float32, "X", 2)
    n, d = X.shape
    idx = out_idx if out_idx is not None else torch.empty((n, k), dtype=torch.int32, device=X.device)
    dist = out_dist if out_dist is not None else torch.empty((n, k), dtype=torch.float32, device=X.device)
    o = _opts(k, margin, timing, stream, algo=algo,
              metric=_lib.MN_L2 if euclidean else _lib.MN_L2SQ)
    _lib.check(_lib.lib().mn_knn_f32(ptr(X), n, d, C.byref(o), ptr(idx), ptr(dist)))
    return KnnResult(idx, dist, last_stats())


@on_device


def knn_l2sq_qc(Qm: torch.Tensor, Cm: torch.Tensor, k: int, q_offset: int = 0, c_offset: int = 0,
                exclude_self: bool = True, margin: int = 16, timing: bool = False,
                stream=None, algo: str = "auto") -> KnnResult:
    """Exact per-shard top-k of queries Q against corpus C (global-id offsets)."""
    Qm = require_cuda(Qm, torch.float32, "Q", 2)
    Cm = require_cuda(Cm, torch.float32, "C", 2)
    nq, d = Qm.shape
    nc, d2 = Cm.shape
    if d != d2:
        raise ValueError("Q and C must have the same feature dimension")
    idx = torch.empty((nq, k), dtype=torch.int32, device=Qm.device)
    dist = torch.empty((nq, k), dtype=torch.float32, device=Qm.device)
    o = _opts(k, margin, timing, stream, exclude_self, algo=algo)
    _lib.check(_lib.lib().mn_knn_f32_qc(ptr(Qm), nq, ptr(Cm), nc, d, q_offset, c_offset,
                                        C.byref(o), ptr(idx), ptr(dist)))
    return KnnResult(idx, dist, last_stats())


@on_device


def merge_parts(part_idx: torch.Tensor, part_dist: torch.Tensor, stream=None):
    """Merge P exact per-shard lists [P, nq, k] into the global top-k."""
    part_idx = require_cuda(part_idx, torch.int32, "part_idx", 3)
    part_dist = require_cuda(part_dist, torch.float32, "part_dist", 3)
    P, nq, k = part_idx.shape
    idx = torch.empty((nq, k), dtype=torch.int32, device=part_idx.device)
    dist = torch.empty((nq, k), dtype=torch.float32, device=part_idx.device)
    _lib.check(_lib.lib().mn_knn_merge_f32(ptr(part_idx), ptr(part_dist), P, nq, k, ptr(idx),
                                           ptr(dist), stream_handle(stream)))
    return idx, dist


@on_device
def build_candidate_graph(means, variances=None, k_neighbors: int = 8,
                          metric: DistanceMetric = DistanceMetric.Bhattacharyya,
                          thickness_weight: ThicknessWeight = ThicknessWeight.Mean,
                          thickness=None, stream=None) -> CandidateEdges:
    """Mirror of MSTStage::build_candidate_graph (mst.rs:312-363) with
    compute_distance (:366-397) and compute_edge_cost (:400-412), through
    mn_mst_candidate_graph_f32.  means / variances [C, F] (the CentroidState
    rows); thickness [C] or None = the mean variance per centroid
    (centroid.rs:107-109).  k = min(k_neighbors, C - 1) edges per node."""
    X = to_device(means).float().contiguous()
    require_cuda(X, torch.float32, "means", 2)
    c, f = X.shape
    V = None
    if variances is not None:
        V = to_device(variances).float().contiguous().to(X.device)
        if tuple(V.shape) != (c, f):
            raise ValueError("variances must have the shape of means")
    if c < 2:
        raise ValueError("build_candidate_graph needs at least 2 centroids (the reference "
                         "computes k = min(k, C - 1) and indexes thickness)")
    T = None
    if thickness is not None:
        T = to_device(thickness).float().contiguous().to(X.device)
    kk = min(k_neighbors, c - 1)
    v = torch.empty((c, kk), dtype=torch.int32, device=X.device)
    dist = torch.empty((c, kk), dtype=torch.float32, device=X.device)
    cost = torch.empty((c, kk), dtype=torch.float32, device=X.device)
    th = torch.empty(c, dtype=torch.float32, device=X.device)
    _lib.check(_lib.lib().mn_mst_candidate_graph_f32(
        ptr(X), ptr(V) if V is not None else None, c, f, k_neighbors, int(metric),
        int(thickness_weight), ptr(T) if T is not None else None, ptr(th), ptr(v), ptr(dist),
        ptr(cost), stream_handle(stream)))
    u = torch.arange(c, device=X.device, dtype=torch.int64).repeat_interleave(kk)
    vv = v.reshape(-1).to(torch.int64)
    return CandidateEdges(u, vv, dist.reshape(-1), th[u], th[vv], cost.reshape(-1), th)


def cos_last_stats() -> dict:
    st = _lib.KnnStats()
    _lib.check(_lib.lib().mn_cos_last_stats(C.byref(st)))
    return st.as_dict()


@on_device


def knn_cos_columns(X: torch.Tensor, topk: int, eps: float = 1.0, sigma: float = 1.0,
                    p: float = 2.0, margin: int = 16, timing: bool = False, stream=None):
    """Rectified-cosine kNN of the FEATURE columns of X [n, f] (each column is a
    node with an n-long profile; graph.rs:214 transposes the centroids).
    Returns (idx [f, topk] int32, dist [f, topk] f64, w [f, topk] f64, stats);
    bit-exact vs test_helpers.rs:77-126 semantics."""
    X = require_cuda(X, torch.float32, "X", 2)
    n, f = X.shape
    idx = torch.empty((f, topk), dtype=torch.int32, device=X.device)
    dist = torch.empty((f, topk), dtype=torch.float64, device=X.device)
    w = torch.empty((f, topk), dtype=torch.float64, device=X.device)
    o = _lib.CosOpts(topk=topk, margin=margin, eps=eps, sigma=sigma, p=p,
                     timing=1 if timing else 0, reserved0=0, stream=stream_handle(stream))
    _lib.check(_lib.lib().mn_knn_cos_columns_f32(ptr(X), n, f, C.byref(o), ptr(idx), ptr(dist),
                                                 ptr(w)))
    return idx, dist, w, cos_last_stats()


def bf16_last_stats() -> dict:
    st = _lib.KnnStats()
    _lib.check(_lib.lib().mn_bf16_last_stats(C.byref(st)))
    return st.as_dict()


@on_device


def knn_cos_bf16(X: torch.Tensor, topk: int, eps: float = 1.0, sigma: float = 1.0,
                 p: float = 2.0, margin: int = 16, timing: bool = False, stream=None):
    """Item graph of config 5: rectified-cosine kNN over the ROWS of a bf16
    matrix X [n, d] — the legacy adjacency builder's distance, weight, filter and
    (dist, j) order (src_legacy/laplacian.rs:245-290, test_helpers.rs:77-126) on
    the exactly widened values.  Returns (idx [n, topk] int32 (-1 empty),
    dist [n, topk] f64, w [n, topk] f64, stats); bit-exact."""
    X = require_cuda(X, torch.bfloat16, "X", 2)
    n, d = X.shape
    idx = torch.empty((n, topk), dtype=torch.int32, device=X.device)
    dist = torch.empty((n, topk), dtype=torch.float64, device=X.device)
    w = torch.empty((n, topk), dtype=torch.float64, device=X.device)
    o = _lib.CosOpts(topk=topk, margin=margin, eps=eps, sigma=sigma, p=p,
                     timing=1 if timing else 0, reserved0=0, stream=stream_handle(stream))
    _lib.check(_lib.lib().mn_knn_cos_bf16(ptr(X), n, d, C.byref(o), ptr(idx), ptr(dist), ptr(w)))
    return idx, dist, w, bf16_last_stats()


@on_device


def knn_cos_bf16_qc(Q: torch.Tensor, C_: torch.Tensor, topk: int, q_offset: int = 0,
                    c_offset: int = 0, eps: float = 1.0, sigma: float = 1.0, p: float = 2.0,
                    margin: int = 16, timing: bool = False, stream=None):
    """Row-shard form of knn_cos_bf16 (queries Q vs corpus shard C_, global ids)."""
    Q = require_cuda(Q, torch.bfloat16, "Q", 2)
    C_ = require_cuda(C_, torch.bfloat16, "C", 2)
    if Q.shape[1] != C_.shape[1]:
        raise ValueError("Q and C must have the same feature dimension")
    nq, d = Q.shape
    idx = torch.empty((nq, topk), dtype=torch.int32, device=Q.device)
    dist = torch.empty((nq, topk), dtype=torch.float64, device=Q.device)
    w = torch.empty((nq, topk), dtype=torch.float64, device=Q.device)
    o = _lib.CosOpts(topk=topk, margin=margin, eps=eps, sigma=sigma, p=p,
                     timing=1 if timing else 0, reserved0=0, stream=stream_handle(stream))
    _lib.check(_lib.lib().mn_knn_cos_bf16_qc(ptr(Q), nq, ptr(C_), C_.shape[0], d, q_offset,
                                             c_offset, C.byref(o), ptr(idx), ptr(dist), ptr(w)))
    return idx, dist, w, bf16_last_stats()
