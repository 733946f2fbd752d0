"""Row-sharded multi-GPU kNN graph build, one process per GPU.

The production entry is the library's mn_knn_sharded_f32 (knn_sharded_capi
below: RCCL inside the library).  Its symmetric form — each rank sweeps its
share of the node-wide symmetric tile table (mn_sym_share_table), the partial
lists of every row go to the row's owner, which merges and certifies them — is
mirrored by sharded_knn_sym over torch.distributed, so the exchange pattern
runs under `gloo` on the CPU with stand-in stages (tests/test_dist.py).

The per-shard form (sharded_knn):

Rank r owns rows [r*n_loc, (r+1)*n_loc) of X as its corpus shard (resident).
1. all-gather the query rows (every row of X) over RCCL/xGMI;
2. exact per-shard top-k of ALL queries against the local shard
   (mn_knn_f32_qc with global-id offsets: certified per shard);
3. one all-to-all: each query's owner receives the R per-shard lists of its rows;
4. merge by (dist, global id) (mn_knn_merge_f32) -> the owner's rows of the graph.
Exact: the global top-k is contained in the union of exact per-shard top-k lists and
a pair's distance is the same arithmetic on every shard.

`knn_fn` / `merge_fn` default to the HIP ops; tests inject CPU stand-ins to check the
exchange pattern under the `gloo` backend.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def sharded_knn(X_shard: torch.Tensor, k: int, knn_fn=None, merge_fn=None, group=None):
    """Returns (idx [n_loc, k] int32 global ids, dist [n_loc, k] f32) for this rank's rows."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_loc, d = X_shard.shape
    if knn_fn is None or merge_fn is None:
        from .knn import knn_l2sq_qc, merge_parts
        knn_fn = knn_fn or (lambda Q, C, kk, c_off: (lambda r: (r.idx, r.dist))(
            knn_l2sq_qc(Q, C, kk, q_offset=0, c_offset=c_off)))
        merge_fn = merge_fn or merge_parts
    sizes = [torch.zeros(1, dtype=torch.int64, device=X_shard.device) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([n_loc], dtype=torch.int64, device=X_shard.device),
                    group=group)
    if any(int(s.item()) != n_loc for s in sizes):
        raise ValueError("sharded_knn: every rank must hold the same number of rows")
    Xall = torch.empty((world * n_loc, d), dtype=X_shard.dtype, device=X_shard.device)
    dist.all_gather_into_tensor(Xall, X_shard.contiguous(), group=group)
    part_i, part_d = knn_fn(Xall, X_shard, k, rank * n_loc)   # [world*n_loc, k] each
    recv_i = torch.empty((world, n_loc, k), dtype=part_i.dtype, device=part_i.device)
    recv_d = torch.empty((world, n_loc, k), dtype=part_d.dtype, device=part_d.device)
    dist.all_to_all_single(recv_i.view(world, -1), part_i.contiguous().view(world, -1), group=group)
    dist.all_to_all_single(recv_d.view(world, -1), part_d.contiguous().view(world, -1), group=group)
    return merge_fn(recv_i, recv_d)


def share_table(nbk: int, rank: int, world: int):
    """mn_sym_share_table: rank's entries (I, Jfirst, tiles, stride) of the
    node-wide symmetric tile table over nbk row blocks (host only)."""
    import ctypes as C
    import numpy as np
    from . import _lib
    n = C.c_int64()
    _lib.check(_lib.lib().mn_sym_share_table(nbk, rank, world, None, 0, C.byref(n)))
    out = np.zeros((max(n.value, 1), 4), np.int32)
    _lib.check(_lib.lib().mn_sym_share_table(nbk, rank, world, out.ctypes.data_as(C.c_void_p),
                                             n.value, C.byref(n)))
    return out[:n.value]


def sharded_knn_sym(X_shard: torch.Tensor, k: int, share_fn, finish_fn, group=None):
    """The symmetric form's exchange (mn_knn_sharded_f32, shard.hip): all-gather
    of the shards, share_fn(Xall, k, rank, world) -> this rank's partial lists of
    ALL rows [N, k] (the exact top-k of the pairs in its share of the tile table),
    one all-to-all so each row's owner holds the R partial lists, finish_fn(parts_idx
    [R, n_loc, k], parts_dist, row0) -> the owner's rows (merge + certify)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_loc, d = X_shard.shape
    Xall = torch.empty((world * n_loc, d), dtype=X_shard.dtype, device=X_shard.device)
    dist.all_gather_into_tensor(Xall, X_shard.contiguous(), group=group)
    part_i, part_d = share_fn(Xall, k, rank, world)
    recv_i = torch.empty((world, n_loc, k), dtype=part_i.dtype, device=part_i.device)
    recv_d = torch.empty((world, n_loc, k), dtype=part_d.dtype, device=part_d.device)
    dist.all_to_all_single(recv_i.view(world, -1), part_i.contiguous().view(world, -1), group=group)
    dist.all_to_all_single(recv_d.view(world, -1), part_d.contiguous().view(world, -1), group=group)
    return finish_fn(recv_i, recv_d, rank * n_loc)


# ---- the same build behind the library's C entry (caller-owned RCCL comm) ----

_QUIESCE_AT_EXIT = []


def quiesce(timeout_s: float = 60.0) -> None:
    """mn_shard_quiesce: wait for the background release of failed sharded
    calls (their communicators aborted, their buffers freed once the device
    work queued on them drained)."""
    from . import _lib
    _lib.check(_lib.lib().mn_shard_quiesce(float(timeout_s)))


def _quiesce_at_exit():
    from . import _lib
    for L in list(_lib._LOADED.values()):
        L.mn_shard_quiesce(60.0)


class RcclComm:
    """An RCCL communicator created through the library (mn_rccl_comm_init):
    rank 0 makes the 128-byte id (`unique_id()`), every rank passes it here."""

    def __init__(self, uid: bytes, world: int, rank: int):
        import atexit
        import ctypes as C
        from . import _lib
        if not _QUIESCE_AT_EXIT:  # no release thread may outlive the process's GPU state
            atexit.register(_quiesce_at_exit)
            _QUIESCE_AT_EXIT.append(True)
        self._lib = _lib
        buf = C.create_string_buffer(bytes(uid), 128)
        h = C.c_void_p()
        _lib.check(_lib.lib().mn_rccl_comm_init(buf, world, rank, C.byref(h)))
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C
        from . import _lib
        buf = C.create_string_buffer(128)
        _lib.check(_lib.lib().mn_rccl_unique_id(buf))
        return buf.raw

    def close(self):
        if self.handle:
            self._lib.check(self._lib.lib().mn_rccl_comm_destroy(self.handle))
            self.handle = None


def set_collective_timeout(seconds: float) -> None:
    """mn_rccl_set_timeout: the deadline of one collective of
    mn_knn_sharded_f32 (process-wide; past it the communicator is aborted and
    the call raises MN_ECOMM)."""
    from . import _lib
    _lib.check(_lib.lib().mn_rccl_set_timeout(float(seconds)))


def knn_sharded_capi(X_shard: torch.Tensor, k: int, comm: RcclComm, query_chunk: int = 0,
                     margin: int = 16, timing: bool = False, stream=None):
    """mn_knn_sharded_f32: this rank's rows of the global exact kNN graph
    (idx [n_loc, k] int32 global ids, dist [n_loc, k] f32)."""
    import ctypes as C
    from . import _lib
    from ._torch import ptr, require_cuda, stream_handle
    X_shard = require_cuda(X_shard, torch.float32, "X_shard", 2)
    n, d = X_shard.shape
    idx = torch.empty((n, k), dtype=torch.int32, device=X_shard.device)
    dd = torch.empty((n, k), dtype=torch.float32, device=X_shard.device)
    o = _lib.KnnOpts(k=k, metric=_lib.MN_L2SQ, exclude_self=1, margin=margin,
                     timing=1 if timing else 0, algo=_lib.MN_KNN_AUTO,
                     stream=stream_handle(stream))
    _lib.check(_lib.lib().mn_knn_sharded_f32(ptr(X_shard), n, d, comm.handle, C.byref(o),
                                             query_chunk, ptr(idx), ptr(dd)))
    return idx, dd


def knn_sharded_sim(X_all: torch.Tensor, k: int, world: int, timing: bool = False, stream=None,
                    algo: int | None = None, threads: bool = False):
    """mn_knn_sharded_sim_f32: the sharded build of `world` ranks on this
    device — mn_knn_sharded_f32's driver over the loopback transport (X_all =
    the shards, rank r's at r * n / world).  `algo` (default AUTO) picks the
    form as the RCCL entry would: AUTO / BF16X1 the symmetric form, F32 /
    BF16X3 the per-shard form.  Returns (idx [n, k] int32, dist [n, k] f32,
    rank_ms [world][3] = per rank the stage A / B / C milliseconds, stats).
    threads=True: mn_knn_sharded_threads_f32 — one host thread per rank, the
    ranks concurrent, every collective checked for the same order on every
    rank (a divergence raises MN_ECOMM instead of hanging)."""
    import ctypes as C
    import numpy as np
    from . import _lib
    from ._torch import ptr, require_cuda, stream_handle
    from .knn import last_stats
    X_all = require_cuda(X_all, torch.float32, "X_all", 2)
    n, d = X_all.shape
    idx = torch.empty((n, k), dtype=torch.int32, device=X_all.device)
    dd = torch.empty((n, k), dtype=torch.float32, device=X_all.device)
    ms = np.zeros((world, 3), dtype=np.float32)
    o = _lib.KnnOpts(k=k, metric=_lib.MN_L2SQ, exclude_self=1, margin=0,
                     timing=1 if timing else 0,
                     algo=_lib.MN_KNN_AUTO if algo is None else algo,
                     stream=stream_handle(stream))
    fn = _lib.lib().mn_knn_sharded_threads_f32 if threads else _lib.lib().mn_knn_sharded_sim_f32
    _lib.check(fn(ptr(X_all), n, d, world, C.byref(o), ptr(idx), ptr(dd),
                  ms.ctypes.data_as(C.c_void_p)))
    return idx, dd, ms, last_stats()
