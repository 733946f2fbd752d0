"""Multi-process (world size 2, gloo, CPU) check of the row-sharded kNN exchange:
shard offsets, all-gather of queries, all-to-all of per-shard lists and the
(dist, id) merge reproduce the global exact kNN of the oracle.  The per-shard
kNN and the merge are CPU stand-ins here (the HIP ops are covered by -m gpu)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

N, D, K = 96, 8, 5


def _full_lists():
    import datagen
    X = datagen.uniform(N, D, seed=13)
    X[10] = X[40]  # exact ties across shards
    idx, dd = O.knn_l2sq(X, N - 1)  # every row's full sorted list (exact oracle arithmetic)
    return X, idx, dd


def _shard_knn_cpu(full_idx, full_d, c_off, n_loc):
    def fn(Q, C, k, c_offset):
        assert c_offset == c_off
        nq = Q.shape[0]
        oi = np.full((nq, k), -1, np.int32)
        od = np.full((nq, k), np.inf, np.float32)
        for q in range(nq):
            sel = (full_idx[q] >= c_offset) & (full_idx[q] < c_offset + n_loc)
            ii, dd = full_idx[q][sel][:k], full_d[q][sel][:k]
            oi[q, :len(ii)], od[q, :len(dd)] = ii, dd
        return torch.from_numpy(oi), torch.from_numpy(od)
    return fn


def _merge_cpu(pi, pd):
    P, nq, k = pi.shape
    pi, pd = pi.numpy(), pd.numpy()
    oi = np.full((nq, k), -1, np.int32)
    od = np.full((nq, k), np.inf, np.float32)
    for q in range(nq):
        c = [(pd[p, q, r], pi[p, q, r]) for p in range(P) for r in range(k) if pi[p, q, r] >= 0]
        c.sort()
        for r, (dv, iv) in enumerate(c[:k]):
            oi[q, r], od[q, r] = iv, dv
    return torch.from_numpy(oi), torch.from_numpy(od)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.join(os.path.dirname(here), "matternet-rs_amd"))
        from surfface_hip.dist import sharded_knn
        X, fi, fd = _full_lists()
        n_loc = N // world
        shard = torch.from_numpy(X[rank * n_loc:(rank + 1) * n_loc].copy())
        idx, dd = sharded_knn(shard, K, knn_fn=_shard_knn_cpu(fi, fd, rank * n_loc, n_loc),
                              merge_fn=_merge_cpu)
        out[rank] = (idx.numpy().tolist(), dd.numpy().tolist())
    finally:
        dist.destroy_process_group()


def test_sharded_knn_exchange_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    X, _, _ = _full_lists()
    ridx, rdist = O.knn_l2sq(X, K)
    got_i = np.concatenate([np.array(out[r][0]) for r in range(world)])
    got_d = np.concatenate([np.array(out[r][1], np.float32) for r in range(world)])
    np.testing.assert_array_equal(got_i, ridx)
    np.testing.assert_array_equal(got_d.view(np.uint32), rdist.view(np.uint32))
