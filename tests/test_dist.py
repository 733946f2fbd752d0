"""Multi-process (world size 2 and 3, gloo, CPU) check of the row-sharded kNN
exchange: shard offsets, all-gather of the shards, all-to-all of the lists and
the (dist, id) merge reproduce the global exact kNN of the oracle — for the
per-shard form and for the symmetric form, whose stand-in share takes exactly
the pairs of the rank's share of the library's node-wide tile table
(mn_sym_share_table, the schedule mn_knn_sharded_f32 runs).  The kernels are
CPU stand-ins here (the HIP stages are covered by -m gpu)."""
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


TILE = 8  # rows per tile of the stand-in share (the kernel's is 256)


def _sym_share_cpu(full_idx, full_d):
    """Stand-in for stage B: per row, the exact top-k over the pairs of the
    tiles in this rank's share of the table (both directions off the diagonal)."""
    n = full_idx.shape[0]
    Dm = np.full((n, n), np.inf, np.float32)
    for q in range(n):
        Dm[q, full_idx[q]] = full_d[q]

    def fn(Xall, k, rank, world):
        from surfface_hip.dist import share_table
        nbk = (n + TILE - 1) // TILE
        mask = np.zeros((n, n), bool)
        for I, Jf, cnt, st in share_table(nbk, rank, world):
            for t in range(cnt):
                J = Jf + t * st
                a = slice(I * TILE, min(n, I * TILE + TILE))
                b = slice(J * TILE, min(n, J * TILE + TILE))
                mask[a, b] = True
                mask[b, a] = True
        np.fill_diagonal(mask, False)
        oi = np.full((n, k), -1, np.int32)
        od = np.full((n, k), np.inf, np.float32)
        for q in range(n):
            js = np.nonzero(mask[q])[0]
            order = sorted(zip(Dm[q, js].tolist(), js.tolist()))[:k]
            for r, (dv, jv) in enumerate(order):
                oi[q, r], od[q, r] = jv, dv
        return torch.from_numpy(oi), torch.from_numpy(od)
    return fn


def _sym_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.join(os.path.dirname(here), "matternet-rs_amd"))
        from surfface_hip.dist import sharded_knn_sym
        X, fi, fd = _full_lists()
        n_loc = N // world
        shard = torch.from_numpy(X[rank * n_loc:(rank + 1) * n_loc].copy())
        idx, dd = sharded_knn_sym(shard, K, _sym_share_cpu(fi, fd),
                                  lambda pi, pd, row0: _merge_cpu(pi, pd))
        out[rank] = (idx.numpy().tolist(), dd.numpy().tolist())
    finally:
        dist.destroy_process_group()


def _run(worker, world):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(worker, args=(world, port, out), nprocs=world, join=True)
    X, _, _ = _full_lists()
    ridx, rdist = O.knn_l2sq(X, K)
    got_i = np.concatenate([np.array(out[r][0]) for r in range(world)])
    got_d = np.concatenate([np.array(out[r][1], np.float32) for r in range(world)])
    np.testing.assert_array_equal(got_i, ridx)
    np.testing.assert_array_equal(got_d.view(np.uint32), rdist.view(np.uint32))


def test_symmetric_schedule_exchange_world2():
    _run(_sym_worker, 2)


def test_symmetric_schedule_exchange_world3():
    _run(_sym_worker, 3)


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
