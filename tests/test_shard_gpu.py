"""Row-sharded kNN on one GPU: the C4 exchange simulated with
8 shards through mn_knn_f32_qc + mn_knn_merge_f32 at the C2 size, and the C
entry mn_knn_sharded_f32 on a single-rank RCCL communicator.  Both must be
bit-identical to the unsharded graph."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _uniform(n, d, seed=42):
    import surfface_hip as S
    X = torch.empty((n, d), dtype=torch.float32, device="cuda")
    S._lib.check(S.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, seed, 0,
                                             torch.cuda.current_stream().cuda_stream))
    return X


def test_eight_simulated_shards_at_c2_size_bit_exact():
    import surfface_hip as S
    n, d, k, R = 1_000_000, 768, 32, 8
    X = _uniform(n, d)
    full = S.knn_l2sq(X, k)
    n_loc = n // R
    parts_i, parts_d = [], []
    for r in range(R):
        res = S.knn_l2sq_qc(X, X[r * n_loc:(r + 1) * n_loc], k, q_offset=0, c_offset=r * n_loc)
        parts_i.append(res.idx)
        parts_d.append(res.dist)
    idx, dist = S.merge_parts(torch.stack(parts_i), torch.stack(parts_d))
    assert torch.equal(idx, full.idx)
    assert torch.equal(dist.view(torch.int32), full.dist.view(torch.int32))


def test_capi_sharded_entry_single_rank():
    import surfface_hip as S
    from surfface_hip.dist import RcclComm, knn_sharded_capi
    X = _uniform(50_000, 96, seed=3)
    comm = RcclComm(RcclComm.unique_id(), 1, 0)
    try:
        idx, dist = knn_sharded_capi(X, 16, comm, query_chunk=20_000)
    finally:
        comm.close()
    full = S.knn_l2sq(X, 16)
    assert torch.equal(idx, full.idx)
    assert torch.equal(dist.view(torch.int32), full.dist.view(torch.int32))


def test_c4_one_rank_share_8m_queries_vs_1m_shard():
    """Config 4 (8M x 768, k=32, 8 GPUs), ONE rank's full share on one GPU:
    all 8M queries (the all-gathered X) against rank 7's resident 1M-row shard
    (global ids 7M..8M-1), through the same 2M-query mn_knn_f32_qc chunks the
    multi-GPU path runs (surfface_hip/dist.py, bench.py knn_fn).  64 sampled
    queries (16 inside the shard: self excluded) bit-exact vs the oracle's
    per-shard form; time and device memory recorded."""
    import json
    import time

    import surfface_hip as S
    from oracle import oracle as O
    n_tot, d, k, R, rank, chunk = 8_000_000, 768, 32, 8, 7, 2_000_000
    n_loc = n_tot // R
    c_off = rank * n_loc
    stream = torch.cuda.current_stream().cuda_stream
    Xall = torch.empty((n_tot, d), dtype=torch.float32, device="cuda")
    for r0 in range(0, n_tot, n_loc):  # the same counter stream as every rank's shard
        S._lib.check(S.lib().mn_fill_uniform_f32(Xall[r0:r0 + n_loc].data_ptr(), n_loc, d, 42,
                                                 r0, stream))
    shard = Xall[c_off:c_off + n_loc]
    idx = torch.empty((n_tot, k), dtype=torch.int32, device="cuda")
    dist = torch.empty((n_tot, k), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    free0, total = torch.cuda.mem_get_info()
    t0 = time.perf_counter()
    stats = []
    for a0 in range(0, n_tot, chunk):
        r = S.knn_l2sq_qc(Xall[a0:a0 + chunk], shard, k, q_offset=a0, c_offset=c_off, timing=True)
        idx[a0:a0 + chunk].copy_(r.idx)
        dist[a0:a0 + chunk].copy_(r.dist)
        stats.append(r.stats)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    free1, _ = torch.cuda.mem_get_info()
    rec = {"s_total": round(el, 2), "pairs_per_s": n_tot * n_loc / el,
           "device_used_gb_after": round((total - free1) / 2**30, 1),
           "device_used_gb_inputs": round((total - free0) / 2**30, 1),
           "chunks": [{kk: (round(v, 1) if isinstance(v, float) else v)
                       for kk, v in st.items() if kk in ("ms_total", "ms_sweep", "ms_sample",
                                                          "n_uncertified", "n_escalated",
                                                          "n_candidates")} for st in stats]}
    print("C4 one-rank share", json.dumps(rec))
    rng = np.random.default_rng(4)
    q = np.concatenate([rng.choice(c_off, 48, replace=False),
                        c_off + rng.choice(n_loc, 16, replace=False)]).astype(np.int64)
    qsel = torch.from_numpy(q).cuda()
    Qh = Xall[qsel].cpu().numpy()
    Ch = shard.cpu().numpy()
    ri, rd = O.knn_l2sq_qc(Qh, q, Ch, c_off, k)
    np.testing.assert_array_equal(idx[qsel].cpu().numpy(), ri)
    np.testing.assert_array_equal(dist[qsel].cpu().numpy().view(np.uint32), rd.view(np.uint32))
    # rows no certificate settles are rescanned exactly: a handful in 8M
    assert sum(st["n_uncertified"] for st in stats) <= 32
    # properties on every row: sorted, ids inside the shard, no self pair
    assert bool((dist[:, 1:] >= dist[:, :-1]).all())
    assert int(idx.min()) >= c_off and int(idx.max()) < c_off + n_loc
    own = torch.arange(c_off, c_off + n_loc, device="cuda", dtype=torch.int32)[:, None]
    assert not bool((idx[c_off:c_off + n_loc] == own).any())
