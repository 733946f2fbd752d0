"""Row-sharded kNN on one GPU: the symmetric sharded build
(mn_knn_sharded_sim_f32: every rank's stages in turn, the exchange a strided
read) at the C2 size and at the full C4 size, the per-shard form
(mn_knn_f32_qc + mn_knn_merge_f32) it falls back to, and the C entry
mn_knn_sharded_f32 on a single-rank RCCL communicator.  All bit-identical to
the unsharded graph."""
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
    """The symmetric sharded schedule with 8 ranks at the C2 size: every tile
    of the node-wide table on exactly one rank, partial lists merged and
    certified by the rows' owners — the unsharded graph bit for bit."""
    import json

    import surfface_hip as S
    from surfface_hip.dist import knn_sharded_sim
    n, d, k, R = 1_000_000, 768, 32, 8
    X = _uniform(n, d)
    full = S.knn_l2sq(X, k)
    idx, dist, ms, st = knn_sharded_sim(X, k, R, timing=True)
    print("C2 as 8 simulated ranks", json.dumps({"rank_ms": ms.round(2).tolist(),
                                                 "n_uncertified": st["n_uncertified"],
                                                 "n_candidates": st["n_candidates"]}))
    assert torch.equal(idx, full.idx)
    assert torch.equal(dist.view(torch.int32), full.dist.view(torch.int32))
    # the shares are balanced: the largest stage-B time within 15% of the mean
    assert ms[:, 1].max() <= 1.15 * ms[:, 1].mean()


@pytest.mark.parametrize("R", [2, 3])
def test_simulated_shards_small_and_clustered(R):
    """Fewer ranks, a world that does not divide the 8-group rounds evenly,
    and clustered rows with exact duplicates across shards."""
    import surfface_hip as S
    from surfface_hip.dist import knn_sharded_sim
    n, d, k = 150_000 - 150_000 % R, 64, 10
    X = _uniform(n, d, seed=11)
    g = torch.Generator(device="cuda").manual_seed(5)
    cent = torch.randn((64, d), device="cuda", generator=g) * 4
    X = (cent[torch.arange(n, device="cuda") % 64] + 0.05 * X).contiguous()
    X[n - 7:] = X[:7]  # exact duplicates in the first and the last shard
    full = S.knn_l2sq(X, k)
    idx, dist, ms, st = knn_sharded_sim(X, k, R, timing=True)
    assert torch.equal(idx, full.idx)
    assert torch.equal(dist.view(torch.int32), full.dist.view(torch.int32))


def test_per_shard_form_eight_shards_bit_exact():
    """The per-shard form (other metrics / generators): exact per-shard top-k
    lists of all queries merged by (dist, id)."""
    import surfface_hip as S
    n, d, k, R = 200_000, 128, 16, 8
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


def test_c4_full_build_as_eight_simulated_ranks():
    """Config 4 (8M x 768, k=32, 8 GPUs) on one GPU: the symmetric sharded
    build with its 8 ranks run in turn.  A rank's share of the real build is
    its stage A + B + C time here (plus the all-gathers and the exchange,
    which the simulation does not run); the largest share must stay within
    8 s.  64 sampled rows (8 per shard) bit-exact vs the oracle's sequential
    f32 fold over all 8M rows; every row sorted with no self pair."""
    import json
    import time

    from oracle import oracle as O
    from surfface_hip.dist import knn_sharded_sim
    import surfface_hip as S
    n_tot, d, k, R = 8_000_000, 768, 32, 8
    n_loc = n_tot // R
    stream = torch.cuda.current_stream().cuda_stream
    Xall = torch.empty((n_tot, d), dtype=torch.float32, device="cuda")
    for r0 in range(0, n_tot, n_loc):  # the same counter stream as every rank's shard
        S._lib.check(S.lib().mn_fill_uniform_f32(Xall[r0:r0 + n_loc].data_ptr(), n_loc, d, 42,
                                                 r0, stream))
    torch.cuda.synchronize()
    free0, total = torch.cuda.mem_get_info()
    t0 = time.perf_counter()
    idx, dist, ms, st = knn_sharded_sim(Xall, k, R, timing=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    free1, _ = torch.cuda.mem_get_info()
    share = ms.sum(axis=1)
    rec = {"s_wall_all_ranks": round(el, 2), "rank_share_s": (share / 1e3).round(3).tolist(),
           "max_share_s": round(float(share.max()) / 1e3, 3),
           "stage_ms_max": ms.max(axis=0).round(1).tolist(),
           "pairs_per_s_at_max_share": n_tot * n_tot / (float(share.max()) / 1e3),
           "n_uncertified": st["n_uncertified"], "n_candidates": st["n_candidates"],
           "device_used_gb": round((total - free1) / 2**30, 1),
           "device_used_gb_inputs": round((total - free0) / 2**30, 1)}
    print("C4 simulated", json.dumps(rec))
    rng = np.random.default_rng(4)
    q = np.concatenate([r * n_loc + rng.choice(n_loc, 8, replace=False) for r in range(R)])
    q = q.astype(np.int64)
    qsel = torch.from_numpy(q).cuda()
    Qh = Xall[qsel].cpu().numpy()
    Ch = Xall.cpu().numpy()
    ri, rd = O.knn_l2sq_qc(Qh, q, Ch, 0, k)
    np.testing.assert_array_equal(idx[qsel].cpu().numpy(), ri)
    np.testing.assert_array_equal(dist[qsel].cpu().numpy().view(np.uint32), rd.view(np.uint32))
    assert st["n_uncertified"] <= 256
    assert bool((dist[:, 1:] >= dist[:, :-1]).all())
    own = torch.arange(0, n_tot, device="cuda", dtype=torch.int32)[:, None]
    assert not bool((idx == own).any())
    assert float(share.max()) <= 8000.0
