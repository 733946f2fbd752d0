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
