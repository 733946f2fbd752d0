"""C4 (8M x 768, 8 simulated ranks) group-shape A/B for the shard table
(tuning build, one process): MN_SYM_GR=4 (default of shard_share) vs 2 (C2's
single-GPU shape); max rank share and stage B, outputs compared."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()
from surfface_hip import _lib  # noqa: E402
from surfface_hip.dist import knn_sharded_sim  # noqa: E402

R, n_loc, d, k = 8, 1_000_000, 768, 32
L = _lib.lib()
st = torch.cuda.current_stream()
X = torch.empty((R * n_loc, d), dtype=torch.float32, device="cuda")
for r0 in range(0, R * n_loc, n_loc):
    _lib.check(L.mn_fill_uniform_f32(X[r0:r0 + n_loc].data_ptr(), n_loc, d, 42, r0, st.cuda_stream))
torch.cuda.synchronize()
ref = None
for v in os.environ.get("C4V", "4;2;4;2").split(";"):
    os.environ["MN_SYM_GR"] = v
    idx, dist, ms, stt = knn_sharded_sim(X, k, R, timing=True, stream=st)
    torch.cuda.synchronize()
    same = None
    if ref is None:
        ref = (idx.clone(), dist.clone())
    else:
        same = bool(torch.equal(ref[0], idx) and torch.equal(ref[1].view(torch.int32), dist.view(torch.int32)))
    share = ms.sum(axis=1)
    print(json.dumps({"MN_SYM_GR": v, "max_share_s": round(float(share.max()) / 1e3, 3),
                      "B_max_ms": round(float(ms[:, 1].max()), 1),
                      "share_spread": round(float(share.max() / share.mean()), 4), "same": same}), flush=True)
    del idx, dist
