"""Symmetric sharded build simulated on one GPU (mn_knn_sharded_sim_f32):
per-rank stage times, uncertified rows (MN_X1_DEBUG=1 prints the reasons),
candidates, bit-exactness vs the single-GPU graph.  Tuning build (MN_SH_* knobs).
  SH_WORLDS="1,8" python scripts/shard_probe.py [n] [d] [k]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()
from surfface_hip import _lib  # noqa: E402
from surfface_hip.dist import knn_sharded_sim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 768
k = int(sys.argv[3]) if len(sys.argv) > 3 else 32
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
torch.cuda.synchronize()
full = S.knn_l2sq(X, k, timing=True)
print(json.dumps({"single": {kk: (round(v, 2) if isinstance(v, float) else v)
                             for kk, v in full.stats.items()}}), flush=True)
for w in [int(x) for x in os.environ.get("SH_WORLDS", "1,8").split(",")]:
    t = time.time()
    idx, dist, ms, st = knn_sharded_sim(X, k, w, timing=True)
    torch.cuda.synchronize()
    same = torch.equal(idx, full.idx) and torch.equal(dist.view(torch.int32), full.dist.view(torch.int32))
    print(json.dumps({"world": w, "wall": round(time.time() - t, 2), "same": bool(same),
                      "stage_ms_max": ms.max(axis=0).round(1).tolist(),
                      "share_ms_max": round(float(ms.sum(axis=1).max()), 1),
                      "n_uncertified": st["n_uncertified"], "n_candidates": st["n_candidates"]}),
          flush=True)
