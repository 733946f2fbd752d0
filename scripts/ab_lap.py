"""Same-process A/B of the item-graph Laplacian (C3's K2 leg) across library
builds: the C2 kNN graph (1M x 768, k 32) once, then
build_laplacian_from_knn (UNION rational, and MAX normalised) under each
library in AB_LIBS (';'-separated paths), CSR outputs compared bit for bit."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
from surfface_hip import _lib  # noqa: E402
from ab_libs import load  # noqa: E402  (tolerant loader)

n, d, k = 1_000_000, 768, 32
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
g = S.knn_l2sq(X, k)
idx, dist = g.idx, g.dist
del X
torch.cuda.synchronize()
VARS = os.environ["AB_LIBS"].split(";")
ref = {}
for r in range(int(os.environ.get("AB_ROUNDS", 3))):
    for v in VARS:
        _lib._LIB = load(v if os.path.isabs(v) else os.path.join(ROOT, v))
        rec = {"round": r, "v": v}
        for mode in ("union", "max"):
            kw = dict(weight_kernel="rational", symmetrise=mode, eps=float("inf"), sigma=1.0, p=2.0,
                      normalize=(mode == "max"))
            S.build_laplacian_from_knn(idx, dist, **kw)
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                L, _ = S.build_laplacian_from_knn(idx, dist, **kw)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            rec[mode + "_ms"] = round(min(ts), 3)
            key = (L.indptr.cpu(), L.indices.cpu(), L.values.cpu())
            if mode not in ref:
                ref[mode] = key
            else:
                rec[mode + "_same"] = bool(torch.equal(ref[mode][0], key[0]) and
                                           torch.equal(ref[mode][1], key[1]) and
                                           torch.equal(ref[mode][2], key[2]))
            del L
        print(json.dumps(rec), flush=True)
