"""A/B of the diffusion kernels (tuning-build MN_DIFFUSE_* knobs) at C3 in one
process: 1M x 768 uniform rows, the C3 feature Laplacian, eta 0.1, 4 steps;
each variant timed and compared bit for bit with the first.
  AB_ENVS="MN_DIFFUSE_V3=1;MN_DIFFUSE_V3=0" python scripts/diffuse_ab.py [reps]"""
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

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n, d = 1_000_000, 768
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
fi, fd, fw, _ = S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0)
L, _ = S.build_laplacian_from_knn(fi, fw, weight_kernel="given", symmetrise="union")
Xd = torch.empty((n, d), dtype=torch.float64, device="cuda")
VERS = os.environ.get("AB_ENVS", "MN_DIFFUSE_V3=1").split(";")
keys = {kv.split("=")[0] for v in VERS for kv in v.split("+")}
ref = None
for r in range(reps):
    for v in VERS:
        for k_ in keys:
            os.environ.pop(k_, None)
        for kv in v.split("+"):
            k_, val = kv.split("=")
            os.environ[k_] = val
        torch.cuda.synchronize()
        t = time.perf_counter()
        S.diffuse_rows(X, L, 0.1, 4, out=Xd)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        if ref is None:
            ref = Xd.clone()
        same = bool(torch.equal(ref.view(torch.int64), Xd.view(torch.int64)))
        print(json.dumps({"rep": r, "v": v, "ms": round(ms, 3), "same_as_first": same}), flush=True)
