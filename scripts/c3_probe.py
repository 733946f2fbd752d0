"""C3 feature-graph leg timing breakdown: rectified-cosine kNN of the 768
feature columns of a 1M x 768 f32 matrix (topk=4), with the library's stage
timers (norms + Gram | select + exact re-rank + finish | fallback).
  python scripts/c3_probe.py [n] [f] [reps]"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
f = int(sys.argv[2]) if len(sys.argv) > 2 else 768
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
X = torch.empty((n, f), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, f, 42, 0, None))
torch.cuda.synchronize()
ref = None
VARS = os.environ.get("C3_VARIANTS", "default").split(";")
keys = {kv.split("=")[0] for v in VARS if v != "default" for kv in v.split("+")}
for r, v in [(r, v) for r in range(reps + 1) for v in VARS]:
    for k_ in keys:
        os.environ.pop(k_, None)
    if v != "default":
        for kv in v.split("+"):
            k_, val = kv.split("=")
            os.environ[k_] = val
    t = time.perf_counter()
    fi, fd, fw, st = S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0, timing=True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) * 1e3
    if ref is None:
        ref = (fi.clone(), fd.clone())
    same = torch.equal(ref[0], fi) and torch.equal(ref[1], fd)
    print(json.dumps({"rep": r, "v": v, "wall_ms": round(wall, 3), "same": bool(same),
                      **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}}),
          flush=True)
