"""lambda-aware search A/B (tuning build, one process): MN_SRCH_V4=1 (16-B
transposing stores) vs 0 (round 5's scalar stores), bench.py's c3 shape:
1M x 768 f32 items, 64 queries, k=32, alpha=0.7; results compared."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()
from surfface_hip import _lib  # noqa: E402

n, f, nq = 1_000_000, 768, 64
X = torch.empty((n, f), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, f, 42, 0, None))
lam = torch.rand(n, dtype=torch.float64, device="cuda")
qrows = torch.arange(0, n, n // nq, device="cuda")[:nq]
Qs = X[qrows].double().contiguous()
lq = lam[qrows].clone().clamp_min(1e-6)
ref = None
for rep in range(3):
    for v in ("1", "0"):
        os.environ["MN_SRCH_V4"] = v
        for hyb in (False, True):
            fn = S.search_lambda_aware_hybrid if hyb else S.search_lambda_aware
            fn(X, lam, Qs, lq, 32, 0.7)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(X, lam, Qs, lq, 32, 0.7)
            e1.record()
            torch.cuda.synchronize()
            key = ("h" if hyb else "s")
            flat = [t for t in (r if isinstance(r, (tuple, list)) else [r]) if torch.is_tensor(t)]
            same = None
            if rep == 0 and v == "1":
                ref = ref or {}
                ref[key] = [t.clone() for t in flat]
            else:
                same = all(torch.equal(a, b) for a, b in zip(ref[key], flat))
            print(json.dumps({"rep": rep, "MN_SRCH_V4": v, "hybrid": hyb,
                              "ms": round(e0.elapsed_time(e1), 3), "same": same}), flush=True)
