"""Phase-1 sample size / list length grid for the bf16x1 generator (C2 shape):
per setting the sample, sweep, re-rank and total times, candidates and
uncertified rows, in one process; outputs compared with the first setting.
  python scripts/grid_x1.py [n] [d] "div:L1,div:L1,..." """
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build
from surfface_hip import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 768
grid = [tuple(int(v) for v in t.split(":")) for t in
        (sys.argv[3] if len(sys.argv) > 3 else "16:16,16:12,16:10,32:8,8:24,24:12").split(",")]
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
torch.cuda.synchronize()
ref = None
for rep in range(2):
    for div, l1 in grid:
        os.environ["MN_X1_SAMPLE_DIV"] = str(div)
        os.environ["MN_X1_L1"] = str(l1)
        out = S.knn_l2sq(X, 32, timing=True, algo="bf16x1")
        torch.cuda.synchronize()
        st = out.stats
        same = None
        if ref is None:
            ref = (out.idx.clone(), out.dist.clone())
        else:
            same = bool(torch.equal(ref[0], out.idx) and torch.equal(ref[1], out.dist))
        print(json.dumps({"rep": rep, "div": div, "L1": l1, "total": round(st["ms_total"], 1),
                          "sample": round(st["ms_sample"], 1), "sweep": round(st["ms_sweep"], 1),
                          "rerank": round(st["ms_rerank"], 1), "esc": st["n_escalated"],
                          "ms_esc": round(st["ms_escalate"], 1), "fb": round(st["ms_fallback"], 1),
                          "cand": st["n_candidates"], "unc": st["n_uncertified"],
                          "same": same}), flush=True)
        del out
