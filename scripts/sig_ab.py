"""Item-graph signals at C3 size, knob variants in one
process (tuning build): the 768 feature signals of a 1M x 768 f32 matrix
against its k=32 union item Laplacian; E/G compared with the first variant.
  SIG_VARIANTS="MN_SIG_FS=0;MN_SIG_FS=64" python scripts/sig_ab.py [n] [d] [reps]"""
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
d = int(sys.argv[2]) if len(sys.argv) > 2 else 768
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
out = S.knn_l2sq(X, 32)
Lit, _ = S.build_laplacian_from_knn(out.idx, out.dist, weight_kernel="rational", symmetrise="union",
                                    eps=float("inf"), sigma=1.0, p=2.0)
torch.cuda.synchronize()
print(json.dumps({"n": n, "d": d, "nnz": Lit.nnz}), flush=True)
VARS = os.environ.get("SIG_VARIANTS", "default").split(";")
keys = {kv.split("=")[0] for v in VARS if v != "default" for kv in v.split("+")}
ref = None
best = {}
for r in range(reps):
    for v in VARS:
        for k_ in keys:
            os.environ.pop(k_, None)
        if v != "default":
            for kv in v.split("+"):
                k_, val = kv.split("=")
                os.environ[k_] = val
        S.signal_energy_and_dispersion(X, Lit)
        torch.cuda.synchronize()
        t = time.perf_counter()
        E, G = S.signal_energy_and_dispersion(X, Lit)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        rec = {"rep": r, "v": v, "ms": round(ms, 3)}
        if ref is None:
            ref = (E.clone(), G.clone())
        else:
            rec["E_rel"] = float(((E - ref[0]).abs() / ref[0].abs().clamp_min(1e-300)).max())
            rec["G_rel"] = float(((G - ref[1]).abs() / ref[1].abs().clamp_min(1e-300)).max())
        best[v] = min(best.get(v, 1e30), ms)
        print(json.dumps(rec), flush=True)
for k_ in keys:
    os.environ.pop(k_, None)
print(json.dumps({"best_ms": best}))
