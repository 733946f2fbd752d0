"""Item-graph signal energies at the C3 shape: X 1M x 768
uniform, its C2 kNN graph -> UNION rational Laplacian, then
signal_energy_and_dispersion timed; AB_ENVS variants (tuning build, ';'
between variants) interleaved in one process, outputs compared.
  AB_ENVS="MN_SIG_NE=8;MN_SIG_NE=4" python scripts/signals_run.py [n] [f] [reps]"""
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
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
X = torch.empty((n, f), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, f, 42, 0, None))
out = S.knn_l2sq(X, 32)
L, _ = S.build_laplacian_from_knn(out.idx, out.dist, weight_kernel="rational", symmetrise="union",
                                  eps=float("inf"), sigma=1.0, p=2.0)
del out
torch.cuda.synchronize()
VERS = os.environ.get("AB_ENVS", "MN_SIG_NONE=0").split(";")
ref = None
for r in range(reps):
    for v in VERS:
        for kv in v.split(","):
            k_, val = kv.split("=")
            os.environ[k_] = val
        torch.cuda.synchronize()
        t = time.perf_counter()
        E, G = S.signal_energy_and_dispersion(X, L)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        if ref is None:
            ref = (E.clone(), G.clone())
        rel = float(((E - ref[0]).abs() / ref[0].abs().clamp_min(1e-300)).max())
        relg = float(((G - ref[1]).abs() / ref[1].abs().clamp_min(1e-300)).max())
        print(json.dumps({"rep": r, "v": v, "ms": round(ms, 3), "nnz": L.nnz,
                          "max_rel_E_vs_first": rel, "max_rel_G_vs_first": relg}), flush=True)
