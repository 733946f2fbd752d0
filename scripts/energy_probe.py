"""K3 energy-rows timing by tau mode (C3 shape): isolates the per-row tau
selection from the Laplacian entry loop.  python scripts/energy_probe.py [n]"""
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
d = 768
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
fi, fd, fw, _ = S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0)
L, _ = S.build_laplacian_from_knn(fi, fw, weight_kernel="given", symmetrise="union")
modes = {"median": S.TauMode.Median, "mean": S.TauMode.Mean, "fixed": S.TauMode.Fixed(0.5)}
ref = {}
for rep in range(3):
    # A/B in one process: LDS entry lists x 2 rows (default) / x 4 rows, the
    # value-linear tau select, the register-resident lists
    for kern, env in (("lds2", {}), ("lds4", {"MN_ENERGY_ROWS": "4"}),
                      ("lds2_lin", {"MN_TAU_SEL": "1"}), ("reg", {"MN_ENERGY_REG": "1"})):
        for kk in ("MN_ENERGY_ROWS", "MN_TAU_SEL", "MN_ENERGY_REG"):
            os.environ.pop(kk, None)
        os.environ.update(env)
        for name, tm in modes.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            E, G, lam = S.energy_rows(X, L, _lib.MN_G_TAUMODE, tm)
            e1.record()
            torch.cuda.synchronize()
            same = None
            if name in ref:
                same = bool(torch.allclose(lam, ref[name], rtol=1e-12, atol=1e-15))
            else:
                ref[name] = lam.clone()
            print(json.dumps({"rep": rep, "kernel": kern, "mode": name,
                              "ms": round(e0.elapsed_time(e1), 3), "nnz": L.nnz,
                              "same_as_first": same}), flush=True)
