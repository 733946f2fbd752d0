"""One K3 energy-rows configuration at the C3 shape, a few timed calls (for
rocprofv3 passes: scripts/pmc_sq.sh).  ER_MODE = median | fixed; MN_* knobs
from the environment (tuning build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()
from surfface_hip import _lib  # noqa: E402

n, d = 1_000_000, 768
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
fi, fd, fw, _ = S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0)
L, _ = S.build_laplacian_from_knn(fi, fw, weight_kernel="given", symmetrise="union")
tm = S.TauMode.Median if os.environ.get("ER_MODE", "median") == "median" else S.TauMode.Fixed(0.5)
for _ in range(3):
    E, G, lam = S.energy_rows(X, L, _lib.MN_G_TAUMODE, tm)
torch.cuda.synchronize()
print("ok", float(lam.sum()))
