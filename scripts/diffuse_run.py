"""The C3 diffusion pre-pass (eta 0.1, 4 steps; energymaps.rs:518-546) on the
1M x 768 rows against the C3 feature Laplacian, a few calls (rocprofv3 passes:
scripts/pmc_sq.sh).  Tuning build (MN_DIFFUSE_* knobs)."""
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
Xd = torch.empty((n, d), dtype=torch.float64, device="cuda")
for _ in range(3):
    S.diffuse_rows(X, L, 0.1, 4, out=Xd)
torch.cuda.synchronize()
print("ok", float(Xd[::9973].sum()))
