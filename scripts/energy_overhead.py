"""Where an energy_rows call's wall time goes at C3 (1M x 768, the feature
Laplacian): wall (Python, synchronised) vs the library's device-side marks
(ms_total: start .. after the rows kernel; ms_rows: the kernel)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
from surfface_hip import _lib  # noqa: E402

n, d = 1_000_000, 768
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
fi, fd, fw, _ = S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0)
L, _ = S.build_laplacian_from_knn(fi, fw, weight_kernel="given", symmetrise="union")
E = torch.empty(n, dtype=torch.float64, device="cuda")
for timing in (False, True, True, False, True):
    torch.cuda.synchronize()
    t = time.perf_counter()
    S.energy_rows(X, L, timing=timing)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) * 1e3
    st = S.energy.last_stats()
    print(json.dumps({"timing": timing, "wall_ms": round(wall, 3), **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}}), flush=True)
# a bare launch-overhead reference: an empty-ish torch op round trip
torch.cuda.synchronize()
t = time.perf_counter()
E.zero_()
torch.cuda.synchronize()
print(json.dumps({"torch_zero_1M_f64_ms": round((time.perf_counter() - t) * 1e3, 3)}))
