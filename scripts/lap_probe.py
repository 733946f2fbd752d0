"""K2 item-Laplacian timing (C3 shape): wall time per call vs the library's
HIP-event span (mn_lap_last_stats.ms_total) for caller-owned (the Python
wrapper) output, to separate kernel time from call overhead.  Run under
rocprofv3 --kernel-trace for the per-kernel timeline.
    python scripts/lap_probe.py [n]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build
from surfface_hip import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
d, k = 768, 32
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
r = S.knn_l2sq(X, k)
del X
torch.cuda.synchronize()
# row segment lengths before the dedupe: k forward slots + in-degree
indeg = torch.bincount(r.idx.reshape(-1).long().clamp(min=0), minlength=n)
seg = indeg + k
edges = [0, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 1 << 40]
hist = {f"<={edges[i + 1]}": int(((seg > edges[i]) & (seg <= edges[i + 1])).sum())
        for i in range(len(edges) - 1)}
big = seg[seg > 512]
print(json.dumps({"seg_hist": hist, "entries_in_rows_gt512": int(big.sum()),
                  "max_seg": int(seg.max())}), flush=True)
# A/B: the bucketed assembly (default) vs the atomic counting-sort path
# (MN_LAP_V1=1): identical CSR and degrees, and both timings
outs = {}
for v in ("1", "0", "1", "0"):
    os.environ["MN_LAP_V1"] = v
    L, deg = S.build_laplacian_from_knn(r.idx, r.dist, weight_kernel="rational",
                                        symmetrise="union", eps=float("inf"), sigma=1.0, p=2.0)
    torch.cuda.synchronize()
    st = S.laplacian.last_stats()
    outs[v] = (L, deg)
    print(json.dumps({"MN_LAP_V1": v, "lib_ms": round(st["ms_total"], 3), "nnz": L.nnz,
                      "big_rows": st["big_rows"], "hub_rows": st["hub_rows"]}), flush=True)
(a, da), (b, db) = outs["1"], outs["0"]
same = (a.nnz == b.nnz and torch.equal(a.indptr, b.indptr) and torch.equal(a.indices, b.indices)
        and torch.equal(a.values.view(torch.int64), b.values.view(torch.int64))
        and torch.equal(da.view(torch.int64), db.view(torch.int64)))
print(json.dumps({"v1_v2_identical": bool(same)}), flush=True)
del outs, a, b, da, db
os.environ.pop("MN_LAP_V1")
for rep in range(6):
    t0 = time.perf_counter()
    L, _ = S.build_laplacian_from_knn(r.idx, r.dist, weight_kernel="rational", symmetrise="union",
                                      eps=float("inf"), sigma=1.0, p=2.0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    st = S.laplacian.last_stats()
    byt = n * k * 8 + L.nnz * 12 + (n + 1) * 8
    print(json.dumps({"rep": rep, "wall_ms": round(wall, 3), "lib_ms": round(st["ms_total"], 3),
                      "nnz": L.nnz, "GB_per_s_wall": round(byt / wall / 1e6, 1),
                      "GB_per_s_lib": round(byt / st["ms_total"] / 1e6, 1),
                      "big_rows": st["big_rows"], "hub_rows": st["hub_rows"]}), flush=True)
    del L
