"""K3 energy-rows A/B at the C3 shape (one process): EAB_VARIANTS=
"default;MN_ENERGY_PROBE=16;MN_TAU_SEL=1" (';' between variants, ',' between
assignments); each variant x tau mode (median, fixed) timed over 5 calls
(min reported), lambda compared with the default variant's."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build
from surfface_hip import _lib  # noqa: E402

n = int(os.environ.get("EAB_N", 1_000_000))
d = 768
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
fi, fd, fw, _ = S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0)
L, _ = S.build_laplacian_from_knn(fi, fw, weight_kernel="given", symmetrise="union")
modes = {"median": S.TauMode.Median, "fixed": S.TauMode.Fixed(0.5)}
keys = set()
variants = os.environ.get("EAB_VARIANTS", "default").split(";")
parsed = []
for v in variants:
    env = {}
    if v != "default":
        for kv in v.split(","):
            k_, val = kv.split("=")
            env[k_] = val
            keys.add(k_)
    parsed.append((v, env))
ref = {}
for v, env in parsed:
    for k_ in keys:
        os.environ.pop(k_, None)
    os.environ.update(env)
    for name, tm in modes.items():
        best = None
        for rep in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            E, G, lam = S.energy_rows(X, L, _lib.MN_G_TAUMODE, tm)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        if name not in ref:
            ref[name] = lam.clone()
            err = 0.0
        else:
            err = float(((lam - ref[name]).abs() / ref[name].abs().clamp_min(1e-300)).max())
        print(json.dumps({"variant": v, "mode": name, "ms": round(best, 3), "nnz": L.nnz,
                          "max_rel_vs_default": err}), flush=True)
for k_ in keys:
    os.environ.pop(k_, None)
# the diffusion pre-pass on the same rows (eta 0.1, 4 steps; bench.py c3 leg)
Xd = torch.empty((n, d), dtype=torch.float64, device="cuda")
S.diffuse_rows(X, L, 0.1, 4, out=Xd)
best = None
for rep in range(3):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    S.diffuse_rows(X, L, 0.1, 4, out=Xd)
    e1.record()
    torch.cuda.synchronize()
    best = e0.elapsed_time(e1) if best is None else min(best, e0.elapsed_time(e1))
print(json.dumps({"diffusion_4_steps_ms": round(best, 3), "GB_per_s": round(n * d * 12 / best / 1e6, 1)}),
      flush=True)
# EAB_SIGNALS=1: the item-graph orientation leg (bench.py c3_legs.item_graph_signals):
# the F feature signals against the C2 item Laplacian
if os.environ.get("EAB_SIGNALS") == "1":
    del Xd
    g = S.knn_l2sq(X, 32, algo="bf16x1")
    Lit, _ = S.build_laplacian_from_knn(g.idx, g.dist, weight_kernel="rational", symmetrise="union",
                                        eps=float("inf"), sigma=1.0, p=2.0)
    del g
    S.signal_energy_and_dispersion(X, Lit)
    best = None
    for rep in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        S.signal_energy_and_dispersion(X, Lit)
        e1.record()
        torch.cuda.synchronize()
        best = e0.elapsed_time(e1) if best is None else min(best, e0.elapsed_time(e1))
    print(json.dumps({"item_graph_signals_ms": round(best, 3), "nnz": Lit.nnz}), flush=True)
