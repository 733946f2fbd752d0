"""K1 microbench: knn_l2sq on n x d uniform f32 rows (library timing stats).
Env MN_L2_PROBE=noepi (bf16x3) / MN_X1_PROBE=noepi (bf16x1 sweep) time the
Gram K loop alone (results invalid)."""
import argparse, json, os, sys, time
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_R, "matternet-rs_amd"))
import torch
import surfface_hip as S
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build
from surfface_hip import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=262144)
ap.add_argument("--d", type=int, default=768)
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--margin", type=int, default=16)
ap.add_argument("--algo", default="auto")
a = ap.parse_args()
X = torch.empty((a.n, a.d), dtype=torch.float32, device="cuda")
_lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), a.n, a.d, 42, 0,
                                          torch.cuda.current_stream().cuda_stream))
for r in range(a.reps):
    torch.cuda.synchronize(); t0 = time.time()
    res = S.knn_l2sq(X, a.k, margin=a.margin, timing=True, algo=a.algo)
    torch.cuda.synchronize(); dt = time.time() - t0
    st = res.stats
    fl = 2.0 * a.n * a.n * a.d
    out = {"n": a.n, "d": a.d, "k": a.k, "algo": a.algo, "used": st["algo"],
           "probe": os.environ.get("MN_L2_PROBE") or os.environ.get("MN_X1_PROBE"),
           "wall_s": round(dt, 4), "ms_gram": round(st["ms_gram"], 2),
           "tflops_alg": round(fl / (st["ms_gram"] * 1e-3) / 1e12, 1),
           "uncert": st["n_uncertified"], "slices": st["slices"],
           "ms_norms": round(st["ms_norms"], 2), "ms_rerank": round(st["ms_rerank"], 2),
           "ms_fallback": round(st["ms_fallback"], 2), "ms_total": round(st["ms_total"], 2)}
    if st["algo"] == 3:
        m0 = st["sample_rows"]
        out.update(ms_sample=round(st["ms_sample"], 2), ms_sweep=round(st["ms_sweep"], 2),
                   sweep_tflops=round(2.0 * a.n * (a.n - m0) * a.d / (st["ms_sweep"] * 1e-3) / 1e12, 1),
                   sample_rows=m0, cands_per_q=round(st["n_candidates"] / a.n, 1),
                   sweep_slices=st["sweep_slices"], sweep_cap=st["sweep_cap"])
    print(json.dumps(out), flush=True)
