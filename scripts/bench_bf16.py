"""Quick C5 item-graph timing: knn_cos_bf16 on n x d uniform bf16 rows."""
import argparse, json, sys, time
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_R, "matternet-rs_amd"))
import torch
import surfface_hip as S

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=262144)
ap.add_argument("--d", type=int, default=3072)
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(1)
X = (torch.rand(a.n, a.d, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
for r in range(a.reps):
    torch.cuda.synchronize(); t0 = time.time()
    i, d, w, st = S.knn_cos_bf16(X, a.k, timing=True)
    torch.cuda.synchronize(); dt = time.time() - t0
    fl = 2.0 * a.n * a.n * a.d
    print(json.dumps({"n": a.n, "d": a.d, "k": a.k, "wall_s": dt, "stats": st,
                      "gram_tflops": fl / (st["ms_gram"] * 1e-3) / 1e12}), flush=True)
