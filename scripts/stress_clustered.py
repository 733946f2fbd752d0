"""Certification stress at scale: the SURVEY §8(d) clustered distribution
(64 blobs sigma 0.1, 1% duplicates, 0.1% zero rows, seed 7) through the kNN
generators; prints per-generator stats and checks sampled rows vs the oracle."""
import argparse, json, os, sys, time
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, "matternet-rs_amd"), _R, os.path.join(_R, "tests")]
import numpy as np
import torch
import datagen
import surfface_hip as S
from oracle import oracle as O

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--d", type=int, default=768)
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--algos", default="bf16x1,bf16x3")
ap.add_argument("--rows", type=int, default=64)
ap.add_argument("--sorted", action="store_true", help="rows sorted along a principal coordinate")
a = ap.parse_args()
t0 = time.time()
X = datagen.clustered(a.n, a.d, seed=7)
if a.sorted:
    X = X[np.argsort(X[:, 0], kind="stable")]
print(json.dumps({"gen_s": round(time.time() - t0, 1)}), flush=True)
Xd = torch.from_numpy(X).cuda()
rows = np.random.default_rng(1).choice(a.n, a.rows, replace=False)
ridx, rdist = O.knn_l2sq_rows(X, a.k, rows)
for algo in a.algos.split(","):
    torch.cuda.synchronize(); t = time.time()
    r = S.knn_l2sq(Xd, a.k, timing=True, algo=algo)
    torch.cuda.synchronize(); dt = time.time() - t
    st = r.stats
    idx, dist = r.idx.cpu().numpy(), r.dist.cpu().numpy()
    ok = bool(np.array_equal(idx[rows], ridx) and np.array_equal(dist[rows].view(np.uint32), rdist.view(np.uint32)))
    print(json.dumps({"algo": algo, "wall_s": round(dt, 3), "rows_bit_exact": ok,
                      "sorted_ok": bool((np.diff(dist, axis=1) >= 0).all()),
                      **{kk: (round(v, 2) if isinstance(v, float) else v) for kk, v in st.items()}}), flush=True)
