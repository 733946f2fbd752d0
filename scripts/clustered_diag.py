"""C2-clustered diagnostics (tests/datagen.clustered, 1M x 768, k=32): the
uncertified-row reasons per re-rank pass (MN_X1_DEBUG=1, stderr) and the
stats of the default path and its variants.
    python scripts/clustered_diag.py [n] [variants ';'-separated]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import datagen  # noqa: E402
import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
variants = (sys.argv[2] if len(sys.argv) > 2 else "default").split(";")
X = torch.from_numpy(datagen.clustered(n, 768, seed=7)).cuda()
os.environ["MN_X1_DEBUG"] = "1"
ref = None
for v in variants:
    env = {} if v == "default" else dict(kv.split("=") for kv in v.split(","))
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    t = time.time()
    r = S.knn_l2sq(X, 32, timing=True)
    torch.cuda.synchronize()
    wall = time.time() - t
    same = None
    if ref is None:
        ref = (r.idx.clone(), r.dist.clone())
    else:
        same = bool(torch.equal(ref[0], r.idx) and torch.equal(ref[1], r.dist))
    print(json.dumps({"variant": v, "wall_s": round(wall, 3), "same_as_first": same,
                      **{k: (round(x, 2) if isinstance(x, float) else x)
                         for k, x in r.stats.items()}}), flush=True)
    for k, x in old.items():
        if x is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = x
