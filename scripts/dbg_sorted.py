import os, sys, json
import numpy as np, torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", ".")
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd"), os.path.join(ROOT, "tests")]
import surfface_hip as S
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build
import datagen
rng = np.random.default_rng(3)
n, d = 20_000, 64
X0 = rng.normal(size=(n, d)) + 0.3
Xs = X0[np.argsort(X0 @ rng.normal(size=d))].astype(np.float32)
for name, X in (("sorted", Xs), ("random", X0.astype(np.float32))):
    bits = datagen.to_bf16_bits(np.ascontiguousarray(X))
    Xt = torch.from_numpy(bits.view(np.int16)).cuda().view(torch.bfloat16)
    for env in ({}, {"MN_BF16_X1": "0"}, {"MN_BF16_TM": "0"}):
        os.environ.pop("MN_BF16_X1", None); os.environ.pop("MN_BF16_TM", None)
        os.environ.update(env)
        i, dd, w, st = S.knn_cos_bf16(Xt, 10)
        print(name, env, json.dumps({k: st[k] for k in ("n_uncertified", "sample_rows", "sweep_slices", "sweep_cap", "slices", "list_len")}), flush=True)
