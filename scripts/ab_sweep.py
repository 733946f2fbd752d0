"""A/B of sweep variants (tuning-build knobs) in ONE process on the same device
and data (guide rule 24): C2 shape by default, interleaved rounds, outputs
compared bit for bit; AB_PROBES times the K-loop probes of each variant.
  AB_ENVS="MN_X1_SYM=1;MN_X1_SYM=0" python scripts/ab_sweep.py [n] [d] [rounds]
(';' between variants, ',' between assignments)."""
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
d = int(sys.argv[2]) if len(sys.argv) > 2 else 768
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
if os.environ.get("AB_DATA") == "clustered":  # the SURVEY §8(d) clustered distribution
    sys.path.append(os.path.join(ROOT, "tests"))
    import datagen  # noqa: E402
    X = torch.from_numpy(datagen.clustered(n, d, seed=7)).cuda()
else:
    X = torch.empty((n, d), dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
torch.cuda.synchronize()
ref = None
VERS = os.environ.get("AB_ENVS", "MN_X1_SYM=1").split(";")
res = {v: [] for v in VERS}
probe = {v: [] for v in VERS}
for r in range(rounds):
    for v in VERS:
        for k_ in {kv.split("=")[0] for vv in VERS for kv in vv.replace("+", ",").split(",")}:
            os.environ.pop(k_, None)  # a variant sets only its own keys
        for kv in v.replace("+", ",").split(","):
            k_, val = kv.split("=")
            os.environ[k_] = val
        os.environ.pop("MN_X1_PROBE", None)
        t = time.time()
        out = S.knn_l2sq(X, 32, timing=True, algo="bf16x1")
        torch.cuda.synchronize()
        st = out.stats
        res[v].append({"ms_sweep": round(st["ms_sweep"], 2), "ms_total": round(st["ms_total"], 2),
                       "ms_rerank": round(st["ms_rerank"], 2), "ms_sample": round(st["ms_sample"], 2),
                       "ms_norms": round(st["ms_norms"], 2),
                       "n_cand": st["n_candidates"], "unc": st["n_uncertified"],
                       "esc": st["n_escalated"], "wall": round(time.time() - t, 3)})
        if ref is None:
            ref = (out.idx.clone(), out.dist.clone())
        else:
            same = torch.equal(ref[0], out.idx) and torch.equal(ref[1].view(torch.int32),
                                                                 out.dist.view(torch.int32))
            res[v][-1]["same_as_first"] = bool(same)
        del out
        pm = {}
        for pk in os.environ.get("AB_PROBES", "noepi").split(","):
            if not pk:
                continue
            os.environ["MN_X1_PROBE"] = pk
            S.knn_l2sq(X, 32, timing=True, algo="bf16x1")
            pm[pk] = round(S.knn.last_stats()["ms_sweep"], 2)
        os.environ.pop("MN_X1_PROBE", None)
        probe[v].append(pm.get("noepi", 0.0))
        print(json.dumps({"round": r, "v": v, **res[v][-1], "probe_ms": pm}), flush=True)
print(json.dumps({"summary": {v: min(x["ms_sweep"] for x in res[v]) for v in VERS},
                  "probe": {v: min(probe[v]) for v in VERS}}))
