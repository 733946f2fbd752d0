"""C5 probe: 1M x 3072 bf16 rectified-cosine kNN (k=32) through the C ABI,
variants by environment (one process; each variant AFTER a warm run):
C5P_VARIANTS="default;MN_BF16_PROBE=noepi;MN_SWEEP_S=4" (';'-separated, ','
between multiple assignments)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build
from surfface_hip import _lib  # noqa: E402

n = int(os.environ.get("C5P_N", 1 << 20))
d = int(os.environ.get("C5P_D", 3072))
dev = torch.device("cuda:0")
L = _lib.lib()
Xb = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
ch = 1 << 17
tmp = torch.empty((min(ch, n), d), dtype=torch.float32, device=dev)
st = torch.cuda.current_stream()
for r0 in range(0, n, ch):
    m = min(ch, n - r0)
    _lib.check(L.mn_fill_uniform_f32(tmp.data_ptr(), m, d, 47, r0, st.cuda_stream))
    Xb[r0:r0 + m].copy_(tmp[:m])
del tmp
torch.cuda.synchronize()
variants = os.environ.get("C5P_VARIANTS", "default").split(";")
ref = None
for rep in range(int(os.environ.get("C5P_REPS", 1))):
    for v in variants:
        env = {}
        if v != "default":
            for kv in v.split(","):
                k_, val = kv.split("=")
                env[k_] = val
        old = {k_: os.environ.get(k_) for k_ in env}
        os.environ.update(env)
        t0 = time.perf_counter()
        idx, dist, w, stt = S.knn_cos_bf16(Xb, 32, eps=1.0, sigma=1.0, p=2.0, timing=True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        for k_, val in old.items():
            if val is None:
                os.environ.pop(k_, None)
            else:
                os.environ[k_] = val
        same = None
        if ref is None:
            ref = (idx.clone(), dist.clone())
        else:
            same = bool(torch.equal(ref[0], idx) and torch.equal(ref[1], dist))
        # the pairs the sweep decides: all n^2 for SW_COS_SYM (sweep_slices -1)
        sweep_rows = n if stt.get("sweep_slices") == -1 else n - stt.get("sample_rows", 0)
        tf = 2.0 * n * sweep_rows * d / (stt["ms_sweep"] * 1e-3) / 1e12 if stt.get("ms_sweep") else None
        print(json.dumps({"rep": rep, "variant": v, "ms": round(ms, 1),
                          "ms_sample": round(stt.get("ms_sample", 0), 1),
                          "ms_sweep": round(stt.get("ms_sweep", 0), 1),
                          "sweep_tflops": tf and round(tf, 1),
                          "ms_rerank": round(stt["ms_rerank"], 1),
                          "uncert": stt["n_uncertified"], "S2": stt.get("sweep_slices"),
                          "same_as_first": same}), flush=True)
        del idx, dist, w
