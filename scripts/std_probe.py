"""K4 timing probe: mn_sorted_index at 1M (std on), certified pass 1 vs the
forced sequential pass 1 (MN_STD_SEQ=1), same process."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "matternet-rs_amd"))
import surfface_hip as S  # noqa: E402
S._lib.select_tuning_library()  # MN_* knobs / timing probes: the tuning build

rng = np.random.default_rng(0)
lam = torch.from_numpy(rng.uniform(0, 1, 1_000_000)).cuda()
for rep in range(3):
    for mode in ("cert", "seq"):
        if mode == "seq":
            os.environ["MN_STD_SEQ"] = "1"
        else:
            os.environ.pop("MN_STD_SEQ", None)
        S.SortedLambdas().build_from(lam)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            sl = S.SortedLambdas().build_from(lam)
        torch.cuda.synchronize()
        print(json.dumps({"rep": rep, "mode": mode, "ms": round((time.perf_counter() - t) * 100, 3),
                          "std": sl.std_dev}), flush=True)
