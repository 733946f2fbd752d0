"""Kernel-level timing of the lambda-aware search at the C3 shape (for rocprofv3)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "matternet-rs_amd"))
import surfface_hip as S  # noqa: E402

n, f, nq = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000, 768, 64
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.rand((n, f), device="cuda", generator=g) * 2 - 1
lam = torch.rand(n, device="cuda", dtype=torch.float64, generator=g)
Q = X[:nq].double().contiguous()
lq = lam[:nq].clone().clamp_min(1e-6)
for _ in range(2):
    S.search_lambda_aware(X, lam, Q, lq, 32, 0.7)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    S.search_lambda_aware(X, lam, Q, lq, 32, 0.7)
torch.cuda.synchronize()
print("ms per call", (time.perf_counter() - t0) / 5 * 1e3)
