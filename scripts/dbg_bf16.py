import sys, numpy as np, torch
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_R, "matternet-rs_amd")); sys.path.insert(0, os.path.join(_R, "tests")); sys.path.insert(0, _R)
import datagen
from oracle import oracle as O
import surfface_hip as S
for (n, d, k) in [(257, 24, 5), (257, 32, 5), (600, 64, 5), (3000, 256, 10)]:
    X = datagen.uniform(n, d, seed=11)
    bits = datagen.to_bf16_bits(X)
    Xf = datagen.bf16_bits_to_f32(bits)
    Xt = torch.from_numpy(bits.view(np.int16)).cuda().view(torch.bfloat16)
    try:
        i, dd, w, st = S.knn_cos_bf16(Xt, k)
    except Exception as e:
        print(n, d, k, "ERR", e, flush=True); break
    i = i.cpu().numpy(); dd = dd.cpu().numpy()
    ri, rd, rw = O.knn_cos(Xf, k)
    bad = np.where(np.any(i != ri, axis=1))[0]
    print(n, d, k, st, "bad rows", len(bad), bad[:10], flush=True)
    for r in bad[:3]:
        print(" row", r, "hip", i[r], dd[r], "\n      ref", ri[r], rd[r], flush=True)
