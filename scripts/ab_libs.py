"""Same-process A/B of two builds of the library (e.g. the HEAD kernel vs a
working-tree change that is not behind a knob): each variant is a library
path, optionally with knobs ('path|MN_X=1,MN_Y=2'); interleaved rounds on the
same device and data, outputs compared bit for bit against the first.
  AB_LIBS="a.so;b.so|MN_SW_V=2" python scripts/ab_libs.py [n] [d] [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "matternet-rs_amd")]
import torch  # noqa: E402

import surfface_hip as S  # noqa: E402
from surfface_hip import _lib  # noqa: E402

WORK = os.environ.get("AB_WORK", "c2")  # c2: knn_l2sq f32; c5: knn_cos_bf16; c3: knn_cos_columns
n = int(sys.argv[1]) if len(sys.argv) > 1 else (1_000_000 if WORK == "c2" else 1 << 20)
d = int(sys.argv[2]) if len(sys.argv) > 2 else (768 if WORK == "c2" else 3072)
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
VARS = os.environ["AB_LIBS"].split(";")


def load(path):
    """_lib._load, tolerating symbols an older build does not export."""
    import ctypes as C
    if path not in _lib._LOADED:
        L = C.CDLL(path)
        for name, (res, args) in _lib.SIGNATURES.items():
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype, fn.argtypes = res, args
        _lib._LOADED[path] = L
    return _lib._LOADED[path]


def main():
    global X
    if WORK in ("c2", "c3"):
        X = torch.empty((n, d), dtype=torch.float32, device="cuda")
        _lib.check(_lib.lib().mn_fill_uniform_f32(X.data_ptr(), n, d, 42, 0, None))
    else:
        X = torch.empty((n, d), dtype=torch.bfloat16, device="cuda")
        tmp = torch.empty((1 << 17, d), dtype=torch.float32, device="cuda")
        for r0 in range(0, n, 1 << 17):
            m = min(1 << 17, n - r0)
            _lib.check(_lib.lib().mn_fill_uniform_f32(tmp.data_ptr(), m, d, 47, r0, None))
            X[r0:r0 + m].copy_(tmp[:m])
        del tmp
    torch.cuda.synchronize()
    ref = None
    best = {v: 1e30 for v in VARS}
    for r in range(rounds):
        for v in VARS:
            path, _, knobs = v.partition("|")
            path = path if os.path.isabs(path) else os.path.join(ROOT, path)
            for kv in [x for x in knobs.split(",") if x]:
                k_, val = kv.split("=")
                os.environ[k_] = val
            _lib._LIB = load(path)
            t = time.time()
            if WORK == "c3":
                fi, fd, fw, st = S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0, timing=True)
                torch.cuda.synchronize()
                rec = {"round": r, "v": v, "wall": round(time.time() - t, 4),
                       **{k_: (round(x, 3) if isinstance(x, float) else x) for k_, x in st.items()}}
                if ref is None:
                    ref = (fi.clone(), fd.clone())
                else:
                    rec["same_as_first"] = bool(torch.equal(ref[0], fi) and torch.equal(ref[1], fd))
                best[v] = min(best[v], st["ms_total"])
                for kv in [x for x in knobs.split(",") if x]:
                    os.environ.pop(kv.split("=")[0], None)
                print(json.dumps(rec), flush=True)
                continue
            if WORK == "c2":
                out = S.knn_l2sq(X, 32, timing=True, algo="bf16x1")
                st = out.stats
            else:
                idx, dist, w, st = S.knn_cos_bf16(X, 32, eps=1.0, sigma=1.0, p=2.0, timing=True)

                class _O:
                    pass
                out = _O()
                out.idx, out.dist = idx, dist.view(torch.int64).view(torch.int32)
            torch.cuda.synchronize()
            rec = {"round": r, "v": v, "ms_sweep": round(st["ms_sweep"], 2),
                   "ms_total": round(st["ms_total"], 2), "ms_sample": round(st["ms_sample"], 2),
                   "ms_rerank": round(st["ms_rerank"], 2), "n_cand": st["n_candidates"],
                   "unc": st["n_uncertified"], "wall": round(time.time() - t, 3)}
            if ref is None:
                ref = (out.idx.clone(), out.dist.clone())
            else:
                rec["same_as_first"] = bool(torch.equal(ref[0], out.idx) and
                                            torch.equal(ref[1].view(torch.int32), out.dist.view(torch.int32)))
            best[v] = min(best[v], st["ms_sweep"])
            for kv in [x for x in knobs.split(",") if x]:
                os.environ.pop(kv.split("=")[0], None)
            del out
            print(json.dumps(rec), flush=True)
    print(json.dumps({"summary_ms_sweep": best}))


if __name__ == "__main__":
    main()
