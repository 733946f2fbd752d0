"""Library calibration for K1 (tuning only, not part of the product path):
the TFLOP/s torch.mm (hipBLASLt / rocBLAS on this image) reaches on the
Gram shape of the sweep, K = 768 fp16 / bf16, f32 accumulate, against which
the hand-written sweep's K loop is read.  Prints one line per shape."""
import json
import sys

import torch


def main():
    dev = torch.device("cuda:0")
    out = []
    for dt in (torch.float16, torch.bfloat16):
        for m, n, k in ((16384, 16384, 768), (32768, 32768, 768), (65536, 65536, 768),
                        (65536, 65536, 1024), (32768, 32768, 4096)):
            a = torch.randn(m, k, device=dev, dtype=dt)
            b = torch.randn(n, k, device=dev, dtype=dt)
            c = torch.empty(m, n, device=dev, dtype=dt)
            for _ in range(3):
                torch.mm(a, b.t(), out=c)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 10
            e0.record()
            for _ in range(it):
                torch.mm(a, b.t(), out=c)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / it
            tf = 2.0 * m * n * k / (ms * 1e-3) / 1e12
            r = {"dtype": str(dt).split(".")[-1], "m": m, "n": n, "k": k, "ms": round(ms, 3),
                 "tflops": round(tf, 1), "frac_of_2500": round(tf / 2500.0, 4)}
            out.append(r)
            print(json.dumps(r), flush=True)
            del a, b, c
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
