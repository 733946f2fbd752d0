"""The library's f32 ln / exp (csrc/glibc_f32.hpp: glibc's logf / expf
restated on the device) vs the HOST glibc — what the reference's f32::ln /
f32::exp call (surfface-core/src/distance.rs:102, 283-289) — on EVERY f32
input: all 2^32 bit patterns through mn_libm_f32, in chunks, 0 mismatches
(NaN matches any NaN).  The Bhattacharyya kernels (mst.hip, bc.hip) use
exactly these functions."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

CHUNK = 1 << 28


@pytest.mark.parametrize("fn", [0, 1], ids=["logf", "expf"])
def test_every_f32_input_matches_host_glibc(fn):
    import surfface_hip as S
    out = torch.empty(CHUNK, dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    bad = 0
    for b0 in range(0, 1 << 32, CHUNK):
        S._lib.check(S.lib().mn_libm_f32(None, CHUNK, b0, fn, out.data_ptr(), s))
        bad += O.libm_mismatch(b0, out.cpu().numpy(), fn)
    assert bad == 0


def test_array_form_and_special_values():
    import surfface_hip as S
    x = np.array([1.0, 0.0, -0.0, np.inf, -np.inf, np.nan, -1.0, 1e-45, 1e-38, 88.7, 88.73,
                  -103.9, -104.0, 0.5, 2.0, 3.4e38], np.float32)
    xd = torch.from_numpy(x).cuda()
    for fn in (0, 1):
        out = torch.empty_like(xd)
        S._lib.check(S.lib().mn_libm_f32(xd.data_ptr(), len(x), 0, fn, out.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream))
        ref = O.libm_f32(x, fn=fn)
        got = out.cpu().numpy()
        same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
        assert same.all(), (fn, x[~same], got[~same], ref[~same])


def test_pow_f64_matches_host_glibc():
    """The library's f64 pow (csrc/glibc_f64.hpp: glibc's pow restated, used
    for the rational kernel's (d / sigma)^p and sorted_index's 2^p) vs the host
    pow (the oracle's or_pow_f64: libm pow): 4M random pairs — the weight
    kernel's x in [0, 4) with p in {0.5, 2, 3, 2.7, 1}, wide x and y, results
    near the subnormal and overflow limits — and the special values."""
    import surfface_hip as S
    rng = np.random.default_rng(7)
    n = 1 << 20
    xs = [rng.random(n) * 4.0,
          np.ldexp(rng.random(n) + 0.5, rng.integers(-1000, 1000, n)),
          0.5 * (1.0 + rng.random(n)),
          rng.random(n) * 4.0]
    ys = [rng.choice([0.5, 2.0, 3.0, 2.7, 1.0], n),
          (rng.random(n) - 0.5) * np.ldexp(1.0, rng.integers(-6, 14, n)),
          1000.0 + 80.0 * rng.random(n),
          rng.random(n) * 8.0 - 2.0]
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 5e-324, 8.9e307, 2.0, 0.5])
    xs.append(np.repeat(sp, len(sp)))
    ys.append(np.tile(sp, len(sp)))
    s = torch.cuda.current_stream().cuda_stream
    for x, y in zip(xs, ys):
        x = np.ascontiguousarray(x, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        out = torch.empty_like(xd)
        S._lib.check(S.lib().mn_libm_pow_f64(xd.data_ptr(), yd.data_ptr(), len(x), out.data_ptr(), s))
        ref = O.pow_f64(x, y)  # host glibc pow (numpy may use a vector math library)
        got = out.cpu().numpy()
        same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
        assert bool(same.all()), (x[~same][:4], y[~same][:4], got[~same][:4], ref[~same][:4])
