"""Race / memory detection on the host side (SURVEY.md §5 "race detection"):
the CPU oracle and the library's host-side planners built with
AddressSanitizer + UndefinedBehaviorSanitizer and run on the CPU.

* the oracle (oracle/Makefile `asan`: tests/native/oracle_asan.c drives every
  entry point on random, one-row, k > n - 1 and NaN-lambda inputs);
* the host C++ that decides what the kernels index — the symmetric block
  tables and their rank shares (gram_sweep2.hpp), the sweep and phase-1 Gram
  slicing / buffer sizing (plan_sweep, plan_gram) and the sharded build's plan
  (shard_sym.hpp) — compiled by hipcc with the sanitizers on the host side
  only (`-Xarch_host -fsanitize=...`; GPU sanitizers are not available).
A sanitizer report makes the program exit non-zero (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1")


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("make") is None,
                    reason="gcc / make not installed")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_asan")
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan", f"ASAN_OUT={exe}"],
                       capture_output=True, text=True)
    assert b.returncode == 0, b.stdout + b.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
    print(r.stdout)
    assert r.returncode == 0 and "rc 0" in r.stdout, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src", ["host_plans_check.hip", "sym_table_check.hip"])
def test_host_planners_under_asan_ubsan(tmp_path, src):
    exe = str(tmp_path / src.replace(".hip", ""))
    b = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17",
                        "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                        "-Xarch_host", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer",
                        "-I", os.path.join(ROOT, "matternet-rs_amd", "csrc"),
                        "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "native", src), "-o", exe],
                       capture_output=True, text=True)
    assert b.returncode == 0, b.stderr[-4000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
    print(r.stdout)
    assert r.returncode == 0 and "bad 0" in r.stdout, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
