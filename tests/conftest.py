"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs the oracle-vs-golden checks, host logic and the C-ABI
export checks on CPU; `-m gpu` runs the parity tests through the C ABI on a
real MI355X.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "matternet-rs_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C ABI)")
