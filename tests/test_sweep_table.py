"""CPU check of the symmetric sweep's block tables (gram_sweep2.hpp
sym_block_table, every order): each upper-triangle tile (I, J >= I) is
covered exactly once, the diagonal tile is only ever a block's first tile,
and the XCD-group table (order 2) has a length the kernel's xcd_remap splits
evenly.  The header's own host code, compiled with hipcc, run on the host."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_sym_block_tables_cover_each_tile_once(tmp_path):
    exe = str(tmp_path / "sym_table_check")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17",
                    "-I", os.path.join(ROOT, "matternet-rs_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "sym_table_check.hip"), "-o", exe],
                   check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0 and "bad 0" in r.stdout, r.stdout + r.stderr
