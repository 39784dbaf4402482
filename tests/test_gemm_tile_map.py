"""The four-wave GEMM's workgroup -> tile maps are bijections (host, no GPU).

native/testing/tile_map_check.hip includes native/kernels/gemm_w4.h and runs
kgs::w4::tile_of -- the exact function the kernel calls -- on the host for the
default map, GROUP_M 8, the XCD-blocked maps (MAP 1-3), GROUP_N (MAP 4) and
split-K grids, over aligned and ragged tile grids: every (slice, tile) must come
from exactly one workgroup, or tiles would be skipped or written twice.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_tile_maps_are_bijections(tmp_path):
    exe = tmp_path / "tile_map_check"
    src = os.path.join(ROOT, "native", "testing", "tile_map_check.hip")
    subprocess.run([HIPCC, "-std=c++17", "-O1", "--offload-host-only", f"-I{ROOT}/native/kernels", src, "-o",
                    str(exe)], check=True, capture_output=True, text=True, cwd=str(tmp_path))
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = r.stdout.splitlines()
    assert lines and all(ln.startswith("ok ") for ln in lines), r.stdout
    # the default map makes all eight XCDs share B columns on a tall grid (the
    # round-3 finding); the blocked map 1 and GROUP_N cut that to two
    assert "ok X=0 grid 32x16 slices 1: bijection, wave-1 B-column sharing 8 XCDs" in lines
    assert "ok X=10000000 grid 32x16 slices 1: bijection, wave-1 B-column sharing 2 XCDs" in lines
    assert "ok X=40000000 grid 32x16 slices 1: bijection, wave-1 B-column sharing 2 XCDs" in lines
    shutil.rmtree(tmp_path, ignore_errors=True)
