"""native/kernels/tile_queue.h's slot-ownership logic on the CPU: the header is
compiled with g++ against a host-only fake of the HIP calls it makes
(tests/native/fakehip) and run, also under AddressSanitizer/UBSan (the pool is
process-lifetime by design, so leak detection is off). The GPU tests in
tests/test_kernels_gpu.py check the same rules on the MI355X with real
concurrent launches."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "tile_queue_host_test.cpp")
INC = os.path.join(ROOT, "tests", "native", "fakehip")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")


@pytest.mark.parametrize("san", [False, True])
def test_tile_queue_ownership_rules_on_host(tmp_path, san):
    exe = str(tmp_path / "tq")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-I", INC, SRC, "-o", exe]
    if san:
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "tile_queue host test: OK" in r.stdout
