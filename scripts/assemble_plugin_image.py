"""Assemble the device-plugin image's final filesystem on the host, no docker.

Runs images/Dockerfile.deviceplugin's build and final stages with
tests/dockerfile_exec.py (the executor the CPU image tests use): the ROCm stage
is served by this machine's /opt/rocm, so the tree ships the same
libamd_smi / libdrm files the image would copy, next to the gpuinfo core the
build stage compiled. The result is what `docker build` would put under /opt/kgs:

    python scripts/assemble_plugin_image.py [--out images/_assembled/deviceplugin]

tests/test_plugin_image_gpu.py runs the plugin from that tree on the MI355X box
with LD_LIBRARY_PATH = the tree's lib/ only.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCKERFILE = os.path.join(ROOT, "images", "Dockerfile.deviceplugin")
DEFAULT_OUT = os.path.join(ROOT, "images", "_assembled", "deviceplugin")


def _relink_sonames(lib: str) -> None:
    """COPY follows symlinks, so libX.so, libX.so.N and libX.so.N.M arrive as
    three identical files; put the ROCm install's links back (the tree is
    pushed to the GPU box on every call: 5.6 MB less)."""
    by_digest: dict = {}
    for name in sorted(os.listdir(lib), key=len, reverse=True):  # the full version first
        path = os.path.join(lib, name)
        if os.path.islink(path) or not os.path.isfile(path):
            continue
        with open(path, "rb") as f:
            d = hashlib.sha256(f.read()).hexdigest()
        if d in by_digest:
            os.unlink(path)
            os.symlink(by_digest[d], path)
        else:
            by_digest[d] = name


def assemble(out: str = DEFAULT_OUT, python: str = sys.executable) -> dict:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from dockerfile_exec import Executor  # noqa: E402

    work = tempfile.mkdtemp(prefix="kgs-dpimg-", dir="/tmp")
    try:
        ex = Executor(DOCKERFILE, ROOT, work, host_stages=("rocm",), python=python)
        ex.run_stage("build")
        final = ex.run_stage(ex.stages[-1].name)
        if os.path.exists(out):
            shutil.rmtree(out)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        shutil.copytree(final, out, symlinks=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)
    _relink_sonames(os.path.join(out, "opt", "kgs", "lib"))
    with open(DOCKERFILE, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    info = {"dockerfile": os.path.relpath(DOCKERFILE, ROOT), "dockerfile_sha256": sha, "assembled_at": time.time(),
            "skipped": [why for _, _, why in ex.skipped], "lib": sorted(os.listdir(os.path.join(out, "opt/kgs/lib"))),
            "native": sorted(os.listdir(os.path.join(out, "opt/kgs/kgs/_native")))}
    with open(os.path.join(out, "ASSEMBLED.json"), "w") as f:
        json.dump(info, f, indent=1)
    return info


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=DEFAULT_OUT)
    a = ap.parse_args(argv)
    print(json.dumps(assemble(a.out), indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
