#!/usr/bin/env python3
"""The parts of create -> GPU-pod-Running that run without docker/kind, timed on
a real MI355X host. The full metric needs a docker + kind host (docs/e2e.md).

  gpuinfo_discover_ms        native KFD/amd-smi discovery (what `kgs create` and
                             the plugin do first)
  plugin_register_ms         plugin server start -> kubelet Register accepted
  plugin_first_list_ms       ... -> first ListAndWatch device list at the kubelet
                             (the moment the node's amd.com/gpu capacity appears)
  plugin_allocate_ms         one Allocate of every device (pod admission)
  plugin_process_selftest_s  `python -m kgs.deviceplugin --self-test` wall time
                             (container cold start: interpreter, grpc, discovery)
  pod_smoke_s                `kgs.workload.entrypoint --smoke`: container command
                             start -> rocminfo + first HIP kernel result
  pod_first_gemm_s           entrypoint start -> first 8192^3 GEMM result (torch
                             import, HIP init, one worker process)

Prints one JSON object; `--out` writes it too.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _median_ms(fn, n=5):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(statistics.median(ts), 3)


def plugin_timings(root="/"):
    from kgs.deviceplugin.fake_kubelet import FakeKubelet
    from kgs.deviceplugin.server import AmdGpuDevicePlugin, RealSource

    src = RealSource(root)
    devs = src.devices()
    with tempfile.TemporaryDirectory(prefix="kgs-dp-") as d:
        kub = FakeKubelet(d)
        kub.start()
        t0 = time.perf_counter()
        plug = AmdGpuDevicePlugin(src, "amd.com/gpu", plugin_dir=d)
        plug.start()
        plug.register()
        t_reg = time.perf_counter()
        plug.notify()
        kub.wait(lambda: bool(kub.device_lists), timeout=10)
        t_list = time.perf_counter()
        ids = [dv.id for dv in devs]
        t1 = time.perf_counter()
        kub.allocate(ids)
        t_alloc = time.perf_counter()
        plug.stop()
        kub.stop()
    return {"devices": len(devs), "plugin_register_ms": round((t_reg - t0) * 1e3, 3),
            "plugin_first_list_ms": round((t_list - t0) * 1e3, 3),
            "plugin_allocate_ms": round((t_alloc - t1) * 1e3, 3)}


def timed_cmd(argv, timeout=900):
    env = dict(os.environ, PYTHONPATH=ROOT)
    t0 = time.perf_counter()
    r = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"{argv} failed ({r.returncode}): {r.stderr[-2000:]}")
    return round(dt, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from kgs import gpuinfo

    res = {"gpuinfo_backend": gpuinfo.backend_name(),
           "gpuinfo_discover_ms": _median_ms(lambda: gpuinfo.discover("/"))}
    res.update(plugin_timings())
    py = sys.executable
    res["plugin_process_selftest_s"] = timed_cmd([py, "-m", "kgs.deviceplugin", "--self-test",
                                                  "--partition-file", "/nonexistent"])
    res["pod_smoke_s"] = timed_cmd([py, "-m", "kgs.workload.entrypoint", "--smoke", "--nproc", "1"])
    res["pod_first_gemm_s"] = timed_cmd([py, "-m", "kgs.workload.entrypoint", "--nproc", "1", "--gemm-size", "8192",
                                         "--gemm-iters", "1"])
    res["note"] = ("components of create->Running measurable without docker/kind; kind create, image pulls "
                   "and the kubelet's own pod start are not included")
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
