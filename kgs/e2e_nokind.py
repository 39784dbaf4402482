"""``kgs bench --no-kind``: the measurable tail of create -> GPU pod Running on a
host without docker/kind, chained into ONE timed flow.

The reference's CI chain (/root/reference/.github/workflows/rocm-ci.yaml:28-39:
create, `kubectl create -f pods/rocm-gpu-test-pod.yaml`, wait Ready, logs) is
kind + kubelet + containerd around two pieces this repository owns: the device
plugin and the pod's entrypoint. This flow runs exactly those pieces, in order,
with the kubelet's device-plugin side played by the in-tree fake kubelet
(kgs.deviceplugin.fake_kubelet -- the same v1beta1 gRPC the real kubelet speaks):

  plugin-process-start  spawn ``python -m kgs.deviceplugin`` (its own process,
                        live discovery with amd-smi) until its socket exists
  plugin-register       ... until its Register reached the kubelet
  capacity              ... until ListAndWatch advertised >= N healthy devices
  allocate              GetPreferredAllocation + Allocate of N devices (the
                        pod-admission RPCs)
  pod-first-gemm        start the pod entrypoint as a child with exactly the
                        Allocate response's envs (which pin ROCr to the
                        allocated GPUs by UUID: ROCR_VISIBLE_DEVICES), until its
                        first checked 8192^3 GEMM result line (``KGS_FIRST_GEMM``
                        from the native probe, or the worker's result when the
                        probe is not built)
  pod-workload          (reported, not in the value) the rest of the pod's run:
                        the torch workers' GEMM / all-reduce workload

What is NOT in the number (needs docker/kind, docs/e2e.md): kind create, image
build/pull, containerd's container start and the kubelet's own pod sync.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

from .timing import PhaseTimer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _wait(pred, timeout: float, what: str, proc=None) -> None:
    deadline = time.monotonic() + timeout
    delay = 0.001
    while not pred():
        if proc is not None and proc.poll() is not None:
            raise RuntimeError(f"{what}: device plugin exited with {proc.returncode}")
        if time.monotonic() > deadline:
            raise TimeoutError(f"{what}: not reached within {timeout:.0f}s")
        time.sleep(delay)
        delay = min(delay * 2, 0.02)


def visible_devices_for(minors: list, root: str = "/") -> str:
    """ROCR_VISIBLE_DEVICES for the allocated render minors: ROCr enumerates GPU
    agents in KFD node order, which is gpuinfo's index order."""
    from . import gpuinfo

    idx = {g.render_minor: g.index for g in gpuinfo.discover(root, use_amdsmi=False).gpus}
    missing = [m for m in minors if m not in idx]
    if missing:
        raise RuntimeError(f"allocated render minors {missing} not in the KFD topology")
    return ",".join(str(idx[m]) for m in minors)


def _line_reader(stream):
    """Lines of ``stream`` through a queue, so the caller can wait on them
    with a deadline (a pod stuck before its first line, e.g. in HIP init, must
    not block the flow forever). ``None`` marks EOF."""
    import queue
    import threading

    q: queue.Queue = queue.Queue()

    def pump():
        try:
            for line in stream:
                q.put(line)
        finally:
            q.put(None)

    threading.Thread(target=pump, name="kgs-pod-stdout", daemon=True).start()
    return q


def run_nokind(gpus: int = 1, dev_root: str = "/", fake_gpus: int = 0, gemm_size: int = 8192,
               timeout: float = 600.0, timings_json: str | None = None, out=print, keep_dir: bool = False,
               advertise: int | None = None) -> int:
    summary = nokind_once(gpus=gpus, dev_root=dev_root, fake_gpus=fake_gpus, gemm_size=gemm_size, timeout=timeout,
                          timings_json=timings_json, keep_dir=keep_dir, advertise=advertise)
    out(json.dumps(summary))
    return 0


def advertised_minors(dev_root: str, n: int | None) -> list | None:
    """Render minors the plugin may advertise for ``--gpus N``: the same
    selection ``kgs create --gpus N`` makes (kgs.cluster.select_gpus)."""
    if n is None:
        return None
    from . import gpuinfo
    from .cluster import select_gpus

    usable = [g for g in gpuinfo.discover(dev_root, use_amdsmi=False).gpus if g.render_minor >= 0 and g.healthy]
    return [g.render_minor for g in select_gpus(usable, n)]


def nokind_once(gpus: int = 1, dev_root: str = "/", fake_gpus: int = 0, gemm_size: int = 8192,
                timeout: float = 600.0, timings_json: str | None = None, keep_dir: bool = False,
                advertise: int | None = None) -> dict:
    """One chained run; returns the summary. ``advertise``: the plugin
    advertises exactly that many GPUs (None = all); the pod takes ``gpus``."""
    import queue

    from .deviceplugin.fake_kubelet import FakeKubelet

    t = PhaseTimer()
    allowed = None if fake_gpus else advertised_minors(dev_root, advertise)
    d = tempfile.mkdtemp(prefix="kgs-nk-", dir="/tmp")  # unix socket paths stay short
    py = sys.executable
    env_base = dict(os.environ)
    env_base["PYTHONPATH"] = REPO + (":" + env_base["PYTHONPATH"] if env_base.get("PYTHONPATH") else "")
    plug_env = dict(env_base)
    if allowed is not None:
        plug_env["KGS_ALLOWED_RENDER_MINORS"] = ",".join(str(m) for m in allowed)
    kub = FakeKubelet(d)
    kub.start()
    plug = None
    result: dict = {}
    try:
        argv = [py, "-m", "kgs.deviceplugin", "--plugin-dir", d, "--dev-root", dev_root,
                "--partition-file", os.path.join(d, "no-partition.json"), "--ready-file", os.path.join(d, "ready"),
                "--health-interval", "1"]
        if fake_gpus:
            argv += ["--fake-gpus", str(fake_gpus)]
        with t.phase("plugin-process-start"):
            plug_log = open(os.path.join(d, "plugin.log"), "w")
            plug = subprocess.Popen(argv, env=plug_env, stdout=plug_log, stderr=subprocess.STDOUT)
            plug_log.close()
            sock = os.path.join(d, "kgs-amdgpu.sock")
            _wait(lambda: os.path.exists(sock), timeout, "plugin socket", plug)
        with t.phase("plugin-register"):
            _wait(lambda: bool(kub.registrations), timeout, "Register", plug)
        with t.phase("capacity") as rec:
            want_cap = len(allowed) if allowed is not None else gpus
            _wait(lambda: kub.capacity() >= max(gpus, want_cap), timeout, f"{want_cap} healthy amd.com/gpu", plug)
            rec["advertised"] = kub.capacity()
            if allowed is not None and rec["advertised"] != len(allowed):
                raise RuntimeError(f"plugin advertised {rec['advertised']} GPUs, expected exactly {len(allowed)}")
        with t.phase("allocate") as rec:
            healthy = [i for i, h, _ in kub.latest_devices() if h == "Healthy"]
            ids = kub.preferred(healthy, [], gpus) if gpus < len(healthy) else healthy[:gpus]
            resp = kub.allocate(ids).container_responses[0]
            envs = dict(resp.envs)
            rec.update(device_ids=ids, device_paths=[s.host_path for s in resp.devices])
        env = dict(env_base, **envs)
        minors = [int(x) for x in envs.get("KGS_RENDER_MINORS", "").split(",") if x]
        if minors and "ROCR_VISIBLE_DEVICES" not in envs:
            # GPUs without a KFD unique_id: Allocate could not pin by UUID
            env["ROCR_VISIBLE_DEVICES"] = visible_devices_for(minors, dev_root)
        res_path = os.path.join(d, "pod_result.json")
        cmd = [py, "-m", "kgs.workload.entrypoint", "--gemm-size", str(gemm_size), "--gemm-iters", "10",
               "--json-out", res_path]
        err_path = os.path.join(d, "pod.stderr")
        with t.phase("pod-first-gemm") as rec:
            with open(err_path, "w") as err:
                pod = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=err, text=True, cwd=REPO)
            lines = _line_reader(pod.stdout)
            try:
                deadline = time.monotonic() + timeout
                first = None
                eof = False
                while True:  # the readiness line, as soon as the pod prints it
                    try:
                        line = lines.get(timeout=max(0.01, deadline - time.monotonic()))
                    except queue.Empty:
                        raise TimeoutError(f"pod first GEMM not reached within {timeout:.0f}s") from None
                    if line is None:
                        eof = True
                        break
                    if line.startswith("KGS_FIRST_GEMM "):
                        first = json.loads(line[len("KGS_FIRST_GEMM "):])
                        break
                if first is not None:
                    if not first.get("ok"):
                        raise RuntimeError(f"pod first-GEMM probe failed: {first}")
                    rec.update(source="kgs-gpuprobe", probe_ready_s=first.get("t_first_gemm_s"))
                else:
                    rec.update(source="worker")  # no probe: the clock stops when the pod's run ends
                    pod.wait(timeout=max(1.0, deadline - time.monotonic()))
            except BaseException:
                pod.kill()
                pod.wait()
                raise
        with t.phase("pod-workload") as rec:
            try:
                rc = pod.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                pod.kill()
                pod.wait()
                raise
            while not eof:  # drain what the pump thread still holds
                eof = lines.get() is None
            pod.stdout.close()
            if rc != 0:
                with open(err_path) as f:
                    raise RuntimeError(f"pod entrypoint failed ({rc}): {f.read()[-2000:]}")
            with open(res_path) as f:
                result = json.load(f)
            rec.update(mode=result.get("mode"), n_gpus=result.get("n_gpus"), in_value=False)
        t.meta.update(pod_result=result, gpus_requested=gpus, fake=bool(fake_gpus), advertised_minors=allowed,
                      allocate_envs=envs, rocr_visible_devices=env.get("ROCR_VISIBLE_DEVICES"))
    finally:
        if plug is not None and plug.poll() is None:
            plug.terminate()
            try:
                plug.wait(timeout=10)
            except subprocess.TimeoutExpired:
                plug.kill()
        kub.stop()
        t.write(timings_json)
        if not keep_dir:
            shutil.rmtree(d, ignore_errors=True)
    phases = {p["phase"]: p["seconds"] for p in t.phases}
    workload_s = phases.pop("pod-workload", None)
    first_src = next((p.get("source") for p in t.phases if p["phase"] == "pod-first-gemm"), None)
    summary = {"metric": "device-plugin start -> first in-pod GEMM (no kind)", "value": round(sum(phases.values()), 4),
               "unit": "s", "gpus": gpus, "advertised": len(allowed) if allowed is not None else None,
               "fake": bool(fake_gpus), "phases": phases,
               "first_gemm_source": first_src,
               "pod_workload_s": workload_s,
               # both readiness points side by side -- the native
               # probe's first checked GEMM, and the end of the torch workload's run
               "to_first_probe_gemm_s": round(sum(phases.values()), 4),
               "to_workload_done_s": round(sum(phases.values()) + (workload_s or 0.0), 4),
               "excluded": "kind create, image build/pull, containerd container start, kubelet pod sync"}
    if result.get("gemm_tflops_total"):
        summary["in_pod_gemm_tflops"] = result["gemm_tflops_total"]
    return summary
