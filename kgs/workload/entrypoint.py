"""gpu-rocm-test pod entrypoint (replaces ``echo Hello from fake ROCm GPU node``).

pods/rocm-gpu-test-pod.yaml runs ``python3 -m kgs.workload.entrypoint --pod``:

1. If the pod got no real GPU (CPU-only host, fake capacity -- BASELINE config 1)
   print the reference's line ``Hello from fake ROCm GPU node``
   (pods/rocm-gpu-test-pod.yaml:9) and hold.
2. Otherwise list the allocated GPUs (native gpuinfo core: the render nodes the
   device plugin passed in), then start one worker process per GPU with
   ``torch.distributed.run`` -- vector add, bf16 MFMA GEMM, RCCL all-reduce
   sweep (:mod:`kgs.workload.worker`) -- and print one JSON result line.
   Before the workers, the native first-GEMM probe (``kgs-gpuprobe``,
   native/probe/gpuprobe.hip: HIP + libkgs_kernels.so, no Python/torch start-up)
   runs one checked 8192^3 GEMM per GPU and prints ``KGS_FIRST_GEMM {...}``:
   the pod's readiness point, ~2 s earlier than the torch worker's first GEMM.
   ``--smoke`` (BASELINE config 2) runs ``rocminfo`` and the HIP vector add
   only: passthrough works and a kernel launches, nothing heavier.
3. ``--pod`` keeps the container Running afterwards (``sleep 3600`` in the
   reference) so ``kubectl logs`` / ``kubectl wait`` behave the same.

The parent never initialises the GPU itself: it counts render nodes and spawns
the workers as children (no exec from a GPU-initialised process).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import time

HELLO_FAKE = "Hello from fake ROCm GPU node"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def allocated_gpus(root: str = "/", environ=None) -> list:
    """The pod's allocation, in HIP device order.

    What the container can see is NOT assumed to be the allocation: a
    privileged container sees every render node of its kind worker. The
    device plugin's Allocate names the GPUs twice -- ``ROCR_VISIBLE_DEVICES``
    (``GPU-<uuid>`` list, the order HIP numbers them) and ``KGS_RENDER_MINORS``
    -- and both filters apply when present."""
    env = os.environ if environ is None else environ
    if env.get("KGS_FAKE_GPUS"):
        return []
    if not os.path.exists(os.path.join(root, "dev/kfd")):
        return []
    try:
        from kgs import gpuinfo

        topo = gpuinfo.discover(root, use_amdsmi=False)
        gpus = [g for g in topo.gpus if g.render_node_present and g.healthy]
    except Exception:
        return []
    alloc = env.get("KGS_RENDER_MINORS")
    if alloc:
        want = {int(x) for x in alloc.split(",") if x.strip()}
        gpus = [g for g in gpus if g.render_minor in want]
    uuids = gpuinfo.parse_rocr_uuids(env.get("ROCR_VISIBLE_DEVICES"))
    if uuids is not None:
        by_uuid = {g.rocr_uuid: g for g in gpus}
        gpus = [by_uuid[u] for u in uuids if u in by_uuid]
    return gpus


def pinned_env(gpus: list, environ=None) -> dict:
    """The environment for this pod's GPU children (probe, torch workers):
    ``ROCR_VISIBLE_DEVICES`` pinned to ``gpus`` by UUID unless Allocate already
    pinned it. Without it a child of a privileged pod would enumerate every GPU
    of the worker and take HIP device 0, whichever GPU that is."""
    from kgs import gpuinfo

    env = dict(os.environ if environ is None else environ)
    if gpus and gpuinfo.parse_rocr_uuids(env.get("ROCR_VISIBLE_DEVICES")) is None:
        try:
            env["ROCR_VISIBLE_DEVICES"] = gpuinfo.rocr_visible_devices(gpus)
        except gpuinfo.GpuInfoUnavailable as e:  # old kernel: only the device nodes isolate the pod
            print(f"kgs workload: WARNING: {e}", file=sys.stderr, flush=True)
    return env


def probe_binary() -> str | None:
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native", "kgs-gpuprobe")
    return exe if os.access(exe, os.X_OK) else None


def run_probe(size: int, timeout: int = 300, env: dict | None = None) -> dict:
    """Native first-GEMM probe over every GPU this process sees.

    The probe prints ``KGS_FIRST_GEMM {...}`` as soon as every device passed
    its checked first GEMM, then runs its throughput loop and prints
    ``KGS_PROBE_TPUT {...}``. The readiness line is forwarded the moment it is
    read (``kgs bench --no-kind`` stops its clock there), not after the probe
    exits. A probe binary that is not built is *skipped*, not a failure: the
    torch workers' GEMM is then the pod's result (``{"skipped": ...}``).
    """
    exe = probe_binary()
    if exe is None:
        return {"skipped": "kgs-gpuprobe not built (python -m kgs.utils.build)"}
    import threading

    import tempfile

    # stderr goes to a file, not a second pipe: a pipe read only after stdout's
    # EOF fills at ~64 KiB (AMD_LOG_LEVEL output) and blocks the probe
    with tempfile.TemporaryFile(mode="w+") as errf:
        proc = subprocess.Popen([exe, "--size", str(size)], stdout=subprocess.PIPE, stderr=errf, text=True,
                                env=env)
        timer = threading.Timer(timeout, proc.kill)
        timer.start()
        res: dict | None = None
        try:
            for line in proc.stdout:
                if line.startswith("KGS_FIRST_GEMM "):
                    print(line.rstrip("\n"), flush=True)
                    res = json.loads(line[len("KGS_FIRST_GEMM "):])
                elif line.startswith("KGS_PROBE_TPUT ") and res is not None:
                    res["throughput"] = json.loads(line[len("KGS_PROBE_TPUT "):])
            rc = proc.wait()
        finally:
            timer.cancel()
        errf.seek(0)
        err = errf.read()
    if res is None:
        sys.stderr.write(err[-2000:])
        why = f"kgs-gpuprobe killed after {timeout}s" if rc < 0 else "no KGS_FIRST_GEMM line"
        return {"ok": False, "rc": rc, "error": why}
    res["rc"] = rc
    return res


def rocminfo_agents(timeout: int = 60, env: dict | None = None) -> dict:
    """GPU agents reported by ``rocminfo`` (run as a child process: the parent
    never initialises the GPU itself)."""
    exe = shutil.which("rocminfo") or shutil.which("rocminfo", path="/opt/rocm/bin")
    if exe is None:
        return {"ok": False, "error": "rocminfo not found"}
    try:
        r = subprocess.run([exe], capture_output=True, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"ok": False, "error": "rocminfo timed out"}
    names = [ln.split(":", 1)[1].strip() for ln in r.stdout.splitlines()
             if ln.strip().startswith("Name:") and "gfx" in ln]
    return {"ok": r.returncode == 0 and bool(names), "gpu_agents": names}


def collect_counters(a, env) -> dict:
    """Run the single-GPU worker (GEMM only) under rocprofv3, one pass per
    counter set, and return the markdown summary plus the raw directory."""
    from kgs.utils.profile import COUNTER_SETS, pmc_command, summarize

    worker = [sys.executable, "-m", "kgs.workload.worker", "--gemm-size", str(a.gemm_size), "--gemm-iters", "5",
              "--skip-allreduce"]
    env1 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    ok = {}
    for name, counters in COUNTER_SETS.items():
        outdir = os.path.join(a.counters_dir, f"pmc_{name}")
        cmd = pmc_command(worker, outdir, counters, name="gemm")
        try:
            r = subprocess.run(cmd, env=env1, capture_output=True, text=True, timeout=a.timeout)
            ok[name] = r.returncode == 0
        except (FileNotFoundError, subprocess.TimeoutExpired) as e:
            ok[name] = f"failed: {e}"
            break
    summary = summarize(a.counters_dir, flops=2.0 * a.gemm_size ** 3)
    print(summary, flush=True)
    return {"dir": a.counters_dir, "passes": ok}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgs-workload")
    ap.add_argument("--pod", action="store_true", help="hold the container after the run (sleep)")
    ap.add_argument("--hold", type=int, default=3600)
    ap.add_argument("--gemm-size", type=int, default=8192)
    ap.add_argument("--gemm-iters", type=int, default=20)
    ap.add_argument("--allreduce-sizes", default="")
    ap.add_argument("--nproc", type=int, default=0, help="override the GPU count")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--timeout", type=int, default=1200)
    ap.add_argument("--counters", action="store_true",
                    help="re-run one GPU's GEMM under rocprofv3 (MFMA busy, LDS conflicts, L2 hit) and summarise")
    ap.add_argument("--counters-dir", default="/tmp/kgs-rocprof")
    ap.add_argument("--smoke", action="store_true", help="config 2: rocminfo + HIP vector add only")
    ap.add_argument("--fp8", action="store_true", help="also report the e4m3 GEMM TFLOPS")
    ap.add_argument("--p2p", action="store_true", help="multi-GPU pods: P2P all-reduce latency vs RCCL")
    ap.add_argument("--no-probe", action="store_true", help="skip the native first-GEMM probe")
    ap.add_argument("--probe-only", action="store_true",
                    help="run the native first-GEMM probe and stop (no torch workers)")
    a = ap.parse_args(argv)

    gpus = allocated_gpus()
    n = a.nproc or len(gpus)
    result: dict = {"mode": "fake" if n == 0 else "gpu", "n_gpus": n, "t_start": time.time()}
    if n == 0:
        print(HELLO_FAKE, flush=True)
    else:
        print(f"kgs workload: {n} GPU(s) allocated", flush=True)
        for g in gpus:
            print(f"  renderD{g.render_minor} {g.bdf} {g.gfx_arch} {g.cu_count} CUs {g.num_xcc} XCDs "
                  f"{g.vram_bytes / 2**30:.0f} GiB numa{g.numa_node}", flush=True)
        env = pinned_env(gpus)
        result["rocr_visible_devices"] = env.get("ROCR_VISIBLE_DEVICES")
        if a.smoke:
            result["rocminfo"] = rocminfo_agents(env=env)
            print(f"rocminfo GPU agents: {result['rocminfo'].get('gpu_agents')}", flush=True)
        if not a.smoke and not a.no_probe and a.gemm_size % 256 == 0:
            result["first_gemm"] = run_probe(a.gemm_size, a.timeout, env)
            # only a probe that ran and failed its check fails the pod
            if "skipped" not in result["first_gemm"] and not result["first_gemm"].get("ok"):
                result["all_ok"] = False
        if a.probe_only:
            return _finish(a, result, rc=0 if result.get("all_ok", True) else 1)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (":" + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        worker = ["-m", "kgs.workload.worker", "--gemm-size", str(a.gemm_size), "--gemm-iters", str(a.gemm_iters)]
        if n == 1:
            # one GPU: no process group to set up, skip torchrun's agent (~1 s)
            env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
            cmd = [sys.executable, *worker]
        else:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                   "--master-addr=127.0.0.1", f"--master-port={_free_port()}", *worker]
        if a.allreduce_sizes:
            cmd += ["--allreduce-sizes", a.allreduce_sizes]
        if a.smoke:
            cmd += ["--skip-gemm", "--skip-allreduce"]
        if a.fp8:
            cmd += ["--fp8"]
        if a.p2p:
            cmd += ["--p2p"]
        ok_before = result.get("all_ok", True)
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout)
        sys.stderr.write(p.stderr[-4000:])
        for line in p.stdout.splitlines():
            if line.startswith("KGS_RESULT "):
                result.update(json.loads(line[len("KGS_RESULT "):]))
                result["all_ok"] = ok_before and result.get("all_ok", True)
            else:
                print(line, flush=True)
        result["worker_rc"] = p.returncode
        if a.counters and p.returncode == 0:
            result["counters"] = collect_counters(a, env)
    return _finish(a, result)


def _finish(a, result: dict, rc: int | None = None) -> int:
    result["t_end"] = time.time()
    line = json.dumps(result)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    if rc is None:
        rc = 0 if result.get("worker_rc", 0) == 0 and result.get("all_ok", True) else 1
    if a.smoke and result.get("n_gpus") and not result.get("rocminfo", {}).get("ok"):
        rc = 1
    if a.pod:
        time.sleep(a.hold)
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
