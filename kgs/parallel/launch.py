"""Single-node self-launch: one worker process per GPU, no torchrun needed.

``python bench.py --gpus 8`` (no ``WORLD_SIZE`` in the environment) becomes a
thin parent that spawns 8 children with the torchrun env contract
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``LOCAL_WORLD_SIZE``/``MASTER_ADDR``/
``MASTER_PORT``), waits for them, and exits with the first non-zero child
status. The parent never initialises the GPU: it only *counts* devices
(``torch.cuda.device_count()`` does not create a HIP context on this image),
so there is no forked/exec'd process that inherited a live GPU context.

Children are started with ``subprocess.Popen`` (fork+exec of a fresh Python
before anything touches the GPU) in their own process group; if one rank
fails the others are terminated so a rendezvous never hangs.

The reference has no multi-process runtime; this is the
launcher for BASELINE.json config 4 (one pod holding 8 GPUs).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def needs_self_launch(nproc: int, env=None) -> bool:
    """True when ``nproc`` ranks are wanted but no launcher set WORLD_SIZE."""
    env = os.environ if env is None else env
    return nproc > 1 and env.get("WORLD_SIZE") in (None, "")


def visible_gpu_count() -> int:
    """Count GPUs without creating a HIP context (safe in the parent)."""
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover - torch is in the image
        return 0


def rank_env(rank: int, world: int, port: int, base=None, addr: str = "127.0.0.1") -> dict:
    env = dict(os.environ if base is None else base)
    env.update({
        "RANK": str(rank),
        "LOCAL_RANK": str(rank),
        "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(world),
        "GROUP_RANK": "0",
        "MASTER_ADDR": addr,
        "MASTER_PORT": str(port),
        # dmabuf IPC is the only mode the host driver supports (RCCL P2P)
        "HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    })
    return env


def spawn_local(nproc: int, argv: Sequence[str], *, require_gpus: bool = True, poll_s: float = 0.05,
                timeout_s: float | None = None) -> int:
    """Run ``[python, *argv]`` as ``nproc`` ranks on this node; return an exit code.

    ``require_gpus``: refuse (exit 1) when fewer than ``nproc`` GPUs are
    visible -- over-subscribing a GPU with several RCCL ranks is not the
    benchmark. CPU/gloo runs pass ``False``.
    """
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    if require_gpus:
        have = visible_gpu_count()
        if have < nproc:
            print(f"[launch] --gpus {nproc} but only {have} GPU(s) visible", file=sys.stderr)
            return 1
    port = free_port()
    procs: list[subprocess.Popen] = []
    for r in range(nproc):
        procs.append(subprocess.Popen([sys.executable, *argv], env=rank_env(r, nproc, port),
                                      start_new_session=True))
    t0 = time.monotonic()
    rc = 0
    try:
        alive = set(range(nproc))
        while alive:
            for r in list(alive):
                st = procs[r].poll()
                if st is None:
                    continue
                alive.discard(r)
                if st != 0 and rc == 0:
                    print(f"[launch] rank {r} exited with {st}; stopping the others", file=sys.stderr)
                    rc = st if st > 0 else 128 - st
                    _terminate(procs)
            if alive and timeout_s is not None and time.monotonic() - t0 > timeout_s:
                print(f"[launch] timeout after {timeout_s:.0f}s", file=sys.stderr)
                rc = rc or 124
                _terminate(procs)
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        _terminate(procs)
        rc = 130
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            _kill_group(p, signal.SIGKILL)
            p.wait()
    return rc


def _kill_group(p: subprocess.Popen, sig) -> None:
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _terminate(procs) -> None:
    for p in procs:
        if p.poll() is None:
            _kill_group(p, signal.SIGTERM)
