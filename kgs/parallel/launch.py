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

import collections
import json
import os
import signal
import socket
import subprocess
import sys
import threading
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


class _Tee:
    """Forward a child's pipe to ours line by line, keeping the last lines
    (the stderr tail of a failing rank goes into the error report) and
    noting whether a JSON result line went by."""

    def __init__(self, src, dst, keep: int = 40):
        self.tail: collections.deque = collections.deque(maxlen=keep)
        self.json_lines = 0
        self._t = threading.Thread(target=self._pump, args=(src, dst), daemon=True)
        self._t.start()

    def _pump(self, src, dst):
        for raw in iter(src.readline, b""):
            line = raw.decode(errors="replace")
            self.tail.append(line.rstrip("\n"))
            if line.startswith("{"):
                self.json_lines += 1
            try:
                dst.write(line)
                dst.flush()
            except ValueError:  # our stream closed during teardown
                pass
        src.close()

    def join(self, timeout: float = 5.0) -> None:
        self._t.join(timeout)


def spawn_local(nproc: int, argv: Sequence[str], *, require_gpus: bool = True, poll_s: float = 0.05,
                timeout_s: float | None = None, error_report: dict | None = None) -> int:
    """Run ``[python, *argv]`` as ``nproc`` ranks on this node; return an exit code.

    ``require_gpus``: refuse (exit 1) when fewer than ``nproc`` GPUs are
    visible -- over-subscribing a GPU with several RCCL ranks is not the
    benchmark. CPU/gloo runs pass ``False``.

    ``timeout_s``: the whole launch is killed after that long (exit 124).
    ``error_report``: on any failure (a rank exits non-zero, or the timeout)
    and when no rank has printed a JSON line, print ONE JSON line to stdout:
    these fields plus ``"status": "error"``, the reason, the failing (or
    still-running) ranks and their stderr tails -- so a driver that parses the
    last JSON line sees a diagnosis, never silence.
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
    outs: list[_Tee] = []
    errs: list[_Tee] = []
    for r in range(nproc):
        p = subprocess.Popen([sys.executable, *argv], env=rank_env(r, nproc, port), start_new_session=True,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        procs.append(p)
        outs.append(_Tee(p.stdout, sys.stdout))
        errs.append(_Tee(p.stderr, sys.stderr))
    t0 = time.monotonic()
    rc = 0
    failure: dict | None = None
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
                    failure = {"reason": f"rank {r} exited with status {st}", "failing_rank": r, "exit_code": st,
                               "ranks": [r]}
                    _terminate(procs)
            if alive and timeout_s is not None and time.monotonic() - t0 > timeout_s:
                print(f"[launch] timeout after {timeout_s:.0f}s", file=sys.stderr)
                rc = rc or 124
                if failure is None:
                    stuck = sorted(alive)
                    failure = {"reason": f"launch timeout after {timeout_s:.0f}s; ranks {stuck} still running",
                               "failing_rank": stuck[0], "exit_code": 124, "ranks": stuck}
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
    for t in outs + errs:
        t.join()
    if failure is not None and error_report is not None and outs and outs[0].json_lines == 0:
        report = dict(error_report)
        report.update(status="error", n_ranks=nproc, elapsed_s=round(time.monotonic() - t0, 2), **failure)
        report["stderr_tail"] = {str(r): list(errs[r].tail)[-20:] for r in failure["ranks"][:4]}
        print(json.dumps(report), flush=True)
    return rc


def inject_fault(rank: int, where: str) -> None:
    """Test hook for the launch failure paths (CPU tests only):
    ``KGS_FAULT=<where>:<rank>:stall:<seconds>`` sleeps that rank at ``where``;
    ``KGS_FAULT=<where>:<rank>:raise`` makes it raise."""
    spec = os.environ.get("KGS_FAULT")
    if not spec:
        return
    parts = spec.split(":")
    if len(parts) < 3 or parts[0] != where or int(parts[1]) != rank:
        return
    if parts[2] == "stall":
        time.sleep(float(parts[3]) if len(parts) > 3 else 3600.0)
    elif parts[2] == "raise":
        raise RuntimeError(f"injected fault at {where} on rank {rank}")


_report_lock = threading.RLock()  # re-entrant: the SIGTERM handler runs on the main thread
_reported = False


def report_once(obj: dict) -> bool:
    """Print ``obj`` as THE JSON line of this process (the result, or the
    error) unless one was already printed: an exception handler, the SIGTERM
    handler and the watchdog can all race to report the same failure, and a
    signal after the result must not add an error line. True if this printed."""
    global _reported
    with _report_lock:
        if _reported:
            return False
        _reported = True
        print(json.dumps(obj), flush=True)
        return True


class Watchdog:
    """Bounds one rank's whole run: after ``timeout_s`` it reports where every
    rank was (rank 0: one JSON error line on stdout) and hard-exits 124, so a
    stalled rank ends a torchrun / driver run cleanly instead of at the
    driver's own limit with no output.

    Ranks publish their phase (``set_phase``) to the rendezvous store as
    ``kgs/phase/<rank>`` = ``<ordinal>:<name>``; rank 0's watchdog reads them
    over a fresh store connection (its main thread may be stuck in a
    collective) and names the ranks that are furthest behind.
    """

    def __init__(self, timeout_s: float | None, rank: int, world: int, report: dict):
        self.phase = "start"
        self.ordinal = 0
        self.rank = rank
        self.world = world
        self.report = report
        self.store = None
        self._t = None
        if timeout_s:
            # rank 0 fires first: it writes the one report (with every rank's
            # phase); the others only end their process, a little later
            timeout_s = timeout_s if rank == 0 else timeout_s + 15.0
            self._t = threading.Timer(timeout_s, self._fire, args=(timeout_s,))
            self._t.daemon = True
            self._t.start()

    def set_phase(self, name: str) -> None:
        self.ordinal += 1
        self.phase = name
        if self.store is not None:
            try:
                self.store.set(f"kgs/phase/{self.rank}", f"{self.ordinal}:{name}")
            except Exception:  # noqa: BLE001 - diagnostics only
                pass

    def _peer_phases(self) -> dict:
        import datetime

        import torch.distributed as dist

        out = {}
        try:
            c = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                              is_master=False, timeout=datetime.timedelta(seconds=5))
            for r in range(self.world):
                key = f"kgs/phase/{r}"
                out[r] = c.get(key).decode() if c.check([key]) else "0:init"
        except Exception as e:  # noqa: BLE001 - store gone: report what we know
            out = {"error": f"store unreachable: {e}"}
        return out

    def _fire(self, timeout_s: float) -> None:
        msg = f"rank {self.rank} watchdog: no completion after {timeout_s:.0f}s (phase: {self.phase})"
        print(f"[kgs] {msg}", file=sys.stderr, flush=True)
        if self.rank == 0:
            rep = {**self.report, "status": "error", "reason": msg, "phase": self.phase, "exit_code": 124}
            if self.world > 1:
                phases = self._peer_phases()
                rep["rank_phases"] = {str(k): v for k, v in phases.items()}
                ords = {r: int(v.split(":", 1)[0]) for r, v in phases.items() if isinstance(r, int)}
                if ords:
                    low = min(ords.values())
                    behind = sorted(r for r, o in ords.items() if o == low)
                    if len(behind) < len(ords):
                        rep["failing_rank"] = behind[0]
                        rep["ranks_behind"] = behind
            rep.setdefault("failing_rank", self.rank)
            report_once(rep)
        os._exit(124)

    def cancel(self) -> None:
        if self._t is not None:
            self._t.cancel()

    def shutdown_bound(self, timeout_s: float) -> None:
        """Switch to a bound on the shutdown alone, once the run's result is
        out: a peer that lags in the process-group teardown must not
        turn a reported result into exit 124. If the teardown runs out, the
        rank leaves with status 0 -- the result line already stands."""
        self.cancel()
        self.set_phase("shutdown")
        self._t = threading.Timer(timeout_s, self._fire_shutdown, args=(timeout_s,))
        self._t.daemon = True
        self._t.start()

    def _fire_shutdown(self, timeout_s: float) -> None:
        print(f"[kgs] rank {self.rank}: process-group shutdown not done after {timeout_s:.0f}s; leaving "
              "(the result was already reported)", file=sys.stderr, flush=True)
        os._exit(0)


def _kill_group(p: subprocess.Popen, sig) -> None:
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _terminate(procs) -> None:
    for p in procs:
        if p.poll() is None:
            _kill_group(p, signal.SIGTERM)
