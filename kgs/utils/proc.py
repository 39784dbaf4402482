"""Subprocess runner with a recorded command plan and dry-run support.

Every external tool the orchestrator drives (kind, kubectl, docker/podman) goes
through :class:`Runner`, so that ``--dry-run`` prints the exact command plan and
tests can assert it. The reference shells out directly from bash
(kind-gpu-sim.sh passim).
"""
from __future__ import annotations

import logging
import os
import shlex
import subprocess
import time
from dataclasses import dataclass, field

log = logging.getLogger("kgs")


class CommandError(RuntimeError):
    def __init__(self, argv, rc, stdout, stderr):
        self.argv, self.rc, self.stdout, self.stderr = list(argv), rc, stdout, stderr
        msg = (stderr or stdout or "").strip().splitlines()
        super().__init__(f"`{shlex.join(self.argv)}` exited {rc}" + (f": {msg[-1]}" if msg else ""))


@dataclass
class Result:
    argv: list
    rc: int
    stdout: str = ""
    stderr: str = ""
    seconds: float = 0.0

    @property
    def ok(self) -> bool:
        return self.rc == 0


@dataclass
class Runner:
    dry_run: bool = False
    env: dict = field(default_factory=dict)
    plan: list = field(default_factory=list)   # every command, in order (also in dry-run)
    echo: bool = False
    # canned stdout for read-only queries in dry-run mode: {argv-prefix-tuple: stdout}
    dry_responses: dict = field(default_factory=dict)

    def _environ(self, extra=None):
        e = dict(os.environ)
        e.update(self.env)
        if extra:
            e.update(extra)
        return e

    def run(self, argv, *, input: str | None = None, check: bool = True, env: dict | None = None,
            mutating: bool = True, timeout: float | None = None) -> Result:
        """Run ``argv``. ``mutating=False`` marks read-only queries, which still
        execute... except in dry-run mode, where they return canned output."""
        argv = [str(a) for a in argv]
        entry = {"argv": argv}
        if input is not None:
            entry["stdin"] = input
        self.plan.append(entry)
        if self.echo:
            log.info("+ %s%s", shlex.join(argv), "  <<stdin" if input is not None else "")
        if self.dry_run:
            out = ""
            for prefix, resp in self.dry_responses.items():
                if tuple(argv[: len(prefix)]) == tuple(prefix):
                    out = resp
                    break
            return Result(argv, 0, out, "")
        t0 = time.perf_counter()
        try:
            p = subprocess.run(argv, input=input, capture_output=True, text=True, env=self._environ(env),
                               timeout=timeout)
        except FileNotFoundError as e:
            if check:
                raise CommandError(argv, 127, "", str(e)) from e
            return Result(argv, 127, "", str(e))
        except subprocess.TimeoutExpired as e:
            if check:
                raise CommandError(argv, 124, e.stdout or "", f"timed out after {timeout}s") from e
            return Result(argv, 124, e.stdout or "", "timeout")
        res = Result(argv, p.returncode, p.stdout, p.stderr, time.perf_counter() - t0)
        if p.stderr and p.returncode == 0:
            log.debug("%s stderr: %s", argv[0], p.stderr.strip())
        if check and p.returncode != 0:
            raise CommandError(argv, p.returncode, p.stdout, p.stderr)
        return res

    def which(self, tool: str) -> str | None:
        from shutil import which

        path = self._environ().get("PATH")
        return which(tool, path=path)
