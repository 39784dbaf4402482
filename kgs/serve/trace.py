"""Fault breadcrumbs for the serving engine.

A GPU memory fault surfaces asynchronously, at the next host sync, with no
kernel name (``hipErrorIllegalAddress`` at the token read-back). Two opt-in
switches attribute it:

* ``KGS_STEP_TRACE=<file>``: one line per engine step before it is launched and
  one after its host sync, written with unbuffered ``os.write`` so the lines
  survive the abort that follows a fault. The step whose ``end`` line is
  missing is the one that faulted (prefill / decode / mixed, its batch).
* ``KGS_SYNC_DEBUG=1`` (with ``KGS_STEP_TRACE``): the model also synchronises
  after every op of the prefill and the (then eager, graphs off) decode and
  writes the op's name: the first op without a line is the faulting one.

Both cost nothing when unset. The reference has no tracing at all.
"""
from __future__ import annotations

import os
import time


class StepTrace:
    def __init__(self, path: str | None, sync_ops: bool = False):
        self.fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644) if path else None
        self.sync_ops = bool(self.fd is not None and sync_ops)
        self.t0 = time.perf_counter()

    @classmethod
    def from_env(cls) -> "StepTrace":
        return cls(os.environ.get("KGS_STEP_TRACE") or None, os.environ.get("KGS_SYNC_DEBUG", "0") == "1")

    @property
    def on(self) -> bool:
        return self.fd is not None

    def mark(self, text: str) -> None:
        if self.fd is not None:
            os.write(self.fd, f"{time.perf_counter() - self.t0:10.4f} {text}\n".encode())

    def op(self, name: str) -> None:
        """After an op: with KGS_SYNC_DEBUG, wait for it and record it."""
        if self.sync_ops:
            import torch

            torch.cuda.synchronize()
            self.mark(f"  ok {name}")


TRACE = StepTrace.from_env()
