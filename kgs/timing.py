"""Per-phase wall-clock timer for the create -> GPU-pod-Running metric.

The reference has no timing at all; its only time bounds are the
60 s ``kubectl wait`` gates (kind-gpu-sim.sh:279, rocm-ci.yaml:35). Every
orchestration phase runs inside ``with timer.phase(name):`` and the totals are
written as one JSON document (``--timings-json``).
"""
from __future__ import annotations

import json
import time
from contextlib import contextmanager
from dataclasses import dataclass, field


@dataclass
class PhaseTimer:
    phases: list = field(default_factory=list)
    t0: float = field(default_factory=time.perf_counter)
    meta: dict = field(default_factory=dict)

    @contextmanager
    def phase(self, name: str, **info):
        start = time.perf_counter()
        rec = {"phase": name, "start_s": round(start - self.t0, 4), **info}
        try:
            yield rec
            rec["ok"] = True
        except BaseException:
            rec["ok"] = False
            raise
        finally:
            rec["seconds"] = round(time.perf_counter() - start, 4)
            self.phases.append(rec)

    def total(self) -> float:
        return round(time.perf_counter() - self.t0, 4)

    def to_dict(self) -> dict:
        return {"total_s": self.total(), "phases": self.phases, **self.meta}

    def write(self, path: str | None) -> None:
        if not path:
            return
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=1)
            f.write("\n")

    def summary(self) -> str:
        w = max([len(p["phase"]) for p in self.phases] + [5])
        lines = [f"{p['phase']:<{w}}  {p['seconds']:8.3f}s{'' if p.get('ok', True) else '  FAILED'}"
                 for p in self.phases]
        lines.append(f"{'total':<{w}}  {self.total():8.3f}s")
        return "\n".join(lines)
