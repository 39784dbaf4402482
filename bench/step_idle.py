#!/usr/bin/env python3
"""GPU idle time per serving step from a rocprofv3 kernel trace of
``python -m kgs.serve bench`` (steps delimited by the sampler's argmax, as in
``decode_step_breakdown.py``): for each of the last N steps, the step period
(argmax end to argmax end) minus the union of every kernel and copy interval
inside it. What is left is time the GPU waited for the host.

  python bench/step_idle.py gpurun_out/r5l/dtrace/d_kernel_trace.csv [more traces] [--last 100]
"""
import argparse
import csv
import statistics


def step_idle(path: str, last: int):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "argmax_rows" in r["Kernel_Name"] or "ArgMax" in r["Kernel_Name"]]
    idle, period = [], []
    for j in range(max(1, len(idx) - last), len(idx)):
        a, b = idx[j - 1], idx[j]
        start, end = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
        busy, cur = 0, start
        for s, e in sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[a + 1:b + 1]):
            s = max(s, cur)
            if e > s:
                busy, cur = busy + e - s, e
        idle.append((end - start - busy) / 1e3)
        period.append((end - start) / 1e3)
    return period, idle


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--last", type=int, default=100)
    a = ap.parse_args(argv)
    for p in a.traces:
        period, idle = step_idle(p, a.last)
        print(f"{p}: {len(period)} steps; period median {statistics.median(period):.1f} mean "
              f"{statistics.fmean(period):.1f} us; GPU idle per step median {statistics.median(idle):.1f} mean "
              f"{statistics.fmean(idle):.1f} max {max(idle):.1f} us ({100 * sum(idle) / sum(period):.2f} %)")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
