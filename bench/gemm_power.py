#!/usr/bin/env python3
"""Sustained GEMM under DVFS: TFLOP/s, board power and GFX clock over time.

The kernel traces of round 3 show back-to-back 8192-class GEMMs slowing by
~40 % within a few milliseconds, for kgs and hipBLASLt alike
(profiles/r3/l2/*dispatches.csv). The headline bench (80 GEMMs after 20 warm-up
GEMMs) runs in that throttled state, where what counts is work per joule.

This runs each backend back-to-back for ``--seconds`` after a ``--cool``
pause, with amd-smi (Python ``amdsmi``) sampled every ``--period`` seconds on a
side thread: socket power, GFX clock and hotspot temperature. One JSON line
per (round, backend): TFLOP/s over the window, mean power and clock, TFLOP/s
per 100 W, and the per-GEMM time trace quantiles.

  python bench/gemm_power.py --mnk 8192 --seconds 2 --rounds 2
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


class Sampler:
    def __init__(self, period: float):
        import amdsmi

        self.amdsmi = amdsmi
        amdsmi.amdsmi_init()
        self.h = amdsmi.amdsmi_get_processor_handles()[0]
        self.period = period
        self.samples = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _one(self):
        a = self.amdsmi
        s = {"t": time.perf_counter()}
        try:
            p = a.amdsmi_get_power_info(self.h)
            s["power_w"] = float(p.get("current_socket_power") or p.get("socket_power") or p.get("average_socket_power") or 0)
        except Exception:  # noqa: BLE001 - metric not exposed
            pass
        try:
            c = a.amdsmi_get_clock_info(self.h, a.AmdSmiClkType.GFX)
            s["gfx_mhz"] = float(c.get("clk") or c.get("cur_clk") or 0)
        except Exception:  # noqa: BLE001
            pass
        try:
            s["temp_c"] = float(a.amdsmi_get_temp_metric(self.h, a.AmdSmiTemperatureType.HOTSPOT,
                                                         a.AmdSmiTemperatureMetric.CURRENT))
        except Exception:  # noqa: BLE001
            pass
        return s

    def _run(self):
        while not self._stop.is_set():
            self.samples.append(self._one())
            self._stop.wait(self.period)

    def window(self, t0, t1):
        ss = [s for s in self.samples if t0 <= s["t"] <= t1]
        out = {}
        for k in ("power_w", "gfx_mhz", "temp_c"):
            v = [s[k] for s in ss if s.get(k)]
            if v:
                out[k] = round(statistics.mean(v), 1)
        out["samples"] = len(ss)
        return out

    def start(self):
        self._t.start()

    def stop(self):
        self._stop.set()
        self._t.join()
        try:
            self.amdsmi.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mnk", default="8192")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--cool", type=float, default=2.0)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--period", type=float, default=0.005)
    ap.add_argument("--backends", default="kgs,hipblaslt",
                    help="kgs, hipblaslt and/or kgs.ops.experiments variant names")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from kgs.ops import gemm_nt

    d = [int(x) for x in a.mnk.split("x")]
    M, N, K = (d * 3)[:3] if len(d) == 1 else d
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fns = {"kgs": lambda: gemm_nt(A, B, out=C), "hipblaslt": lambda: torch.matmul(A, B.T, out=C)}
    for name in a.backends.split(","):  # any other name: a kgs.ops.experiments variant
        if name not in fns:
            from kgs.ops import experiments

            fns[name] = (lambda v: lambda: experiments.gemm_nt(A, B, v, out=C))(name)
    fl = 2.0 * M * N * K
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    # GEMMs per window from a short timing
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        fns["kgs"]()
    e.record()
    e.synchronize()
    n = max(10, int(a.seconds / (s.elapsed_time(e) / 5e3)))
    sm = Sampler(a.period)
    sm.start()
    res = []
    try:
        for rnd in range(a.rounds):
            for name in a.backends.split(","):
                time.sleep(a.cool)
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                evs[0].record()
                for i in range(n):
                    fns[name]()
                    evs[i + 1].record()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                per = [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]
                total_ms = sum(per)
                r = {"round": rnd, "backend": name, "mnk": [M, N, K], "gemms": n,
                     "tflops": round(fl * n / (total_ms * 1e-3) / 1e12, 1),
                     "tflops_first10": round(fl * 10 / (sum(per[:10]) * 1e-3) / 1e12, 1),
                     "tflops_last_half": round(fl * (n - n // 2) / (sum(per[n // 2:]) * 1e-3) / 1e12, 1),
                     "us_p10_p50_p90": [round(1e3 * q, 1) for q in statistics.quantiles(per, n=10)[::4]],
                     **sm.window(t0, t1)}
                if r.get("power_w"):
                    r["tflops_per_100w"] = round(100 * r["tflops"] / r["power_w"], 2)
                print(json.dumps(r), flush=True)
                res.append(r)
    finally:
        sm.stop()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
