#!/usr/bin/env python3
"""Host cost of one GEMM call, and what it does to a short-kernel benchmark.

For each backend (kgs ``gemm_nt``, hipBLASLt through ``torch.matmul``):

* ``host_us``: wall time per call to enqueue ``--calls`` GEMMs while the GPU
  is held busy by a spin kernel (``torch.cuda._sleep``), so the queue never
  pushes back and only the host side is measured;
* ``gpu_us_cold``: events around ``--iters`` launches issued to an idle GPU,
  the way ``bench/gemm_sweep.py`` timed until round 4 -- the first launch's
  host latency is inside the window;
* ``gpu_us_prefilled``: the same with a spin kernel queued before the start
  event, so every launch is already queued when the window opens (pure
  back-to-back GPU time).

    python bench/launch_overhead.py --shapes 4096,8192 --out launch.json
"""
from __future__ import annotations

import argparse
import json
import statistics as st
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

SPIN_CYCLES = 50_000_000  # ~25 ms at ~2 GHz: longer than any enqueue burst below


def host_us(fn, calls: int) -> float:
    torch.cuda.synchronize()
    torch.cuda._sleep(SPIN_CYCLES)
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / calls * 1e6


def gpu_us(fn, iters: int, prefill: bool) -> float:
    torch.cuda.synchronize()
    if prefill:
        torch.cuda._sleep(SPIN_CYCLES // 10)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--shapes", default="4096,8192")
    ap.add_argument("--calls", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from kgs.ops import gemm_nt

    res = []
    for sh in a.shapes.split(","):
        d = [int(x) for x in sh.split("x")]
        M, N, K = (d * 3)[:3] if len(d) == 1 else d
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fns = {"kgs": lambda: gemm_nt(A, B, out=C), "hipblaslt": lambda: torch.matmul(A, B.T, out=C)}
        for f in fns.values():
            for _ in range(3):
                f()
        r = {"shape": [M, N, K]}
        fl = 2.0 * M * N * K
        h = {name: [host_us(f, a.calls) for _ in range(3)] for name, f in fns.items()}
        cold = {name: [] for name in fns}
        pre = {name: [] for name in fns}
        for _ in range(a.rounds):  # backends interleaved, as bench/gemm_sweep.py does
            for name, f in fns.items():
                cold[name].append(gpu_us(f, a.iters, False))
                pre[name].append(gpu_us(f, a.iters, True))
        for name in fns:
            r[name] = {"host_us": round(st.median(h[name]), 2),
                       "gpu_us_cold": round(st.median(cold[name]), 2),
                       "gpu_us_prefilled": round(st.median(pre[name]), 2),
                       "tflops_cold": round(fl / (st.median(cold[name]) * 1e-6) / 1e12, 1),
                       "tflops_prefilled": round(fl / (st.median(pre[name]) * 1e-6) / 1e12, 1)}
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
