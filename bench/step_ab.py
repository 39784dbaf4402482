#!/usr/bin/env python3
"""The bench step (4 x 8192^3 bf16 GEMMs, outputs alternating between two
buffers, kgs/models/gemm_workload.py) under each GEMM path, interleaved in ONE
process (cdna_hip_programming.md rule 24): blocks of --steps steps per path,
--rounds rounds, median and min ms per step and TFLOP/s.

Paths: kgs production ("fast": persistent four-wave grid), kgs "w4_oneshot"
(one workgroup per tile, same K-step), and torch.matmul (hipBLASLt). Use
--seconds to make each block a sustained run (the clock the chip holds under
minutes of load, not the first tens of ms).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--mnk", default="8192")
    ap.add_argument("--gemms", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20, help="steps per timed block")
    ap.add_argument("--seconds", type=float, default=0.0, help="> 0: each block runs this long instead")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--paths", default="fast,w4_oneshot,hipblaslt")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from kgs.ops import gemm_nt

    dims = [int(x) for x in a.mnk.split("x")]
    M, N, K = (dims * 3)[:3] if len(dims) == 1 else dims
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    A = (torch.rand((M, K), generator=g, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand((N, K), generator=g, device=dev) * 2 - 1).bfloat16()
    C = [torch.empty((M, N), device=dev, dtype=torch.bfloat16) for _ in range(2)]
    ref = A.float()[:256] @ B.float().T

    side = torch.cuda.Stream(device=dev)
    main = torch.cuda.current_stream(dev)

    def two_streams(v):
        """The step's independent GEMMs alternated over two streams (odd ones
        on a side stream that joins at the end of the step), so one GEMM's
        tail and the next one's ramp overlap instead of queueing behind the
        stream's kernel barrier. Experiment only: bench.py keeps one stream."""
        def f(i):
            if i == 0:
                side.wait_stream(main)  # before GEMM 0 is queued: GEMM 1 may start on CUs GEMM 0 frees
            if i & 1:
                with torch.cuda.stream(side):
                    gemm_nt(A, B, out=C[i & 1], variant=v)
            else:
                gemm_nt(A, B, out=C[i & 1], variant=v)
            if i == a.gemms - 1:
                main.wait_stream(side)
        return f

    def path(p):
        if p == "hipblaslt":
            return lambda i: torch.matmul(A, B.T, out=C[i & 1])
        if p.endswith("_2s"):
            return two_streams(p[:-3])
        from kgs.ops.gemm import VARIANTS

        if p not in VARIANTS:  # a measured alternative from the experiments library
            from kgs.ops import experiments

            return lambda i: experiments.gemm_nt(A, B, p, out=C[i & 1])
        return lambda i: gemm_nt(A, B, out=C[i & 1], variant=p)

    paths = {p: path(p) for p in a.paths.split(",")}
    from kgs.ops.experiments import NO_OUTPUT

    for p, f in paths.items():  # numerics before timing
        f(0)
        torch.cuda.synchronize()
        if p in NO_OUTPUT:  # a measurement build that does not write C
            continue
        err = ((C[0][:256].float() - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, (p, err)

    def block(f):
        n = a.steps
        if a.seconds > 0:  # calibrate to the requested duration
            n = max(a.steps, int(a.seconds / max(1e-4, calib[f]) ))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            for i in range(a.gemms):
                f(i)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / n

    calib = {}
    for p, f in paths.items():
        for _ in range(3):
            f(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            for i in range(a.gemms):
                f(i)
        torch.cuda.synchronize()
        calib[f] = (time.perf_counter() - t0) / a.steps
    times = {p: [] for p in paths}
    for r in range(a.rounds):
        for p, f in paths.items():
            times[p].append(block(f))
        print(json.dumps({"round": r, **{p: round(v[-1], 4) for p, v in times.items()}}), flush=True)
    fl = 2.0 * M * N * K * a.gemms
    res = {"shape": [M, N, K], "gemms_per_step": a.gemms, "steps_per_block": a.steps, "seconds_per_block": a.seconds,
           "rounds": a.rounds,
           "ms_per_step_median": {p: round(statistics.median(v), 4) for p, v in times.items()},
           "ms_per_step_min": {p: round(min(v), 4) for p, v in times.items()},
           "tflops_median": {p: round(fl / (statistics.median(v) * 1e-3) / 1e12, 1) for p, v in times.items()}}
    print(json.dumps(res), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
