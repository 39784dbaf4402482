#!/usr/bin/env python3
"""Persistent GEMM vs an RCCL-shaped collective on ONE MI355X (VERDICT r3
next-step 4): which first-ticket policy and grid the bench step should use.

The multi-GPU bench step (kgs/models/gemm_workload.py) runs 4 x 8192^3 GEMMs
on the compute stream and a 64 MiB RCCL all-reduce on a side stream. RCCL's
all-reduce kernel is one workgroup per channel, each sitting on a CU for the
length of the collective; a CU that holds one cannot also hold a GEMM
workgroup (the four-wave GEMM takes a whole SIMD's registers per wave and
128 KiB of LDS). One GPU has no peers, so the collective is emulated by its
CU footprint: k workgroups each holding a CU for t microseconds
(``kgs.ops.cu_hold``, 64 KiB LDS each).

  k  RCCL channels: 16 / 32 / 64 (RCCL picks tens of channels for a large
     all-reduce over the 8-GPU xGMI mesh; the sweep brackets it)
  t  duration of a 64 MiB fp32 all-reduce over 8 GPUs: each GPU
     moves 2 * 7/8 * 64 MiB = 117 MiB; at ~1 TB/s (all 7 links) 0.12 ms, at
     ~330 GB/s (typical large-message RCCL busBW) 0.36 ms, on one ring
     (153 GB/s) 0.77 ms -> 100 / 350 / 700 us

GEMM policies (experiments lib, kgs_exp_gemm_w4p_grid, + the production one-shot grid):
  static      persistent, one workgroup per CU, first ticket = rank (production)
  dynamic     persistent, one workgroup per CU, every ticket from the queue
  static_r    persistent on (CUs - k) workgroups, static first ticket
  dynamic_r   the same with dynamic first tickets
  oneshot     one workgroup per tile (no persistence)

Orders:
  before  the collective is issued on the side stream before the GEMMs (the bench step)
  after1  the side stream waits for the first GEMM, then issues the collective
          (a gradient bucket that becomes ready during backward)

Reported per case: step ms (median), the collective's hidden fraction
(gemm + t - step) / t, and step / ideal where ideal = gemm + k t / CUs
(the collective's CU-time spread over the whole chip).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def measure(args) -> dict:
    from kgs.ops import gemm_nt
    from kgs.ops.elementwise import cu_hold
    from kgs.ops.experiments import gemm_w4p_grid

    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    m = args.m
    a = (torch.rand((m, m), generator=g, device=dev) * 2 - 1).bfloat16()
    b = (torch.rand((m, m), generator=g, device=dev) * 2 - 1).bfloat16()
    c = [torch.empty((m, m), device=dev, dtype=torch.bfloat16) for _ in range(2)]
    ref = gemm_nt(a, b, variant="w4_oneshot")
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev, priority=-1 if args.side_priority == "high" else 0)
    ev1 = torch.cuda.Event()

    def gemm_fn(policy, k):
        if policy == "oneshot":
            return lambda i: gemm_nt(a, b, out=c[i & 1], variant="w4_oneshot")
        mode = 2 if policy.startswith("dynamic") else 1
        grid = cus - k if policy.endswith("_r") else 0
        return lambda i: gemm_w4p_grid(a, b, c[i & 1], mode=mode, grid=grid)

    def step(policy, k, t, order):
        run = gemm_fn(policy, k)

        def f():
            if t > 0 and order == "before":
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    cu_hold(k, t, lds_kb=64)
            for i in range(args.gemms):
                run(i)
                if i == 0 and t > 0 and order == "after1":
                    ev1.record(main)
                    side.wait_event(ev1)
                    with torch.cuda.stream(side):
                        cu_hold(k, t, lds_kb=64)
            if t > 0:
                main.wait_stream(side)
        return f

    def timed(f):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(main)
        f()
        e.record(main)
        e.synchronize()
        return s.elapsed_time(e)

    policies = args.policies.split(",")
    ks = [int(x) for x in args.channels.split(",")]
    ts = [float(x) for x in args.usec.split(",")]
    orders = args.orders.split(",")
    # correctness of every policy first (a wrong ticket policy must not be timed)
    for p in policies:
        for k in ks:
            c[0].zero_()
            gemm_fn(p, k)(0)
            torch.cuda.synchronize(dev)
            assert torch.equal(c[0], ref), f"policy {p} (k={k}) differs from the one-shot kernel"
    cases = {}
    for p in policies:
        for k in (ks if p.endswith("_r") else [0]):
            cases[(p, k, 0.0, "none")] = step(p, k, 0.0, "none")
    for k in ks:
        for t in ts:
            cases[("comm_only", k, t, "-")] = (lambda k=k, t=t: cu_hold(k, t, lds_kb=64))
            for p in policies:
                for o in orders:
                    cases[(p, k, t, o)] = step(p, k, t, o)
    for f in cases.values():
        for _ in range(2):
            f()
    torch.cuda.synchronize(dev)
    times = {key: [] for key in cases}
    for _ in range(args.iters):  # interleaved rounds
        for key, f in cases.items():
            times[key].append(timed(f))
    med = {key: statistics.median(v) for key, v in times.items()}
    g_static = med[("static", 0, 0.0, "none")]
    rows = []
    for (p, k, t, o), ms in med.items():
        r = {"policy": p, "channels": k, "usec": t, "order": o, "ms": round(ms, 4)}
        if t > 0 and p != "comm_only":
            r["hidden"] = round((g_static + t * 1e-3 - ms) / (t * 1e-3), 3)
            r["vs_ideal"] = round(ms / (g_static + k * t * 1e-3 / cus), 4)
            r["vs_static_alone"] = round(ms / g_static, 4)
        rows.append(r)
    best = {}
    for k in ks:
        for t in ts:
            for o in orders:
                cand = [(med[(p, k, t, o)], p) for p in policies]
                best[f"k{k}_t{int(t)}_{o}"] = min(cand)[1]
    return {"config": {"gemm": f"{args.gemms} x {m}^3 bf16", "cus": cus, "iters": args.iters,
                       "side_priority": args.side_priority, "standin": "kgs.ops.cu_hold, 64 KiB LDS per workgroup"},
            "gemm_alone_ms": {p: round(med[(p, 0, 0.0, "none")], 4) for p in policies if not p.endswith("_r")},
            "rows": rows, "best_policy": best}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--gemms", type=int, default=4)
    ap.add_argument("--channels", default="16,32,64")
    ap.add_argument("--usec", default="100,350,700")
    ap.add_argument("--orders", default="before,after1")
    ap.add_argument("--policies", default="static,dynamic,static_r,dynamic_r,oneshot")
    ap.add_argument("--side-priority", choices=("normal", "high"), default="normal")
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    res = measure(args)
    print(json.dumps(res), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
