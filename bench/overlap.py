#!/usr/bin/env python3
"""GEMM / collective overlap on ONE MI355X.

The bench step (kgs/models/gemm_workload.py) runs 4 x 8192^3 GEMMs on the
compute stream and, at N > 1, an RCCL all-reduce of a 64 MiB bucket on a side
stream. Every GEMM workgroup holds a whole CU (128 KiB LDS, 512 registers per
wave), so a collective kernel gets CUs only when the dispatcher hands it a CU
that a GEMM workgroup just released. Whether that happens while the GEMMs run
-- or only after them (serial) -- is measured here with the RCCL-shaped
stand-in kernel ``kgs.ops.comm_standin`` (a few tens of long-lived, memory-bound
workgroups: the footprint of a ring all-reduce kernel), since one GPU has no
peers for RCCL itself.

Cases (CUDA-event wall time per step, median over --iters steps):
  gemm        G GEMMs alone
  comm        the stand-in alone
  serial      GEMMs then comm on one stream (the no-overlap bound)
  side        comm first on a normal-priority side stream, then the GEMMs
  side_prio   the same on a high-priority side stream (the bench's choice)
  late_prio   GEMMs first, then comm on the high-priority side stream

hidden = (gemm + comm - case) / comm: 1 = comm fully hidden, 0 = serial.
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
    from kgs.ops.elementwise import comm_standin

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    m = args.m
    a = (torch.rand((m, m), generator=g, device=dev) * 2 - 1).bfloat16()
    b = (torch.rand((m, m), generator=g, device=dev) * 2 - 1).bfloat16()
    c = [torch.empty((m, m), device=dev, dtype=torch.bfloat16) for _ in range(2)]
    n = int(args.bucket_mb * (1 << 20)) // 4
    dst = torch.rand(n, generator=g, device=dev)
    src = torch.rand(n, generator=g, device=dev)
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    side_hi = torch.cuda.Stream(device=dev, priority=-1)

    def gemms():
        for i in range(args.gemms):
            gemm_nt(a, b, out=c[i & 1], variant=args.variant)

    def comm():
        comm_standin(dst, src, blocks=args.blocks, passes=args.passes, lds_kb=args.standin_lds_kb)

    def on(stream, fn):
        stream.wait_stream(main)
        with torch.cuda.stream(stream):
            fn()
        main.wait_stream(stream)

    def case_side(stream):
        def f():
            stream.wait_stream(main)
            with torch.cuda.stream(stream):
                comm()
            gemms()
            main.wait_stream(stream)
        return f

    def case_late(stream):
        def f():
            stream.wait_stream(main)
            gemms()
            with torch.cuda.stream(stream):
                comm()
            main.wait_stream(stream)
        return f

    cases = {
        "gemm": gemms,
        "comm": comm,
        "serial": lambda: (gemms(), comm()),
        "side": case_side(side),
        "side_prio": case_side(side_hi),
        "late_prio": case_late(side_hi),
    }
    for f in cases.values():  # warm up every path (and the clocks)
        for _ in range(3):
            f()
    torch.cuda.synchronize(dev)
    times = {k: [] for k in cases}
    for _ in range(args.iters):  # interleaved rounds
        for k, f in cases.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(main)
            f()
            e.record(main)
            e.synchronize()
            times[k].append(s.elapsed_time(e))
    med = {k: statistics.median(v) for k, v in times.items()}
    tg, tc = med["gemm"], med["comm"]
    out = {
        "config": {"gemm": f"{args.gemms} x {m}^3 bf16 (kgs gemm_nt, variant {args.variant})",
                   "comm_standin_mb": args.bucket_mb, "comm_blocks": args.blocks, "comm_passes": args.passes,
                   "comm_lds_kb": args.standin_lds_kb, "iters": args.iters},
        "ms_median": {k: round(v, 4) for k, v in med.items()},
        "hidden_fraction": {k: round((tg + tc - med[k]) / tc, 3) for k in ("serial", "side", "side_prio", "late_prio")},
        "overlap_efficiency": {k: round(med[k] / (tg + tc), 3) for k in ("serial", "side", "side_prio", "late_prio")},
    }
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--gemms", type=int, default=4)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--blocks", type=int, default=32, help="stand-in workgroups (RCCL channels)")
    ap.add_argument("--passes", type=int, default=3, help="stand-in passes (scales its duration)")
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--variant", default="auto", help="kgs GEMM variant (auto = persistent; w4_oneshot)")
    ap.add_argument("--standin-lds-kb", type=int, default=0,
                    help="LDS per stand-in workgroup (> 32: it needs a CU of its own, like a collective kernel)")
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
