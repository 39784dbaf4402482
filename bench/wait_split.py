#!/usr/bin/env python3
"""Where the persistent GEMM's extra ``SQ_WAIT_ANY`` sits: steady K-loop or tile change.

VERDICT r5 item 2: at 8192^3 the persistent kernel waits +42 % more than
hipBLASLt (profiles/r5/gemm/pmc_r7/) at equal MFMA busy, and a build that writes
no C still waits as much (profiles/r5/gemm/store_drain/). This splits the waits
by varying K at a fixed tile grid (M = N = 8192: 1024 tiles, 4 per CU): a
K-step costs the same waits at every K, a tile change / prologue / epilogue the
same at every K, so per path

    SQ_WAIT_ANY(K) = per_kstep * (K / 64) * tiles_per_cu  +  fixed

and the least-squares line over K in {1024, 2048, 4096, 8192, 16384} gives the
steady part (slope) and the tile-change + launch part (intercept).

Two modes:

  driver   (run under rocprofv3 --pmc, one pass per run): ``--iters`` launches of
           every (path, K) in a fixed order; writes the plan next to the CSVs.
  summary  ``--summary DIR [DIR ...]``: reads the counter CSVs of the passes,
           assigns dispatches to (path, K) in plan order, and fits the lines.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... -d OUT/p1 -o w -- python3 bench/wait_split.py --plan OUT/plan.json
    python3 bench/wait_split.py --summary OUT/p1 [OUT/p2] --plan OUT/plan.json --json OUT/wait_split.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KS = (1024, 2048, 4096, 8192, 16384)
PATHS = ("w4pn_0", "w4pq4x4n_0", "w4_oneshot", "hipblaslt")
# which dispatches belong to a path (kernel-name regex)
MATCH = {"w4pn_0": r"gemm_nt_w4p<", "w4pq4x4n_0": r"gemm_nt_w4p<", "w4_oneshot": r"gemm_nt_w4<",
         "hipblaslt": r"Cijk"}


def drive(a) -> int:
    import torch

    from kgs.ops import experiments, gemm_nt

    M = N = 8192
    plan = []
    for K in a.ks:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for p in a.paths:
            if p == "hipblaslt":
                f = lambda: torch.matmul(A, B.T, out=C)  # noqa: E731
            elif p == "w4_oneshot":
                f = lambda: gemm_nt(A, B, out=C, variant="w4_oneshot")  # noqa: E731
            else:
                f = lambda p=p: experiments.gemm_nt(A, B, p, out=C)  # noqa: E731
            f()  # first call outside the counted block (library kernel selection, code load)
            torch.cuda.synchronize()
            plan.append({"path": p, "K": K, "iters": a.iters, "warm": 1})
            for _ in range(a.iters):
                f()
            torch.cuda.synchronize()
        del A, B, C
    if a.plan:
        with open(a.plan, "w") as fh:
            json.dump({"M": M, "N": N, "plan": plan}, fh, indent=1)
    print("done")
    return 0


def summarise(a) -> int:
    plan = json.load(open(a.plan))
    rows = defaultdict(dict)  # (pass dir, dispatch id) -> counters
    names = {}
    for d in a.summary:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    key = (d, int(r["Dispatch_Id"]))
                    rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
                    rows[key]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    names[key] = r["Kernel_Name"]
    out = {}
    for d in a.summary:
        seq = [k for k in sorted(rows) if k[0] == d and re.search(r"gemm_nt_w4|Cijk", names[k])]
        i = 0
        for step in plan["plan"]:
            n = step["warm"] + step["iters"]
            got = seq[i:i + n][step["warm"]:]
            i += n
            want = MATCH[step["path"]]
            bad = [names[k] for k in got if not re.search(want, names[k])]
            if bad or len(got) != step["iters"]:
                raise SystemExit(f"dispatch order does not match the plan at {step}: {bad[:2]} ({len(got)})")
            cell = out.setdefault(f'{step["path"]}@{step["K"]}', {"path": step["path"], "K": step["K"]})
            for c in rows[got[0]]:
                vals = [rows[k][c] for k in got if c in rows[k]]
                cell[c] = sum(vals) / len(vals)
    fits = {}
    for p in {v["path"] for v in out.values()}:
        pts = sorted((v["K"], v) for v in out.values() if v["path"] == p)
        xs = [k / 64 for k, _ in pts]  # K-steps per tile
        fit = {"K": [k for k, _ in pts]}
        for c in ("SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "_ns"):
            ys = [v.get(c) for _, v in pts]
            if any(y is None for y in ys):
                continue
            n = len(xs)
            mx, my = sum(xs) / n, sum(ys) / n
            sxx = sum((x - mx) ** 2 for x in xs)
            slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx
            icpt = my - slope * mx
            res = max(abs(y - (icpt + slope * x)) for x, y in zip(xs, ys))
            fit[c] = {"per_kstep": round(slope, 1), "fixed": round(icpt, 1), "max_residual": round(res, 1),
                      "values": [round(y, 1) for y in ys]}
        fits[p] = fit
    res = {"shape": "8192 x 8192 x K, 1024 tiles (4 per CU)", "cells": out, "fits": fits}
    print(json.dumps(fits, indent=1))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ks", type=lambda s: [int(x) for x in s.split(",")], default=list(KS))
    ap.add_argument("--paths", type=lambda s: s.split(","), default=list(PATHS))
    ap.add_argument("--plan", default=None, help="driver: write the plan here; summary: read it")
    ap.add_argument("--summary", nargs="+", default=None, help="pass directories to summarise")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    return summarise(a) if a.summary else drive(a)


if __name__ == "__main__":
    raise SystemExit(main())
