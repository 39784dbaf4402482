#!/usr/bin/env python3
"""Where a persistent-GEMM launch loses time at its edges: per-workgroup start
and per-tile end stamps from the production kernel's timing build
(gemm_w4p.h TS, s_memrealtime at 100 MHz), for launches issued back to back
as bench.py issues them.

Per launch it reports the span (first start -> last end), the head (how long
after the first workgroup the others start), the tail (CU time idle after
each workgroup's last tile until the launch's last one), the gap to the next
launch, the per-XCD finish spread and the tile-time distribution by tile
index. The timing build and production are timed against each other first, so
a reader can see whether the stamps perturb the kernel.

    python bench/gemm_tail.py --shapes 8192,8192x4096x14336 --launches 20 --out tail.json
"""
from __future__ import annotations

import argparse
import json
import statistics as st
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def parse_shape(s: str):
    p = [int(x) for x in s.split("x")]
    return (p[0], p[0], p[0]) if len(p) == 1 else tuple(p)


def analyse(st_all, grid: int) -> dict:
    """st_all: int64 [L, grid, 16] host tensor of one shape's launches."""
    tick_us = 0.01  # 100 MHz
    launches = []
    prev_end = None
    for li in range(st_all.shape[0]):
        s = st_all[li, :grid]
        start = s[:, 0].double()
        last = s[:, 14].double()
        ntl = s[:, 15].long()
        t0, t1 = start.min().item(), last.max().item()
        span = (t1 - t0) * tick_us
        head = (start - t0) * tick_us
        tail = (t1 - last) * tick_us
        xcc = (s[:, 1] >> 32).long() & 0xF
        # mean tile time per workgroup after its first tile (tiles 1 .. n-1), and per XCD
        per_tile = ((last - s[:, 2].double()) * tick_us) / (ntl - 1).clamp(min=1).double()
        per_x_fin, per_x_tile = {}, {}
        for x in sorted(set(xcc.tolist())):
            m = xcc == x
            per_x_fin[int(x)] = round((t1 - last[m].max().item()) * tick_us, 2)
            per_x_tile[int(x)] = round(per_tile[m].mean().item(), 2)
        by_idx = {}
        for b in range(grid):
            n = int(min(ntl[b].item(), 11))
            prev = start[b].item()
            for j in range(n):
                e = s[b, 2 + j].item()
                by_idx.setdefault(j, []).append((e - prev) * tick_us)
                prev = e
        exit_ = s[:, 13].double()
        rec = {
            "span_us": round(span, 2),
            # the last workgroup's exit (queue exit counter + reset) after the launch's last tile end
            "exit_after_last_tile_us": round((exit_.max().item() - t1) * tick_us, 2),
            "head_mean_us": round(head.mean().item(), 2), "head_max_us": round(head.max().item(), 2),
            "tail_mean_us": round(tail.mean().item(), 2), "tail_max_us": round(tail.max().item(), 2),
            "edge_idle_frac": round((head.mean().item() + tail.mean().item()) / span, 4),
            "tiles_per_wg": sorted(set(ntl.tolist())),
            "xcd_finish_before_last_us": per_x_fin,
            "xcd_mean_tile_us": per_x_tile,
            "tile_us_median_by_index": {j: round(st.median(v), 2) for j, v in by_idx.items()},
            "tile_us_p10_p90_by_index": {j: [round(sorted(v)[len(v) // 10], 2), round(sorted(v)[(9 * len(v)) // 10], 2)]
                                         for j, v in by_idx.items()},
        }
        if prev_end is not None:
            rec["gap_from_previous_us"] = round((t0 - prev_end) * tick_us, 2)
        prev_end = t1
        launches.append(rec)
    body = launches[1:] if len(launches) > 2 else launches
    keys = ("span_us", "exit_after_last_tile_us", "head_mean_us", "head_max_us", "tail_mean_us", "tail_max_us", "edge_idle_frac")
    summary = {k: round(st.median([r[k] for r in body]), 4) for k in keys}
    gaps = [r["gap_from_previous_us"] for r in body if "gap_from_previous_us" in r]
    if gaps:
        summary["gap_from_previous_us"] = round(st.median(gaps), 2)
    xs = sorted(body[0]["xcd_mean_tile_us"])
    summary["xcd_mean_tile_us"] = {x: round(st.median([r["xcd_mean_tile_us"][x] for r in body]), 2) for x in xs}
    summary["xcd_finish_before_last_us"] = {x: round(st.median([r["xcd_finish_before_last_us"][x] for r in body]), 2)
                                            for x in xs}
    mid = st_all[st_all.shape[0] // 2, :grid]
    raw = {"t0": int(mid[:, 0].min().item()),
           "rows": [[int(v) for v in mid[b].tolist()] for b in range(grid)]}
    return {"summary": summary, "launches": launches, "raw_middle_launch": raw}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--shapes", default="8192,8192x4096x14336")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--maps", default="prod",
                    help="comma list of tile maps (kgs.ops.experiments.STAMP_MAPS names) or 'prod'")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    from kgs.ops import experiments as ex
    from kgs.ops import gemm_nt

    dev = torch.device("cuda", 0)
    res = []
    for sh, mp in [(sh, mp) for sh in a.shapes.split(",") for mp in a.maps.split(",")]:
        M, N, K = parse_shape(sh)
        map_ = ex.production_map(M, N, K) if mp == "prod" else mp
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        A = (torch.rand((M, K), generator=g, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand((N, K), generator=g, device=dev) * 2 - 1).bfloat16()
        C = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
        C2 = torch.empty_like(C)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        grid = min((M // 256) * (N // 256), cus)
        L = a.launches
        stamps = torch.zeros((L, grid, 16), dtype=torch.int64, device=dev)
        # same bits as production
        ex.gemm_w4p_stamps(A, B, C2, stamps[0], map_)
        gemm_nt(A, B, out=C)
        torch.cuda.synchronize()
        same = bool(torch.equal(C, C2))  # the maps change only the tile order: same bits everywhere
        # timing build vs production, interleaved blocks of L launches
        ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
        t_prod, t_ts = [], []
        for _ in range(3):
            for which in ("prod", "ts"):
                e0, e1 = ev(), ev()
                e0.record()
                for i in range(L):
                    if which == "prod":
                        gemm_nt(A, B, out=C)
                    else:
                        ex.gemm_w4p_stamps(A, B, C2, stamps[i], map_)
                e1.record()
                torch.cuda.synchronize()
                (t_prod if which == "prod" else t_ts).append(e0.elapsed_time(e1) * 1e3 / L)
        stamps.zero_()
        for i in range(L):
            ex.gemm_w4p_stamps(A, B, C2, stamps[i], map_)
        torch.cuda.synchronize()
        an = analyse(stamps.cpu(), grid)
        r = {"shape": [M, N, K], "map": map_, "grid": grid, "bitwise_production": same,
             "us_per_launch_production": round(st.median(t_prod), 2),
             "us_per_launch_timing_build": round(st.median(t_ts), 2), **an}
        print(json.dumps({k: v for k, v in r.items() if k not in ("launches", "raw_middle_launch")}), flush=True)
        res.append(r)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
