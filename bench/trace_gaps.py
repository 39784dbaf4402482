#!/usr/bin/env python3
"""Kernel durations and inter-kernel gaps from a rocprofv3 kernel trace CSV:
per kernel name, the median duration; over consecutive dispatches of the
matching kernels, the median idle gap (start of one minus end of the one
before) -- the dispatch / ramp cost between back-to-back GEMMs.

    python bench/trace_gaps.py gpurun_out/X/btrace/..._kernel_trace.csv --match gemm_nt_w4p
"""
import argparse
import csv
import glob
import json
import statistics


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="gemm")
    ap.add_argument("--skip", type=int, default=20, help="first matching dispatches to skip (warm-up)")
    a = ap.parse_args(argv)
    path = a.trace if a.trace.endswith(".csv") else glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(path)) if a.match in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[a.skip:]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    gaps = [(int(b["Start_Timestamp"]) - int(a_["End_Timestamp"])) / 1e3 for a_, b in zip(rows, rows[1:])]
    out = {"trace": path, "dispatches": len(rows), "duration_us_median": round(statistics.median(dur), 2),
           "gap_us_median": round(statistics.median(gaps), 2), "gap_us_p90": round(sorted(gaps)[int(0.9 * len(gaps))], 2),
           "gap_share": round(sum(g for g in gaps if g < 1000) / (sum(dur) + sum(g for g in gaps if g < 1000)), 4)}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
