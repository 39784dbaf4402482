#!/usr/bin/env python3
"""Read a rocprofv3 kernel trace of bench/overlap.py and report, per comm
stand-in dispatch, how much of its lifetime ran concurrently with a GEMM
dispatch (interval intersection on the GPU timestamps).

usage: python bench/overlap_trace.py <rocprofv3 -d dir> [--out file.json]
"""
import argparse
import csv
import glob
import json
import os


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(rows, key=lambda x: x[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.dir)
    gemm = [(s, e) for n, s, e in rows if "gemm_nt" in n]
    comm = [(s, e) for n, s, e in rows if "comm_standin" in n]
    res = []
    for s, e in comm:
        ov = sum(max(0, min(e, ge) - max(s, gs)) for gs, ge in gemm)
        res.append({"comm_us": round((e - s) / 1e3, 1), "concurrent_with_gemm_us": round(ov / 1e3, 1),
                    "concurrent_fraction": round(ov / max(1, e - s), 3)})
    summary = {"gemm_dispatches": len(gemm), "comm_dispatches": len(comm),
               "comm_with_any_gemm_overlap": sum(1 for r in res if r["concurrent_with_gemm_us"] > 0),
               "median_concurrent_fraction": sorted(r["concurrent_fraction"] for r in res)[len(res) // 2] if res else None,
               "per_comm": res}
    print(json.dumps({k: v for k, v in summary.items() if k != "per_comm"}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
