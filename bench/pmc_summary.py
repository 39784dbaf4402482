#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel (name filter), the mean over its
dispatches of every counter, plus dispatch counts. Several pass directories can
be merged (each pass is its own run, the same program and dispatch order).

    python bench/pmc_summary.py DIR [DIR ...] --match gemm_nt_w4 [--json out.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics
from collections import defaultdict


def load(dirs, match):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows = defaultdict(dict)
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if not re.search(match, r["Kernel_Name"]):
                        continue
                    key = (r["Dispatch_Id"], r["Kernel_Name"])
                    rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
                    rows[key]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    meta[r["Kernel_Name"]] = {"grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                                              "lds": int(r["LDS_Block_Size"]), "vgpr": int(r["VGPR_Count"]),
                                              "agpr": int(r["Accum_VGPR_Count"]), "sgpr": int(r["SGPR_Count"])}
            for (_, name), cs in rows.items():
                for c, v in cs.items():
                    per[name][c].append(v)
    return per, meta


def short(name: str) -> str:
    m = re.search(r"(\w+)<([^()]*)>\(", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name[:120]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default=".")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    per, meta = load(a.dirs, a.match)
    out = {}
    for name, cs in per.items():
        out[short(name)] = {"meta": meta.get(name, {}),
                            "dispatches": max(len(v) for k, v in cs.items() if k != "_ns"),
                            **{c: round(statistics.mean(v), 1) for c, v in sorted(cs.items())}}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
