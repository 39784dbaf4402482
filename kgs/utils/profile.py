#!/usr/bin/env python3
"""rocprofv3 helpers: counter sets, command builder, CSV -> markdown summary.

Used by the in-pod entrypoint (``kgs.workload.entrypoint --counters``, BASELINE
config 3: "bf16 MFMA GEMM smoke with rocprof counters") and by
``bench/prof_summary.py`` for the committed ``profiles/``.

Counter sets follow the gfx950 slot limits (MI355X_MICROARCH.md "rocprofv3 PMC
slots": 8 SQ, 4 TCC, 2 GRBM per pass) and are never combined with tracing in
one run (the pool refuses --pmc together with sys/runtime tracing).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import statistics

COUNTER_SETS = {
    "pipe": ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT",
             "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE"],
    "mfma": ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"],
    "l2": ["TCC_HIT_sum", "TCC_MISS_sum", "GRBM_GUI_ACTIVE"],
}


def pmc_command(cmd: list, outdir: str, counters: list, name: str = "run") -> list:
    """``rocprofv3 --pmc ... -- <cmd>`` (the program itself after ``--``, no
    env/bash hop in between)."""
    return ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", outdir, "-o", name, "--", *cmd]


def trace_command(cmd: list, outdir: str, name: str = "run") -> list:
    return ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", outdir, "-o", name, "--", *cmd]


def short(name: str) -> str:
    n = name.split("(")[0]
    if "gemm_nt_256w4" in n:
        return "kgs gemm_nt_256w4 (round-1 4-wave experiment)"
    if "gemm_nt_w4" in n:
        return "kgs gemm_nt_w4 (4-wave, production) " + n.split("<")[-1].rstrip(">") if "<" in n else n
    if "gemm_nt_256" in n:
        return "kgs gemm_nt_256 (8-wave ping-pong) " + n.split("<")[-1].rstrip(">") if "<" in n else n
    if "Cijk" in n:
        return "hipBLASLt " + n[:60]
    return n[:70]


def summarize(d: str, flops: float = 2.0 * 8192 ** 3, simds: int = 1024) -> str:
    out = []
    tr = glob.glob(os.path.join(d, "trace", "*_kernel_trace.csv"))
    if tr:
        rows = list(csv.DictReader(open(tr[0])))
        by = collections.defaultdict(list)
        meta = {}
        for r in rows:
            k = short(r["Kernel_Name"])
            by[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
            meta[k] = (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("LDS_Block_Size"),
                       r.get("Workgroup_Size_X") or r.get("Workgroup_Size"), r.get("Grid_Size_X") or r.get("Grid_Size"))
        out.append("## Kernel trace (rocprofv3 --kernel-trace --stats)\n")
        out.append("| kernel | dispatches | median ms | min ms | TFLOP/s (median) | VGPR | AGPR | LDS B | WG | grid |")
        out.append("|---|---|---|---|---|---|---|---|---|---|")
        for k, v in sorted(by.items(), key=lambda kv: -statistics.median(kv[1])):
            med = statistics.median(v)
            is_gemm = any(s in k for s in ("gemm", "hipBLASLt"))
            tf = f"{flops / (med * 1e-3) / 1e12:.0f}" if is_gemm else "-"
            m = meta[k]
            out.append(f"| {k} | {len(v)} | {med:.4f} | {min(v):.4f} | {tf} | {m[0]} | {m[1]} | {m[2]} | {m[3]} | "
                       f"{m[4]} |")
        out.append("")
    for pdir in sorted(glob.glob(os.path.join(d, "pmc*"))):
        f = glob.glob(os.path.join(pdir, "*_counter_collection.csv"))
        if not f:
            continue
        rows = list(csv.DictReader(open(f[0])))
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in rows:
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        names = sorted({c for k in agg.values() for c in k})
        out.append(f"## Counters: {os.path.basename(pdir)} (mean per dispatch)\n")
        out.append("| kernel | " + " | ".join(names) + " | derived |")
        out.append("|---|" + "---|" * (len(names) + 1))
        for k, c in agg.items():
            if not any(s in k for s in ("gemm", "hipBLASLt", "vadd")):
                continue
            m = {n: statistics.mean(v) for n, v in c.items()}
            dv = []
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
                dv.append(f"MFMA busy/SIMD vs GPU cycles {m['SQ_VALU_MFMA_BUSY_CYCLES'] / simds / (m['GRBM_GUI_ACTIVE'] / 8):.1%}")
            if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
                dv.append(f"LDS conflict cycles {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.1%} of LDS active")
            if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
                dv.append(f"wait {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.0%} / inst-stall "
                          f"{m.get('SQ_WAIT_INST_ANY', 0) / m['SQ_WAVE_CYCLES']:.0%} / active "
                          f"{m.get('SQ_ACTIVE_INST_ANY', 0) / m['SQ_WAVE_CYCLES']:.0%}")
            if "TCC_HIT_sum" in m:
                dv.append(f"L2 hit {m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.1%}")
            out.append(f"| {k} | " + " | ".join(f"{m.get(n, 0):.3e}" for n in names) + " | " + "; ".join(dv) + " |")
        out.append("")
    return "\n".join(out)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("dir")
    ap.add_argument("--flops", type=float, default=2.0 * 8192 ** 3)
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args(argv)
    print(summarize(a.dir, a.flops, a.simds))


if __name__ == "__main__":
    main()
