#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace + PMC passes) as markdown.

  python bench/prof_summary.py gpurun_out/round > profiles/gemm_8192.md

Reads <dir>/trace/*_kernel_trace.csv and every <dir>/pmc*/ *_counter_collection.csv;
groups dispatches by kernel name; reports median duration, TFLOP/s for the
GEMM kernels (8192^3 unless --flops), and per-kernel counter means with the
derived ratios used in the write-ups (MFMA busy per SIMD / GPU cycles, LDS bank
conflict share, L2 hit rate, effective clock).
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(name: str) -> str:
    n = name.split("(")[0]
    if "gemm_nt_256w4" in n:
        return "kgs gemm_nt_256w4 (4-wave)"
    if "gemm_nt_256" in n:
        return "kgs gemm_nt_256 (8-wave ping-pong) " + n.split("<")[-1].rstrip(">") if "<" in n else n
    if "Cijk" in n:
        return "hipBLASLt " + n[:60]
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--flops", type=float, default=2.0 * 8192 ** 3)
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args()
    out = []
    tr = glob.glob(os.path.join(a.dir, "trace", "*_kernel_trace.csv"))
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
            tf = a.flops / (med * 1e-3) / 1e12 if ("gemm" in k or "Cijk" in k or "hipBLASLt" in k) else None
            m = meta[k]
            out.append(f"| {k} | {len(v)} | {med:.4f} | {min(v):.4f} | {tf:.0f} |" if tf else
                       f"| {k} | {len(v)} | {med:.4f} | {min(v):.4f} | - |")
            out[-1] += f" {m[0]} | {m[1]} | {m[2]} | {m[3]} | {m[4]} |"
        out.append("")
    for pdir in sorted(glob.glob(os.path.join(a.dir, "pmc*"))):
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
            if not any(s in k for s in ("gemm", "hipBLASLt")):
                continue
            m = {n: statistics.mean(v) for n, v in c.items()}
            d = []
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
                d.append(f"MFMA busy/SIMD vs GPU cycles {m['SQ_VALU_MFMA_BUSY_CYCLES'] / a.simds / (m['GRBM_GUI_ACTIVE'] / 8):.1%}")
            if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
                d.append(f"LDS conflict cycles {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.1%} of LDS active")
            if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
                d.append(f"wait {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.0%} / inst-stall "
                         f"{m.get('SQ_WAIT_INST_ANY', 0) / m['SQ_WAVE_CYCLES']:.0%} / active "
                         f"{m.get('SQ_ACTIVE_INST_ANY', 0) / m['SQ_WAVE_CYCLES']:.0%}")
            if "TCC_HIT_sum" in m:
                d.append(f"L2 hit {m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.1%}")
            out.append(f"| {k} | " + " | ".join(f"{m.get(n, 0):.3e}" for n in names) + " | " + "; ".join(d) + " |")
        out.append("")
    print("\n".join(out))


if __name__ == "__main__":
    main()
