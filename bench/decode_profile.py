#!/usr/bin/env python3
"""Decode kernels under rocprofv3 counters: a fixed, HBM-streaming workload per
kernel so per-dispatch counters (FETCH_SIZE, MFMA busy) can be set against the
kernel-trace durations. Run it three times, once per pass (one rocprofv3 pass per run):

  rocprofv3 --kernel-trace --stats ... -- python3 bench/decode_profile.py
  rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE ... -- python3 bench/decode_profile.py
  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE ... -- python3 bench/decode_profile.py

and summarise with ``python bench/decode_profile.py --summarize <dir>``.

Workload (Llama-3-8B decode shapes):
  * paged decode attention, batch 256, 544-token contexts, 32 q / 8 kv heads,
    16 layers' caches walked in turn (the KV streams from HBM);
  * skinny GEMM, gate|up 28672x4096 at batch 16, fused RMS+SwiGLU epilogue,
    over a ring of weight copies larger than the MALL;
  * split-K 256x256 GEMM, down 4096x14336 at batch 256, 8 slices.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run(iters: int = 8) -> None:
    import torch

    from kgs.ops import decode as D
    from kgs.ops.gemm import gemm_nt_splitk

    dev = "cuda"
    torch.manual_seed(0)
    # attention
    B, H, HKV, ctx, layers = 256, 32, 8, 544, 16
    npg = (ctx + D.PAGE - 1) // D.PAGE
    cache = D.PagedKVCache(layers, 1 + B * npg, HKV, dev)
    cache.data.normal_()
    bt = (1 + torch.arange(B * npg, device=dev, dtype=torch.int32)).reshape(B, npg)
    ctx_lens = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    q = torch.randn(B, (H + 2 * HKV) * D.HEAD_DIM, device=dev).bfloat16()
    for i in range(iters):
        D.paged_decode_attention(q, cache.layer(i % layers), bt, ctx_lens, H, HKV)
    torch.cuda.synchronize()
    del cache
    # skinny gate|up, fused RMS + SwiGLU
    n, k, m = 28672, 4096, 16
    ws = [D.PackedWeight((torch.randn(n, k, device=dev) * k ** -0.5).bfloat16(), swiglu=True) for _ in range(8)]
    x = torch.randn(m, k, device=dev).bfloat16()
    ss = x.float().pow(2).sum(-1)
    for i in range(iters):
        D.skinny_gemm(x, ws[i % len(ws)], rms=ss)
    torch.cuda.synchronize()
    del ws
    # split-K down at batch 256
    n, k, m = 4096, 14336, 256
    wd = [(torch.randn(n, k, device=dev) * k ** -0.5).bfloat16() for _ in range(8)]
    xd = torch.randn(m, k, device=dev).bfloat16()
    for i in range(iters):
        gemm_nt_splitk(xd, wd[i % len(wd)], 8)
    torch.cuda.synchronize()


def _short(name: str) -> str:
    n = name.split("(")[0]
    for key, label in (("paged_decode", "paged_decode_attention"), ("paged_reduce", "paged_reduce"),
                       ("skinny", "skinny_gemm " + n.split("<")[-1].rstrip(">") if "<" in n else "skinny"),
                       ("gemm_nt_256", "gemm_nt_256 split-K"), ("splitk_reduce", "splitk_reduce")):
        if key in n:
            return label
    return ""


def summarize(d: str) -> str:
    out = ["# Decode kernels: rocprofv3 counters against kernel-trace time", "",
           "Workload: `bench/decode_profile.py` (HBM-streaming operands; see its docstring).", ""]
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "*_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            k = _short(r["Kernel_Name"])
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = _short(r["Kernel_Name"])
            if k:
                ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # algorithmic bytes per dispatch (what the kernel must read at least)
    algo = {"paged_decode_attention": 256 * 544 * 8 * 2 * 128 * 2, "gemm_nt_256 split-K": 4096 * 14336 * 2,
            "skinny_gemm 2, 1, 16, false": 28672 * 4096 * 2}
    out.append("| kernel | dispatches | median us | algorithmic MB | algorithmic TB/s | FETCH_SIZE MB | "
               "FETCH / algorithmic | MFMA busy |")
    out.append("|---|---:|---:|---:|---:|---:|---:|---:|")
    for k in sorted(dur, key=lambda s: -statistics.median(dur[s])):
        t = statistics.median(dur[k])
        c = {n: statistics.mean(v) for n, v in ctr[k].items()}
        fetch = c.get("FETCH_SIZE")
        mb = f"{fetch / 1024:.1f}" if fetch is not None else "-"
        ab = algo.get(k)
        amb = f"{ab / 2 ** 20:.1f}" if ab else "-"
        abw = f"{ab / t / 1e12:.2f}" if ab else "-"
        ratio = f"{fetch * 1024 / ab:.2f}" if ab and fetch is not None else "-"
        mf = "-"
        if c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and c.get("GRBM_GUI_ACTIVE"):
            mf = f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (c['GRBM_GUI_ACTIVE'] / 8):.1%}"
        out.append(f"| {k} | {len(dur[k])} | {t * 1e6:.1f} | {amb} | {abw} | {mb} | {ratio} | {mf} |")
    out.append("")
    out.append("FETCH_SIZE (KB, summed over the TCC channels rocprofv3 reports) reads about half of the bytes the")
    out.append("kernels must stream, on every kernel alike, so it is quoted as a ratio only. The bandwidth figures")
    out.append("are algorithmic bytes over kernel-trace time. MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs over")
    out.append("GRBM_GUI_ACTIVE / 8 XCDs. Decode kernels are bandwidth-bound by design, so MFMA busy stays low, except")
    out.append("for the batch-256 split-K GEMM, which sits near the ridge point.")
    out.append("")
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--summarize", metavar="DIR")
    a = ap.parse_args(argv)
    if a.summarize:
        print(summarize(a.summarize))
        return 0
    run(a.iters)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
