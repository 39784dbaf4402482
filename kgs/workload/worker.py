"""Per-GPU worker of the gpu-rocm-test pod (one process per allocated GPU).

Runs, on every rank: the HIP vector-add smoke (BASELINE config 2), a bf16 MFMA
GEMM correctness check and TFLOPS measurement (config 3), then -- with more
than one GPU -- an RCCL all-reduce bandwidth sweep over xGMI (config 4). Rank 0
prints one ``KGS_RESULT {json}`` line with every rank's numbers.

Launched by :mod:`kgs.workload.entrypoint` through ``torch.distributed.run``.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm-size", type=int, default=8192)
    ap.add_argument("--gemm-iters", type=int, default=20)
    ap.add_argument("--vadd-elems", type=int, default=1 << 26)
    ap.add_argument("--allreduce-sizes", default="")
    ap.add_argument("--allreduce-iters", type=int, default=20)
    ap.add_argument("--skip-gemm", action="store_true")
    ap.add_argument("--skip-allreduce", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="also run the e4m3 GEMM (scaled fp8 MFMA)")
    ap.add_argument("--p2p", action="store_true",
                    help="with >1 GPU: P2P (IPC/xGMI) all-reduce latency vs RCCL, 1 KiB..8 MiB")
    return ap.parse_args(argv)


def vector_add_check(dev, n: int) -> dict:
    import torch

    from kgs.ops import vector_add

    a = torch.rand(n, device=dev)
    b = torch.rand(n, device=dev)
    c = vector_add(a, b)
    ok = bool(torch.allclose(c, a + b))
    torch.cuda.synchronize(dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 10
    s.record()
    for _ in range(iters):
        vector_add(a, b, out=c)
    e.record()
    torch.cuda.synchronize(dev)
    ms = s.elapsed_time(e) / iters
    return {"ok": ok, "elems": n, "ms": round(ms, 4), "gbs": round(3 * 4 * n / (ms * 1e-3) / 1e9, 1)}


def gemm_check(dev, size: int, iters: int) -> dict:
    import torch

    from kgs.ops import fast_path_ok, gemm_nt

    g = torch.Generator(device=dev)
    g.manual_seed(7)
    A = (torch.rand(size, size, generator=g, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand(size, size, generator=g, device=dev) * 2 - 1).bfloat16()
    C = torch.empty(size, size, device=dev, dtype=torch.bfloat16)
    gemm_nt(A, B, out=C)
    rows = min(size, 512)
    ref = A[:rows].float() @ B.float().T
    err = ((C[:rows].float() - ref).abs().max() / ref.abs().max()).item()
    for _ in range(3):
        gemm_nt(A, B, out=C)
    torch.cuda.synchronize(dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        gemm_nt(A, B, out=C)
    e.record()
    torch.cuda.synchronize(dev)
    ms = s.elapsed_time(e) / iters
    return {"size": size, "rel_err": err, "ok": err < 2e-2, "ms": round(ms, 4),
            "tflops": round(2.0 * size ** 3 / (ms * 1e-3) / 1e12, 1),
            "kernel": "gemm_nt_w4p" if fast_path_ok(A, B, C) else "gemm_nt_generic"}


def gemm_fp8_check(dev, size: int, iters: int) -> dict:
    """The same GEMM on OCP e4m3 operands (scaled fp8 MFMA), per-tensor scales."""
    import torch

    from kgs.ops import gemm_fp8_nt, quantize_fp8

    g = torch.Generator(device=dev)
    g.manual_seed(11)
    qa, sa = quantize_fp8(torch.rand(size, size, generator=g, device=dev) * 2 - 1)
    qb, sb = quantize_fp8(torch.rand(size, size, generator=g, device=dev) * 2 - 1)
    C = torch.empty(size, size, device=dev, dtype=torch.bfloat16)
    gemm_fp8_nt(qa, qb, sa, sb, out=C)
    rows = min(size, 512)
    ref = (qa[:rows].float() * sa) @ (qb.float() * sb).T
    err = ((C[:rows].float() - ref).abs().max() / ref.abs().max()).item()
    for _ in range(3):
        gemm_fp8_nt(qa, qb, sa, sb, out=C)
    torch.cuda.synchronize(dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        gemm_fp8_nt(qa, qb, sa, sb, out=C)
    e.record()
    torch.cuda.synchronize(dev)
    ms = s.elapsed_time(e) / iters
    return {"size": size, "rel_err": err, "ok": err < 2e-2, "ms": round(ms, 4),
            "tflops": round(2.0 * size ** 3 / (ms * 1e-3) / 1e12, 1), "dtype": "fp8_e4m3"}


def main(argv=None) -> int:
    a = _args(argv)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import torch

    from kgs.parallel import dist as kdist

    ctx = kdist.init_from_env()
    dev = ctx.device
    res = {"rank": ctx.rank, "host": socket.gethostname(), "device": str(dev)}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        res["gpu"] = {"name": p.name, "arch": getattr(p, "gcnArchName", ""), "cus": p.multi_processor_count,
                      "hbm_gib": round(p.total_memory / 2**30, 1)}
        t0 = time.perf_counter()
        res["vector_add"] = vector_add_check(dev, a.vadd_elems)
        if not a.skip_gemm:
            res["gemm"] = gemm_check(dev, a.gemm_size, a.gemm_iters)
            if a.fp8:
                res["gemm_fp8"] = gemm_fp8_check(dev, a.gemm_size, a.gemm_iters)
        res["compute_s"] = round(time.perf_counter() - t0, 3)
    results = kdist.all_gather_object(ctx, res)
    sweep = None
    if ctx.distributed and not a.skip_allreduce:
        from kgs.parallel.allreduce import allreduce_sweep

        sizes = [int(x) for x in a.allreduce_sizes.split(",") if x] or None
        sweep = [p.as_dict() for p in allreduce_sweep(sizes, iters=a.allreduce_iters, device=dev)]
    p2p_rows = None
    if ctx.distributed and a.p2p and dev.type == "cuda":
        from kgs.parallel.p2p_allreduce import P2PAllReduce, latency_sweep

        ar = P2PAllReduce(group=ctx.group, max_bytes=8 << 20, device=dev)
        p2p_rows = latency_sweep(ar, iters=20)
        ar.close()
    if ctx.rank == 0:
        gemm_tf = [r.get("gemm", {}).get("tflops", 0.0) for r in results]
        out = {"world_size": ctx.world_size, "ranks": results,
               "gemm_tflops_total": round(sum(gemm_tf), 1),
               "all_ok": all(r.get("vector_add", {}).get("ok", True) and r.get("gemm", {}).get("ok", True)
                             and r.get("gemm_fp8", {}).get("ok", True) for r in results)}
        if any("gemm_fp8" in r for r in results):
            out["gemm_fp8_tflops_total"] = round(sum(r.get("gemm_fp8", {}).get("tflops", 0.0) for r in results), 1)
        if p2p_rows:
            out["p2p_allreduce"] = p2p_rows
        if sweep:
            out["allreduce"] = sweep
            out["allreduce_peak_busbw_gbs"] = round(max(p["busbw_gbs"] for p in sweep), 1)
        print("KGS_RESULT " + json.dumps(out), flush=True)
    kdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
