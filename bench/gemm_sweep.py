#!/usr/bin/env python3
"""GEMM sweep on one MI355X: kgs HIP kernel vs torch.matmul (hipBLASLt).

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24), random
U[-1,1) operands (rule 25). Prints one JSON line per shape and writes
gpurun_out/gemm_sweep.json.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops import gemm_nt  # noqa: E402


_rand = None


def _gemm(v):
    """Production variants through kgs.ops; measured alternatives (and, with a
    wrong result, the timing probes) through the opt-in kgs.ops.experiments."""
    from kgs.ops import experiments
    from kgs.ops.gemm import VARIANTS

    if v in VARIANTS:
        return lambda A, B, out: gemm_nt(A, B, out=out, variant=v)
    if v.startswith("w4x_"):  # w4x_bmX_bnY[_sS][_tT]: four-wave kernel, X x Y tiles, S K-slices, T stages
        from kgs.ops.gemm import gemm_nt_w4x

        f = v.split("_")
        bm, bn = int(f[1][2:]), int(f[2][2:])
        opt = {t[0]: int(t[1:]) for t in f[3:]}  # sS: K slices, tT: LDS stages
        s, st = opt.get("s", 1), opt.get("t", 2)
        return lambda A, B, out: gemm_nt_w4x(A, B, bn=bn, nslice=s, out=out, bm=bm, stages=st)
    return lambda A, B, out: experiments.gemm_nt(A, B, v, out=out, allow_wrong=True)


def _gemm_fp8(v):
    from kgs.ops import experiments, gemm_fp8_nt
    from kgs.ops.gemm import FP8_VARIANTS

    if v in FP8_VARIANTS:
        return lambda qa, qb, sa, sb, out: gemm_fp8_nt(qa, qb, sa, sb, out=out, variant=v)
    return lambda qa, qb, sa, sb, out: experiments.gemm_fp8_nt(qa, qb, sa, sb, v, out=out)


def time_fn(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096,8192")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/gemm_sweep.json")
    ap.add_argument("--variants", default="auto", help="comma list of kgs variants: auto,fast,w4,generic")
    ap.add_argument("--dtype", choices=("bf16", "fp8"), default="bf16",
                    help="fp8: kgs gemm_fp8_nt (e4m3, scaled MFMA) vs torch._scaled_mm (hipBLASLt fp8)")
    ap.add_argument("--data", choices=("uniform", "normal"), default="uniform",
                    help="operand distribution: U[-1,1) or N(0,1) (activation/weight-like)")
    a = ap.parse_args()
    global _rand
    _rand = (lambda *sh: torch.rand(*sh, device="cuda") * 2 - 1) if a.data == "uniform" else \
        (lambda *sh: torch.randn(*sh, device="cuda"))
    if a.dtype == "fp8":
        return sweep_fp8(a)
    res = []
    for s in a.shapes.split(","):
        dims = [int(x) for x in s.split("x")]
        M, N, K = (dims * 3)[:3] if len(dims) == 1 else dims
        A = _rand(M, K).bfloat16()
        B = _rand(N, K).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        C2 = torch.empty_like(C)
        fns = {f"kgs_{v}": (lambda v=v: _gemm(v)(A, B, out=C)) for v in a.variants.split(",")}
        fns["hipblaslt"] = lambda: torch.matmul(A, B.T, out=C2)
        for f in fns.values():
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(a.rounds):  # interleaved rounds in one process
            for k, f in fns.items():
                times[k].append(time_fn(f, a.iters))
        errs = {}
        for v in a.variants.split(","):
            _gemm(v)(A, B, out=C)
            errs[v] = ((C.float() - C2.float()).abs().max() / C2.float().abs().max()).item()
        fl = 2.0 * M * N * K
        r = {"shape": [M, N, K]}
        for k, ts in times.items():
            r[f"{k}_tflops_median"] = round(fl / (sorted(ts)[len(ts) // 2] * 1e-3) / 1e12, 1)
            r[f"{k}_tflops_best"] = round(fl / (min(ts) * 1e-3) / 1e12, 1)
        r["rel_err_vs_hipblaslt"] = errs
        print(json.dumps(r), flush=True)
        res.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


def sweep_fp8(a):
    from kgs.ops import gemm_fp8_nt, quantize_fp8

    res = []
    for s in a.shapes.split(","):
        dims = [int(x) for x in s.split("x")]
        M, N, K = (dims * 3)[:3] if len(dims) == 1 else dims
        qa, sa = quantize_fp8(_rand(M, K))
        qb, sb = quantize_fp8(_rand(N, K))
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        C2 = torch.empty_like(C)
        ta = torch.tensor(sa, device="cuda")
        tb = torch.tensor(sb, device="cuda")
        fns = {f"kgs_fp8_{v}": (lambda v=v: _gemm_fp8(v)(qa, qb, sa, sb, out=C))
               for v in a.variants.split(",")}
        try:
            torch._scaled_mm(qa, qb.T, scale_a=ta, scale_b=tb, out_dtype=torch.bfloat16)
            fns["hipblaslt_fp8"] = lambda: torch._scaled_mm(qa, qb.T, scale_a=ta, scale_b=tb,
                                                           out_dtype=torch.bfloat16, out=C2)
        except Exception as e:  # pragma: no cover - depends on the torch build
            print(f"torch._scaled_mm unavailable: {e}", file=sys.stderr)
        for f in fns.values():
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                times[k].append(time_fn(f, a.iters))
        ref = (qa.float() * sa) @ (qb.float() * sb).T
        errs = {}
        for v in a.variants.split(","):
            _gemm_fp8(v)(qa, qb, sa, sb, out=C)
            errs[v] = ((C.float() - ref).abs().max() / ref.abs().max()).item()
        if "hipblaslt_fp8" in fns:
            errs["hipblaslt_fp8"] = ((C2.float() - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * M * N * K
        r = {"shape": [M, N, K], "dtype": "fp8_e4m3"}
        for k, ts in times.items():
            r[f"{k}_tflops_median"] = round(fl / (sorted(ts)[len(ts) // 2] * 1e-3) / 1e12, 1)
            r[f"{k}_tflops_best"] = round(fl / (min(ts) * 1e-3) / 1e12, 1)
        r["rel_err_vs_fp32_dequant"] = errs
        print(json.dumps(r), flush=True)
        res.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
