#!/usr/bin/env python3
"""Why is 8192x4096x14336 slower per K-step than 8192^3? (round 3 probe)

Measures kgs (production four-wave kernel, plus GROUP_M / order variants from
the experiments library) and hipBLASLt on M x N x K with the operands' leading
dimension optionally padded (``lda = ldb = LD``: A and B are views into wider
buffers), so the effect of the row stride can be separated from the effect of
K. Reports TFLOP/s and microseconds per 256x256x64 K-step per CU:
``t_kernel / (tiles / 256 * K / 64)``.

  python bench/gemm_stride_probe.py --cases 8192x4096x14336,8192x4096x14336@16384,8192x4096x16384
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops import gemm_nt  # noqa: E402


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
    ap.add_argument("--cases", default="8192x4096x14336,8192x4096x14336@16384,8192x4096x16384,8192x8192x8192")
    ap.add_argument("--variants", default="fast", help="kgs variants (production) and experiment names")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from kgs.ops import experiments
    from kgs.ops.gemm import VARIANTS

    res = []
    for case in a.cases.split(","):
        shape, _, ld = case.partition("@")
        M, N, K = (int(x) for x in shape.split("x"))
        LD = int(ld) if ld else K
        Abuf = (torch.rand(M, LD, device="cuda") * 2 - 1).bfloat16()
        Bbuf = (torch.rand(N, LD, device="cuda") * 2 - 1).bfloat16()
        A, B = Abuf[:, :K], Bbuf[:, :K]
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        C2 = torch.empty_like(C)
        fns = {}
        for v in a.variants.split(","):
            if v in VARIANTS:
                fns[f"kgs_{v}"] = (lambda v=v: gemm_nt(A, B, out=C, variant=v))
            else:
                fns[f"kgs_{v}"] = (lambda v=v: experiments.gemm_nt(A, B, v, out=C, allow_wrong=True))
        fns["hipblaslt"] = lambda: torch.matmul(A, B.T, out=C2)
        for f in fns.values():
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                times[k].append(time_fn(f, a.iters))
        fl = 2.0 * M * N * K
        ksteps_per_cu = (M // 256) * (N // 256) / 256 * (K // 64)
        r = {"case": case, "M": M, "N": N, "K": K, "ld": LD}
        for k, ts in times.items():
            t = sorted(ts)[len(ts) // 2]
            r[k] = {"tflops": round(fl / (t * 1e-3) / 1e12, 1), "ms": round(t, 4),
                    "us_per_kstep_per_cu": round(t * 1e3 / ksteps_per_cu, 4)}
        for v in a.variants.split(","):
            fns[f"kgs_{v}"]()
            fns["hipblaslt"]()
            torch.cuda.synchronize()
            r[f"kgs_{v}"]["rel_err"] = ((C.float() - C2.float()).abs().max() / C2.float().abs().max()).item()
        print(json.dumps(r), flush=True)
        res.append(r)
        del Abuf, Bbuf, A, B, C, C2
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
