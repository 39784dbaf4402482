#!/usr/bin/env python3
"""All four operand layouts of the bf16 GEMM (kgs.ops.gemm_bf16) against
torch.matmul (hipBLASLt handles every layout natively) and against
transpose-copy + NT, interleaved in one process on random data."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops import gemm_bf16, gemm_nt, transpose  # noqa: E402


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
    ap.add_argument("--out", default="gpurun_out/gemm_layouts.json")
    a = ap.parse_args()
    res = []
    for s in a.shapes.split(","):
        dims = [int(x) for x in s.split("x")]
        M, N, K = (dims * 3)[:3] if len(dims) == 1 else dims
        for ta, tb in ((False, True), (False, False), (True, False), (True, True)):
            A = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16() if ta else \
                (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16() if tb else \
                (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            C2 = torch.empty_like(C)
            opA = A.t() if ta else A
            opB = B.t() if tb else B
            fns = {
                "kgs": lambda: gemm_bf16(A, B, trans_a=ta, trans_b=tb, out=C),
                "kgs_transpose_then_nt": lambda: gemm_nt(transpose(A) if ta else A, B if tb else transpose(B), out=C),
                "hipblaslt": lambda: torch.matmul(opA, opB, out=C2),
            }
            for f in fns.values():
                f()
            torch.cuda.synchronize()
            ts = {k: [] for k in fns}
            for _ in range(a.rounds):
                for k, f in fns.items():
                    ts[k].append(time_fn(f, a.iters))
            gemm_bf16(A, B, trans_a=ta, trans_b=tb, out=C)
            torch.matmul(opA, opB, out=C2)
            err = ((C.float() - C2.float()).abs().max() / C2.float().abs().max()).item()
            fl = 2.0 * M * N * K
            name = ("T" if ta else "N") + ("N" if tb else "T")  # BLAS naming of op(A), op(B) for C = op(A) op(B)
            r = {"shape": [M, N, K], "layout": f"A{'[K][M]' if ta else '[M][K]'} B{'[N][K]' if tb else '[K][N]'}",
                 "blas": name, "rel_err_vs_hipblaslt": err}
            for k, v in ts.items():
                r[f"{k}_tflops"] = round(fl / (sorted(v)[len(v) // 2] * 1e-3) / 1e12, 1)
            print(json.dumps(r), flush=True)
            res.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
