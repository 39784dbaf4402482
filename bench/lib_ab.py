#!/usr/bin/env python3
"""Two builds of the kernel library, interleaved in ONE process (VERDICT r4
next-step 2, step 1: isolate the round-4 GEMM drop).

``--lib-b`` is another build of ``libkgs_kernels.so`` (e.g. the tree before a
change, built with ``python -m kgs.utils.build --only kernels --out DIR`` from a
``git worktree``); ``--lib-a`` defaults to this tree's. Both are loaded with
ctypes (RTLD_LOCAL: each keeps its own symbols and code objects) and called
through the same C entry point, ``kgs_gemm_bf16_nt`` (auto variant), on the same
operands, in interleaved rounds with hipBLASLt (``torch.matmul``) as the
box-speed yardstick -- same box, same clocks, same thermal state. Outputs are
compared bitwise against each other. One JSON line per shape.

  python bench/lib_ab.py --lib-b gpurun_ab/prepack/libkgs_kernels.so \\
      --shapes 4096,8192,8192x4096x14336,4096x8192x14336,16384x16384x8192
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

VP, I = ctypes.c_void_p, ctypes.c_int


def load(path: str):
    so = ctypes.CDLL(os.path.abspath(path))  # RTLD_LOCAL
    so.kgs_gemm_bf16_nt.argtypes = [VP] * 4 + [I] * 8 + [VP]
    so.kgs_gemm_bf16_nt.restype = I
    return so


def caller(so, A, B, C):
    M, K = A.shape
    N = B.shape[0]

    def f():
        s = torch.cuda.current_stream().cuda_stream
        rc = so.kgs_gemm_bf16_nt(A.data_ptr(), B.data_ptr(), C.data_ptr(), None, M, N, K, A.stride(0), B.stride(0),
                                 C.stride(0), 0, 0, s)
        if rc:
            raise RuntimeError(f"kgs_gemm_bf16_nt rc={rc}")
    return f


def time_fn(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--lib-a", default=os.path.join(ROOT, "kgs", "_native", "libkgs_kernels.so"))
    ap.add_argument("--lib-b", required=True)
    ap.add_argument("--shapes", default="4096,8192,8192x4096x14336,4096x8192x14336,16384x16384x8192")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    la, lb = load(a.lib_a), load(a.lib_b)
    res = []
    for s in a.shapes.split(","):
        dims = [int(x) for x in s.split("x")]
        M, N, K = (dims * 3)[:3] if len(dims) == 1 else dims
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        Ca, Cb, Ch = (torch.empty(M, N, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        fns = {"a": caller(la, A, B, Ca), "b": caller(lb, A, B, Cb),
               "hipblaslt": lambda: torch.matmul(A, B.T, out=Ch)}
        for f in fns.values():
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                times[k].append(time_fn(f, a.iters))
        fl = 2.0 * M * N * K
        r = {"shape": [M, N, K], "bitwise_a_eq_b": bool(torch.equal(Ca, Cb))}
        for k, ts in times.items():
            r[f"{k}_tflops_median"] = round(fl / (statistics.median(ts) * 1e-3) / 1e12, 1)
        r["a_over_b"] = round(r["a_tflops_median"] / r["b_tflops_median"], 4)
        r["a_over_hipblaslt"] = round(r["a_tflops_median"] / r["hipblaslt_tflops_median"], 4)
        r["b_over_hipblaslt"] = round(r["b_tflops_median"] / r["hipblaslt_tflops_median"], 4)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"lib_a": a.lib_a, "lib_b": a.lib_b, "rounds": a.rounds, "iters": a.iters, "shapes": res},
                      f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
