#!/usr/bin/env python3
"""Minimal GEMM driver for rocprofv3 (kernel trace / PMC counters).

Runs ``--iters`` launches of the kgs gfx950 GEMM and, with --torch, the same
number of torch.matmul (hipBLASLt) launches on identical random operands.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops import gemm_nt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mnk", default="8192")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--torch", action="store_true")
ap.add_argument("--variant", default="auto", help="kgs.ops.gemm variant or a kgs.ops.experiments name")
a = ap.parse_args()
d = [int(x) for x in a.mnk.split("x")]
M, N, K = (d * 3)[:3] if len(d) == 1 else d
A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
if a.variant == "auto":
    run = lambda: gemm_nt(A, B, out=C)  # noqa: E731
else:
    from kgs.ops import experiments
    from kgs.ops.gemm import VARIANTS

    run = (lambda: gemm_nt(A, B, out=C, variant=a.variant)) if a.variant in VARIANTS else \
        (lambda: experiments.gemm_nt(A, B, a.variant, out=C))
for _ in range(a.iters):
    run()
if a.torch:
    for _ in range(a.iters):
        torch.matmul(A, B.T, out=C)
torch.cuda.synchronize()
print("done")
