#!/usr/bin/env python3
"""Run each GEMM layout a few times (for rocprofv3 counter passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops import gemm_bf16  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
for ta, tb in ((False, True), (False, False), (True, False), (True, True)):
    A = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
    B = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
    for _ in range(5):
        gemm_bf16(A, B, trans_a=ta, trans_b=tb)
    torch.cuda.synchronize()
print("done")
