#!/usr/bin/env python3
"""Timing probes for the A-transposed layout (wrong results by construction):
ta=2 keeps the transposed DMA but reads with ds_read_b128, ta=3 keeps the
tr reads but stages with the NT DMA pattern."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops import _lib, gemm_nt  # noqa: E402

n = 8192
A = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
B = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
C = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
so = _lib.lib()


def run(ta):
    rc = so.kgs_gemm_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), None, n, n, n, n, n, n, ta, 0, 0,
                          _lib.stream_handle(A.device))
    assert rc == 0, rc


fns = {"nt": lambda: gemm_nt(A, B, out=C), "a_trans": lambda: run(1), "probe_trdma_b128read": lambda: run(2),
       "probe_ntdma_trread": lambda: run(3)}
for f in fns.values():
    f()
torch.cuda.synchronize()
ts = {k: [] for k in fns}
for _ in range(5):
    for k, f in fns.items():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        ts[k].append(s.elapsed_time(e) / 10)
print(json.dumps({k: round(2 * n ** 3 / (sorted(v)[2] * 1e-3) / 1e12, 1) for k, v in ts.items()}))
