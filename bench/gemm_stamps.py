#!/usr/bin/env python3
"""Where does a phase's time go? Runs the production GEMM schedule built with
s_memtime stamps (native/experiments/gemm_experiments.hip, S bit 16) at 8192^3 and reports, per
wave group, the mean cycles of each section of a phase:

  read   reads + LDS-DMA issue + vmcnt wait      bar1   first barrier + lgkmcnt
  mfma   16 MFMAs issued                         bar2   second barrier
(diagnostic build: the stamps themselves cost a few % of wave cycles)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops import _lib, experiments, gemm_nt  # noqa: E402

so = experiments.lib()
SN = so.kgs_gemm_stamp_n()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
A = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
B = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
C = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
st = torch.zeros(4 * SN, dtype=torch.int64, device="cuda")
for _ in range(20):  # warm clocks
    gemm_nt(A, B, out=C)
rc = so.kgs_gemm_bf16_nt_stamps(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, st.data_ptr(),
                               _lib.stream_handle(A.device))
assert rc == 0, rc
torch.cuda.synchronize()
assert torch.equal(C, gemm_nt(A, B)), "stamped build must compute the same product"
v = st.cpu().view(4, 4, 8, 8, 5)  # block, iteration, phase, wave, point
res = {}
for grp, waves in (("waves0-3", range(4)), ("waves4-7", range(4, 8))):
    secs = {"read": [], "bar1": [], "mfma": [], "bar2": [], "phase": []}
    for b in range(4):
        for it in range(4):
            for qp in range(8):
                for w in waves:
                    p = v[b, it, qp, w].tolist()
                    secs["read"].append(p[1] - p[0])
                    secs["bar1"].append(p[2] - p[1])
                    secs["mfma"].append(p[3] - p[2])
                    secs["bar2"].append(p[4] - p[3])
                    secs["phase"].append(p[4] - p[0])
    res[grp] = {k: round(statistics.mean(x), 1) for k, x in secs.items()}
    res[grp]["median_phase"] = statistics.median(secs["phase"])
# absolute timeline of one SIMD's two waves (0 and 4) over the first 8 phases of block 0
base = v[0, 0, 0, 0, 0].item()
timeline = {f"w{w}": [[int(x - base) for x in v[0, 0, qp, w].tolist()] for qp in range(8)] for w in (0, 4)}
print(json.dumps({"shape": [n, n, n], "cycles_per_section": res, "timeline_P0_to_P4": timeline,
                  "ideal_mfma_block": 16 * 16, "note": "s_memtime ticks = shader cycles"}, indent=1))
