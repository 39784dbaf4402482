#!/usr/bin/env python3
"""Decode-batch GEMMs on one MI355X: the four-wave kernel at tile widths 256 /
128 (and 128-row tiles for batches <= 128) with 1-8 K-slices (kgs.ops.gemm.gemm_nt_w4x) against hipBLASLt
(torch.matmul) and the 8-wave split-K kernel, on the Llama-3-8B projection
shapes at serving batches. Weights stream from HBM (a fresh weight copy per
call rotates through a pool larger than the 256 MiB Infinity Cache), as in
decode. Interleaved rounds, medians. One JSON line per (batch, shape).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="128,192,256,384,512")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from kgs.ops.gemm import gemm_nt_splitk, gemm_nt_w4x

    dev = torch.device("cuda", 0)
    res = []
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        pool = max(2, (1 << 30) // (N * K * 2) + 1)  # > 1 GiB of weights: each call reads from HBM
        Ws = [(torch.rand(N, K, device=dev) * 2 - 1).bfloat16() for _ in range(pool)]
        for M in [int(x) for x in a.batches.split(",")]:
            x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ref = (x.float() @ Ws[0].float().T)
            cands = {"hipblaslt": lambda w: torch.matmul(x, w.T, out=out)}
            for bm in ((256, 128) if M <= 128 else (256,)):
                for bn in (256, 128):
                    if N % bn:
                        continue
                    for ns in (1, 2, 4, 8):
                        if (K // ns) % 128 or K % ns:
                            continue
                        tag = f"w4_bn{bn}_s{ns}" if bm == 256 else f"w4_bm128_bn{bn}_s{ns}"
                        cands[tag] = (lambda w, bn=bn, ns=ns, bm=bm: gemm_nt_w4x(x, w, bn=bn, nslice=ns, out=out,
                                                                                 bm=bm))
            for ns in (4, 8):
                if (K // ns) % 8 == 0:
                    cands[f"pp_splitk{ns}"] = (lambda w, ns=ns: gemm_nt_splitk(x, w, ns, out=out))
            errs = {}
            for k, f in cands.items():
                f(Ws[0])
                torch.cuda.synchronize()
                errs[k] = float(((out.float() - ref).abs().max() / ref.abs().max()).item())
            times = {k: [] for k in cands}
            for _ in range(a.rounds):
                for k, f in cands.items():
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for i in range(a.iters):
                        f(Ws[i % pool])
                    e.record()
                    e.synchronize()
                    times[k].append(s.elapsed_time(e) * 1e3 / a.iters)
            med = {k: round(statistics.median(v), 2) for k, v in times.items()}
            best = min(med, key=med.get)
            r = {"shape": name, "M": M, "N": N, "K": K, "us": med, "best": best,
                 "speedup_vs_hipblaslt": round(med["hipblaslt"] / med[best], 3),
                 "max_rel_err": round(max(errs.values()), 5)}
            print(json.dumps(r), flush=True)
            res.append(r)
        del Ws
        torch.cuda.empty_cache()
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            for r in res:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
