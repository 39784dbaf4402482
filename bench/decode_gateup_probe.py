#!/usr/bin/env python3
"""Decode gate|up + SwiGLU at batch 128-512 (Llama-3-8B: [M, 4096] x [28672, 4096]^T):
routing candidates vs hipBLASLt, weights streamed from HBM (a ring of copies
larger than the MALL, as a 32-layer decode step sees them).

Candidates (gate|up at batch 256 was 67 us, ~58 % of
the weight-streaming floor):
  swiglu_bmXXX_bnYYY  the four-wave kernel with SwiGLU in its epilogue
  sk_bnYYY_sS         split-K S slices (fp32 partials, reduce) + silu_mul
  skf_bnYYY_sS        split-K S slices + ONE fused reduce-and-SwiGLU pass
  hipblaslt           torch.matmul + silu_mul
  p<any of the above> the same on weights packed tile-panel major
                      (kgs.ops.gemm.pack_w4x_weight, PACKB), e.g. pswiglu_bm256_bn128
A ``_tT`` suffix runs the four-wave kernel with T LDS stages (3 or 4); ``_nt``
streams the weights non-temporally (B loads only; two stages).
With ``--proj down`` (x [M, 14336] . W [4096, 14336]^T, no SwiGLU), ``qkv``
([6144, 4096]) or ``o`` ([4096, 4096]) the candidates are w4x_bmXXX_bnYYY[_sS][_tT],
pw4x_... and hipblaslt.
One JSON line per (batch, variant): median us, weight GB/s, max rel err vs
hipBLASLt + silu_mul.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="128,256,512")
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--ring-gb", type=float, default=1.5)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--variants", default=(
        "swiglu_bm256_bn128,swiglu_bm256_bn256,swiglu_bm128_bn256,swiglu_bm128_bn128,"
        "sk_bn256_s2,sk_bn256_s4,sk_bn128_s2,skf_bn256_s2,skf_bn256_s4,skf_bn128_s2,hipblaslt"))
    ap.add_argument("--proj", choices=("gateup", "down", "qkv", "o"), default="gateup",
                    help="down / qkv / o: a plain projection (no SwiGLU), Llama-3-8B shapes")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from kgs.ops.gemm import (gemm_nt_w4x, gemm_nt_w4x_splitk_swiglu, gemm_nt_w4x_swiglu, pack_w4x_weight,
                              reserve_splitk_workspace)
    from kgs.ops.transformer import silu_mul

    dev = torch.device("cuda", 0)
    down = a.proj != "gateup"  # plain projection
    N, K = {"down": (a.hidden, a.inter), "qkv": (a.hidden + 2 * 1024, a.hidden), "o": (a.hidden, a.hidden),
            "gateup": (2 * a.inter, a.hidden)}[a.proj]
    wbytes = N * K * 2
    ring = max(2, int(a.ring_gb * 1e9 // wbytes))
    ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(ring)]
    reserve_splitk_workspace(dev, 4 * 512 * N)
    packed = {}  # (bn, swiglu) -> ring of packed copies

    def ring_of(bn, sw):
        if (bn, sw) not in packed:
            packed.clear()  # one packed ring at a time (HBM)
            torch.cuda.empty_cache()
            packed[(bn, sw)] = [pack_w4x_weight(w, bn, swiglu=sw) for w in ws]
        return packed[(bn, sw)]

    def make(v, x):
        if v == "hipblaslt":
            return (lambda i: torch.matmul(x, ws[i].T)) if down else (lambda i: silu_mul(torch.matmul(x, ws[i].T)))
        pk = v.startswith("p")
        v = v[1:] if pk else v
        f = v.split("_")
        nt = "nt" in f
        f = [t for t in f if t != "nt"]
        opt = {t[0]: int(t[1:]) for t in f[1:] if t[0] in "st"}  # sS: K slices, tT: LDS stages
        s, st = opt.get("s", 1), opt.get("t", 2)
        if f[0] in ("swiglu", "w4x"):
            bm, bn = int(f[1][2:]), int(f[2][2:])
        else:
            bm, bn = 256, int(f[1][2:])
        sw = f[0] == "swiglu"
        w = (lambda i: ring_of(bn, sw)[i]) if pk else (lambda i: ws[i])
        if sw:
            return lambda i: gemm_nt_w4x_swiglu(x, w(i), bn=bn, bm=bm, stages=st, nt_weights=nt)
        if f[0] == "skf":  # split-K partials + fused reduce-and-SwiGLU
            return lambda i: gemm_nt_w4x_splitk_swiglu(x, w(i), bn=bn, nslice=s)
        if down:
            return lambda i: gemm_nt_w4x(x, w(i), bn=bn, nslice=s, bm=bm, stages=st, nt_weights=nt)
        return lambda i: silu_mul(gemm_nt_w4x(x, w(i), bn=bn, nslice=s, bm=bm, stages=st))

    res = []
    for m in (int(t) for t in a.batches.split(",")):
        x = (torch.randn(m, K, device=dev)).bfloat16()
        ref = torch.matmul(x, ws[0].T)
        ref = (ref if down else silu_mul(ref)).float()
        for v in a.variants.split(","):
            try:
                fn = make(v, x)
                got = fn(0).float()
            except Exception as e:  # a shape the variant does not take
                print(json.dumps({"batch": m, "variant": v, "error": str(e)[:200]}), flush=True)
                continue
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            for i in range(ring):
                fn(i)
            torch.cuda.synchronize()
            ts = []
            for it in range(a.iters):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn(it % ring)
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            us = statistics.median(ts)
            r = {"batch": m, "variant": v, "us": round(us, 2), "weight_TBps": round(wbytes / us / 1e6, 2),
                 "rel_err": round(err, 5)}
            print(json.dumps(r), flush=True)
            res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
