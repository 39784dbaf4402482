#!/usr/bin/env python3
"""Decode-kernel microbenchmarks on one MI355X: the skinny GEMM on the Llama-3-8B
projection shapes (vs torch.matmul = hipBLASLt on the unpacked weight) and the
paged decode attention (vs KV bytes). Prints one JSON line per measurement.

  python bench/decode_bench.py [--gemm] [--attn] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

SWEEP = False
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
SHAPES_70B = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
              "lm_head": (128256, 8192)}


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def bench_gemm(iters, ms, ring_bytes=3 << 30):
    """Each call reads a different copy of the weight (a ring of copies larger
    than the 256 MB MALL), as a real decode step streams 32 layers' weights."""
    from kgs.ops.decode import PackedWeight, choose_ksplit, skinny_gemm

    for name, (n, k) in SHAPES.items():
        copies = max(2, min(64, ring_bytes // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * k ** -0.5).to(torch.bfloat16) for _ in range(copies)]
        pws = [PackedWeight(w) for w in ws]
        for m in ms:
            x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            it = {"i": 0}

            def kgs_call():
                it["i"] = (it["i"] + 1) % copies
                skinny_gemm(x, pws[it["i"]], out=out)

            def torch_call():
                it["i"] = (it["i"] + 1) % copies
                torch.matmul(x, ws[it["i"]].T, out=out)

            t_k = _time(kgs_call, iters)
            t_t = _time(torch_call, iters)
            sweep = {}
            if SWEEP:
                from kgs.ops.decode import skinny_geometry

                nch = k // skinny_geometry(m)[1]
                for ks in [d for d in range(1, nch + 1) if nch % d == 0 and d <= 64]:
                    def ks_call(ks=ks):
                        it["i"] = (it["i"] + 1) % copies
                        skinny_gemm(x, pws[it["i"]], out=out, ksplit=ks)
                    sweep[ks] = round(_time(ks_call, iters), 2)
            ref = x.float() @ ws[0].float().T
            err = ((skinny_gemm(x, pws[0]).float() - ref).abs().max() / ref.abs().max()).item()
            byts = n * k * 2 + m * k * 2 + m * n * 2
            print(json.dumps({"op": "skinny_gemm", "shape": name, "m": m, "n": n, "k": k, "copies": copies,
                              "ksplit": choose_ksplit(m, n, k), "us": round(t_k, 2), "tbps": round(byts / t_k / 1e6, 2),
                              "torch_us": round(t_t, 2), "torch_tbps": round(byts / t_t / 1e6, 2),
                              "speedup": round(t_t / t_k, 3), "rel_err": round(err, 5), "ksplit_us": sweep}),
                  flush=True)
        del ws, pws
        torch.cuda.empty_cache()


def bench_wide(iters, ms, ring_bytes=3 << 30):
    """Large decode batches (M >= 128): the kgs 256x256 prefill GEMM (gemm_nt)
    against hipBLASLt, weights HBM-streamed as in bench_gemm."""
    from kgs.ops.gemm import gemm_nt, gemm_nt_splitk

    for name, (n, k) in SHAPES.items():
        copies = max(2, min(64, ring_bytes // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * k ** -0.5).to(torch.bfloat16) for _ in range(copies)]
        for m in ms:
            x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            it = {"i": 0}

            def kgs_call():
                it["i"] = (it["i"] + 1) % copies
                gemm_nt(x, ws[it["i"]], out=out)

            def torch_call():
                it["i"] = (it["i"] + 1) % copies
                torch.matmul(x, ws[it["i"]].T, out=out)

            t_k = _time(kgs_call, iters)
            t_t = _time(torch_call, iters)
            splits = {}
            for ns in (2, 4, 8, 16):
                if k % ns or (k // ns) % 128:
                    continue

                def sk_call(ns=ns):
                    it["i"] = (it["i"] + 1) % copies
                    gemm_nt_splitk(x, ws[it["i"]], ns, out=out)
                splits[ns] = round(_time(sk_call, iters), 2)
            ref = x.float() @ ws[0].float().T
            err = ((gemm_nt_splitk(x, ws[0], 4).float() - ref).abs().max() / ref.abs().max()).item()
            byts = n * k * 2 + m * k * 2 + m * n * 2
            print(json.dumps({"op": "gemm_nt_wide", "splitk_us": splits, "splitk_rel_err": round(err, 5), "shape": name, "m": m, "n": n, "k": k, "copies": copies,
                              "us": round(t_k, 2), "tbps": round(byts / t_k / 1e6, 2), "torch_us": round(t_t, 2),
                              "speedup": round(t_t / t_k, 3)}), flush=True)
        del ws
        torch.cuda.empty_cache()


def tune_gemm(iters, ms, ring_bytes=2 << 30, fp8=False):
    """Time every (variant, split-K) of the skinny GEMM per Llama shape and batch
    bucket with HBM-streamed weights; print the best and a TUNED table."""
    from kgs.ops.decode import PackedWeight, _mt, skinny_gemm, skinny_geometry, skinny_variants

    table = {}
    for name, (n, k) in SHAPES.items():
        copies = max(2, min(32, ring_bytes // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * k ** -0.5).to(torch.bfloat16) for _ in range(copies)]
        pws = [PackedWeight(w, fp8=fp8) for w in ws]
        for m in ms:
            x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            it = {"i": 0}

            def torch_call():
                it["i"] = (it["i"] + 1) % copies
                torch.matmul(x, ws[it["i"]].T, out=out)

            t_t = _time(torch_call, iters)
            res = {}
            for v in skinny_variants(m):
                rps, kpc, mpad = skinny_geometry(m, v)
                if n % rps or k % kpc:
                    continue
                nch, nstrip = k // kpc, n // rps
                for ks in [d for d in range(1, nch + 1) if nch % d == 0 and nstrip * d <= 2048 and
                           (d == 1 or d * mpad * n * 4 <= (64 << 20))]:
                    def call(v=v, ks=ks):
                        it["i"] = (it["i"] + 1) % copies
                        skinny_gemm(x, pws[it["i"]], out=out, ksplit=ks, variant=v)
                    res[(v, ks)] = _time(call, iters)
            (bv, bks), bt = min(res.items(), key=lambda kv: kv[1])
            table[(_mt(m), n, k)] = (bv, bks)
            print(json.dumps({"op": "skinny_tune_fp8" if fp8 else "skinny_tune", "shape": name, "m": m, "n": n, "k": k, "best_variant": bv,
                              "best_ksplit": bks, "us": round(bt, 2), "tbps": round(n * k * 2 / bt / 1e6, 2),
                              "torch_us": round(t_t, 2), "speedup": round(t_t / bt, 3),
                              "all": {f"{v}/{ks}": round(t, 1) for (v, ks), t in sorted(res.items())}}), flush=True)
        del ws, pws
        torch.cuda.empty_cache()
    print("TUNED = " + repr(table), flush=True)


def bench_attn(iters):
    from kgs.ops.decode import PagedKVCache, decode_splits, paged_decode_attention

    heads, hkv = 32, 8
    for b, ctx in ((1, 4096), (16, 1024), (64, 1024), (64, 4096), (256, 1024), (256, 2048)):
        pages_per_seq = (ctx + 31) // 32
        total = b * pages_per_seq
        cache = PagedKVCache(1, total, hkv, "cuda")
        cache.data.uniform_(-1, 1)
        bt = torch.randperm(total, device="cuda").int().reshape(b, pages_per_seq).contiguous()
        ctx_t = torch.full((b,), ctx, dtype=torch.int32, device="cuda")
        q = (torch.randn(b, heads * 128, device="cuda")).to(torch.bfloat16)
        out = torch.empty(b, heads * 128, dtype=torch.bfloat16, device="cuda")
        t = _time(lambda: paged_decode_attention(q, cache.layer(0), bt, ctx_t, heads, hkv, out=out), iters)
        byts = b * ctx * hkv * 128 * 2 * 2
        pps, ns = decode_splits(b, hkv, pages_per_seq)
        print(json.dumps({"op": "paged_decode", "batch": b, "ctx": ctx, "heads": heads, "kv_heads": hkv,
                          "nsplit": ns, "us": round(t, 2), "tbps": round(byts / t / 1e6, 2)}), flush=True)
        del cache
        torch.cuda.empty_cache()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", action="store_true")
    ap.add_argument("--attn", action="store_true")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ms", default="1,16,32,64,128,256")
    ap.add_argument("--sweep", action="store_true", help="time every valid split-K factor")
    ap.add_argument("--tune", action="store_true", help="time every tile variant x split-K; print a TUNED table")
    ap.add_argument("--fp8", action="store_true", help="--tune the weight-only fp8 (W8A16) kernels")
    ap.add_argument("--wide", action="store_true", help="kgs 256x256 GEMM vs hipBLASLt at M >= 128")
    ap.add_argument("--model", choices=("llama3-8b", "llama3-70b"), default="llama3-8b")
    a = ap.parse_args(argv)
    if a.model == "llama3-70b":
        SHAPES.clear()
        SHAPES.update(SHAPES_70B)
    global SWEEP
    SWEEP = a.sweep
    if a.tune:
        tune_gemm(a.iters, [int(v) for v in a.ms.split(",")], fp8=a.fp8)
        return 0
    if a.wide:
        bench_wide(a.iters, [int(v) for v in a.ms.split(",")])
        return 0
    both = not (a.gemm or a.attn)
    if a.gemm or both:
        bench_gemm(a.iters, [int(v) for v in a.ms.split(",")])
    if a.attn or both:
        bench_attn(a.iters)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
