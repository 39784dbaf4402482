"""Flash-attention forward and fused block-op timings on one MI355X.

    python bench/attention_bench.py [--batch 4 --seq 2048 --heads 32 --kv-heads 8]

Prints one JSON line per measurement: the kgs kernel (``kgs.ops.attention_qkv``,
reading q/k/v straight from the fused QKV buffer) against PyTorch-ROCm's
``scaled_dot_product_attention`` on pre-transposed [B, H, S, D] tensors (its best
case: the layout change is not timed), and the fused RMSNorm / RoPE / SwiGLU
kernels against their PyTorch expressions. Random (gaussian) data.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters=20, warmup=3):
    import torch

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(argv=None) -> int:
    import torch

    from kgs.ops import transformer as T

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma list: attn,ops")
    ap.add_argument("--w4", action="store_true",
                    help="also time the one-wave-per-SIMD named-register kernel (kgs.ops.experiments, seq % 256 == 0)")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved timing rounds (medians reported)")
    a = ap.parse_args(argv)
    only = set(a.only.split(",")) if a.only else {"attn", "ops"}
    dev = "cuda"
    b, s, nh, nkv, hd = a.batch, a.seq, a.heads, a.kv_heads, 128
    t = b * s
    torch.manual_seed(0)
    if "attn" in only:
        qkv = torch.randn(t, (nh + 2 * nkv) * hd, device=dev).to(torch.bfloat16)
        out = torch.empty(t, nh * hd, device=dev, dtype=torch.bfloat16)
        q = qkv[:, :nh * hd].reshape(b, s, nh, hd).transpose(1, 2).contiguous()
        k = qkv[:, nh * hd:(nh + nkv) * hd].reshape(b, s, nkv, hd).transpose(1, 2).contiguous()
        v = qkv[:, (nh + nkv) * hd:].reshape(b, s, nkv, hd).transpose(1, 2).contiguous()
        for causal in (True, False):
            import statistics

            flops = 4.0 * b * nh * s * s * hd * (0.5 if causal else 1.0)
            fns = {"kgs": lambda: T.attention_qkv(qkv, b, s, nh, nkv, causal=causal, out=out),
                   "sdpa": lambda: torch.nn.functional.scaled_dot_product_attention(
                       q, k, v, is_causal=causal, enable_gqa=True)}
            out4 = torch.empty_like(out)
            if a.w4:
                from kgs.ops import experiments

                fns["kgs_w4"] = lambda: experiments.attention_qkv_w4(qkv, b, s, nh, nkv, causal=causal, out=out4)
            times = {n: [] for n in fns}
            for _ in range(a.rounds):
                for n, f in fns.items():
                    times[n].append(_time(f, a.iters))
            ms, ms_t = statistics.median(times["kgs"]), statistics.median(times["sdpa"])
            ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal, enable_gqa=True)
            ref = ref.transpose(1, 2).reshape(t, nh * hd).float()
            err = (out.float() - ref).abs().max().item()
            rec = {"op": "attention_fwd", "causal": causal, "batch": b, "seq": s, "heads": nh,
                   "kv_heads": nkv, "kgs_ms": round(ms, 4), "kgs_tflops": round(flops / ms / 1e9, 1),
                   "sdpa_ms": round(ms_t, 4), "sdpa_tflops": round(flops / ms_t / 1e9, 1),
                   "speedup": round(ms_t / ms, 2), "max_abs_err_vs_sdpa": round(err, 5)}
            if a.w4:
                for n in ("kgs_w4",):
                    ms4 = statistics.median(times[n])
                    rec.update({f"{n}_ms": round(ms4, 4), f"{n}_tflops": round(flops / ms4 / 1e9, 1)})
                rec.update(kgs_w4_max_abs_err_vs_sdpa=round((out4.float() - ref).abs().max().item(), 5))
            print(json.dumps(rec), flush=True)
        del qkv, q, k, v, out
    if "ops" in only:
        h, inter = a.hidden, a.inter
        x = torch.randn(t, h, device=dev).to(torch.bfloat16)
        d = torch.randn(t, h, device=dev).to(torch.bfloat16)
        w = torch.ones(h, device=dev, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        ms = _time(lambda: T.add_rmsnorm(x, d, w, out=y), a.iters)

        def torch_addnorm():
            xs = x + d
            xf = xs.float()
            return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()).to(torch.bfloat16)

        ms_t = _time(torch_addnorm, a.iters)
        gb = 4 * t * h * 2 / 1e9
        print(json.dumps({"op": "add_rmsnorm", "rows": t, "cols": h, "kgs_ms": round(ms, 4),
                          "kgs_GBps": round(gb / ms * 1e3, 1), "torch_ms": round(ms_t, 4),
                          "speedup": round(ms_t / ms, 2)}), flush=True)
        qkv = torch.randn(t, (nh + 2 * nkv) * hd, device=dev).to(torch.bfloat16)
        cos, sin = T.rope_tables(s, hd, 500000.0, dev)
        ms = _time(lambda: T.rope_qkv_(qkv, cos, sin, nh + nkv, hd, s), a.iters)
        ms_t = _time(lambda: T.ref_rope_qkv(qkv, cos, sin, nh + nkv, hd, s), a.iters)
        gb = 2 * t * (nh + nkv) * hd * 2 / 1e9
        print(json.dumps({"op": "rope_qkv", "tokens": t, "heads": nh + nkv, "kgs_ms": round(ms, 4),
                          "kgs_GBps": round(gb / ms * 1e3, 1), "torch_ms": round(ms_t, 4),
                          "speedup": round(ms_t / ms, 2)}), flush=True)
        del qkv
        gu = torch.randn(t, 2 * inter, device=dev).to(torch.bfloat16)
        o = torch.empty(t, inter, device=dev, dtype=torch.bfloat16)
        ms = _time(lambda: T.silu_mul(gu, out=o), a.iters)
        ms_t = _time(lambda: torch.nn.functional.silu(gu[:, :inter]) * gu[:, inter:], a.iters)
        gb = 3 * t * inter * 2 / 1e9
        print(json.dumps({"op": "silu_mul", "rows": t, "inter": inter, "kgs_ms": round(ms, 4),
                          "kgs_GBps": round(gb / ms * 1e3, 1), "torch_ms": round(ms_t, 4),
                          "speedup": round(ms_t / ms, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
