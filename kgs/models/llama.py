"""Llama-3-architecture decoder (random init) whose every projection runs on the
hand-written gfx950 GEMMs -- the measurable in-pod stand-in for BASELINE.json
config 5 (``vllm-rocm-pod.yaml``: Llama-3-8B bf16 TP=1 on one MI355X). vLLM
itself ships in its own image (docs/vllm.md); this model shows the same
architecture's prefill on the kgs kernels, with no network and no checkpoint.

* projections: fused QKV [q + 2 kv heads], O, fused gate|up, down, lm-head on
  :func:`kgs.ops.gemm_nt` (bf16) or :class:`kgs.ops.Fp8Linear` (W8A8 e4m3:
  per-tensor weight scales, per-token dynamic activation scales produced by
  the fused norm / SwiGLU / row-quantise kernels, no host sync);
* attention: :func:`kgs.ops.attention_qkv` -- the hand-written flash-attention
  forward (causal, GQA) reading q/k/v in place from the QKV output;
* residual add + RMSNorm, rotate-half RoPE and SwiGLU's ``silu(g) * u`` as one
  fused kernel each (``native/kernels/transformer.hip``).

``backend="torch"`` runs the same weights and the same math through PyTorch-ROCm
(``torch.matmul`` = hipBLASLt, ``scaled_dot_product_attention``, elementwise
ops), so the backends can be compared numerically and for speed.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch


@dataclass
class LlamaConfig:
    hidden: int = 4096
    intermediate: int = 14336
    heads: int = 32
    kv_heads: int = 8
    layers: int = 32
    vocab: int = 128256
    rope_theta: float = 500000.0
    eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    @classmethod
    def llama3_8b(cls, layers: int = 32) -> "LlamaConfig":
        return cls(layers=layers)

    @classmethod
    def llama3_70b(cls, layers: int = 80) -> "LlamaConfig":
        """141 GB of bf16 weights: fits one 288 GB MI355X with room for the KV cache."""
        return cls(hidden=8192, intermediate=28672, heads=64, kv_heads=8, layers=layers)

    @classmethod
    def named(cls, name: str, layers: int | None = None) -> "LlamaConfig":
        f = {"llama3-8b": cls.llama3_8b, "llama3-70b": cls.llama3_70b}[name]
        return f() if layers is None else f(layers=layers)

    def params(self) -> int:
        h, i, kv = self.hidden, self.intermediate, self.kv_heads * self.head_dim
        per_layer = h * (h + 2 * kv) + h * h + 2 * h * i + i * h
        return self.layers * per_layer + 2 * self.vocab * h


def _rms_norm(x, w, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


def _rope_torch(q, k, cos, sin):
    # q, k: [B, H, S, D]; rotate-half (neox) pairs (i, i + D/2)
    def rot(x):
        xf = x.float()
        x1, x2 = xf[..., : xf.shape[-1] // 2], xf[..., xf.shape[-1] // 2:]
        return torch.cat((x1 * cos - x2 * sin, x2 * cos + x1 * sin), dim=-1).to(x.dtype)

    return rot(q), rot(k)


class _Proj:
    """One projection on the selected backend (weights [out, in], no bias)."""

    def __init__(self, w: torch.Tensor, backend: str):
        self.backend = backend
        if backend == "fp8":
            from kgs.ops import Fp8Linear

            self.f8 = Fp8Linear(w)
            self.w = None
        else:
            self.w = w

    def __call__(self, x2d: torch.Tensor) -> torch.Tensor:
        if self.backend == "kgs":
            from kgs.ops import gemm_nt

            return gemm_nt(x2d, self.w)
        if self.backend == "fp8":
            return self.f8(x2d)
        return x2d @ self.w.T


class LlamaModel:
    """Prefill-only forward (no KV cache: the whole prompt in one pass)."""

    def __init__(self, cfg: LlamaConfig, device="cuda", backend: str = "kgs", seed: int = 0,
                 dtype=torch.bfloat16):
        self.cfg, self.backend = cfg, backend
        g = torch.Generator(device=device).manual_seed(seed)

        def rnd(*shape, scale):
            return (torch.randn(*shape, device=device, generator=g) * scale).to(dtype)

        h, i, kvd = cfg.hidden, cfg.intermediate, cfg.kv_heads * cfg.head_dim
        self.embed = rnd(cfg.vocab, h, scale=0.02)
        self.layers = []
        for _ in range(cfg.layers):
            self.layers.append({
                "ln1": torch.ones(h, device=device, dtype=dtype),
                "qkv": _Proj(rnd(h + 2 * kvd, h, scale=h ** -0.5), backend),
                "o": _Proj(rnd(h, h, scale=h ** -0.5), backend),
                "ln2": torch.ones(h, device=device, dtype=dtype),
                "gate_up": _Proj(rnd(2 * i, h, scale=h ** -0.5), backend),
                "down": _Proj(rnd(h, i, scale=i ** -0.5), backend),
            })
        self.norm = torch.ones(h, device=device, dtype=dtype)
        self.lm_head = _Proj(rnd(cfg.vocab, h, scale=h ** -0.5), backend)

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        if self.backend == "torch":
            return self._forward_torch(tokens)
        from kgs.ops.gemm import gemm_swiglu
        from kgs.ops.transformer import add_rmsnorm, attention_qkv, rope_qkv_, rope_tables

        cfg = self.cfg
        b, s = tokens.shape
        h, hd, nh, nkv = cfg.hidden, cfg.head_dim, cfg.heads, cfg.kv_heads
        cos, sin = self._tables(s, lambda: rope_tables(s, hd, cfg.rope_theta, tokens.device))
        x = self.embed[tokens].reshape(b * s, h)
        if self.backend == "fp8":
            return self._forward_fp8(x, b, s, cos, sin)
        y = add_rmsnorm(x, None, self.layers[0]["ln1"], cfg.eps)
        for i, L in enumerate(self.layers):
            qkv = L["qkv"](y)
            rope_qkv_(qkv, cos, sin, nh + nkv, hd, s)
            a = attention_qkv(qkv, b, s, nh, nkv, head_dim=hd, causal=True)
            y = self._add_norm(x, a, L["o"], L["ln2"])  # x += o-proj
            act = gemm_swiglu(y, L["gate_up"].w)  # SwiGLU in the GEMM epilogue
            nxt = self.layers[i + 1]["ln1"] if i + 1 < len(self.layers) else self.norm
            y = self._add_norm(x, act, L["down"], nxt)  # x += down-proj
        return self.lm_head(y).reshape(b, s, cfg.vocab)

    def _add_norm(self, x, a, proj, w):
        """x += proj(a) and return rmsnorm(x) * w; on aligned operands the add
        runs in the GEMM's store (kgs.ops.gemm.gemm_nt_add_, bitwise the same)."""
        from kgs.ops.gemm import addc_ok, gemm_nt_add_
        from kgs.ops.transformer import add_rmsnorm

        if addc_ok(a, proj.w, x):
            gemm_nt_add_(a, proj.w, x)
            return add_rmsnorm(x, None, w, self.cfg.eps)
        return add_rmsnorm(x, proj(a), w, self.cfg.eps)

    def _forward_fp8(self, x, b, s, cos, sin):
        """W8A8: every producer (norm, SwiGLU, attention-output quantiser) emits
        e4m3 rows with per-token scales; the GEMMs dequantise per row in their
        epilogue (kgs_gemm_fp8_nt_rows). Attention and the residual stay bf16."""
        from kgs.ops.transformer import (add_rmsnorm_fp8, attention_qkv, quantize_rows_fp8, rope_qkv_,
                                         silu_mul_fp8)

        cfg = self.cfg
        hd, nh, nkv = cfg.head_dim, cfg.heads, cfg.kv_heads
        y8, ys = add_rmsnorm_fp8(x, None, self.layers[0]["ln1"], cfg.eps)
        for i, L in enumerate(self.layers):
            qkv = L["qkv"].f8.forward_q(y8, ys)
            rope_qkv_(qkv, cos, sin, nh + nkv, hd, s)
            a8, as_ = quantize_rows_fp8(attention_qkv(qkv, b, s, nh, nkv, head_dim=hd, causal=True))
            y8, ys = add_rmsnorm_fp8(x, L["o"].f8.forward_q(a8, as_), L["ln2"], cfg.eps)
            m8, ms = silu_mul_fp8(L["gate_up"].f8.forward_q(y8, ys))
            nxt = self.layers[i + 1]["ln1"] if i + 1 < len(self.layers) else self.norm
            y8, ys = add_rmsnorm_fp8(x, L["down"].f8.forward_q(m8, ms), nxt, cfg.eps)
        return self.lm_head.f8.forward_q(y8, ys).reshape(b, s, cfg.vocab)

    def _tables(self, s, make):
        if getattr(self, "_rope_key", None) != s:
            self._rope_key, self._rope = s, make()
        return self._rope

    def _forward_torch(self, tokens: torch.Tensor) -> torch.Tensor:
        cfg = self.cfg
        b, s = tokens.shape
        h, hd, nh, nkv = cfg.hidden, cfg.head_dim, cfg.heads, cfg.kv_heads
        dev = tokens.device

        def make():
            inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, device=dev, dtype=torch.float32) / hd))
            ang = torch.arange(s, device=dev, dtype=torch.float32)[:, None] * inv[None, :]
            return ang.cos(), ang.sin()

        cos, sin = self._tables(s, make)
        x = self.embed[tokens].reshape(b * s, h)
        for L in self.layers:
            y = _rms_norm(x, L["ln1"], cfg.eps)
            qkv = L["qkv"](y)
            q = qkv[:, :h].reshape(b, s, nh, hd).transpose(1, 2)
            k = qkv[:, h:h + nkv * hd].reshape(b, s, nkv, hd).transpose(1, 2)
            v = qkv[:, h + nkv * hd:].reshape(b, s, nkv, hd).transpose(1, 2)
            q, k = _rope_torch(q, k, cos, sin)
            a = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
            x = x + L["o"](a.transpose(1, 2).reshape(b * s, h).contiguous())
            y = _rms_norm(x, L["ln2"], cfg.eps)
            gu = L["gate_up"](y)
            act = torch.nn.functional.silu(gu[:, :cfg.intermediate]) * gu[:, cfg.intermediate:]
            x = x + L["down"](act.contiguous())
        x = _rms_norm(x, self.norm, cfg.eps)
        return self.lm_head(x).reshape(b, s, cfg.vocab)

    def gemm_flops(self, tokens: int) -> float:
        """Projection FLOPs of one prefill (2 per MAC), attention excluded."""
        cfg = self.cfg
        h, i, kvd = cfg.hidden, cfg.intermediate, cfg.kv_heads * cfg.head_dim
        per_layer = h * (h + 2 * kvd) + h * h + 2 * h * i + i * h
        return 2.0 * tokens * (cfg.layers * per_layer + cfg.vocab * h)


def prefill_bench(cfg: LlamaConfig, batch: int, seq: int, backend: str = "kgs", iters: int = 3,
                  warmup: int = 1, device="cuda") -> dict:
    model = LlamaModel(cfg, device=device, backend=backend)
    g = torch.Generator(device=device).manual_seed(1)
    tokens = torch.randint(0, cfg.vocab, (batch, seq), device=device, generator=g)
    for _ in range(warmup):
        model.forward(tokens)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        logits = model.forward(tokens)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    n = batch * seq
    return {"backend": backend, "layers": cfg.layers, "batch": batch, "seq": seq, "ms": round(dt * 1e3, 2),
            "prefill_tokens_per_s": round(n / dt, 1),
            "gemm_tflops": round(model.gemm_flops(n) / dt / 1e12, 1),
            "logits_finite": bool(torch.isfinite(logits.float()).all().item()),
            "params_b": round(cfg.params() / 1e9, 2)}


def main(argv=None) -> int:  # pragma: no cover - GPU
    import argparse
    import json

    ap = argparse.ArgumentParser(description="Llama-3-8B-architecture prefill on the kgs GEMMs")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--backends", default="kgs,torch,fp8")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args(argv)
    cfg = LlamaConfig.llama3_8b(layers=a.layers)
    for be in a.backends.split(","):
        print(json.dumps(prefill_bench(cfg, a.batch, a.seq, backend=be, iters=a.iters)), flush=True)
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":  # pragma: no cover
    raise SystemExit(main())
