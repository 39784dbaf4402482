"""Fused decoder-block ops on the gfx950 kernels (``native/kernels/transformer.hip``
and ``native/kernels/attention.hip``), plus the plain-PyTorch fp32 references the
tests compare them with.

* :func:`add_rmsnorm` -- ``x += d`` (bf16 residual stream, in place) then
  ``rmsnorm(x) * w``; :func:`rms_norm` without the add
* :func:`rope_qkv_` -- rotate-half RoPE on the q and k heads of a fused QKV
  projection output, in place
* :func:`silu_mul` -- SwiGLU ``silu(gate) * up`` from a fused gate|up output
* :func:`add_rmsnorm_fp8`, :func:`silu_mul_fp8`, :func:`quantize_rows_fp8` -- the
  same producers emitting e4m3 rows + per-row scales for
  :func:`kgs.ops.gemm.gemm_fp8_rows` (W8A8, per-token dynamic activation scales)
* :func:`attention_qkv` -- causal/full GQA flash attention (head_dim 128) reading
  q, k, v straight out of the fused QKV buffer and writing ``[tokens, H*128]``

Every op raises :class:`kgs.ops.NativeUnavailable` when the native library is
missing -- there is no silent PyTorch fallback.
"""
from __future__ import annotations

import math

import torch

from . import _lib


def _need(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be on a GPU")
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name} must be bf16")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must be a row-major 2-D matrix")


def add_rmsnorm(x: torch.Tensor, d: torch.Tensor | None, w: torch.Tensor, eps: float = 1e-5,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """``x += d`` (when ``d`` is given; bf16, in place) and return ``rmsnorm(x) * w``.

    cols must be a multiple of 512 (up to 8192)."""
    _need(x, "x")
    rows, cols = x.shape
    if d is not None:
        _need(d, "d")
        if d.shape != x.shape or d.stride(0) != x.stride(0):
            raise ValueError("d must match x in shape and row stride")
    if w.shape != (cols,) or w.dtype != torch.bfloat16 or not w.is_contiguous():
        raise ValueError("w must be a contiguous bf16 vector of length cols")
    y = torch.empty((rows, cols), dtype=torch.bfloat16, device=x.device) if out is None else out
    _need(y, "out")
    rc = _lib.lib().kgs_add_rmsnorm_bf16(x.data_ptr(), 0 if d is None else d.data_ptr(),
                                         0 if d is None else x.data_ptr(), w.data_ptr(), y.data_ptr(), rows, cols,
                                         x.stride(0), y.stride(0), float(eps), _lib.stream_handle(x.device))
    _lib.check(rc, "add_rmsnorm")
    return y


def splitk_add_rmsnorm(partials: torch.Tensor, x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5,
                       out: torch.Tensor | None = None) -> torch.Tensor:
    """``x += bf16(sum(partials))`` (in place) and return ``rmsnorm(x) * w``:
    the split-K reduce of a decode projection fused with the residual add and
    norm after it. ``partials``: contiguous fp32 ``[nslice, rows, cols]``
    (``kgs.ops.gemm.gemm_nt_w4x_partials``); cols a multiple of 2048 up to 8192.
    The delta is rounded to bf16 as the unfused reduce would round it."""
    _need(x, "x")
    rows, cols = x.shape
    if partials.dtype != torch.float32 or partials.dim() != 3 or tuple(partials.shape[1:]) != (rows, cols) or \
            not partials.is_contiguous():
        raise ValueError("partials must be a contiguous fp32 [nslice, rows, cols] tensor")
    if w.shape != (cols,) or w.dtype != torch.bfloat16 or not w.is_contiguous():
        raise ValueError("w must be a contiguous bf16 vector of length cols")
    y = torch.empty((rows, cols), dtype=torch.bfloat16, device=x.device) if out is None else out
    _need(y, "out")
    rc = _lib.lib().kgs_splitk_add_rmsnorm_bf16(partials.data_ptr(), partials.shape[0], x.data_ptr(), w.data_ptr(),
                                                y.data_ptr(), rows, cols, x.stride(0), y.stride(0), float(eps),
                                                _lib.stream_handle(x.device))
    _lib.check(rc, "splitk_add_rmsnorm")
    return y


def argmax_rows(x: torch.Tensor) -> torch.Tensor:
    """``x.argmax(dim=-1)`` for bf16 GPU logits ``[rows, cols]`` (cols % 8 == 0):
    int64, the first index of each row's maximum (NaN counts as the maximum)."""
    _need(x, "x")
    rows, cols = x.shape
    out = torch.empty(rows, dtype=torch.int64, device=x.device)
    rc = _lib.lib().kgs_argmax_rows_bf16(x.data_ptr(), out.data_ptr(), rows, cols, x.stride(0),
                                         _lib.stream_handle(x.device))
    _lib.check(rc, "argmax_rows")
    return out


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    return add_rmsnorm(x, None, w, eps)


def _fp8_out(rows, cols, device):
    from .gemm import FP8_DTYPE

    return (torch.empty((rows, cols), dtype=FP8_DTYPE, device=device),
            torch.empty(rows, dtype=torch.float32, device=device))


def add_rmsnorm_fp8(x: torch.Tensor, d: torch.Tensor | None, w: torch.Tensor, eps: float = 1e-5):
    """As :func:`add_rmsnorm`, but the normalised rows come back as e4m3 with a
    per-row scale: returns ``(y8, scales)``, ``y ~= y8.float() * scales[:, None]``."""
    _need(x, "x")
    rows, cols = x.shape
    if d is not None:
        _need(d, "d")
        if d.shape != x.shape or d.stride(0) != x.stride(0):
            raise ValueError("d must match x in shape and row stride")
    if w.shape != (cols,) or w.dtype != torch.bfloat16 or not w.is_contiguous():
        raise ValueError("w must be a contiguous bf16 vector of length cols")
    y8, ys = _fp8_out(rows, cols, x.device)
    rc = _lib.lib().kgs_add_rmsnorm_fp8(x.data_ptr(), 0 if d is None else d.data_ptr(),
                                        0 if d is None else x.data_ptr(), w.data_ptr(), y8.data_ptr(), ys.data_ptr(),
                                        rows, cols, x.stride(0), y8.stride(0), float(eps),
                                        _lib.stream_handle(x.device))
    _lib.check(rc, "add_rmsnorm_fp8")
    return y8, ys


def quantize_rows_fp8(x: torch.Tensor):
    """bf16 rows -> ``(e4m3 rows, per-row f32 scales)`` in one pass (cols % 512 == 0)."""
    _need(x, "x")
    rows, cols = x.shape
    y8, ys = _fp8_out(rows, cols, x.device)
    rc = _lib.lib().kgs_quant_rows_fp8(x.data_ptr(), y8.data_ptr(), ys.data_ptr(), rows, cols, x.stride(0),
                                       y8.stride(0), _lib.stream_handle(x.device))
    _lib.check(rc, "quantize_rows_fp8")
    return y8, ys


def silu_mul_fp8(gu: torch.Tensor):
    """SwiGLU into e4m3 rows with per-row scales: ``(a8, scales)``."""
    _need(gu, "gu")
    rows, w2 = gu.shape
    inter = w2 // 2
    y8, ys = _fp8_out(rows, inter, gu.device)
    rc = _lib.lib().kgs_silu_mul_fp8(gu.data_ptr(), y8.data_ptr(), ys.data_ptr(), rows, inter, gu.stride(0),
                                     y8.stride(0), _lib.stream_handle(gu.device))
    _lib.check(rc, "silu_mul_fp8")
    return y8, ys


def rope_tables(seq: int, head_dim: int, theta: float, device) -> tuple[torch.Tensor, torch.Tensor]:
    """fp32 ``cos``/``sin`` of ``pos * theta**(-2i/head_dim)``, shape [seq, head_dim/2]."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, device=device, dtype=torch.float32) / head_dim))
    ang = torch.arange(seq, device=device, dtype=torch.float32)[:, None] * inv[None, :]
    return ang.cos().contiguous(), ang.sin().contiguous()


def rope_qkv_(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, heads: int, head_dim: int, seq: int,
              positions: torch.Tensor | None = None) -> torch.Tensor:
    """Rotate (in place) the first ``heads`` heads of every token row of ``qkv``
    (q heads then k heads). Positions are ``token % seq`` unless given."""
    _need(qkv, "qkv")
    for t in (cos, sin):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.shape[-1] != head_dim // 2:
            raise ValueError("cos/sin must be contiguous fp32 [max_pos, head_dim/2]")
    pos = 0
    if positions is not None:
        if positions.dtype != torch.int32 or not positions.is_contiguous():
            raise ValueError("positions must be contiguous int32")
        pos = positions.data_ptr()
    rc = _lib.lib().kgs_rope_qkv_bf16(qkv.data_ptr(), cos.data_ptr(), sin.data_ptr(), pos, qkv.shape[0], heads,
                                      head_dim, qkv.stride(0), seq, _lib.stream_handle(qkv.device))
    _lib.check(rc, "rope_qkv")
    return qkv


def silu_mul(gu: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``silu(gu[:, :I]) * gu[:, I:]`` for a fused gate|up output of width 2I."""
    _need(gu, "gu")
    rows, w2 = gu.shape
    inter = w2 // 2
    out = torch.empty((rows, inter), dtype=torch.bfloat16, device=gu.device) if out is None else out
    _need(out, "out")
    rc = _lib.lib().kgs_silu_mul_bf16(gu.data_ptr(), out.data_ptr(), rows, inter, gu.stride(0), out.stride(0),
                                      _lib.stream_handle(gu.device))
    _lib.check(rc, "silu_mul")
    return out


def attention_qkv(qkv: torch.Tensor, batch: int, seq: int, heads: int, kv_heads: int, head_dim: int = 128,
                  causal: bool = True, scale: float | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Flash attention over a fused QKV buffer ``[batch*seq, (heads + 2*kv_heads) * head_dim]``
    (q heads, then k heads, then v heads per token). Returns ``[batch*seq, heads*head_dim]``."""
    _need(qkv, "qkv")
    if qkv.shape[0] != batch * seq or qkv.shape[1] < (heads + 2 * kv_heads) * head_dim:
        raise ValueError("qkv shape does not match batch/seq/heads")
    out = torch.empty((batch * seq, heads * head_dim), dtype=torch.bfloat16, device=qkv.device) \
        if out is None else out
    _need(out, "out")
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    ld = qkv.stride(0)
    esz = qkv.element_size()
    base = qkv.data_ptr()
    rc = _lib.lib().kgs_attn_fwd_bf16(base, base + heads * head_dim * esz, base + (heads + kv_heads) * head_dim * esz,
                                      out.data_ptr(), batch, seq, heads, kv_heads, head_dim, ld, ld, ld, out.stride(0),
                                      float(scale), 1 if causal else 0, _lib.stream_handle(qkv.device))
    _lib.check(rc, "attention")
    return out


def attention_chunk(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int, kv_heads: int,
                    head_dim: int = 128, scale: float | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Causal flash attention of one sequence's prefill CHUNK over its whole
    context: ``q`` rows ``[S, >= heads*128]`` are the last S positions (S % 128
    == 0), ``k``/``v`` ``[Sk, >= kv_heads*128]`` every key up to and including
    them (Sk - S % 64 == 0) -- row i sees keys 0 .. Sk - S + i. Any row strides."""
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _need(t, n)
    S, Sk = q.shape[0], k.shape[0]
    if v.shape[0] != Sk:
        raise ValueError("k and v differ in length")
    out = torch.empty((S, heads * head_dim), dtype=torch.bfloat16, device=q.device) if out is None else out
    _need(out, "out")
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    rc = _lib.lib().kgs_attn_fwd_bf16_ex(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), 1, S, Sk, heads,
                                         kv_heads, head_dim, q.stride(0), k.stride(0), v.stride(0), out.stride(0),
                                         float(scale), 1, _lib.stream_handle(q.device))
    _lib.check(rc, "attention_chunk")
    return out


def ref_attention_chunk(q, k, v, heads, kv_heads, head_dim=128, scale=None):
    """fp32 reference of :func:`attention_chunk` (bottom-right causal)."""
    S, Sk = q.shape[0], k.shape[0]
    qf = q[:, :heads * head_dim].float().reshape(S, heads, head_dim).transpose(0, 1)
    kf = k[:, :kv_heads * head_dim].float().reshape(Sk, kv_heads, head_dim).transpose(0, 1)
    vf = v[:, :kv_heads * head_dim].float().reshape(Sk, kv_heads, head_dim).transpose(0, 1)
    rep = heads // kv_heads
    kf, vf = kf.repeat_interleave(rep, 0), vf.repeat_interleave(rep, 0)
    mask = torch.arange(Sk, device=q.device)[None, :] <= (Sk - S + torch.arange(S, device=q.device))[:, None]
    o = torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, attn_mask=mask, scale=scale)
    return o.transpose(0, 1).reshape(S, heads * head_dim)


# ----------------------------------------------------------------------------
# fp32 PyTorch references (tests, the "torch" model backend)

def ref_add_rmsnorm(x, d, w, eps=1e-5):
    """Returns (new residual bf16, normalised bf16) with the kernel's rounding points."""
    xs = x if d is None else (x.float() + d.float()).to(torch.bfloat16)
    xf = xs.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return xs, y.to(torch.bfloat16)


def ref_rope_qkv(qkv, cos, sin, heads, head_dim, seq):
    t = qkv.shape[0]
    x = qkv[:, :heads * head_dim].float().reshape(t, heads, head_dim)
    pos = torch.arange(t, device=qkv.device) % seq
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    x1, x2 = x[..., :head_dim // 2], x[..., head_dim // 2:]
    rot = torch.cat((x1 * c - x2 * s, x2 * c + x1 * s), dim=-1)
    out = qkv.clone()
    out[:, :heads * head_dim] = rot.reshape(t, heads * head_dim).to(qkv.dtype)
    return out


def ref_silu_mul(gu):
    i = gu.shape[1] // 2
    g, u = gu[:, :i].float(), gu[:, i:].float()
    return (g * torch.sigmoid(g) * u).to(torch.bfloat16)


def ref_attention_qkv(qkv, batch, seq, heads, kv_heads, head_dim=128, causal=True, scale=None):
    t = batch * seq
    q = qkv[:, :heads * head_dim].float().reshape(batch, seq, heads, head_dim).transpose(1, 2)
    k = qkv[:, heads * head_dim:(heads + kv_heads) * head_dim].float().reshape(batch, seq, kv_heads, head_dim)
    v = qkv[:, (heads + kv_heads) * head_dim:(heads + 2 * kv_heads) * head_dim].float().reshape(
        batch, seq, kv_heads, head_dim)
    rep = heads // kv_heads
    k = k.transpose(1, 2).repeat_interleave(rep, dim=1)
    v = v.transpose(1, 2).repeat_interleave(rep, dim=1)
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=scale)
    return o.transpose(1, 2).reshape(t, heads * head_dim)
