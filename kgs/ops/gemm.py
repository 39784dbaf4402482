"""bf16 MFMA GEMM ops backed by ``native/kernels/gemm_bf16.hip``.

``gemm_nt(a, b)`` computes ``a @ b.T`` for ``a: [M, K]``, ``b: [N, K]`` (both
K-contiguous bf16 on a gfx950 device), with optional fused bias + activation in
the kernel epilogue. :func:`gemm_bf16` covers the other layouts: operands stored
K-major are read with ``ds_read_b64_tr_b16``, so no transpose copy is made.
``gemm_fp8_nt`` is the same pipeline on OCP e4m3 operands with the scaled fp8
MFMA and a per-tensor dequant scale. ``matmul`` and ``Linear`` are built on
these; the backward pass uses the transposed-read layouts, so every FLOP of the
in-pod workload runs on the hand-written MFMA kernel.
"""
from __future__ import annotations

import os

import torch

from . import _lib

EPI = {None: 0, "none": 0, "bias": 1, "gelu": 2, "relu": 3, "silu": 4}
# Production kernels only; the measured alternatives and timing probes are in
# kgs.ops.experiments (a separate, opt-in library).
# "fast" = the four-wave kernel (gemm_w4.h), the aligned hot path, launched as the
# persistent grid (gemm_w4p.h) when K >= 384; "w4_oneshot" = its one-shot grid
# (one workgroup per tile, for A/B and tests); "pingpong" =
# the 8-wave kernel it replaced there (still behind bounded / fp8 / K-major).
VARIANTS = {"auto": 0, "fast": 3, "w4": 3, "w4_oneshot": 4, "pingpong": 1, "generic": 2, "bounded": 16}


def _check_operand(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name} must be bfloat16, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must be on a GPU")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must be a 2-D row-major (stride(1)==1) matrix")


def gemm_nt(
    a: torch.Tensor,
    b: torch.Tensor,
    bias: torch.Tensor | None = None,
    act: str | None = None,
    out: torch.Tensor | None = None,
    variant: str = "auto",
) -> torch.Tensor:
    """``act(a @ b.T + bias)`` in bf16 with f32 accumulation.

    act: None | "bias" (bias only) | "gelu" | "relu" | "silu"; a non-None act or
    bias implies the bias epilogue (a zero bias is allocated if act is given
    without one).
    """
    _check_operand(a, "a")
    _check_operand(b, "b")
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise ValueError(f"inner dims differ: a {tuple(a.shape)} b {tuple(b.shape)}")
    if a.device != b.device:
        raise ValueError("a and b on different devices")
    epi_name = act if act is not None else ("bias" if bias is not None else None)
    if epi_name not in EPI:
        raise ValueError(f"unknown activation {act!r}")
    epi = EPI[epi_name]
    if epi and bias is None:
        bias = torch.zeros(N, dtype=torch.bfloat16, device=a.device)
    if bias is not None:
        if bias.dtype != torch.bfloat16 or bias.numel() != N or not bias.is_contiguous():
            raise ValueError("bias must be a contiguous bf16 vector of length N")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out")
        if tuple(out.shape) != (M, N):
            raise ValueError(f"out has shape {tuple(out.shape)}, expected {(M, N)}")
    rc = _lib.lib().kgs_gemm_bf16_nt(
        a.data_ptr(),
        b.data_ptr(),
        out.data_ptr(),
        bias.data_ptr() if bias is not None else None,
        M,
        N,
        K,
        a.stride(0),
        b.stride(0),
        out.stride(0),
        epi,
        VARIANTS[variant],
        _lib.stream_handle(a.device),
    )
    _lib.check(rc, f"gemm_nt[{M}x{N}x{K}]")
    return out


_SPLITK_WS: dict = {}


def reserve_splitk_workspace(device: torch.device, floats: int) -> torch.Tensor:
    """The per-GPU fp32 partial-tile buffer, grown to at least ``floats``. Call
    it up front (before hipGraph capture: a buffer first allocated inside a
    capture would belong to the graph's pool). A buffer it replaces is retired,
    not freed -- graphs captured earlier still point at it."""
    from .decode import device_key, retire

    key = device_key(device)
    ws = _SPLITK_WS.get(key)
    if ws is None or ws.numel() < floats:
        retire(ws)
        ws = _SPLITK_WS[key] = torch.empty(floats, dtype=torch.float32, device=device)
    return ws


def gemm_nt_splitk(a: torch.Tensor, b: torch.Tensor, nslice: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """``a @ b.T`` (bf16, f32 accumulation) over ``nslice`` K-slices: the 256x256
    pipeline writes fp32 partial tiles, a reduce kernel sums them. For short-M
    (decode-batch) GEMMs whose N / 256 tiles leave most CUs idle.
    ``(K / nslice) % 8 == 0``; % 128 with M, N % 256 == 0 takes the aligned path."""
    _check_operand(a, "a")
    _check_operand(b, "b")
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise ValueError(f"inner dims differ: a {tuple(a.shape)} b {tuple(b.shape)}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    need = nslice * M * N
    from .decode import device_key

    ws = _SPLITK_WS.get(device_key(a.device))
    if ws is None or ws.numel() < need:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("gemm_nt_splitk: reserve_splitk_workspace() before hipGraph capture")
        ws = reserve_splitk_workspace(a.device, need)
    rc = _lib.lib().kgs_gemm_bf16_nt_splitk(a.data_ptr(), b.data_ptr(), out.data_ptr(), ws.data_ptr(), M, N, K,
                                            a.stride(0), b.stride(0), out.stride(0), nslice,
                                            _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm_nt_splitk[{M}x{N}x{K}/{nslice}]")
    return out


W4X_BK = 64  # the four-wave kernel's K-tile (gemm_w4.h BK)


class PanelWeight:
    """A ``[N, K]`` bf16 weight re-laid out tile-panel major for the four-wave
    kernel's PACKB mode (``native/kernels/gemm_w4.h``): ``[N / bn][K / 64][bn][64]``,
    so each K-step's ``bn x 64`` B block is one contiguous run in HBM. For a
    fused gate|up weight packed with ``swiglu=True`` each panel holds the
    tile's gate / up 32-row groups interleaved, as the SwiGLU epilogue stages
    them. Only valid with the ``bn`` it was packed for."""

    def __init__(self, data: torch.Tensor, n: int, k: int, bn: int, swiglu: bool):
        self.data, self.shape, self.bn, self.swiglu = data, (n, k), bn, swiglu

    def __repr__(self):
        return f"PanelWeight(shape={self.shape}, bn={self.bn}, swiglu={self.swiglu})"


def pack_w4x_weight(w: torch.Tensor, bn: int, swiglu: bool = False) -> PanelWeight:
    """Pack ``w [N, K]`` for :func:`gemm_nt_w4x` / :func:`gemm_nt_w4x_swiglu`
    with ``packed=`` (see :class:`PanelWeight`). ``N % bn == 0``, ``K % 64 == 0``;
    with ``swiglu`` the rows are ``[gate; up]`` (``N = 2I``) and ``bn % 64 == 0``."""
    if w.dim() != 2 or w.dtype != torch.bfloat16:
        raise ValueError("pack_w4x_weight: a 2-D bf16 weight")
    N, K = w.shape
    if bn not in (128, 256) or N % bn or K % W4X_BK:
        raise ValueError(f"pack_w4x_weight: [{N}, {K}] does not tile by {bn} x {W4X_BK}")
    if swiglu:
        # panel tn, 32-row group g: gate rows (even g) / up rows (odd g) of the
        # tile's bn / 2 output columns, in the order the kernel's DMA j stages them
        i, h = N // 2, bn // 2
        gate = w[:i].reshape(i // h, h // 32, 32, K)
        up = w[i:].reshape(i // h, h // 32, 32, K)
        w = torch.stack((gate, up), dim=2).reshape(N, K)
    data = w.reshape(N // bn, bn, K // W4X_BK, W4X_BK).permute(0, 2, 1, 3).contiguous()
    return PanelWeight(data, N, K, bn, swiglu)


def _w4x_flags(packed: int, stages: int, nt_weights: bool = False) -> int:
    if stages not in (2, 3, 4):
        raise ValueError(f"stages must be 2, 3 or 4, got {stages}")
    if nt_weights and stages != 2:
        raise ValueError("nt_weights runs with two LDS stages only")
    return packed | (2 if nt_weights else 0) | (stages - 2) << 4


def _packed_operand(b, bn, swiglu):
    if not isinstance(b, PanelWeight):
        return b, b.shape, b.stride(0), 0
    if b.bn != bn or b.swiglu != swiglu:
        raise ValueError(f"{b!r} used with bn={bn}, swiglu={swiglu}")
    return b.data, b.shape, b.shape[1], 1


def gemm_nt_w4x(a: torch.Tensor, b, bn: int = 256, nslice: int = 1,
                out: torch.Tensor | None = None, bm: int = 256, stages: int = 2,
                nt_weights: bool = False) -> torch.Tensor:
    """``a @ b.T`` on the four-wave kernel with ``bm`` x ``bn`` tiles (256 or 128
    each), any M (rows past M read as zeros), over ``nslice`` K-slices (fp32
    partials + reduce when > 1): the decode-batch GEMM path.
    ``N % bn == 0`` and ``(K / nslice) % 128 == 0``. ``b`` is a ``[N, K]`` tensor
    or a :class:`PanelWeight` packed with the same ``bn``. ``stages``: LDS
    stages (3 / 4 keep more K-tiles in flight; only where they fit in 160 KiB).
    ``nt_weights``: ``b``'s loads non-temporal (decode weights each CU streams
    once), ``a``'s loads default (two stages only)."""
    _check_operand(a, "a")
    b, bshape, ldb, packed = _packed_operand(b, bn, False)
    if not packed:
        _check_operand(b, "b")
    M, K = a.shape
    N, K2 = bshape
    if K != K2:
        raise ValueError(f"inner dims differ: a {tuple(a.shape)} b {tuple(bshape)}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    ws_ptr = None
    if nslice > 1:
        from .decode import device_key

        need = nslice * M * N
        ws = _SPLITK_WS.get(device_key(a.device))
        if ws is None or ws.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("gemm_nt_w4x: reserve_splitk_workspace() before hipGraph capture")
            ws = reserve_splitk_workspace(a.device, need)
        ws_ptr = ws.data_ptr()
    rc = _lib.lib().kgs_gemm_bf16_nt_w4x_ex(a.data_ptr(), b.data_ptr(), out.data_ptr(), ws_ptr, M, N, K, a.stride(0),
                                            ldb, out.stride(0), int(bn), int(nslice), int(bm),
                                            _w4x_flags(packed, stages, nt_weights), _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm_nt_w4x[{M}x{N}x{K} {bm}x{bn}/{nslice}]")
    return out


def addc_ok(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor) -> bool:
    """Whether :func:`gemm_nt_add_` takes these operands: the aligned
    four-wave path (M, N multiples of 256, K of 128, 16-B aligned rows).
    ``KGS_PREFILL_ADDC=0`` says no to everything (A/B against the unfused pair)."""
    if os.environ.get("KGS_PREFILL_ADDC", "1") != "1":
        return False
    if not (a.is_cuda and b.is_cuda and c.is_cuda) or any(t.dtype != torch.bfloat16 for t in (a, b, c)):
        return False
    if a.stride(1) != 1 or b.stride(1) != 1 or c.stride(1) != 1 or a.dim() != 2 or b.dim() != 2 or c.dim() != 2:
        return False
    M, K = a.shape
    N = b.shape[0]
    if b.shape[1] != K or tuple(c.shape) != (M, N):
        return False
    return bool(_lib.lib().kgs_gemm_bf16_nt_w4_ok(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, a.stride(0),
                                                   b.stride(0), c.stride(0)))


def gemm_nt_add_(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """In place ``c = bf16(c + bf16(a @ b.T))``: a projection whose residual add
    runs in the GEMM's store (EPI_ADDC), with the roundings of ``gemm_nt`` followed
    by ``add_rmsnorm``'s add. Aligned four-wave operands only (:func:`addc_ok`);
    persistent above one tile per CU."""
    if not addc_ok(a, b, c):
        raise ValueError("gemm_nt_add_: operands outside the aligned four-wave path (see addc_ok)")
    M, K = a.shape
    N = b.shape[0]
    rc = _lib.lib().kgs_gemm_bf16_nt_addc(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                                          c.stride(0), _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm_nt_add_[{M}x{N}x{K}]")
    return c


def gemm_nt_w4x_partials(a: torch.Tensor, b, bn: int, nslice: int, bm: int = 256, stages: int = 2,
                         nt_weights: bool = False) -> torch.Tensor:
    """The split-K four-wave GEMM WITHOUT its reduce: returns the fp32 partial
    products ``[nslice, M, N]`` (a view of the per-GPU split-K workspace, valid
    until the next split-K call on the stream) for a fused consumer --
    ``kgs.ops.transformer.splitk_add_rmsnorm`` or ``kgs.ops.decode.rope_cache_``."""
    if nslice < 2:
        raise ValueError("partials need nslice >= 2")
    _check_operand(a, "a")
    b, bshape, ldb, packed = _packed_operand(b, bn, False)
    if not packed:
        _check_operand(b, "b")
    M, K = a.shape
    N, K2 = bshape
    if K != K2:
        raise ValueError(f"inner dims differ: a {tuple(a.shape)} b {tuple(bshape)}")
    from .decode import device_key

    need = nslice * M * N
    ws = _SPLITK_WS.get(device_key(a.device))
    if ws is None or ws.numel() < need:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("gemm_nt_w4x_partials: reserve_splitk_workspace() before hipGraph capture")
        ws = reserve_splitk_workspace(a.device, need)
    rc = _lib.lib().kgs_gemm_bf16_nt_w4x_ex(a.data_ptr(), b.data_ptr(), None, ws.data_ptr(), M, N, K, a.stride(0),
                                            ldb, N, int(bn), int(nslice), int(bm),
                                            _w4x_flags(packed, stages, nt_weights),
                                            _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm_nt_w4x_partials[{M}x{N}x{K} {bm}x{bn}/{nslice}]")
    return ws[:need].view(nslice, M, N)


def gemm_nt_w4x_swiglu(a: torch.Tensor, w_gate_up, bn: int = 128,
                       out: torch.Tensor | None = None, bm: int = 256, stages: int = 2,
                       nt_weights: bool = False) -> torch.Tensor:
    """``silu(a @ gate.T) * (a @ up.T)`` for a fused gate|up weight ``[2I, K]``
    (gate rows first) on the four-wave kernel, the SwiGLU applied in the GEMM
    epilogue: returns ``[M, I]`` (both products rounded to bf16 first, as
    ``gemm_nt`` + ``kgs.ops.transformer.silu_mul`` round them). Any M;
    ``2I % bn == 0``, ``K % 128 == 0``. ``w_gate_up`` may be a
    :class:`PanelWeight` from ``pack_w4x_weight(w, bn, swiglu=True)``."""
    _check_operand(a, "a")
    w, wshape, ldb, packed = _packed_operand(w_gate_up, bn, True)
    if not packed:
        _check_operand(w, "w_gate_up")
    M, K = a.shape
    N, K2 = wshape
    if K != K2:
        raise ValueError(f"inner dims differ: a {tuple(a.shape)} w {tuple(wshape)}")
    if out is None:
        out = torch.empty((M, N // 2), dtype=torch.bfloat16, device=a.device)
    rc = _lib.lib().kgs_gemm_bf16_nt_w4x_swiglu_ex(a.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K,
                                                   a.stride(0), ldb, out.stride(0), int(bn), int(bm),
                                                   _w4x_flags(packed, stages, nt_weights),
                                                   _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm_nt_w4x_swiglu[{M}x{N}x{K} {bm}x{bn}]")
    return out


def gemm_nt_w4x_splitk_swiglu(a: torch.Tensor, w_gate_up: torch.Tensor, bn: int = 256, nslice: int = 2,
                              bm: int = 256, out: torch.Tensor | None = None) -> torch.Tensor:
    """SwiGLU over a fused gate|up weight as a split-K GEMM (fp32 partials in the
    split-K workspace) + one reduce-and-SwiGLU pass: returns ``[M, I]`` with the
    roundings of ``gemm_nt`` + ``silu_mul``. For decode batches where the
    epilogue-fused kernel (:func:`gemm_nt_w4x_swiglu`) leaves CUs idle."""
    parts = gemm_nt_w4x_partials(a, w_gate_up, bn=bn, nslice=nslice, bm=bm)
    M, N = a.shape[0], w_gate_up.shape[0]
    if out is None:
        out = torch.empty((M, N // 2), dtype=torch.bfloat16, device=a.device)
    rc = _lib.lib().kgs_splitk_reduce_swiglu_bf16(parts.data_ptr(), out.data_ptr(), int(nslice), M, N // 2,
                                                  out.stride(0), _lib.stream_handle(a.device))
    _lib.check(rc, f"splitk_reduce_swiglu[{nslice}x{M}x{N // 2}]")
    return out


def gemm_swiglu(a: torch.Tensor, w_gate_up: torch.Tensor) -> torch.Tensor:
    """SwiGLU MLP input projection ``silu(a @ gate.T) * (a @ up.T)`` -> ``[M, I]``:
    fused into the four-wave GEMM's epilogue (256x256 tiles; 256x128 when
    ``2I % 256 != 0``) when the shape allows, else GEMM + ``silu_mul``. Same
    bits either way."""
    N, K = w_gate_up.shape
    ok = (a.dim() == 2 and a.dtype == torch.bfloat16 and w_gate_up.dtype == torch.bfloat16 and a.is_cuda
          and a.stride(1) == 1 and w_gate_up.stride(1) == 1 and K % 128 == 0 and N % 128 == 0
          and a.stride(0) % 8 == 0 and w_gate_up.stride(0) % 8 == 0 and (N // 2) % 8 == 0
          and a.data_ptr() % 16 == 0 and w_gate_up.data_ptr() % 16 == 0 and a.shape[1] == K)
    if ok:
        return gemm_nt_w4x_swiglu(a, w_gate_up, bn=256 if N % 256 == 0 else 128)
    from .transformer import silu_mul

    return silu_mul(gemm_nt(a, w_gate_up))


FP8_DTYPE = torch.float8_e4m3fn  # OCP e4m3 -- gfx950's MFMA fp8 format (not MI300's fnuz)
FP8_MAX = 448.0
# fp8: "fast" = the 8-wave aligned pipeline; "w4p" = the four-wave persistent
# kernel (gemm_w4f8.h: K >= 768, "auto" takes it with more 256x256 tiles than CUs)
FP8_VARIANTS = {"auto": 0, "fast": 1, "w4p": 3, "bounded": 16}


def quantize_fp8(x: torch.Tensor, scale: float | None = None) -> tuple[torch.Tensor, float]:
    """Per-tensor e4m3 quantisation: returns ``(x_fp8, scale)`` with
    ``x ~= x_fp8.float() * scale`` (scale = amax / 448 unless given)."""
    if scale is None:
        amax = float(x.detach().abs().max().float().item()) if x.numel() else 0.0
        scale = amax / FP8_MAX if amax > 0 else 1.0
    q = (x.float() / scale).clamp(-FP8_MAX, FP8_MAX).to(FP8_DTYPE)
    return q, float(scale)


def quantize_fp8_dev(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Dynamic per-tensor e4m3 quantisation on the GPU (native/kernels/quant_fp8.hip).

    Returns ``(q, scale)`` where ``scale`` is a 1-element f32 DEVICE tensor
    (``x ~= q.float() * scale``); nothing is copied to the host, so the call is
    graph-capturable. ``x``: contiguous f32/bf16, numel % 8 == 0."""
    if x.dtype not in (torch.float32, torch.bfloat16) or not x.is_cuda or not x.is_contiguous():
        raise ValueError("quantize_fp8_dev needs a contiguous f32/bf16 GPU tensor")
    if x.numel() % 8:
        raise ValueError("numel must be a multiple of 8")
    q = torch.empty(x.shape, dtype=FP8_DTYPE, device=x.device)
    out2 = torch.empty(2, dtype=torch.float32, device=x.device)
    rc = _lib.lib().kgs_quantize_fp8(x.data_ptr(), x.numel(), 1 if x.dtype == torch.bfloat16 else 0, q.data_ptr(),
                                     out2.data_ptr(), _lib.stream_handle(x.device))
    _lib.check(rc, "quantize_fp8")
    return q, out2[1:2]


def gemm_fp8_nt(
    a: torch.Tensor,
    b: torch.Tensor,
    scale_a: float | torch.Tensor = 1.0,
    scale_b: float = 1.0,
    bias: torch.Tensor | None = None,
    act: str | None = None,
    out: torch.Tensor | None = None,
    variant: str = "auto",
) -> torch.Tensor:
    """``act(scale_a*scale_b * (a @ b.T) + bias)`` in bf16 from e4m3 operands.

    a: [M, K], b: [N, K], both ``torch.float8_e4m3fn`` K-contiguous on a gfx950
    device; K % 16 == 0 (K % 256 and M, N % 256 for the aligned path). f32
    accumulation on the scaled 16x16x128 fp8 MFMA (2x the bf16 MFMA rate).
    """
    for t, name in ((a, "a"), (b, "b")):
        if t.dtype != FP8_DTYPE:
            raise TypeError(f"{name} must be {FP8_DTYPE}, got {t.dtype}")
        if not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
            raise ValueError(f"{name} must be a 2-D row-major GPU matrix")
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise ValueError(f"inner dims differ: a {tuple(a.shape)} b {tuple(b.shape)}")
    epi_name = act if act is not None else ("bias" if bias is not None else None)
    if epi_name not in EPI:
        raise ValueError(f"unknown activation {act!r}")
    epi = EPI[epi_name]
    if epi and bias is None:
        bias = torch.zeros(N, dtype=torch.bfloat16, device=a.device)
    if bias is not None and (bias.dtype != torch.bfloat16 or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("bias must be a contiguous bf16 vector of length N")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out")
        if tuple(out.shape) != (M, N):
            raise ValueError(f"out has shape {tuple(out.shape)}, expected {(M, N)}")
    if isinstance(scale_a, torch.Tensor):
        # device-resident (dynamic) activation scale: read in the kernel epilogue
        if scale_a.dtype != torch.float32 or scale_a.numel() != 1 or scale_a.device != a.device:
            raise ValueError("a device scale_a must be a 1-element f32 tensor on a's device")
        alpha, alpha_ptr = float(scale_b), scale_a.data_ptr()
    else:
        alpha, alpha_ptr = float(scale_a) * float(scale_b), None
    rc = _lib.lib().kgs_gemm_fp8_nt_dev(
        a.data_ptr(), b.data_ptr(), out.data_ptr(), bias.data_ptr() if bias is not None else None,
        M, N, K, a.stride(0), b.stride(0), out.stride(0), alpha, alpha_ptr, epi,
        FP8_VARIANTS[variant], _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm_fp8_nt[{M}x{N}x{K}]")
    return out


def gemm_fp8_rows(
    a: torch.Tensor,
    a_scales: torch.Tensor,
    b: torch.Tensor,
    scale_b: float = 1.0,
    bias: torch.Tensor | None = None,
    out: torch.Tensor | None = None,
    variant: str = "auto",
) -> torch.Tensor:
    """``a_scales[m] * scale_b * (a @ b.T) (+ bias)`` in bf16 from e4m3 operands with
    per-row (per-token) activation scales -- the output of the fused quantising
    producers in :mod:`kgs.ops.transformer` (``add_rmsnorm_fp8``, ``silu_mul_fp8``,
    ``quantize_rows_fp8``)."""
    for t, name in ((a, "a"), (b, "b")):
        if t.dtype != FP8_DTYPE:
            raise TypeError(f"{name} must be {FP8_DTYPE}, got {t.dtype}")
        if not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
            raise ValueError(f"{name} must be a 2-D row-major GPU matrix")
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise ValueError(f"inner dims differ: a {tuple(a.shape)} b {tuple(b.shape)}")
    if a_scales.dtype != torch.float32 or a_scales.numel() != M or not a_scales.is_contiguous():
        raise ValueError("a_scales must be a contiguous f32 vector of length M")
    if bias is not None and (bias.dtype != torch.bfloat16 or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("bias must be a contiguous bf16 vector of length N")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out")
    rc = _lib.lib().kgs_gemm_fp8_nt_rows(
        a.data_ptr(), b.data_ptr(), out.data_ptr(), bias.data_ptr() if bias is not None else None,
        M, N, K, a.stride(0), b.stride(0), out.stride(0), float(scale_b), a_scales.data_ptr(),
        EPI["bias"] if bias is not None else 0, FP8_VARIANTS[variant], _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm_fp8_rows[{M}x{N}x{K}]")
    return out


def fast_path_ok(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> bool:
    M, K = a.shape
    N = b.shape[0]
    c_ptr = out.data_ptr() if out is not None else 0
    ldc = out.stride(0) if out is not None else N
    return bool(
        _lib.lib().kgs_gemm_bf16_nt_fast_ok(a.data_ptr(), b.data_ptr(), c_ptr, M, N, K, a.stride(0), b.stride(0), ldc)
    )


def transpose(x: torch.Tensor) -> torch.Tensor:
    """Materialised ``x.T`` for a row-major bf16 matrix (HIP LDS-tiled transpose)."""
    from .elementwise import transpose_bf16

    return transpose_bf16(x)


TR_READ_A = False        # route K-major A through ds_read_b64_tr_b16 (else transpose + NT)
TR_READ_B_MAX_M = 4096   # K-major B: tr reads up to this M, transpose + NT above


def gemm_bf16(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
         bias: torch.Tensor | None = None, act: str | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """``op(a) @ op(b)`` for row-major bf16 matrices, any of the four layouts:

    * ``trans_a=False``: ``a`` is [M, K];  ``trans_a=True``: ``a`` is [K, M] (use ``a.T``)
    * ``trans_b=False``: ``b`` is [K, N];  ``trans_b=True``: ``b`` is [N, K] (the NT layout)

    (so ``gemm_bf16(a, b) == a @ b`` and ``gemm_bf16(a, b, trans_b=True) == a @ b.T``).
    A K-major operand is either read in place through the pipeline's
    transposed-read path (``ds_read_b64_tr_b16``, aligned shapes) or
    materialised by the 6.3 TB/s HIP transpose and fed to the NT kernel,
    whichever measured faster for the shape (module constants below).
    """
    _check_operand(a, "a")
    _check_operand(b, "b")
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N, K2 = (b.shape[0], b.shape[1]) if trans_b else (b.shape[1], b.shape[0])
    if K != K2:
        raise ValueError(f"inner dims differ: op(a) {M}x{K}, op(b) {K2}x{N}")
    ta, tb = int(trans_a), int(not trans_b)  # kernel flags: 1 = operand stored [K][rows]
    if ta and not TR_READ_A:
        # measured: the tr-read A path runs ~20 % behind a 6.3 TB/s transpose + NT
        # at 8192^3 and ties at 4096^3 (profiles/gemm_layouts.json)
        a, ta = transpose(a), 0
    if tb and M > TR_READ_B_MAX_M:
        # the B transpose costs ~ 476/M of the GEMM time; above M = 4096 it is
        # cheaper than the tr-read path's LDS cost (profiles/gemm_layouts.json)
        b, tb = transpose(b), 0
    if not ta and not tb:
        return gemm_nt(a, b, bias=bias, act=act, out=out)
    epi_name = act if act is not None else ("bias" if bias is not None else None)
    if epi_name not in EPI:
        raise ValueError(f"unknown activation {act!r}")
    epi = EPI[epi_name]
    if epi and bias is None:
        bias = torch.zeros(N, dtype=torch.bfloat16, device=a.device)
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    so = _lib.lib()
    ok = so.kgs_gemm_bf16_layout_ok(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                                    out.stride(0), ta, tb)
    if not ok or (bias is not None and bias.data_ptr() % 8):
        aa = transpose(a) if ta else a
        bb = transpose(b) if tb else b
        return gemm_nt(aa, bb, bias=bias, act=act, out=out)
    rc = so.kgs_gemm_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), bias.data_ptr() if bias is not None else None,
                          M, N, K, a.stride(0), b.stride(0), out.stride(0), ta, tb, epi,
                          _lib.stream_handle(a.device))
    _lib.check(rc, f"gemm[{M}x{N}x{K}, ta={ta}, tb={tb}]")
    return out


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b`` with ``b: [K, N]`` row-major (transposed-read path, no transpose copy)."""
    return gemm_bf16(a, b)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, act):
        ctx.save_for_backward(x, w, bias)
        ctx.act = act
        if act in (None, "none"):
            return gemm_nt(x, w, bias=bias)
        if not any(ctx.needs_input_grad[:3]):
            return gemm_nt(x, w, bias=bias, act=act)  # inference: activation fused in the epilogue
        # training keeps the pre-activation for the backward pass: GEMM with the
        # bias epilogue, then the activation in torch (cheap, memory-bound)
        z = gemm_nt(x, w, bias=bias)
        ctx.z = z
        return _act(z, act)

    @staticmethod
    def backward(ctx, gy):
        x, w, bias = ctx.saved_tensors
        gy = gy.contiguous()
        if ctx.act not in (None, "none"):
            z = ctx.z.float().requires_grad_(True)
            with torch.enable_grad():
                y = _act(z, ctx.act)
            (gz,) = torch.autograd.grad(y, z, gy.float())
            gy = gz.to(torch.bfloat16).contiguous()
        # dX[M,K] = dY[M,N] . W[N,K]      (W read K-major: transposed-read path)
        gx = gemm_bf16(gy, w)
        # dW[N,K] = dY^T[N,M] . X[M,K]    (both operands M-major)
        gw = gemm_bf16(gy, x, trans_a=True)
        gb = gy.float().sum(0).to(torch.bfloat16) if bias is not None else None
        return gx, gw, gb, None


def _act(z: torch.Tensor, act: str) -> torch.Tensor:
    if act == "gelu":
        return torch.nn.functional.gelu(z, approximate="tanh")
    if act == "relu":
        return torch.relu(z)
    if act == "silu":
        return torch.nn.functional.silu(z)
    if act == "bias":
        return z
    raise ValueError(act)


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None):
    """Differentiable ``act(x @ w.T + bias)`` on the HIP GEMM (x: [M,K], w: [N,K])."""
    return _LinearFn.apply(x, w, bias, act)


class Linear(torch.nn.Module):
    """bf16 ``nn.Linear`` whose forward and backward GEMMs run on the HIP kernel."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, act: str | None = None,
                 device=None):
        super().__init__()
        w = torch.empty(out_features, in_features, dtype=torch.bfloat16, device=device)
        torch.nn.init.normal_(w, std=in_features ** -0.5)
        self.weight = torch.nn.Parameter(w)
        self.bias = torch.nn.Parameter(torch.zeros(out_features, dtype=torch.bfloat16, device=device)) if bias else None
        self.act = act

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        y = linear(x.reshape(-1, shp[-1]).contiguous(), self.weight, self.bias, self.act)
        return y.reshape(*shp[:-1], y.shape[-1])


class Fp8Linear(torch.nn.Module):
    """W8A8 inference Linear on the fp8 MFMA GEMM.

    The weight is quantised once to e4m3 with a per-tensor host scale. Each
    forward quantises the activation on the GPU (dynamic per-tensor scale,
    device-resident) and runs ``gemm_fp8_nt`` with the bias/activation epilogue
    fused: two small kernels and one GEMM, no host synchronisation
    (hipGraph-capturable)."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None):
        super().__init__()
        qw, sw = quantize_fp8(weight.detach())
        self.register_buffer("qweight", qw.contiguous())
        self.w_scale = sw
        self.register_buffer("bias", None if bias is None else bias.detach().to(torch.bfloat16).contiguous())
        self.act = act

    @classmethod
    def from_linear(cls, lin: torch.nn.Module) -> "Fp8Linear":
        return cls(lin.weight, getattr(lin, "bias", None), getattr(lin, "act", None))

    def forward_q(self, x8: torch.Tensor, x_scales: torch.Tensor) -> torch.Tensor:
        """Pre-quantised activation (e4m3 rows + per-row f32 scales, e.g. from
        ``kgs.ops.add_rmsnorm_fp8``); bias only (no activation epilogue)."""
        if self.act is not None:
            raise ValueError("forward_q supports no fused activation")
        return gemm_fp8_rows(x8, x_scales, self.qweight, self.w_scale, bias=self.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        qx, sx = quantize_fp8_dev(x.reshape(-1, shp[-1]).contiguous())
        y = gemm_fp8_nt(qx, self.qweight, sx, self.w_scale, bias=self.bias, act=self.act)
        return y.reshape(*shp[:-1], y.shape[-1])
