"""Decode-path ops on ``native/kernels/decode.hip`` -- the one-token-per-sequence
half of LLM serving, which is HBM-bound on the weights and the KV cache.

* :func:`pack_weight` / :class:`PackedWeight` -- a ``[N, K]`` bf16 weight
  rearranged ONCE into MFMA A-fragment order (``[N/16][K/32][64][8]``), so the
  skinny GEMM streams it as contiguous 1 KB wave loads straight into registers.
* :func:`skinny_gemm` -- ``x[M, K] @ W^T`` for a decode batch ``M <= 256``
  (split-K with an in-kernel last-arriver reduction when ``N`` is small).
* :class:`PagedKVCache` -- ``[layers, pages, kv_heads, K|V, 32 x 128]`` bf16
  pages whose element order IS the MFMA operand order of the decode attention
  (:func:`kv_index_tables`); a 32-token page of one KV head is 16 KB.
* :func:`rope_cache_` -- RoPE on the q/k heads of fused QKV rows + scatter of k/v
  into their cache slots, one launch.
* :func:`paged_decode_attention` -- GQA decode attention over the paged cache
  (context split across waves, log-sum-exp merge by the last split, one launch).

Every op raises :class:`kgs.ops.NativeUnavailable` when the native library is
missing; the ``ref_*`` functions are the plain-PyTorch fp32 references (they run
on CPU too and define the cache layout for tests).
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib

PAGE = 32
HEAD_DIM = 128
CUS = 256  # MI355X compute units (grid sizing)


# ----------------------------------------------------------------------------
# weights

def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """``[N, K]`` -> ``[N/16, K/32, 64, 8]``: lane ``g*16 + r`` of fragment
    ``(nt, kk)`` holds ``W[16 nt + r, 32 kk + 8 g : +8]`` (16x16x32 bf16 A map)."""
    n, k = w.shape
    if n % 16 or k % 32:
        raise ValueError(f"pack_weight needs N % 16 == 0 and K % 32 == 0, got {tuple(w.shape)}")
    return w.reshape(n // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


def unpack_weight(p: torch.Tensor) -> torch.Tensor:
    nt, kk = p.shape[:2]
    return p.reshape(nt, kk, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(nt * 16, kk * 32)


def swiglu_rows(n2: int) -> torch.Tensor:
    """Row order of a fused gate|up weight ``[2I, K]`` (gate rows first) in which
    16-row tile ``t`` holds gate rows ``8t..8t+7`` then up rows ``8t..8t+7``: the
    skinny GEMM's SwiGLU epilogue pairs them lane-to-lane (``lane ^ 32``)."""
    if n2 % 32:
        raise ValueError("fused gate|up weight needs 2I % 32 == 0")
    inter = n2 // 2
    return torch.arange(n2).reshape(2, inter // 8, 8).permute(1, 0, 2).reshape(n2)


def rope_rows(n: int, heads: int, kv_heads: int) -> torch.Tensor:
    """Row order of a fused qkv weight ``[(H + 2 HKV) * 128, K]`` in which every
    q / k head's 16-row tile ``t`` holds dims ``8t..8t+7`` then ``64+8t..64+8t+7``
    (v heads unchanged): the skinny GEMM's RoPE epilogue pairs each rotate-half
    partner lane-to-lane (``lane ^ 32``)."""
    if n != (heads + 2 * kv_heads) * HEAD_DIM:
        raise ValueError(f"qkv weight of {n} rows does not match {heads} + 2 x {kv_heads} heads of {HEAD_DIM}")
    head = torch.arange(HEAD_DIM).reshape(2, 8, 8).permute(1, 0, 2).reshape(HEAD_DIM)
    rot = heads + kv_heads
    q_k = (torch.arange(rot)[:, None] * HEAD_DIM + head[None, :]).reshape(-1)
    return torch.cat([q_k, torch.arange(rot * HEAD_DIM, n)])


def pack_swiglu(w: torch.Tensor) -> torch.Tensor:
    return pack_weight(w[swiglu_rows(w.shape[0]).to(w.device)])


FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0


class PackedWeight:
    """A projection weight in skinny-GEMM fragment order (plus its shape).

    * ``swiglu=True``: a fused gate|up weight whose GEMM emits ``silu(g) * u``;
    * ``fold``: an RMSNorm weight ``[K]`` folded into the columns (``W * fold``),
      for GEMMs that apply the norm in their epilogue (``rms=``);
    * ``fp8=True``: weight-only fp8 (W8A16): OCP e4m3 with one scale per output
      row, dequantised to bf16 in registers (half the HBM bytes per step);
    * ``rope=(H, HKV)``: a fused qkv weight in :func:`rope_rows` order, for the
      GEMM whose epilogue applies RoPE and writes the KV cache (``rope=`` of
      :func:`skinny_gemm`); its output is in the original order."""

    __slots__ = ("data", "n", "k", "swiglu", "fp8", "wscale", "rope")

    def __init__(self, w: torch.Tensor, swiglu: bool = False, fold: torch.Tensor | None = None, fp8: bool = False,
                 rope: tuple | None = None):
        self.n, self.k = w.shape
        self.swiglu, self.fp8, self.rope = swiglu, fp8, rope
        if swiglu and rope:
            raise ValueError("a weight is either SwiGLU- or RoPE-packed")
        rows = swiglu_rows(self.n).to(w.device) if swiglu else \
            rope_rows(self.n, *rope).to(w.device) if rope else None
        if fold is not None:
            w = w.float() * fold.float()[None, :]
        if fp8:
            wf = w.float()
            scale = wf.abs().amax(1).clamp(min=1e-12) / FP8_MAX
            q = (wf / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8).view(torch.uint8)
            if rows is not None:
                q, scale = q[rows], scale[rows]
            self.data = pack_weight(q)
            self.wscale = scale.float().contiguous()
        else:
            w = w.to(torch.bfloat16)
            self.data = pack_weight(w[rows] if rows is not None else w)
            self.wscale = None

    @property
    def n_out(self) -> int:
        return self.n // 2 if self.swiglu else self.n

    def unpacked(self) -> torch.Tensor:
        """The weight as the kernel sees it (dequantised for fp8), in original row order."""
        p = unpack_weight(self.data)
        if self.fp8:
            p = (p.view(FP8).float() * self.wscale[:, None]).to(torch.bfloat16)
        if self.swiglu or self.rope:
            rows = swiglu_rows(self.n) if self.swiglu else rope_rows(self.n, *self.rope)
            inv = torch.empty(self.n, dtype=torch.long, device=p.device)
            inv[rows.to(p.device)] = torch.arange(self.n, device=p.device)
            p = p[inv]
        return p


# tile variants of native/kernels/decode.hip (id -> (R W-row tiles per wave,
# MT 16-column x tiles, KC k-steps per x chunk)); 0 = default for the batch size
SKINNY_VARIANTS = {
    1: (1, 1, 16), 2: (1, 1, 8), 3: (2, 1, 16),
    4: (1, 2, 16), 5: (1, 2, 8), 6: (2, 2, 8), 7: (2, 2, 16),
    8: (1, 4, 16), 9: (1, 4, 4), 10: (1, 4, 8), 11: (2, 4, 4), 12: (2, 4, 8),
    13: (2, 8, 2), 14: (2, 8, 4), 15: (4, 8, 2), 16: (1, 8, 4),
    17: (2, 16, 2), 18: (1, 16, 4), 19: (1, 16, 2),
    20: (1, 1, 8), 21: (2, 1, 8),
}
# variants whose four waves split one strip's K range (decode.hip skinny KIN):
# strips of 16 R rows, chunks of 4 x KC k-steps, no cross-workgroup split-K
KIN_VARIANTS = frozenset({20, 21})
_DEFAULT_VARIANT = {1: 1, 2: 4, 4: 8, 8: 13, 16: 17}

# Measured routing per (MT, N, K) on MI355X with weights streamed from HBM
# (bench/decode_bench.py --tune, profiles/decode_tune.md): (variant, ksplit) of
# the skinny GEMM where it beat hipBLASLt, None where hipBLASLt won. Shapes:
# Llama-3-8B qkv 6144x4096, o 4096x4096, gate|up 28672x4096, down 4096x14336,
# lm_head 128256x4096.
_QKV, _O, _GU, _DOWN, _LM = (6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)
TUNED: dict = {
    (1, *_QKV): (1, 2), (1, *_O): (20, 1), (1, *_GU): (3, 1), (1, *_DOWN): (1, 4), (1, *_LM): (1, 1),
    (2, *_QKV): (4, 2), (2, *_O): (4, 4), (2, *_GU): (6, 1), (2, *_DOWN): (4, 4), (2, *_LM): (6, 1),
    (4, *_QKV): None, (4, *_O): (9, 4), (4, *_GU): (11, 1), (4, *_DOWN): (10, 4), (4, *_LM): (11, 1),
    (8, *_QKV): None, (8, *_O): None, (8, *_GU): None, (8, *_DOWN): (16, 4), (8, *_LM): None,
    (16, *_QKV): None, (16, *_O): None, (16, *_GU): None, (16, *_DOWN): None, (16, *_LM): None,
}
# few-row batches: (variant, ksplit, up to M) -- the in-workgroup K split
# (variant 20) wins while x is a few rows (each wave reads its B fragments
# straight from L2, so x traffic grows with M); profiles/r2/skinny_kin_tune.jsonl
TUNED_TINY: dict = {_QKV: (20, 1, 8), _GU: (20, 1, 4), _DOWN: (20, 1, 2)}
TUNED_TINY_FP8: dict = {_GU: (21, 1, 4), _DOWN: (21, 7, 4)}
# the same sweep for weight-only fp8 (--tune --fp8): (variant, ksplit) per (MT, N, K)
TUNED_FP8: dict = {
    (1, *_QKV): (20, 1), (2, *_QKV): (5, 4), (4, *_QKV): (9, 4),
    (1, *_O): (20, 1), (2, *_O): (5, 4), (4, *_O): (10, 4),
    (1, *_GU): (1, 1), (2, *_GU): (7, 1), (4, *_GU): (12, 2),
    (1, *_DOWN): (1, 7), (2, *_DOWN): (5, 8), (4, *_DOWN): (9, 8),
    (1, *_LM): (1, 1), (2, *_LM): (6, 1), (4, *_LM): (11, 1),
}
# Decode batches above the fused range: K slices of the split-K 256x256 GEMM
# (kgs.ops.gemm.gemm_nt_splitk) per (batch bucket, N, K) where it beat both
# hipBLASLt and the skinny GEMM (bench/decode_bench.py --wide,
# profiles/decode_wide_gemm.jsonl): down 1.89x / 1.14x / 1.48x at 128 / 256 /
# 512, qkv 1.22x at 256, o 1.07x at 128. gate|up (fp32 partials too large) and
# the rest stay on hipBLASLt.
SPLITK_TUNED: dict = {
    (128, *_DOWN): 16, (128, *_O): 8,
    (256, *_QKV): 8, (256, *_DOWN): 8,
    (512, *_DOWN): 8,
    # Llama-3-70B (decode without packed copies, `--model llama3-70b`; bench/decode_bench.py --wide
    # --model llama3-70b): down 1.55x / 1.83x / 2.3x at 64 / 128 / 256, qkv 1.40x and o 1.47x at 256;
    # 1 = the plain 256x256 GEMM (gate|up at 256: 1.22x)
    (64, 8192, 28672): 8,
    (128, 10240, 8192): 4, (128, 8192, 8192): 8, (128, 8192, 28672): 8,
    (256, 10240, 8192): 4, (256, 8192, 8192): 8, (256, 8192, 28672): 8, (256, 57344, 8192): 1,
}
SPLITK_WS_FLOATS = 8 * 256 * 8192  # the largest entry above (M x N x slices)

# Decode batches 49-512 on the four-wave kernel (kgs.ops.gemm.gemm_nt_w4x):
# (tile width, K slices, tile height) per (batch bucket, N, K) where it beat
# hipBLASLt and the 8-wave split-K, weights streamed from HBM
# (bench/decode_w4x_sweep.py, profiles/r2/decode_w4x_sweep.jsonl and
# decode_w4x_bm128.jsonl, decode_w4x_lm_head.jsonl; speed-up vs hipBLASLt in the comments). Batches up to
# 128 take 128-row tiles (no MFMAs on padding rows: qkv / o / down 3-20 %
# faster than 256-row tiles at 64-128 rows, and ahead of the fused skinny
# GEMMs from 49 rows up). Buckets not listed stay on the routes below.
_W4X_BUCKETS = (64, 96, 128, 192, 256, 384, 512)
W4X_MIN_BATCH = 49
W4X_TUNED: dict = {
    (64, *_QKV): (128, 4, 128), (96, *_QKV): (128, 8, 128), (128, *_QKV): (128, 4, 128),  # 1.99/4.39/3.31
    (64, *_O): (128, 8, 128), (96, *_O): (128, 8, 128), (128, *_O): (128, 8, 128),  # 4.95/2.27/2.22
    (64, *_GU): (128, 1, 128), (96, *_GU): (128, 1, 128), (128, *_GU): (128, 1, 128),  # 1.16/1.15/1.14
    (64, *_DOWN): (128, 8, 128), (96, *_DOWN): (128, 8, 128), (128, *_DOWN): (128, 8, 128),  # 1.75/2.07/2.29
    (64, *_LM): (256, 1, 128), (96, *_LM): (256, 1, 128), (128, *_LM): (256, 1, 128),  # 1.18/1.22/1.24
    (192, *_QKV): (128, 4, 256), (256, *_QKV): (128, 4, 256), (384, *_QKV): (128, 2, 256),  # 1.39/1.49/1.06
    # o at 192-256 rows: 128-row tiles, 4 slices (half the fp32 partials of 256-row tiles x 8 slices;
    # probe 29.6 / 30.6 vs 32.9 / 33.7 us, serving b256 +0.8 % A/B/A, profiles/r3/decode/route_ab)
    (192, *_O): (128, 4, 128), (256, *_O): (128, 4, 128), (384, *_O): (128, 4, 256),  # -/-/1.02
    (512, *_O): (128, 4, 256),  # 1.10
    (192, *_GU): (128, 1, 256), (256, *_GU): (128, 1, 256), (512, *_GU): (256, 1, 256),  # 1.07/1.06/1.06
    (192, *_DOWN): (128, 8, 256), (256, *_DOWN): (128, 8, 256), (384, *_DOWN): (128, 4, 256),  # 2.7/1.5/1.4
    (512, *_DOWN): (128, 4, 256),  # 1.45
}


def _apply_w4x_override(spec: str) -> None:
    """``KGS_W4X_ROUTES="256,4096,4096=128,4,128,4;..."``: (bucket, N, K) =
    (bn, slices, bm[, stages]) entries replacing W4X_TUNED's, for same-box
    routing A/B runs (scripts/gpu.sh route_ab); ``=none`` removes an entry."""
    for item in filter(None, (s.strip() for s in spec.split(";"))):
        key, _, val = item.partition("=")
        k = tuple(int(t) for t in key.split(","))
        if len(k) != 3 or k[0] not in _W4X_BUCKETS:
            raise ValueError(f"KGS_W4X_ROUTES: bad key {key!r}")
        if val.strip() == "none":
            W4X_TUNED.pop(k, None)
            continue
        v = tuple(int(t) for t in val.split(","))
        if len(v) not in (3, 4):
            raise ValueError(f"KGS_W4X_ROUTES: bad route {val!r}")
        W4X_TUNED[k] = v


if os.environ.get("KGS_W4X_ROUTES"):
    _apply_w4x_override(os.environ["KGS_W4X_ROUTES"])


def w4x_route(m: int, n: int, k: int):
    """(tile width, K slices, tile height[, LDS stages]) of the four-wave
    decode GEMM for batch m, or None. The tuple's order is
    ``gemm_nt_w4x_partials``'s (bn, nslice, bm, stages) positional order."""
    if m < W4X_MIN_BATCH or m > 512:
        return None
    b = next(x for x in _W4X_BUCKETS if m <= x)
    return W4X_TUNED.get((b, n, k))


def w4x_stages(route) -> int:
    """LDS stages of a W4X_TUNED route (2 unless the entry names 3 or 4)."""
    return route[3] if len(route) > 3 else 2


# Decode weights are read once per step by one CU each: their loads go
# non-temporal (gemm_w4.h AUX 52, B's loads only; the activations, re-read by
# every workgroup from L2, keep the default policy). gate|up at batch 256:
# 69.1 -> 68.0 us row-major, 67.5 -> 64.9 us tile-panel packed
# (profiles/r4/decode/README.md); batch-256 serving, two A/B/A passes on one
# box: 18 247 -> 18 302 output tok/s (profiles/r5/decode/README.md). On by
# default since round 5: the fault that kept it opt-in in round 4 was the
# graph memset node of the persistent GEMM's ticket slot, not these loads
# (profiles/r5/fault/README.md; the nt kernels differ from the default ones
# only in the nt bit of B's buffer loads). KGS_NT_WEIGHTS=0 turns it off.
NT_WEIGHTS = os.environ.get("KGS_NT_WEIGHTS", "1") == "1"


def w4x_nt(route) -> bool:
    """Stream this route's weights non-temporally (two-stage routes only)."""
    return NT_WEIGHTS and w4x_stages(route) == 2


def w4x_split_bns(n: int, k: int) -> set:
    """Tile widths the split-K four-wave routes use for an ``[n, k]`` weight
    (the bn a tile-panel copy must be packed with)."""
    return {r[0] for (_, rn, rk), r in W4X_TUNED.items() if (rn, rk) == (n, k) and r[1] > 1}


def splitk_slices(m: int, n: int, k: int) -> int | None:
    """K slices for a decode GEMM of batch m (bucketed to a power of two), or
    None when the split-K kernel is not the measured winner."""
    mb = 1 << max(0, (m - 1).bit_length())
    return SPLITK_TUNED.get((mb, n, k))


SKINNY_DEFAULT_MAX_M = 32  # untuned shapes: skinny GEMM up to this batch, hipBLASLt above


def _mt(m: int) -> int:
    if not 0 < m <= 256:
        raise ValueError(f"skinny GEMM batch must be 1..256, got {m}")
    return 1 if m <= 16 else 2 if m <= 32 else 4 if m <= 64 else 8 if m <= 128 else 16


def skinny_variants(m: int) -> list[int]:
    mt = _mt(m)
    return [v for v, (_, vmt, _) in SKINNY_VARIANTS.items() if vmt == mt]


def skinny_geometry(m: int, variant: int = 0) -> tuple[int, int, int]:
    """(rows of W per workgroup strip, k per x chunk, padded batch) -- mirrors
    ``kgs_skinny_variant_geometry`` in decode.hip."""
    mt = _mt(m)
    v = variant or _DEFAULT_VARIANT[mt]
    r, vmt, kc = SKINNY_VARIANTS[v]
    if vmt != mt:
        raise ValueError(f"variant {variant} is for {16 * vmt}-column batches, not M={m}")
    if v in KIN_VARIANTS:
        return 16 * r, 128 * kc, 16 * mt
    return 64 * r, 32 * kc, 16 * mt


def choose_ksplit(m: int, n: int, k: int, cus: int = CUS, variant: int = 0) -> int:
    """Largest divisor of the k-chunk count that keeps the grid within one
    workgroup per CU (measured best: long-running streaming workgroups,
    profiles/decode_kernels.md) and the fp32 slabs within 64 MB (1 = no split)."""
    rps, kpc, mpad = skinny_geometry(m, variant)
    nstrip, nchunks = n // rps, k // kpc
    best = 1
    for d in range(2, nchunks + 1):
        if nchunks % d:
            continue
        if nstrip * d > max(cus, nstrip) or d * mpad * n * 4 > (64 << 20):
            break
        best = d
    return best


def skinny_config(m: int, n: int, k: int, fp8: bool = False) -> tuple[int, int]:
    """(variant, ksplit) for a skinny-GEMM call: the tuned entry, else the defaults."""
    tiny = (TUNED_TINY_FP8 if fp8 else TUNED_TINY).get((n, k))
    if tiny is not None and m <= tiny[2]:
        return tiny[:2]
    hit = (TUNED_FP8 if fp8 else TUNED).get((_mt(m), n, k))
    if hit is not None:
        return hit
    v = _DEFAULT_VARIANT[_mt(m)]
    return v, choose_ksplit(m, n, k, variant=v)


def use_skinny(m: int, n: int, k: int) -> bool:
    """Decode routing: True = skinny GEMM, False = the library GEMM (hipBLASLt)."""
    if not 0 < m <= 256:
        return False
    key = (_mt(m), n, k)
    if key in TUNED:
        return TUNED[key] is not None
    return m <= SKINNY_DEFAULT_MAX_M


_WS: dict = {}
# Workspaces replaced by larger ones. hipGraphs captured before the growth still
# hold the old device pointers, so the old buffers must outlive them: they are
# kept here for the life of the process instead of going back to the caching
# allocator (where they could be reused, or released to the driver and fault).
_RETIRED: list = []


def device_key(device: torch.device) -> int:
    """Normalised per-GPU cache key: torch.device("cuda") and "cuda:0" differ as
    dict keys but name the same workspace."""
    return device.index if device.index is not None else torch.cuda.current_device()


def retire(*bufs) -> None:
    _RETIRED.extend(b for b in bufs if b is not None)


def _workspace(device: torch.device, floats: int, ints: int):
    """Per-device split-K slab buffer and zeroed ticket counters (the kernel
    re-arms the counters it uses). GEMMs of one device are stream-ordered."""
    key = device_key(device)
    ws, cnt = _WS.get(key, (None, None))
    if ws is None or ws.numel() < floats:
        retire(ws)
        ws = torch.empty(max(floats, 1 << 20), dtype=torch.float32, device=device)
    if cnt is None or cnt.numel() < ints:
        retire(cnt)
        cnt = torch.zeros(max(ints, 4096), dtype=torch.int32, device=device)
    _WS[key] = (ws, cnt)
    return ws, cnt


EPI_SWIGLU, EPI_RMS, EPI_RESID = 1, 2, 4


def skinny_gemm(x: torch.Tensor, w: PackedWeight, out: torch.Tensor | None = None,
                ksplit: int | None = None, variant: int = 0, rms: torch.Tensor | None = None,
                resid_ss: torch.Tensor | None = None, zero: torch.Tensor | None = None,
                eps: float = 1e-5, rope: dict | None = None) -> torch.Tensor:
    """``x @ W^T`` (bf16, fp32 accumulate) for ``x: [M <= 256, K]`` row-major;
    ``silu(x @ Wg^T) * (x @ Wu^T)`` for a ``swiglu`` weight. Fused epilogues:

    * ``rms`` (fp32 ``[M]`` row sums of squares of x): RMSNorm folded in -- the
      rows are scaled by ``rsqrt(rms / K + eps)`` (the norm weight must be folded
      into W, ``PackedWeight(..., fold=w)``);
    * ``resid_ss`` (fp32 ``[M]``): ``out`` is the residual stream, updated in
      place (``out += x @ W^T``), and the new rows' sums of squares are added
      into ``resid_ss`` (for the next ``rms`` consumer);
    * ``zero`` (fp32 ``[M]``): cleared at kernel start (a consumed statistic);
    * ``rope`` (a ``rope=(H, HKV)``-packed qkv weight): dict of ``cos``, ``sin``
      (fp32 ``[max_pos, 64]``), ``positions`` and ``slots`` (int32 ``[M]``) and
      ``cache`` (the layer's bf16 pages): q / k rotated at their positions, k / v
      written into their cache slots -- :func:`rope_cache_` in the epilogue."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be a row-major bf16 GPU matrix")
    m, k = x.shape
    if k != w.k:
        raise ValueError(f"inner dims differ: x {tuple(x.shape)} vs W [{w.n}, {w.k}]")
    if w.fp8 and _mt(m) > 4:
        raise ValueError("fp8 (W8A16) skinny GEMM covers batches <= 64")
    if variant == 0 and ksplit is None:
        variant, ks = skinny_config(m, w.n, k, fp8=w.fp8)
        if rope is not None and SKINNY_VARIANTS[variant][0] != 1:
            # the RoPE epilogue is built for one-tile waves (R 1): the batch's default variant
            variant = _DEFAULT_VARIANT[_mt(m)]
            ks = choose_ksplit(m, w.n, k, variant=variant)
    else:
        ks = ksplit if ksplit is not None else choose_ksplit(m, w.n, k, variant=variant)
    rps, kpc, mpad = skinny_geometry(m, variant)
    if w.n % rps or k % kpc:
        raise ValueError(f"skinny GEMM needs N % {rps} == 0 and K % {kpc} == 0 (N={w.n}, K={k})")
    epi = (EPI_SWIGLU if w.swiglu else 0) | (EPI_RMS if rms is not None else 0) | \
        (EPI_RESID if resid_ss is not None else 0)
    for t, name in ((rms, "rms"), (resid_ss, "resid_ss"), (zero, "zero")):
        if t is not None and (t.dtype != torch.float32 or t.numel() < m or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous fp32 vector of >= M elements")
    if resid_ss is not None:
        if w.swiglu or out is None or tuple(out.shape) != (m, w.n):
            raise ValueError("resid_ss needs the residual stream as out [M, N] (and no swiglu)")
    if out is None:
        out = torch.empty((m, w.n_out), dtype=torch.bfloat16, device=x.device)
    ws, cnt = _workspace(x.device, ks * mpad * w.n if ks > 1 else 0, w.n // rps)
    if (rope is not None) != bool(w.rope):
        raise ValueError("rope= needs a rope-packed qkv weight (PackedWeight(..., rope=(H, HKV))) and vice versa")
    if rope is not None:
        if w.fp8 or resid_ss is not None:
            raise ValueError("the RoPE epilogue is bf16-weight only and writes a fresh qkv output")
        cache = rope["cache"]
        if cache.dtype != torch.bfloat16 or not cache.is_contiguous():
            raise ValueError("the RoPE epilogue writes a bf16 KV cache")
        for key in ("positions", "slots"):
            v = rope[key]
            if v.dtype != torch.int32 or not v.is_contiguous() or v.numel() < m:
                raise ValueError(f"{key} must be a contiguous int32 vector of >= M elements")
        rc = _lib.lib().kgs_skinny_gemm_bf16_rope(
            w.data.data_ptr(), x.data_ptr(), out.data_ptr(), ws.data_ptr(), cnt.data_ptr(), m, w.n, k, x.stride(0),
            out.stride(0), ks, variant, EPI_RMS if rms is not None else 0,
            rms.data_ptr() if rms is not None else None, 1.0 / k, float(eps), rope["cos"].data_ptr(),
            rope["sin"].data_ptr(), rope["positions"].data_ptr(), rope["slots"].data_ptr(), cache.data_ptr(),
            w.rope[0], w.rope[1], _lib.stream_handle(x.device))
        _lib.check(rc, f"skinny_gemm_rope[{m}x{w.n}x{k}, variant={variant}, ksplit={ks}]")
        return out
    rc = _lib.lib().kgs_skinny_gemm_bf16_fused(
        w.data.data_ptr(), x.data_ptr(), out.data_ptr(), ws.data_ptr(), cnt.data_ptr(), m, w.n, k, x.stride(0),
        out.stride(0), ks, variant, epi, rms.data_ptr() if rms is not None else None,
        resid_ss.data_ptr() if resid_ss is not None else None, zero.data_ptr() if zero is not None else None,
        1.0 / k, float(eps), w.wscale.data_ptr() if w.fp8 else None, _lib.stream_handle(x.device))
    _lib.check(rc, f"skinny_gemm[{m}x{w.n}x{k}, variant={variant}, ksplit={ks}, epi={epi}, fp8={w.fp8}]")
    return out


def reserve_workspace(device) -> None:
    """Allocate the largest split-K slab buffers the decode GEMMs can ask for up
    front (skinny: 64 MB; the 256x256 split-K kernel: SPLITK_WS_FLOATS), e.g.
    before hipGraph capture."""
    from .gemm import reserve_splitk_workspace

    _workspace(torch.device(device), 16 << 20, 1 << 16)
    reserve_splitk_workspace(torch.device(device), SPLITK_WS_FLOATS)


# ----------------------------------------------------------------------------
# paged KV cache

def kv_index_tables(device="cpu") -> tuple[torch.Tensor, torch.Tensor]:
    """``(K_IDX, V_IDX)``, each ``[32, 128]`` int64: the position of token ``tau``,
    dim ``d`` inside a page's K / V region (``kv_k_index`` / ``kv_v_index`` in
    decode.hip). K is in S^T = K.Q^T A-fragment order, V in O^T = V^T.P^T
    A-fragment order with the token order S^T's accumulator produces."""
    tau = torch.arange(PAGE, device=device)[:, None]
    d = torch.arange(HEAD_DIM, device=device)[None, :]
    k_idx = (((tau >> 4) * 4 + (d >> 5)) * 64 + ((d >> 3) & 3) * 16 + (tau & 15)) * 8 + (d & 7)
    v_idx = ((d >> 4) * 64 + ((tau >> 2) & 3) * 16 + (d & 15)) * 8 + (tau & 3) + 4 * (tau >> 4)
    return k_idx, v_idx


class PagedKVCache:
    """All layers' KV pages in one allocation: ``[layers, pages, kv_heads, 2, 4096]``
    (2 = K then V region of a 32-token page) in bf16, or in OCP e4m3
    (``dtype="fp8"``: scale 1, saturating -- half the bytes the decode attention
    streams and twice the tokens per GB). Pages are handed out by the
    scheduler's block allocator (kgs.serve)."""

    def __init__(self, layers: int, pages: int, kv_heads: int, device, dtype="bf16"):
        self.layers, self.pages, self.kv_heads = layers, pages, kv_heads
        tdt = {"bf16": torch.bfloat16, torch.bfloat16: torch.bfloat16, "fp8": FP8, FP8: FP8}[dtype]
        self.data = torch.zeros(layers, pages, kv_heads, 2, PAGE * HEAD_DIM, dtype=tdt, device=device)

    def layer(self, i: int) -> torch.Tensor:
        return self.data[i]

    @property
    def fp8(self) -> bool:
        return self.data.dtype == FP8

    @staticmethod
    def bytes_per_page(layers: int, kv_heads: int, dtype="bf16") -> int:
        return layers * kv_heads * 2 * PAGE * HEAD_DIM * (1 if dtype == "fp8" else 2)


def rope_cache_(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, positions: torch.Tensor,
                slots: torch.Tensor, cache_layer: torch.Tensor, heads: int, kv_heads: int,
                partials: torch.Tensor | None = None) -> torch.Tensor:
    """In place: rotate the q and k heads of every row of the fused ``qkv``
    ``[T, (H + 2 HKV) * 128]`` at ``positions[t]``, and write k, v into cache slot
    ``slots[t]`` (``page * 32 + offset``; < 0 skips the write).

    ``partials`` (fp32 ``[nslice, T, (H + 2 HKV) * 128]``, from
    ``kgs.ops.gemm.gemm_nt_w4x_partials``): the projection arrives as split-K
    partial products; they are reduced (bf16-rounded like the unfused reduce)
    in the same launch and ``qkv`` is output only."""
    t = qkv.shape[0]
    if qkv.dtype != torch.bfloat16 or not qkv.is_cuda or qkv.stride(1) != 1:
        raise ValueError("qkv must be a row-major bf16 GPU matrix")
    nslice = 0
    if partials is not None:
        if partials.dtype != torch.float32 or partials.dim() != 3 or not partials.is_contiguous() or \
                tuple(partials.shape[1:]) != (t, (heads + 2 * kv_heads) * HEAD_DIM):
            raise ValueError("partials must be contiguous fp32 [nslice, T, (H + 2 HKV) * 128]")
        nslice = partials.shape[0]
    for v, name in ((positions, "positions"), (slots, "slots")):
        if v.dtype != torch.int32 or not v.is_contiguous() or v.numel() != t:
            raise ValueError(f"{name} must be a contiguous int32 vector of length {t}")
    for v in (cos, sin):
        if v.dtype != torch.float32 or not v.is_contiguous() or v.shape[-1] != HEAD_DIM // 2:
            raise ValueError("cos/sin must be contiguous fp32 [max_pos, 64]")
    if cache_layer.dtype not in (torch.bfloat16, FP8) or not cache_layer.is_contiguous():
        raise ValueError("cache_layer must be a contiguous bf16 or e4m3 page array")
    rc = _lib.lib().kgs_rope_cache_bf16(qkv.data_ptr(), cos.data_ptr(), sin.data_ptr(), positions.data_ptr(),
                                        slots.data_ptr(), cache_layer.data_ptr(), t, heads, kv_heads, HEAD_DIM,
                                        qkv.stride(0), 1 if cache_layer.dtype == FP8 else 0,
                                        None if partials is None else partials.data_ptr(), nslice,
                                        _lib.stream_handle(qkv.device))
    _lib.check(rc, "rope_cache")
    return qkv


def decode_splits(batch: int, kv_heads: int, max_pages: int, cus: int = CUS, min_pages: int = 4) -> tuple[int, int]:
    """(pages_per_split, nsplit) for a block-table width of ``max_pages``.

    Split each context so that the grid holds about two waves per CU:
    ``nsplit = ceil(2 * CUs / (batch * kv_heads))``. Every split keeps at least
    ``min_pages`` pages (a one-page split is all launch and merge overhead: 52
    us for batch 1 x 4096 tokens with 1-page splits, profiles/decode_kernels.md).
    So batch 1-8 takes eight splits, batch 16 four and batch 32 two. From batch
    64 up, one split per (sequence, KV head) is fastest. It is paired with the
    two-page register pipeline, which the kernel runs for grids of up to 1024
    waves (``kgs_paged_decode_bf16``).

    Round-3 measurements (``profiles/r3/decode/paged_sweep_ctx*.log``, table
    width 64 pages):

    * 1024 cached tokens: batch 64 52 us (was 100 with the old rule of two
      splits and no pipeline); batch 128 92 us (was 124);
    * 528 tokens: batch 64 30 us (was 59), batch 128 50 us (was 72);
    * 2000 tokens: within 2 % of the best split everywhere.

    The old rule split large batches whenever the table held 64 pages or more;
    without the pipeline, each split paid one page latency per page."""
    groups = max(1, batch * kv_heads)
    want = max(1, math.ceil(2 * cus / groups))
    nsplit = max(1, min(math.ceil(max_pages / min_pages), want))
    pps = math.ceil(max_pages / nsplit)
    return pps, math.ceil(max_pages / pps)


_AWS: dict = {}


def _attn_workspace(b: int, heads: int, kv_heads: int, nsplit: int, device) -> tuple:
    """(po, pml, cnt) split-merge workspace of the paged decode attention
    (None x 3 for one split); grown on demand, one per device."""
    if nsplit <= 1:
        return None, None, None
    need = b * heads * nsplit
    key = device_key(device)
    po, pml, cnt = _AWS.get(key, (None, None, None))
    if po is None or po.numel() < need * HEAD_DIM or cnt.numel() < b * kv_heads:
        retire(po, pml, cnt)
        po = torch.empty(max(need, 1 << 14) * HEAD_DIM, dtype=torch.float32, device=device)
        pml = torch.empty(max(need, 1 << 14) * 2, dtype=torch.float32, device=device)
        cnt = torch.zeros(max(b * kv_heads, 4096), dtype=torch.int32, device=device)
        _AWS[key] = (po, pml, cnt)
    return po, pml, cnt


def rope_paged_decode_attention(partials: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                                positions: torch.Tensor, slots: torch.Tensor, cache_layer: torch.Tensor,
                                block_tables: torch.Tensor, ctx_lens: torch.Tensor, heads: int, kv_heads: int,
                                out: torch.Tensor | None = None, scale: float | None = None,
                                pages_per_split: int | None = None, pipe: bool | None = None) -> torch.Tensor:
    """:func:`rope_cache_` (partials form) and :func:`paged_decode_attention` in
    ONE launch (``kgs_paged_decode_rope_bf16``): ``partials`` fp32
    ``[nslice, B, (H + 2 HKV) * 128]`` from ``gemm_nt_w4x_partials`` of the
    fused qkv projection. Each attention wave reduces, rotates and caches its
    own (sequence, KV head) rows, so the rotated q never goes through memory
    and the rope_cache launch disappears. Same cache contents and output as the
    two launches. ``slots[b]`` must lie in the last page of ``ctx_lens[b]``
    (the engine's assignment)."""
    nh = heads + 2 * kv_heads
    if partials.dtype != torch.float32 or partials.dim() != 3 or not partials.is_contiguous() or \
            partials.shape[2] != nh * HEAD_DIM or not partials.is_cuda:
        raise ValueError("partials must be contiguous fp32 GPU [nslice, B, (H + 2 HKV) * 128]")
    b = partials.shape[1]
    if partials.shape[0] not in (2, 4, 8):
        raise ValueError("rope_paged_decode_attention: 2, 4 or 8 K slices (compile-time in the kernel)")
    if heads % kv_heads or heads // kv_heads > 6:
        raise ValueError("rope_paged_decode_attention: GQA group of at most 6 q heads per KV head")
    for v, name in ((positions, "positions"), (slots, "slots"), (ctx_lens, "ctx_lens")):
        if v.dtype != torch.int32 or not v.is_contiguous() or v.numel() != b:
            raise ValueError(f"{name} must be a contiguous int32 vector of length {b}")
    for v in (cos, sin):
        if v.dtype != torch.float32 or not v.is_contiguous() or v.shape[-1] != HEAD_DIM // 2:
            raise ValueError("cos/sin must be contiguous fp32 [max_pos, 64]")
    if cache_layer.dtype not in (torch.bfloat16, FP8) or not cache_layer.is_contiguous():
        raise ValueError("cache_layer must be a contiguous bf16 or e4m3 page array")
    if block_tables.dtype != torch.int32 or not block_tables.is_contiguous() or block_tables.shape[0] != b:
        raise ValueError("block_tables must be contiguous int32 [B, max_pages]")
    max_pages = block_tables.shape[1]
    if pages_per_split is None:
        pps, nsplit = decode_splits(b, kv_heads, max_pages)
    else:
        pps, nsplit = pages_per_split, math.ceil(max_pages / pages_per_split)
    if out is None:
        out = torch.empty((b, heads * HEAD_DIM), dtype=torch.bfloat16, device=partials.device)
    po, pml, cnt = _attn_workspace(b, heads, kv_heads, nsplit, partials.device)
    scale = 1.0 / math.sqrt(HEAD_DIM) if scale is None else scale
    rc = _lib.lib().kgs_paged_decode_rope_bf16(
        partials.data_ptr(), partials.shape[0], cos.data_ptr(), sin.data_ptr(), positions.data_ptr(),
        slots.data_ptr(), cache_layer.data_ptr(), block_tables.data_ptr(), ctx_lens.data_ptr(), out.data_ptr(),
        po.data_ptr() if po is not None else None, pml.data_ptr() if pml is not None else None,
        cnt.data_ptr() if cnt is not None else None, b, heads, kv_heads, HEAD_DIM, max_pages, pps, nsplit,
        out.stride(0), float(scale), 1 if cache_layer.dtype == FP8 else 0, -1 if pipe is None else int(bool(pipe)),
        _lib.stream_handle(partials.device))
    _lib.check(rc, "rope_paged_decode_attention")
    return out


def paged_decode_attention(q: torch.Tensor, cache_layer: torch.Tensor, block_tables: torch.Tensor,
                           ctx_lens: torch.Tensor, heads: int, kv_heads: int, out: torch.Tensor | None = None,
                           scale: float | None = None, pages_per_split: int | None = None,
                           pipe: bool | None = None) -> torch.Tensor:
    """One query token per sequence: ``q`` rows ``[B, >= H*128]`` (e.g. the rotated
    q heads at the front of the fused QKV rows), ``block_tables`` int32
    ``[B, max_pages]``, ``ctx_lens`` int32 ``[B]`` (cached tokens incl. the new
    one). Returns ``[B, H*128]`` bf16."""
    b = q.shape[0]
    if q.dtype != torch.bfloat16 or not q.is_cuda or q.stride(1) != 1:
        raise ValueError("q must be a row-major bf16 GPU matrix")
    if block_tables.dtype != torch.int32 or not block_tables.is_contiguous() or block_tables.shape[0] != b:
        raise ValueError("block_tables must be contiguous int32 [B, max_pages]")
    if ctx_lens.dtype != torch.int32 or not ctx_lens.is_contiguous() or ctx_lens.numel() != b:
        raise ValueError("ctx_lens must be contiguous int32 [B]")
    max_pages = block_tables.shape[1]
    if pages_per_split is None:
        pps, nsplit = decode_splits(b, kv_heads, max_pages)
    else:
        pps, nsplit = pages_per_split, math.ceil(max_pages / pages_per_split)
    if out is None:
        out = torch.empty((b, heads * HEAD_DIM), dtype=torch.bfloat16, device=q.device)
    po, pml, cnt = _attn_workspace(b, heads, kv_heads, nsplit, q.device)
    scale = 1.0 / math.sqrt(HEAD_DIM) if scale is None else scale
    rc = _lib.lib().kgs_paged_decode_bf16_ex(q.data_ptr(), cache_layer.data_ptr(), block_tables.data_ptr(),
                                             ctx_lens.data_ptr(), out.data_ptr(),
                                             po.data_ptr() if po is not None else None,
                                             pml.data_ptr() if pml is not None else None,
                                             cnt.data_ptr() if cnt is not None else None, b, heads, kv_heads, HEAD_DIM,
                                             max_pages, pps, nsplit, q.stride(0), out.stride(0), float(scale),
                                             1 if cache_layer.dtype == FP8 else 0,
                                             -1 if pipe is None else int(bool(pipe)), _lib.stream_handle(q.device))
    _lib.check(rc, "paged_decode_attention")
    return out


# ----------------------------------------------------------------------------
# plain-PyTorch references (fp32 math; CPU or GPU)

def ref_cache_write(cache_layer: torch.Tensor, k: torch.Tensor, v: torch.Tensor, slots: torch.Tensor) -> None:
    """Scatter ``k, v: [T, HKV, 128]`` into ``cache_layer [pages, HKV, 2, 4096]``."""
    k_idx, v_idx = kv_index_tables(cache_layer.device)
    keep = slots >= 0
    slots = slots[keep].long()
    k, v = k[keep], v[keep]
    page, tau = slots // PAGE, slots % PAGE
    hkv = cache_layer.shape[1]

    def cvt(t):
        if cache_layer.dtype == FP8:  # saturating, like the kernel
            return t.float().clamp(-FP8_MAX, FP8_MAX).to(FP8)
        return t.to(cache_layer.dtype)

    for h in range(hkv):
        cache_layer[page[:, None], h, 0, k_idx[tau]] = cvt(k[:, h])
        cache_layer[page[:, None], h, 1, v_idx[tau]] = cvt(v[:, h])


_KV_IDX: dict = {}


def gather_kv(cache_layer: torch.Tensor, pages: torch.Tensor, ctx: int, rows: int | None = None
              ) -> tuple[torch.Tensor, torch.Tensor]:
    """The first ``ctx`` cached tokens of one sequence as contiguous row-major
    ``k``, ``v`` ``[rows, kv_heads * 128]`` bf16 (rows ``ctx .. rows-1`` zero) --
    the keys/values a prefill chunk attends to (``rows`` pads them to the
    chunk's q-blocks). Vectorised torch gathers through the page layout's index
    tables; an fp8 cache is widened to bf16."""
    rows = ctx if rows is None else rows
    dev = cache_layer.device
    key = (dev.type, dev.index)
    if key not in _KV_IDX:
        _KV_IDX[key] = kv_index_tables(dev)
    k_idx, v_idx = _KV_IDX[key]
    hkv = cache_layer.shape[1]
    npg = (ctx + PAGE - 1) // PAGE
    sel = cache_layer[pages[:npg].long()]  # [npg, hkv, 2, 4096]
    out = []
    for region, idx in ((0, k_idx), (1, v_idx)):
        t = sel[:, :, region][..., idx]  # [npg, hkv, 32, 128]
        t = t.permute(0, 2, 1, 3).reshape(npg * PAGE, hkv * HEAD_DIM)[:ctx].to(torch.bfloat16)
        if rows > ctx:
            t = torch.cat([t, t.new_zeros(rows - ctx, hkv * HEAD_DIM)])
        out.append(t.contiguous())
    return out[0], out[1]


def ref_gather_kv(cache_layer: torch.Tensor, pages: torch.Tensor, ctx: int) -> tuple[torch.Tensor, torch.Tensor]:
    """The first ``ctx`` tokens of one sequence: ``(k, v)``, each ``[ctx, HKV, 128]`` fp32."""
    k_idx, v_idx = kv_index_tables(cache_layer.device)
    pos = torch.arange(ctx, device=cache_layer.device)
    page = pages.long()[pos // PAGE]
    tau = pos % PAGE
    hkv = cache_layer.shape[1]
    k = torch.stack([cache_layer[page[:, None], h, 0, k_idx[tau]] for h in range(hkv)], dim=1)
    v = torch.stack([cache_layer[page[:, None], h, 1, v_idx[tau]] for h in range(hkv)], dim=1)
    return k.float(), v.float()


def ref_paged_decode(q: torch.Tensor, cache_layer: torch.Tensor, block_tables: torch.Tensor, ctx_lens: torch.Tensor,
                     heads: int, kv_heads: int, scale: float | None = None) -> torch.Tensor:
    scale = 1.0 / math.sqrt(HEAD_DIM) if scale is None else scale
    rep = heads // kv_heads
    outs = []
    for i in range(q.shape[0]):
        ctx = int(ctx_lens[i])
        k, v = ref_gather_kv(cache_layer, block_tables[i], ctx)
        qi = q[i, :heads * HEAD_DIM].float().reshape(heads, HEAD_DIM)
        kk = k.repeat_interleave(rep, dim=1)  # [ctx, H, D]
        vv = v.repeat_interleave(rep, dim=1)
        s = torch.einsum("hd,thd->ht", qi, kk) * scale
        p = torch.softmax(s, dim=-1)
        outs.append(torch.einsum("ht,thd->hd", p, vv).reshape(-1))
    return torch.stack(outs)


def ref_rope_rows(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, positions: torch.Tensor,
                  heads: int) -> torch.Tensor:
    """Rotate-half RoPE of the first ``heads`` 128-wide heads of each row (fp32 result)."""
    t = x.shape[0]
    xf = x[:, :heads * HEAD_DIM].float().reshape(t, heads, HEAD_DIM)
    c, s = cos[positions.long()][:, None, :], sin[positions.long()][:, None, :]
    x1, x2 = xf[..., :HEAD_DIM // 2], xf[..., HEAD_DIM // 2:]
    return torch.cat((x1 * c - x2 * s, x2 * c + x1 * s), dim=-1).reshape(t, heads * HEAD_DIM)
