"""Opt-in access to the measured GEMM alternatives (``libkgs_experiments.so``).

Production code never imports this module: ``kgs.ops.gemm_nt`` exposes only the
correct production kernels (auto / fast / generic / bounded). The kernels here
are the alternatives and timing probes behind ``profiles/gemm_tuning.md``
(source: ``native/experiments/gemm_experiments.hip``). Entries with
``probe=True`` compute a WRONG product by construction (they exist to time one
cost in isolation) and are only callable with ``allow_wrong=True``.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from functools import lru_cache
from pathlib import Path

import torch

from . import _lib
from .gemm import EPI, _check_operand

LIB_PATH = Path(os.environ.get("KGS_EXPERIMENTS_LIB", _lib.NATIVE_DIR / "libkgs_experiments.so"))


@dataclass(frozen=True)
class Experiment:
    id: int
    what: str
    probe: bool = False  # wrong result by construction (timing only)
    epilogue: bool = True  # supports the bias/activation epilogues


BF16 = {
    "w4_bk32": Experiment(3, "round-1 4-wave try: BK=32 4-deep ring, one barrier per 64 MFMAs"),
    "pp_prio": Experiment(4, "s_setprio around the MFMA blocks", epilogue=False),
    "pp_gm8": Experiment(5, "GROUP_M 8", epilogue=False),
    "pp_v0": Experiment(6, "first schedule (12/4/8/0 reads, look-ahead 5)", epilogue=False),
    "pp_gm2": Experiment(7, "GROUP_M 2", epilogue=False),
    "pp_gm16": Experiment(8, "GROUP_M 16", epilogue=False),
    "probe_2xmfma": Experiment(9, "every MFMA block doubled", probe=True, epilogue=False),
    "p32": Experiment(10, "32-MFMA phases, 160 KiB ring"),
    "probe_l2": Experiment(11, "all blocks load tile (0,0)", probe=True, epilogue=False),
    "lockstep": Experiment(12, "no ping-pong stagger", epilogue=False),
    "lockstep_1bar": Experiment(13, "lockstep, one barrier per phase", epilogue=False),
    "pl": Experiment(14, "lockstep with in-wave software pipelining"),
    "narrow_store": Experiment(15, "2 x 8-B store tail", epilogue=False),
    "persistent": Experiment(20, "persistent tile walk"),
    "vgpr_stage": Experiment(21, "VGPR staging, 4 phases in flight"),
    "vgpr_stage2": Experiment(22, "VGPR staging, 2 phases in flight"),
}
FP8 = {"gm8": 17, "gm16": 18, "gm2": 19, "gn4": 20, "gn8": 21, "gn2": 22}
# fp8 four-wave persistent kernel (gemm_w4f8.h, native/experiments/gemm_w4h.hip):
# w4f8_X_B1_R_P -> id 40..
_W4F8_CFG = ((0, 12, 24, 1), (0, 12, 12, 2), (0, 10, 12, 2), (0, 16, 24, 1), (0, 10, 24, 1), (0, 12, 20, 2),
             (8, 12, 24, 1), (140000000, 12, 24, 1), (0, 14, 12, 2), (0, 12, 8, 3), (0, 10, 8, 3), (0, 12, 6, 4))
W4F8 = {f"w4f8_{x}_{b1}_{r}_{p}": 40 + i for i, (x, b1, r, p) in enumerate(_W4F8_CFG)}
# gemm_w4h (native/experiments/gemm_w4h.hip): 4 waves x 128x128, two barriers
# per 128-MFMA K-step; name w4h_ORD_B1_R_P_X -> table id in gemm_w4h.hip (barrier 1 after MFMA B1, R
# MFMAs after barrier 2, P reads per MFMA there)
_W4H_CFG = ((1, 24, 20, 1, 0), (1, 24, 20, 1, 160000), (1, 24, 20, 1, 320000), (1, 24, 20, 1, 480000),
            (1, 20, 20, 1, 160000), (1, 20, 24, 1, 320000),
            # round 3: GROUP_M 2 / 8 / 16 / 32 with the production schedule
            (1, 24, 20, 1, 2), (1, 24, 20, 1, 8), (1, 24, 20, 1, 16), (1, 24, 20, 1, 32),
            # round 3: XCD-blocked tile maps (gemm_w4.h blocked_tile) MAP 1 / 2 / 3
            (1, 24, 20, 1, 10000000), (1, 24, 20, 1, 20000000), (1, 24, 20, 1, 30000000),
            # MAP 4: GROUP_N (the default map with M and N exchanged), G = 4 / 8 / 2
            (1, 24, 20, 1, 40000000), (1, 24, 20, 1, 40000008), (1, 24, 20, 1, 40000002),
            # DMA operand order (X / 10^8): B first / interleaved, with MAP 4 and with the default map
            (1, 24, 20, 1, 140000000), (1, 24, 20, 1, 240000000), (1, 24, 20, 1, 100000000),
            (1, 24, 20, 1, 200000000))
W4H = {f"w4h_{o}_{b}_{r}_{p}_{x}": i + 1 for i, (o, b, r, p, x) in enumerate(_W4H_CFG)}
# round 3: the persistent four-wave kernel (native/kernels/gemm_w4p.h, named accumulator AGPRs),
# name w4p_X -> id 101.. (X: gemm_w4.h knob bag: tile map, DMA operand order); K >= 384
_W4P_X = (0, 140000000, 8, 10000000, 140000008, 40000000, 100000000, 200000000, 140000002)
W4H.update({f"w4p_{x}": 101 + i for i, x in enumerate(_W4P_X)})
# the same with the static tile walk (no ticket queue): w4ps_X -> 121..
W4H.update({f"w4ps_{x}": 121 + i for i, x in enumerate((0, 140000000, 8, 140000008))})
# round 4: C stored non-temporally (gemm_w4p.h NTST): w4pn_X -> 131..
W4H.update({"w4pn_0": 131, "w4pn_140000008": 132, "w4pn_8": 133, "w4pn_140000000": 134})
# round 4: LDS layout 1 (gemm_w4p.h Lay<1>: rows DMA'd by consecutive lanes in address order,
# placed for conflict-free fragment reads): w4pl_X -> 135..
W4H.update({"w4pl_0": 135, "w4pl_140000008": 136, "w4pl_8": 137, "w4pl_140000000": 138})
# round 4: MFMA order inside a k-sub: i-major (w4po0_X) / n-major (w4po2_X) instead of the growing square
W4H.update({"w4po0_0": 139, "w4po2_0": 140, "w4po0_140000008": 141, "w4po2_140000008": 142})
# round 5: C store measurement builds (gemm_w4p.h (L / 100) % 10): C not written (w4px_0, output
# garbage) / s_waitcnt vmcnt(0) after each tile's stores (w4pd_0)
W4H.update({"w4px_0": 143, "w4pd_0": 144})
# ... and K-step 0 after an epilogue waiting vmcnt(ND + stores): w4pw_0
W4H.update({"w4pw_0": 145})
# round 6: deferred C stores (gemm_w4p.h DD, SPS): w4pq<DD>x<SPS>[n]_<X> (n: non-temporal stores) -> 146..
W4H.update({"w4pq8x2n_0": 146, "w4pq4x4n_0": 147, "w4pq8x1n_0": 148, "w4pq10x2n_0": 149, "w4pq16x1n_0": 150,
            "w4pq8x2_0": 151, "w4pq8x2_140000008": 152, "w4pq12x1n_0": 153, "w4pq8x2n_140000008": 154,
            "w4pq8x2n_8": 155, "w4pq1x16n_0": 156, "w4pq2x8n_0": 157, "w4pq3x6n_0": 158, "w4pq2x10n_0": 159,
            "w4pq4x5n_0": 160, "w4pq4x4_140000008": 161, "w4pq4x4n_140000008": 162, "w4pq4x4_0": 163,
            "w4pq4x4_8": 164, "w4pq2x8_140000008": 165, "w4pq2x8_0": 166})
# round 6: one barrier per K-step (gemm_w4p.h OB), DMA window W MFMAs: w4pb[w<W>][q<DD>x<SPS>][t]_<X>
# (nt C stores unless t) -> 167..
W4H.update({"w4pb_0": 167, "w4pbw48_0": 168, "w4pbw32_0": 169, "w4pbq4x4_0": 170, "w4pbt_140000008": 171,
            "w4pbt_8": 172, "w4pbt_0": 173, "w4pbw64_0": 174})
# round 6: K-step schedule (gemm_w4p.h (L / 10^7) % 10): w4pk<B1>r<R>[q4x4n]_<X> -> 175..
W4H.update({"w4pk20r20q4x4n_0": 175, "w4pk24r16q4x4n_0": 176, "w4pk20r16q4x4n_0": 177, "w4pk18r16q4x4n_0": 178,
            "w4pk24r16_140000008": 179, "w4pk20r16_140000008": 180, "w4pk20r24q4x4n_0": 181,
            "w4pk18r24q4x4n_0": 182, "w4pk24r24q4x4n_0": 183, "w4pk20r24_140000008": 184})
NO_OUTPUT = frozenset({"w4px_0"})  # timing only: C is not written


@lru_cache(maxsize=1)
def lib() -> ctypes.CDLL:
    _lib.lib()  # torch's HIP runtime first, then the production library (shared runtime)
    if not LIB_PATH.exists():
        raise _lib.NativeUnavailable(f"{LIB_PATH} is missing: `python -m kgs.utils.build --only experiments`")
    so = ctypes.CDLL(str(LIB_PATH))
    vp, i = ctypes.c_void_p, ctypes.c_int
    so.kgs_exp_gemm_bf16_nt.argtypes = [vp] * 4 + [i] * 8 + [vp]
    so.kgs_exp_gemm_bf16_nt.restype = i
    so.kgs_exp_gemm_fp8_nt.argtypes = [vp] * 3 + [i] * 6 + [ctypes.c_float, i, vp]
    so.kgs_exp_gemm_fp8_nt.restype = i
    so.kgs_gemm_bf16_nt_stamps.argtypes = [vp] * 3 + [i] * 6 + [vp] * 2
    so.kgs_gemm_bf16_nt_stamps.restype = i
    so.kgs_gemm_stamp_n.restype = i
    so.kgs_exp_gemm_w4h.argtypes = [vp] * 3 + [i] * 7 + [vp]
    so.kgs_exp_gemm_w4h.restype = i
    so.kgs_exp_gemm_w4p_grid.argtypes = [vp] * 3 + [i] * 8 + [vp]
    so.kgs_exp_gemm_w4p_grid.restype = i
    L = ctypes.c_long
    so.kgs_exp_attn4_fwd_bf16.argtypes = [vp] * 4 + [i] * 6 + [L] * 4 + [ctypes.c_float, i, vp, i, vp]
    so.kgs_exp_attn4_fwd_bf16.restype = i
    so.kgs_exp_gemm_w4p_stamps.argtypes = [vp] * 3 + [i] * 7 + [vp] * 3
    so.kgs_exp_gemm_w4p_stamps.restype = i
    so.kgs_exp_gemm_w4p_waits.argtypes = [vp] * 3 + [i] * 7 + [vp] * 3
    so.kgs_exp_gemm_w4p_waits.restype = i
    so.kgs_exp_gemm_fp8_w4f8.argtypes = [vp] * 3 + [i] * 6 + [ctypes.c_float, i, vp]
    so.kgs_exp_gemm_fp8_w4f8.restype = i
    return so


def gemm_nt(a: torch.Tensor, b: torch.Tensor, variant: str, bias: torch.Tensor | None = None,
            act: str | None = None, out: torch.Tensor | None = None, allow_wrong: bool = False) -> torch.Tensor:
    """``act(a @ b.T + bias)`` on experimental kernel ``variant`` (aligned shapes only)."""
    if variant in W4H:
        if bias is not None or act is not None:
            raise ValueError("w4h variants have no epilogue")
        _check_operand(a, "a")
        _check_operand(b, "b")
        M, K = a.shape
        N = b.shape[0]
        if out is None:
            out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
        rc = lib().kgs_exp_gemm_w4h(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                                    out.stride(0), W4H[variant], _lib.stream_handle(a.device))
        _lib.check(rc, f"experiment {variant}[{M}x{N}x{K}]")
        return out
    ex = BF16[variant]
    if ex.probe and not allow_wrong:
        raise ValueError(f"{variant} is a timing probe with a wrong result; pass allow_wrong=True")
    _check_operand(a, "a")
    _check_operand(b, "b")
    M, K = a.shape
    N = b.shape[0]
    epi_name = act if act is not None else ("bias" if bias is not None else None)
    epi = EPI[epi_name]
    if epi and not ex.epilogue:
        raise ValueError(f"{variant} has no epilogue variant")
    if epi and bias is None:
        bias = torch.zeros(N, dtype=torch.bfloat16, device=a.device)
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    rc = lib().kgs_exp_gemm_bf16_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                    bias.data_ptr() if bias is not None else None, M, N, K, a.stride(0),
                                    b.stride(0), out.stride(0), epi, ex.id, _lib.stream_handle(a.device))
    _lib.check(rc, f"experiment {variant}[{M}x{N}x{K}]")
    return out


def gemm_fp8_nt(a: torch.Tensor, b: torch.Tensor, scale_a: float, scale_b: float, variant: str,
                out: torch.Tensor | None = None) -> torch.Tensor:
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if variant in W4F8:
        rc = lib().kgs_exp_gemm_fp8_w4f8(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                                         b.stride(0), out.stride(0), float(scale_a) * float(scale_b), W4F8[variant],
                                         _lib.stream_handle(a.device))
        _lib.check(rc, f"fp8 experiment {variant}[{M}x{N}x{K}]")
        return out
    rc = lib().kgs_exp_gemm_fp8_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                                   out.stride(0), float(scale_a) * float(scale_b), FP8[variant],
                                   _lib.stream_handle(a.device))
    _lib.check(rc, f"fp8 experiment {variant}[{M}x{N}x{K}]")
    return out


def gemm_w4p_grid(a, b, out, mode: int = 1, grid: int = 0) -> None:
    """The persistent GEMM (default map) with first-ticket ``mode`` (1 = static,
    2 = from the queue) on ``grid`` workgroups (0 = one per CU), on the current
    stream. ``a`` [M, K], ``b`` [N, K], ``out`` [M, N], bf16 row-major."""
    M, K = a.shape
    N = b.shape[0]
    _lib.check(lib().kgs_exp_gemm_w4p_grid(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                                           b.stride(0), out.stride(0), int(mode), int(grid),
                                           _lib.stream_handle(a.device)), "kgs_exp_gemm_w4p_grid")


# tile maps of the timing build (gemm_w4h.hip kgs_exp_gemm_w4p_stamps)
STAMP_MAPS = {"default": 0, "mirror_g8": 1, "g8": 2, "mirror": 3, "blk1": 4, "blk2": 5, "blk3": 6}


def production_map(M: int, N: int, K: int) -> str:
    """The tile map gemm_persistent.hip's launcher uses for an aligned problem."""
    tall, longk = M > N, K > 8192
    return "mirror_g8" if tall and longk else "mirror" if tall else "g8" if longk else "default"


def gemm_w4p_stamps(a, b, out, stamps: torch.Tensor, map_: int | str = 0) -> int:
    """The persistent GEMM's timing build (gemm_w4p.h TS) on the current
    stream: ``stamps`` is an int64 [>= grid, 16] device tensor that receives
    per-workgroup start / per-tile end stamps (s_memrealtime, 100 MHz), HW_ID
    and XCC_ID. ``map_``: a STAMP_MAPS name or id. Returns the grid."""
    if isinstance(map_, str):
        map_ = STAMP_MAPS[map_]
    M, K = a.shape
    N = b.shape[0]
    if stamps.dtype != torch.int64 or stamps.dim() != 2 or stamps.shape[1] != 16 or not stamps.is_contiguous():
        raise ValueError("stamps must be a contiguous int64 [grid, 16] tensor")
    grid = ctypes.c_int(0)
    tiles = (M // 256) * (N // 256)
    if stamps.shape[0] < min(tiles, torch.cuda.get_device_properties(a.device).multi_processor_count):
        raise ValueError("stamps has fewer rows than the grid")
    _lib.check(lib().kgs_exp_gemm_w4p_stamps(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                                             b.stride(0), out.stride(0), int(map_), stamps.data_ptr(),
                                             ctypes.byref(grid), _lib.stream_handle(a.device)),
               "kgs_exp_gemm_w4p_stamps")
    return grid.value


def attention_qkv_w4(qkv: torch.Tensor, batch: int, seq: int, heads: int, kv_heads: int, head_dim: int = 128,
                     causal: bool = True, scale: float | None = None, out: torch.Tensor | None = None,
                     stamps: torch.Tensor | None = None) -> torch.Tensor:
    """:func:`kgs.ops.transformer.attention_qkv` on the one-wave-per-SIMD,
    named-register kernel (native/experiments/attention_w4.h; ``seq % 256 == 0``).
    ``stamps``: an int64 [64, 4, 64, 8] tensor selects the timing build (per
    workgroup < 64, wave and tile: s_memtime at the tile start and after each
    section)."""
    if stamps is not None and (stamps.dtype != torch.int64 or stamps.numel() < 64 * 4 * 64 * 8):
        raise ValueError("stamps must be an int64 tensor of 64 * 4 * 64 * 8 elements")
    import math

    if qkv.dtype != torch.bfloat16 or not qkv.is_cuda or qkv.stride(1) != 1:
        raise ValueError("qkv must be a row-major bf16 GPU tensor")
    if qkv.shape[0] != batch * seq or qkv.shape[1] < (heads + 2 * kv_heads) * head_dim:
        raise ValueError("qkv shape does not match batch/seq/heads")
    out = torch.empty((batch * seq, heads * head_dim), dtype=torch.bfloat16, device=qkv.device) \
        if out is None else out
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    ld, esz, base = qkv.stride(0), qkv.element_size(), qkv.data_ptr()
    rc = lib().kgs_exp_attn4_fwd_bf16(base, base + heads * head_dim * esz, base + (heads + kv_heads) * head_dim * esz,
                                      out.data_ptr(), batch, seq, seq, heads, kv_heads, head_dim, ld, ld, ld,
                                      out.stride(0), float(scale), 1 if causal else 0,
                                      stamps.data_ptr() if stamps is not None else None, 0,
                                      _lib.stream_handle(qkv.device))
    _lib.check(rc, "attention_qkv_w4")
    return out


def gemm_w4p_waits(a, b, out, stamps: torch.Tensor, variant: int = 0) -> int:
    """The persistent GEMM's wait-stamp build (gemm_w4p.h WSB): computes ``a @ b.T`` into ``out`` and
    fills ``stamps`` (int64 ``[>= grid, 4, 16]``, per wave: s_memtime cycles of [category][lgkm wait,
    barrier 1, vm wait, barrier 2] for category 0 = a tile's K-steps 0-1, 1 = the steady loop, 2 = the
    last two, then start, end, tiles). Variant: 0 production nt + deferred 4 x 4, 1 nt only, 2 tall
    long-K map, 3 map 0 temporal C. Returns the grid."""
    import ctypes

    M, K = a.shape
    N = b.shape[0]
    if stamps.dtype != torch.int64 or not stamps.is_contiguous() or stamps.dim() != 3 or tuple(stamps.shape[1:]) != (4, 16):
        raise ValueError("stamps: contiguous int64 [grid, 4, 16]")
    cus = torch.cuda.get_device_properties(a.device).multi_processor_count
    if stamps.shape[0] < min((M // 256) * (N // 256), cus):
        raise ValueError("stamps: fewer rows than the persistent grid")
    g = ctypes.c_int(0)
    _lib.check(lib().kgs_exp_gemm_w4p_waits(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                                            b.stride(0), out.stride(0), int(variant), stamps.data_ptr(),
                                            ctypes.byref(g), _lib.stream_handle(a.device)), "kgs_exp_gemm_w4p_waits")
    return g.value
