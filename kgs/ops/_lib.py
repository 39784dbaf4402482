"""ctypes binding to ``kgs/_native/libkgs_kernels.so`` (the gfx950 HIP kernels).

The library exports a plain C ABI (see ``native/kernels/*.hip``): raw device
pointers, sizes and a ``hipStream_t``. Torch is imported first so that the
library's ``libamdhip64.so.7`` dependency resolves (by SONAME) to the HIP runtime
torch already loaded -- one HIP runtime per process, shared streams.

There is deliberately no silent fallback: on a machine with a GPU, a missing or
unloadable library raises ``NativeUnavailable`` (the driver checks that the
native code is what runs).
"""
from __future__ import annotations

import ctypes
import os
from functools import lru_cache
from pathlib import Path

NATIVE_DIR = Path(__file__).resolve().parents[1] / "_native"
LIB_PATH = Path(os.environ.get("KGS_KERNELS_LIB", NATIVE_DIR / "libkgs_kernels.so"))


class NativeUnavailable(RuntimeError):
    pass


class KernelError(RuntimeError):
    pass


_ERRS = {-1: "bad shape", -2: "bad alignment / not eligible for this variant", -3: "bad argument"}

_c_void_p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_long = ctypes.c_long

_SIGS = {
    "kgs_gemm_bf16_nt": ([_c_void_p, _c_void_p, _c_void_p, _c_void_p] + [_c_int] * 8 + [_c_void_p], _c_int),
    "kgs_gemm_bf16_nt_addc": ([_c_void_p, _c_void_p, _c_void_p] + [_c_int] * 6 + [_c_void_p], _c_int),
    "kgs_tile_queue_stats": ([_c_int, ctypes.POINTER(_c_long)], _c_int),
    "kgs_tile_queue_check": ([_c_int, ctypes.POINTER(_c_long)], _c_int),
    "kgs_tile_queue_slot": ([_c_void_p, ctypes.POINTER(_c_void_p)], _c_int),
    "kgs_gemm_bf16_nt_fast_ok": ([_c_void_p, _c_void_p, _c_void_p] + [_c_int] * 6, _c_int),
    "kgs_gemm_bf16_nt_bounded_ok": ([_c_void_p, _c_void_p, _c_void_p] + [_c_int] * 6, _c_int),
    "kgs_gemm_bf16_nt_w4_ok": ([_c_void_p, _c_void_p, _c_void_p] + [_c_int] * 6, _c_int),
    "kgs_gemm_bf16_nt_splitk": ([_c_void_p] * 4 + [_c_int] * 7 + [_c_void_p], _c_int),
    "kgs_gemm_bf16_nt_w4x": ([_c_void_p] * 4 + [_c_int] * 9 + [_c_void_p], _c_int),
    "kgs_gemm_bf16_nt_w4x_ex": ([_c_void_p] * 4 + [_c_int] * 10 + [_c_void_p], _c_int),
    "kgs_gemm_fp8_nt": ([_c_void_p, _c_void_p, _c_void_p, _c_void_p] + [_c_int] * 6 + [ctypes.c_float, _c_int, _c_int,
                                                                                     _c_void_p], _c_int),
    "kgs_gemm_fp8_nt_ok": ([_c_void_p, _c_void_p, _c_void_p] + [_c_int] * 7, _c_int),
    "kgs_gemm_fp8_nt_dev": ([_c_void_p, _c_void_p, _c_void_p, _c_void_p] + [_c_int] * 6 +
                            [ctypes.c_float, _c_void_p, _c_int, _c_int, _c_void_p], _c_int),
    "kgs_quantize_fp8": ([_c_void_p, _c_long, _c_int, _c_void_p, _c_void_p, _c_void_p], _c_int),
    "kgs_gemm_bf16": ([_c_void_p, _c_void_p, _c_void_p, _c_void_p] + [_c_int] * 9 + [_c_void_p], _c_int),
    "kgs_gemm_bf16_layout_ok": ([_c_void_p, _c_void_p, _c_void_p] + [_c_int] * 8, _c_int),
    "kgs_vector_add_f32": ([_c_void_p, _c_void_p, _c_void_p, _c_long, _c_void_p], _c_int),
    "kgs_cu_hold": ([_c_int, ctypes.c_double, _c_int, _c_void_p], _c_int),
    "kgs_comm_standin_f32": ([_c_void_p, _c_void_p, _c_long, _c_int, _c_int, _c_int, _c_void_p], _c_int),
    "kgs_vector_add_bf16": ([_c_void_p, _c_void_p, _c_void_p, _c_long, _c_void_p], _c_int),
    "kgs_transpose_bf16": ([_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p], _c_int),
    "kgs_transpose_bf16_v": ([_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_void_p], _c_int),
    "kgs_vector_add_f32_v": ([_c_void_p, _c_void_p, _c_void_p, _c_long, _c_int, _c_void_p], _c_int),
    "kgs_vector_add_bf16_v": ([_c_void_p, _c_void_p, _c_void_p, _c_long, _c_int, _c_void_p], _c_int),
    "kgs_checksum_bf16": ([_c_void_p, _c_long, _c_void_p, _c_void_p], _c_int),
    # fused decoder-block ops (native/kernels/transformer.hip, attention.hip)
    "kgs_add_rmsnorm_bf16": ([_c_void_p] * 5 + [_c_int, _c_int, _c_long, _c_long, ctypes.c_float, _c_void_p], _c_int),
    "kgs_rope_qkv_bf16": ([_c_void_p] * 4 + [_c_long, _c_int, _c_int, _c_long, _c_int, _c_void_p], _c_int),
    "kgs_silu_mul_bf16": ([_c_void_p, _c_void_p, _c_long, _c_int, _c_long, _c_long, _c_void_p], _c_int),
    "kgs_add_rmsnorm_fp8": ([_c_void_p] * 6 + [_c_int, _c_int, _c_long, _c_long, ctypes.c_float, _c_void_p], _c_int),
    "kgs_quant_rows_fp8": ([_c_void_p] * 3 + [_c_int, _c_int, _c_long, _c_long, _c_void_p], _c_int),
    "kgs_silu_mul_fp8": ([_c_void_p] * 3 + [_c_long, _c_int, _c_long, _c_long, _c_void_p], _c_int),
    "kgs_gemm_fp8_nt_rows": ([_c_void_p, _c_void_p, _c_void_p, _c_void_p] + [_c_int] * 6 +
                             [ctypes.c_float, _c_void_p, _c_int, _c_int, _c_void_p], _c_int),
    "kgs_attn_fwd_bf16_ex": ([_c_void_p] * 4 + [_c_int] * 6 + [_c_long] * 4 + [ctypes.c_float, _c_int, _c_void_p],
                             _c_int),
    "kgs_attn_fwd_bf16": ([_c_void_p] * 4 + [_c_int] * 5 + [_c_long] * 4 + [ctypes.c_float, _c_int, _c_void_p],
                          _c_int),
    # decode path (native/kernels/decode.hip)
    "kgs_skinny_geometry": ([_c_int, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int), ctypes.POINTER(_c_int)], _c_int),
    "kgs_skinny_gemm_bf16": ([_c_void_p] * 5 + [_c_int] * 3 + [_c_long, _c_long, _c_int, _c_void_p], _c_int),
    "kgs_skinny_gemm_bf16_v": ([_c_void_p] * 5 + [_c_int] * 3 + [_c_long, _c_long, _c_int, _c_int, _c_void_p], _c_int),
    "kgs_skinny_gemm_bf16_ex": ([_c_void_p] * 5 + [_c_int] * 3 + [_c_long, _c_long] + [_c_int] * 3 + [_c_void_p],
                                _c_int),
    "kgs_skinny_gemm_bf16_fused": ([_c_void_p] * 5 + [_c_int] * 3 + [_c_long, _c_long] + [_c_int] * 3 +
                                   [_c_void_p] * 3 + [ctypes.c_float, ctypes.c_float, _c_void_p, _c_void_p], _c_int),
    "kgs_skinny_variant_geometry": ([_c_int, _c_int] + [ctypes.POINTER(_c_int)] * 3, _c_int),
    "kgs_rope_cache_bf16": ([_c_void_p] * 6 + [_c_long, _c_int, _c_int, _c_int, _c_long, _c_int, _c_void_p, _c_int,
                                                  _c_void_p], _c_int),
    "kgs_gemm_bf16_nt_w4x_swiglu": ([_c_void_p] * 3 + [_c_int] * 8 + [_c_void_p], _c_int),
    "kgs_gemm_bf16_nt_w4x_swiglu_ex": ([_c_void_p] * 3 + [_c_int] * 9 + [_c_void_p], _c_int),
    "kgs_skinny_gemm_bf16_rope": ([_c_void_p] * 5 + [_c_int] * 3 + [_c_long, _c_long] + [_c_int] * 3 +
                                  [_c_void_p, ctypes.c_float, ctypes.c_float] + [_c_void_p] * 5 + [_c_int, _c_int,
                                                                                                  _c_void_p], _c_int),
    "kgs_argmax_rows_bf16": ([_c_void_p, _c_void_p, _c_int, _c_int, _c_long, _c_void_p], _c_int),
    "kgs_splitk_add_rmsnorm_bf16": ([_c_void_p, _c_int] + [_c_void_p] * 3 + [_c_int, _c_int, _c_long, _c_long,
                                                                              ctypes.c_float, _c_void_p], _c_int),
    "kgs_paged_decode_bf16": ([_c_void_p] * 8 + [_c_int] * 7 + [_c_long, _c_long, ctypes.c_float, _c_int, _c_void_p],
                              _c_int),
    "kgs_splitk_reduce_swiglu_bf16": ([_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p], _c_int),
    "kgs_paged_decode_bf16_ex": ([_c_void_p] * 8 + [_c_int] * 7 + [_c_long, _c_long, ctypes.c_float, _c_int, _c_int,
                                                                   _c_void_p], _c_int),
    "kgs_paged_decode_rope_bf16": ([_c_void_p, _c_int] + [_c_void_p] * 11 + [_c_int] * 7 +
                                   [_c_long, ctypes.c_float, _c_int, _c_int, _c_void_p], _c_int),
    # peer-to-peer all-reduce (native/kernels/allreduce_p2p.hip)
    "kgs_ar_signal_bytes": ([], _c_int),
    "kgs_ar_max_blocks": ([], _c_int),
    "kgs_ar_max_ranks": ([], _c_int),
    "kgs_ar_ipc_handle_bytes": ([], _c_int),
    "kgs_ar_alloc": ([ctypes.c_size_t, _c_int, ctypes.POINTER(_c_void_p)], _c_int),
    "kgs_ar_free": ([_c_void_p], _c_int),
    "kgs_ar_ipc_handle": ([_c_void_p, ctypes.c_char_p], _c_int),
    "kgs_ar_ipc_open": ([ctypes.c_char_p, ctypes.POINTER(_c_void_p)], _c_int),
    "kgs_ar_ipc_close": ([_c_void_p], _c_int),
    "kgs_ar_run": ([ctypes.POINTER(_c_void_p), ctypes.POINTER(_c_void_p), _c_int, _c_int, _c_void_p, _c_void_p,
                    _c_long, _c_long, _c_int, _c_int, ctypes.c_uint, _c_int, ctypes.c_double, _c_void_p, _c_void_p],
                   _c_int),
}


@lru_cache(maxsize=1)
def lib() -> ctypes.CDLL:
    import torch  # noqa: F401  -- must precede the load (shared HIP runtime)

    if not LIB_PATH.exists():
        raise NativeUnavailable(
            f"{LIB_PATH} is missing: build it with `python -m kgs.utils.build` (hipcc --offload-arch=gfx950)"
        )
    try:
        so = ctypes.CDLL(str(LIB_PATH))
    except OSError as e:  # pragma: no cover - depends on the box
        raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, (args, res) in _SIGS.items():
        fn = getattr(so, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
    return so


def available() -> bool:
    try:
        lib()
        return True
    except NativeUnavailable:
        return False


def check(rc: int, what: str) -> None:
    if rc == 0:
        return
    if rc < 0:
        raise KernelError(f"{what}: {_ERRS.get(rc, rc)}")
    raise KernelError(f"{what}: hipError_t {rc}")


def stream_handle(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def tile_queue_stats(device: int = 0) -> dict:
    """The persistent GEMMs' ticket-slot pool on ``device`` (tile_queue.h):
    slots allocated, owned by streams, owned by captured launches, and the
    launches that found no slot (they ran the one-shot grid)."""
    out = (_c_long * 5)()
    check(lib().kgs_tile_queue_stats(int(device), out), "kgs_tile_queue_stats")
    return {"slots": out[0], "stream_slots": out[1], "capture_slots": out[2], "fallbacks": out[3],
            "grow_failures": out[4]}


def tile_queue_check(device: int = 0) -> dict:
    """The ticket-slot pool's quiescent invariant (tile_queue.h): with no
    persistent GEMM in flight every word of every slot is zero. Synchronises
    the device first. ``dirty_slots`` > 0 means a launch left its tickets
    behind or something wrote into the pool (the next eager launch on that
    slot would take wrong tickets); ``slot_addr`` / ``words`` are the first
    dirty slot's device address and its 16 words. ``error_slots``: slots whose
    error word a persistent GEMM set when it read a ticket no launch could
    have issued (it stopped taking tiles: that launch's output is incomplete)."""
    import torch

    torch.cuda.synchronize(device)
    out = (_c_long * 22)()
    check(lib().kgs_tile_queue_check(int(device), out), "kgs_tile_queue_check")
    r = {"dirty_slots": out[0], "dirty_words": out[1], "first_value": out[2], "first_word": out[3],
         "error_slots": out[21]}
    if out[0]:
        r["slot_addr"] = hex(out[4])
        r["words"] = [f"{w & 0xffffffff:08x}" for w in out[5:21]]
    return r


def neighbours(addr: int, device: int = 0, span: int = 256 << 20) -> list:
    """The caching allocator's segments (and their last active blocks) within
    ``span`` bytes of a device address: what sits next to a corrupted word."""
    import torch

    out = []
    for seg in torch.cuda.memory_snapshot():
        if seg.get("device", 0) != device:
            continue
        lo, size = seg["address"], seg["total_size"]
        if lo - span <= addr <= lo + size + span:
            blocks = [(hex(b["address"]), b["size"], b["state"]) for b in seg.get("blocks", [])
                      if b["state"] == "active_allocated"]
            out.append({"segment": hex(lo), "end": hex(lo + size), "bytes_to_addr": addr - (lo + size),
                        "pool": seg.get("segment_pool_id"), "stream": seg.get("stream"), "blocks": blocks[-4:]})
    return sorted(out, key=lambda d: abs(d["bytes_to_addr"]))[:6]
