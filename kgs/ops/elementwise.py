"""Memory-bound HIP ops: vector add (config-2 smoke), transpose, checksum."""
from __future__ import annotations

import torch

from . import _lib


def _dev_check(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda:
            raise ValueError("tensor must be on a GPU")
        if not t.is_contiguous():
            raise ValueError("tensor must be contiguous")


def vector_add(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, variant: int = 0) -> torch.Tensor:
    """``a + b`` elementwise (f32 or bf16) on the HIP vector-add kernel.

    variant selects a streaming configuration (0 = default; 1-6 are the measured
    alternatives in native/kernels/elementwise.hip)."""
    _dev_check(a, b)
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError("a and b must match in shape and dtype")
    out = torch.empty_like(a) if out is None else out
    _dev_check(out)
    n = a.numel()
    if a.dtype == torch.float32:
        fn = _lib.lib().kgs_vector_add_f32_v
    elif a.dtype == torch.bfloat16:
        fn = _lib.lib().kgs_vector_add_bf16_v
    else:
        raise TypeError(f"unsupported dtype {a.dtype}")
    _lib.check(fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), n, variant, _lib.stream_handle(a.device)),
               "vector_add")
    return out


def comm_standin(dst: torch.Tensor, src: torch.Tensor, blocks: int = 32, passes: int = 1,
                 lds_kb: int = 0) -> torch.Tensor:
    """``dst += src`` (f32) on a fixed number of workgroups, ``passes`` times: the
    footprint of a ring collective's kernel (a few tens of long-lived,
    memory-bound workgroups) on one GPU, for GEMM/comm overlap measurements.
    ``lds_kb`` > 32 reserves enough LDS that a workgroup needs a CU of its own
    (cannot share one with a 128 KiB GEMM workgroup)."""
    _dev_check(dst, src)
    if dst.dtype != torch.float32 or src.dtype != torch.float32 or dst.shape != src.shape:
        raise ValueError("comm_standin needs two f32 tensors of one shape")
    _lib.check(_lib.lib().kgs_comm_standin_f32(dst.data_ptr(), src.data_ptr(), dst.numel(), int(blocks), int(passes),
                                               int(lds_kb) * 1024, _lib.stream_handle(dst.device)), "comm_standin")
    return dst


def cu_hold(blocks: int, usec: float, lds_kb: int = 64, device=None) -> None:
    """A collective's CU footprint by time: ``blocks`` workgroups (RCCL
    channels), each holding a CU for ``usec`` microseconds from when it starts,
    on the current stream. ``lds_kb`` > 32: no 128 KiB GEMM workgroup fits on
    the same CU (bench/overlap_rccl.py)."""
    _lib.check(_lib.lib().kgs_cu_hold(int(blocks), float(usec), int(lds_kb) * 1024, _lib.stream_handle(device)),
               "cu_hold")


def transpose_bf16(x: torch.Tensor, variant: int = 0) -> torch.Tensor:
    """Materialised ``x.T`` (variant 0 = auto: 16-B path when shapes allow,
    1 = element-wise tile, 2 = force the 16-B path)."""
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("transpose_bf16 needs a row-major bf16 matrix")
    if not x.is_cuda:
        raise ValueError("tensor must be on a GPU")
    rows, cols = x.shape
    out = torch.empty((cols, rows), dtype=torch.bfloat16, device=x.device)
    rc = _lib.lib().kgs_transpose_bf16_v(x.data_ptr(), out.data_ptr(), rows, cols, x.stride(0), rows, variant,
                                         _lib.stream_handle(x.device))
    _lib.check(rc, "transpose_bf16")
    return out


def checksum(x: torch.Tensor) -> torch.Tensor:
    """Device-side (sum, sum|x|) of a bf16 tensor as a 2-element f32 tensor."""
    _dev_check(x)
    if x.dtype != torch.bfloat16 or x.numel() % 8:
        raise ValueError("checksum needs bf16 with numel % 8 == 0")
    out = torch.zeros(2, dtype=torch.float32, device=x.device)
    _lib.check(
        _lib.lib().kgs_checksum_bf16(x.data_ptr(), x.numel(), out.data_ptr(), _lib.stream_handle(x.device)),
        "checksum",
    )
    return out
