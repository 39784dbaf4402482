"""HIP/CDNA4 kernels exposed to PyTorch (gfx950 only).

* :func:`gemm_nt`, :func:`matmul`, :func:`linear`, :class:`Linear` -- bf16 MFMA GEMM
  (``native/kernels/gemm_bf16.hip``)
* :func:`vector_add`, :func:`transpose_bf16`, :func:`checksum` -- memory-bound
  helpers (``native/kernels/elementwise.hip``)
* :func:`add_rmsnorm`, :func:`rope_qkv_`, :func:`silu_mul`, :func:`attention_qkv` --
  fused decoder-block ops and flash attention (``native/kernels/transformer.hip``,
  ``native/kernels/attention.hip``)

Importing this package does not touch the GPU; the native library is loaded on
first use and raises :class:`NativeUnavailable` if it is missing.
"""
from ._lib import KernelError, NativeUnavailable, available  # noqa: F401


def __getattr__(name):  # lazy: keep `import kgs.ops` free of torch for CPU-only tools
    if name in ("gemm_nt", "matmul", "linear", "Linear", "fast_path_ok", "transpose", "EPI", "gemm_fp8_nt",
                "quantize_fp8", "gemm_bf16", "quantize_fp8_dev", "Fp8Linear", "gemm_fp8_rows"):
        from . import gemm

        return getattr(gemm, name)
    if name in ("add_rmsnorm", "rms_norm", "rope_qkv_", "rope_tables", "silu_mul", "attention_qkv",
                "add_rmsnorm_fp8", "silu_mul_fp8", "quantize_rows_fp8"):
        from . import transformer

        return getattr(transformer, name)
    if name in ("vector_add", "transpose_bf16", "checksum"):
        from . import elementwise

        return getattr(elementwise, name)
    raise AttributeError(name)
