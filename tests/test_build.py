"""The native build: every HIP object is gfx950-only and exports the C ABI."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "kgs", "_native")
KLIB = os.path.join(NATIVE, "libkgs_kernels.so")


@pytest.fixture(scope="module", autouse=True)
def built():
    from kgs.utils.build import build_all

    build_all(verbose=False)


def test_kernel_library_exports():
    out = subprocess.run(["nm", "-D", "--defined-only", KLIB], capture_output=True, text=True, check=True).stdout
    for sym in ("kgs_gemm_bf16_nt", "kgs_gemm_bf16_nt_fast_ok", "kgs_vector_add_f32", "kgs_vector_add_bf16",
                "kgs_transpose_bf16", "kgs_checksum_bf16"):
        assert sym in out, sym


def test_code_objects_are_gfx950_only():
    data = open(KLIB, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"gfx1100", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in data


def test_incremental_build_is_noop():
    from kgs.utils.build import build_all

    st = build_all(verbose=False)
    assert all(v in ("fresh",) or v.startswith("skipped") for v in st.values()), st


def test_graft_entry_build_imports():
    import __graft_entry__

    __graft_entry__.build()
