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


def test_kernel_dir_holds_only_production_sources():
    """``native/kernels/`` (the production library)
    holds only code the production library compiles: every header there is
    reached from a production ``.hip`` file, and nothing there includes an
    experiments-only header. Measured alternatives live in ``native/experiments/``."""
    import re
    from pathlib import Path

    kdir = Path(ROOT) / "native" / "kernels"
    inc = re.compile(r'#include\s+"([^"]+)"')
    reached, todo = set(), [p.name for p in kdir.glob("*.hip")]
    while todo:
        name = todo.pop()
        if name in reached:
            continue
        reached.add(name)
        for dep in inc.findall((kdir / name).read_text()):
            assert (kdir / dep).exists(), f"{name} includes {dep}, which is not in native/kernels"
            todo.append(dep)
    headers = {p.name for p in kdir.glob("*.h")}
    assert headers <= reached, sorted(headers - reached)
    gens = {p.name for p in kdir.glob("gen_*.py")}
    assert gens == {"gen_acc_regs.py"}, gens  # acc_regs.h's generator (the persistent GEMM's AGPR map)


def test_build_manifest_matches_the_tree():
    """Every build records what each library was built from
    (``kgs/_native/build_manifest.json``); right after a build the check finds
    every target's output and inputs unchanged, and the kernels record names
    the persistent GEMM's headers and the gfx950-only compile line."""
    import json

    from kgs.utils.build import MANIFEST, check_manifest

    res = check_manifest()
    assert res["ok"], res
    man = json.load(open(os.path.join(NATIVE, MANIFEST)))
    k = man["targets"]["kernels"]
    assert {"native/kernels/gemm_w4p.h", "native/kernels/tile_queue.h", "native/kernels/gemm_bf16.hip"} <= set(k["inputs"])
    assert "--offload-arch=gfx950" in k["compile"] and man["arch"] == "gfx950"


def test_manifest_check_names_a_stale_library(tmp_path):
    """A source edited after the build, and a library replaced after it, are
    both reported by target name."""
    from pathlib import Path

    from kgs.utils.build import CXX, Target, build_target, check_manifest, write_manifest

    src = tmp_path / "one.cpp"
    src.write_text("extern \"C\" int one() { return 1; }\n")
    t = Target("one", tmp_path / "libone.so", [src], CXX, flags=["-O2", "-fPIC"])
    assert build_target(t, jobs=1, objroot=tmp_path / "obj")
    write_manifest(tmp_path, [t], {"one": "built"})
    assert check_manifest(tmp_path) == {"ok": True, "targets": {"one": "ok"}}
    src.write_text("extern \"C\" int one() { return 2; }\n")
    r = check_manifest(tmp_path)
    assert not r["ok"] and "inputs changed" in r["targets"]["one"] and str(src) in r["targets"]["one"]
    Path(t.output).write_bytes(b"not the recorded library")
    assert check_manifest(tmp_path)["targets"]["one"] == "output differs from the recorded build"
