#!/usr/bin/env python3
"""Per-kernel instruction diff of one kernel source between two trees.

Compiles ``native/kernels/<src>`` of this tree and of another git revision
(a temporary ``git worktree``) for gfx950 with ``-save-temps`` and compares the
instruction stream of every kernel, with basic-block labels normalised (adding a
kernel renumbers the labels of the ones after it). Answers "did this change
touch the code of kernels it was not meant to?" without a GPU.

  python bench/isa_diff.py gemm_persistent.hip --rev HEAD~1
"""
from __future__ import annotations

import argparse
import difflib
import re
import subprocess
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"


def kernels(asm: str) -> dict[str, list[str]]:
    out = {}
    for m in re.finditer(r"^(_Z\S+):[^\n]*$", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        body = [re.sub(r"\.L\w+?\d+_", ".L_", ln.split(";")[0].strip()) for ln in asm[m.end():end].splitlines()]
        out[m.group(1)] = [ln for ln in body if ln and not ln.startswith(".")]
    return out


def compile_asm(src: Path, workdir: Path) -> str:
    workdir.mkdir(parents=True, exist_ok=True)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", str(src), "-o", "x.o",
                    "-save-temps=obj"], cwd=workdir, check=True, capture_output=True, timeout=1800)
    (s,) = workdir.glob(f"{src.stem}-hip-amdgcn-amd-amdhsa-gfx950.s")
    return s.read_text()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("src", help="file under native/kernels/")
    ap.add_argument("--rev", default="HEAD~1")
    ap.add_argument("--rename", action="append", default=[], metavar="REGEX=REPL",
                    help="rewrite this tree's kernel names before matching (a template that gained "
                         "defaulted parameters mangles differently), e.g. 'ELi0ELi0ELi2EEEv=ELi0EEEv'")
    a = ap.parse_args(argv)
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        wt = td / "wt"
        subprocess.run(["git", "worktree", "add", "-f", str(wt), a.rev], cwd=ROOT, check=True, capture_output=True)
        try:
            old = kernels(compile_asm(wt / "native" / "kernels" / a.src, td / "old"))
        finally:
            subprocess.run(["git", "worktree", "remove", "--force", str(wt)], cwd=ROOT, capture_output=True)
        new = kernels(compile_asm(ROOT / "native" / "kernels" / a.src, td / "new"))
        for rule in a.rename:
            pat, repl = rule.split("=", 1)
            new = {re.sub(pat, repl, k): v for k, v in new.items()}
    same = [n for n in old if old[n] == new.get(n)]
    changed = [n for n in old if n in new and old[n] != new[n]]
    print(f"{a.src} vs {a.rev}: {len(same)} kernels instruction-identical, {len(changed)} changed, "
          f"{len(set(new) - set(old))} new, {len(set(old) - set(new))} removed")
    for n in changed:
        d = [ln for ln in difflib.unified_diff(old[n], new[n], lineterm="", n=0)
             if ln[:1] in "+-" and ln[:3] not in ("+++", "---")]
        print(f"  changed {n}: {len(d)} lines, e.g. {d[:4]}")
    for n in sorted(set(new) - set(old)):
        print(f"  new {n} ({len(new[n])} instructions)")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
