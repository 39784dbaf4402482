"""In-tree native build for kgs (gfx950 only).

Builds, with the ROCm toolchain in ``/opt/rocm``:

* ``kgs/_native/libkgs_kernels.so`` -- every ``native/kernels/*.hip`` (bf16 MFMA
  GEMM, vector add, transpose, checksum, P2P all-reduce) behind a C ABI that
  ``kgs/ops/_lib.py`` loads with ctypes. Built with ``-fvisibility=hidden``:
  only the ``KGS_EXPORT`` production entry points are exported.
* ``kgs/_native/kgs-gpuprobe`` -- the pod's first-GEMM readiness probe: HIP
  host code linked against ``libkgs_kernels.so`` (no Python, no torch), one
  thread per visible GPU running the production GEMM with a sampled check.
* ``kgs/_native/kgs-graph-memset-repro`` -- a pure-HIP check of hipGraph memset
  nodes (native/probe/graph_memset_repro.hip), no torch, no kgs library.
* ``kgs/_native/libkgs_experiments.so`` -- ``native/experiments/*.hip``, the
  measured GEMM alternatives and timing probes (some wrong by construction),
  opt-in through ``kgs.ops.experiments`` and never loaded by production code.
* ``kgs/_native/libkgs_gpuinfo.so`` + ``kgs/_native/kgs-gpuinfo`` -- the C++
  device-enumeration core (KFD sysfs topology + amd-smi) used by the device
  plugin, also as a standalone CLI.
* ``kgs/_native/libamd_smi_stub.so`` -- a test double of the amd-smi C API
  (ECC counts and xGMI link states from a text file) for the CPU tests of the
  plugin's health path; loaded only through ``KGS_AMDSMI_LIB``.
* ``kgs/_native/_serve*.so`` -- the continuous-batching scheduler and paged-KV
  block allocator of ``kgs.serve`` (C++17, pybind11).
* ``kgs/_native/kgs-rccl-bench`` -- single-process multi-GPU RCCL all-reduce
  sweep (ncclCommInitAll), the C++ twin of ``kgs.parallel.allreduce``.

Everything is compiled for ``--offload-arch=gfx950`` and nothing else. The
build is incremental (mtime based) and parallel; ``python -m kgs.utils.build``
or ``__graft_entry__.build()`` drive it. No JIT cache is used, so the built
``.so`` files travel with the repo snapshot to the GPU box.

Every build writes ``kgs/_native/build_manifest.json``: per target, the sha256
of the output and of every source and header it was built from, the compiler
line and the toolchain version. ``python -m kgs.utils.build --check`` (and
``smoke()``) compare it against the tree: a library that no longer matches its
sources, or a source edited after the last build, is reported by name.

The reference has no native build at all; its only native components are Go
device plugins cloned and built inside docker (kind-gpu-sim.sh:180-228).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import subprocess
import sys
from dataclasses import dataclass, field
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
NATIVE = REPO / "native"
OUT = REPO / "kgs" / "_native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = "gfx950"

HIPCC = str(ROCM / "bin" / "hipcc")
MANIFEST = "build_manifest.json"
CXX = os.environ.get("CXX", "g++")

HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
    "-munsafe-fp-atomics",
]


@dataclass
class Target:
    name: str
    output: Path
    sources: list[Path]
    compiler: str
    flags: list[str] = field(default_factory=list)
    link_flags: list[str] = field(default_factory=list)
    shared: bool = True
    headers: list[Path] = field(default_factory=list)
    optional: bool = False  # skip (with a warning) if a dependency is missing

    def stale(self) -> bool:
        if not self.output.exists():
            return True
        out_m = self.output.stat().st_mtime
        deps = list(self.sources) + list(self.headers) + [Path(__file__)]
        return any(p.exists() and p.stat().st_mtime > out_m for p in deps)


def _pybind_includes() -> list[str]:
    try:
        import pybind11  # noqa: WPS433

        inc = [pybind11.get_include()]
    except Exception:  # pragma: no cover - pybind11 is in the image
        return []
    import sysconfig

    inc.append(sysconfig.get_paths()["include"])
    return [f"-I{p}" for p in inc]


def _py_ext_suffix() -> str:
    import sysconfig

    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


# ``--only`` group names: the device-plugin image builds ``gpuinfo`` (the three
# targets of the enumeration core) and nothing that needs hipcc.
GROUPS = {
    "gpuinfo": ("gpuinfo-lib", "gpuinfo-py", "gpuinfo-cli"),
    "gpu": ("kernels", "gpuprobe", "experiments", "rccl-bench", "memset-repro"),
}


def expand_only(only: list[str] | None) -> list[str] | None:
    if not only:
        return None
    out: list[str] = []
    for name in only:
        for t in GROUPS.get(name, (name,)):
            if t not in out:
                out.append(t)
    return out


def amdsmi_header(rocm: Path | None = None) -> Path:
    return (rocm or ROCM) / "include" / "amd_smi" / "amdsmi.h"


def targets(out: Path | None = None) -> list[Target]:
    odir = Path(out) if out is not None else OUT
    kdir = NATIVE / "kernels"
    gdir = NATIVE / "gpuinfo"
    rdir = NATIVE / "rccl_bench"
    sdir = NATIVE / "serve"
    k_headers = sorted(kdir.glob("*.h"))
    g_headers = sorted(gdir.glob("*.h"))
    amdsmi_ok = amdsmi_header().exists()
    smi_flags = ["-DKGS_HAVE_AMDSMI=1", f"-I{ROCM / 'include'}"] if amdsmi_ok else []
    # amd-smi is dlopen'ed at run time (native/gpuinfo/smi.cpp): headers only, no link dependency
    smi_link = ["-ldl"]
    core = [gdir / "gpuinfo.cpp", gdir / "smi.cpp"]
    ts = [
        Target(
            "kernels",
            odir / "libkgs_kernels.so",
            sorted(kdir.glob("*.hip")),
            HIPCC,
            flags=HIP_FLAGS + ["-fvisibility=hidden", f"-I{kdir}"],
            headers=k_headers,
        ),
        Target(
            "gpuprobe",
            odir / "kgs-gpuprobe",
            [NATIVE / "probe" / "gpuprobe.hip"],
            HIPCC,
            flags=[f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-Wall"],
            link_flags=[f"-L{odir}", "-lkgs_kernels", "-Wl,-rpath,$ORIGIN", "-pthread"],
            shared=False,
        ),
        Target(
            "memset-repro",
            odir / "kgs-graph-memset-repro",
            [NATIVE / "probe" / "graph_memset_repro.hip"],
            HIPCC,
            flags=[f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-Wall"],
            link_flags=[],
            shared=False,
        ),
        Target(
            "experiments",
            odir / "libkgs_experiments.so",
            sorted((NATIVE / "experiments").glob("*.hip")),
            HIPCC,
            flags=HIP_FLAGS + ["-fvisibility=hidden", f"-I{kdir}"],
            headers=k_headers + sorted((NATIVE / "experiments").glob("*.h")),
        ),
        Target(
            "gpuinfo-lib",
            odir / "libkgs_gpuinfo.so",
            core + [gdir / "gpuinfo_capi.cpp"],
            CXX,
            flags=["-O2", "-std=c++17", "-fPIC", "-Wall", f"-I{gdir}"] + smi_flags,
            link_flags=smi_link,
            headers=g_headers,
        ),
        Target(
            "gpuinfo-py",
            odir / f"_gpuinfo{_py_ext_suffix()}",
            core + [gdir / "gpuinfo_py.cpp"],
            CXX,
            flags=["-O2", "-std=c++17", "-fPIC", "-Wall", f"-I{gdir}"] + smi_flags + _pybind_includes(),
            link_flags=smi_link,
            headers=g_headers,
        ),
        Target(
            "gpuinfo-cli",
            odir / "kgs-gpuinfo",
            core + [gdir / "gpuinfo_cli.cpp"],
            CXX,
            flags=["-O2", "-std=c++17", "-Wall", f"-I{gdir}"] + smi_flags,
            link_flags=smi_link,
            shared=False,
            headers=g_headers,
        ),
        Target(
            "amdsmi-stub",
            odir / "libamd_smi_stub.so",
            [gdir / "testing" / "amdsmi_stub.cpp"],
            CXX,
            flags=["-O2", "-std=c++17", "-fPIC", "-Wall", f"-I{ROCM / 'include'}"],
            optional=True,
        ),
        Target(
            "serve-py",
            odir / f"_serve{_py_ext_suffix()}",
            [sdir / "scheduler.cpp", sdir / "serve_py.cpp"],
            CXX,
            flags=["-O2", "-std=c++17", "-fPIC", "-Wall", f"-I{sdir}"] + _pybind_includes(),
            headers=sorted(sdir.glob("*.h")),
        ),
        Target(
            "rccl-bench",
            odir / "kgs-rccl-bench",
            [rdir / "rccl_bench.cpp"],
            HIPCC,
            flags=[f"--offload-arch={ARCH}", "-O2", "-std=c++17", f"-I{ROCM / 'include'}"],
            link_flags=[f"-L{ROCM / 'lib'}", "-lrccl", f"-Wl,-rpath,{ROCM / 'lib'}"],
            shared=False,
            optional=True,
        ),
    ]
    return [t for t in ts if all(s.exists() for s in t.sources)]


def _compile_one(t: Target, src: Path, obj: Path) -> None:
    cmd = [t.compiler, *t.flags, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_target(t: Target, jobs: int = 8, verbose: bool = False, objroot: Path | None = None) -> bool:
    """Build one target; returns True if it was (re)built."""
    if not t.stale():
        return False
    objdir = (objroot or REPO / "build" / "obj") / t.name
    objdir.mkdir(parents=True, exist_ok=True)
    objs = [objdir / (s.stem + ".o") for s in t.sources]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_compile_one, t, s, o) for s, o in zip(t.sources, objs)]
        for f in futs:
            f.result()
    t.output.parent.mkdir(parents=True, exist_ok=True)
    tmp = t.output.with_name(t.output.name + ".tmp")
    link = [t.compiler]
    if t.compiler == HIPCC:
        link.append(f"--offload-arch={ARCH}")
    if t.shared:
        link.append("-shared")
    link += [str(o) for o in objs] + ["-o", str(tmp)] + t.link_flags
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, t.output)
    if verbose:
        print(f"[kgs.build] built {t.output}", file=sys.stderr)
    return True


def build_all(jobs: int | None = None, verbose: bool = True, only: list[str] | None = None,
              out: str | os.PathLike | None = None, require_amdsmi: bool = False) -> dict[str, str]:
    """Build every native target (or the ``only`` targets / groups) into
    ``out`` (default ``kgs/_native``). Returns {name: "built"|"fresh"|"skipped: why"}.

    This is the ONE build definition: ``images/Dockerfile.deviceplugin`` runs
    ``python3 -m kgs.utils.build --only gpuinfo --require-amdsmi --out ...``
    in its build stage instead of hand-written compiler lines.
    """
    only = expand_only(only)
    outdir = Path(out).resolve() if out is not None else None
    sel = [t for t in targets(outdir) if not only or t.name in only]
    if only:
        unknown = sorted(set(only) - {t.name for t in targets(outdir)})
        if unknown:
            raise RuntimeError(f"unknown build target(s) {unknown}; have {[t.name for t in targets(outdir)]} "
                               f"and groups {sorted(GROUPS)}")
    if any(t.compiler == HIPCC for t in sel) and not Path(HIPCC).exists():
        raise RuntimeError(f"hipcc not found at {HIPCC}; set ROCM_PATH")
    if require_amdsmi and not amdsmi_header().exists():
        raise RuntimeError(f"--require-amdsmi: {amdsmi_header()} not found (set ROCM_PATH to a tree with "
                           "include/amd_smi); the device plugin's ECC/xGMI health needs it")
    jobs = jobs or min(8, os.cpu_count() or 4)
    objroot = (outdir / ".obj") if outdir is not None else None
    status: dict[str, str] = {}
    for t in sel:
        try:
            status[t.name] = "built" if build_target(t, jobs=jobs, verbose=verbose, objroot=objroot) else "fresh"
        except RuntimeError as e:
            if t.optional:
                status[t.name] = f"skipped: {str(e).splitlines()[0]}"
                if verbose:
                    print(f"[kgs.build] optional target {t.name} skipped:\n{e}", file=sys.stderr)
            else:
                raise
    write_manifest(outdir if outdir is not None else OUT, sel, status)
    return status


def _sha256(p: Path) -> str:
    h = hashlib.sha256()
    with open(p, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def _rel(p: Path) -> str:
    try:
        return str(Path(p).resolve().relative_to(REPO))
    except ValueError:
        return str(p)


def _toolchain(compiler: str) -> str:
    try:
        r = subprocess.run([compiler, "--version"], capture_output=True, text=True, timeout=60)
        return " | ".join(line for line in r.stdout.splitlines()[:2] if line)
    except (OSError, subprocess.SubprocessError):
        return "unknown"


def _record(t: Target) -> dict:
    return {"output": _rel(t.output), "output_sha256": _sha256(t.output),
            "inputs": {_rel(p): _sha256(p) for p in [*t.sources, *t.headers] if p.exists()},
            "compile": [Path(t.compiler).name, *t.flags], "link": t.link_flags,
            "toolchain": _toolchain(t.compiler)}


def write_manifest(outdir: Path, sel: list[Target], status: dict[str, str]) -> Path:
    """Merge the records of the targets built or found fresh into the manifest."""
    path = outdir / MANIFEST
    try:
        man = json.loads(path.read_text())
    except (OSError, ValueError):
        man = {}
    man.setdefault("targets", {})
    man["arch"], man["mode"] = ARCH, "in-tree (kgs.utils.build), no JIT cache"
    for t in sel:
        if t.output.exists() and not status.get(t.name, "").startswith("skipped"):
            man["targets"][t.name] = _record(t)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + ".tmp")
    tmp.write_text(json.dumps(man, indent=1, sort_keys=True) + "\n")
    os.replace(tmp, path)
    return path


def check_manifest(out: str | os.PathLike | None = None) -> dict:
    """Compare the manifest against the tree. Returns {"ok", "targets": {name:
    "ok" | why}}: a target is not ok when its output is missing or differs from
    the recorded hash (rebuilt or replaced since), or when one of its inputs
    changed (the library predates the source)."""
    outdir = Path(out) if out is not None else OUT
    try:
        man = json.loads((outdir / MANIFEST).read_text())
    except (OSError, ValueError) as e:
        return {"ok": False, "error": f"no manifest: {e}", "targets": {}}
    res: dict[str, str] = {}
    for name, rec in man.get("targets", {}).items():
        outp = REPO / rec["output"] if not Path(rec["output"]).is_absolute() else Path(rec["output"])
        if not outp.exists():
            res[name] = "output missing"
            continue
        if _sha256(outp) != rec["output_sha256"]:
            res[name] = "output differs from the recorded build"
            continue
        changed = [k for k, v in rec["inputs"].items()
                   if not (REPO / k).exists() or _sha256(REPO / k) != v]
        res[name] = f"inputs changed since the build: {changed}" if changed else "ok"
    return {"ok": bool(res) and all(v == "ok" for v in res.values()), "targets": res}


def clean() -> None:
    shutil.rmtree(REPO / "build" / "obj", ignore_errors=True)
    for p in OUT.glob("*"):
        if p.is_dir():
            shutil.rmtree(p, ignore_errors=True)  # __pycache__
        elif p.name != "__init__.py":
            p.unlink()


def main(argv: list[str] | None = None) -> int:
    import argparse

    ap = argparse.ArgumentParser(prog="python -m kgs.utils.build", description=__doc__.splitlines()[0])
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--only", nargs="*", default=None,
                    help=f"targets or groups ({', '.join(sorted(GROUPS))})")
    ap.add_argument("--out", default=None, help="output directory (default kgs/_native)")
    ap.add_argument("--require-amdsmi", action="store_true",
                    help="fail unless the amd-smi header is found (device-plugin image)")
    ap.add_argument("--check", action="store_true",
                    help="build nothing: compare the build manifest against the tree (exit 1 if stale)")
    a = ap.parse_args(argv)
    if a.check:
        res = check_manifest(a.out)
        print(json.dumps(res, indent=1))
        return 0 if res["ok"] else 1
    if a.clean:
        clean()
    st = build_all(jobs=a.jobs, only=a.only, out=a.out, require_amdsmi=a.require_amdsmi)
    if a.out is not None:
        shutil.rmtree(Path(a.out) / ".obj", ignore_errors=True)
    for k, v in st.items():
        print(f"{k:14s} {v}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
