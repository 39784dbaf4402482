"""Execute a Dockerfile's stages on the host, without docker (CPU tests).

No docker daemon exists here or on the GPU boxes, and the hermetic fakes only
record ``docker build`` argv -- which let a Dockerfile whose build step could
not link pass every test (Missing 1). This runs the real
instructions instead:

* ``FROM <image> AS <name>`` starts a stage whose filesystem is a temp dir;
* ``COPY <src>... <dst>`` copies from the build context (the repo) into it;
  ``COPY --from=<stage>`` reads the earlier stage's temp dir, or -- for stages
  listed in ``host_stages`` (the ROCm release image) -- the host filesystem,
  which is a ROCm install in this container;
* ``WORKDIR`` / ``ENV`` / ``ARG`` are tracked; ``ENV`` values that are absolute
  paths are mapped into the stage dir;
* ``RUN`` runs under bash with that env in the mapped WORKDIR. ``pip install``
  (no network) is skipped after checking every requirement is pinned with
  ``==``; a RUN that names an absolute path cannot be mapped and is reported in
  ``skipped`` (the test asserts the stages it executes have none).

Only the instruction subset the in-tree Dockerfiles use is implemented.
"""
from __future__ import annotations

import glob
import os
import re
import shlex
import shutil
import subprocess
from dataclasses import dataclass, field


@dataclass
class Stage:
    name: str
    image: str
    instrs: list = field(default_factory=list)  # (op, args-string)


def parse(path: str, build_args: dict | None = None) -> tuple[dict, list]:
    """Returns ({global ARG: value}, [Stage])."""
    text = open(path).read()
    text = re.sub(r"\\\n", " ", text)  # line continuations
    gargs: dict = {}
    stages: list[Stage] = []
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        op, _, rest = line.partition(" ")
        op = op.upper()
        rest = rest.strip()
        if op == "ARG" and not stages:
            k, _, v = rest.partition("=")
            gargs[k] = (build_args or {}).get(k, v)
            continue
        if op == "FROM":
            parts = rest.split()
            image = re.sub(r"\$\{(\w+)\}", lambda m: gargs.get(m.group(1), ""), parts[0])
            name = parts[2] if len(parts) >= 3 and parts[1].upper() == "AS" else str(len(stages))
            stages.append(Stage(name, image))
            continue
        stages[-1].instrs.append((op, rest))
    return gargs, stages


def unpinned_requirements(run: str) -> list:
    """Requirements of a ``pip install`` RUN that are not pinned with ``==``."""
    bad = []
    for cmd in run.split("&&"):
        toks = shlex.split(cmd)
        if "pip" not in toks[:2] or "install" not in toks:
            continue
        for tok in toks[toks.index("install") + 1:]:
            if tok.startswith("-"):
                continue
            if "==" not in tok:
                bad.append(tok)
    return bad


class Executor:
    def __init__(self, dockerfile: str, context: str, workroot: str, host_stages=("rocm",),
                 build_args: dict | None = None, python: str | None = None):
        self.dockerfile = dockerfile
        self.context = context
        self.workroot = workroot
        self.host_stages = set(host_stages)
        self.gargs, self.stages = parse(dockerfile, build_args)
        self.roots: dict = {}
        self.envs: dict = {}
        self.skipped: list = []
        self.ran: list = []
        self.python = python

    def stage(self, name: str) -> Stage:
        for s in self.stages:
            if s.name == name:
                return s
        raise KeyError(name)

    def _map(self, root: str, p: str, workdir: str) -> str:
        if not p.startswith("/"):
            p = os.path.join(workdir, p)
        return os.path.join(root, p.lstrip("/"))

    def _copy(self, root: str, args: str, workdir: str) -> None:
        toks = shlex.split(args)
        src_root = self.context
        from_stage = None
        while toks and toks[0].startswith("--"):
            flag = toks.pop(0)
            if flag.startswith("--from="):
                from_stage = flag.split("=", 1)[1]
        *srcs, dst = toks
        if from_stage is not None:
            src_root = "/" if from_stage in self.host_stages else self.roots[from_stage]
        dst_path = self._map(root, dst, workdir)
        expanded = []
        for s in srcs:
            base = os.path.join(src_root, s.lstrip("/")) if from_stage else os.path.join(src_root, s)
            hits = sorted(glob.glob(base)) if any(c in s for c in "*?[") else [base]
            if not hits or not all(os.path.exists(h) or os.path.islink(h) for h in hits):
                raise FileNotFoundError(f"COPY {args}: {s} not found in "
                                        f"{'stage ' + from_stage if from_stage else 'build context'}")
            expanded += hits
        into_dir = dst.endswith("/") or len(expanded) > 1
        for h in expanded:
            if os.path.isdir(h):  # docker copies a directory's contents
                shutil.copytree(h, dst_path, dirs_exist_ok=True, symlinks=False)
            else:
                target = os.path.join(dst_path, os.path.basename(h)) if into_dir else dst_path
                os.makedirs(os.path.dirname(target), exist_ok=True)
                shutil.copy2(h, target)  # follows symlinks, as COPY does

    def run_stage(self, name: str, skip_pip: bool = True) -> str:
        st = self.stage(name)
        root = os.path.join(self.workroot, f"stage-{st.name}")
        os.makedirs(root, exist_ok=True)
        self.roots[st.name] = root
        workdir = "/"
        env: dict = {}
        for op, args in st.instrs:
            if op == "WORKDIR":
                workdir = args if args.startswith("/") else os.path.join(workdir, args)
                os.makedirs(self._map(root, workdir, "/"), exist_ok=True)
            elif op == "ENV":
                for kv in shlex.split(args):
                    k, _, v = kv.partition("=")
                    env[k] = ":".join(self._map(root, x, "/") if x.startswith("/") else x for x in v.split(":"))
            elif op == "COPY":
                self._copy(root, args, workdir)
            elif op == "RUN":
                if "pip install" in args and skip_pip:
                    bad = unpinned_requirements(args)
                    if bad:
                        raise AssertionError(f"{self.dockerfile}: unpinned pip requirement(s) {bad}")
                    self.skipped.append((st.name, args, "pip (no network)"))
                    continue
                if re.search(r"(^|[\s\"'=])/(?!dev/null)[A-Za-z]", args):
                    self.skipped.append((st.name, args, "absolute path"))
                    continue
                run_env = dict(os.environ, **env)
                if self.python:
                    bindir = os.path.join(self.workroot, "bin")
                    os.makedirs(bindir, exist_ok=True)
                    link = os.path.join(bindir, "python3")
                    if not os.path.exists(link):
                        os.symlink(self.python, link)
                    run_env["PATH"] = bindir + ":" + run_env.get("PATH", "")
                r = subprocess.run(["bash", "-c", args], cwd=self._map(root, workdir, "/"), env=run_env,
                                   capture_output=True, text=True)
                if r.returncode != 0:
                    raise RuntimeError(f"stage {st.name}: RUN {args}\n  failed ({r.returncode}):\n"
                                       f"{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
                self.ran.append((st.name, args))
            # ARG / ENTRYPOINT / CMD / LABEL / EXPOSE: nothing to execute
        self.envs[st.name] = env
        return root
