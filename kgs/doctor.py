"""``kgs doctor``: host preflight before ``kgs create``.

The reference lists its prerequisites in a table (docker|podman, kind, kubectl,
git, sed -- /root/reference/Readme.md:29-35) and discovers missing ones
mid-run. ``kgs doctor`` checks what this provisioner needs up front, and the
MI355X-specific pieces the reference never had to care about:

* container runtime, kind, kubectl present (and their versions);
* ``/dev/kfd`` and the ``/dev/dri/renderD*`` nodes exist and are read/write for
  this user (the kind node containers bind-mount them);
* the native gpuinfo core finds the GPUs, they are gfx950, healthy, and the
  xGMI mesh is complete (every pair linked: what RCCL's rings need);
* the local registry port is free or already ours;
* the in-tree native build (HIP kernels, first-GEMM probe, gpuinfo core) is
  present and newer than its sources (WARN otherwise: the workload image
  rebuilds it, but a host-side ``kgs bench --no-kind`` runs what is in the tree).

Each check is OK / WARN / FAIL; exit status 1 if any FAIL. ``--json`` for tools.
"""
from __future__ import annotations

import json
import os
import socket
from dataclasses import dataclass

from . import config as C
from .utils.proc import Runner


@dataclass
class Check:
    name: str
    status: str  # OK | WARN | FAIL
    detail: str

    def as_dict(self):
        return {"name": self.name, "status": self.status, "detail": self.detail}


def _tool_version(runner: Runner, argv: list) -> str:
    r = runner.run(argv, check=False, mutating=False, timeout=20)
    out = (r.stdout or r.stderr).strip().splitlines()
    return out[0] if r.ok and out else ""


def check_tools(runner: Runner, runtime: str | None) -> list:
    out = []
    rts = [runtime] if runtime else ["docker", "podman"]
    found = [rt for rt in rts if runner.which(rt)]
    if found:
        out.append(Check("container runtime", "OK", f"{found[0]} ({_tool_version(runner, [found[0], '--version'])})"))
    else:
        out.append(Check("container runtime", "FAIL", f"none of {', '.join(rts)} on PATH"))
    for tool, argv in (("kind", ["kind", "version"]), ("kubectl", ["kubectl", "version", "--client"])):
        if runner.which(tool):
            out.append(Check(tool, "OK", _tool_version(runner, argv) or "present"))
        else:
            out.append(Check(tool, "FAIL", f"{tool} not on PATH"))
    return out


def check_devices(root: str) -> list:
    out = []
    kfd = os.path.join(root, "dev", "kfd")
    if not os.path.exists(kfd):
        return [Check("/dev/kfd", "WARN", "absent: CPU-only host, `kgs create` will use the fake-capacity path")]
    out.append(Check("/dev/kfd", "OK" if os.access(kfd, os.R_OK | os.W_OK) else "FAIL",
                     "read/write" if os.access(kfd, os.R_OK | os.W_OK) else "not read/write for this user "
                     "(add it to the render/video groups)"))
    try:
        from kgs import gpuinfo

        topo = gpuinfo.discover(root)
    except Exception as e:  # native core missing or unreadable sysfs
        out.append(Check("gpuinfo", "FAIL", f"discovery failed: {e}"))
        return out
    gpus = topo.gpus
    if not gpus:
        out.append(Check("GPUs", "FAIL", "/dev/kfd exists but no GPU node in the KFD topology"))
        return out
    archs = sorted({g.gfx_arch for g in gpus})
    out.append(Check("GPUs", "OK" if archs == ["gfx950"] else "WARN",
                     f"{len(gpus)} x {','.join(archs)} (MI355X is gfx950)"))
    bad_nodes = [g.render_minor for g in gpus
                 if not os.access(os.path.join(root, "dev", "dri", f"renderD{g.render_minor}"), os.R_OK | os.W_OK)]
    out.append(Check("render nodes", "FAIL" if bad_nodes else "OK",
                     f"renderD{bad_nodes} not read/write" if bad_nodes else
                     f"renderD{[g.render_minor for g in gpus]} read/write"))
    unhealthy = [g.index for g in gpus if not g.healthy]
    out.append(Check("health", "FAIL" if unhealthy else "OK",
                     f"unhealthy: {unhealthy}" if unhealthy else "all healthy"))
    if len(gpus) > 1:
        missing = [(a.index, b.index) for i, a in enumerate(gpus) for b in gpus[i + 1:]
                   if not topo.xgmi_connected(a, b)]
        out.append(Check("xGMI mesh", "WARN" if missing else "OK",
                         f"pairs without a direct xGMI link: {missing}" if missing else
                         f"all {len(gpus) * (len(gpus) - 1) // 2} pairs directly linked"))
    numa = sorted({g.numa_node for g in gpus})
    out.append(Check("NUMA", "OK", f"GPUs on NUMA nodes {numa}"))
    return out


def check_registry_port(port: int, runner: Runner, runtime: str | None) -> Check:
    with socket.socket() as s:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        try:
            s.bind(("127.0.0.1", port))
            return Check("registry port", "OK", f"127.0.0.1:{port} free")
        except OSError:
            pass
    rt = runtime or next((r for r in ("docker", "podman") if runner.which(r)), None)
    if rt:
        r = runner.run([rt, "ps", "-q", "-f", f"name=^{C.REGISTRY_NAME}$"], check=False, mutating=False)
        if r.ok and r.stdout.strip():
            return Check("registry port", "OK", f"{port} held by the existing {C.REGISTRY_NAME} (reused)")
    return Check("registry port", "FAIL", f"{port} in use by something else (use --registry-port)")


def check_native_build() -> Check:
    from .utils import build

    missing, stale = [], []
    for t in build.targets():
        if not t.output.exists():
            (stale if t.optional else missing).append(t.name)
        elif t.stale():
            stale.append(t.name)
    if missing:
        return Check("native build", "WARN", f"not built: {', '.join(missing)} (python -m kgs.utils.build)")
    if stale:
        return Check("native build", "WARN", f"older than sources: {', '.join(stale)} (python -m kgs.utils.build)")
    return Check("native build", "OK", f"{len(build.targets())} targets fresh for {build.ARCH}")


def run_doctor(settings: C.Settings, as_json: bool = False, runner: Runner | None = None) -> int:
    runner = runner or Runner()
    checks = check_tools(runner, settings.runtime)
    checks += check_devices(settings.dev_root)
    checks.append(check_registry_port(settings.registry_port, runner, settings.runtime))
    checks.append(check_native_build())
    failed = any(c.status == "FAIL" for c in checks)
    if as_json:
        print(json.dumps({"ok": not failed, "checks": [c.as_dict() for c in checks]}, indent=1))
    else:
        w = max(len(c.name) for c in checks)
        for c in checks:
            print(f"{c.status:4}  {c.name:<{w}}  {c.detail}")
        print("ready for `kgs create rocm`" if not failed else "fix the FAIL lines above first")
    return 1 if failed else 0
