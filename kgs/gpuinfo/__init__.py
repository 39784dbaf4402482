"""Python view of the native GPU enumeration core (``native/gpuinfo``).

``discover(root)`` returns a :class:`Topology` built by the C++ core
(pybind11 module ``kgs._native._gpuinfo``; ctypes over
``libkgs_gpuinfo.so`` as a second path). There is no pure-Python parser: the
device plugin and CLI always see what the native core sees.

The reference has no discovery at all -- it writes a constant capacity of 2
into each worker's status (kind-gpu-sim.sh:113).
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass, field
from functools import lru_cache
from pathlib import Path

NATIVE_DIR = Path(__file__).resolve().parents[1] / "_native"
XGMI = 11
PCIE = 2


class GpuInfoUnavailable(RuntimeError):
    pass


@dataclass
class Link:
    to_node: int
    type: int
    weight: int = 0
    max_bandwidth_mbs: int = 0

    @property
    def is_xgmi(self) -> bool:
        return self.type == XGMI


@dataclass
class Gpu:
    index: int
    node_id: int
    render_minor: int
    bdf: str = ""
    gpu_id: int = 0
    unique_id: str = "0"
    hive_id: str = "0"
    gfx_arch: str = ""
    gfx_target_version: int = 0
    vendor_id: int = 0
    device_id: int = 0
    simd_count: int = 0
    cu_count: int = 0
    num_xcc: int = 0
    lds_kb: int = 0
    wave_size: int = 0
    max_clock_mhz: int = 0
    vram_bytes: int = 0
    numa_node: int = -1
    uuid: str = ""
    # amd-smi health sample (-1 = not available)
    ecc_correctable: int = -1
    ecc_uncorrectable: int = -1
    ecc_deferred: int = -1
    xgmi_links_total: int = -1
    xgmi_links_up: int = -1
    xgmi_links_down: int = -1
    smi_links: list = field(default_factory=list)  # [{to_index, type, hops, weight, p2p}] from amd-smi
    properties_readable: bool = True
    render_node_present: bool = False
    healthy: bool = False
    health_reason: str = ""
    links: list = field(default_factory=list)

    @property
    def device_id_str(self) -> str:
        """Stable kubelet device ID: the PCI address when known, else the node id."""
        return self.bdf if self.bdf and self.bdf != "0000:00:00.0" else f"kfd-node-{self.node_id}"

    @property
    def render_path(self) -> str:
        return f"/dev/dri/renderD{self.render_minor}"

    @property
    def rocr_uuid(self) -> str:
        """The agent UUID ROCr reports and matches in ``ROCR_VISIBLE_DEVICES``:
        ``GPU-`` + the KFD ``unique_id`` as 16 hex digits ("" when the kernel
        exposes no unique_id). Unlike an index, it names the same GPU whatever
        else the process can see (privileged or not, any enumeration order)."""
        try:
            uid = int(self.unique_id)
        except (TypeError, ValueError):
            return ""
        return f"GPU-{uid:016x}" if uid else ""

    def xgmi_peers(self) -> set:
        return {lk.to_node for lk in self.links if lk.is_xgmi}


@dataclass
class Topology:
    root: str
    kfd_present: bool
    topology_present: bool
    amdsmi_used: bool
    cpu_nodes: int
    gpus: list
    warnings: list
    amdsmi_library: str = ""
    smi_topology_checked: bool = False  # amd-smi's link matrix compared with the KFD io_links
    smi_topology_agrees: bool = False

    def by_node(self) -> dict:
        return {g.node_id: g for g in self.gpus}

    def xgmi_connected(self, a: Gpu, b: Gpu) -> bool:
        return b.node_id in a.xgmi_peers() or a.node_id in b.xgmi_peers()

    @property
    def healthy_gpus(self) -> list:
        return [g for g in self.gpus if g.healthy]


def _parse(js: str) -> Topology:
    d = json.loads(js)
    gpus = []
    for g in d["gpus"]:
        links = [Link(**lk) for lk in g.pop("links")]
        gpus.append(Gpu(links=links, **g))
    return Topology(
        root=d["root"], kfd_present=d["kfd_present"], topology_present=d["topology_present"],
        amdsmi_used=d["amdsmi_used"], cpu_nodes=d["cpu_nodes"], gpus=gpus, warnings=d["warnings"],
        amdsmi_library=d.get("amdsmi_library", ""), smi_topology_checked=d.get("smi_topology_checked", False),
        smi_topology_agrees=d.get("smi_topology_agrees", False),
    )


@lru_cache(maxsize=1)
def _backend():
    try:
        from kgs._native import _gpuinfo  # type: ignore

        return ("pybind", _gpuinfo)
    except ImportError:
        pass
    so = NATIVE_DIR / "libkgs_gpuinfo.so"
    if so.exists():
        lib = ctypes.CDLL(str(so))
        lib.kgs_gpuinfo_discover_json.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_long]
        lib.kgs_gpuinfo_discover_json.restype = ctypes.c_long
        return ("ctypes", lib)
    raise GpuInfoUnavailable(
        f"native gpuinfo core not built ({NATIVE_DIR}); run `python -m kgs.utils.build`"
    )


def backend_name() -> str:
    return _backend()[0]


def discover_json(root: str = "/", use_amdsmi: bool = True) -> str:
    kind, mod = _backend()
    if kind == "pybind":
        return mod.discover_json(str(root), use_amdsmi)
    n = mod.kgs_gpuinfo_discover_json(str(root).encode(), int(use_amdsmi), None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    mod.kgs_gpuinfo_discover_json(str(root).encode(), int(use_amdsmi), buf, n + 1)
    return buf.value.decode()


def discover(root: str | os.PathLike = "/", use_amdsmi: bool = True) -> Topology:
    return _parse(discover_json(str(root), use_amdsmi))


def rocr_visible_devices(gpus) -> str:
    """``ROCR_VISIBLE_DEVICES`` value pinning a process to exactly ``gpus`` (in
    that order: HIP device i is ``gpus[i]``). Raises if a GPU has no UUID --
    an index list would silently mean other GPUs in a privileged container."""
    ids = [g.rocr_uuid for g in gpus]
    missing = [g.render_minor for g, u in zip(gpus, ids) if not u]
    if missing:
        raise GpuInfoUnavailable(f"no KFD unique_id for renderD{missing}: cannot pin by UUID")
    return ",".join(ids)


def parse_rocr_uuids(value: str | None) -> list | None:
    """The ``GPU-<hex>`` entries of a ``ROCR_VISIBLE_DEVICES`` value, lower-case;
    None when it is unset or holds anything but UUIDs (indices)."""
    if not value:
        return None
    items = [x.strip() for x in value.split(",") if x.strip()]
    if not items or not all(x.upper().startswith("GPU-") for x in items):
        return None
    return ["GPU-" + x[4:].lower() for x in items]


def health(root: str, node_id: int, render_minor: int) -> tuple:
    kind, mod = _backend()
    if kind == "pybind":
        return tuple(mod.health(str(root), node_id, render_minor))
    t = discover(root, use_amdsmi=False)
    g = t.by_node().get(node_id)
    return (bool(g and g.healthy), g.health_reason if g else "KFD node gone")


class HealthMonitor:
    """Stateful per-GPU health (native ``HealthMonitor``, native/gpuinfo/gpuinfo.h):
    the sysfs checks plus amd-smi's uncorrectable-ECC count and xGMI link
    status against a baseline taken at the first check. ``check`` returns a dict
    with ``healthy``, ``reason`` and the sample (``ecc_*``, ``xgmi_links_*``,
    ``amdsmi``). Without the pybind core it degrades to the stateless sysfs check.
    """

    def __init__(self, root: str = "/", use_amdsmi: bool = True, ecc_tolerance: int | None = None):
        if ecc_tolerance is None:
            ecc_tolerance = int(os.environ.get("KGS_ECC_UNCORRECTABLE_TOLERANCE", "0"))
        self.root = str(root)
        kind, mod = _backend()
        self._native = mod.HealthMonitor(self.root, use_amdsmi, int(ecc_tolerance)) if kind == "pybind" else None

    @property
    def amdsmi_used(self) -> bool:
        return bool(self._native is not None and self._native.amdsmi_used)

    def check(self, node_id: int, render_minor: int, bdf: str = "") -> dict:
        if self._native is not None:
            return dict(self._native.check(node_id, render_minor, bdf))
        ok, why = health(self.root, node_id, render_minor)
        return {"healthy": ok, "reason": why, "amdsmi": False}
