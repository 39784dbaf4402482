"""Write a synthetic KFD/DRM tree of an 8 x MI355X host.

Property values are copied from a real gfx950 node captured on an MI355X box
(tests/fixtures/kfd_box1): 256 CUs (simd_count 1024), 8 XCCs, 160 KiB LDS,
288 GiB HBM3E, 2400 MHz, vendor 0x1002 / device 0x75a3, render minors
128 + 8*i, every GPU pair joined by one xGMI link (io_link type 11, weight 15).
Used by tests, by ``kgs create --fake-gpus`` dry runs and by the device plugin's
self-test; nothing here touches real devices.
"""
from __future__ import annotations

import os
from pathlib import Path

GFX950_PROPS = {
    "cpu_cores_count": 0,
    "simd_count": 1024,
    "mem_banks_count": 1,
    "caches_count": 546,
    "io_links_count": 8,
    "p2p_links_count": 1,
    "cpu_core_id_base": 0,
    "simd_id_base": 2147487816,
    "max_waves_per_simd": 8,
    "lds_size_in_kb": 160,
    "gds_size_in_kb": 0,
    "num_gws": 64,
    "wave_front_size": 64,
    "array_count": 32,
    "simd_arrays_per_engine": 1,
    "cu_per_simd_array": 9,
    "simd_per_cu": 4,
    "max_slots_scratch_cu": 32,
    "gfx_target_version": 90500,
    "vendor_id": 4098,
    "device_id": 30115,
    "location_id": 0,
    "domain": 0,
    "drm_render_minor": 0,
    "hive_id": 9825122081130393499,
    "num_sdma_engines": 2,
    "num_sdma_xgmi_engines": 14,
    "num_sdma_queues_per_engine": 8,
    "num_cp_queues": 24,
    "max_engine_clk_fcompute": 2400,
    "local_mem_size": 0,
    "unique_id": 0,
    "num_xcc": 8,
    "max_engine_clk_ccompute": 5008,
}
HBM_BYTES = 288 * (1 << 30)
# PCI buses of the 8 OAM slots (any distinct values do)
BUSES = [0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xE5, 0xF5]


def _write(p: Path, text: str) -> None:
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(text)


def _props(d: dict) -> str:
    return "".join(f"{k} {v}\n" for k, v in d.items())


def make_fake_mi355x(root: str | os.PathLike, n_gpus: int = 8, cpu_sockets: int = 2, render_base: int = 128,
                     render_step: int = 8, with_kfd: bool = True, xgmi: bool = True) -> Path:
    """Create the tree under ``root``; returns ``root`` as a Path."""
    root = Path(root)
    topo = root / "sys/class/kfd/kfd/topology"
    _write(topo / "generation_id", "1\n")
    _write(topo / "system_properties", "platform_oem 0\nplatform_id 0\nplatform_rev 0\n")
    nodes = topo / "nodes"
    for c in range(cpu_sockets):
        _write(nodes / str(c) / "properties", _props({"cpu_cores_count": 128, "simd_count": 0,
                                                      "mem_banks_count": 1, "io_links_count": n_gpus}))
        _write(nodes / str(c) / "gpu_id", "0\n")
    if with_kfd:
        _write(root / "dev/kfd", "")
    for i in range(n_gpus):
        nid = cpu_sockets + i
        minor = render_base + render_step * i
        p = dict(GFX950_PROPS)
        p["drm_render_minor"] = minor
        p["location_id"] = BUSES[i % len(BUSES)] << 8
        p["unique_id"] = 0xA6FF75A300000000 + i
        nd = nodes / str(nid)
        _write(nd / "properties", _props(p))
        _write(nd / "gpu_id", f"{28000 + 206 * i}\n")
        _write(nd / "name", "ip discovery\n")
        _write(nd / "mem_banks/0/properties", _props({"heap_type": 1, "size_in_bytes": HBM_BYTES,
                                                      "flags": 0, "width": 8192, "mem_clk_max": 2000}))
        link = 0
        # PCIe link to the CPU socket owning this GPU
        sock = i * cpu_sockets // max(1, n_gpus)
        _write(nd / f"io_links/{link}/properties",
               _props({"type": 2, "node_from": nid, "node_to": sock, "weight": 20,
                       "max_bandwidth": 63000, "flags": 1}))
        link += 1
        if xgmi:
            for j in range(n_gpus):
                if j == i:
                    continue
                _write(nd / f"io_links/{link}/properties",
                       _props({"type": 11, "version_major": 0, "node_from": nid, "node_to": cpu_sockets + j,
                               "weight": 15, "min_bandwidth": 76000, "max_bandwidth": 76000, "flags": 1}))
                link += 1
        _write(root / f"dev/dri/renderD{minor}", "")
        _write(root / f"sys/class/drm/renderD{minor}/device/numa_node", f"{sock}\n")
    return root


def remove_gpu_device(root: str | os.PathLike, render_minor: int) -> None:
    """Fault injection: the render node disappears (GPU lost / reset)."""
    p = Path(root) / f"dev/dri/renderD{render_minor}"
    if p.exists():
        p.unlink()


def restore_gpu_device(root: str | os.PathLike, render_minor: int) -> None:
    _write(Path(root) / f"dev/dri/renderD{render_minor}", "")
