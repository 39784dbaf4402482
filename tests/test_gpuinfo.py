"""Native gpuinfo core against the captured MI355X box tree and the synthetic 8-GPU tree."""
import json
import os
import subprocess

import pytest

from kgs import gpuinfo
from kgs.gpuinfo.fake import make_fake_mi355x, remove_gpu_device

HERE = os.path.dirname(__file__)
BOX = os.path.join(HERE, "fixtures", "kfd_box1")
CLI = os.path.join(os.path.dirname(HERE), "kgs", "_native", "kgs-gpuinfo")


def test_backend_is_native():
    assert gpuinfo.backend_name() in ("pybind", "ctypes")


def test_captured_box():
    t = gpuinfo.discover(BOX, use_amdsmi=False)
    assert t.kfd_present and t.topology_present and t.cpu_nodes == 2
    assert len(t.gpus) == 1
    g = t.gpus[0]
    assert (g.node_id, g.render_minor, g.bdf, g.gfx_arch) == (4, 144, "0000:5a:00.0", "gfx950")
    assert g.cu_count == 256 and g.num_xcc == 8 and g.lds_kb == 160 and g.wave_size == 64
    assert g.vram_bytes == 309220868096 and g.max_clock_mhz == 2400 and g.numa_node == 0
    assert g.healthy and g.links == []  # peers are cgroup-hidden on the box


def test_fake_eight(tmp_path):
    root = make_fake_mi355x(tmp_path)
    t = gpuinfo.discover(root, use_amdsmi=False)
    assert [g.render_minor for g in t.gpus] == [128 + 8 * i for i in range(8)]
    assert [g.numa_node for g in t.gpus] == [0, 0, 0, 0, 1, 1, 1, 1]
    for g in t.gpus:
        assert len(g.xgmi_peers()) == 7 and all(lk.max_bandwidth_mbs == 76000 for lk in g.links if lk.is_xgmi)
    assert t.xgmi_connected(t.gpus[0], t.gpus[7])
    assert len({g.device_id_str for g in t.gpus}) == 8


def test_health_detects_missing_node(tmp_path):
    root = make_fake_mi355x(tmp_path, n_gpus=2)
    assert gpuinfo.health(str(root), 2, 128) == (True, "ok")
    remove_gpu_device(root, 128)
    ok, why = gpuinfo.health(str(root), 2, 128)
    assert not ok and "renderD128" in why
    t = gpuinfo.discover(root, use_amdsmi=False)
    assert [g.healthy for g in t.gpus] == [False, True]


def test_no_kfd(tmp_path):
    root = make_fake_mi355x(tmp_path, n_gpus=1, with_kfd=False)
    t = gpuinfo.discover(root, use_amdsmi=False)
    assert not t.kfd_present and not t.gpus[0].healthy
    assert any("/dev/kfd" in w for w in t.warnings)
    empty = gpuinfo.discover(tmp_path / "nothing", use_amdsmi=False)
    assert not empty.topology_present and empty.gpus == []


def test_gfx_name():
    from kgs._native import _gpuinfo

    assert _gpuinfo.gfx_name(90500) == "gfx950"
    assert _gpuinfo.gfx_name(90402) == "gfx942"
    assert _gpuinfo.gfx_name(100300) == "gfx1030"


@pytest.mark.skipif(not os.path.exists(CLI), reason="kgs-gpuinfo not built")
def test_cli_json_matches_module(tmp_path):
    root = make_fake_mi355x(tmp_path, n_gpus=4)
    out = subprocess.run([CLI, "--root", str(root), "--json", "--no-amdsmi"], capture_output=True, text=True,
                         check=True).stdout
    d = json.loads(out)
    assert [g["render_minor"] for g in d["gpus"]] == [128, 136, 144, 152]
    table = subprocess.run([CLI, "--root", str(root)], capture_output=True, text=True, check=True).stdout
    assert "gfx950" in table and "X X X" in table


def test_ctypes_backend_agrees(tmp_path):
    import ctypes

    root = make_fake_mi355x(tmp_path, n_gpus=2)
    so = ctypes.CDLL(str(gpuinfo.NATIVE_DIR / "libkgs_gpuinfo.so"))
    so.kgs_gpuinfo_discover_json.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_long]
    so.kgs_gpuinfo_discover_json.restype = ctypes.c_long
    n = so.kgs_gpuinfo_discover_json(str(root).encode(), 0, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    so.kgs_gpuinfo_discover_json(str(root).encode(), 0, buf, n + 1)
    assert json.loads(buf.value.decode()) == json.loads(gpuinfo.discover_json(str(root), False))
