"""amd-smi health and topology in the native gpuinfo core.

The amd-smi C API is served by a stub library (native/gpuinfo/testing/
amdsmi_stub.cpp, loaded through KGS_AMDSMI_LIB) whose ECC counters and xGMI link
states come from a text file the tests rewrite while the plugin runs: an
uncorrectable-ECC rise or a dropped xGMI link must flip the device to Unhealthy
on ListAndWatch, and a counter reset / link restore must bring it back."""
import os
import tempfile

import pytest

from kgs.deviceplugin.fake_kubelet import FakeKubelet
from kgs.deviceplugin.server import AmdGpuDevicePlugin, RealSource
from kgs.gpuinfo.fake import make_fake_mi355x

NATIVE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kgs", "_native")
STUB = os.path.join(NATIVE, "libamd_smi_stub.so")

pytestmark = pytest.mark.skipif(not os.path.exists(STUB), reason="amd-smi stub not built (python -m kgs.utils.build)")


class StubSmi:
    """Writes the stub's state file: one `gpu` line per device, `link` lines."""

    def __init__(self, path, gpus):
        self.path = path
        self.gpus = {g.render_minor: {"bdf": g.bdf, "uuid": f"uuid-{g.render_minor}", "corr": 0, "uncorr": 0,
                                      "deferred": 0, "links": "1111111"} for g in gpus}
        self.links = []
        self.write()

    def write(self):
        lines = [f"gpu {m} {v['bdf']} {v['uuid']} {v['corr']} {v['uncorr']} {v['deferred']} {v['links']}"
                 for m, v in sorted(self.gpus.items())]
        lines += [f"link {a} {b} {t} {h} {w}" for a, b, t, h, w in self.links]
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            f.write("\n".join(lines) + "\n")
        os.replace(tmp, self.path)


@pytest.fixture
def smi_host(monkeypatch):
    d = tempfile.mkdtemp(prefix="kgs", dir="/tmp")
    root = str(make_fake_mi355x(os.path.join(d, "host"), n_gpus=4))
    from kgs import gpuinfo

    gpus = gpuinfo.discover(root, use_amdsmi=False).gpus
    stub = StubSmi(os.path.join(d, "smi_state.txt"), gpus)
    for i, a in enumerate(gpus):  # the fake tree is a full xGMI mesh
        for b in gpus[i + 1:]:
            stub.links.append((a.render_minor, b.render_minor, "xgmi", 1, 15))
    stub.write()
    monkeypatch.setenv("KGS_AMDSMI_LIB", STUB)
    monkeypatch.setenv("KGS_AMDSMI_STUB_STATE", stub.path)
    monkeypatch.delenv("KGS_NO_AMDSMI", raising=False)
    yield root, stub, d
    import shutil

    shutil.rmtree(d, ignore_errors=True)


def test_discover_uses_amdsmi_and_cross_checks_links(smi_host):
    from kgs import gpuinfo

    root, stub, _ = smi_host
    stub.gpus[128]["corr"] = 5
    stub.write()
    t = gpuinfo.discover(root)
    assert t.amdsmi_used and t.amdsmi_library.endswith("libamd_smi_stub.so")
    g0 = t.gpus[0]
    assert g0.uuid == "uuid-128" and g0.ecc_correctable == 5 and g0.ecc_uncorrectable == 0
    assert g0.xgmi_links_total == 7 and g0.xgmi_links_up == 7 and g0.xgmi_links_down == 0
    assert {p["to_index"] for p in g0.smi_links} == {1, 2, 3}
    assert all(p["type"] == gpuinfo.XGMI and p["hops"] == 1 and p["p2p"] == 1 for p in g0.smi_links)
    assert t.smi_topology_checked and t.smi_topology_agrees and not t.warnings


def test_topology_disagreement_is_reported(smi_host):
    from kgs import gpuinfo

    root, stub, _ = smi_host
    stub.links = [lk for lk in stub.links if {lk[0], lk[1]} != {128, 136}]  # amd-smi: PCIe between GPU 0 and 1
    stub.write()
    t = gpuinfo.discover(root)
    assert t.smi_topology_checked and not t.smi_topology_agrees
    assert any("disagree on GPU 0 -> 1" in w for w in t.warnings)


def test_no_amdsmi_without_opt_in(smi_host, monkeypatch):
    from kgs import gpuinfo

    root, _, _ = smi_host
    monkeypatch.delenv("KGS_AMDSMI_LIB")
    t = gpuinfo.discover(root)  # a non-"/" root never touches the host's amd-smi
    assert not t.amdsmi_used and t.gpus[0].ecc_uncorrectable == -1


def test_health_monitor_ecc_and_link_baselines(smi_host):
    from kgs import gpuinfo

    root, stub, _ = smi_host
    g = gpuinfo.discover(root, use_amdsmi=False).gpus[1]
    stub.gpus[g.render_minor]["uncorr"] = 2  # errors from before the plugin started: the baseline
    stub.write()
    hm = gpuinfo.HealthMonitor(root)
    assert hm.amdsmi_used
    st = hm.check(g.node_id, g.render_minor, g.bdf)
    assert st["healthy"] and st["amdsmi"] and st["ecc_uncorrectable"] == 2
    stub.gpus[g.render_minor]["uncorr"] = 3
    stub.write()
    st = hm.check(g.node_id, g.render_minor, g.bdf)
    assert not st["healthy"] and "uncorrectable ECC errors rose from 2 to 3" in st["reason"]
    stub.gpus[g.render_minor]["uncorr"] = 0  # GPU reset: counters cleared -> re-baseline
    stub.write()
    assert hm.check(g.node_id, g.render_minor, g.bdf)["healthy"]
    stub.gpus[g.render_minor]["links"] = "1101111"
    stub.write()
    st = hm.check(g.node_id, g.render_minor, g.bdf)
    assert not st["healthy"] and "xGMI link 2 down" in st["reason"]
    stub.gpus[g.render_minor]["links"] = "1111111"
    stub.write()
    assert hm.check(g.node_id, g.render_minor, g.bdf)["healthy"]
    # a tolerance lets a bounded number of new errors pass
    tol = gpuinfo.HealthMonitor(root, ecc_tolerance=2)
    assert tol.check(g.node_id, g.render_minor, g.bdf)["healthy"]
    stub.gpus[g.render_minor]["uncorr"] = 2
    stub.write()
    assert tol.check(g.node_id, g.render_minor, g.bdf)["healthy"]
    stub.gpus[g.render_minor]["uncorr"] = 3
    stub.write()
    assert not tol.check(g.node_id, g.render_minor, g.bdf)["healthy"]


def test_list_and_watch_flips_on_ecc_and_recovers(smi_host):
    """The plugin streams Unhealthy when amd-smi reports new uncorrectable errors
    on a device, refuses to allocate it, and re-advertises it after recovery."""
    import grpc

    root, stub, d = smi_host
    dpdir = os.path.join(d, "dp")
    kub = FakeKubelet(dpdir)
    kub.start()
    src = RealSource(root, use_amdsmi=True)
    plug = AmdGpuDevicePlugin(src, plugin_dir=dpdir, health_interval=0.1)
    try:
        plug.start()
        plug.register()
        plug.notify()
        assert kub.wait_capacity(4)
        assert not plug.health_tick()  # first tick takes the baselines: nothing flips
        dev = [x for x in src.devices() if x.render_minor == 144][0]
        stub.gpus[144]["uncorr"] = 1
        stub.write()
        assert plug.health_tick()
        assert kub.wait_health(dev.id, "Unhealthy")
        assert kub.capacity() == 3
        with pytest.raises(grpc.RpcError):
            kub.allocate([dev.id])
        from prometheus_client import generate_latest

        from kgs.deviceplugin.metrics import make_registry

        text = generate_latest(make_registry(plug)).decode()
        assert f'kgs_gpu_ecc_errors{{id="{dev.id}",kind="uncorrectable"}} 1.0' in text
        assert f'kgs_gpu_xgmi_links{{id="{dev.id}",state="up"}} 7.0' in text
        stub.gpus[144]["uncorr"] = 0  # reset
        stub.write()
        assert plug.health_tick()
        assert kub.wait_health(dev.id, "Healthy")
        assert kub.capacity() == 4
    finally:
        plug.stop()
        kub.stop()
