"""Device plugin (T2 of SURVEY.md §4): real gRPC over unix sockets against a
fake kubelet, on a fake 8 x MI355X sysfs tree and on the captured box tree."""
import os
import tempfile
import threading
import time

import grpc
import pytest

from kgs.deviceplugin import api
from kgs.deviceplugin.fake_kubelet import FakeKubelet
from kgs.deviceplugin.server import AmdGpuDevicePlugin, FakeSource, RealSource, load_partition
from kgs.gpuinfo.fake import make_fake_mi355x, remove_gpu_device, restore_gpu_device

FIXTURE_BOX = os.path.join(os.path.dirname(__file__), "fixtures", "kfd_box1")


@pytest.fixture
def short_tmp():
    # unix socket paths must stay < 108 bytes
    d = tempfile.mkdtemp(prefix="kgs", dir="/tmp")
    yield d
    import shutil

    shutil.rmtree(d, ignore_errors=True)


@pytest.fixture
def host8(short_tmp):
    return str(make_fake_mi355x(os.path.join(short_tmp, "host")))


@pytest.fixture
def cluster(short_tmp, host8):
    dpdir = os.path.join(short_tmp, "dp")
    kub = FakeKubelet(dpdir)
    kub.start()
    src = RealSource(host8, use_amdsmi=False)
    plug = AmdGpuDevicePlugin(src, plugin_dir=dpdir, health_interval=0.1)
    plug.start()
    plug.register()
    plug.notify()
    assert kub.wait_capacity(8)
    yield kub, plug, src, host8
    plug.stop()
    kub.stop()


def test_register_and_list_and_watch(cluster):
    kub, plug, src, _ = cluster
    reg = kub.registrations[-1]
    assert reg.version == "v1beta1"
    assert reg.resource_name == "amd.com/gpu"
    assert reg.endpoint == "kgs-amdgpu.sock"
    assert reg.options.get_preferred_allocation_available
    assert kub.options.get_preferred_allocation_available and not kub.options.pre_start_required
    devs = kub.latest_devices()
    assert len(devs) == 8 and kub.capacity() == 8
    assert all(h == "Healthy" for _, h, _ in devs)
    # NUMA topology hints: 4 GPUs per socket
    assert sorted(n[0] for _, _, n in devs) == [0, 0, 0, 0, 1, 1, 1, 1]


def test_allocate_gives_kfd_and_render_nodes(cluster):
    kub, plug, src, host = cluster
    ids = [d.id for d in src.devices()][:2]
    resp = kub.allocate(ids)
    c = resp.container_responses[0]
    paths = [(s.container_path, s.host_path, s.permissions) for s in c.devices]
    assert paths[0] == ("/dev/kfd", "/dev/kfd", "rw")
    assert ("/dev/dri/renderD128", "/dev/dri/renderD128", "rw") in paths
    assert ("/dev/dri/renderD136", "/dev/dri/renderD136", "rw") in paths
    assert len(paths) == 3
    assert c.envs["KGS_RENDER_MINORS"] == "128,136"
    assert c.annotations["kgs.amd.com/gpus"] == ",".join(ids)
    for _, h, _ in paths:
        assert os.path.exists(os.path.join(host, h.lstrip("/")))


def test_allocate_pins_rocr_to_the_allocated_gpus_by_uuid(cluster):
    """Allocate of renderD136 returns exactly that GPU's
    ROCr UUID (GPU-<KFD unique_id as 16 hex digits>), so even a privileged
    container -- which sees every render node of its worker -- runs on it; an
    8-GPU allocation lists all eight, in the same order as KGS_RENDER_MINORS."""
    kub, plug, src, host = cluster
    d136 = next(d for d in src.devices() if d.render_minor == 136)
    c = kub.allocate([d136.id]).container_responses[0]
    assert c.envs["KGS_RENDER_MINORS"] == "136"
    # fake tree: unique_id = 0xA6FF75A300000000 + index (kgs/gpuinfo/fake.py)
    assert c.envs["ROCR_VISIBLE_DEVICES"] == f"GPU-{0xA6FF75A300000000 + d136.index:016x}" == "GPU-a6ff75a300000001"
    ids = [d.id for d in src.devices()]
    c8 = kub.allocate(list(reversed(ids))).container_responses[0]  # kubelet order does not matter
    uu = c8.envs["ROCR_VISIBLE_DEVICES"].split(",")
    assert uu == [f"GPU-{0xA6FF75A300000000 + i:016x}" for i in range(8)]
    assert c8.envs["KGS_RENDER_MINORS"] == ",".join(str(128 + 8 * i) for i in range(8))
    assert len(set(uu)) == 8


def test_allocate_without_unique_id_sets_no_index_pin(short_tmp):
    """A GPU without a KFD unique_id cannot be pinned by UUID; Allocate then
    sets no ROCR_VISIBLE_DEVICES at all rather than an index list (which would
    name other GPUs in a privileged container)."""
    host = make_fake_mi355x(os.path.join(short_tmp, "h0"), n_gpus=2)
    for p in (host / "sys/class/kfd/kfd/topology/nodes").glob("*/properties"):
        p.write_text("".join(ln if not ln.startswith("unique_id ") else "unique_id 0\n"
                             for ln in p.read_text().splitlines(keepends=True)))
    dpdir = os.path.join(short_tmp, "dp0")
    kub = FakeKubelet(dpdir)
    kub.start()
    src = RealSource(str(host), use_amdsmi=False)
    plug = AmdGpuDevicePlugin(src, plugin_dir=dpdir)
    plug.start()
    plug.register()
    try:
        c = kub.allocate([src.devices()[0].id]).container_responses[0]
        assert "ROCR_VISIBLE_DEVICES" not in c.envs and c.envs["KGS_RENDER_MINORS"] == "128"
    finally:
        plug.stop()
        kub.stop()


def test_allocate_unknown_device_rejected(cluster):
    kub, *_ = cluster
    with pytest.raises(grpc.RpcError) as ei:
        kub.allocate(["0000:ff:00.0"])
    assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_health_flip_streams_unhealthy_then_recovers(cluster):
    kub, plug, src, host = cluster
    sick = [d.id for d in src.devices() if d.render_minor == 144][0]
    remove_gpu_device(host, 144)
    assert plug.health_tick()
    assert kub.wait_health(sick, "Unhealthy")
    assert kub.capacity() == 7
    with pytest.raises(grpc.RpcError) as ei:
        kub.allocate([sick])
    assert ei.value.code() == grpc.StatusCode.FAILED_PRECONDITION
    restore_gpu_device(host, 144)
    assert plug.health_tick()
    assert kub.wait_health(sick, "Healthy")
    assert kub.capacity() == 8
    assert not plug.health_tick()  # no change -> no update


def test_kfd_loss_marks_all_unhealthy(cluster):
    kub, plug, src, host = cluster
    os.unlink(os.path.join(host, "dev/kfd"))
    assert plug.health_tick()
    assert kub.wait_capacity(0)


def test_preferred_allocation_packs_numa(cluster):
    kub, plug, src, _ = cluster
    ids = [d.id for d in src.devices()]
    # 4 GPUs from all 8: one socket
    got = kub.preferred(ids, [], 4)
    numas = {d.numa for d in src.devices() if d.id in got}
    assert len(got) == 4 and len(numas) == 1
    # must-include a socket-1 GPU -> the rest come from socket 1
    got = kub.preferred(ids, [ids[5]], 4)
    assert ids[5] in got and {d.numa for d in src.devices() if d.id in got} == {1}
    got = kub.preferred(ids, [], 8)
    assert sorted(got) == sorted(ids)


def test_kubelet_restart_reregisters(short_tmp, host8):
    dpdir = os.path.join(short_tmp, "dp")
    kub = FakeKubelet(dpdir)
    kub.start()
    plug = AmdGpuDevicePlugin(RealSource(host8, use_amdsmi=False), plugin_dir=dpdir, health_interval=0.2)
    t = threading.Thread(target=plug.serve_forever, kwargs={"poll": 0.05}, daemon=True)
    t.start()
    try:
        assert kub.wait(lambda: len(kub.registrations) == 1 and bool(kub.device_lists), timeout=15)
        kub.restart()
        assert kub.wait(lambda: len(kub.registrations) >= 2, timeout=15)
        assert kub.wait_capacity(8, timeout=15)
        deadline = time.monotonic() + 10
        while plug.registrations < 2 and time.monotonic() < deadline:
            time.sleep(0.05)
        assert plug.registrations >= 2
    finally:
        plug.stop()
        t.join(timeout=10)
        kub.stop()


def test_partition_filtering(short_tmp, host8):
    import json

    pf = os.path.join(short_tmp, "gpus.json")
    with open(pf, "w") as f:
        json.dump({"nodes": {"c-worker": [128, 136, 144, 152], "c-worker2": [160, 168, 176, 184],
                             "c-worker3": []}}, f)
    a = load_partition(pf, "c-worker")
    b = load_partition(pf, "c-worker2")
    assert a == {128, 136, 144, 152} and b == {160, 168, 176, 184}
    assert load_partition(pf, "c-worker3") == set()
    assert load_partition(pf, "unknown-node") == set()
    assert load_partition(None, "x") is None
    src = RealSource(host8, a, use_amdsmi=False)
    assert [d.render_minor for d in src.devices()] == [128, 136, 144, 152]
    os.environ["KGS_ALLOWED_RENDER_MINORS"] = "184"
    try:
        assert load_partition(pf, "c-worker") == {184}
    finally:
        del os.environ["KGS_ALLOWED_RENDER_MINORS"]


def test_captured_box_tree():
    src = RealSource(FIXTURE_BOX, use_amdsmi=False)
    devs = src.devices()
    assert len(devs) == 1
    d = devs[0]
    assert d.render_minor == 144 and d.id == "0000:5a:00.0" and d.healthy
    assert d.meta["gfx"] == "gfx950" and d.meta["cus"] == 256 and d.meta["vram_gib"] == 288.0


def test_fake_source_plugin(short_tmp):
    dpdir = os.path.join(short_tmp, "dp")
    kub = FakeKubelet(dpdir)
    kub.start()
    src = FakeSource(2)
    plug = AmdGpuDevicePlugin(src, plugin_dir=dpdir)
    plug.start()
    plug.register()
    plug.notify()
    try:
        assert kub.wait_capacity(2)
        r = kub.allocate(["fake-amdgpu-0"])
        assert len(r.container_responses[0].devices) == 0
        assert r.container_responses[0].envs["KGS_FAKE_GPUS"] == "fake-amdgpu-0"
        src.set_unhealthy("fake-amdgpu-1")
        assert plug.health_tick()
        assert kub.wait_health("fake-amdgpu-1", "Unhealthy")
        assert kub.capacity() == 1
    finally:
        plug.stop()
        kub.stop()


def test_register_rejects_wrong_version(short_tmp):
    dpdir = os.path.join(short_tmp, "dp")
    kub = FakeKubelet(dpdir)
    kub.start()
    try:
        with grpc.insecure_channel(f"unix://{kub.sock}") as ch:
            stub = ch.unary_unary(api.method_path("Registration", "Register"),
                                  request_serializer=api.RegisterRequest.SerializeToString,
                                  response_deserializer=api.Empty.FromString)
            with pytest.raises(grpc.RpcError):
                stub(api.RegisterRequest(version="v1alpha", endpoint="x", resource_name="amd.com/gpu"), timeout=5)
    finally:
        kub.stop()


def test_self_test_cli(host8, capsys):
    from kgs.deviceplugin.__main__ import main

    rc = main(["--self-test", "--dev-root", host8, "--no-amdsmi", "--partition-file", "/nonexistent"])
    out = capsys.readouterr().out
    assert rc == 0, out
    assert '"capacity": 8' in out and '"paths_exist": true' in out


def test_serve_forever_stops_promptly(short_tmp, host8):
    dpdir = os.path.join(short_tmp, "dp")
    kub = FakeKubelet(dpdir)
    kub.start()
    plug = AmdGpuDevicePlugin(RealSource(host8, use_amdsmi=False), plugin_dir=dpdir)
    t = threading.Thread(target=plug.serve_forever, kwargs={"poll": 0.05}, daemon=True)
    t.start()
    assert kub.wait(lambda: bool(kub.device_lists), timeout=15)
    t0 = time.monotonic()
    plug.stop()
    t.join(timeout=10)
    assert not t.is_alive() and time.monotonic() - t0 < 10
    assert not os.path.exists(plug.socket_path)
    kub.stop()


def test_prometheus_metrics(cluster):
    from prometheus_client import generate_latest

    from kgs.deviceplugin.metrics import make_registry

    kub, plug, src, host = cluster
    kub.allocate([src.devices()[0].id])
    remove_gpu_device(host, 136)
    plug.health_tick()
    text = generate_latest(make_registry(plug)).decode()
    assert 'kgs_deviceplugin_devices{health="Healthy"} 7.0' in text
    assert 'kgs_deviceplugin_devices{health="Unhealthy"} 1.0' in text
    assert "kgs_deviceplugin_allocations_total 1.0" in text
    assert "kgs_deviceplugin_registrations_total 1.0" in text
    assert "kgs_deviceplugin_health_flips_total 1.0" in text
    assert 'render_minor="136"' in text


def test_entrypoint_does_not_assume_isolation(host8):
    """The pod entrypoint on a privileged worker view (all 8 render nodes
    visible): its allocation is what Allocate named, and the children it starts
    are pinned to exactly those GPUs by UUID, in HIP device order."""
    from kgs.workload.entrypoint import allocated_gpus, pinned_env

    everything = allocated_gpus(host8, environ={})
    assert len(everything) == 8  # no allocation envs: what is visible
    env = {"KGS_RENDER_MINORS": "144,136"}
    got = allocated_gpus(host8, environ=env)
    assert sorted(g.render_minor for g in got) == [136, 144]
    pin = pinned_env(got, environ=env)["ROCR_VISIBLE_DEVICES"]
    assert pin == ",".join(g.rocr_uuid for g in got) and pin.count("GPU-") == 2
    # Allocate's own pin (upper-case hex is the same UUID) wins and sets the order
    env = {"ROCR_VISIBLE_DEVICES": "GPU-A6FF75A300000007,GPU-a6ff75a300000002"}
    got = allocated_gpus(host8, environ=env)
    assert [g.render_minor for g in got] == [184, 144]
    assert pinned_env(got, environ=env)["ROCR_VISIBLE_DEVICES"] == env["ROCR_VISIBLE_DEVICES"]
    # an index list is not a pin: replaced by the UUIDs
    assert pinned_env(got, environ={"ROCR_VISIBLE_DEVICES": "0,1"})["ROCR_VISIBLE_DEVICES"] == \
        "GPU-a6ff75a300000007,GPU-a6ff75a300000002"
    assert allocated_gpus(host8, environ={"KGS_FAKE_GPUS": "fake-amdgpu-0"}) == []


def test_fake_kubelet_waits_on_state_not_list_count(short_tmp):
    """a wait keyed on "one more list than before" returned
    on the plugin's own late register()/notify() list (still Healthy). The
    state waits only return once the latest list shows the state."""
    kub = FakeKubelet(os.path.join(short_tmp, "dpw"))
    healthy = [("gpu-0", "Healthy", [0]), ("gpu-1", "Healthy", [0])]
    kub.device_lists.append(healthy)

    def feed():
        time.sleep(0.1)
        with kub._cv:  # the stale list lands first ...
            kub.device_lists.append(list(healthy))
            kub._cv.notify_all()
        time.sleep(0.2)
        with kub._cv:  # ... then the flip
            kub.device_lists.append([("gpu-0", "Healthy", [0]), ("gpu-1", "Unhealthy", [0])])
            kub._cv.notify_all()

    t = threading.Thread(target=feed)
    t0 = time.monotonic()
    t.start()
    assert kub.wait_health("gpu-1", "Unhealthy", timeout=5)
    assert time.monotonic() - t0 >= 0.25 and kub.capacity() == 1
    assert kub.wait_capacity(1, timeout=0.1) and not kub.wait_capacity(2, timeout=0.1)
    t.join()
