"""From-scratch kubelet device plugin advertising real ``amd.com/gpu`` devices.

Lifecycle (kubelet device-plugin protocol v1beta1):

1. discover GPUs with the native core (:mod:`kgs.gpuinfo`), keep the ones this
   node owns (partition file written by ``kgs create``);
2. serve ``v1beta1.DevicePlugin`` on ``<plugin-dir>/kgs-amdgpu.sock``;
3. ``Register`` with the kubelet on ``<plugin-dir>/kubelet.sock``;
4. stream the device list on ``ListAndWatch`` and re-send it whenever a GPU's
   health flips (device nodes present + KFD node alive, plus amd-smi
   uncorrectable-ECC count and xGMI link status against a baseline; polled);
5. on ``Allocate`` hand the container ``/dev/kfd`` and the allocated
   ``/dev/dri/renderD<minor>`` nodes, plus ``ROCR_VISIBLE_DEVICES=GPU-<uuid>,...``
   for exactly those GPUs. The device nodes isolate an unprivileged container
   (ROCr only enumerates GPUs whose render node it can open); the UUIDs also pin
   a privileged one, which sees every render node of its worker;
6. ``GetPreferredAllocation`` keeps multi-GPU pods on one xGMI island / NUMA
   node (:mod:`kgs.deviceplugin.allocator`);
7. if the kubelet restarts (it wipes the plugin directory) the plugin notices
   its socket is gone, restarts its server and re-registers.

The reference deploys the upstream Go plugin without the
``/var/lib/kubelet/device-plugins`` mount (kind-gpu-sim.sh:248-276), so it can
never register; capacity there only comes from the status patch (:113).
"""
from __future__ import annotations

import json
import logging
import os
import socket
import threading
import time
from concurrent import futures
from dataclasses import dataclass, field

import grpc

from . import api
from .allocator import DevInfo, preferred

log = logging.getLogger("kgs.deviceplugin")

RESOURCE_NAME = "amd.com/gpu"
SOCKET_NAME = "kgs-amdgpu.sock"


@dataclass
class PluginDevice:
    id: str
    index: int
    numa: int = -1
    node_id: int = -1
    render_minor: int = -1
    healthy: bool = True
    reason: str = "ok"
    xgmi_peers: frozenset = frozenset()
    fake: bool = False
    meta: dict = field(default_factory=dict)


# ------------------------------------------------------------------ sources --
class RealSource:
    """GPUs from the native gpuinfo core, filtered to this node's partition."""

    def __init__(self, root: str = "/", allowed_minors: set | None = None, use_amdsmi: bool = True):
        from kgs import gpuinfo

        self.root = root
        self.allowed = allowed_minors
        self.use_amdsmi = use_amdsmi
        self._devs: list[PluginDevice] = []
        # stateful: ECC / xGMI baselines are taken at the first health tick
        self.monitor = gpuinfo.HealthMonitor(root, use_amdsmi=use_amdsmi)
        self.last_sample: dict = {}
        self.rescan()

    def rescan(self) -> None:
        from kgs import gpuinfo

        topo = gpuinfo.discover(self.root, use_amdsmi=self.use_amdsmi)
        self.amdsmi_used = topo.amdsmi_used
        self.amdsmi_library = topo.amdsmi_library
        devs = []
        for g in topo.gpus:
            if g.render_minor < 0:
                continue  # unreadable node: not ours to offer
            if self.allowed is not None and g.render_minor not in self.allowed:
                continue
            devs.append(PluginDevice(
                id=g.device_id_str, index=g.index, numa=g.numa_node, node_id=g.node_id,
                render_minor=g.render_minor, healthy=g.healthy, reason=g.health_reason,
                xgmi_peers=frozenset(g.xgmi_peers()),
                meta={"gfx": g.gfx_arch, "cus": g.cu_count, "vram_gib": round(g.vram_bytes / 2**30, 1),
                      "uuid": g.uuid, "bdf": g.bdf, "rocr_uuid": g.rocr_uuid},
            ))
        self._devs = devs

    def devices(self) -> list:
        return list(self._devs)

    def refresh(self) -> bool:
        """Re-evaluate health (sysfs + amd-smi ECC / xGMI against the baseline);
        True if any device changed state."""
        changed = False
        for d in self._devs:
            st = self.monitor.check(d.node_id, d.render_minor, d.meta.get("bdf", ""))
            self.last_sample[d.id] = st
            ok, why = bool(st["healthy"]), st["reason"]
            if ok != d.healthy:
                log.warning("device %s (renderD%d) health %s -> %s: %s", d.id, d.render_minor,
                            d.healthy, ok, why)
                changed = True
            d.healthy, d.reason = ok, why
        return changed

    def device_specs(self, d: PluginDevice) -> list:
        return [api.DeviceSpec(container_path=f"/dev/dri/renderD{d.render_minor}",
                               host_path=f"/dev/dri/renderD{d.render_minor}", permissions="rw")]

    common_specs = [api.DeviceSpec(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")]


class FakeSource:
    """N simulated GPUs (the reference's fake capacity, served through a real
    plugin instead of a status patch). Allocate hands out no device nodes."""

    def __init__(self, n: int, numa_split: int = 2):
        self._devs = [PluginDevice(id=f"fake-amdgpu-{i}", index=i, numa=(i * numa_split) // max(1, n),
                                   fake=True) for i in range(n)]
        self._fail: set = set()

    def devices(self) -> list:
        return list(self._devs)

    def set_unhealthy(self, dev_id: str, unhealthy: bool = True) -> None:
        (self._fail.add if unhealthy else self._fail.discard)(dev_id)

    def refresh(self) -> bool:
        changed = False
        for d in self._devs:
            ok = d.id not in self._fail
            if ok != d.healthy:
                changed = True
            d.healthy, d.reason = ok, "ok" if ok else "fault injected"
        return changed

    def device_specs(self, d):
        return []

    common_specs: list = []


def load_partition(path: str | None, node_name: str | None) -> set | None:
    """Render minors this node may advertise, from ``kgs create``'s partition
    file ``{"nodes": {"<node>": [minors...]}}``. None = no restriction."""
    env = os.environ.get("KGS_ALLOWED_RENDER_MINORS")
    if env is not None:
        return {int(x) for x in env.replace(",", " ").split()}
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        data = json.load(f)
    nodes = data.get("nodes", {})
    if node_name and node_name in nodes:
        return set(nodes[node_name])
    if node_name and nodes:
        return set()  # partitioned host, this node owns nothing
    return None


def mark_ready(path: str | None, status: dict) -> None:
    """Readiness file for the DaemonSet probe (registered, or idle by design)."""
    if not path:
        return
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(status, f)
    os.replace(tmp, path)


def _wait_listening(path: str, timeout: float) -> None:
    deadline = time.monotonic() + timeout
    delay = 0.0005
    while True:
        with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
            try:
                s.connect(path)
                return
            except OSError:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"plugin socket {path} not accepting connections")
        time.sleep(delay)
        delay = min(delay * 2, 0.05)


# ------------------------------------------------------------------- plugin --
class AmdGpuDevicePlugin:
    def __init__(self, source, resource_name: str = RESOURCE_NAME, plugin_dir: str = api.DEVICE_PLUGIN_PATH,
                 socket_name: str = SOCKET_NAME, health_interval: float = 5.0, kubelet_socket: str | None = None,
                 ready_file: str | None = None):
        self.source = source
        self.ready_file = ready_file
        self.resource_name = resource_name
        self.plugin_dir = plugin_dir
        self.socket_name = socket_name
        self.socket_path = os.path.join(plugin_dir, socket_name)
        self.kubelet_socket = kubelet_socket or os.path.join(plugin_dir, api.KUBELET_SOCKET)
        self.health_interval = health_interval
        self._server = None
        self._cv = threading.Condition()
        self._version = 0          # bumps on every device-list change
        self._stop = threading.Event()
        # serialises stop() with serve_forever's restart; re-entrant because
        # stop() also runs from a SIGTERM handler on the serving thread
        self._life = threading.RLock()
        self.registrations = 0
        self.allocations = 0
        self.health_flips = 0

    # ---- gRPC service ---------------------------------------------------------
    def GetDevicePluginOptions(self, request, context):
        return api.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def _device_msgs(self):
        out = []
        for d in self.source.devices():
            msg = api.Device(ID=d.id, health=api.HEALTHY if d.healthy else api.UNHEALTHY)
            if d.numa >= 0:
                msg.topology.nodes.add(ID=d.numa)
            out.append(msg)
        return out

    def ListAndWatch(self, request, context):
        log.info("ListAndWatch: stream opened (%d devices)", len(self.source.devices()))
        seen = -1
        while not self._stop.is_set() and context.is_active():
            with self._cv:
                if seen == self._version:
                    self._cv.wait(timeout=1.0)
                    if seen == self._version:
                        continue
                seen = self._version
            yield api.ListAndWatchResponse(devices=self._device_msgs())
        log.info("ListAndWatch: stream closed")

    def GetPreferredAllocation(self, request, context):
        infos = {d.id: DevInfo(d.id, d.index, d.numa, d.node_id, d.xgmi_peers) for d in self.source.devices()}
        resp = api.PreferredAllocationResponse()
        for cr in request.container_requests:
            ids = preferred(cr.available_deviceIDs, cr.must_include_deviceIDs, cr.allocation_size, infos)
            resp.container_responses.add(deviceIDs=ids)
            log.info("GetPreferredAllocation: size=%d avail=%d -> %s", cr.allocation_size,
                     len(cr.available_deviceIDs), ids)
        return resp

    def Allocate(self, request, context):
        devs = {d.id: d for d in self.source.devices()}
        resp = api.AllocateResponse()
        for cr in request.container_requests:
            ids = list(cr.devices_ids)
            unknown = [i for i in ids if i not in devs]
            if unknown:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown device ids {unknown}")
            sick = [i for i in ids if not devs[i].healthy]
            if sick:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, f"unhealthy devices {sick}")
            # HIP device i of the container is the i-th GPU by KFD order, in
            # every list below (render minors, ROCr UUIDs)
            ids.sort(key=lambda i: devs[i].index)
            car = resp.container_responses.add()
            car.devices.extend(self.source.common_specs)
            minors = []
            for i in ids:
                car.devices.extend(self.source.device_specs(devs[i]))
                minors.append(str(devs[i].render_minor))
            car.envs["KGS_GPU_IDS"] = ",".join(ids)
            if any(devs[i].fake for i in ids):
                car.envs["KGS_FAKE_GPUS"] = ",".join(ids)
            else:
                car.envs["KGS_RENDER_MINORS"] = ",".join(minors)
                # Pin ROCr to exactly these GPUs by UUID. The device nodes
                # alone isolate an unprivileged container, but a privileged one
                # gets every /dev/dri node of its kind worker; an index list
                # would name other GPUs there, a UUID cannot.
                uuids = [devs[i].meta.get("rocr_uuid", "") for i in ids]
                if all(uuids):
                    car.envs["ROCR_VISIBLE_DEVICES"] = ",".join(uuids)
                else:
                    log.warning("Allocate %s: no KFD unique_id for %s; ROCR_VISIBLE_DEVICES not set, "
                                "only the device nodes isolate this container", ids,
                                [i for i, u in zip(ids, uuids) if not u])
            car.annotations["kgs.amd.com/gpus"] = ",".join(ids)
            self.allocations += 1
            log.info("Allocate: %s -> %s", ids, [d.host_path for d in car.devices])
        return resp

    def PreStartContainer(self, request, context):
        return api.PreStartContainerResponse()

    # ---- server / registration -----------------------------------------------
    def _handlers(self):
        def uu(fn, req, resp):
            return grpc.unary_unary_rpc_method_handler(fn, request_deserializer=req.FromString,
                                                       response_serializer=resp.SerializeToString)

        return grpc.method_handlers_generic_handler("v1beta1.DevicePlugin", {
            "GetDevicePluginOptions": uu(self.GetDevicePluginOptions, api.Empty, api.DevicePluginOptions),
            "ListAndWatch": grpc.unary_stream_rpc_method_handler(
                self.ListAndWatch, request_deserializer=api.Empty.FromString,
                response_serializer=api.ListAndWatchResponse.SerializeToString),
            "GetPreferredAllocation": uu(self.GetPreferredAllocation, api.PreferredAllocationRequest,
                                         api.PreferredAllocationResponse),
            "Allocate": uu(self.Allocate, api.AllocateRequest, api.AllocateResponse),
            "PreStartContainer": uu(self.PreStartContainer, api.PreStartContainerRequest,
                                    api.PreStartContainerResponse),
        })

    def start(self) -> None:
        os.makedirs(self.plugin_dir, exist_ok=True)
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=16))
        self._server.add_generic_rpc_handlers((self._handlers(),))
        self._server.add_insecure_port(f"unix://{self.socket_path}")
        self._server.start()
        # wait until the socket accepts (the kubelet dials it right after
        # Register). A raw unix-socket connect answers in ~0.1 ms; gRPC's
        # channel_ready_future polls connectivity and took ~200 ms here, on the
        # create -> plugin-Ready path (profiles/e2e_components.json).
        _wait_listening(self.socket_path, timeout=10.0)
        log.info("serving %s on %s", self.resource_name, self.socket_path)

    def stop(self, grace: float = 1.0) -> None:
        with self._life:
            self._stop.set()
            with self._cv:
                self._cv.notify_all()
            if self._server is not None:
                self._server.stop(grace).wait()
                self._server = None
        if os.path.exists(self.socket_path):
            try:
                os.unlink(self.socket_path)
            except OSError:
                pass

    def register(self, timeout: float = 10.0) -> None:
        req = api.RegisterRequest(
            version=api.VERSION, endpoint=self.socket_name, resource_name=self.resource_name,
            options=api.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True),
        )
        with grpc.insecure_channel(f"unix://{self.kubelet_socket}") as ch:
            stub = ch.unary_unary(api.method_path("Registration", "Register"),
                                  request_serializer=api.RegisterRequest.SerializeToString,
                                  response_deserializer=api.Empty.FromString)
            stub(req, timeout=timeout)
        self.registrations += 1
        log.info("registered %s with kubelet (%s)", self.resource_name, self.kubelet_socket)

    def notify(self) -> None:
        with self._cv:
            self._version += 1
            self._cv.notify_all()

    def health_tick(self) -> bool:
        changed = self.source.refresh()
        if changed:
            self.health_flips += 1
            self.notify()
        return changed

    def _kubelet_id(self):
        try:
            st = os.stat(self.kubelet_socket)
            return (st.st_ino, st.st_ctime_ns)
        except FileNotFoundError:
            return None

    def serve_forever(self, poll: float = 1.0) -> None:
        """Start, register and keep registered until stop()."""
        self.start()
        self._wait_kubelet_and_register()
        kubelet_id = self._kubelet_id()
        next_health = time.monotonic() + self.health_interval
        while not self._stop.is_set():
            self._stop.wait(poll)
            if self._stop.is_set():
                break
            if time.monotonic() >= next_health:
                self.health_tick()
                next_health = time.monotonic() + self.health_interval
            cur = self._kubelet_id()
            if not os.path.exists(self.socket_path) or (cur is not None and cur != kubelet_id):
                log.warning("kubelet restarted (socket %s); re-registering",
                            "gone" if not os.path.exists(self.socket_path) else "changed")
                with self._life:  # a stop() now either precedes the restart or tears it down
                    if self._server is not None:
                        self._server.stop(0).wait()
                        self._server = None
                    if self._stop.is_set():  # stop() raced the restart: do not come back up
                        break
                    self.start()
                if self._stop.is_set():  # stop() ran inside the block (signal on this thread)
                    self.stop(0)
                    break
                self._wait_kubelet_and_register()
                kubelet_id = self._kubelet_id()

    def _wait_kubelet_and_register(self) -> None:
        delay = 0.2
        while not self._stop.is_set():
            try:
                self.register()
                self.notify()
                mark_ready(self.ready_file, {"state": "registered", "resource": self.resource_name,
                                             "devices": len(self.source.devices())})
                return
            except grpc.RpcError as e:
                log.warning("kubelet registration failed (%s); retrying in %.1fs", e.code() if hasattr(e, "code")
                            else e, delay)
                self._stop.wait(delay)
                delay = min(delay * 2, 5.0)
