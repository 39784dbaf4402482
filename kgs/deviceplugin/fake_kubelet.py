"""A minimal kubelet device-manager stand-in, speaking real gRPC over a unix socket.

It serves ``v1beta1.Registration/Register`` on ``<dir>/kubelet.sock``; when a
plugin registers, it dials the plugin's endpoint, reads its options, and keeps
a ``ListAndWatch`` stream open, recording every device list it receives --
what the kubelet does to compute a node's ``amd.com/gpu`` capacity. Tests and
the on-GPU self-check drive ``allocate``/``preferred`` through it.

Simulating a kubelet restart (``restart()``) wipes the socket directory the way
the real kubelet does, which is what the plugin's re-registration logic keys on.
"""
from __future__ import annotations

import logging
import os
import threading
from concurrent import futures

import grpc

from . import api

log = logging.getLogger("kgs.fake_kubelet")


class FakeKubelet:
    def __init__(self, plugin_dir: str):
        self.dir = plugin_dir
        self.sock = os.path.join(plugin_dir, api.KUBELET_SOCKET)
        self.registrations: list = []
        self.device_lists: list = []      # every ListAndWatch update
        self.options = None
        self._server = None
        self._chan = None
        self._watch = None
        self._cv = threading.Condition()

    # --- Registration service ---
    def _register(self, req, context):
        if req.version != api.VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {req.version}")
        with self._cv:
            self.registrations.append(req)
            self._cv.notify_all()
        threading.Thread(target=self._connect_plugin, args=(req.endpoint,), daemon=True).start()
        return api.Empty()

    def _connect_plugin(self, endpoint: str) -> None:
        path = os.path.join(self.dir, endpoint)
        self._chan = grpc.insecure_channel(f"unix://{path}")
        opts = self._chan.unary_unary(api.method_path("DevicePlugin", "GetDevicePluginOptions"),
                                      request_serializer=api.Empty.SerializeToString,
                                      response_deserializer=api.DevicePluginOptions.FromString)
        try:
            self.options = opts(api.Empty(), timeout=5)
        except grpc.RpcError as e:  # pragma: no cover
            log.error("GetDevicePluginOptions failed: %s", e)
            return
        law = self._chan.unary_stream(api.method_path("DevicePlugin", "ListAndWatch"),
                                      request_serializer=api.Empty.SerializeToString,
                                      response_deserializer=api.ListAndWatchResponse.FromString)
        try:
            for resp in law(api.Empty()):
                with self._cv:
                    self.device_lists.append([(d.ID, d.health, [n.ID for n in d.topology.nodes])
                                              for d in resp.devices])
                    self._cv.notify_all()
        except grpc.RpcError:
            pass  # stream ends when the plugin stops or we restart

    def start(self) -> None:
        os.makedirs(self.dir, exist_ok=True)
        if os.path.exists(self.sock):
            os.unlink(self.sock)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        handler = grpc.method_handlers_generic_handler("v1beta1.Registration", {
            "Register": grpc.unary_unary_rpc_method_handler(
                self._register, request_deserializer=api.RegisterRequest.FromString,
                response_serializer=api.Empty.SerializeToString),
        })
        self._server.add_generic_rpc_handlers((handler,))
        self._server.add_insecure_port(f"unix://{self.sock}")
        self._server.start()

    def stop(self) -> None:
        if self._chan is not None:
            self._chan.close()
            self._chan = None
        if self._server is not None:
            self._server.stop(0).wait()
            self._server = None

    def restart(self) -> None:
        """Kubelet restart: stop, wipe every socket in the directory, start again."""
        self.stop()
        for n in os.listdir(self.dir):
            p = os.path.join(self.dir, n)
            if n.endswith(".sock") or os.path.basename(p) == api.KUBELET_SOCKET:
                try:
                    os.unlink(p)
                except OSError:
                    pass
        self.start()

    # --- helpers ---
    def wait(self, pred, timeout: float = 10.0) -> bool:
        with self._cv:
            return self._cv.wait_for(pred, timeout=timeout)

    def latest_devices(self):
        with self._cv:
            return self.device_lists[-1] if self.device_lists else None

    def capacity(self) -> int:
        d = self.latest_devices() or []
        return sum(1 for _, h, _ in d if h == api.HEALTHY)

    def health(self) -> dict:
        """{device id: health} of the latest list ({} before the first)."""
        return {i: h for i, h, _ in (self.latest_devices() or [])}

    # Waits key on the STATE the latest list shows, never on how many lists
    # arrived: the plugin's register() / notify() lists can land after a test
    # took a count, and a stale "Healthy" list then satisfies "one more list".
    def wait_health(self, dev_id: str, state: str, timeout: float = 10.0) -> bool:
        return self.wait(lambda: self.health().get(dev_id) == state, timeout=timeout)

    def wait_capacity(self, n: int, timeout: float = 10.0) -> bool:
        return self.wait(lambda: bool(self.device_lists) and self.capacity() == n, timeout=timeout)

    def _endpoint_channel(self):
        reg = self.registrations[-1]
        return grpc.insecure_channel(f"unix://{os.path.join(self.dir, reg.endpoint)}")

    def allocate(self, ids: list):
        with self._endpoint_channel() as ch:
            fn = ch.unary_unary(api.method_path("DevicePlugin", "Allocate"),
                                request_serializer=api.AllocateRequest.SerializeToString,
                                response_deserializer=api.AllocateResponse.FromString)
            req = api.AllocateRequest()
            req.container_requests.add(devices_ids=ids)
            return fn(req, timeout=5)

    def preferred(self, available: list, must: list, size: int):
        with self._endpoint_channel() as ch:
            fn = ch.unary_unary(api.method_path("DevicePlugin", "GetPreferredAllocation"),
                                request_serializer=api.PreferredAllocationRequest.SerializeToString,
                                response_deserializer=api.PreferredAllocationResponse.FromString)
            req = api.PreferredAllocationRequest()
            req.container_requests.add(available_deviceIDs=available, must_include_deviceIDs=must,
                                       allocation_size=size)
            return list(fn(req, timeout=5).container_responses[0].deviceIDs)
