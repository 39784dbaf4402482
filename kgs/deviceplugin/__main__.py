"""``python -m kgs.deviceplugin`` -- the amdgpu-dp-ds container entrypoint.

  --dev-root /            where host /dev and /sys are visible (DaemonSet mounts them)
  --plugin-dir DIR        kubelet device-plugin dir (hostPath /var/lib/kubelet/device-plugins)
  --partition-file F      render minors per node, written by `kgs create` (/etc/kgs/gpus.json)
  --node-name NAME        this node (downward API NODE_NAME)
  --fake-gpus N           advertise N simulated GPUs (CPU-only hosts, BASELINE config 1)
  --self-test             discover, print the Allocate response for every device and check
                          the device paths exist, then exit (used on the GPU box)
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import sys
import tempfile
import threading

from . import api
from .server import AmdGpuDevicePlugin, FakeSource, RealSource, load_partition, mark_ready


def _args(argv=None):
    ap = argparse.ArgumentParser(prog="kgs-deviceplugin", description="kgs amd.com/gpu device plugin")
    ap.add_argument("--resource", default=os.environ.get("KGS_RESOURCE", "amd.com/gpu"))
    ap.add_argument("--dev-root", default=os.environ.get("KGS_DEV_ROOT", "/"))
    ap.add_argument("--plugin-dir", default=os.environ.get("KGS_PLUGIN_DIR", api.DEVICE_PLUGIN_PATH))
    ap.add_argument("--partition-file", default=os.environ.get("KGS_PARTITION_FILE", "/etc/kgs/gpus.json"))
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME"))
    ap.add_argument("--fake-gpus", type=int, default=int(os.environ.get("KGS_FAKE_GPUS", "0") or 0))
    ap.add_argument("--health-interval", type=float, default=float(os.environ.get("KGS_HEALTH_INTERVAL", "5")))
    ap.add_argument("--no-amdsmi", action="store_true")
    ap.add_argument("--ready-file", default=os.environ.get("KGS_READY_FILE", "/tmp/kgs-dp-ready"))
    ap.add_argument("--metrics-port", type=int, default=int(os.environ.get("KGS_METRICS_PORT", "0") or 0),
                    help="serve Prometheus metrics on this port (0 = off)")
    ap.add_argument("--self-test", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    return ap.parse_args(argv)


def make_source(a):
    if a.fake_gpus > 0:
        return FakeSource(a.fake_gpus)
    allowed = load_partition(a.partition_file, a.node_name)
    return RealSource(a.dev_root, allowed, use_amdsmi=not a.no_amdsmi)


def _loaded(name: str) -> str:
    """Path of the first mapped shared object whose file name contains ``name``."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split(None, 5)[-1].strip()
                if name in os.path.basename(path):
                    return path
    except OSError:
        pass
    return ""


def self_test(a) -> int:
    """Serve on a private dir with the fake kubelet; Allocate every device."""
    from .fake_kubelet import FakeKubelet

    src = make_source(a)
    devs = src.devices()
    with tempfile.TemporaryDirectory(prefix="kgs-dp-") as d:
        kub = FakeKubelet(d)
        kub.start()
        plug = AmdGpuDevicePlugin(src, a.resource, plugin_dir=d)
        plug.start()
        plug.register()
        plug.notify()
        ok = kub.wait(lambda: bool(kub.device_lists), timeout=10)
        report = {"devices": [dv.__dict__ | {"xgmi_peers": sorted(dv.xgmi_peers)} for dv in devs],
                  "kubelet_saw": kub.latest_devices(), "capacity": kub.capacity(), "allocate": None,
                  "paths_exist": None,
                  # which amd-smi answered (the shipped image's lib/ or the host's)
                  "amdsmi_used": bool(getattr(src, "amdsmi_used", False)),
                  "amdsmi_library": getattr(src, "amdsmi_library", ""),
                  "amdsmi_loaded_from": _loaded("libamd_smi"),
                  "gpuinfo_loaded_from": _loaded("kgs_gpuinfo") or _loaded("_gpuinfo")}
        if ok and devs:
            resp = kub.allocate([dv.id for dv in devs])
            specs = [(s.container_path, s.host_path, s.permissions) for s in resp.container_responses[0].devices]
            report["allocate"] = {"devices": specs, "envs": dict(resp.container_responses[0].envs)}
            report["paths_exist"] = all(os.path.exists(os.path.join(a.dev_root, h.lstrip("/"))) for _, h, _ in specs)
        plug.stop()
        kub.stop()
    print(json.dumps(report, indent=1, default=str))
    good = ok and (report["paths_exist"] in (True, None)) and report["capacity"] == len(devs)
    return 0 if good else 1


def main(argv=None) -> int:
    a = _args(argv)
    logging.basicConfig(level=logging.DEBUG if a.verbose else logging.INFO,
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s", stream=sys.stderr)
    if a.self_test:
        return self_test(a)
    src = make_source(a)
    logging.getLogger("kgs.deviceplugin").info(
        "node=%s devices=%s", a.node_name, [(d.id, d.render_minor, d.healthy) for d in src.devices()])
    stop = threading.Event()
    if not src.devices() and a.fake_gpus <= 0:
        # A GPU-labelled worker that owns no GPU (all-on-first partition, or a
        # CPU-only host using the reference's patched fake capacity): registering
        # an empty amd.com/gpu list would make the kubelet zero the capacity, so
        # stay idle (and Ready) instead.
        logging.getLogger("kgs.deviceplugin").info("no GPUs for this node; idle (not registering)")
        mark_ready(a.ready_file, {"state": "idle", "devices": 0})
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        signal.signal(signal.SIGINT, lambda *_: stop.set())
        while not stop.wait(3600):
            pass
        return 0
    plug = AmdGpuDevicePlugin(src, a.resource, plugin_dir=a.plugin_dir, health_interval=a.health_interval,
                              ready_file=a.ready_file)
    if a.metrics_port:
        from .metrics import serve

        serve(plug, a.metrics_port)

    def _term(signum, frame):
        plug.stop()

    signal.signal(signal.SIGTERM, _term)
    signal.signal(signal.SIGINT, _term)
    try:
        plug.serve_forever()
    finally:
        plug.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
