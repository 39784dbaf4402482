#!/usr/bin/env python3
"""Where the device plugin's start-up time goes (the `plugin-process-start`
phase of `kgs bench --no-kind`): imports, KFD discovery, amd-smi discovery and
the health monitor's baseline, each timed on its own. Prints one JSON line."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    t = {}
    t0 = time.perf_counter()
    from kgs.deviceplugin import server  # noqa: F401  (grpc + protobuf descriptors)

    t["import_server_s"] = time.perf_counter() - t0
    from kgs import gpuinfo

    for smi in (False, True):
        t1 = time.perf_counter()
        topo = gpuinfo.discover("/", use_amdsmi=smi)
        t[f"discover_amdsmi_{int(smi)}_s"] = time.perf_counter() - t1
        t[f"gpus_amdsmi_{int(smi)}"] = len(topo.gpus)
    t1 = time.perf_counter()
    mon = gpuinfo.HealthMonitor("/", use_amdsmi=True)
    t["health_monitor_init_s"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    src = server.RealSource("/", None, use_amdsmi=True)
    t["real_source_s"] = time.perf_counter() - t1
    t["devices"] = [d.id for d in src.devices()]
    del mon
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in t.items()}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
