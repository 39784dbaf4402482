"""Prometheus metrics for the device plugin (``--metrics-port``).

Exposed gauges/counters are computed at scrape time from the plugin's state:

  kgs_deviceplugin_devices{health="Healthy"|"Unhealthy"}   advertised amd.com/gpu
  kgs_deviceplugin_device_healthy{id,render_minor,numa}     1/0 per device
  kgs_deviceplugin_allocations_total                        Allocate container responses
  kgs_deviceplugin_registrations_total                      kubelet registrations
  kgs_deviceplugin_health_flips_total                       health transitions streamed
  kgs_gpu_ecc_errors{id,kind=correctable|uncorrectable|deferred}   amd-smi totals (last health tick)
  kgs_gpu_xgmi_links{id,state=up|down}                      amd-smi xGMI link status (last health tick)

The reference has no observability beyond ``echo``.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily


class PluginCollector:
    def __init__(self, plugin):
        self.plugin = plugin

    def collect(self):
        devs = self.plugin.source.devices()
        g = GaugeMetricFamily("kgs_deviceplugin_devices", "amd.com/gpu devices advertised", labels=["health"])
        healthy = sum(1 for d in devs if d.healthy)
        g.add_metric(["Healthy"], healthy)
        g.add_metric(["Unhealthy"], len(devs) - healthy)
        yield g
        per = GaugeMetricFamily("kgs_deviceplugin_device_healthy", "1 if the device is healthy",
                                labels=["id", "render_minor", "numa"])
        for d in devs:
            per.add_metric([d.id, str(d.render_minor), str(d.numa)], 1.0 if d.healthy else 0.0)
        yield per
        samples = getattr(self.plugin.source, "last_sample", {}) or {}
        ecc = GaugeMetricFamily("kgs_gpu_ecc_errors", "amd-smi accumulated ECC error counts", labels=["id", "kind"])
        links = GaugeMetricFamily("kgs_gpu_xgmi_links", "amd-smi xGMI link status", labels=["id", "state"])
        for dev_id, st in sorted(samples.items()):
            if not st.get("amdsmi"):
                continue
            for kind in ("correctable", "uncorrectable", "deferred"):
                v = st.get(f"ecc_{kind}", -1)
                if v is not None and v >= 0:
                    ecc.add_metric([dev_id, kind], float(v))
            for state in ("up", "down"):
                v = st.get(f"xgmi_links_{state}", -1)
                if v is not None and v >= 0:
                    links.add_metric([dev_id, state], float(v))
        yield ecc
        yield links
        for name, attr, doc in (("allocations", "allocations", "Allocate container responses"),
                                ("registrations", "registrations", "kubelet registrations"),
                                ("health_flips", "health_flips", "health transitions streamed")):
            c = CounterMetricFamily(f"kgs_deviceplugin_{name}", doc)
            c.add_metric([], float(getattr(self.plugin, attr, 0)))
            yield c


def make_registry(plugin) -> CollectorRegistry:
    reg = CollectorRegistry()
    reg.register(PluginCollector(plugin))
    return reg


def serve(plugin, port: int, addr: str = "0.0.0.0"):
    """Start the HTTP exporter in a daemon thread; returns (server, thread)."""
    from prometheus_client import start_http_server

    return start_http_server(port, addr=addr, registry=make_registry(plugin))
