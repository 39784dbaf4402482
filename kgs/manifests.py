"""Kubernetes / kind manifests rendered from Python (no heredocs).

Each renderer returns plain dicts; :func:`dump` turns them into YAML. The
shapes mirror the reference's heredocs where they are part of the contract
(kind-gpu-sim.sh:86-97 kind config, :131-141 registry ConfigMap, :248-276 plugin
DaemonSet) and differ where the reference is broken:

* kind config: containerd reads per-registry ``hosts.toml`` from
  ``config_path`` (kind's documented local-registry setup), instead of the
  deprecated ``registry.mirrors`` table *plus* hosts.toml + a SIGHUP that
  targets a host PID (Q2/Q3); the certs.d tree and the GPU partition file are
  bind-mounted into the nodes, so no per-node ``docker exec`` is needed;
* GPU workers bind-mount ``/dev/kfd`` and their ``/dev/dri/renderD*`` nodes;
* the plugin DaemonSet mounts the kubelet device-plugin dir, ``/dev``, ``/sys``
  and ``/etc/kgs`` (the reference mounts nothing for ROCm, Q7) and has a
  readiness probe, so ``kubectl wait`` means "registered", not "started".
"""
from __future__ import annotations

import json

import yaml

from . import config as C


class _Dumper(yaml.SafeDumper):
    def ignore_aliases(self, data):  # never emit &id001 anchors for shared sub-dicts
        return True


_RESOLVER = yaml.resolver.Resolver()


def _str_presenter(dumper, data):
    if "\n" in data:
        return dumper.represent_scalar("tag:yaml.org,2002:str", data, style="|")
    # strings that would read back as bool/int/null ("true", "5000", "") get
    # double quotes -- the repo's yamllint style (quote-type: double)
    if data == "" or _RESOLVER.resolve(yaml.ScalarNode, data, (True, False)) != "tag:yaml.org,2002:str":
        return dumper.represent_scalar("tag:yaml.org,2002:str", data, style='"')
    return dumper.represent_scalar("tag:yaml.org,2002:str", data)


_Dumper.add_representer(str, _str_presenter)


def dump(obj) -> str:
    if isinstance(obj, list):
        return "---\n".join(yaml.dump(o, Dumper=_Dumper, sort_keys=False, default_flow_style=False) for o in obj)
    return yaml.dump(obj, Dumper=_Dumper, sort_keys=False, default_flow_style=False)


# ----------------------------------------------------------------- kind ------
def containerd_patch() -> str:
    return (
        '[plugins."io.containerd.grpc.v1.cri".registry]\n'
        f'  config_path = "{C.CERTS_D}"\n'
    )


def hosts_toml(registry_name: str = C.REGISTRY_NAME, internal_port: int = C.REGISTRY_INTERNAL_PORT) -> str:
    # kind-gpu-sim.sh:122-125
    return f'[host."http://{registry_name}:{internal_port}"]\n  capabilities = ["pull", "resolve"]\n'


def kind_config(workers: list, certs_dir: str | None, partition_file: str | None,
                kind_node_image: str | None = None) -> dict:
    """``workers``: list of dicts {"render_minors": [...], "kfd": bool} (one per worker)."""
    common_mounts = []
    if certs_dir:
        common_mounts.append({"hostPath": certs_dir, "containerPath": C.CERTS_D, "readOnly": True})
    cp = {"role": "control-plane"}
    if common_mounts:
        cp["extraMounts"] = list(common_mounts)
    if kind_node_image:
        cp["image"] = kind_node_image
    nodes = [cp]
    for w in workers:
        n = {"role": "worker"}
        mounts = list(common_mounts)
        if partition_file:
            mounts.append({"hostPath": partition_file,
                           "containerPath": f"{C.PARTITION_DIR_IN_NODE}/{C.PARTITION_FILE}", "readOnly": True})
        if w.get("kfd"):
            mounts.append({"hostPath": "/dev/kfd", "containerPath": "/dev/kfd"})
            for m in w.get("render_minors", []):
                mounts.append({"hostPath": f"/dev/dri/renderD{m}", "containerPath": f"/dev/dri/renderD{m}"})
        if mounts:
            n["extraMounts"] = mounts
        if kind_node_image:
            n["image"] = kind_node_image
        nodes.append(n)
    return {
        "kind": "Cluster",
        "apiVersion": "kind.x-k8s.io/v1alpha4",
        "containerdConfigPatches": [containerd_patch()],
        "nodes": nodes,
    }


# ------------------------------------------------------------- registry ------
def registry_configmap(port: int) -> dict:
    # KEP-1755 (kind-gpu-sim.sh:131-141)
    return {
        "apiVersion": "v1",
        "kind": "ConfigMap",
        "metadata": {"name": C.LOCAL_REGISTRY_CM_NAME, "namespace": C.LOCAL_REGISTRY_CM_NAMESPACE},
        "data": {"localRegistryHosting.v1": f'host: "localhost:{port}"\nhelp: "{C.LOCAL_REGISTRY_HELP}"\n'},
    }


# -------------------------------------------------------------- plugin -------
def plugin_daemonset(image: str, fake_gpus: int = 0, health_interval: float = 5.0) -> dict:
    tol = [{"key": C.TAINT[0], "operator": "Equal", "value": C.TAINT[1], "effect": C.TAINT[2]}]
    env = [
        {"name": "NODE_NAME", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
        {"name": "KGS_HEALTH_INTERVAL", "value": str(health_interval)},
        {"name": "KGS_METRICS_PORT", "value": str(C.PLUGIN_METRICS_PORT)},
        {"name": "PYTHONUNBUFFERED", "value": "1"},
    ]
    if fake_gpus:
        env.append({"name": "KGS_FAKE_GPUS", "value": str(fake_gpus)})
    mounts = [
        {"name": "device-plugin", "mountPath": C.KUBELET_DP_DIR},
        {"name": "dev", "mountPath": "/dev"},
        {"name": "sys", "mountPath": "/sys", "readOnly": True},
        {"name": "kgs-etc", "mountPath": C.PARTITION_DIR_IN_NODE, "readOnly": True},
    ]
    vols = [
        {"name": "device-plugin", "hostPath": {"path": C.KUBELET_DP_DIR, "type": "DirectoryOrCreate"}},
        {"name": "dev", "hostPath": {"path": "/dev"}},
        {"name": "sys", "hostPath": {"path": "/sys"}},
        {"name": "kgs-etc", "hostPath": {"path": C.PARTITION_DIR_IN_NODE, "type": "DirectoryOrCreate"}},
    ]
    return {
        "apiVersion": "apps/v1",
        "kind": "DaemonSet",
        "metadata": {"name": C.PLUGIN_DS_NAME, "namespace": C.PLUGIN_NAMESPACE},
        "spec": {
            "selector": {"matchLabels": {"app": C.PLUGIN_APP_LABEL}},
            "updateStrategy": {"type": "RollingUpdate"},
            "template": {
                "metadata": {"labels": {"app": C.PLUGIN_APP_LABEL}},
                "spec": {
                    "priorityClassName": "system-node-critical",
                    "nodeSelector": {C.LABEL_HARDWARE[0]: C.LABEL_HARDWARE[1]},
                    "tolerations": tol,
                    "containers": [{
                        "name": C.PLUGIN_CONTAINER,
                        "image": image,
                        "imagePullPolicy": "IfNotPresent",
                        "command": ["python3", "-m", "kgs.deviceplugin"],
                        "env": env,
                        "securityContext": {"privileged": True},
                        "ports": [{"name": "metrics", "containerPort": C.PLUGIN_METRICS_PORT}],
                        "readinessProbe": {
                            "exec": {"command": ["test", "-f", "/tmp/kgs-dp-ready"]},
                            "periodSeconds": 1,
                            "failureThreshold": 1,
                        },
                        "volumeMounts": mounts,
                    }],
                    "volumes": vols,
                },
            },
        },
    }


def partition_file(nodes: dict) -> str:
    """``{"nodes": {"<node-name>": [render minors]}}`` for the plugin."""
    return json.dumps({"nodes": {k: sorted(v) for k, v in nodes.items()}}, indent=1) + "\n"


# ---------------------------------------------------------------- pods -------
def gpu_test_pod(image: str, gpus: int = 1, command: list | None = None, name: str = C.TEST_POD_NAME) -> dict:
    """The pods/rocm-gpu-test-pod.yaml layout (pods/rocm-gpu-test-pod.yaml:1-19)
    with the workload image, a memory /dev/shm for RCCL, and N GPUs."""
    return {
        "apiVersion": "v1",
        "kind": "Pod",
        "metadata": {"name": name},
        "spec": {
            "containers": [{
                "name": C.TEST_POD_CONTAINER,
                "image": image,
                "command": command or ["python3", "-m", "kgs.workload.entrypoint", "--pod"],
                "resources": {"limits": {C.RESOURCE_NAME: gpus}},
                "volumeMounts": [{"name": "dshm", "mountPath": "/dev/shm"}],
            }],
            "nodeSelector": {C.LABEL_HARDWARE[0]: C.LABEL_HARDWARE[1]},
            "tolerations": [{"key": C.TAINT[0], "operator": "Equal", "value": C.TAINT[1], "effect": C.TAINT[2]}],
            "volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory", "sizeLimit": "16Gi"}}],
        },
    }


STATIC_POD_REGISTRY = "localhost:5000"  # what pods/*.yaml are written against (the reference default port)


def render_static_pod(name: str, registry_host: str) -> str:
    """``pods/<name>.yaml`` with its in-tree images moved to ``registry_host``
    (``localhost:<--registry-port>``), so ``--registry-port=N`` clusters can run
    the shipped pods: ``kgs pod rocm-gpu-test --registry-port=N | kubectl create -f -``.
    Images from public registries (e.g. the vLLM pod) are left alone."""
    from pathlib import Path

    pods = Path(__file__).resolve().parents[1] / "pods"
    stem = name[:-5] if name.endswith(".yaml") else name
    path = pods / f"{stem}.yaml"
    if not path.exists():
        path = pods / f"{stem}-pod.yaml"
    if not path.exists():
        avail = sorted(p.stem for p in pods.glob("*.yaml"))
        raise UnknownPod(f"ERROR: no pod manifest {name!r} in pods/ (have: {', '.join(avail)})")
    text = path.read_text()
    return text.replace(f"image: {STATIC_POD_REGISTRY}/", f"image: {registry_host}/")


class UnknownPod(ValueError):
    pass
