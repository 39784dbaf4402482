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


# Llama-3-8B architecture (config.json only: no weights, no tokenizer). vLLM
# builds the model from it and --load-format=dummy random-initialises the
# weights, so the pod starts on an offline host (BASELINE config 5, synthetic
# weights). Kept in sync with kgs.models.llama.LlamaConfig.llama3_8b() by a test.
LLAMA3_8B_HF_CONFIG = {
    "architectures": ["LlamaForCausalLM"],
    "model_type": "llama",
    "attention_bias": False,
    "attention_dropout": 0.0,
    "bos_token_id": 128000,
    "eos_token_id": 128001,
    "hidden_act": "silu",
    "hidden_size": 4096,
    "initializer_range": 0.02,
    "intermediate_size": 14336,
    "max_position_embeddings": 8192,
    "mlp_bias": False,
    "num_attention_heads": 32,
    "num_hidden_layers": 32,
    "num_key_value_heads": 8,
    "pretraining_tp": 1,
    "rms_norm_eps": 1e-05,
    "rope_scaling": None,
    "rope_theta": 500000.0,
    "tie_word_embeddings": False,
    "torch_dtype": "bfloat16",
    "use_cache": True,
    "vocab_size": 128256,
}
VLLM_MODEL_DIR = "/models/llama3-8b"
VLLM_CONFIGMAP = "vllm-llama3-8b-config"


def vllm_rocm_pod(image: str = C.VLLM_ROCM_IMAGE) -> list:
    """``pods/vllm-rocm-pod.yaml``: a ConfigMap holding the Llama-3-8B
    ``config.json`` plus the serving Pod that mounts it at ``/models/llama3-8b``.

    Mirrors /root/reference/pods/vllm-cpu-pod.yaml:1-38 (name pattern, port
    8000, /dev/shm memory emptyDir, GPU nodeSelector/toleration with the value
    quoted -- Q12) with a real ``amd.com/gpu: 1``. NOT privileged, unlike the
    reference's CPU pod (:24-25): a privileged container gets every render node
    of its kind worker, so a 1-GPU pod could run on another pod's GPU. The
    device plugin's Allocate passes /dev/kfd, the one render node and
    ``ROCR_VISIBLE_DEVICES=GPU-<uuid>``, which is all vLLM needs. Offline by
    construction: the model is a local path (no hub id), weights are
    ``--load-format=dummy`` and ``--skip-tokenizer-init`` means no tokenizer is
    needed (requests send token ids)."""
    cm = {
        "apiVersion": "v1",
        "kind": "ConfigMap",
        "metadata": {"name": VLLM_CONFIGMAP},
        "data": {"config.json": json.dumps(LLAMA3_8B_HF_CONFIG, indent=2) + "\n"},
    }
    pod = {
        "apiVersion": "v1",
        "kind": "Pod",
        "metadata": {"name": "vllm-rocm-pod"},
        "spec": {
            "containers": [{
                "name": "vllm-rocm-container",
                "image": image,
                "ports": [{"containerPort": 8000}],
                "env": [
                    {"name": "HF_HUB_OFFLINE", "value": "1"},
                    {"name": "TRANSFORMERS_OFFLINE", "value": "1"},
                ],
                "command": ["python3", "-m", "vllm.entrypoints.openai.api_server"],
                "args": [
                    f"--model={VLLM_MODEL_DIR}",
                    "--served-model-name=llama3-8b",
                    "--load-format=dummy",
                    "--skip-tokenizer-init",
                    "--dtype=bfloat16",
                    "--tensor-parallel-size=1",
                    "--max-model-len=8192",
                    "--gpu-memory-utilization=0.90",
                    "--port=8000",
                ],
                "resources": {"limits": {C.RESOURCE_NAME: 1}},
                "readinessProbe": {"httpGet": {"path": "/health", "port": 8000},
                                   "periodSeconds": 5, "failureThreshold": 120},
                "volumeMounts": [
                    {"name": "dshm", "mountPath": "/dev/shm"},
                    {"name": "model-config", "mountPath": VLLM_MODEL_DIR, "readOnly": True},
                ],
            }],
            "nodeSelector": {C.LABEL_HARDWARE[0]: C.LABEL_HARDWARE[1]},
            "tolerations": [{"key": C.TAINT[0], "operator": "Equal", "value": C.TAINT[1], "effect": C.TAINT[2]}],
            "volumes": [
                {"name": "dshm", "emptyDir": {"medium": "Memory", "sizeLimit": "16Gi"}},
                {"name": "model-config", "configMap": {"name": VLLM_CONFIGMAP}},
            ],
            "restartPolicy": "Never",
        },
    }
    return [cm, pod]


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
