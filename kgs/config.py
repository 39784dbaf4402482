"""Defaults and the observable contract kept from the reference.

Every value here is something a user of ``kind-gpu-sim.sh`` can observe (flag
defaults, names, labels, taints, resource names, image tags); they are kept
byte-identical. Citations are to /root/reference/kind-gpu-sim.sh.
"""
from __future__ import annotations

from dataclasses import dataclass, field

# --- flag defaults (kind-gpu-sim.sh:4-7) -------------------------------------
DEFAULT_REGISTRY_PORT = 5000
# Docker-Hub library images are pulled through a public mirror to dodge Docker
# Hub rate limits -- the reference's patch_dockerfile sed-rewrites FROM lines to
# this mirror (kind-gpu-sim.sh:144-178, :5); here it is a build argument.
BASE_MIRROR = "public.ecr.aws/docker/library"
REGISTRY_IMAGE = f"{BASE_MIRROR}/registry:2"
# Pinned bases (the reference pins nothing for ROCm, Q6). gfx950 needs ROCm >= 7.0.
ROCM_BASE_IMAGE = "docker.io/rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.8.0"
ROCM_DEV_IMAGE = "docker.io/rocm/dev-ubuntu-22.04:7.0"          # amd-smi source of the plugin image
# The ROCm release images above live on Docker Hub under this prefix;
# --rocm-mirror=<registry>/<path> swaps it (the C13 mirror rewrite, applied to
# the ROCm images: the reference rewrites only its library bases, :144-178).
ROCM_REGISTRY = "docker.io/rocm"
PY_BUILD_IMAGE = "python:3.12.8-bookworm"
PY_SLIM_IMAGE = "python:3.12.8-slim-bookworm"
VLLM_ROCM_IMAGE = "docker.io/rocm/vllm:rocm7.0.0_vllm_0.10.2_20251006"
DEFAULT_CLUSTER_NAME = "kind-gpu-sim"
DEFAULT_IMAGE_NAME = "not-set"

# --- generated artefacts / names (kind-gpu-sim.sh:68-69) ----------------------
CONFIG_FILE = "kind-config.yaml"
REGISTRY_NAME = "kind-registry"
REGISTRY_INTERNAL_PORT = 5000
KIND_NETWORK = "kind"

# --- node contract (kind-gpu-sim.sh:107-117) -----------------------------------
LABEL_HARDWARE = ("hardware-type", "gpu")
LABEL_WORKER_ROLE = ("node-role.kubernetes.io/worker", "")
LABEL_ROCM_PRESENT = ("rocm.amd.com/gpu.present", "true")
TAINT = ("gpu", "true", "NoSchedule")
RESOURCE_NAME = "amd.com/gpu"
FAKE_GPUS_PER_WORKER = 2  # the reference's patched capacity (kind-gpu-sim.sh:113)
DEFAULT_WORKERS = 2       # 1 control-plane + 2 workers (kind-gpu-sim.sh:93-96)

# kgs additions (node labels carrying what the plugin on that node may advertise)
LABEL_GPU_PARTITION = "kgs.amd.com/gpu-partition"
PARTITION_DIR_IN_NODE = "/etc/kgs"
PARTITION_FILE = "gpus.json"

# --- registry plumbing (kind-gpu-sim.sh:89-92, :120-142) ----------------------
CERTS_D = "/etc/containerd/certs.d"
LOCAL_REGISTRY_CM_NAMESPACE = "kube-public"
LOCAL_REGISTRY_CM_NAME = "local-registry-hosting"
LOCAL_REGISTRY_HELP = "https://kind.sigs.k8s.io/docs/user/local-registry/"

# --- device plugin deploy (kind-gpu-sim.sh:242-283) ----------------------------
PLUGIN_IMAGE_REPO = "amdgpu-dp"
PLUGIN_IMAGE_TAG = "dev"
PLUGIN_DS_NAME = "amdgpu-device-plugin-daemonset"
PLUGIN_NAMESPACE = "kube-system"
PLUGIN_APP_LABEL = "amdgpu-device-plugin"
PLUGIN_CONTAINER = "amdgpu-dp-ds"
PLUGIN_READY_TIMEOUT_S = 60
PLUGIN_METRICS_PORT = 9464  # Prometheus exporter of the plugin (kgs addition)
KUBELET_DP_DIR = "/var/lib/kubelet/device-plugins"

# --- workload images (in-tree Dockerfiles, images/) ---------------------------
WORKLOAD_IMAGE_REPO = "kgs-rocm-test"
WORKLOAD_IMAGE_TAG = "dev"

# --- pods (pods/rocm-gpu-test-pod.yaml) ----------------------------------------
TEST_POD_NAME = "gpu-rocm-test"
TEST_POD_CONTAINER = "gpu-sim"
TEST_POD_READY_TIMEOUT_S = 60

SUCCESS_FMT_FAKE = " Simulated GPU Kind cluster is ready for '{gpu_type}'!"  # kind-gpu-sim.sh:388
SUCCESS_FMT_REAL = " MI355X Kind cluster is ready for '{gpu_type}' ({n} amd.com/gpu advertised)!"
USAGE = "Usage: {prog} {{create [rocm]|delete|load|status|bench|doctor}} [--registry-port=N] [--cluster-name=S] " \
        "[--image-name=S] [--runtime=docker|podman] [--dry-run] ..."


@dataclass
class Settings:
    """Resolved CLI settings (one object threads through every phase)."""

    registry_port: int = DEFAULT_REGISTRY_PORT
    cluster_name: str = DEFAULT_CLUSTER_NAME
    image_name: str = DEFAULT_IMAGE_NAME
    runtime: str | None = None           # docker | podman | None = autodetect
    workers: int = DEFAULT_WORKERS
    gpus: int | None = None              # advertise exactly N of the host's GPUs (None = all healthy)
    gpu_partition: str = "all-on-first"  # all-on-first | split | fake
    fake_gpus: int | None = None         # force the fake path with N per worker
    fake_mode: str = "patch"             # patch (reference) | plugin (kgs fake plugin)
    registry_bind: str = "127.0.0.1"     # Q4: do not publish the registry on all interfaces
    registry_image: str | None = None    # None = <base_mirror>/registry:2
    base_mirror: str = BASE_MIRROR       # C13: registry prefix for library base images
    rocm_base_image: str = ROCM_BASE_IMAGE
    rocm_dev_image: str = ROCM_DEV_IMAGE
    rocm_mirror: str | None = None       # replaces ROCM_REGISTRY in the ROCm image references
    kind_node_image: str | None = None
    config_file: str = CONFIG_FILE
    dry_run: bool = False
    keep_on_fail: bool = False
    skip_build: bool = False
    timings_json: str | None = None
    plugin_image: str | None = None      # override the built image
    ready_timeout_s: int = PLUGIN_READY_TIMEOUT_S
    dev_root: str = "/"                  # host root for /dev and /sys discovery (tests use a fake tree)
    extra: dict = field(default_factory=dict)

    def library_image(self, name: str) -> str:
        """``name`` (e.g. ``python:3.12.8-slim-bookworm``) from the configured library mirror."""
        return f"{self.base_mirror.rstrip('/')}/{name}"

    def rocm_image(self, ref: str) -> str:
        """A ROCm release image (``docker.io/rocm/<name>:<tag>``) from the
        ``--rocm-mirror`` registry when one is set; other references as given."""
        if self.rocm_mirror and ref.startswith(ROCM_REGISTRY + "/"):
            return self.rocm_mirror.rstrip("/") + ref[len(ROCM_REGISTRY):]
        return ref

    @property
    def registry_container_image(self) -> str:
        return self.registry_image or self.library_image("registry:2")

    def plugin_build_args(self) -> list[str]:
        """``--build-arg`` list for images/Dockerfile.deviceplugin."""
        return ["--build-arg", f"PY_IMAGE={self.library_image(PY_SLIM_IMAGE)}",
                "--build-arg", f"BUILD_IMAGE={self.library_image(PY_BUILD_IMAGE)}",
                "--build-arg", f"ROCM_IMAGE={self.rocm_image(self.rocm_dev_image)}"]

    @property
    def registry_host(self) -> str:
        return f"localhost:{self.registry_port}"
