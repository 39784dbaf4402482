"""Cluster lifecycle: ``create`` / ``delete`` / ``load`` / ``status``.

Python replacement for kind-gpu-sim.sh's function layer (L1-L6 in SURVEY.md
§1). The observable contract (names, labels, taint, resource, image tags,
registry wiring, success/error strings) is kept; the mechanics are
MI355X-first:

* GPUs come from the native enumeration core, not a constant. A host with
  ``/dev/kfd`` and gfx950 nodes gets real passthrough: worker containers
  bind-mount ``/dev/kfd`` and their ``renderD*`` nodes and the in-tree device
  plugin registers the real ``amd.com/gpu`` devices (kubelet-managed capacity).
  A host without them (or ``--fake-gpus``) takes the reference's fake path:
  ``amd.com/gpu`` capacity patched into node status (kind-gpu-sim.sh:113), or
  served by the plugin's fake source (``--fake-mode plugin``).
* GPUs are partitioned across workers (``--gpu-partition``): with
  ``all-on-first`` (default) worker 1 owns every GPU so a single pod can take
  all 8; ``split`` deals them out NUMA-contiguously. The partition is a JSON
  file bind-mounted into every worker; each node's plugin advertises only its
  share, so 8 physical GPUs never show up as 16.
* Registry hosts.toml files are bind-mounted (containerd ``config_path``), so
  node configuration needs no ``docker exec`` and no containerd SIGHUP.
* Labels and taints are applied with one ``kubectl`` call each for all workers.
* Readiness is polled for pod existence, then ``kubectl wait`` (no blind
  ``sleep 5``, Q11), then the advertised capacity is confirmed.
* Every phase is timed (``--timings-json``).
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import sys
import time
from pathlib import Path

from . import config as C
from . import manifests
from .runtime import ContainerRuntime
from .timing import PhaseTimer
from .utils.proc import CommandError, Runner

log = logging.getLogger("kgs")
REPO_ROOT = Path(__file__).resolve().parents[1]


class ProvisionError(RuntimeError):
    """A failure that maps to exit status 1 with a user-facing message."""


def plan_partitions(gpus: list, workers: int, mode: str) -> list:
    """Render minors per worker. ``gpus``: objects with render_minor, numa_node."""
    minors = [g for g in gpus if getattr(g, "render_minor", -1) >= 0]
    out = [[] for _ in range(workers)]
    if workers <= 0 or not minors:
        return out
    if mode == "all-on-first":
        out[0] = [g.render_minor for g in minors]
    elif mode == "split":
        # NUMA-contiguous blocks: sort by (numa, index) then deal consecutive chunks
        order = sorted(minors, key=lambda g: (getattr(g, "numa_node", -1), getattr(g, "index", 0)))
        per, extra = divmod(len(order), workers)
        i = 0
        for w in range(workers):
            k = per + (1 if w < extra else 0)
            out[w] = [g.render_minor for g in order[i:i + k]]
            i += k
    elif mode == "fake":
        pass
    else:
        raise ProvisionError(f"unknown --gpu-partition {mode!r} (all-on-first|split)")
    return out


def select_gpus(gpus: list, n: int | None) -> list:
    """The ``n`` GPUs to advertise (``kgs create --gpus N``), out of the host's
    healthy ones: one xGMI island first, then the fewest NUMA nodes, then the
    lowest indices -- the device plugin's GetPreferredAllocation scoring
    (kgs/deviceplugin/allocator.py), applied at cluster level. ``None`` = all.
    The reference advertises a fixed count per worker (kind-gpu-sim.sh:113)."""
    if n is None:
        return list(gpus)
    if n < 1:
        raise ProvisionError(f"ERROR: --gpus must be >= 1 (got {n})")
    if n > len(gpus):
        raise ProvisionError(f"ERROR: --gpus {n} but the host has only {len(gpus)} healthy GPU(s) "
                             f"(renderD{[g.render_minor for g in gpus]})")
    from .deviceplugin.allocator import DevInfo, preferred

    infos = {str(g.render_minor): DevInfo(str(g.render_minor), g.index, getattr(g, "numa_node", -1),
                                          getattr(g, "node_id", -1), frozenset(g.xgmi_peers()))
             for g in gpus}
    ids = preferred([str(g.render_minor) for g in gpus], [], n, infos)
    chosen = {int(i) for i in ids}
    return [g for g in gpus if g.render_minor in chosen]


class Provisioner:
    def __init__(self, settings: C.Settings, runner: Runner | None = None, timer: PhaseTimer | None = None,
                 workdir: str | os.PathLike | None = None, out=None):
        self.s = settings
        self.runner = runner or Runner(dry_run=settings.dry_run)
        self.timer = timer or PhaseTimer()
        self.workdir = Path(workdir or os.getcwd())
        self.out = out or (lambda msg: print(msg, flush=True))
        self.rt: ContainerRuntime | None = None
        self.topology = None
        self.fake = False
        self.partitions: list = []
        self.selected: list = []
        self.created_cluster = False

    # ------------------------------------------------------------ helpers ----
    @property
    def context(self) -> str:
        return f"kind-{self.s.cluster_name}"

    def kind(self, *args, **kw):
        return self.runner.run(["kind", *args], **kw)

    def kubectl(self, *args, **kw):
        return self.runner.run(["kubectl", "--context", self.context, *args], **kw)

    @property
    def state_dir(self) -> Path:
        return self.workdir / ".kgs" / self.s.cluster_name

    def generated_worker_names(self) -> list:
        """kind's node names, in the order of the kind config's worker list
        (``<cluster>-worker``, ``-worker2``, ... ``-worker10``): the order the
        partition plan and the partition file use."""
        return [f"{self.s.cluster_name}-worker"] + [f"{self.s.cluster_name}-worker{i}"
                                                    for i in range(2, self.s.workers + 1)]

    def worker_names(self) -> list:
        """The cluster's worker nodes in natural order. kubectl lists nodes
        lexicographically (``worker, worker10, worker2``), which must not be
        zipped with the partition plan."""
        names = self.generated_worker_names()
        if self.runner.dry_run:
            return names
        r = self.kubectl("get", "nodes", "-o", "jsonpath={range .items[*]}{.metadata.name}{\"\\n\"}{end}",
                         mutating=False)
        got = [n for n in r.stdout.split() if n and "control-plane" not in n]
        return sorted(got, key=_natural_key) or names

    def partition_of(self) -> dict:
        """{worker node name: render minors} -- by name, never by list position."""
        return dict(zip(self.generated_worker_names(), self.partitions))

    def cluster_exists(self) -> bool:
        r = self.kind("get", "clusters", check=False, mutating=False)
        return self.s.cluster_name in r.stdout.split()

    def ensure_runtime(self) -> ContainerRuntime:
        if self.rt is None:
            self.rt = ContainerRuntime.detect(self.runner, self.s.runtime)
        return self.rt

    # ------------------------------------------------------------ discover ---
    def discover(self) -> None:
        if self.s.fake_gpus is not None:
            if self.s.gpus is not None:
                raise ProvisionError("ERROR: --gpus selects real GPUs to advertise; with --fake-gpus the "
                                     "count is --fake-gpus per worker")
            self.fake = True
            self.partitions = [[] for _ in range(self.s.workers)]
            return
        try:
            from . import gpuinfo

            self.topology = gpuinfo.discover(self.s.dev_root, use_amdsmi=False)
        except Exception as e:  # native core missing: treat as CPU-only host
            log.warning("GPU discovery unavailable (%s); using the fake capacity path", e)
            self.topology = None
        gpus = self.topology.gpus if self.topology else []
        usable = [g for g in gpus if g.render_minor >= 0 and g.healthy]
        if not self.topology or not self.topology.kfd_present or not usable:
            if self.s.gpus is not None:
                raise ProvisionError(f"ERROR: --gpus {self.s.gpus} needs real GPUs, but none were found under "
                                     f"{self.s.dev_root} (/dev/kfd + gfx nodes); for the simulated path use "
                                     "--fake-gpus N")
            self.fake = True
            self.partitions = [[] for _ in range(self.s.workers)]
            return
        self.fake = False
        self.selected = select_gpus(usable, self.s.gpus)
        self.partitions = plan_partitions(self.selected, self.s.workers, self.s.gpu_partition)

    @property
    def fake_per_worker(self) -> int:
        return self.s.fake_gpus if self.s.fake_gpus is not None else C.FAKE_GPUS_PER_WORKER

    @property
    def expected_capacity(self) -> int:
        if self.fake:
            return self.fake_per_worker * self.s.workers
        return sum(len(p) for p in self.partitions)

    # ------------------------------------------------------------ registry ---
    def start_registry(self) -> None:
        rt = self.ensure_runtime()
        name = C.REGISTRY_NAME
        self.out(f"Starting local registry on port {self.s.registry_port}...")
        if rt.is_running(name):
            self.out(f"Registry '{name}' already running.")
            return
        if rt.exists(name):  # stopped container from an earlier run: restart it
            rt.cr("start", name)
            return
        rt.cr("run", "-d", "--restart=always", "-p",
              f"{self.s.registry_bind}:{self.s.registry_port}:{C.REGISTRY_INTERNAL_PORT}",
              "--name", name, self.s.registry_container_image)

    def write_node_files(self) -> tuple:
        """certs.d tree + partition file (bind-mounted into the nodes)."""
        sd = self.state_dir
        certs = sd / "certs.d"
        host_dir = certs / self.s.registry_host
        part = sd / C.PARTITION_FILE
        if not self.runner.dry_run:
            host_dir.mkdir(parents=True, exist_ok=True)
            (host_dir / "hosts.toml").write_text(manifests.hosts_toml())
            part.write_text(manifests.partition_file(self.partition_of()))
        return str(certs.resolve()), str(part.resolve())

    def write_kind_config(self) -> Path:
        certs, part = self.write_node_files()
        workers = [{"kfd": (not self.fake) and bool(p), "render_minors": p} for p in self.partitions]
        cfg = manifests.kind_config(workers, certs, part, self.s.kind_node_image)
        path = self.workdir / self.s.config_file
        text = manifests.dump(cfg)
        if not self.runner.dry_run:
            path.write_text(text)
        else:
            self.out(f"# {path}\n{text}")
        return path

    def apply_registry_configmap(self) -> None:
        self.kubectl("apply", "-f", "-", input=manifests.dump(manifests.registry_configmap(self.s.registry_port)))

    # --------------------------------------------------------------- nodes ---
    def configure_nodes(self) -> list:
        workers = self.worker_names()
        labels = [f"{C.LABEL_HARDWARE[0]}={C.LABEL_HARDWARE[1]}",
                  f"{C.LABEL_WORKER_ROLE[0]}={C.LABEL_WORKER_ROLE[1]}",
                  f"{C.LABEL_ROCM_PRESENT[0]}={C.LABEL_ROCM_PRESENT[1]}"]
        self.kubectl("label", "node", *workers, *labels, "--overwrite")
        self.kubectl("taint", "node", *workers, f"{C.TAINT[0]}={C.TAINT[1]}:{C.TAINT[2]}", "--overwrite")
        if not self.fake:
            owned = self.partition_of()
            for w in workers:
                self.kubectl("label", "node", w, f"{C.LABEL_GPU_PARTITION}={len(owned.get(w, []))}", "--overwrite")
        elif self.s.fake_mode == "patch":
            patch = json.dumps([{"op": "add", "path": "/status/capacity/amd.com~1gpu",
                                 "value": str(self.fake_per_worker)}])
            for w in workers:
                self.kubectl("patch", "node", w, "--type=json", f"-p={patch}", "--subresource=status")
        return workers

    def prepull(self, nodes: list, images: list) -> None:
        """Pull ``images`` into the nodes' containerd from the local registry
        (``crictl pull`` inside each kind node), so the test pod does not pay a
        multi-GB pull after it is scheduled. Runs in the background during
        ``create`` while the plugin is deployed and becomes Ready."""
        rt = self.ensure_runtime()
        for node in nodes:
            for img in images:
                rt.cr("exec", node, "crictl", "pull", img, check=False)

    # -------------------------------------------------------------- plugin ---
    def plugin_image(self) -> str:
        if self.s.plugin_image:
            return self.s.plugin_image
        rt = self.ensure_runtime()
        repo = f"{C.PLUGIN_IMAGE_REPO}:{C.PLUGIN_IMAGE_TAG}"
        return f"localhost/{repo}" if rt.name == "podman" else f"{self.s.registry_host}/{repo}"

    def build_plugin_image(self) -> str:
        """Build (or pick) the plugin image and make it pullable by the nodes."""
        self.plugin_image_stage1()
        return self.plugin_image_stage2()

    def plugin_image_stage1(self) -> None:
        """Everything that does not need the cluster: docker build + push to the
        local registry (podman: build + tag). Runs concurrently with
        ``kind create cluster`` in ``create`` -- a cold image build is the
        longest phase after cluster creation, and the reference runs it after."""
        rt = self.ensure_runtime()
        image = self.plugin_image()
        if self.s.plugin_image or self.s.skip_build:
            return
        tag = f"{self.s.registry_host}/{C.PLUGIN_IMAGE_REPO}:{C.PLUGIN_IMAGE_TAG}"
        self.out(" Building kgs ROCm device plugin image...")
        env = {"BUILDAH_FORMAT": "docker"} if rt.name == "podman" else None
        rt.cr("build", "-t", tag, *self.s.plugin_build_args(),
              "-f", str(REPO_ROOT / "images" / "Dockerfile.deviceplugin"), str(REPO_ROOT), env=env)
        if rt.name == "docker":
            rt.cr("push", tag)
        else:
            rt.cr("tag", tag, image)

    def plugin_image_stage2(self) -> str:
        """The cluster-dependent part: side-load into the kind nodes where the
        nodes cannot pull it (podman, or a prebuilt image not in the registry)."""
        rt = self.ensure_runtime()
        image = self.plugin_image()
        if self.s.plugin_image or self.s.skip_build:
            self.out(f"Using prebuilt device-plugin image {image}")
            if rt.name == "podman" or self.s.plugin_image:
                rt.load_into_kind(image, self.s.cluster_name)
        elif rt.name == "podman":
            rt.save_and_kind_load(image, self.s.cluster_name)
        return image

    def deploy_plugin(self, image: str) -> None:
        fake_gpus = self.fake_per_worker if (self.fake and self.s.fake_mode == "plugin") else 0
        ds = manifests.plugin_daemonset(image, fake_gpus=fake_gpus)
        self.kubectl("apply", "-f", "-", input=manifests.dump(ds))

    def wait_plugin_ready(self) -> None:
        sel = f"app={C.PLUGIN_APP_LABEL}"
        deadline = time.monotonic() + self.s.ready_timeout_s
        if not self.runner.dry_run:
            # Q11: wait for the DaemonSet to create pods instead of a fixed sleep
            while True:
                r = self.kubectl("get", "pods", "-n", C.PLUGIN_NAMESPACE, "-l", sel, "-o", "name",
                                 check=False, mutating=False)
                if r.ok and r.stdout.strip():
                    break
                if time.monotonic() > deadline:
                    raise ProvisionError("ERROR: ROCm plugin pods not ready in time")
                time.sleep(0.25)
        remaining = max(1, int(deadline - time.monotonic()))
        r = self.kubectl("wait", "--for=condition=Ready", "-n", C.PLUGIN_NAMESPACE, "pod", "-l", sel,
                         f"--timeout={remaining}s", check=False)
        if not r.ok:
            self._diagnose_plugin()
            raise ProvisionError("ERROR: ROCm plugin pods not ready in time")

    def _diagnose_plugin(self) -> None:
        for args in (("get", "pods", "-n", C.PLUGIN_NAMESPACE, "-l", f"app={C.PLUGIN_APP_LABEL}", "-o", "wide"),
                     ("logs", "-n", C.PLUGIN_NAMESPACE, "-l", f"app={C.PLUGIN_APP_LABEL}", "--tail=50")):
            r = self.kubectl(*args, check=False, mutating=False)
            if r.stdout:
                print(r.stdout, file=sys.stderr)

    def allocatable(self) -> dict:
        r = self.kubectl("get", "nodes", "-o", "json", check=False, mutating=False)
        if not r.ok or not r.stdout.strip():
            return {}
        data = json.loads(r.stdout)
        out = {}
        for n in data.get("items", []):
            v = n.get("status", {}).get("allocatable", {}).get(C.RESOURCE_NAME)
            if v is not None:
                out[n["metadata"]["name"]] = int(v)
        return out

    def wait_capacity(self, timeout_s: float = 60.0) -> int:
        want = self.expected_capacity
        if self.runner.dry_run:
            return want
        deadline = time.monotonic() + timeout_s
        have = 0
        while time.monotonic() < deadline:
            have = sum(self.allocatable().values())
            if have >= want:
                return have
            time.sleep(0.25)
        raise ProvisionError(f"ERROR: only {have} of {want} {C.RESOURCE_NAME} advertised after {timeout_s:.0f}s")

    # ---------------------------------------------------------- reconcile ---
    SHAPE_FILE = "cluster.json"

    def desired_shape(self) -> dict:
        """What this create would build: the parts of the kind config that an
        existing cluster cannot be changed to in place (node list and the
        /dev/kfd + renderD extraMounts are fixed at `kind create` time)."""
        return {"fake": bool(self.fake), "workers": int(self.s.workers),
                "partitions": [list(p) for p in (self.partitions or [])] if not self.fake else [],
                "registry_port": int(self.s.registry_port)}

    def write_shape(self) -> None:
        if self.runner.dry_run:
            return
        self.state_dir.mkdir(parents=True, exist_ok=True)
        (self.state_dir / self.SHAPE_FILE).write_text(json.dumps(self.desired_shape(), indent=1) + "\n")

    def check_drift(self) -> None:
        """Q15 reconcile, with drift detection: re-running create on an existing
        cluster is fine only if it would build the same cluster. A cluster made
        on the fake (CPU-only) path and re-created on a GPU host has workers
        without /dev/kfd mounts; a changed partition or worker count likewise
        cannot be applied in place -- fail now with a clear instruction instead
        of timing out on capacity later."""
        want = self.desired_shape()
        path = self.state_dir / self.SHAPE_FILE
        have = None
        if path.exists():
            try:
                have = json.loads(path.read_text())
            except ValueError:
                have = None
        diffs = []
        if have is not None:
            for key, label in (("fake", "GPU path (fake capacity vs real /dev/kfd passthrough)"),
                               ("workers", "worker count"), ("partitions", "GPU partition (render minors per worker)"),
                               ("registry_port", "registry port")):
                if have.get(key) != want[key]:
                    diffs.append(f"{label}: existing {have.get(key)!r}, requested {want[key]!r}")
        else:
            # created by another tool / an older kgs: the node list is still checkable
            n = len(self.worker_names())
            if n != want["workers"]:
                diffs.append(f"worker count: existing {n}, requested {want['workers']}")
        if diffs:
            raise ProvisionError(
                f"ERROR: kind cluster '{self.s.cluster_name}' exists with a different shape -- "
                + "; ".join(diffs)
                + f". These are fixed when kind creates the nodes: run `kgs delete --cluster-name={self.s.cluster_name}`"
                  " first, then create again.")
        if have is None:
            self.write_shape()

    # --------------------------------------------------------------- verbs ---
    def create(self, gpu_type: str = "rocm") -> int:
        if gpu_type != "rocm":
            raise ProvisionError(
                f" Unknown GPU type: {gpu_type}" + (" (the nvidia path is not part of this MI355X-native build)"
                                                    if gpu_type == "nvidia" else ""))
        t = self.timer
        with t.phase("runtime"):
            self.ensure_runtime()
        with t.phase("discover") as rec:
            self.discover()
            rec.update(fake=self.fake, partitions=self.partitions)
        with t.phase("registry"):
            self.start_registry()
        with t.phase("kind-config"):
            cfg = self.write_kind_config()
        # the plugin image builds while kind creates the cluster (dry-run and
        # --serial keep the reference's sequential order)
        build = None
        if not self.runner.dry_run and not self.s.extra.get("serial"):
            build = _Background(self.plugin_image_stage1)
        try:
            with t.phase("kind-create") as rec:
                if not self.runner.dry_run and self.cluster_exists():
                    self.check_drift()
                    self.out(f"Kind cluster '{self.s.cluster_name}' already exists; reconciling.")
                    rec["reused"] = True
                else:
                    args = ["create", "cluster", "--name", self.s.cluster_name, "--config", str(cfg)]
                    self.kind(*args)
                    self.created_cluster = True
                    self.write_shape()
            with t.phase("registry-network"):
                why = self.ensure_runtime().network_connect(C.KIND_NETWORK, C.REGISTRY_NAME)
                if why is not None and not self.runner.dry_run:
                    # without it the nodes cannot pull localhost:<port>/amdgpu-dp:dev and the
                    # user would only see a 60 s "plugin pods not ready" timeout (Q5)
                    raise ProvisionError(f"ERROR: could not attach {C.REGISTRY_NAME} to network "
                                         f"{C.KIND_NETWORK}: {why}")
            with t.phase("nodes") as rec:
                rec["workers"] = self.configure_nodes()
            prepull_images = self.s.extra.get("prepull") or []
            if prepull_images and not self.runner.dry_run:
                # GPU pods only land on GPU workers; pull there while the plugin comes up
                owned = self.partition_of()
                gpu_nodes = [w for w in rec["workers"] if self.fake or owned.get(w)] or rec["workers"]
                pulls = _Background(lambda: self.prepull(gpu_nodes, prepull_images))
            else:
                pulls = None
            with t.phase("registry-configmap"):
                self.apply_registry_configmap()
            with t.phase("plugin-image") as rec:
                if build is not None:
                    rec["overlapped_build_s"] = build.join()
                    image = self.plugin_image_stage2()
                else:
                    image = self.build_plugin_image()
            with t.phase("plugin-deploy"):
                self.deploy_plugin(image)
            with t.phase("plugin-ready"):
                self.wait_plugin_ready()
            with t.phase("capacity") as rec:
                rec["amd.com/gpu"] = self.wait_capacity()
            if pulls is not None:
                with t.phase("prepull-wait") as rec:
                    rec["overlapped_pull_s"] = pulls.join()
        except (ProvisionError, CommandError):
            if build is not None:
                build.join(reraise=False)
            if self.created_cluster and not self.s.keep_on_fail and not self.runner.dry_run:
                self.out(f"create failed; deleting cluster '{self.s.cluster_name}' (use --keep-on-fail to keep it)")
                self.kind("delete", "cluster", "--name", self.s.cluster_name, check=False)
            raise
        finally:
            self.timer.meta.update(cluster=self.s.cluster_name, fake=self.fake, runtime=getattr(self.rt, "name", None))
            self.timer.write(self.s.timings_json)
        if self.fake:
            self.out(C.SUCCESS_FMT_FAKE.format(gpu_type=gpu_type))
        else:
            self.out(C.SUCCESS_FMT_REAL.format(gpu_type=gpu_type, n=self.expected_capacity))
        return 0

    def delete(self, keep_registry: bool = False) -> int:
        """Delete the cluster, then stop and remove the registry
        (kind-gpu-sim.sh:338-361). ``keep_registry`` leaves the registry and
        the images pushed to it (``kgs bench --sweep`` between its points)."""
        rt = self.ensure_runtime()
        if self.cluster_exists() or self.runner.dry_run:
            self.out(f"Deleting kind cluster '{self.s.cluster_name}'...")
            self.kind("delete", "cluster", "--name", self.s.cluster_name)
        else:
            self.out(f"Kind cluster '{self.s.cluster_name}' does not exist. Skipping delete.")
        if keep_registry:
            if not self.runner.dry_run:
                shutil.rmtree(self.state_dir, ignore_errors=True)
            return 0
        name = C.REGISTRY_NAME
        self.out(f"Stopping {name} (if running)...")
        if rt.running_id(name) or self.runner.dry_run:  # Q10: test the output, not the exit code
            if not rt.cr("stop", name, check=False).ok:
                self.out(f"Warning: Failed to stop {name}")
        else:
            self.out(f"No running container named '{name}' to stop.")
        self.out(f"Removing {name} (if exists)...")
        if rt.exists(name) or self.runner.dry_run:
            if not rt.cr("rm", name, check=False).ok:
                self.out(f"Warning: Failed to remove {name}")
        else:
            self.out(f"No container named '{name}' to remove.")
        if not self.runner.dry_run:
            shutil.rmtree(self.state_dir, ignore_errors=True)
        return 0

    def load(self) -> int:
        if not self.s.image_name or self.s.image_name == C.DEFAULT_IMAGE_NAME:
            raise ProvisionError("ERROR: load needs --image-name=<image>")
        self.ensure_runtime().load_into_kind(self.s.image_name, self.s.cluster_name)
        return 0

    def status(self, as_json: bool = False) -> int:
        info = {"cluster": self.s.cluster_name, "exists": self.cluster_exists()}
        if info["exists"]:
            info["allocatable"] = self.allocatable()
            r = self.kubectl("get", "pods", "-n", C.PLUGIN_NAMESPACE, "-l", f"app={C.PLUGIN_APP_LABEL}",
                             "-o", "wide", check=False, mutating=False)
            info["plugin_pods"] = r.stdout.strip().splitlines()
        if as_json:
            self.out(json.dumps(info, indent=1))
        else:
            self.out(f"cluster {info['cluster']}: {'present' if info['exists'] else 'absent'}")
            for n, v in info.get("allocatable", {}).items():
                self.out(f"  {n}: {C.RESOURCE_NAME}={v}")
            for line in info.get("plugin_pods", []):
                self.out(f"  {line}")
        return 0


def _natural_key(name: str) -> list:
    """``worker2`` < ``worker10`` (digit runs compare as numbers)."""
    import re

    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", name)]


class _Background:
    """Run ``fn`` on a thread; ``join`` re-raises its exception in the caller."""

    def __init__(self, fn):
        import threading

        self._exc = None
        self._t0 = time.monotonic()
        self._dt = None

        def run():
            try:
                fn()
            except BaseException as e:  # surfaced by join()
                self._exc = e
            finally:
                self._dt = time.monotonic() - self._t0

        self._thread = threading.Thread(target=run, name="kgs-image-build", daemon=True)
        self._thread.start()

    def join(self, reraise: bool = True) -> float:
        self._thread.join()
        if reraise and self._exc is not None:
            raise self._exc
        return round(self._dt or 0.0, 4)
