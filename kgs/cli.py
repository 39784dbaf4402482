"""``kgs`` command line -- drop-in for ``kind-gpu-sim.sh``.

  kgs create [rocm] [--registry-port=N] [--cluster-name=S] [--runtime=docker|podman]
                    [--gpus=N] [--workers=N] [--gpu-partition=all-on-first|split] [--fake-gpus=N]
                    [--fake-mode=patch|plugin] [--timings-json=F] [--dry-run] [--keep-on-fail]
  kgs delete [--cluster-name=S]
  kgs load   --image-name=IMG [--cluster-name=S]
  kgs status [--json]
  kgs bench  [--gpus=N] [--pod-gpus=M] create --gpus N -> gpu-rocm-test (M GPUs, default N) Running,
             [--sweep=1,2,4,8]        per-phase JSON; --sweep repeats it per advertised count
             [--no-kind]              the docker-free chained tail instead (plugin -> pod -> GEMM)
  kgs images [--workload] [--plugin] [--amdsmi-lib]  build the in-tree images
  kgs pod NAME [--registry-port=N]   print pods/NAME.yaml with the image on the
                                     configured local registry (| kubectl create -f -)

Flags are accepted in both ``--k=v`` and ``--k v`` form and anywhere on the line
(the reference scans all argv for its three flags, kind-gpu-sim.sh:31-43). Unlike
the reference, an unknown flag is an error, and the GPU type is a real
positional (Q1). Usage errors exit 1, as ``usage()`` does (kind-gpu-sim.sh:364-367).
"""
from __future__ import annotations

import argparse
import logging
import sys

from . import config as C

VERBS = ("create", "delete", "load", "status", "bench", "images", "doctor", "pod")


class _Parser(argparse.ArgumentParser):
    def error(self, message):  # exit 1 like the reference's usage()
        self.print_usage(sys.stderr)
        print(f"{self.prog}: error: {message}", file=sys.stderr)
        raise SystemExit(1)


def build_parser(prog: str = "kgs") -> argparse.ArgumentParser:
    ap = _Parser(prog=prog, description="MI355X-native kind GPU provisioner (kind-gpu-sim compatible)",
                 usage=C.USAGE.format(prog=prog))
    ap.add_argument("verb", nargs="?", choices=VERBS)
    ap.add_argument("gpu_type", nargs="?", default="rocm")
    ap.add_argument("--registry-port", type=int, default=C.DEFAULT_REGISTRY_PORT)
    ap.add_argument("--cluster-name", default=C.DEFAULT_CLUSTER_NAME)
    ap.add_argument("--image-name", default=C.DEFAULT_IMAGE_NAME)
    ap.add_argument("--runtime", choices=("docker", "podman"), default=None)
    ap.add_argument("--workers", type=int, default=C.DEFAULT_WORKERS)
    ap.add_argument("--gpu-partition", choices=("all-on-first", "split"), default="all-on-first")
    ap.add_argument("--fake-gpus", type=int, default=None,
                    help="force the simulated path with N amd.com/gpu per worker (reference default: 2)")
    ap.add_argument("--fake-mode", choices=("patch", "plugin"), default="patch",
                    help="fake capacity via node-status patch (reference) or via the plugin's fake source")
    ap.add_argument("--registry-bind", default="127.0.0.1")
    ap.add_argument("--kind-node-image", default=None)
    ap.add_argument("--base-mirror", default=C.BASE_MIRROR,
                    help="registry prefix for library base images (python, registry); reference: patch_dockerfile")
    ap.add_argument("--rocm-base-image", default=C.ROCM_BASE_IMAGE, help="PyTorch-ROCm base of the workload image")
    ap.add_argument("--rocm-dev-image", default=C.ROCM_DEV_IMAGE,
                    help="ROCm image the device-plugin build copies the amd-smi header and libraries from "
                         "(docs/deviceplugin.md: pull size, lighter sources)")
    ap.add_argument("--rocm-mirror", default=None,
                    help=f"registry prefix replacing {C.ROCM_REGISTRY} in the ROCm image references "
                         "(plugin amd-smi stage, workload base), e.g. a pull-through cache")
    ap.add_argument("--plugin-image", default=None, help="use a prebuilt device-plugin image")
    ap.add_argument("--skip-build", action="store_true")
    ap.add_argument("--ready-timeout", type=int, default=C.PLUGIN_READY_TIMEOUT_S)
    ap.add_argument("--timings-json", default=None)
    ap.add_argument("--dev-root", default="/", help="host root for GPU discovery (tests)")
    ap.add_argument("--dry-run", action="store_true", help="print the command plan, change nothing")
    ap.add_argument("--keep-on-fail", action="store_true")
    ap.add_argument("--serial", action="store_true",
                    help="build the plugin image after the cluster (default: concurrently with kind create)")
    ap.add_argument("--json", action="store_true")
    # bench/images options
    ap.add_argument("--gpus", type=int, default=None,
                    help="advertise exactly N of the host's healthy GPUs (one xGMI island, fewest NUMA nodes; "
                         "default: all). bench: also the test pod's request unless --pod-gpus")
    ap.add_argument("--pod-gpus", type=int, default=None,
                    help="bench: amd.com/gpu requested by the test pod (default: --gpus, or 1)")
    ap.add_argument("--sweep", default=None,
                    help="bench: comma list of advertised GPU counts, e.g. 1,2,4,8 (one create..delete per count)")
    ap.add_argument("--sweep-json", default=None, help="bench --sweep: write the per-count JSON here")
    ap.add_argument("--pod-timeout", type=int, default=C.TEST_POD_READY_TIMEOUT_S)
    ap.add_argument("--keep", action="store_true", help="bench: keep the cluster afterwards")
    ap.add_argument("--no-kind", action="store_true",
                    help="bench: no docker/kind -- plugin process -> kubelet register -> capacity -> Allocate -> pod "
                         "entrypoint first GEMM, chained and timed (kgs/e2e_nokind.py)")
    ap.add_argument("--gemm-size", type=int, default=8192, help="bench --no-kind: the pod's first GEMM size")
    ap.add_argument("--workload-image", default=None)
    ap.add_argument("--workload", action="store_true")
    ap.add_argument("--plugin", action="store_true")
    ap.add_argument("--amdsmi-lib", action="store_true",
                    help="images: build the small amd-smi source image (images/Dockerfile.amdsmi-lib) for "
                         "--rocm-dev-image")
    ap.add_argument("-v", "--verbose", action="store_true")
    return ap


def settings_from(a) -> C.Settings:
    return C.Settings(
        registry_port=a.registry_port, cluster_name=a.cluster_name, image_name=a.image_name, runtime=a.runtime,
        workers=a.workers, gpus=a.gpus, gpu_partition=a.gpu_partition, fake_gpus=a.fake_gpus, fake_mode=a.fake_mode,
        registry_bind=a.registry_bind, kind_node_image=a.kind_node_image, dry_run=a.dry_run,
        keep_on_fail=a.keep_on_fail, skip_build=a.skip_build, timings_json=a.timings_json,
        plugin_image=a.plugin_image, ready_timeout_s=a.ready_timeout, dev_root=a.dev_root,
        base_mirror=a.base_mirror, rocm_base_image=a.rocm_base_image, rocm_dev_image=a.rocm_dev_image,
        rocm_mirror=a.rocm_mirror, extra={"serial": a.serial},
    )


def _parse_counts(text: str) -> list:
    try:
        counts = [int(x) for x in text.replace(" ", "").split(",") if x]
    except ValueError:
        counts = []
    if not counts or any(c < 1 for c in counts):
        raise SystemExit(f"--sweep wants a comma list of GPU counts >= 1, e.g. 1,2,4,8 (got {text!r})")
    return counts


def main(argv=None, prog: str = "kgs") -> int:
    ap = build_parser(prog)
    a = ap.parse_intermixed_args(argv)
    logging.basicConfig(level=logging.DEBUG if a.verbose else logging.INFO, format="%(message)s",
                        stream=sys.stderr)
    if a.verb is None:
        print(C.USAGE.format(prog=prog), file=sys.stderr)
        return 1
    from .cluster import Provisioner, ProvisionError
    from .runtime import RuntimeNotFound
    from .utils.proc import CommandError
    from .e2e import result_timeout

    s = settings_from(a)
    p = Provisioner(s)
    try:
        if a.verb == "create":
            return p.create(a.gpu_type)
        if a.verb == "delete":
            return p.delete()
        if a.verb == "load":
            return p.load()
        if a.verb == "status":
            return p.status(as_json=a.json)
        if a.verb == "pod":
            from .manifests import UnknownPod, render_static_pod

            try:
                sys.stdout.write(render_static_pod(a.gpu_type, s.registry_host))
            except UnknownPod as e:
                print(str(e), file=sys.stderr)
                return 1
            return 0
        if a.verb == "bench" and a.sweep:
            from .e2e import run_sweep

            counts = _parse_counts(a.sweep)
            if a.no_kind:
                kw = dict(dev_root=a.dev_root, fake_gpus=a.fake_gpus or 0, gemm_size=a.gemm_size,
                          timeout=result_timeout(a.pod_timeout))
                return run_sweep(None, counts, pod_gpus=a.pod_gpus, sweep_json=a.sweep_json, out=p.out,
                                 no_kind=True, **kw)

            def make(n):
                st = settings_from(a)
                st.gpus = n
                st.timings_json = f"{a.timings_json}.gpus{n}.json" if a.timings_json else None
                return Provisioner(st, runner=p.runner, out=p.out)

            return run_sweep(make, counts, pod_gpus=a.pod_gpus, sweep_json=a.sweep_json, out=p.out,
                             pod_timeout=a.pod_timeout, keep=False, workload_image=a.workload_image)
        if a.verb == "bench" and a.no_kind:
            from .e2e_nokind import run_nokind

            return run_nokind(gpus=a.pod_gpus or a.gpus or 1, advertise=a.gpus, dev_root=a.dev_root,
                              fake_gpus=a.fake_gpus or 0, gemm_size=a.gemm_size,
                              timeout=result_timeout(a.pod_timeout), timings_json=a.timings_json)
        if a.verb == "bench":
            from .e2e import run_e2e

            return run_e2e(p, gpus=a.pod_gpus or a.gpus or 1, pod_timeout=a.pod_timeout, keep=a.keep,
                           workload_image=a.workload_image)
        if a.verb == "doctor":
            from .doctor import run_doctor

            return run_doctor(s, as_json=a.json)
        if a.verb == "images":
            from .images import build_images

            only_lib = a.amdsmi_lib and not (a.workload or a.plugin)
            return build_images(p, workload=not only_lib and (a.workload or not a.plugin),
                                plugin=not only_lib and (a.plugin or not a.workload), amdsmi_lib=a.amdsmi_lib)
    except (ProvisionError, RuntimeNotFound) as e:
        print(str(e), file=sys.stderr)
        return 1
    except TimeoutError as e:  # a bench wait ran out (pod result, plugin capacity, ...)
        print(f"ERROR: {e}", file=sys.stderr)
        return 1
    except CommandError as e:
        print(f"ERROR: {e}", file=sys.stderr)
        if e.stderr:
            print(e.stderr.rstrip(), file=sys.stderr)
        return 1
    finally:
        if s.dry_run and p.runner.plan:
            import shlex

            print("# command plan:", file=sys.stderr)
            for step in p.runner.plan:
                print("  " + shlex.join(step["argv"]) + ("  <<stdin" if "stdin" in step else ""), file=sys.stderr)
    return 1
