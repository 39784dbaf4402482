"""``kgs bench``: the headline metric -- cluster create -> GPU pod Running.

Phases (all in one PhaseTimer, written to ``--timings-json``):
  workload-image  the gpu-rocm-test image exists locally, or is built (and
                  pushed to the local registry) now -- explicitly, before the
                  cluster, instead of a late ImagePullBackOff after scheduling
  create phases (kgs.cluster.Provisioner.create)
  pod-apply       kubectl apply the gpu-rocm-test pod (N x amd.com/gpu)
  pod-running     kubectl wait --for=jsonpath={.status.phase}=Running
  pod-ready       kubectl wait --for=condition=Ready
and the headline ``create_to_running_s`` = start of create .. pod Running. The
pod's own result line (GEMM TFLOPS, all-reduce busBW) is parsed from its logs
when it has finished its run.

Mirrors the reference CI (rocm-ci.yaml:28-39: create, kubectl create pod,
kubectl wait Ready --timeout=60s, kubectl logs), timed phase by phase. Needs a
docker/podman + kind + kubectl host; none exists in the build container or on
the gpurun boxes, so the e2e number is produced by this tool on such a host
(BASELINE.md says which numbers were measured where).
"""
from __future__ import annotations

import json
import time

from . import config as C
from . import manifests


def workload_image(p) -> str:
    rt = p.ensure_runtime()
    repo = f"{C.WORKLOAD_IMAGE_REPO}:{C.WORKLOAD_IMAGE_TAG}"
    return f"localhost/{repo}" if rt.name == "podman" else f"{p.s.registry_host}/{repo}"


def run_e2e(p, gpus: int = 1, pod_timeout: int = C.TEST_POD_READY_TIMEOUT_S, keep: bool = False,
            workload_image: str | None = None, pod_command: list | None = None) -> int:
    summary = e2e_once(p, gpus=gpus, pod_timeout=pod_timeout, keep=keep, workload_image=workload_image,
                       pod_command=pod_command)
    p.out(json.dumps(summary))
    return 0


def result_timeout(pod_timeout: float) -> float:
    """Seconds to wait for the test pod's result line once it is Ready."""
    return max(1.0, pod_timeout * 10.0)


def e2e_once(p, gpus: int = 1, pod_timeout: int = C.TEST_POD_READY_TIMEOUT_S, keep: bool = False,
             workload_image: str | None = None, pod_command: list | None = None,
             keep_registry: bool = False) -> dict:
    """One create -> pod Running -> logs (-> delete) pass; returns the summary.
    ``keep_registry``: the final delete leaves the local registry (and the
    images in it) for the next pass."""
    t = p.timer
    t_start = time.perf_counter()
    image = workload_image or globals()["workload_image"](p)
    with t.phase("workload-image") as rec:
        rec["image"] = image
        if workload_image:
            rec["provided"] = True  # a user-supplied image: their registry, their build
        elif p.runner.dry_run or p.ensure_runtime().image_exists(image):
            rec["cached"] = True
            if not p.runner.dry_run and p.ensure_runtime().name == "docker":
                # built earlier, but the registry may be a fresh one (kgs delete
                # removes it): the nodes pull from the registry, so push (a no-op
                # upload when the registry already has the layers)
                p.start_registry()
                p.ensure_runtime().cr("push", image)
                rec["pushed"] = True
        else:
            from .images import build_images

            p.out(f"workload image {image} not found locally; building it")
            build_images(p, workload=True, plugin=False)
            rec["built"] = True
    if p.ensure_runtime().name != "podman" and not p.s.extra.get("no_prepull"):
        # pull the (multi-GB) workload image into the GPU workers during create,
        # overlapped with plugin deploy/readiness, instead of after scheduling
        p.s.extra["prepull"] = [image]
    p.create("rocm")
    if p.ensure_runtime().name == "podman" and not workload_image:
        with t.phase("workload-image-load"):
            p.rt.load_into_kind(image, p.s.cluster_name)
    pod = manifests.gpu_test_pod(image, gpus=gpus, command=pod_command)
    name = pod["metadata"]["name"]
    result = {}
    try:
        with t.phase("pod-apply"):
            p.kubectl("apply", "-f", "-", input=manifests.dump(pod))
        with t.phase("pod-running"):
            p.kubectl("wait", "--for=jsonpath={.status.phase}=Running", f"pod/{name}", f"--timeout={pod_timeout}s")
        running_s = time.perf_counter() - t_start
        with t.phase("pod-ready"):
            p.kubectl("wait", "--for=condition=Ready", f"pod/{name}", f"--timeout={pod_timeout}s")
        with t.phase("pod-logs"):
            # the pod's result line comes after its workload (GEMM sweep,
            # all-reduce), well after Ready: the same bound as the --no-kind
            # chain, scaled by --pod-timeout (600 s at the default 60 s)
            wait_s = result_timeout(pod_timeout)
            deadline = time.monotonic() + (wait_s if not p.runner.dry_run else 0)
            while True:
                r = p.kubectl("logs", f"pod/{name}", check=False, mutating=False)
                for line in r.stdout.splitlines():
                    if line.startswith("{") and '"mode"' in line:
                        result = json.loads(line)
                if result or time.monotonic() > deadline:
                    break
                time.sleep(2)
            if not result and not p.runner.dry_run:
                raise TimeoutError(f"pod/{name}: no result line in its logs within {wait_s:.0f}s "
                                   f"(--pod-timeout {pod_timeout}s x 10)")
        t.meta.update(create_to_running_s=round(running_s, 4), gpus_requested=gpus, pod_result=result)
    finally:
        t.write(p.s.timings_json)
        if not keep and not p.runner.dry_run:
            p.delete(keep_registry=keep_registry)
    summary = {"metric": "cluster-create->GPU-pod-Running", "value": t.meta.get("create_to_running_s"),
               "unit": "s", "gpus": gpus, "advertised": p.expected_capacity, "fake": p.fake,
               "phases": {ph["phase"]: ph["seconds"] for ph in t.phases}}
    if result.get("gemm_tflops_total"):
        summary["in_pod_gemm_tflops"] = result["gemm_tflops_total"]
    return summary


def run_sweep(make_provisioner, counts: list, pod_gpus: int | None = None, sweep_json: str | None = None,
              out=print, no_kind: bool = False, **kw) -> int:
    """``kgs bench --sweep 1,2,4,8``: the headline at each advertised-GPU count.

    For every N: a fresh ``create --gpus N`` (exactly N GPUs advertised) ->
    gpu-rocm-test pod requesting ``pod_gpus`` (default N: the pod takes all of
    them, BASELINE config 4; ``--pod-gpus 1`` is config 3) -> Running -> logs
    (in-pod GEMM TFLOPS) -> delete. With ``no_kind`` each point is the no-kind
    chained tail instead (kgs/e2e_nokind.py). One JSON document: the per-N
    points plus a ``table`` of create->Running seconds and in-pod TFLOPS.
    A failing point is recorded with its error and the sweep goes on, so one
    bad count does not hide the others; the exit status is then 1.
    """
    points = []
    last = None
    for i, n in enumerate(counts):
        want = pod_gpus or n
        try:
            if no_kind:
                from .e2e_nokind import nokind_once

                pt = nokind_once(gpus=want, advertise=n, **kw)
            else:
                # the registry (with the plugin and workload images) outlives
                # the points; the last one removes it as `kgs delete` does
                last = make_provisioner(n)
                pt = e2e_once(last, gpus=want, keep_registry=i < len(counts) - 1, **kw)
            pt["ok"] = True
        except Exception as e:  # noqa: BLE001 - recorded per point
            pt = {"ok": False, "error": f"{type(e).__name__}: {e}"}
        pt.update(advertised=n, pod_gpus=want)
        points.append(pt)
    if last is not None and not points[-1]["ok"] and not last.runner.dry_run:
        last.delete()  # a failed last point: still leave no registry behind
    doc = {
        "metric": ("device-plugin start -> first in-pod GEMM (no kind)" if no_kind
                   else "cluster-create->GPU-pod-Running"),
        "unit": "s",
        "sweep": list(counts),
        "points": points,
        "table": [{"advertised": pt["advertised"], "pod_gpus": pt["pod_gpus"], "seconds": pt.get("value"),
                   "in_pod_gemm_tflops": pt.get("in_pod_gemm_tflops"), "ok": pt["ok"]} for pt in points],
    }
    text = json.dumps(doc, indent=1)
    if sweep_json:
        with open(sweep_json, "w") as f:
            f.write(text + "\n")
    out(text)
    return 0 if all(pt["ok"] for pt in points) else 1
