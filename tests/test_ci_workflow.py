"""Rehearse .github/workflows/rocm-ci.yaml hermetically.

VERDICT r2 noted that rocm-ci.yaml had never run. GitHub runners are out of
reach, but the workflow's own shell steps can run, in order, against the
stateful fake kind/kubectl/docker from tests/fakebin. The steps covered are:
the native build, the plugin image, `create rocm` on the CPU-only fake path,
the workload image, the test pod, its log check, and `delete`. Network-only
steps (curl downloads, pip installs) are skipped after checking that their
versions are pinned. A step that would fail on a runner because of our code
(a wrong verb, a missing file, a log line the grep does not find) fails here.
"""
import os
import subprocess
import sys

import yaml

from test_cli import world  # noqa: F401 - the fake-tool fixture

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WF = os.path.join(ROOT, ".github", "workflows", "rocm-ci.yaml")


def _steps():
    wf = yaml.safe_load(open(WF))
    (job,) = wf["jobs"].values()
    return [s for s in job["steps"] if "run" in s]


def test_rocm_ci_steps_run_against_the_fakes(world, tmp_path):  # noqa: F811
    work = tmp_path / "ci"
    work.mkdir()
    for name in ("pods", "kind-gpu-sim.sh", "kgs", "images", "native"):
        (work / name).symlink_to(os.path.join(ROOT, name))
    env = dict(os.environ, PYTHONPATH=ROOT, PYTHON=sys.executable)
    env["PATH"] = f"{os.path.dirname(sys.executable)}:{env['PATH']}"
    native_out = str(tmp_path / "kgs-native")
    ran, skipped = [], []
    for step in _steps():
        cmd = step["run"]
        if "curl " in cmd or "pip install" in cmd:
            if "pip install" in cmd:
                assert all("==" in t for t in cmd.split("install", 1)[1].split() if not t.startswith("-")), cmd
            skipped.append(cmd)
            continue
        cmd = cmd.replace("/tmp/kgs-native", native_out).replace("python -m", f"{sys.executable} -m")
        r = subprocess.run(["bash", "-eo", "pipefail", "-c", cmd], cwd=str(work), env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, f"step {step.get('name', cmd)!r} failed:\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}"
        ran.append(step.get("name", cmd))
    # the native core the plugin image ships was built by the same command
    assert any(n.startswith("_gpuinfo") for n in os.listdir(native_out))
    # plugin + workload images built and pushed to the local registry, the pod ran, the cluster is gone
    builds = [a for a in world.calls("docker", "build")]
    assert any("Dockerfile.deviceplugin" in " ".join(a) for a in builds)
    assert any("Dockerfile.rocm-test" in " ".join(a) for a in builds)
    assert "Hello from fake ROCm GPU node" in (work / "pod.log").read_text()
    assert (work / "create-timings.json").exists()
    assert world.state()["clusters"] == {}
    assert len(ran) >= 6 and len(skipped) == 2


def test_tests_workflow_fails_on_native_build_and_pins_rocm():
    """the CPU tier's native build must not be masked
    (``|| true`` let it run on the Python fallback), and the gfx950 build job
    must use a pinned ROCm image, not a moving ``:latest`` (the reference's
    unpinned-upstream drift, Q6)."""
    from kgs import config

    wf = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "tests.yaml")))
    runs = [s["run"] for job in wf["jobs"].values() for s in job["steps"] if "run" in s]
    assert not any("|| true" in r or "|| :" in r for r in runs), runs
    build = [r for r in runs if "kgs.utils.build" in r]
    assert build and all("--only gpuinfo" in r for r in build)
    images = [job["container"] for job in wf["jobs"].values() if "container" in job]
    assert images == [config.ROCM_DEV_IMAGE]
    assert all(not i.endswith(":latest") and ":" in i.rsplit("/", 1)[-1] for i in images)
