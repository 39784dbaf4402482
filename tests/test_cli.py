"""T1: the CLI against stateful fake kind/kubectl/docker/podman
binaries on PATH. Asserts the reference's observable contract (§2.2) and the
deliberate fixes (Q1-Q15)."""
import json
import os
import stat
import sys

import pytest
import yaml

from kgs import config as C
from kgs.cli import main
from kgs.gpuinfo.fake import make_fake_mi355x

FAKE_TOOL = os.path.join(os.path.dirname(__file__), "fakebin", "fake_tool.py")


@pytest.fixture
def world(tmp_path, monkeypatch):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    os.chmod(FAKE_TOOL, os.stat(FAKE_TOOL).st_mode | stat.S_IEXEC | stat.S_IXGRP | stat.S_IXOTH)
    for tool in ("kind", "kubectl", "docker", "podman", "systemctl"):
        (bindir / tool).symlink_to(FAKE_TOOL)
    py_dir = os.path.dirname(sys.executable)
    monkeypatch.setenv("PATH", f"{bindir}:{py_dir}:/usr/bin:/bin")
    monkeypatch.setenv("KGS_FAKE_STATE", str(tmp_path / "state.json"))
    monkeypatch.setenv("KGS_FAKE_LOG", str(tmp_path / "log.jsonl"))
    monkeypatch.delenv("KGS_FAKE_FAIL", raising=False)
    work = tmp_path / "work"
    work.mkdir()
    monkeypatch.chdir(work)
    empty_root = tmp_path / "nogpu"
    empty_root.mkdir()

    class W:
        path = tmp_path
        cwd = work
        nogpu = str(empty_root)

        @staticmethod
        def state():
            p = tmp_path / "state.json"
            return json.loads(p.read_text()) if p.exists() else {}

        @staticmethod
        def log():
            p = tmp_path / "log.jsonl"
            return [json.loads(x) for x in p.read_text().splitlines()] if p.exists() else []

        @staticmethod
        def calls(tool, *prefix):
            return [e["argv"] for e in W.log() if e["tool"] == tool and e["argv"][: len(prefix)] == list(prefix)]

        @staticmethod
        def kubectl_calls(*prefix):
            out = []
            for e in W.log():
                if e["tool"] != "kubectl":
                    continue
                a = e["argv"]
                if a[:1] == ["--context"]:
                    a = a[2:]
                if a[: len(prefix)] == list(prefix):
                    out.append((a, e["stdin"]))
            return out

    return W


def run(*args):
    return main(list(args))


def test_create_fake_path_matches_reference_contract(world, capsys):
    rc = run("create", "--dev-root", world.nogpu)
    out = capsys.readouterr().out
    assert rc == 0
    assert "Simulated GPU Kind cluster is ready for 'rocm'!" in out
    st = world.state()
    # registry: name, restart policy, port mapping bound to localhost (Q4), on the kind network
    reg = st["containers"]["kind-registry"]
    assert reg["running"] and "--restart=always" in reg["args"]
    assert "127.0.0.1:5000:5000" in reg["args"] and reg["image"] == C.REGISTRY_IMAGE
    assert "kind" in reg["networks"]
    cl = st["clusters"]["kind-gpu-sim"]
    assert sorted(cl["nodes"]) == ["kind-gpu-sim-control-plane", "kind-gpu-sim-worker", "kind-gpu-sim-worker2"]
    for n in ("kind-gpu-sim-worker", "kind-gpu-sim-worker2"):
        node = cl["nodes"][n]
        assert node["labels"] == {"hardware-type": "gpu", "node-role.kubernetes.io/worker": "",
                                  "rocm.amd.com/gpu.present": "true"}
        assert node["taints"] == ["gpu=true:NoSchedule"]
        assert node["capacity"] == {"amd.com/gpu": "2"}  # kind-gpu-sim.sh:113
    cp = cl["nodes"]["kind-gpu-sim-control-plane"]
    assert cp["labels"] == {} and cp["taints"] == []
    kinds = [o["kind"] for o in cl["objects"]]
    assert kinds == ["ConfigMap", "DaemonSet"]
    cm = cl["objects"][0]
    assert cm["metadata"] == {"name": "local-registry-hosting", "namespace": "kube-public"}
    assert 'host: "localhost:5000"' in cm["data"]["localRegistryHosting.v1"]
    ds = cl["objects"][1]
    assert ds["metadata"] == {"name": "amdgpu-device-plugin-daemonset", "namespace": "kube-system"}
    tpl = ds["spec"]["template"]
    assert tpl["metadata"]["labels"] == {"app": "amdgpu-device-plugin"}
    assert tpl["spec"]["nodeSelector"] == {"hardware-type": "gpu"}
    assert tpl["spec"]["tolerations"] == [{"key": "gpu", "operator": "Equal", "value": "true",
                                           "effect": "NoSchedule"}]
    ctr = tpl["spec"]["containers"][0]
    assert ctr["name"] == "amdgpu-dp-ds" and ctr["image"] == "localhost:5000/amdgpu-dp:dev"
    assert ctr["securityContext"] == {"privileged": True} and ctr["imagePullPolicy"] == "IfNotPresent"
    mounts = {m["mountPath"] for m in ctr["volumeMounts"]}
    assert {"/var/lib/kubelet/device-plugins", "/dev", "/sys", "/etc/kgs"} <= mounts  # Q7 fixed
    assert "localhost:5000/amdgpu-dp:dev" in st["registry_images"]
    # kind config: config_path + bind-mounted hosts.toml (Q2/Q3), 1 CP + 2 workers
    cfg = yaml.safe_load((world.cwd / "kind-config.yaml").read_text())
    assert cfg["kind"] == "Cluster" and cfg["apiVersion"] == "kind.x-k8s.io/v1alpha4"
    assert [n["role"] for n in cfg["nodes"]] == ["control-plane", "worker", "worker"]
    assert 'config_path = "/etc/containerd/certs.d"' in cfg["containerdConfigPatches"][0]
    hosts = world.cwd / ".kgs" / "kind-gpu-sim" / "certs.d" / "localhost:5000" / "hosts.toml"
    assert hosts.read_text() == '[host."http://kind-registry:5000"]\n  capabilities = ["pull", "resolve"]\n'
    # no per-node docker exec / SIGHUP (Q2), labels + taint batched in one call each
    assert world.calls("docker", "exec") == []
    assert len(world.kubectl_calls("label")) == 1 and len(world.kubectl_calls("taint")) == 1
    # no GPU passthrough mounts on a CPU-only host
    assert all(m["containerPath"] not in ("/dev/kfd",) for n in cfg["nodes"] for m in n.get("extraMounts", []))


def test_create_real_gpus_all_on_first(world, tmp_path, capsys):
    host = make_fake_mi355x(tmp_path / "host8")
    rc = run("create", "rocm", "--dev-root", str(host), "--timings-json", str(tmp_path / "t.json"))
    out = capsys.readouterr().out
    assert rc == 0, out
    assert "8 amd.com/gpu advertised" in out
    cfg = yaml.safe_load((world.cwd / "kind-config.yaml").read_text())
    w1, w2 = cfg["nodes"][1], cfg["nodes"][2]
    w1_paths = [m["containerPath"] for m in w1["extraMounts"]]
    assert "/dev/kfd" in w1_paths and sum(p.startswith("/dev/dri/renderD") for p in w1_paths) == 8
    assert "/dev/kfd" not in [m["containerPath"] for m in w2["extraMounts"]]
    part = json.loads((world.cwd / ".kgs" / "kind-gpu-sim" / "gpus.json").read_text())
    assert part["nodes"]["kind-gpu-sim-worker"] == [128 + 8 * i for i in range(8)]
    assert part["nodes"]["kind-gpu-sim-worker2"] == []
    st = world.state()["clusters"]["kind-gpu-sim"]
    # capacity comes from the plugin (kubelet-managed), never from a status patch (H5)
    assert world.kubectl_calls("patch") == []
    assert st["nodes"]["kind-gpu-sim-worker"]["allocatable"] == {"amd.com/gpu": "8"}
    assert st["nodes"]["kind-gpu-sim-worker"]["labels"]["kgs.amd.com/gpu-partition"] == "8"
    t = json.loads((tmp_path / "t.json").read_text())
    names = [p["phase"] for p in t["phases"]]
    assert names == ["runtime", "discover", "registry", "kind-config", "kind-create", "registry-network", "nodes",
                     "registry-configmap", "plugin-image", "plugin-deploy", "plugin-ready", "capacity"]
    assert t["fake"] is False and all(p["ok"] for p in t["phases"])


def test_create_split_partition(world, tmp_path):
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("create", "--dev-root", str(host), "--gpu-partition", "split") == 0
    part = json.loads((world.cwd / ".kgs" / "kind-gpu-sim" / "gpus.json").read_text())["nodes"]
    assert part["kind-gpu-sim-worker"] == [128, 136, 144, 152]  # NUMA 0
    assert part["kind-gpu-sim-worker2"] == [160, 168, 176, 184]  # NUMA 1
    st = world.state()["clusters"]["kind-gpu-sim"]["nodes"]
    assert st["kind-gpu-sim-worker"]["allocatable"] == {"amd.com/gpu": "4"}
    assert st["kind-gpu-sim-worker2"]["allocatable"] == {"amd.com/gpu": "4"}


def test_create_is_idempotent(world, capsys):
    assert run("create", "--dev-root", world.nogpu) == 0
    assert run("create", "--dev-root", world.nogpu) == 0
    out = capsys.readouterr().out
    assert "Registry 'kind-registry' already running." in out
    assert "already exists; reconciling" in out
    assert len(world.calls("kind", "create", "cluster")) == 1  # Q15
    assert len(world.calls("docker", "run")) == 1


def test_create_detects_drift_fake_to_real(world, tmp_path, capsys):
    """A cluster made on the CPU-only (fake) path has no /dev/kfd mounts; a
    second create on a GPU host must fail fast with a delete-first message
    instead of timing out on capacity."""
    assert run("create", "--dev-root", world.nogpu) == 0
    host = make_fake_mi355x(tmp_path / "host8")
    capsys.readouterr()
    assert run("create", "--dev-root", str(host)) == 1
    out = capsys.readouterr()
    msg = out.out + out.err
    assert "different shape" in msg and "GPU path" in msg and "kgs delete" in msg
    assert len(world.calls("kind", "create", "cluster")) == 1
    assert "kind-gpu-sim" in world.state()["clusters"]  # the existing cluster is left alone
    # after delete the GPU create goes through
    assert run("delete") == 0
    assert run("create", "--dev-root", str(host)) == 0


def test_create_detects_partition_and_worker_drift(world, tmp_path, capsys):
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("create", "--dev-root", str(host)) == 0
    capsys.readouterr()
    assert run("create", "--dev-root", str(host), "--gpu-partition", "split") == 1
    out = capsys.readouterr()
    assert "GPU partition" in out.out + out.err
    assert run("create", "--dev-root", str(host)) == 0  # same shape: reconcile


def test_delete_then_delete_again(world, capsys):
    assert run("create", "--dev-root", world.nogpu) == 0
    assert run("delete") == 0
    st = world.state()
    assert st["clusters"] == {} and "kind-registry" not in st["containers"]
    capsys.readouterr()
    assert run("delete") == 0
    out = capsys.readouterr().out
    assert "Kind cluster 'kind-gpu-sim' does not exist. Skipping delete." in out
    assert "No running container named 'kind-registry' to stop." in out
    assert "No container named 'kind-registry' to remove." in out
    assert not (world.cwd / ".kgs" / "kind-gpu-sim").exists()


def test_load_docker_and_podman(world):
    assert run("create", "--dev-root", world.nogpu) == 0
    assert run("load", "--image-name=myimg:1") == 0
    assert world.calls("kind", "load", "docker-image") == [["load", "docker-image", "myimg:1", "--name",
                                                             "kind-gpu-sim"]]
    assert run("load", "--image-name", "myimg:2", "--runtime", "podman") == 0
    saves = world.calls("podman", "save")
    assert saves and saves[0][1] == "myimg:2"
    archive = saves[0][saves[0].index("-o") + 1]
    assert archive != "/tmp/image.tar" and not os.path.exists(archive)  # Q9: private, removed
    assert world.calls("kind", "load", "image-archive")[0][2] == archive


def test_load_requires_image(world, capsys):
    assert run("load") == 1
    assert "--image-name" in capsys.readouterr().err


def test_usage_and_bad_verbs(world, capsys):
    assert run() == 1
    assert "Usage:" in capsys.readouterr().err
    with pytest.raises(SystemExit) as e:
        run("frobnicate")
    assert e.value.code == 1
    assert run("create", "nvidia", "--dev-root", world.nogpu) == 1
    assert "Unknown GPU type: nvidia" in capsys.readouterr().err
    with pytest.raises(SystemExit) as e:
        run("create", "--no-such-flag")
    assert e.value.code == 1


def test_flags_anywhere_both_forms(world):
    # Q1: flags before the verb, `=` and space forms; gpu type stays positional
    assert run("--cluster-name=foo", "create", "--registry-port", "5001", "rocm", "--dev-root", world.nogpu) == 0
    st = world.state()
    assert "foo" in st["clusters"]
    assert "127.0.0.1:5001:5000" in st["containers"]["kind-registry"]["args"]
    cm = st["clusters"]["foo"]["objects"][0]
    assert 'host: "localhost:5001"' in cm["data"]["localRegistryHosting.v1"]
    assert (world.cwd / ".kgs" / "foo" / "certs.d" / "localhost:5001" / "hosts.toml").exists()
    assert all(a[1] == "kind-foo" for a in world.calls("kubectl"))


def test_plugin_not_ready_rolls_back(world, monkeypatch, capsys):
    monkeypatch.setenv("KGS_FAKE_FAIL", "plugin-ready")
    assert run("create", "--dev-root", world.nogpu) == 1
    assert "ERROR: ROCm plugin pods not ready in time" in capsys.readouterr().err
    assert world.state()["clusters"] == {}
    assert run("create", "--dev-root", world.nogpu, "--keep-on-fail") == 1
    assert "kind-gpu-sim" in world.state()["clusters"]


def test_kind_create_failure_exit_1(world, monkeypatch, capsys):
    monkeypatch.setenv("KGS_FAKE_FAIL", "kind-create")
    assert run("create", "--dev-root", world.nogpu) == 1
    assert "failed to create cluster" in capsys.readouterr().err


def test_podman_runtime(world):
    assert run("create", "--runtime", "podman", "--dev-root", world.nogpu) == 0
    build = [e for e in world.log() if e["tool"] == "podman" and e["argv"][0] == "build"][0]
    assert build["env"]["KIND_EXPERIMENTAL_PROVIDER"] == "podman"
    assert build["env"]["BUILDAH_FORMAT"] == "docker"
    ds = world.state()["clusters"]["kind-gpu-sim"]["objects"][1]
    assert ds["spec"]["template"]["spec"]["containers"][0]["image"] == "localhost/amdgpu-dp:dev"
    assert world.calls("kind", "load", "image-archive")
    assert world.calls("podman", "push") == []


def test_docker_preferred_when_both_present(world):
    assert run("create", "--dev-root", world.nogpu) == 0
    assert world.calls("docker", "run") and not world.calls("podman", "run")  # Q14


def test_fake_mode_plugin(world):
    assert run("create", "--fake-gpus", "3", "--fake-mode", "plugin") == 0
    assert world.kubectl_calls("patch") == []
    nodes = world.state()["clusters"]["kind-gpu-sim"]["nodes"]
    assert nodes["kind-gpu-sim-worker"]["allocatable"] == {"amd.com/gpu": "3"}
    ds = world.state()["clusters"]["kind-gpu-sim"]["objects"][1]
    env = {e["name"]: e.get("value") for e in ds["spec"]["template"]["spec"]["containers"][0]["env"]}
    assert env["KGS_FAKE_GPUS"] == "3"


def test_dry_run_executes_nothing(world, capsys):
    assert run("create", "--dry-run", "--dev-root", world.nogpu) == 0
    assert world.log() == []
    err = capsys.readouterr().err
    assert "kind create cluster --name kind-gpu-sim" in err
    assert not (world.cwd / "kind-config.yaml").exists()


def test_status(world, capsys):
    assert run("create", "--dev-root", world.nogpu) == 0
    capsys.readouterr()
    assert run("status", "--json") == 0
    info = json.loads(capsys.readouterr().out)
    assert info["exists"] and info["allocatable"] == {"kind-gpu-sim-worker": 2, "kind-gpu-sim-worker2": 2}


def test_bench_e2e(world, tmp_path, capsys):
    rc = run("bench", "--dev-root", world.nogpu, "--timings-json", str(tmp_path / "e2e.json"))
    assert rc == 0
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith('{"metric"')]
    summary = json.loads(lines[-1])
    assert summary["metric"] == "cluster-create->GPU-pod-Running" and summary["value"] > 0
    t = json.loads((tmp_path / "e2e.json").read_text())
    assert [p["phase"] for p in t["phases"]][-4:] == ["pod-apply", "pod-running", "pod-ready", "pod-logs"]
    # a fresh host: the workload image is built (and pushed) first, as its own phase
    assert t["phases"][0]["phase"] == "workload-image" and t["phases"][0].get("built")
    builds = [a for a in world.calls("docker", "build") if "localhost:5000/kgs-rocm-test:dev" in a]
    assert builds and any(a[:2] == ["push", "localhost:5000/kgs-rocm-test:dev"] for a in world.calls("docker"))
    assert t["pod_result"]["mode"] == "fake"
    pod = [o for o in world.log() if o["tool"] == "kubectl" and "apply" in o["argv"] and o["stdin"]
           and "kind: Pod" in o["stdin"]]
    doc = yaml.safe_load(pod[0]["stdin"])
    assert doc["metadata"]["name"] == "gpu-rocm-test"
    assert doc["spec"]["containers"][0]["name"] == "gpu-sim"
    assert doc["spec"]["containers"][0]["resources"]["limits"] == {"amd.com/gpu": 1}
    assert world.state()["clusters"] == {}  # bench deletes unless --keep
    # the workload image was pre-pulled into the workers during create
    pulls = [e["argv"] for e in world.log() if e["tool"] == "docker" and e["argv"][:1] == ["exec"]
             and "crictl" in e["argv"]]
    assert pulls and all(a[-1] == "localhost:5000/kgs-rocm-test:dev" for a in pulls)
    assert any(p["phase"] == "prepull-wait" for p in t["phases"])


def test_bench_result_wait_follows_pod_timeout(world, tmp_path, monkeypatch, capsys):
    """the wait for the pod's result line is --pod-timeout
    x 10 (not a fixed 600 s), and a pod that never prints one fails the bench
    (exit 1) instead of reporting an empty result."""
    import time

    from kgs.e2e import result_timeout

    assert result_timeout(60) == 600 and result_timeout(1) == 10
    monkeypatch.setenv("KGS_FAKE_FAIL", "pod-no-result")
    t0 = time.monotonic()
    assert run("bench", "--dev-root", world.nogpu, "--pod-timeout", "1") == 1
    assert 9 <= time.monotonic() - t0 < 60
    assert "no result line" in capsys.readouterr().err
    assert world.state()["clusters"] == {}  # still cleaned up


def test_bench_uses_cached_workload_image_and_registry_port(world, tmp_path, capsys):
    """An image already present is not rebuilt; --registry-port flows into the
    pod's image reference."""
    rc = run("bench", "--dev-root", world.nogpu, "--registry-port=5123", "--timings-json", str(tmp_path / "a.json"))
    assert rc == 0
    t = json.loads((tmp_path / "a.json").read_text())
    assert t["phases"][0].get("built")
    rc = run("bench", "--dev-root", world.nogpu, "--registry-port=5123", "--timings-json", str(tmp_path / "b.json"))
    assert rc == 0
    t = json.loads((tmp_path / "b.json").read_text())
    assert t["phases"][0].get("cached") and not t["phases"][0].get("built")
    pods = [yaml.safe_load(o["stdin"]) for o in world.log() if o["tool"] == "kubectl" and o["stdin"]
            and "kind: Pod" in o["stdin"]]
    assert pods and all(p["spec"]["containers"][0]["image"] == "localhost:5123/kgs-rocm-test:dev" for p in pods)


def test_bench_no_kind_fake_chain(world, tmp_path, capsys):
    """`kgs bench --no-kind`: the real plugin process, kubelet Register,
    ListAndWatch capacity, Allocate and the pod entrypoint, chained and timed."""
    rc = run("bench", "--no-kind", "--fake-gpus", "2", "--gpus", "2", "--timings-json", str(tmp_path / "nk.json"))
    assert rc == 0
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith('{"metric"')][-1]
    s = json.loads(line)
    assert s["metric"].startswith("device-plugin start -> first in-pod GEMM") and s["value"] > 0
    assert list(s["phases"]) == ["plugin-process-start", "plugin-register", "capacity", "allocate", "pod-first-gemm"]
    t = json.loads((tmp_path / "nk.json").read_text())
    assert t["pod_result"]["mode"] == "fake" and t["allocate_envs"]["KGS_FAKE_GPUS"].count(",") == 1
    alloc = [p for p in t["phases"] if p["phase"] == "allocate"][0]
    assert len(alloc["device_ids"]) == 2


def test_gpuprobe_rejects_bad_sizes_before_touching_the_gpu():
    """The native first-GEMM probe validates its shape on the host (the GEMM
    grid assumes 256-multiples) and exits 2 without any HIP call."""
    import subprocess

    from kgs.workload.entrypoint import probe_binary

    exe = probe_binary()
    if exe is None:
        pytest.skip("kgs-gpuprobe not built")
    for bad in (["--size", "1000"], ["--size", "0"], ["--iters", "-1"], ["--bogus"]):
        r = subprocess.run([exe, *bad], capture_output=True, text=True, timeout=60)
        assert r.returncode == 2, (bad, r.stdout, r.stderr)
        assert "KGS_FIRST_GEMM" not in r.stdout


def test_entrypoint_probe_line_parsing(tmp_path, monkeypatch, capsys):
    """run_probe echoes the probe's KGS_FIRST_GEMM line and returns it parsed;
    a probe that prints no line, or reports a failed check, makes the pod fail."""
    from kgs.workload import entrypoint

    def fake(body: str) -> str:
        exe = tmp_path / f"probe{len(list(tmp_path.iterdir()))}"
        exe.write_text("#!/bin/sh\n" + body + "\n")
        exe.chmod(0o755)
        return str(exe)

    good = fake('echo \'KGS_FIRST_GEMM {"ok":true,"n_gpus":1,"t_first_gemm_s":0.25,"devices":[]}\'')
    monkeypatch.setattr(entrypoint, "probe_binary", lambda: good)
    res = entrypoint.run_probe(256, timeout=30)
    assert res["ok"] is True and res["rc"] == 0 and res["t_first_gemm_s"] == 0.25
    assert capsys.readouterr().out.startswith("KGS_FIRST_GEMM ")
    bad = fake('echo \'KGS_FIRST_GEMM {"ok":false,"devices":[]}\'; exit 1')
    monkeypatch.setattr(entrypoint, "probe_binary", lambda: bad)
    assert entrypoint.run_probe(256, timeout=30)["ok"] is False
    silent = fake("exit 3")
    monkeypatch.setattr(entrypoint, "probe_binary", lambda: silent)
    res = entrypoint.run_probe(256, timeout=30)
    assert res["ok"] is False and res["rc"] == 3
    monkeypatch.setattr(entrypoint, "probe_binary", lambda: None)
    assert "not built" in entrypoint.run_probe(256)["skipped"]


def test_entrypoint_forwards_readiness_before_the_probe_exits(tmp_path, monkeypatch):
    """the KGS_FIRST_GEMM line is forwarded when read, not when the
    probe (which goes on to its throughput loop) has exited."""
    import time

    from kgs.workload import entrypoint

    exe = tmp_path / "probe"
    exe.write_text("#!/bin/sh\necho 'KGS_FIRST_GEMM {\"ok\":true,\"devices\":[]}'\nsleep 2\n"
                   "echo 'KGS_PROBE_TPUT {\"iters\":5,\"devices\":[{\"device\":0,\"tflops\":1600.0}]}'\n")
    exe.chmod(0o755)
    monkeypatch.setattr(entrypoint, "probe_binary", lambda: str(exe))
    writes = []

    class Rec:
        def write(self, text):
            writes.append((time.monotonic(), text))

        def flush(self):
            pass

    monkeypatch.setattr(sys, "stdout", Rec())
    res = entrypoint.run_probe(256, timeout=30)
    t_end = time.monotonic()
    t_line = [t for t, x in writes if x.startswith("KGS_FIRST_GEMM")][0]
    assert t_end - t_line > 1.5
    assert res["ok"] and res["throughput"]["devices"][0]["tflops"] == 1600.0


def test_entrypoint_missing_probe_does_not_fail_the_pod(tmp_path, monkeypatch):
    from kgs.workload import entrypoint

    class G:
        render_minor, bdf, gfx_arch, cu_count, num_xcc, vram_bytes, numa_node = 128, "0000:05:00.0", "gfx950", \
            256, 8, 288 << 30, 0
        rocr_uuid = "GPU-a6ff75a300000000"

    monkeypatch.setattr(entrypoint, "allocated_gpus", lambda: [G()])
    monkeypatch.setattr(entrypoint, "probe_binary", lambda: None)
    out = tmp_path / "r.json"
    assert entrypoint.main(["--probe-only", "--json-out", str(out)]) == 0
    r = json.loads(out.read_text())
    assert "skipped" in r["first_gemm"] and r.get("all_ok", True)


def test_pod_verb_renders_static_pods_on_the_configured_registry(world, capsys):
    assert run("pod", "rocm-gpu-test", "--registry-port=5123") == 0
    doc = yaml.safe_load(capsys.readouterr().out)
    assert doc["metadata"]["name"] == "gpu-rocm-test"
    assert doc["spec"]["containers"][0]["image"] == "localhost:5123/kgs-rocm-test:dev"
    assert run("pod", "vllm-rocm-pod", "--registry-port=5123") == 0
    assert "docker.io/rocm/vllm" in capsys.readouterr().out  # public images untouched
    assert run("pod", "no-such-pod") == 1


def test_shell_wrapper_is_executable():
    p = os.path.join(os.path.dirname(os.path.dirname(__file__)), "kind-gpu-sim.sh")
    assert os.access(p, os.X_OK)


def test_base_mirror_rewrites_base_images(world):
    """C13 analog: the reference sed-patches FROM lines to a public mirror
    (kind-gpu-sim.sh:144-178); kgs passes the mirror as build arguments."""
    assert run("create", "--dev-root", world.nogpu, "--base-mirror=mirror.example:5001/library") == 0
    build = world.calls("docker", "build")[0]
    assert "PY_IMAGE=mirror.example:5001/library/python:3.12.8-slim-bookworm" in build
    assert "BUILD_IMAGE=mirror.example:5001/library/python:3.12.8-bookworm" in build
    reg = world.state()["containers"][C.REGISTRY_NAME]
    assert reg["image"] == "mirror.example:5001/library/registry:2"


def test_rocm_images_are_mirrorable_and_overridable(world, tmp_path):
    """the plugin image's ROCm stage (a multi-GB
    Docker Hub pull made for one header directory and three .so files) takes
    --rocm-mirror (the C13 rewrite, kind-gpu-sim.sh:144-178) and --rocm-dev-image,
    and both reach the `docker build` argv."""
    assert run("create", "--dev-root", world.nogpu, "--rocm-mirror=mirror.example:5001/rocm") == 0
    build = world.calls("docker", "build")[0]
    assert "ROCM_IMAGE=mirror.example:5001/rocm/dev-ubuntu-22.04:7.0" in build
    assert not any("docker.io/rocm" in x for x in build), build
    assert run("delete") == 0
    n = len(world.calls("docker", "build"))
    assert run("create", "--dev-root", world.nogpu, "--rocm-dev-image=registry.local/amdsmi-lib:7.0.0",
               "--rocm-mirror=mirror.example:5001/rocm") == 0
    build = world.calls("docker", "build")[n]
    assert "ROCM_IMAGE=registry.local/amdsmi-lib:7.0.0" in build  # not a docker.io/rocm ref: left alone
    # the workload image's PyTorch-ROCm base takes the same mirror
    from kgs import config as Cfg

    s = Cfg.Settings(rocm_mirror="mirror.example:5001/rocm")
    assert s.rocm_image(Cfg.ROCM_BASE_IMAGE) == "mirror.example:5001/rocm/" + Cfg.ROCM_BASE_IMAGE.split("/", 2)[2]
    assert Cfg.Settings().rocm_image(Cfg.ROCM_BASE_IMAGE) == Cfg.ROCM_BASE_IMAGE


def test_default_base_images_use_public_mirror(world):
    assert run("create", "--dev-root", world.nogpu) == 0
    build = world.calls("docker", "build")[0]
    assert f"PY_IMAGE={C.BASE_MIRROR}/python:3.12.8-slim-bookworm" in build


def test_doctor_cpu_only_host(world, capsys):
    """No /dev/kfd: runtime/kind/kubectl OK (fakes on PATH), devices WARN, exit 0."""
    assert run("doctor", "--dev-root", world.nogpu, "--json", "--registry-port", "0") == 0
    rep = json.loads(capsys.readouterr().out)
    st = {c["name"]: c["status"] for c in rep["checks"]}
    assert st["container runtime"] == "OK" and st["kind"] == "OK" and st["kubectl"] == "OK"
    assert st["/dev/kfd"] == "WARN" and rep["ok"] is True


def test_doctor_fake_mi355x_box(world, tmp_path, capsys):
    root = str(make_fake_mi355x(str(tmp_path / "host8")))
    assert run("doctor", "--dev-root", root, "--json", "--registry-port", "0") == 0
    rep = json.loads(capsys.readouterr().out)
    st = {c["name"]: (c["status"], c["detail"]) for c in rep["checks"]}
    assert st["GPUs"][0] == "OK" and "8 x gfx950" in st["GPUs"][1]
    assert st["xGMI mesh"] == ("OK", "all 28 pairs directly linked")
    assert st["health"][0] == "OK"


def test_doctor_native_build_check(monkeypatch):
    """The native-build check reports missing and stale targets as WARN."""
    from pathlib import Path

    from kgs import doctor
    from kgs.utils import build

    class T:
        def __init__(self, name, exists, stale, optional=False):
            self.name, self.optional = name, optional
            self.output = Path("/") if exists else Path("/nonexistent/kgs-x")
            self._stale = stale

        def stale(self):
            return self._stale

    monkeypatch.setattr(build, "targets", lambda: [T("kernels", True, False), T("gpuprobe", True, False)])
    c = doctor.check_native_build()
    assert c.status == "OK" and "2 targets fresh" in c.detail
    monkeypatch.setattr(build, "targets", lambda: [T("kernels", True, True), T("gpuprobe", False, True)])
    c = doctor.check_native_build()
    assert c.status == "WARN" and "not built: gpuprobe" in c.detail
    monkeypatch.setattr(build, "targets", lambda: [T("kernels", True, True), T("rccl-bench", False, True, True)])
    c = doctor.check_native_build()
    assert c.status == "WARN" and "older than sources: kernels, rccl-bench" in c.detail


def test_doctor_missing_tools_fails(world, monkeypatch, capsys):
    monkeypatch.setenv("PATH", "/nonexistent")
    assert run("doctor", "--dev-root", world.nogpu, "--registry-port", "0") == 1
    out = capsys.readouterr().out
    assert "FAIL" in out and "kind not on PATH" in out


def test_plugin_image_builds_concurrently_with_kind_create(world, tmp_path):
    tj = tmp_path / "t.json"
    assert run("create", "--dev-root", world.nogpu, "--timings-json", str(tj)) == 0
    phases = {p["phase"]: p for p in json.loads(tj.read_text())["phases"]}
    assert "overlapped_build_s" in phases["plugin-image"]
    # the pushed image is in the registry before the DaemonSet is applied
    log = world.log()
    push = next(i for i, e in enumerate(log) if e["tool"] == "docker" and e["argv"][:1] == ["push"])
    apply_ds = next(i for i, e in enumerate(log) if e["tool"] == "kubectl" and "apply" in e["argv"]
                    and e["stdin"] and "DaemonSet" in e["stdin"])
    assert push < apply_ds


def test_serial_flag_keeps_reference_order(world):
    assert run("create", "--dev-root", world.nogpu, "--serial") == 0
    log = world.log()
    kind_create = next(i for i, e in enumerate(log) if e["tool"] == "kind" and e["argv"][:2] == ["create", "cluster"])
    build = next(i for i, e in enumerate(log) if e["tool"] == "docker" and e["argv"][:1] == ["build"])
    assert kind_create < build


# ---- advertised-GPU count --------------------------------
@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_create_advertises_exactly_n_gpus(world, tmp_path, capsys, n):
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("create", "--gpus", str(n), "--dev-root", str(host)) == 0
    assert f"({n} amd.com/gpu advertised)" in capsys.readouterr().out
    cfg = yaml.safe_load((world.cwd / "kind-config.yaml").read_text())
    renders = [m["containerPath"] for node in cfg["nodes"] for m in node.get("extraMounts", [])
               if m["containerPath"].startswith("/dev/dri/renderD")]
    assert len(renders) == n
    part = json.loads((world.cwd / ".kgs" / "kind-gpu-sim" / "gpus.json").read_text())["nodes"]
    chosen = part["kind-gpu-sim-worker"]
    assert len(chosen) == n and part["kind-gpu-sim-worker2"] == []
    # one NUMA node (4 GPUs per socket on the fake host), lowest indices: 128, 136, ...
    assert chosen == [128 + 8 * i for i in range(n)]
    st = world.state()["clusters"]["kind-gpu-sim"]
    assert st["nodes"]["kind-gpu-sim-worker"]["allocatable"] == {"amd.com/gpu": str(n)}
    assert st["nodes"]["kind-gpu-sim-worker"]["labels"]["kgs.amd.com/gpu-partition"] == str(n)


def test_create_gpus_split_over_workers(world, tmp_path):
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("create", "--gpus", "4", "--gpu-partition", "split", "--dev-root", str(host)) == 0
    part = json.loads((world.cwd / ".kgs" / "kind-gpu-sim" / "gpus.json").read_text())["nodes"]
    assert sum(len(v) for v in part.values()) == 4 and all(len(v) == 2 for v in part.values())


def test_create_gpus_changed_is_drift(world, tmp_path, capsys):
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("create", "--gpus", "2", "--dev-root", str(host)) == 0
    assert run("create", "--gpus", "2", "--dev-root", str(host)) == 0  # same shape: reconcile
    capsys.readouterr()
    assert run("create", "--gpus", "4", "--dev-root", str(host)) == 1
    err = capsys.readouterr().err
    assert "different shape" in err and "GPU partition" in err


def test_create_gpus_errors(world, tmp_path, capsys):
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("create", "--gpus", "9", "--dev-root", str(host)) == 1
    assert "only 8 healthy GPU(s)" in capsys.readouterr().err
    assert run("create", "--gpus", "1", "--dev-root", world.nogpu) == 1
    assert "needs real GPUs" in capsys.readouterr().err
    assert world.state().get("clusters", {}) == {}  # refused before anything was created


def test_select_gpus_prefers_one_xgmi_island():
    from kgs import gpuinfo
    from kgs.cluster import select_gpus

    import tempfile

    d = tempfile.mkdtemp(prefix="kgs-sel", dir="/tmp")
    gpus = gpuinfo.discover(str(make_fake_mi355x(os.path.join(d, "h"))), use_amdsmi=False).gpus
    # drop every xGMI link of GPU 0: it must not be picked into a 2-GPU set
    for g in gpus:
        g.links = [lk for lk in g.links if lk.to_node != gpus[0].node_id] if g is not gpus[0] else \
            [lk for lk in g.links if not lk.is_xgmi]
    pick = select_gpus(gpus, 2)
    assert gpus[0] not in pick and len(pick) == 2
    assert select_gpus(gpus, None) == gpus


def test_bench_sweep_dry_run_plan(world, tmp_path, capsys):
    """`kgs bench --sweep 1,2,4,8 --dry-run`: one create (N renderD mounts) ->
    pod (N GPUs) -> delete per count, nothing executed."""
    host = make_fake_mi355x(tmp_path / "host8")
    rc = run("bench", "--sweep", "1,2,4,8", "--dry-run", "--dev-root", str(host),
             "--sweep-json", str(tmp_path / "sweep.json"))
    cap = capsys.readouterr()
    assert rc == 0, cap.err
    assert world.log() == []
    doc = json.loads((tmp_path / "sweep.json").read_text())
    assert [p["advertised"] for p in doc["points"]] == [1, 2, 4, 8]
    assert [p["pod_gpus"] for p in doc["points"]] == [1, 2, 4, 8]
    assert all(p["ok"] for p in doc["points"]) and [t["advertised"] for t in doc["table"]] == [1, 2, 4, 8]
    # the printed kind configs carry 1, 2, 4, 8 render nodes in order
    cfgs = [c for c in cap.out.split("# ") if "kind: Cluster" in c]
    counts = [c.count("containerPath: /dev/dri/renderD") for c in cfgs]
    assert counts == [1, 2, 4, 8]
    assert cap.err.count("kind create cluster --name kind-gpu-sim") == 4
    pods = [c for c in cap.err.split("\n") if "kubectl" in c and "apply" in c]
    assert len(pods) >= 4


def test_bench_sweep_runs_each_count(world, tmp_path, capsys):
    host = make_fake_mi355x(tmp_path / "host8")
    rc = run("bench", "--sweep", "1,8", "--pod-gpus", "1", "--dev-root", str(host),
             "--sweep-json", str(tmp_path / "s.json"))
    assert rc == 0
    doc = json.loads((tmp_path / "s.json").read_text())
    assert [(p["advertised"], p["pod_gpus"], p["ok"]) for p in doc["points"]] == [(1, 1, True), (8, 1, True)]
    assert all(p["value"] > 0 for p in doc["points"])
    # each point created and deleted its own cluster
    assert len(world.calls("kind", "create", "cluster")) == 2 and world.state()["clusters"] == {}
    pods = [yaml.safe_load(o["stdin"]) for o in world.log() if o["tool"] == "kubectl" and o["stdin"]
            and "kind: Pod" in o["stdin"]]
    assert [p["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] for p in pods] == [1, 1]


def test_bench_sweep_records_a_failing_point(world, tmp_path, monkeypatch):
    host = make_fake_mi355x(tmp_path / "host8")
    rc = run("bench", "--sweep", "2,16", "--dev-root", str(host), "--sweep-json", str(tmp_path / "s.json"))
    assert rc == 1
    pts = json.loads((tmp_path / "s.json").read_text())["points"]
    assert pts[0]["ok"] and not pts[1]["ok"] and "only 8 healthy" in pts[1]["error"]


# ---- create-path correctness ------------------------------
def test_registry_network_failure_is_an_error(world, monkeypatch, capsys):
    monkeypatch.setenv("KGS_FAKE_FAIL", "network-connect")
    assert run("create", "--dev-root", world.nogpu) == 1
    err = capsys.readouterr().err
    assert "could not attach kind-registry to network kind" in err and "permission denied" in err
    assert world.state()["clusters"] == {}  # rolled back


def test_ten_workers_partition_labels_match_the_file(world, tmp_path):
    """kubectl lists worker, worker10, worker2 ...; labels must follow node
    names, not list position."""
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("create", "--workers", "10", "--gpu-partition", "split", "--dev-root", str(host)) == 0
    part = json.loads((world.cwd / ".kgs" / "kind-gpu-sim" / "gpus.json").read_text())["nodes"]
    nodes = world.state()["clusters"]["kind-gpu-sim"]["nodes"]
    assert len(part) == 10
    for name, minors in part.items():
        assert nodes[name]["labels"]["kgs.amd.com/gpu-partition"] == str(len(minors)), name
        assert nodes[name]["allocatable"].get("amd.com/gpu", "0") in (str(len(minors)), "0")
    assert part["kind-gpu-sim-worker10"] == [] and len(part["kind-gpu-sim-worker2"]) == 1


def test_natural_worker_order():
    from kgs.cluster import _natural_key

    names = ["c-worker", "c-worker10", "c-worker2", "c-worker3"]
    assert sorted(names, key=_natural_key) == ["c-worker", "c-worker2", "c-worker3", "c-worker10"]


def test_bench_no_kind_advertises_the_same_selection(world, tmp_path, capsys):
    """`kgs bench --no-kind --gpus 4 --pod-gpus 1` on the fake 8-GPU host: the
    plugin process advertises exactly the 4 GPUs `create --gpus 4` would, and
    the pod is allocated one of them (BASELINE config 3 shape)."""
    host = make_fake_mi355x(tmp_path / "host8")
    rc = run("bench", "--no-kind", "--gpus", "4", "--pod-gpus", "1", "--dev-root", str(host),
             "--timings-json", str(tmp_path / "nk.json"))
    assert rc == 0
    s = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith('{"metric"')][-1])
    assert s["advertised"] == 4 and s["gpus"] == 1
    t = json.loads((tmp_path / "nk.json").read_text())
    assert t["advertised_minors"] == [128, 136, 144, 152]
    cap = [p for p in t["phases"] if p["phase"] == "capacity"][0]
    assert cap["advertised"] == 4
    alloc = [p for p in t["phases"] if p["phase"] == "allocate"][0]
    assert len(alloc["device_ids"]) == 1
    assert t["allocate_envs"]["KGS_RENDER_MINORS"] in {"128", "136", "144", "152"}


def test_bench_sweep_keeps_the_registry_between_points(world, tmp_path):
    """The nodes pull the workload image from the local registry: the sweep
    must not remove the registry between points (a fresh, empty one would leave
    every later pod in ImagePullBackOff), and a locally cached image is pushed
    again. After the last point the registry is gone, as after `kgs delete`."""
    host = make_fake_mi355x(tmp_path / "host8")
    assert run("bench", "--sweep", "1,2,4", "--dev-root", str(host)) == 0
    runs = world.calls("docker", "run")
    assert len([a for a in runs if "kind-registry" in a]) == 1  # started once, reused by points 2 and 3
    assert world.calls("docker", "rm") == [["rm", "kind-registry"]]  # removed once, at the end
    pushes = [a for a in world.calls("docker", "push") if a[1].endswith("kgs-rocm-test:dev")]
    assert len(pushes) == 3  # built + pushed once, re-pushed (cached) by the next two points
    assert "kind-registry" not in world.state()["containers"]


def test_images_amdsmi_lib_builds_the_light_source(world, capsys):
    assert run("images", "--amdsmi-lib", "--dev-root", world.nogpu) == 0
    builds = world.calls("docker", "build")
    assert len(builds) == 1 and any("Dockerfile.amdsmi-lib" in x for x in builds[0])
    assert "UBUNTU_IMAGE=public.ecr.aws/docker/library/ubuntu:22.04" in builds[0]
    assert "--rocm-dev-image=localhost:5000/kgs-amdsmi-lib:7.0" in capsys.readouterr().out
