#!/usr/bin/env python3
"""Stateful stand-in for kind / kubectl / docker / podman / systemctl (T1 tests).

Installed as symlinks named after each tool on a temporary PATH. Every call is
appended to $KGS_FAKE_LOG as JSON ({"tool", "argv", "stdin"}); the simulated
world (containers, networks, clusters, nodes, pods, images) lives in
$KGS_FAKE_STATE. Behaviour follows the real tools closely enough for the
orchestrator's control flow: error strings for "already connected", exit codes
for missing containers, kind node naming, kubelet-managed capacity once the
device-plugin DaemonSet is applied (from the bind-mounted partition file), etc.
Fault injection: $KGS_FAKE_FAIL = comma list of {plugin-ready, kind-create,
push, pod-running, pod-no-result, network-connect}. Node lists come back sorted by name, as
the real kubectl prints them (worker, worker10, worker2, ...).
"""
import fcntl
import json
import os
import sys

import yaml

TOOL = os.path.basename(sys.argv[0])
ARGS = sys.argv[1:]
STATE = os.environ.get("KGS_FAKE_STATE", "/tmp/kgs-fake-state.json")
LOG = os.environ.get("KGS_FAKE_LOG", "/tmp/kgs-fake-log.jsonl")
FAIL = set(filter(None, os.environ.get("KGS_FAKE_FAIL", "").split(",")))


def load():
    if os.path.exists(STATE):
        with open(STATE) as f:
            return json.load(f)
    return {"containers": {}, "networks": {}, "clusters": {}, "images": [], "registry_images": []}


def save(st):
    with open(STATE, "w") as f:
        json.dump(st, f, indent=1)


def out(s=""):
    sys.stdout.write(s)


def err(msg, rc=1):
    sys.stderr.write(msg + "\n")
    sys.exit(rc)


# The orchestrator runs some tools concurrently (the plugin image builds while
# kind creates the cluster); serialise whole invocations on a lock next to the
# state file, so the read-modify-write of the simulated world stays atomic.
_lock = open(STATE + ".lock", "a")
fcntl.flock(_lock, fcntl.LOCK_EX)

stdin = None
if not sys.stdin.isatty():
    try:
        stdin = sys.stdin.read()
    except Exception:
        stdin = None
with open(LOG, "a") as f:
    f.write(json.dumps({"tool": TOOL, "argv": ARGS, "stdin": stdin,
                        "env": {k: os.environ.get(k) for k in ("KIND_EXPERIMENTAL_PROVIDER", "DOCKER_HOST",
                                                               "BUILDAH_FORMAT")}}) + "\n")

st = load()


# ------------------------------------------------------------------ docker ---
def container_tool():
    cs = st["containers"]
    if not ARGS:
        err("usage")
    cmd = ARGS[0]
    if cmd == "inspect":
        name = ARGS[-1]
        if name not in cs:
            err(f"Error: No such object: {name}")
        out(("true" if cs[name]["running"] else "false") + "\n")
    elif cmd == "ps":
        running_only = "-a" not in " ".join(ARGS) and "-aq" not in ARGS
        name = None
        for a in ARGS:
            if a.startswith("name="):
                name = a[len("name="):].strip("^$").lstrip("/").lstrip("?").lstrip("/")
        for n, c in cs.items():
            if name and n != name:
                continue
            if running_only and not c["running"]:
                continue
            out(c["id"] + "\n")
    elif cmd == "run":
        name = ARGS[ARGS.index("--name") + 1]
        if name in cs:
            err(f'docker: Error response from daemon: Conflict. The container name "/{name}" is already in use.',
                125)
        cs[name] = {"id": f"{abs(hash(name)) % 10**12:012x}", "running": True, "image": ARGS[-1],
                    "networks": ["bridge"], "args": ARGS}
        out(cs[name]["id"] + "\n")
    elif cmd == "start":
        cs[ARGS[1]]["running"] = True
    elif cmd == "stop":
        if ARGS[1] not in cs:
            err(f"Error: No such container: {ARGS[1]}")
        cs[ARGS[1]]["running"] = False
    elif cmd == "rm":
        if ARGS[1] not in cs:
            err(f"Error: No such container: {ARGS[1]}")
        del cs[ARGS[1]]
    elif cmd == "network" and ARGS[1] == "connect":
        net, name = ARGS[2], ARGS[3]
        if "network-connect" in FAIL:
            err(f"Error response from daemon: failed to add interface to network {net}: permission denied")
        if net not in st["networks"]:
            err(f"Error response from daemon: network {net} not found")
        if net in cs[name]["networks"]:
            err(f"Error response from daemon: endpoint with name {name} already exists in network {net}")
        cs[name]["networks"].append(net)
    elif cmd == "build":
        tag = ARGS[ARGS.index("-t") + 1]
        if tag not in st["images"]:
            st["images"].append(tag)
        out(f"Successfully tagged {tag}\n")
    elif cmd == "push":
        if "push" in FAIL:
            err("push failed")
        if ARGS[1] not in st["images"]:
            err(f"An image does not exist locally with the tag: {ARGS[1]}")
        st["registry_images"].append(ARGS[1])
    elif cmd == "tag":
        st["images"].append(ARGS[2])
    elif cmd == "save":
        path = ARGS[ARGS.index("-o") + 1]
        with open(path, "w") as f:
            f.write("archive of " + ARGS[1])
    elif cmd == "image" and ARGS[1] == "inspect":
        if ARGS[2] not in st["images"]:
            err("no such image")
        out("[]\n")
    else:
        err(f"fake {TOOL}: unsupported {ARGS}")


# -------------------------------------------------------------------- kind ---
def kind_tool():
    cl = st["clusters"]
    if ARGS[:2] == ["get", "clusters"]:
        for n in cl:
            out(n + "\n")
        if not cl:
            sys.stderr.write("No kind clusters found.\n")
    elif ARGS[:2] == ["create", "cluster"]:
        if "kind-create" in FAIL:
            err("ERROR: failed to create cluster: boom")
        name = ARGS[ARGS.index("--name") + 1]
        cfgp = ARGS[ARGS.index("--config") + 1]
        if name in cl:
            err(f'ERROR: failed to create cluster: node(s) already exist for a cluster with the name "{name}"')
        cfg = yaml.safe_load(open(cfgp))
        nodes = {}
        w = 0
        for n in cfg["nodes"]:
            if n["role"] == "control-plane":
                nn = f"{name}-control-plane"
            else:
                w += 1
                nn = f"{name}-worker" + ("" if w == 1 else str(w))
            nodes[nn] = {"role": n["role"], "labels": {}, "taints": [], "capacity": {}, "allocatable": {},
                         "mounts": n.get("extraMounts", [])}
        cl[name] = {"nodes": nodes, "config": cfg, "objects": [], "pods": {}, "loaded": []}
        st["networks"].setdefault("kind", [])
        out(f"Creating cluster \"{name}\" ...\n")
    elif ARGS[:2] == ["delete", "cluster"]:
        name = ARGS[ARGS.index("--name") + 1]
        cl.pop(name, None)
        if not cl:
            st["networks"].pop("kind", None)
    elif ARGS[:2] == ["get", "nodes"]:
        name = ARGS[ARGS.index("--name") + 1]
        for n in cl.get(name, {}).get("nodes", {}):
            out(n + "\n")
    elif ARGS[:2] == ["load", "docker-image"] or ARGS[:2] == ["load", "image-archive"]:
        name = ARGS[ARGS.index("--name") + 1]
        if name not in cl:
            err(f"ERROR: unknown cluster \"{name}\"")
        cl[name]["loaded"].append(ARGS[2])
    else:
        err(f"fake kind: unsupported {ARGS}")


# ----------------------------------------------------------------- kubectl ---
def _cluster():
    ctx = None
    if "--context" in ARGS:
        ctx = ARGS[ARGS.index("--context") + 1]
    name = ctx[len("kind-"):] if ctx else next(iter(st["clusters"]), None)
    if name not in st["clusters"]:
        err(f"error: context \"{ctx}\" does not exist")
    return st["clusters"][name]


def _partition(c):
    for n, node in c["nodes"].items():
        for m in node["mounts"]:
            if m["containerPath"] == "/etc/kgs/gpus.json" and os.path.exists(m["hostPath"]):
                return json.load(open(m["hostPath"]))["nodes"]
    return {}


def _apply_plugin(c, ds):
    env = {e["name"]: e.get("value") for e in ds["spec"]["template"]["spec"]["containers"][0].get("env", [])}
    fake = int(env.get("KGS_FAKE_GPUS") or 0)
    part = _partition(c)
    for n, node in c["nodes"].items():
        if node["labels"].get("hardware-type") != "gpu":
            continue
        if fake:
            node["capacity"]["amd.com/gpu"] = str(fake)
        elif part.get(n):
            node["capacity"]["amd.com/gpu"] = str(len(part[n]))
        node["allocatable"] = dict(node["capacity"])
    c["plugin_pods"] = [f"pod/amdgpu-device-plugin-daemonset-{i}" for i, (n, node) in
                        enumerate(c["nodes"].items()) if node["labels"].get("hardware-type") == "gpu"]


def kubectl_tool():
    a = [x for i, x in enumerate(ARGS) if not (x == "--context" or (i > 0 and ARGS[i - 1] == "--context"))]
    c = _cluster()
    verb = a[0]
    if verb == "get" and a[1] == "nodes":
        if "json" in a:
            items = [{"metadata": {"name": n, "labels": v["labels"]},
                      "spec": {"taints": v["taints"]},
                      "status": {"capacity": v["capacity"], "allocatable": v["allocatable"]}}
                     for n, v in sorted(c["nodes"].items())]
            out(json.dumps({"items": items}))
        else:
            out("\n".join(sorted(c["nodes"])) + "\n")
    elif verb == "label":
        names = [x for x in a[2:] if "=" not in x and not x.startswith("-")]
        kvs = [x for x in a[2:] if "=" in x and not x.startswith("-")]
        for n in names:
            for kv in kvs:
                k, v = kv.split("=", 1)
                c["nodes"][n]["labels"][k] = v
    elif verb == "taint":
        names = [x for x in a[2:] if ":" not in x and not x.startswith("-")]
        t = [x for x in a[2:] if ":" in x][0]
        for n in names:
            if t not in c["nodes"][n]["taints"]:
                c["nodes"][n]["taints"].append(t)
    elif verb == "patch":
        n = a[2]
        p = [x for x in a if x.startswith("-p=")][0][3:]
        for op in json.loads(p):
            key = op["path"].split("/")[-1].replace("~1", "/")
            c["nodes"][n]["capacity"][key] = op["value"]
            c["nodes"][n]["allocatable"][key] = op["value"]
    elif verb in ("apply", "create"):
        text = stdin or ""
        if "-f" in a and a[a.index("-f") + 1] != "-":
            with open(a[a.index("-f") + 1]) as f:
                text = f.read()
        for doc in yaml.safe_load_all(text):
            if not doc:
                continue
            c["objects"].append(doc)
            if doc["kind"] == "DaemonSet":
                _apply_plugin(c, doc)
            if doc["kind"] == "Pod":
                c["pods"][doc["metadata"]["name"]] = {"phase": "Running", "spec": doc["spec"]}
    elif verb == "get" and a[1] == "pods":
        for p in c.get("plugin_pods", []):
            out(p + "\n")
    elif verb == "wait":
        if any("amdgpu-device-plugin" in x for x in a) and "plugin-ready" in FAIL:
            err("error: timed out waiting for the condition on pods/amdgpu-device-plugin-daemonset-0")
        if any(x.startswith("pod/") for x in a) and "pod-running" in FAIL:
            err("error: timed out waiting for the condition on pods/gpu-rocm-test")
        out("condition met\n")
    elif verb == "logs":
        if any("gpu-rocm-test" in x for x in a):
            out("Hello from fake ROCm GPU node\n")
            if "pod-no-result" not in FAIL:
                out(json.dumps({"mode": "fake", "n_gpus": 0}) + "\n")
        else:
            out("plugin log line\n")
    elif verb == "delete":
        c["pods"].pop(a[-1].split("/")[-1], None)
    else:
        err(f"fake kubectl: unsupported {ARGS}")


if TOOL in ("docker", "podman"):
    container_tool()
elif TOOL == "kind":
    kind_tool()
elif TOOL == "kubectl":
    kubectl_tool()
elif TOOL == "systemctl":
    pass
else:
    err(f"unknown fake tool {TOOL}")
save(st)
