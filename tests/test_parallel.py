"""Distributed paths on CPU: gloo, world_size 2 (the RCCL code paths are the
same torch.distributed calls; the GPU box only has one GPU)."""
import json
import os
import sys
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _T:
    """A tensor sent by value: torch's queue pickling shares tensor storage by
    file descriptor, which the parent cannot open once the worker has exited."""

    def __init__(self, t):
        self.dtype = t.dtype
        self.a = t.detach().cpu().float().numpy().copy() if t.is_floating_point() else t.detach().cpu().numpy().copy()


def _pack(v):
    if isinstance(v, torch.Tensor):
        return _T(v)
    if isinstance(v, (list, tuple)):
        return type(v)(_pack(x) for x in v)
    if isinstance(v, dict):
        return {k: _pack(x) for k, x in v.items()}
    return v


def _unpack(v):
    if isinstance(v, _T):
        return torch.from_numpy(v.a).to(v.dtype)
    if isinstance(v, (list, tuple)):
        return type(v)(_unpack(x) for x in v)
    if isinstance(v, dict):
        return {k: _unpack(x) for k, x in v.items()}
    return v


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        q.put((rank, _pack(fn(rank, world))))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(fn, world=2, attempts=3):
    """Run fn(rank, world) on `world` gloo ranks. The rendezvous port is picked
    free but can be taken by a concurrent test (pytest -n) before rank 0 binds
    it: such a run is retried on a new port; any other worker error is raised."""
    ctx = mp.get_context("spawn")
    for attempt in range(attempts):
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
        for p in ps:
            p.start()
        res = {r: _unpack(v) for r, v in (q.get(timeout=120) for _ in ps)}
        for p in ps:
            p.join(timeout=60)
        errs = [v for v in res.values() if isinstance(v, str)]
        if not errs:
            return res
        if attempt + 1 < attempts and any("address already in use" in e.lower() or "eaddrinuse" in e.lower()
                                          for e in errs):
            continue
        raise AssertionError(f"worker failed: {errs}")
    return res


def _init_and_reduce(rank, world):
    from kgs.parallel import dist as kdist

    ctx = kdist.init_from_env(expected_world=world, device_type="cpu")
    assert ctx.backend == "gloo" and ctx.world_size == world and ctx.rank == rank
    m = kdist.max_over_ranks(ctx, float(rank * 10))
    g = kdist.all_gather_object(ctx, {"r": rank})
    kdist.barrier(ctx)
    return (m, [x["r"] for x in g])


def test_init_from_env_gloo():
    res = _spawn(_init_and_reduce)
    assert res[0] == (10.0, [0, 1]) and res[1] == (10.0, [0, 1])


def _sweep(rank, world):
    from kgs.parallel import dist as kdist
    from kgs.parallel.allreduce import allreduce_sweep

    kdist.init_from_env(device_type="cpu")
    pts = allreduce_sweep([1024, 1 << 16], iters=3, warmup=1, device=torch.device("cpu"))
    return [(p.bytes, p.correct, p.busbw_gbs > 0, round(p.busbw_gbs / p.algbw_gbs, 3)) for p in pts]


def test_allreduce_sweep_gloo():
    res = _spawn(_sweep)
    assert res[0] == res[1] or all(a[:3] == b[:3] for a, b in zip(res[0], res[1]))
    for nbytes, ok, pos, ratio in res[0]:
        assert ok and pos and ratio == 1.0  # 2(n-1)/n = 1 at n=2


def _bucketer(rank, world):
    from kgs.parallel import dist as kdist
    from kgs.parallel.allreduce import GradBucketer

    kdist.init_from_env(device_type="cpu")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    b = GradBucketer(model.parameters(), bucket_mb=0.001)  # tiny buckets -> several buckets
    nb = len(b.buckets)
    x = torch.randn(8, 16) * (rank + 1)
    model(x).pow(2).sum().backward()
    b.wait()
    grads = [p.grad.clone() for p in model.parameters()]
    # reference: average of both ranks' local grads, computed here via all_gather
    b.remove()
    for p in model.parameters():
        p.grad = None
    model(x).pow(2).sum().backward()
    local = [p.grad.clone() for p in model.parameters()]
    ref = []
    for t in local:
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        ref.append(sum(parts) / world)
    return nb, all(torch.allclose(g, r, atol=1e-5) for g, r in zip(grads, ref))


def test_grad_bucketer_matches_average():
    res = _spawn(_bucketer)
    for nb, ok in res.values():
        assert nb >= 2 and ok


def test_single_process_context():
    from kgs.parallel import dist as kdist

    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    ctx = kdist.init_from_env(device_type="cpu")
    assert not ctx.distributed and ctx.group is None
    assert kdist.max_over_ranks(ctx, 3.5) == 3.5
    with pytest.raises(SystemExit):
        kdist.init_from_env(expected_world=2, device_type="cpu")


def _bench_rank(rank, world):
    import contextlib
    import io
    import json
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.main(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--gemm-m", "64", "--gemm-n", "64", "--gemm-k", "64",
                         "--allreduce-mb", "0.25", "--backend", "torch", "--cpu"])
    out = buf.getvalue().strip()
    return rc, (json.loads(out) if out else None)


def test_bench_distributed_plumbing_gloo():
    """bench.py's multi-rank path (barriers, max-over-ranks, bucket all-reduce,
    rank-0-only JSON) on 2 CPU ranks; the GPU run uses the same code on RCCL."""
    res = _spawn(_bench_rank)
    rc0, j0 = res[0]
    rc1, j1 = res[1]
    assert rc0 == 0 and rc1 == 0
    assert j1 is None  # only rank 0 prints
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in j0
    assert j0["n_gpus"] == 2 and j0["steps"] == 2 and j0["scaling"] == "weak"
    assert j0["config"]["parallelism"] == "dp2" and j0["config"]["global_batch"] == 8
    assert j0["ms_per_step"] > 0 and j0["backend"] == "torch"
    assert abs(j0["value"] - 2 * j0["per_gpu_tflops"]) <= 0.011  # aggregate = world x per-GPU (rounded)


MLP_DIMS = [64, 96, 48, 32]


def _mlp_dp(rank, world):
    from kgs.models.mlp import train_dp
    from kgs.parallel import dist as kdist

    ctx = kdist.init_from_env(device_type="cpu")
    r = train_dp(MLP_DIMS, steps=4, global_batch=64, lr=0.1, backend="torch", device="cpu", group=ctx.group,
                 bucket_mb=0.01, dtype=torch.float32)  # tiny buckets: several all-reduces per step
    return [p.detach().clone() for p in r["model"].parameters()], r["losses"]


def test_mlp_dp_matches_single_process_full_batch():
    """DP over 2 gloo ranks (bucketed, backward-overlapped all-reduce) must train
    the same weights as one process on the whole batch."""
    from kgs.models.mlp import train_dp

    res = _spawn(_mlp_dp)
    ref = train_dp(MLP_DIMS, steps=4, global_batch=64, lr=0.1, backend="torch", device="cpu",
                   dtype=torch.float32)
    ref_params = [p.detach() for p in ref["model"].parameters()]
    for rank in (0, 1):
        params, losses = res[rank]
        for p, q in zip(params, ref_params):
            torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-5)
        assert abs(losses[-1] - ref["losses"][-1]) < 1e-5
    assert ref["losses"][-1] < ref["losses"][0]


def _tp_weights(din=64, dff=128, dout=48, dtype=torch.float32, device="cpu"):
    g = torch.Generator().manual_seed(7)
    w1 = (torch.randn(dff, din, generator=g) * din ** -0.5).to(dtype).to(device)
    b1 = (torch.randn(dff, generator=g) * 0.1).to(dtype).to(device)
    w2 = (torch.randn(dout, dff, generator=g) * dff ** -0.5).to(dtype).to(device)
    b2 = (torch.randn(dout, generator=g) * 0.1).to(dtype).to(device)
    x = torch.randn(32, din, generator=g).to(dtype).to(device)
    return x, w1, b1, w2, b2


def _tp_rank(rank, world):
    from kgs.parallel import dist as kdist
    from kgs.parallel.tensor_parallel import TPMLP, make_reducer

    ctx = kdist.init_from_env(device_type="cpu")
    x, w1, b1, w2, b2 = _tp_weights()
    mlp = TPMLP(w1, b1, w2, b2, world, rank, make_reducer(ctx.group), backend="torch")
    return mlp(x)


def test_tensor_parallel_mlp_gloo():
    """Column(gelu) -> row split over 2 ranks + one all-reduce == the full MLP."""
    from kgs.parallel.tensor_parallel import reference_mlp

    res = _spawn(_tp_rank)
    x, w1, b1, w2, b2 = _tp_weights()
    ref = reference_mlp(x, w1, b1, w2, b2)
    for r in (0, 1):
        torch.testing.assert_close(res[r], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_self_launches_n_ranks_cpu(world):
    """`python bench.py --gpus N` without torchrun: the parent spawns N ranks
    (torchrun env contract) and rank 0 prints exactly one valid JSON line."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--cpu",
                        "--backend", "torch", "--gemm-m", "64", "--gemm-n", "64", "--gemm-k", "64",
                        "--steps", "2", "--warmup", "1", "--allreduce-mb", "0.25"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == world and j["config"]["parallelism"] == f"dp{world}"
    assert len(j["per_rank_ms_per_step"]) == world
    assert j["ms_per_step"] == max(j["per_rank_ms_per_step"])
    assert j["allreduce_busbw_gbs"] > 0 and j["allreduce_ms_in_step"] > 0


def test_self_launch_propagates_rank_failure(tmp_path):
    """One failing rank fails the whole launch (non-zero) and the surviving
    ranks are stopped instead of hanging in a rendezvous."""
    from kgs.parallel import launch

    script = tmp_path / "w.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "if r == 1: sys.exit(7)\n"
                      "time.sleep(60)\n")
    import time

    t0 = time.monotonic()
    rc = launch.spawn_local(3, [str(script)], require_gpus=False)
    assert rc == 7
    assert time.monotonic() - t0 < 30


def test_self_launch_refuses_missing_gpus():
    from kgs.parallel import launch

    assert launch.needs_self_launch(2, {}) and not launch.needs_self_launch(2, {"WORLD_SIZE": "2"})
    assert not launch.needs_self_launch(1, {})
    # this container has no GPU: asking for 2 real GPUs must fail fast, before spawning
    if launch.visible_gpu_count() < 2:
        assert launch.spawn_local(2, ["-c", "pass"], require_gpus=True) == 1


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "KGS_FAULT", "KGS_LAUNCH_PARENT")}
    env["OMP_NUM_THREADS"] = "1"
    env.update(extra)
    return env


_TINY = ["--cpu", "--backend", "torch", "--gemm-m", "64", "--gemm-n", "64", "--gemm-k", "64",
         "--steps", "2", "--warmup", "1", "--allreduce-mb", "0.25"]


def _error_line(stdout):
    lines = [json.loads(ln) for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return lines[0]


def test_bench_stalled_rank_fails_fast_with_error_json():
    """one of 8 gloo ranks stalls; the run ends inside
    its launch timeout, exits non-zero and prints ONE error JSON line naming
    the rank that is behind."""
    import subprocess
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", *_TINY,
                        "--launch-timeout", "25", "--rendezvous-timeout", "20"],
                       capture_output=True, text=True, env=_bench_env(KGS_FAULT="warmup:5:stall:600"), timeout=200)
    dt = time.monotonic() - t0
    assert p.returncode != 0
    assert dt < 25 + 30 + 30, dt
    err = _error_line(p.stdout)
    assert err["status"] == "error" and err["n_gpus"] == 8 and err["value"] is None
    assert err["metric"].startswith("in-pod bf16 GEMM TFLOPS")
    assert err["failing_rank"] == 5, err
    assert err["rank_phases"]["5"].endswith(":setup") and err["rank_phases"]["0"].endswith(":warmup")
    assert err["ranks_behind"] == [5]


def test_bench_raising_rank_kills_all_within_seconds():
    import subprocess
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", *_TINY,
                        "--launch-timeout", "120"],
                       capture_output=True, text=True, env=_bench_env(KGS_FAULT="setup:2:raise"), timeout=200)
    dt = time.monotonic() - t0
    assert p.returncode != 0
    assert dt < 60, dt  # not the 120 s watchdog: the launcher stops the peers
    err = _error_line(p.stdout)
    assert err["status"] == "error" and err["failing_rank"] == 2
    assert any("injected fault at setup on rank 2" in ln for ln in err["stderr_tail"]["2"])


def test_bench_missing_rank_fails_at_rendezvous():
    """torchrun-style launch where one rank never starts: the rendezvous
    timeout (not the collective timeout) ends rank 0 with an error line."""
    import subprocess

    from kgs.parallel.launch import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = _bench_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                     MASTER_PORT=str(free_port()))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", *_TINY,
                        "--rendezvous-timeout", "5", "--launch-timeout", "60"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode != 0
    err = _error_line(p.stdout)
    assert err["status"] == "error" and err["phase"] == "rendezvous", err


def test_distinct_device_check():
    import datetime

    import torch.distributed as dist

    from kgs.parallel.dist import DeviceConflict, check_distinct_devices
    from kgs.parallel.launch import free_port

    store = dist.TCPStore("127.0.0.1", free_port(), 1, is_master=True, timeout=datetime.timedelta(seconds=5))
    check_distinct_devices(store, 0, 1, "0:3:0/uuid-a", 5)
    store.set("kgs/dev/1", "0:3:0/uuid-a")  # a second rank claiming the same GPU
    with pytest.raises(DeviceConflict, match=r"ranks \[0, 1\]"):
        check_distinct_devices(store, 0, 2, "0:3:0/uuid-a", 5)


def _torchrun(nproc, *extra, fault=None, timeout=240):
    import subprocess

    from kgs.parallel.launch import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = _bench_env(**({"KGS_FAULT": fault} if fault else {}))
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                           os.path.join(root, "bench.py"), "--gpus", str(nproc), *_TINY, *extra],
                          capture_output=True, text=True, env=env, timeout=timeout, cwd="/tmp")


def test_bench_under_torchrun_agent_store():
    """The driver's launch (torch.distributed.run, static rendezvous: the agent
    hosts the store and the ranks are its clients) works with our own store."""
    p = _torchrun(2)
    assert p.returncode == 0, p.stderr[-2000:]
    j = _error_line(p.stdout)
    assert j["n_gpus"] == 2 and "status" not in j


def test_bench_under_torchrun_failing_rank_reports():
    """torchrun tears the job down when a rank raises; rank 0 turns the agent's
    SIGTERM into the error line, and the launcher exits non-zero."""
    p = _torchrun(2, "--launch-timeout", "120", fault="setup:1:raise")
    assert p.returncode != 0
    j = _error_line(p.stdout)
    assert j["status"] == "error" and j["value"] is None


def test_pick_device_index_one_gpu_per_rank_launchers():
    """a rank that sees exactly one GPU (SLURM --gpus-per-task=1,
    one container per rank) uses it whatever its LOCAL_RANK; with several
    visible GPUs LOCAL_RANK must index one."""
    from kgs.parallel.dist import DeviceConflict, pick_device_index

    assert pick_device_index(5, 1) == 0
    assert pick_device_index(3, 8) == 3
    with pytest.raises(DeviceConflict):
        pick_device_index(9, 8)
    assert pick_device_index(9, 8, allow_shared_device=True) == 1
    with pytest.raises(DeviceConflict):
        pick_device_index(0, 0)


def test_watchdog_shutdown_bound_keeps_a_reported_result(tmp_path):
    """after the result line, a lagging teardown ends the rank with
    status 0 (the shutdown-only bound), not the run watchdog's 124."""
    import subprocess
    import sys
    import time

    code = ("import time, sys; sys.path.insert(0, %r)\n"
            "from kgs.parallel.launch import Watchdog\n"
            "wd = Watchdog(1.0, 0, 1, {'metric': 'x'})\n"
            "wd.shutdown_bound(0.5)\n"
            "time.sleep(5)\n") % ROOT
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (r.returncode, r.stderr)
    assert time.monotonic() - t0 < 4.5
    assert "shutdown not done" in r.stderr and "watchdog: no completion" not in r.stderr


def _bench_inproc(*extra):
    import contextlib
    import io

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from kgs.parallel import launch

    launch._reported = False  # one JSON line per process; these tests call main() more than once
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.main(["--gpus", "1", "--steps", "2", "--warmup", "1", "--gemm-m", "128", "--gemm-n", "64",
                         "--gemm-k", "96", "--backend", "torch", "--cpu", "--yardstick-steps", "2", *extra])
    lines = [json.loads(ln) for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, buf.getvalue()
    return rc, lines[0]


def test_bench_line_carries_same_box_yardstick_and_full_check(monkeypatch):
    """the default run checks the last timed output in full
    against fp32 (rel_err) and times the vendor GEMM interleaved with the kgs
    step (hipblaslt_tflops, ratio_vs_hipblaslt). value / ms_per_step stay the
    timed region's: value = 4 GEMMs x 2MNK / ms_per_step."""
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    rc, j = _bench_inproc()
    assert rc == 0 and "status" not in j
    for key in ("rel_err", "hipblaslt_tflops", "ratio_vs_hipblaslt", "yardstick"):
        assert key in j, key
    assert 0 <= j["rel_err"] < 1e-2
    ys = j["yardstick"]
    assert ys["rounds"] == 3 and len(ys["kgs_ms"]) == 3 and len(ys["ref_ms"]) == 3
    assert j["ratio_vs_hipblaslt"] == pytest.approx(ys["ref_ms_per_step"] / ys["kgs_ms_per_step"], rel=1e-3)
    flops = 4 * 2.0 * 128 * 64 * 96
    assert j["value"] == pytest.approx(flops / (j["ms_per_step"] * 1e-3) / 1e12, abs=0.011, rel=2e-3)
    # the yardstick is untimed extra: its kgs median is not what value reports
    assert j["ms_per_step"] == max(j["per_rank_ms_per_step"])
    rc0, j0 = _bench_inproc("--yardstick-rounds", "0")
    assert rc0 == 0 and "ratio_vs_hipblaslt" not in j0 and "rel_err" in j0


def test_bench_fails_loudly_on_a_wrong_timed_output(monkeypatch):
    from kgs.models.gemm_workload import GemmWorkload

    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    real = GemmWorkload.step

    def corrupt(self, reference=False):
        real(self, reference)
        if not reference:
            self.c[(self.g - 1) & 1][3, 5] += 1e3  # one wrong element in the timed output
    monkeypatch.setattr(GemmWorkload, "step", corrupt)
    rc, j = _bench_inproc()
    assert rc == 1
    assert j["status"] == "error" and j["phase"] == "check" and j["rel_err"] > 1e-2 and j["value"] is None
