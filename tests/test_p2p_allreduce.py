"""Peer-to-peer xGMI all-reduce (native/kernels/allreduce_p2p.hip).

GPU tests compare bitwise against the fp32 sum of the ranks' tensors in rank
order (the kernel sums peers 0..N-1 in f32 on every rank). Two shapes of
"multi-rank" fit a one-GPU box: N ranks played by one launch in one process (no IPC),
and N processes sharing the GPU through IPC handles (the real code path).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bare(world, oneshot_max=None):
    from kgs.parallel.p2p_allreduce import P2PAllReduce

    ar = object.__new__(P2PAllReduce)
    ar.world = world
    ar.max_blocks = 128
    ar.oneshot_max_bytes = oneshot_max if oneshot_max is not None else ((1 << 20) if world <= 4 else (256 << 10))
    ar._epoch = 0
    return ar


def test_algo_and_grid_selection():
    ar = _bare(8)
    assert ar.pick_algo(4096) == "oneshot"
    assert ar.pick_algo(256 << 10) == "oneshot"
    assert ar.pick_algo((256 << 10) + 16) == "twoshot"
    assert _bare(2).pick_algo(8 << 20) == "oneshot"  # two ranks: two-shot saves nothing
    assert ar.blocks_for(16, "oneshot") == 1
    assert ar.blocks_for(512 * 16 * 3, "oneshot") == 3
    assert ar.blocks_for(1 << 30, "twoshot") == 128


def test_epoch_never_zero():
    ar = _bare(2)
    ar._epoch = 0xFFFFFFFE
    assert ar._next_epoch() == 0xFFFFFFFF
    assert ar._next_epoch() == 1  # wraps past 0 (flags start zeroed)


def _inputs(world, n, dtype, device):
    return [((torch.arange(n, device=device, dtype=torch.float32) * (r + 3)) % 61 - 30).to(dtype) / 4
            for r in range(world)]


def _ref(xs):
    acc = xs[0].float()
    for x in xs[1:]:
        acc = acc + x.float()
    return acc.to(xs[0].dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("algo", ["oneshot", "twoshot"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_local_ranks_bitwise(world, algo, dtype):
    from kgs.parallel.p2p_allreduce import P2PAllReduce

    ar = P2PAllReduce.local_ranks(world, max_bytes=8 << 20, device="cuda", timeout_s=3.0)
    try:
        esz = torch.tensor([], dtype=dtype).element_size()
        for nbytes in (16, 1008, 4096, (1 << 20) + 48, 8 << 20):
            xs = _inputs(world, nbytes // esz, dtype, "cuda")
            for _ in range(2):
                outs = ar.all_reduce_local(xs, algo=algo)
                ar.check()  # fail fast on a barrier timeout
            ref = _ref(xs)
            for o in outs:
                assert torch.equal(o, ref), (algo, dtype, nbytes)
        ar.check()
    finally:
        ar.close()


@pytest.mark.gpu
def test_graph_capture_replays_with_device_epochs():
    """Captured once, replayed with new inputs: each replay must synchronise
    afresh (device-side epochs), not pass on the flags of the capture-time call."""
    from kgs.parallel.p2p_allreduce import P2PAllReduce

    world, n = 4, 1 << 16
    ar = P2PAllReduce.local_ranks(world, max_bytes=1 << 20, device="cuda", timeout_s=3.0)
    try:
        xs = [torch.zeros(n, device="cuda") for _ in range(world)]
        outs = [torch.empty(n, device="cuda") for _ in range(world)]
        ar.all_reduce_local(xs, outs=outs)  # warm up outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                ar.all_reduce_local(xs, outs=outs)
        torch.cuda.current_stream().wait_stream(s)
        for it in range(5):
            for r in range(world):
                xs[r].fill_(float(r + 1 + it))
            g.replay()
            torch.cuda.synchronize()
            ar.check()
            want = float(sum(r + 1 + it for r in range(world)))
            for o in outs:
                assert torch.all(o == want), (it, o[:4])
    finally:
        ar.close()


@pytest.mark.gpu
def test_missing_peer_times_out_instead_of_hanging():
    from kgs.parallel.p2p_allreduce import P2PAllReduce

    ar = P2PAllReduce.local_ranks(2, max_bytes=1 << 20, device="cuda", timeout_s=0.05)
    try:
        x = torch.ones(1024, device="cuda")
        out = torch.empty_like(x)
        # launch rank 0 only: its barrier can never complete
        ar._launch(0, x, out, "oneshot", ar._next_epoch(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="timed out"):
            ar.check()
    finally:
        ar.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_ipc_two_processes():
    """Two processes, IPC-mapped staging buffers (same GPU on a one-GPU box)."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "workers", "p2p_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == 2 and res["ok"], res


@pytest.mark.gpu
def test_tensor_parallel_mlp_on_p2p_allreduce():
    """4-way TP MLP on the HIP GEMM, row-parallel partials summed by the P2P
    kernel (one launch plays the 4 ranks): every rank gets the same output, and
    it matches the unsplit MLP to bf16 accuracy."""
    from kgs.parallel.p2p_allreduce import P2PAllReduce
    from kgs.parallel.tensor_parallel import reference_mlp, tp_mlp_local

    g = torch.Generator(device="cuda").manual_seed(3)
    din, dff, dout, world = 1024, 4096, 1024, 4
    x = (torch.randn(512, din, device="cuda", generator=g)).bfloat16()
    w1 = (torch.randn(dff, din, device="cuda", generator=g) * din ** -0.5).bfloat16()
    b1 = (torch.randn(dff, device="cuda", generator=g) * 0.1).bfloat16()
    w2 = (torch.randn(dout, dff, device="cuda", generator=g) * dff ** -0.5).bfloat16()
    b2 = (torch.randn(dout, device="cuda", generator=g) * 0.1).bfloat16()
    ar = P2PAllReduce.local_ranks(world, max_bytes=8 << 20, device="cuda", timeout_s=3.0)
    try:
        outs = tp_mlp_local(x, w1, b1, w2, b2, world, p2p_local=ar)
        torch.cuda.synchronize()
        ar.check()
    finally:
        ar.close()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ref = reference_mlp(x, w1, b1, w2, b2)
    rel = ((outs[0].float() - ref).norm() / ref.norm()).item()
    assert rel < 2e-2, rel
