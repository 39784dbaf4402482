"""Data-parallel MLP training on the HIP kernels: the DP gradient-sync pattern of
SURVEY.md §2.6 run as a real training loop instead of a synthetic bucket.

One process per GPU. Every rank holds a full replica of a stack of
``kgs.ops.Linear`` layers, whose forward and backward GEMMs run on the gfx950
MFMA kernel. Each rank trains on its own shard of a synthetic regression batch.
Parameter gradients are packed into buckets (:class:`kgs.parallel.allreduce.GradBucketer`);
a bucket is all-reduced over RCCL as soon as backward has produced all its
gradients, so the collectives overlap the rest of backward. ``wait()`` before
the optimizer step is the only synchronisation point.

``backend="torch"`` swaps in ``torch.nn.Linear`` (CPU / gloo tests, and the
hipBLASLt comparison on a GPU). The reference has no training code (SURVEY.md
§2.6); nothing here is ported.
"""
from __future__ import annotations

import time

import torch


class MLP(torch.nn.Module):
    def __init__(self, dims: list, act: str = "gelu", backend: str = "kgs", device=None, dtype=torch.bfloat16,
                 seed: int = 0):
        super().__init__()
        self.backend = backend
        g = torch.Generator(device="cpu").manual_seed(seed)
        layers = []
        for i, (din, dout) in enumerate(zip(dims[:-1], dims[1:])):
            last = i == len(dims) - 2
            a = None if last else act
            if backend == "kgs":
                from kgs.ops.gemm import Linear

                lin = Linear(din, dout, bias=True, act=a, device=device)
            else:
                lin = _TorchLinear(din, dout, act=a, device=device, dtype=dtype)
            with torch.no_grad():  # identical init on every rank and for both backends
                lin.weight.copy_(torch.randn(dout, din, generator=g) * din ** -0.5)
                lin.bias.zero_()
            layers.append(lin)
        self.layers = torch.nn.ModuleList(layers)

    def forward(self, x):
        for lin in self.layers:
            x = lin(x)
        return x

    def flops_per_sample(self) -> float:
        """fwd + bwd GEMM FLOPs per sample (2 for fwd, 4 for bwd per MAC)."""
        return 6.0 * sum(lin.weight.numel() for lin in self.layers)


class _TorchLinear(torch.nn.Linear):
    def __init__(self, din, dout, act=None, device=None, dtype=None):
        super().__init__(din, dout, bias=True, device=device, dtype=dtype)
        self.act = act

    def forward(self, x):
        y = super().forward(x)
        if self.act == "gelu":
            y = torch.nn.functional.gelu(y, approximate="tanh")
        elif self.act == "relu":
            y = torch.relu(y)
        elif self.act == "silu":
            y = torch.nn.functional.silu(y)
        return y


def synthetic_batch(step: int, batch: int, din: int, dout: int, device, dtype, seed: int = 1234):
    """Deterministic (step-indexed) regression batch from a fixed random teacher."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    teacher = torch.randn(dout, din, generator=g) * din ** -0.5
    gs = torch.Generator(device="cpu").manual_seed(seed + 1 + step)
    x = torch.randn(batch, din, generator=gs)
    y = torch.tanh(x @ teacher.T)
    return x.to(device=device, dtype=dtype), y.to(device=device, dtype=dtype)


def train_dp(dims: list, steps: int = 10, global_batch: int = 1024, lr: float = 0.05, backend: str = "kgs",
             device=None, group=None, bucket_mb: float = 64.0, dtype=torch.bfloat16, warmup: int = 2) -> dict:
    """Run ``steps`` SGD steps of data-parallel training; call on every rank.

    The global batch is split evenly over the ranks (rank r takes rows
    r*B/N .. (r+1)*B/N of the step's batch), gradients are averaged with the
    bucketed, backward-overlapped all-reduce, and every rank applies the same
    update, so all replicas stay identical (checked by the tests).
    """
    import torch.distributed as dist

    from kgs.parallel.allreduce import GradBucketer

    distributed = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if distributed else 1
    rank = dist.get_rank(group) if distributed else 0
    if global_batch % world:
        raise ValueError("global_batch must divide evenly over the ranks")
    per = global_batch // world
    device = torch.device(device) if device is not None else torch.device("cpu")
    model = MLP(dims, backend=backend, device=device, dtype=dtype)
    params = list(model.parameters())
    bucketer = GradBucketer(params, bucket_mb=bucket_mb, group=group) if world > 1 else None
    losses, times = [], []
    sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)
    for step in range(steps):
        x, y = synthetic_batch(step, global_batch, dims[0], dims[-1], device, dtype)
        x, y = x[rank * per:(rank + 1) * per].contiguous(), y[rank * per:(rank + 1) * per].contiguous()
        sync()
        t0 = time.perf_counter()
        for p in params:
            p.grad = None
        out = model(x)
        loss = torch.nn.functional.mse_loss(out.float(), y.float())
        loss.backward()
        if bucketer is not None:
            bucketer.wait()
        with torch.no_grad():
            for p in params:
                p.add_(p.grad, alpha=-lr)
        sync()
        times.append(time.perf_counter() - t0)
        lv = loss.detach()
        if distributed:
            dist.all_reduce(lv, group=group)
            lv = lv / world
        losses.append(float(lv))
    if bucketer is not None:
        bucketer.remove()
    timed = times[warmup:] or times
    ms = 1e3 * sum(timed) / len(timed)
    return {
        "losses": losses,
        "ms_per_step": ms,
        "tflops_per_rank": model.flops_per_sample() * per / (ms * 1e-3) / 1e12,
        "world": world,
        "params": sum(p.numel() for p in params),
        "model": model,
    }
