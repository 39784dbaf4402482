"""RCCL collectives for the in-pod workload (torch.distributed, backend "nccl" = RCCL).

* :func:`allreduce_sweep` -- nccl-tests-style all-reduce sweep: for each message
  size, time ``iters`` back-to-back all-reduces and report algorithm bandwidth
  (bytes / t) and bus bandwidth (algbw * 2(n-1)/n), the number to hold against
  the xGMI roofline (one ring ~ one 153 GB/s link; RCCL's multi-ring / tree
  channels over the 8-GPU full mesh can use all 7 links). BASELINE.json config 4.
* :class:`GradBucketer` -- data-parallel gradient sync: gradients are packed
  into flat buckets (default 64 MiB: large enough that the per-collective
  latency is amortised, few enough to overlap with the backward pass) and each
  bucket is all-reduced asynchronously as soon as all its gradients are ready,
  on RCCL's own stream, overlapping the rest of backward.

The reference has no collectives; nothing here is a port.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

DEFAULT_SIZES = [1 << s for s in range(10, 31, 2)]  # 1 KiB .. 1 GiB


@dataclass
class SweepPoint:
    bytes: int
    dtype: str
    ms: float
    algbw_gbs: float
    busbw_gbs: float
    correct: bool

    def as_dict(self):
        return self.__dict__.copy()


def bus_factor(world: int) -> float:
    return 2.0 * (world - 1) / world if world > 1 else 0.0


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def allreduce_sweep(sizes=None, dtype=torch.float32, iters: int = 20, warmup: int = 5, device=None,
                    group=None, check: bool = True) -> list:
    """Run on every rank; returns the same list of :class:`SweepPoint` on all ranks
    (times are the max over ranks)."""
    sizes = sizes or DEFAULT_SIZES
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                        else torch.device("cpu"))
    esize = torch.tensor([], dtype=dtype).element_size()
    out = []
    for nbytes in sizes:
        n = max(1, nbytes // esize)
        buf = torch.empty(n, dtype=dtype, device=device)
        correct = True
        if check:
            buf.fill_(rank + 1)
            dist.all_reduce(buf, group=group)
            expect = world * (world + 1) / 2
            correct = bool(torch.all(buf == expect).item())
        for _ in range(warmup):
            dist.all_reduce(buf, group=group)
        _sync(device)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(buf, group=group)
        _sync(device)
        dt = (time.perf_counter() - t0) / iters
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dt = float(t.item())
        real = n * esize
        algbw = real / dt / 1e9
        out.append(SweepPoint(real, str(dtype).replace("torch.", ""), dt * 1e3, algbw, algbw * bus_factor(world),
                              correct))
    return out


class GradBucketer:
    """Bucketed, overlapped gradient all-reduce for data parallelism.

    ``GradBucketer(model.parameters(), bucket_mb=64)`` registers post-accumulate
    hooks; call :meth:`wait` after ``loss.backward()`` (before the optimizer
    step). Gradients are averaged over the group.
    """

    def __init__(self, params, bucket_mb: float = 64.0, group=None, average: bool = True):
        self.group = group
        self.world = dist.get_world_size(group)
        self.average = average
        params = [p for p in params if p.requires_grad]
        # reverse order: gradients of the last layers arrive first in backward
        params = list(reversed(params))
        cap = int(bucket_mb * (1 << 20))
        self.buckets = []
        cur, size = [], 0
        for p in params:
            nb = p.numel() * p.element_size()
            if cur and (size + nb > cap or p.dtype != cur[0].dtype or p.device != cur[0].device):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            self.buckets.append(cur)
        self._flat = []
        self._pending = [0] * len(self.buckets)
        self._work = [None] * len(self.buckets)
        self._index = {}
        for bi, b in enumerate(self.buckets):
            n = sum(p.numel() for p in b)
            self._flat.append(torch.zeros(n, dtype=b[0].dtype, device=b[0].device))
            off = 0
            for p in b:
                self._index[id(p)] = (bi, off)
                off += p.numel()
            self._pending[bi] = len(b)
        self._remaining = list(self._pending)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for b in self.buckets for p in b]

    def _on_grad(self, p):
        bi, off = self._index[id(p)]
        flat = self._flat[bi]
        flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
        self._remaining[bi] -= 1
        if self._remaining[bi] == 0:
            if self.average:
                flat.div_(self.world)
            self._work[bi] = dist.all_reduce(flat, group=self.group, async_op=True)

    def wait(self) -> None:
        for bi, b in enumerate(self.buckets):
            w = self._work[bi]
            if w is None:  # a parameter got no gradient this step: reduce what we have
                flat = self._flat[bi]
                if self.average:
                    flat.div_(self.world)
                dist.all_reduce(flat, group=self.group)
            else:
                w.wait()
            flat = self._flat[bi]
            off = 0
            for p in b:
                if p.grad is not None:
                    p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
                off += p.numel()
            self._work[bi] = None
            self._remaining[bi] = self._pending[bi]

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
