"""Tensor parallelism (Megatron-style column/row split) on the HIP GEMM, with the
row-parallel reduction on the P2P xGMI all-reduce.

SURVEY.md §2.6: the reference runs vLLM at TP=1 and turns the custom
all-reduce off (/root/reference/pods/vllm-cpu-pod.yaml:17-20); TP>1 is where
the small-message all-reduce matters. This module is the in-repo consumer of
:class:`kgs.parallel.p2p_allreduce.P2PAllReduce`:

* :class:`ColumnParallelLinear` -- W split by output rows; every rank computes
  its slice of the activations, no communication.
* :class:`RowParallelLinear` -- W split by input columns; every rank computes a
  partial product of the full output, summed across ranks by ONE all-reduce
  (P2P one-shot/two-shot kernel when the group's GPUs are IPC-mapped, RCCL
  otherwise). The bias is added once, after the sum.
* :class:`TPMLP` -- column(gelu) -> row: one all-reduce per MLP, the
  transformer-block pattern.

Each rank holds shard ``rank`` of the weights (same seed on every rank, so the
full matrices never need to be sent). ``backend="torch"`` runs the same math
with torch GEMMs (CPU / gloo tests).
"""
from __future__ import annotations

import torch


def _linear(x, w, bias, act, backend):
    if backend == "kgs":
        from kgs.ops.gemm import gemm_nt

        y = gemm_nt(x, w, bias=bias, act=act)
        return y
    y = x @ w.T
    if bias is not None:
        y = y + bias
    if act == "gelu":
        y = torch.nn.functional.gelu(y, approximate="tanh")
    return y


def shard_rows(w: torch.Tensor, world: int, rank: int) -> torch.Tensor:
    n = w.shape[0]
    if n % world:
        raise ValueError(f"{n} output rows do not split over {world} ranks")
    return w[rank * n // world:(rank + 1) * n // world].contiguous()


def shard_cols(w: torch.Tensor, world: int, rank: int) -> torch.Tensor:
    k = w.shape[1]
    if k % world:
        raise ValueError(f"{k} input columns do not split over {world} ranks")
    return w[:, rank * k // world:(rank + 1) * k // world].contiguous()


class ColumnParallelLinear(torch.nn.Module):
    def __init__(self, weight: torch.Tensor, bias: torch.Tensor | None, world: int, rank: int, act=None,
                 backend="kgs"):
        super().__init__()
        self.weight = torch.nn.Parameter(shard_rows(weight, world, rank), requires_grad=False)
        self.bias = None if bias is None else torch.nn.Parameter(
            bias[rank * bias.numel() // world:(rank + 1) * bias.numel() // world].contiguous(), requires_grad=False)
        self.act, self.backend = act, backend

    def forward(self, x):
        return _linear(x, self.weight, self.bias, self.act, self.backend)


class RowParallelLinear(torch.nn.Module):
    def __init__(self, weight: torch.Tensor, bias: torch.Tensor | None, world: int, rank: int, reducer,
                 backend="kgs"):
        super().__init__()
        self.weight = torch.nn.Parameter(shard_cols(weight, world, rank), requires_grad=False)
        self.bias = None if bias is None else torch.nn.Parameter(bias.contiguous(), requires_grad=False)
        self.reducer, self.backend = reducer, backend

    def partial(self, x_shard):
        return _linear(x_shard, self.weight, None, None, self.backend)

    def forward(self, x_shard):
        y = self.reducer(self.partial(x_shard))
        return y + self.bias if self.bias is not None else y


class TPMLP(torch.nn.Module):
    """y = W2 . gelu(W1 . x + b1) + b2 with W1 column-split and W2 row-split."""

    def __init__(self, w1, b1, w2, b2, world: int, rank: int, reducer, backend="kgs"):
        super().__init__()
        self.up = ColumnParallelLinear(w1, b1, world, rank, act="gelu", backend=backend)
        self.down = RowParallelLinear(w2, b2, world, rank, reducer, backend=backend)

    def forward(self, x):
        return self.down(self.up(x))


def make_reducer(group=None, p2p=None):
    """Sum over the group: the P2P kernel when ``p2p`` (a P2PAllReduce) is given
    and the tensor fits, RCCL/gloo otherwise."""
    import torch.distributed as dist

    def reduce(t):
        if p2p is not None:
            return p2p.all_reduce(t.contiguous())
        t = t.contiguous()
        dist.all_reduce(t, group=group)
        return t

    return reduce


def reference_mlp(x, w1, b1, w2, b2):
    h = torch.nn.functional.gelu(x.float() @ w1.float().T + b1.float(), approximate="tanh")
    return h @ w2.float().T + b2.float()


def tp_mlp_local(x, w1, b1, w2, b2, world: int, p2p_local=None, backend="kgs"):
    """All ``world`` TP ranks in one process on one GPU (tests / single-GPU
    rehearsal): per-rank partials, reduced by the one-launch P2P kernel
    (``P2PAllReduce.local_ranks``) or by a plain sum."""
    partials = []
    for r in range(world):
        up = ColumnParallelLinear(w1, b1, world, r, act="gelu", backend=backend)
        down = RowParallelLinear(w2, None, world, r, reducer=None, backend=backend)
        partials.append(down.partial(up(x)))
    if p2p_local is not None:
        outs = p2p_local.all_reduce_local(partials)
        return [o + b2 for o in outs]
    s = partials[0].float()
    for p in partials[1:]:
        s = s + p.float()
    return [(s + b2.float()).to(partials[0].dtype) for _ in range(world)]
