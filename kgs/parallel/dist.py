"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

``torch.distributed`` backend ``"nccl"`` *is* RCCL on ROCm. Each rank binds to
``cuda:LOCAL_RANK``. Without a GPU (CI, this container) the same code runs on
``gloo`` so the distributed paths are tested on CPU with world_size > 1.

The reference has no distributed runtime at all; this is the
data plane the in-pod workload needs for BASELINE.json config 4.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: Any = None
    group: Any = None
    initialized_here: bool = False

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_from_env(expected_world: int | None = None, backend: str | None = None, timeout_s: float = 600.0,
                  device_type: str | None = None) -> DistContext:
    """Initialise from torchrun-style env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*).

    With WORLD_SIZE unset (or 1) this is a single-process context and no process
    group is created. ``expected_world`` is a sanity check against ``--gpus``.
    """
    import torch
    import torch.distributed as dist

    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", rank)
    if expected_world is not None and expected_world != world:
        if world == 1 and expected_world > 1:
            raise SystemExit(
                f"--gpus {expected_world} needs one process per GPU: launch with "
                f"`python -m torch.distributed.run --nproc-per-node {expected_world} --master-addr 127.0.0.1 ...`"
            )
        raise SystemExit(f"WORLD_SIZE={world} does not match --gpus {expected_world}")

    use_gpu = torch.cuda.is_available() if device_type is None else device_type == "cuda"
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev_index = local_rank % max(1, ndev)
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")

    ctx = DistContext(rank=rank, world_size=world, local_rank=local_rank, device=device)
    if world > 1:
        be = backend or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            kw = {}
            if be == "nccl":
                kw["device_id"] = device
            dist.init_process_group(be, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
            ctx.initialized_here = True
        ctx.backend = be
        ctx.group = dist.group.WORLD
    return ctx


def barrier(ctx: DistContext) -> None:
    if ctx.distributed:
        import torch.distributed as dist

        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def max_over_ranks(ctx: DistContext, value: float) -> float:
    if not ctx.distributed:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_object(ctx: DistContext, obj):
    if not ctx.distributed:
        return [obj]
    import torch.distributed as dist

    out = [None] * ctx.world_size
    dist.all_gather_object(out, obj)
    return out


def shutdown(ctx: DistContext, timeout_s: float = 60.0) -> None:
    """Tear the process group down so that no rank exits while a peer still
    holds live transport state towards it.

    A gloo rank whose peer process has already exited can abort in its
    transport thread ("terminate called without an active exception", seen on
    8-rank CPU runs). So: barrier (all collectives done), drop our references and
    destroy the group, then a store-side exit barrier -- every rank counts itself
    out and leaves only once all have destroyed theirs. Rank 0 hosts the store
    and is therefore the last to go.
    """
    if not ctx.initialized_here:
        return
    import gc
    import time

    import torch.distributed as dist

    store = None
    try:
        if ctx.world_size > 1:
            store = dist.distributed_c10d._get_default_store()
            barrier(ctx)
    except Exception:  # pragma: no cover - best effort on a broken group
        store = None
    ctx.group = None
    try:
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        pass
    gc.collect()
    if store is None:
        return
    try:
        store.add("kgs/exit", 1)
        deadline = time.monotonic() + timeout_s
        while store.add("kgs/exit", 0) < ctx.world_size and time.monotonic() < deadline:
            time.sleep(0.01)
        if ctx.rank == 0:  # give the others a moment to read the final count
            deadline = time.monotonic() + 2.0
            while store.add("kgs/exit_ack", 0) < ctx.world_size - 1 and time.monotonic() < deadline:
                time.sleep(0.01)
        else:
            store.add("kgs/exit_ack", 1)
    except Exception:  # pragma: no cover - rank 0's store already gone: nothing left to protect
        pass
