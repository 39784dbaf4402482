"""RCCL (torch.distributed "nccl") on the GPUs this process can see: a
one-process group on a one-GPU box (the collective path still runs through
RCCL's kernels), the xGMI sweep when launched with more ranks."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kgs.parallel.allreduce import allreduce_sweep  # noqa: E402


def main():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    pts = allreduce_sweep(sizes=[1 << 10, 1 << 16, 1 << 20, 16 << 20], iters=5, warmup=2, device=dev)
    ok = all(p.correct for p in pts)
    if rank == 0:
        print(json.dumps({"world": world, "backend": dist.get_backend(), "ok": ok,
                          "points": [p.as_dict() for p in pts]}), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
