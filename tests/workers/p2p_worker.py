"""torchrun worker for tests/test_p2p_allreduce.py: every rank maps every other
rank's staging buffers over IPC and checks the P2P all-reduce bitwise against
the fp32 sum in rank order. On a one-GPU box all ranks share cuda:0 (IPC within
one device); on a multi-GPU node each rank has its own GPU (xGMI)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from kgs.parallel import dist as kdist  # noqa: E402
from kgs.parallel.p2p_allreduce import P2PAllReduce  # noqa: E402


def main():
    # gloo: the handle exchange needs no RCCL; both ranks may share the one GPU of a test box
    ctx = kdist.init_from_env(backend="gloo", allow_shared_device=True)
    rank, world = ctx.rank, ctx.world_size
    ar = P2PAllReduce(group=ctx.group, max_bytes=4 << 20, device=ctx.device, timeout_s=5.0)
    ok = True
    results = []
    for dtype in (torch.float32, torch.bfloat16):
        esz = torch.tensor([], dtype=dtype).element_size()
        for nbytes in (16, 4096, 65536 + 16, 1 << 20, 4 << 20):
            for algo in ("oneshot", "twoshot"):
                n = nbytes // esz
                xs = [((torch.arange(n, device=ctx.device, dtype=torch.float32) * (r + 1)) % 97 - 48).to(dtype) / 8
                      for r in range(world)]
                ref = xs[0].float()
                for r in range(1, world):
                    ref = ref + xs[r].float()
                ref = ref.to(dtype)
                for _ in range(3):  # repeated calls exercise the epoch flags
                    y = ar.all_reduce(xs[rank], algo=algo)
                    ar.check()  # fail fast on a barrier timeout
                good = bool(torch.equal(y, ref))
                ok &= good
                results.append({"dtype": str(dtype), "bytes": nbytes, "algo": algo, "ok": good})
    ar.check()
    ar.close()
    if rank == 0:
        print(json.dumps({"world": world, "ok": ok, "cases": results}), flush=True)
    kdist.shutdown(ctx)
    return 0 if ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
