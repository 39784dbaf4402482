#!/usr/bin/env python3
"""P2P all-reduce with cached vs uncached staging buffers, one GPU.

The staging buffers are ordinary cached device memory. Their cross-GPU
correctness rests on the flag protocol's L2 write-back before each flag and
its invalidate after each poll (native/kernels/allreduce_p2p.hip
block_barrier, pinned in the ISA by tests/test_kernel_resources.py). The
alternative is uncached staging, like the signal blocks. This measures what
that alternative costs on the paths one GPU can run: local ranks (one launch
plays N ranks on one GPU, so every staging access is local), one- and
two-shot, interleaved rounds, medians. Cross-GPU (xGMI) reads are not
measurable on a 1-GPU box.

    python bench/p2p_staging_ab.py --out gpurun_out/p2p_staging_ab.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--sizes-kib", default="64,512,4096")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from kgs.parallel.p2p_allreduce import P2PAllReduce

    rows = []
    for world in [int(x) for x in a.worlds.split(",")]:
        ars = {mode: P2PAllReduce.local_ranks(world, max_bytes=8 << 20, staging_uncached=(mode == "uncached"))
               for mode in ("cached", "uncached")}
        for kib in [int(x) for x in a.sizes_kib.split(",")]:
            n = kib * 1024 // 2
            ins = [torch.full((n,), float(r + 1), dtype=torch.bfloat16, device="cuda") for r in range(world)]
            want = float(sum(range(1, world + 1)))
            for algo in ("oneshot", "twoshot"):
                times = {m: [] for m in ars}
                for mode, ar in ars.items():  # numerics first
                    outs = ar.all_reduce_local(ins, algo=algo)
                    torch.cuda.synchronize()
                    err = int(ar.err.item())
                    wrong = [int((o != want).sum()) for o in outs]
                    if err or any(wrong):
                        raise SystemExit(json.dumps({"failure": {"world": world, "kib": kib, "algo": algo,
                                                                 "mode": mode, "err": err, "wrong": wrong,
                                                                 "at": "first call of the cell"}}))
                for _ in range(a.rounds):
                    for mode, ar in ars.items():
                        outs = [torch.empty_like(x) for x in ins]
                        for _ in range(5):
                            ar.all_reduce_local(ins, algo=algo, outs=outs)
                        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        s.record()
                        for _ in range(a.iters):
                            ar.all_reduce_local(ins, algo=algo, outs=outs)
                        e.record()
                        e.synchronize()
                        times[mode].append(s.elapsed_time(e) / a.iters * 1e3)
                        # every timed block ends checked: the last call's outputs and the barrier error word
                        # (a timed-out barrier in any call of the block sets it and stays set)
                        err = int(ar.err.item())
                        wrong = [int((o != want).sum()) for o in outs]
                        if err or any(wrong):
                            raise SystemExit(json.dumps({"failure": {"world": world, "kib": kib, "algo": algo,
                                                                     "mode": mode, "err": err, "wrong": wrong,
                                                                     "block_ms": times[mode][-1] / 1e3 * a.iters}}))
                row = {"world": world, "kib": kib, "algo": algo,
                       **{f"{m}_us": round(statistics.median(v), 2) for m, v in times.items()}}
                row["uncached_over_cached"] = round(row["uncached_us"] / row["cached_us"], 3)
                rows.append(row)
                print(json.dumps(row), flush=True)
        for ar in ars.values():
            ar.check()
            ar.close()
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
