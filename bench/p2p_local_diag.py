#!/usr/bin/env python3
"""Diagnose a wrong P2P all-reduce result with local ranks (one GPU): every call
checked, the error word read after every call (a barrier timeout sets bit
1 << phase), first failure reported with the wrong elements' positions.

    python bench/p2p_local_diag.py --world 8 --kib 64 --algos oneshot,twoshot --calls 200
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--kib", type=int, default=64)
    ap.add_argument("--algos", default="oneshot,twoshot")
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--uncached", action="store_true")
    ap.add_argument("--timeout", type=float, default=2.0)
    a = ap.parse_args(argv)
    from kgs.parallel.p2p_allreduce import P2PAllReduce

    ar = P2PAllReduce.local_ranks(a.world, max_bytes=8 << 20, timeout_s=a.timeout, staging_uncached=a.uncached)
    n = a.kib * 1024 // 2
    ins = [torch.full((n,), float(r + 1), dtype=torch.bfloat16, device="cuda") for r in range(a.world)]
    want = float(sum(range(1, a.world + 1)))
    algos = a.algos.split(",")
    bad = None
    for i in range(a.calls):
        algo = algos[i % len(algos)]
        outs = ar.all_reduce_local(ins, algo=algo)
        torch.cuda.synchronize()
        err = int(ar.err.item())
        wrong = [int((o != want).sum()) for o in outs]
        if err or any(wrong):
            idx = (outs[0] != want).nonzero().flatten()[:8].tolist()
            vals = outs[0][idx].float().tolist() if idx else []
            bad = {"call": i, "algo": algo, "err": err, "wrong_per_rank": wrong, "first_idx": idx, "vals": vals,
                   "blocks": ar.blocks_for(n * 2, algo)}
            break
    res = {"world": a.world, "kib": a.kib, "algos": algos, "calls": a.calls, "uncached": a.uncached,
           "first_failure": bad}
    print(json.dumps(res), flush=True)
    ar.close()
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
