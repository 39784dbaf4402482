#!/usr/bin/env python3
"""Memory-bound kernels on one MI355X: HIP vector add (every streaming
configuration) and the bf16 transpose, against the torch equivalents, in GB/s
of HBM traffic. Interleaved rounds in one process; writes a JSON summary."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgs.ops.elementwise import transpose_bf16, vector_add  # noqa: E402


def time_fn(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def run(fns, nbytes, rounds, iters):
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    ts = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            ts[k].append(time_fn(f, iters))
    return {k: round(nbytes / (sorted(v)[len(v) // 2] * 1e-3) / 1e9, 1) for k, v in ts.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=1 << 28)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/elementwise.json")
    a = ap.parse_args()
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        x = torch.rand(a.elems, device="cuda").to(dt)
        y = torch.rand(a.elems, device="cuda").to(dt)
        z = torch.empty_like(x)
        ok = all(torch.equal(vector_add(x, y, variant=v), x + y) for v in range(7))
        fns = {f"kgs_v{v}": (lambda v=v: vector_add(x, y, out=z, variant=v)) for v in range(7)}
        fns["torch_add"] = lambda: torch.add(x, y, out=z)
        fns["torch_copy"] = lambda: z.copy_(x)
        gbs = run(fns, 3 * x.numel() * x.element_size(), a.rounds, a.iters)
        gbs["torch_copy"] = round(gbs["torch_copy"] * 2 / 3, 1)  # copy moves 2 arrays, not 3
        res[f"vector_add_{str(dt).split('.')[-1]}"] = {"gbs": gbs, "bitwise_ok": ok, "bytes": 3 * x.numel() * x.element_size()}
        print(json.dumps({f"vector_add_{dt}": gbs, "ok": ok}), flush=True)
        del x, y, z
    for (r, c) in ((8192, 8192), (16384, 4096), (4096, 11008)):
        m = torch.randn(r, c, device="cuda").bfloat16()
        ok = all(torch.equal(transpose_bf16(m, variant=v), m.t().contiguous()) for v in (1, 2))
        fns = {"kgs_auto": lambda: transpose_bf16(m), "kgs_elementwise": lambda: transpose_bf16(m, variant=1),
               "torch_t_contiguous": lambda: m.t().contiguous()}
        gbs = run(fns, 2 * m.numel() * 2, a.rounds, a.iters)
        res[f"transpose_{r}x{c}"] = {"gbs": gbs, "bitwise_ok": ok}
        print(json.dumps({f"transpose_{r}x{c}": gbs, "ok": ok}), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
