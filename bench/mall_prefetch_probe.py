#!/usr/bin/env python3
"""Does touching a decode projection's weights into the Infinity Cache, on a
side stream while the PREVIOUS projection runs, speed the projection up?

Batch-256 Llama-3-8B decode shapes on the production routes (tile-panel
weights, non-temporal weight loads, fp32 split-K partials without the reduce):
  pair "down>qkv": down [4096, 14336] then the next layer's qkv [6144, 4096]
  pair "gateup>down": gate|up + SwiGLU [28672, 4096] then down
Weights rotate through rings larger than the 256 MiB cache, as a 32-layer step
sees them. Per iteration, events around each GEMM on the main stream; in the
"touch" arm, ``kgs_exp_mall_touch`` (native/experiments/prefetch_exp.hip,
``--nwg`` workgroups) reads the second GEMM's weights on a side stream that
starts with the first GEMM. Medians over ``--iters``; arms interleaved.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--pairs", default="down>qkv,gateup>down,o>gateup")
    ap.add_argument("--nwg", default="32,64")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--ring-gb", type=float, default=1.5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from kgs.ops import experiments
    from kgs.ops.gemm import gemm_nt_w4x_partials, gemm_nt_w4x_swiglu, pack_w4x_weight, reserve_splitk_workspace

    dev = torch.device("cuda", 0)
    lib = experiments.lib()
    lib.kgs_exp_mall_touch.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p]
    lib.kgs_exp_mall_touch.restype = ctypes.c_int
    sink = torch.zeros(256, dtype=torch.int32, device=dev)
    shapes = {"qkv": (6144, 4096, 128, 4), "o": (4096, 4096, 128, 4), "down": (4096, 14336, 128, 8),
              "gateup": (28672, 4096, 128, 1)}  # N, K, bn, K slices (W4X_TUNED, bucket 256)
    reserve_splitk_workspace(dev, 8 * 256 * 6144)
    rings, xs = {}, {}
    for name in {p for pair in a.pairs.split(",") for p in pair.split(">")}:
        N, K, bn, _ = shapes[name]
        n = max(2, int(a.ring_gb * 1e9 // (N * K * 2)))
        rings[name] = [pack_w4x_weight((torch.randn(N, K, device=dev) * 0.02).bfloat16(), bn,
                                       swiglu=name == "gateup") for _ in range(n)]
        xs[name] = torch.randn(256, K, device=dev).bfloat16()
        torch.cuda.empty_cache()

    def gemm(name, i):
        N, K, bn, s = shapes[name]
        w = rings[name][i % len(rings[name])]
        if name == "gateup":
            return gemm_nt_w4x_swiglu(xs[name], w, bn=bn, bm=256, nt_weights=True)
        return gemm_nt_w4x_partials(xs[name], w, bn, s, bm=128 if name == "o" else 256, nt_weights=True)

    side = torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream(dev)
    res = []
    for pair in a.pairs.split(","):
        first, second = pair.split(">")
        arms = ["plain"] + [f"touch{n}" for n in a.nwg.split(",")]
        t = {arm: {"first": [], "second": [], "both": []} for arm in arms}
        for it in range(a.iters + 3):
            for arm in arms:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
                if arm != "plain":
                    side.wait_stream(main_s)
                    w = rings[second][it % len(rings[second])].data
                    with torch.cuda.stream(side):
                        rc = lib.kgs_exp_mall_touch(w.data_ptr(), w.numel() * 2, int(arm[5:]), sink.data_ptr(),
                                                    side.cuda_stream)
                        assert rc == 0, rc
                gemm(first, it)
                ev[1].record()
                gemm(second, it)
                ev[2].record()
                if arm != "plain":
                    main_s.wait_stream(side)
                ev[2].synchronize()
                if it >= 3:
                    t[arm]["first"].append(ev[0].elapsed_time(ev[1]) * 1e3)
                    t[arm]["second"].append(ev[1].elapsed_time(ev[2]) * 1e3)
                    t[arm]["both"].append(ev[0].elapsed_time(ev[2]) * 1e3)
        r = {"pair": pair, **{arm: {k: round(statistics.median(v), 2) for k, v in d.items()} for arm, d in t.items()}}
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
