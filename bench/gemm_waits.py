#!/usr/bin/env python3
"""Where a persistent GEMM wave waits: lgkm (LDS reads) vs barrier 1 vs vm (DMA) vs barrier 2.

VERDICT r5 item 2 asked for the persistent kernel's extra ``SQ_WAIT_ANY`` to be attributed to its
wait kinds. bench/wait_split.py showed the extra is per K-step, not at the tile change. This uses the
wait-stamp build (native/kernels/gemm_w4p.h, L digit 10^6): every wave reads ``s_memtime`` before and
after each of a K-step's waits and barriers. The cycles are summed per category: a tile's K-steps
0-1, the steady loop, and the last two K-steps, which load the next tile.

The stamps cost cycles of their own (an SMEM read and its wait, six per K-step), so the build runs
slower than production. Read the numbers as shares of that build's K-step, not as production time.

    python bench/gemm_waits.py --shapes 8192,8192x4096x14336 --out gpurun_out/gemm_waits.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

CATS = ("tile_start", "steady", "tile_end")
KINDS = ("lgkm_wait", "barrier1", "vm_wait", "barrier2")
VARIANTS = {0: "production nt + deferred 4x4 (3-8 tiles/CU)", 1: "nt C, nothing deferred",
            2: "tall long-K map (mirrored G8)", 3: "map 0, temporal C"}


def one(M, N, K, variant, launches):
    from kgs.ops import experiments, gemm_nt

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    a = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).bfloat16()
    ref = gemm_nt(a, b, variant="w4_oneshot")
    out = torch.empty_like(ref)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    st = torch.zeros((cus, 4, 16), dtype=torch.int64, device=dev)
    for _ in range(3):
        experiments.gemm_w4p_waits(a, b, out, st, variant)
    torch.cuda.synchronize()
    sums = None
    for _ in range(launches):
        st.zero_()
        grid = experiments.gemm_w4p_waits(a, b, out, st, variant)
        torch.cuda.synchronize()
        s = st[:grid].cpu().double()
        sums = s if sums is None else sums + s
    assert torch.equal(out, ref), "the wait-stamp build must compute the production image"
    waves = sums.shape[0] * 4
    ws = sums[:, :, :12].reshape(waves, 3, 4)  # [wave][category][kind]
    total = (sums[:, :, 13] - sums[:, :, 12]).reshape(waves)
    tiles = sums[:, :, 14].reshape(waves)
    ksteps = tiles * (K // 64)
    res = {"shape": [M, N, K], "variant": variant, "what": VARIANTS[variant], "launches": launches,
           "waves": waves, "cycles_per_wave": round(float(total.mean()) / launches, 1),
           "ksteps_per_wave": round(float(ksteps.mean()) / launches, 2)}
    per = {}
    for ci, cname in enumerate(CATS):
        for ki, kname in enumerate(KINDS):
            v = ws[:, ci, ki]
            per[f"{cname}.{kname}"] = {"cycles_per_wave": round(float(v.mean()) / launches, 1),
                                       "share_of_wave_cycles": round(float(v.sum() / total.sum()), 4)}
    res["waits"] = per
    steady_ks = (ksteps - tiles * 4) / launches  # K-steps in the steady category (all but 2 + 2 per tile)
    res["steady_cycles_per_kstep"] = {k: round(float(ws[:, 1, ki].sum() / launches / steady_ks.sum()), 1)
                                      for ki, k in enumerate(KINDS)}
    res["cycles_per_kstep_all"] = round(float(total.sum() / ksteps.sum()), 1)
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--shapes", default="8192,8192x4096x14336,16384x16384x8192")
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    rows = []
    for sh in a.shapes.split(","):
        d = [int(x) for x in sh.split("x")]
        M, N, K = (d * 3)[:3] if len(d) == 1 else d
        tiles = (M // 256) * (N // 256)
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        if M > N and K > 8192:
            variants = [2]
        elif 2 * cus < tiles <= 8 * cus:
            variants = [0, 1]
        else:
            variants = [3]
        for v in variants:
            r = one(M, N, K, v, a.launches)
            rows.append(r)
            print(json.dumps(r), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
