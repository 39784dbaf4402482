#!/usr/bin/env python3
"""Paged decode attention: context splits per sequence vs batch (Llama-3-8B
heads: 32 q / 8 kv x 128, bf16 pages), at a serving-like context. Picks the
split count that the decode_splits() heuristic should produce. One JSON line
per (batch, nsplit) with the median kernel time and the KV bytes / time."""
import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="32,64,128,256")
    ap.add_argument("--ctx", type=int, default=528)
    ap.add_argument("--table-pages", type=int, default=64, help="block-table width (the graph bucket)")
    ap.add_argument("--splits", default="1,2,4,8,16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pipe", default="auto", help="auto | 0 | 1 | both: the two-page register pipeline")
    a = ap.parse_args()
    from kgs.ops.decode import PAGE, PagedKVCache, decode_splits, paged_decode_attention

    dev = torch.device("cuda", 0)
    H, HKV = 32, 8
    for b in [int(x) for x in a.batches.split(",")]:
        tp = a.table_pages
        cache = PagedKVCache(1, b * tp + 8, HKV, dev)
        lay = cache.layer(0)
        lay.copy_((torch.randn(lay.shape, device=dev) * 0.5).to(lay.dtype))
        bt = torch.randperm(b * tp, device=dev).view(b, tp).int().contiguous()
        ctx = torch.full((b,), a.ctx, dtype=torch.int32, device=dev)
        q = (torch.randn(b, H * 128, device=dev)).bfloat16()
        kv_bytes = b * math.ceil(a.ctx / PAGE) * PAGE * HKV * 128 * 2 * 2
        auto = decode_splits(b, HKV, tp)
        pipes = {"auto": [None], "0": [False], "1": [True], "both": [False, True]}[a.pipe]
        for ns, pipe in [(int(x), p) for x in a.splits.split(",") for p in pipes]:
            pps = math.ceil(tp / ns)
            for _ in range(3):
                paged_decode_attention(q, lay, bt, ctx, H, HKV, pages_per_split=pps, pipe=pipe)
            ts = []
            for _ in range(a.iters):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                paged_decode_attention(q, lay, bt, ctx, H, HKV, pages_per_split=pps, pipe=pipe)
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            us = statistics.median(ts)
            print(json.dumps({"batch": b, "nsplit": math.ceil(tp / pps), "pps": pps, "us": round(us, 2),
                              "TBps": round(kv_bytes / us / 1e6, 2), "auto_pps_nsplit": auto, "pipe": pipe}), flush=True)
        del cache, lay
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
