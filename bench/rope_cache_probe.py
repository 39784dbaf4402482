#!/usr/bin/env python3
"""Prompt-pass RoPE + KV write (kgs.ops.decode.rope_cache_) at 16 384 rows,
Llama-3-8B heads: with every cache write, and with the slots at -1 (rotation
only) -- the difference is the cost of the paged K / V writes."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> int:
    from kgs.ops.decode import PAGE, PagedKVCache, rope_cache_
    from kgs.ops.transformer import rope_tables

    dev = torch.device("cuda", 0)
    T, H, HKV = 16384, 32, 8
    qkv = (torch.randn(T, (H + 2 * HKV) * 128, device=dev) * 0.1).bfloat16()
    cos, sin = rope_tables(4096, 128, 500000.0, dev)
    pos = (torch.arange(T, device=dev) % 512).int()
    cache = PagedKVCache(1, T // PAGE + 8, HKV, dev)
    slots = (torch.arange(T, device=dev) + PAGE).int()  # page 0 is the null page
    none = torch.full_like(slots, -1)
    res = {}
    for name, sl in (("writes", slots), ("no_writes", none)):
        for _ in range(3):
            rope_cache_(qkv, cos, sin, pos, sl, cache.layer(0), H, HKV)
        ts = []
        for _ in range(30):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            rope_cache_(qkv, cos, sin, pos, sl, cache.layer(0), H, HKV)
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        res[name] = round(statistics.median(ts), 2)
    print(json.dumps({"rows": T, "us": res}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
