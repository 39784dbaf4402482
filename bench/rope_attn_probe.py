#!/usr/bin/env python3
"""Batch-256 decode attention with its qkv reduce + RoPE + KV write: the two
launches (rope_cache on split-K partials, then paged_decode_attention) against
the fused launch (rope_paged_decode_attention, KGS_ROPE_ATTN=1), and the
attention alone, back to back on one stream. Llama-3-8B heads (32 q / 8 kv x
128), 4 qkv K-slices, contexts of --ctx tokens, scattered pages. Prints one JSON
line per variant (median us over --iters launches). Run under rocprofv3 --pmc
for counters (profiles/r3/decode/README.md)."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=528)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--variants", default="two,fused,attn")
    a = ap.parse_args()
    from kgs.ops.decode import (PAGE, PagedKVCache, paged_decode_attention, rope_cache_,
                                rope_paged_decode_attention)
    from kgs.ops.transformer import rope_tables

    dev = torch.device("cuda", 0)
    b, heads, hkv, hd, nslice = a.batch, 32, 8, 128, 4
    nh = heads + 2 * hkv
    max_pages = (a.ctx + PAGE - 1) // PAGE
    npages = b * max_pages + 8
    bt = torch.randperm(npages, device=dev)[: b * max_pages].int().view(b, max_pages).contiguous()
    ctxs = torch.full((b,), a.ctx, dtype=torch.int32, device=dev)
    last = ctxs.long() - 1
    slots = (bt.gather(1, (last // PAGE).view(-1, 1)).view(-1).long() * PAGE + last % PAGE).int().contiguous()
    pos = last.int().contiguous()
    cos, sin = rope_tables(4096, hd, 500000.0, dev)
    parts = torch.randn(nslice, b, nh * hd, device=dev).contiguous()
    cache = PagedKVCache(1, npages, hkv, dev)
    cache.layer(0).copy_((torch.randn(cache.layer(0).shape, device=dev) * 0.5).bfloat16())
    qkv = torch.empty((b, nh * hd), dtype=torch.bfloat16, device=dev)
    out = torch.empty((b, heads * hd), dtype=torch.bfloat16, device=dev)
    lay = cache.layer(0)

    def two():
        rope_cache_(qkv, cos, sin, pos, slots, lay, heads, hkv, partials=parts)
        paged_decode_attention(qkv, lay, bt, ctxs, heads, hkv, out=out)

    def fused():
        rope_paged_decode_attention(parts, cos, sin, pos, slots, lay, bt, ctxs, heads, hkv, out=out)

    def attn():
        paged_decode_attention(qkv, lay, bt, ctxs, heads, hkv, out=out)

    fns = {"two": two, "fused": fused, "attn": attn}
    for v in a.variants.split(","):
        fn = fns[v]
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        kv_mb = b * a.ctx * hkv * 2 * hd * 2 / 1e6
        print(json.dumps({"variant": v, "batch": b, "ctx": a.ctx, "us": round(statistics.median(ts), 2),
                          "kv_MB": round(kv_mb, 1)}), flush=True)


if __name__ == "__main__":
    main()
