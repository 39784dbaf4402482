"""Uninitialised-memory probe of the serving path.

Fresh device memory holds whatever it held before: on a box that just ran
another process it can be the driver's release poison, on a fresh one zeros.
A kernel that reads memory nobody wrote (an over-read, a missing store, a
counter never reset) therefore behaves differently from run to run -- and if
it turns such a value into an address, it faults only sometimes.

This probe makes that difference deterministic. Before anything else it fills
the PyTorch caching allocator with a chosen 32-bit pattern (one big block the
engine's large allocations are carved from, plus small-pool segments), frees
it back to the cache without releasing it, then builds the serving engine and
runs a short offline generate. Two processes with two patterns (default 0 and
0x00000400: small positive as an index, a subnormal as bf16 -- neither can
turn into a wild address) must produce bitwise-identical tokens, logits
checksum and KV cache; a difference names an uninitialised read. Prints one
JSON line.

  python bench/uninit_probe.py --pattern 0x400 --fill-gb 90 --out gpurun_out/u1.json
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def prefill_cache(pattern: int, fill_gb: float, small_mb: int) -> dict:
    import torch

    dev = torch.device("cuda", 0)
    n = int(fill_gb * (1 << 30)) // 4
    big = torch.full((n,), pattern, dtype=torch.int32, device=dev)
    # small pool (blocks <= 1 MiB live in 2 MiB segments): 512 KiB tensors
    small = [torch.full((128 * 1024,), pattern, dtype=torch.int32, device=dev) for _ in range(small_mb * 2)]
    torch.cuda.synchronize()
    del big, small  # back to the cache, not to the driver
    st = torch.cuda.memory_stats(dev)
    return {"reserved_gb": round(st["reserved_bytes.all.current"] / 2**30, 1)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--pattern", default="0", help="32-bit fill value (int, 0x.. accepted)")
    ap.add_argument("--fill-gb", type=float, default=90.0)
    ap.add_argument("--small-mb", type=int, default=256)
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--input-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=16)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--num-pages", type=int, default=6144)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    pattern = int(a.pattern, 0)

    import numpy as np
    import torch

    t0 = time.perf_counter()
    fill = prefill_cache(pattern, a.fill_gb, a.small_mb)

    from kgs.models.llama import LlamaConfig
    from kgs.serve.bench import _graph_widths, _prompts
    from kgs.serve.engine import EngineConfig, LLMEngine, SamplingParams

    mc = LlamaConfig.named("llama3-8b", a.layers)
    ec = EngineConfig(num_pages=a.num_pages, max_batch=a.max_batch, max_model_len=2048,
                      cuda_graphs=not a.no_graphs)
    eng = LLMEngine(mc, ec, device="cuda", backend="kgs")
    if not a.no_graphs:
        eng.warmup(widths=_graph_widths(a))
    last = {}
    real_sample = eng._sample

    def sample(ids, logits):  # keep a checksum of every step's logits
        lf = logits.float()
        last["logits"] = last.get("logits", 0.0) + float(lf.abs().sum().item())
        last["nan"] = last.get("nan", 0) + int(torch.isnan(lf).sum().item())
        return real_sample(ids, logits)

    eng._sample = sample
    prompts = _prompts(a.requests, a.input_len, mc.vocab, seed=3)
    outs = eng.generate(prompts, SamplingParams(max_tokens=a.output_len, ignore_eos=True))
    torch.cuda.synchronize()
    toks = np.array([r.output for r in outs], dtype=np.int64)
    cache = eng.model.cache.data
    # per-layer sums of the cache's 32-bit words (every page, used or not)
    sums = [int(cache[i].view(torch.int32).sum(dtype=torch.int64).item()) for i in range(cache.shape[0])]
    ck = hashlib.sha256(np.array(sums, dtype=np.int64).tobytes()).hexdigest()
    from kgs.ops._lib import tile_queue_check

    tq = tile_queue_check(0)
    res = {"tile_queue": tq, "pattern": hex(pattern), "fill": fill, "graphs": not a.no_graphs, "requests": a.requests,
           "tokens_sha": hashlib.sha256(toks.tobytes()).hexdigest(), "logits_abs_sum": last.get("logits"),
           "logit_nans": last.get("nan"), "cache_sha": ck, "stats": dict(eng.stats),
           "seconds": round(time.perf_counter() - t0, 1)}
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
