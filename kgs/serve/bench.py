"""Offline serving throughput of :class:`kgs.serve.LLMEngine` (BASELINE config 5
stand-in): N requests of synthetic random-token prompts, fixed output length
(EOS ignored), continuous batching, Llama-3-8B architecture with random-init
bf16 weights on one MI355X. Prints one JSON line.

Optional baseline (``--hf``): the same architecture in HF ``transformers``
(``LlamaForCausalLM``, SDPA attention, eager ``generate`` with static batches)
on the same GPU -- what a PyTorch user gets without a serving engine.

  python -m kgs.serve bench [--requests 256] [--input-len 512] [--output-len 256]
                            [--max-batch 256] [--layers 32] [--hf] [--request-rate R]
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch


def _prompts(n, length, vocab, seed=0, shared=0):
    """n random prompts of `length` tokens; the first `shared` tokens are one
    common prefix (a system prompt) when shared > 0."""
    rng = np.random.default_rng(seed)
    head = rng.integers(3, vocab, size=min(shared, length)).tolist()
    return [head + rng.integers(3, vocab, size=length - len(head)).tolist() for _ in range(n)]


def _graph_widths(a):
    """Page-table width buckets a run with these lengths can hit (captured up front)."""
    widths = sorted({w for w in (8, 16, 32, 64, 128, 256)
                     if w >= (a.input_len + 32) // 32 and w <= 2 * ((a.input_len + a.output_len) // 32 + 1)})
    return widths or None


def run_engine(a) -> dict:
    from kgs.models.llama import LlamaConfig

    from .engine import EngineConfig, LLMEngine, SamplingParams

    mc = LlamaConfig.named(a.model, a.layers)
    ec = EngineConfig(max_batch=a.max_batch, max_model_len=a.max_model_len, cuda_graphs=not a.no_graphs,
                      max_prefill_tokens=a.max_prefill_tokens, fused_max_batch=a.fused_max_batch,
                      decode_weights=a.decode_weights, kv_cache_dtype=a.kv_cache_dtype,
                      chunked_prefill=a.chunked_prefill, prefix_caching=a.prefix_caching,
                      packed_decode=not a.no_packed_decode, prefill_weights=a.prefill_weights,
                      fuse_splitk=not a.no_fuse_splitk, w4x_panels=not a.no_w4x_panels,
                      gate_up_panels=not a.no_gate_up_panels, overlap=a.overlap != "off")
    t0 = time.perf_counter()
    eng = LLMEngine(mc, ec, device="cuda", backend="kgs")
    t_load = time.perf_counter() - t0
    t0 = time.perf_counter()
    if not a.no_graphs:
        eng.warmup(widths=_graph_widths(a))
    # one short request end to end (prefill + decode paths compiled/allocated)
    eng.generate(_prompts(1, 16, mc.vocab, seed=9), SamplingParams(max_tokens=4, ignore_eos=True))
    torch.cuda.synchronize()
    t_warm = time.perf_counter() - t0
    prompts = _prompts(a.requests, a.input_len, mc.vocab, shared=a.shared_prefix)
    params = SamplingParams(max_tokens=a.output_len, ignore_eos=True)
    if a.gc_freeze:
        import gc

        gc.collect()
        gc.freeze()  # the engine's long-lived objects leave the collector's scans
    for k in eng.stats:
        eng.stats[k] = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = eng.generate(prompts, params)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_out = sum(len(r.output) for r in outs)
    n_in = a.requests * a.input_len
    from kgs.ops._lib import tile_queue_check
    from kgs.ops.decode import NT_WEIGHTS

    tq = tile_queue_check(0)  # the persistent GEMMs' ticket pool must be all zero again
    if os.environ.get("KGS_HOST_PHASES_OUT"):
        with open(os.environ["KGS_HOST_PHASES_OUT"], "w") as f:
            json.dump(eng.host_phases(), f)
    ttft = sorted(r.t_first - r.t_arrival for r in outs)
    tpot = sorted((r.t_done - r.t_first) / max(1, len(r.output) - 1) for r in outs)
    return {
        "metric": f"offline serving throughput (kgs.serve, {a.model} arch, random init)", "model": a.model,
        "backend": "kgs", "requests": a.requests, "input_len": a.input_len, "output_len": a.output_len,
        "max_batch": a.max_batch, "layers": a.layers, "num_pages": eng.num_pages, "cuda_graphs": not a.no_graphs,
        "fused_max_batch": a.fused_max_batch, "decode_weights": a.decode_weights,
        "kv_cache_dtype": a.kv_cache_dtype, "prefill_weights": a.prefill_weights,
        "fuse_splitk": not a.no_fuse_splitk, "w4x_panels": not a.no_w4x_panels,
        "gate_up_panels": eng.model.gate_up_panels is not None, "overlap": eng.overlap,
        "nt_weights": NT_WEIGHTS,
        "chunked_prefill": a.chunked_prefill,
        "prefix_caching": a.prefix_caching, "shared_prefix": a.shared_prefix,
        "prefix_hit_tokens": int(eng.sched.prefix_hit_tokens),
        "seconds": round(dt, 3), "output_tok_per_s": round(n_out / dt, 1),
        "total_tok_per_s": round((n_out + n_in) / dt, 1), "requests_per_s": round(a.requests / dt, 3),
        "ttft_p50_ms": round(1e3 * ttft[len(ttft) // 2], 1), "tpot_p50_ms": round(1e3 * tpot[len(tpot) // 2], 2),
        "load_s": round(t_load, 1), "warmup_s": round(t_warm, 1), "stats": dict(eng.stats),
        "tile_queue_dirty_slots": tq["dirty_slots"],
    }


def _pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else float("nan")


def run_online(a, mc=None, device="cuda", backend="kgs") -> dict:
    """Online serving: requests arrive as a Poisson process at --request-rate
    req/s (the arrival schedule is drawn up front, seeded), the engine runs
    continuously and admits each request once its arrival time has passed.
    Latencies are measured from the scheduled arrival: TTFT, TPOT (per request,
    (t_done - t_first) / (tokens - 1)), ITL (every gap between two tokens of a
    request) and end-to-end latency, p50/p99 -- the metrics of vLLM's
    benchmark_serving, without the HTTP hop."""
    from kgs.models.llama import LlamaConfig

    from .engine import EngineConfig, LLMEngine, SamplingParams

    mc = mc or LlamaConfig.named(getattr(a, "model", "llama3-8b"), a.layers)
    ec = EngineConfig(max_batch=a.max_batch, max_model_len=a.max_model_len, cuda_graphs=not a.no_graphs,
                      max_prefill_tokens=a.max_prefill_tokens, fused_max_batch=a.fused_max_batch,
                      decode_weights=a.decode_weights, kv_cache_dtype=a.kv_cache_dtype,
                      chunked_prefill=getattr(a, "chunked_prefill", 0),
                      prefix_caching=getattr(a, "prefix_caching", False),
                      packed_decode=not getattr(a, "no_packed_decode", False),
                      overlap=getattr(a, "overlap", "auto") == "on",  # auto: off (TTFT, see --overlap)
                      **({"num_pages": 256} if device == "cpu" else {}))
    eng = LLMEngine(mc, ec, device=device, backend=backend)
    if not a.no_graphs:
        eng.warmup(widths=_graph_widths(a))
    eng.generate(_prompts(1, 16, mc.vocab, seed=9), SamplingParams(max_tokens=4, ignore_eos=True))
    if device != "cpu":
        torch.cuda.synchronize()
    rng = np.random.default_rng(1)
    arrivals = np.cumsum(rng.exponential(1.0 / a.request_rate, size=a.requests))
    prompts = _prompts(a.requests, a.input_len, mc.vocab, shared=getattr(a, "shared_prefix", 0))
    params = SamplingParams(max_tokens=a.output_len, ignore_eos=True)
    tok_times: dict = {}
    done = []
    t0 = time.perf_counter()
    i = 0
    while i < a.requests or eng.has_work():
        now = time.perf_counter() - t0
        while i < a.requests and arrivals[i] <= now:
            rid = eng.add_request(prompts[i], params)
            eng.requests[rid].t_arrival = t0 + arrivals[i]
            tok_times[rid] = []
            i += 1
        if not eng.has_work():
            time.sleep(max(0.0, min(0.01, arrivals[i] - now)))
            continue
        for rid, _tok, fin in eng.step():
            tok_times[rid].append(time.perf_counter())
            if fin:
                done.append(eng.requests.pop(rid))
    dt = time.perf_counter() - t0
    ttft = [r.t_first - r.t_arrival for r in done]
    tpot = [(r.t_done - r.t_first) / max(1, len(r.output) - 1) for r in done]
    e2e = [r.t_done - r.t_arrival for r in done]
    itl = [b - c for ts in tok_times.values() for c, b in zip(ts, ts[1:])]
    n_out = sum(len(r.output) for r in done)
    ms = lambda v: round(1e3 * v, 2)  # noqa: E731
    return {
        "metric": "online serving (kgs.serve, Poisson arrivals, Llama-3-8B arch, random init)",
        "backend": "kgs", "requests": a.requests, "request_rate": a.request_rate, "input_len": a.input_len,
        "output_len": a.output_len, "max_batch": a.max_batch, "layers": a.layers,
        "chunked_prefill": getattr(a, "chunked_prefill", 0), "prefix_caching": getattr(a, "prefix_caching", False),
        "shared_prefix": getattr(a, "shared_prefix", 0), "prefix_hit_tokens": int(eng.sched.prefix_hit_tokens),
        "seconds": round(dt, 3), "output_tok_per_s": round(n_out / dt, 1),
        "requests_per_s": round(len(done) / dt, 3),
        "ttft_ms": {"p50": ms(_pct(ttft, .5)), "p99": ms(_pct(ttft, .99)), "mean": ms(float(np.mean(ttft)))},
        "tpot_ms": {"p50": ms(_pct(tpot, .5)), "p99": ms(_pct(tpot, .99)), "mean": ms(float(np.mean(tpot)))},
        "itl_ms": {"p50": ms(_pct(itl, .5)), "p99": ms(_pct(itl, .99))},
        "e2e_ms": {"p50": ms(_pct(e2e, .5)), "p99": ms(_pct(e2e, .99))},
        "stats": dict(eng.stats),
    }


def run_hf(a) -> dict:
    """HF transformers eager generate, static batches of max_batch, same shapes."""
    import transformers

    cfg = transformers.LlamaConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336,
                                   num_hidden_layers=a.layers, num_attention_heads=32, num_key_value_heads=8,
                                   max_position_embeddings=8192, rope_theta=500000.0, rms_norm_eps=1e-5,
                                   torch_dtype="bfloat16", attn_implementation="sdpa")
    torch.set_default_dtype(torch.bfloat16)
    with torch.device("cuda"):
        model = transformers.LlamaForCausalLM(cfg)
    torch.set_default_dtype(torch.float32)
    model.eval()
    prompts = torch.tensor(_prompts(a.requests, a.input_len, 128256), device="cuda")
    bs = min(a.max_batch, a.requests)
    gen = dict(max_new_tokens=a.output_len, min_new_tokens=a.output_len, do_sample=False, pad_token_id=0)
    with torch.no_grad():
        model.generate(prompts[:1, :16], max_new_tokens=2, do_sample=False, pad_token_id=0)  # warm up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_out = 0
        for i in range(0, a.requests, bs):
            out = model.generate(prompts[i:i + bs], attention_mask=torch.ones_like(prompts[i:i + bs]), **gen)
            n_out += (out.shape[1] - a.input_len) * out.shape[0]
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    return {"metric": "offline generation throughput (HF transformers eager generate, same arch)",
            "backend": f"hf-transformers-{transformers.__version__}", "requests": a.requests,
            "input_len": a.input_len, "output_len": a.output_len, "batch": bs, "layers": a.layers,
            "seconds": round(dt, 3), "output_tok_per_s": round(n_out / dt, 1),
            "total_tok_per_s": round((n_out + a.requests * a.input_len) / dt, 1)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m kgs.serve bench", description=__doc__.splitlines()[0])
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--input-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--max-prefill-tokens", type=int, default=16384)
    ap.add_argument("--model", choices=("llama3-8b", "llama3-70b"), default="llama3-8b")
    ap.add_argument("--layers", type=int, default=None, help="default: the model's (32 / 80)")
    ap.add_argument("--no-packed-decode", action="store_true",
                    help="one weight copy: decode on hipBLASLt / split-K (needed for llama3-70b on one GPU)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-fuse-splitk", action="store_true",
                    help="reduce split-K decode projections in their own launch (A/B against the fused consumers)")
    ap.add_argument("--no-w4x-panels", action="store_true",
                    help="split-K decode projections read the row-major weights (A/B against the panel copies)")
    ap.add_argument("--gc-freeze", action="store_true",
                    help="gc.collect() + gc.freeze() after warm-up (A/B: collector pauses in the step loop)")
    ap.add_argument("--overlap", choices=("auto", "on", "off"), default="auto",
                    help="plan and launch step t+1 before step t's tokens are read back (EngineConfig.overlap). "
                         "auto: on offline, off online -- online it trades TTFT for TPOT (32 req/s: TTFT p50 "
                         "+4 ms, TPOT -7 %%; profiles/r5/overlap/README.md)")
    ap.add_argument("--no-gate-up-panels", action="store_true",
                    help="unsplit SwiGLU decode routes read the row-major gate|up (A/B against the panel copies)")
    ap.add_argument("--fused-max-batch", type=int, default=48,
                    help="decode batches up to this run the fused skinny-GEMM layer (0 = never)")
    ap.add_argument("--decode-weights", choices=("bf16", "fp8"), default="bf16",
                    help="fp8 = weight-only fp8 decode GEMMs (W8A16); the headline is bf16")
    ap.add_argument("--prefill-weights", choices=("bf16", "fp8"), default="bf16",
                    help="fp8 = W8A8 prompt pass (e4m3 weights, per-row activation scales); the headline is bf16")
    ap.add_argument("--kv-cache-dtype", choices=("bf16", "fp8"), default="bf16",
                    help="fp8 = e4m3 KV pages (half the attention bytes); the headline is bf16")
    ap.add_argument("--chunked-prefill", type=int, default=0,
                    help="> 0: mixed steps of at most this many rows (prompt chunks + decodes)")
    ap.add_argument("--prefix-caching", action="store_true", help="reuse cached pages of shared prompt prefixes")
    ap.add_argument("--shared-prefix", type=int, default=0,
                    help="the first N prompt tokens are common to every request (a system prompt)")
    ap.add_argument("--request-rate", type=float, default=0.0,
                    help="> 0: online mode, Poisson arrivals at this many requests/s (TTFT/TPOT/ITL p50/p99)")
    ap.add_argument("--hf", action="store_true", help="also run the HF transformers baseline")
    ap.add_argument("--hf-only", action="store_true")
    a = ap.parse_args(argv)
    if a.layers is None:
        a.layers = 80 if a.model == "llama3-70b" else 32
    if a.model == "llama3-70b" and not a.no_packed_decode and a.decode_weights == "bf16":
        a.no_packed_decode = True  # two bf16 copies of 70B (282 GB) leave no room for the KV cache
    if a.request_rate > 0:
        print(json.dumps(run_online(a)), flush=True)
        return 0
    if not a.hf_only:
        print(json.dumps(run_engine(a)), flush=True)
        torch.cuda.empty_cache()
    if a.hf or a.hf_only:
        print(json.dumps(run_hf(a)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
