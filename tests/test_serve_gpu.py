"""kgs.serve on the GPU: the kgs backend (skinny GEMM, paged decode attention,
fused RoPE/KV write, flash-attention prefill, hipGraph decode) generates what
the full-recompute oracle of the same weights generates, with and without
graphs, including batches past the skinny-GEMM crossover."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _cfg():
    from kgs.models.llama import LlamaConfig

    return LlamaConfig(hidden=512, intermediate=1024, heads=4, kv_heads=1, layers=2, vocab=1024)


def _engine(graphs, **kw):
    from kgs.serve import EngineConfig, LLMEngine

    ec = EngineConfig(num_pages=256, max_batch=kw.pop("max_batch", 8), max_model_len=1024, cuda_graphs=graphs, **kw)
    return LLMEngine(_cfg(), ec, device="cuda", backend="kgs")


def _oracle_check(eng, prompts, outs, tol=3e-2):
    oracle = eng.model.oracle
    oracle_ref = type(oracle)(oracle.cfg, device="cuda", backend="torch", seed=0)
    for prompt, req in zip(prompts, outs):
        seq = list(prompt)
        for tok in req.output:
            logits = oracle_ref.forward(torch.tensor([seq], device="cuda"))[0, -1].float()
            assert logits[tok] >= logits.max() - tol * logits.abs().max(), (len(seq), tok, int(logits.argmax()))
            seq.append(tok)


@pytest.mark.parametrize("graphs", [False, True])
def test_engine_kgs_matches_oracle(graphs):
    from kgs.serve import SamplingParams

    eng = _engine(graphs)
    rng = np.random.default_rng(0)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (7, 130, 64, 300, 33)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=8, ignore_eos=True))
    assert all(len(r.output) == 8 for r in outs)
    if graphs:
        assert eng.stats["graph_replays"] > 0
    _oracle_check(eng, prompts, outs)


def test_graphs_equal_eager():
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(1)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (40, 90, 12)]
    p = SamplingParams(max_tokens=10, ignore_eos=True)
    a = [r.output for r in _engine(False).generate(prompts, p)]
    b = [r.output for r in _engine(True).generate(prompts, p)]
    assert a == b


def test_large_decode_batch_unfused_path():
    from kgs.serve import SamplingParams

    n = 72  # above fused_max_batch 64: add_rmsnorm / silu_mul + hipBLASLt / skinny routing
    eng = _engine(True, max_batch=128)
    rng = np.random.default_rng(2)
    prompts = [rng.integers(3, 1024, size=20).tolist() for _ in range(n)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=3, ignore_eos=True))
    assert all(len(r.output) == 3 for r in outs)
    _oracle_check(eng, prompts[:4], outs[:4])


def test_fused_and_unfused_decode_agree():
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(3)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (50, 9, 140)]
    p = SamplingParams(max_tokens=12, ignore_eos=True)
    fused = _engine(False, fused_max_batch=64)
    unfused = _engine(False, fused_max_batch=0)
    a = fused.generate(prompts, p)
    b = unfused.generate(prompts, p)
    _oracle_check(fused, prompts, a)
    _oracle_check(unfused, prompts, b)


def test_equal_length_prefill_batched_attention():
    from kgs.serve import SamplingParams

    eng = _engine(True)
    rng = np.random.default_rng(4)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (90, 120, 128, 100)]  # all pad to 128
    outs = eng.generate(prompts, SamplingParams(max_tokens=5, ignore_eos=True))
    _oracle_check(eng, prompts, outs)


def test_fp8_decode_weights_engine():
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(5)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (40, 70)]
    eng = _engine(True, decode_weights="fp8")
    outs = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
    assert all(len(r.output) == 6 for r in outs)
    # weight-only fp8: the chosen tokens stay near the bf16 oracle's top logit
    _oracle_check(eng, prompts, outs, tol=0.12)


def test_fp8_kv_cache_engine():
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(6)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (40, 130)]
    eng = _engine(True, kv_cache_dtype="fp8")
    assert eng.model.cache.fp8
    outs = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
    _oracle_check(eng, prompts, outs, tol=0.12)


@pytest.mark.parametrize("S,ctx,H,HKV", [(128, 128, 32, 8), (256, 384, 4, 1), (128, 1024, 8, 8), (384, 0, 32, 8)])
def test_attention_chunk_matches_reference(S, ctx, H, HKV):
    """Flash attention of a prefill chunk (last S of ctx + S positions) over its
    whole context, strided q (inside fused QKV rows) against fp32 SDPA."""
    from kgs.ops.transformer import attention_chunk, ref_attention_chunk

    g = torch.Generator(device="cuda").manual_seed(S + ctx)
    qkv = torch.randn(S, (H + 2 * HKV) * 128, device="cuda", generator=g).bfloat16()
    k = torch.randn(ctx + S, HKV * 128, device="cuda", generator=g).bfloat16()
    v = torch.randn(ctx + S, HKV * 128, device="cuda", generator=g).bfloat16()
    out = attention_chunk(qkv, k, v, H, HKV)
    ref = ref_attention_chunk(qkv, k, v, H, HKV)
    err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("graphs", [False, True])
def test_chunked_prefill_engine_matches_oracle(graphs):
    """Mixed steps (256-row budget) on the kgs kernels: long prompts split over
    chunks that attend to their cached context (gather + chunk attention),
    decodes in the same steps; generations match the oracle, and the same as
    whole-prompt prefill."""
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(3)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (40, 700, 300, 129, 5)]
    p = SamplingParams(max_tokens=6, ignore_eos=True)
    eng = _engine(graphs, chunked_prefill=256)
    outs = eng.generate(prompts, p)
    assert eng.stats["mixed_steps"] >= 4 and all(len(r.output) == 6 for r in outs)
    _oracle_check(eng, prompts, outs)
    assert eng.sched.check_invariants() == ""


def test_prefix_caching_engine_matches_oracle():
    """Shared 300-token system prompt: later requests reuse its cached pages
    (their first chunk attends to the gathered prefix) and still generate what
    the oracle generates."""
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(11)
    system = rng.integers(3, 1024, size=300).tolist()
    prompts = [system + rng.integers(3, 1024, size=n).tolist() for n in (5, 40, 77, 130)]
    eng = _engine(True, prefix_caching=True, chunked_prefill=512)
    p = SamplingParams(max_tokens=5, ignore_eos=True)
    outs = eng.generate(prompts[:1], p) + eng.generate(prompts[1:], p)
    assert eng.sched.prefix_hit_tokens >= 3 * 256
    _oracle_check(eng, prompts, outs)
    assert eng.sched.check_invariants() == ""


def test_fp8_kv_with_chunked_prefill_and_prefix_caching():
    """fp8 (e4m3) KV pages under chunked prefill + prefix caching: the chunk
    context is gathered from fp8 pages (widened to bf16). Tokens stay close to
    the bf16 engine's (fp8 KV rounding may flip near-ties, so compare the
    oracle with a wider margin)."""
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(13)
    system = rng.integers(3, 1024, size=260).tolist()
    prompts = [system + rng.integers(3, 1024, size=n).tolist() for n in (9, 300)]
    eng = _engine(True, prefix_caching=True, chunked_prefill=256, kv_cache_dtype="fp8")
    p = SamplingParams(max_tokens=4, ignore_eos=True)
    outs = eng.generate(prompts[:1], p) + eng.generate(prompts[1:], p)
    assert eng.sched.prefix_hit_tokens >= 256 and eng.stats["mixed_steps"] >= 2
    _oracle_check(eng, prompts, outs, tol=0.12)


def test_data_parallel_replica_on_gpu():
    """One replica process on cuda:0 (the --data-parallel worker path on a GPU:
    spawn, its own HIP context, hipGraphs) generates what the in-process engine
    generates."""
    import asyncio
    import dataclasses

    from kgs.serve import EngineConfig, SamplingParams
    from kgs.serve.dp import DPEngineLoop

    ec = EngineConfig(num_pages=256, max_batch=8, max_model_len=1024, cuda_graphs=True)
    rng = np.random.default_rng(21)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (30, 200)]
    p = SamplingParams(max_tokens=5, ignore_eos=True)
    runner = DPEngineLoop(1, dataclasses.asdict(_cfg()), ec, device="cuda", backend="kgs", start_timeout=240)
    try:
        async def one(prompt):
            q: asyncio.Queue = asyncio.Queue()
            runner.submit(prompt, p, asyncio.get_running_loop(), q)
            assert (await q.get())[0] == "id"
            out = []
            while True:
                _, t, fin, _, _ = await q.get()
                out.append(t)
                if fin:
                    return out

        async def all_():
            return await asyncio.gather(*(one(pr) for pr in prompts))

        got = asyncio.run(all_())
    finally:
        runner.shutdown()
    ref = _engine(True).generate(prompts, p)
    assert got == [r.output for r in ref]


def test_unpacked_decode_gqa8_engine_matches_oracle():
    """packed_decode=False (one weight copy, the Llama-3-70B layout on one GPU):
    decode on hipBLASLt / split-K GEMMs, GQA 8:1 attention; matches the oracle."""
    from kgs.models.llama import LlamaConfig
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    cfg = LlamaConfig(hidden=1024, intermediate=2048, heads=8, kv_heads=1, layers=2, vocab=1024)
    eng = LLMEngine(cfg, EngineConfig(num_pages=256, max_batch=8, max_model_len=1024, packed_decode=False),
                    device="cuda", backend="kgs")
    assert eng.model.packed is None and eng.model.fused_max_batch == 0
    rng = np.random.default_rng(23)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (20, 150, 300)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=5, ignore_eos=True))
    _oracle_check(eng, prompts, outs)


def test_fp8_prefill_engine():
    """W8A8 prompt pass (prefill_weights='fp8'): generations stay within fp8
    rounding of the bf16 oracle (the decode and the KV writes stay bf16)."""
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(29)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (64, 200)]
    eng = _engine(True, prefill_weights="fp8")
    assert eng.model.prefill_f8 is not None
    outs = eng.generate(prompts, SamplingParams(max_tokens=4, ignore_eos=True))
    _oracle_check(eng, prompts, outs, tol=0.12)


def test_fp8_prefill_with_chunked_prefill():
    """W8A8 projections in mixed (chunk + decode) steps."""
    from kgs.serve import SamplingParams

    rng = np.random.default_rng(31)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (40, 600)]
    eng = _engine(True, prefill_weights="fp8", chunked_prefill=256)
    outs = eng.generate(prompts, SamplingParams(max_tokens=4, ignore_eos=True))
    assert eng.stats["mixed_steps"] >= 3
    _oracle_check(eng, prompts, outs, tol=0.12)


@pytest.mark.parametrize("b", [64, 128, 192, 256])
def test_splitk_fused_decode_llama8b_layer(b):
    """Decode through one Llama-3-8B-shaped layer, where qkv / o / down run
    split-K on the four-wave kernel (and gate|up unsplit): with
    their partials reduced inside RoPE/KV-write and add+RMSNorm and SwiGLU in
    the gate|up epilogue, the KV cache is bit-identical and the logits agree
    with the unfused launches."""
    from kgs.models.llama import LlamaConfig
    from kgs.ops.decode import PAGE
    from kgs.serve.model import ServingModel

    cfg = LlamaConfig(hidden=4096, intermediate=14336, heads=32, kv_heads=8, layers=1, vocab=2048)
    ctx = 40
    outs, caches = [], []
    # (fuse_splitk, rope_attn): the third run folds rope_cache into the attention launch (KGS_ROPE_ATTN=1)
    for fuse, rope_attn in ((False, False), (True, False)) + (((True, True),) if b in (64, 256) else ()):
        torch.manual_seed(0)
        m = ServingModel(cfg, device="cuda", num_pages=b * 2 + 8, max_model_len=256, fuse_splitk=fuse,
                         packed_decode=False)
        m.rope_attn = rope_attn
        assert (m._splitk_route(b, 0, "qkv") is not None) == fuse
        assert (m._swiglu_route(b) is not None) == fuse  # gate|up unsplit on the four-wave kernel at 128 / 256
        bt = torch.arange(b * 2, dtype=torch.int32, device="cuda").view(b, 2)
        g = torch.Generator(device="cuda").manual_seed(1)
        lay = m.cache.layer(0)
        lay.copy_((torch.randn(lay.shape, generator=g, device="cuda") * 0.5).to(lay.dtype))
        tokens = torch.randint(0, cfg.vocab, (b,), generator=g, device="cuda")
        pos = torch.full((b,), ctx - 1, dtype=torch.int32, device="cuda")
        slots = (bt[:, (ctx - 1) // PAGE] * PAGE + (ctx - 1) % PAGE).contiguous()
        ctx_lens = torch.full((b,), ctx, dtype=torch.int32, device="cuda")
        outs.append(m.decode(tokens, pos, slots, bt, ctx_lens).float())
        caches.append(lay.clone())
        torch.cuda.synchronize()
        del m
    for j in range(1, len(outs)):
        assert torch.equal(caches[0], caches[j]), j
        err = ((outs[0] - outs[j]).abs().max() / outs[0].abs().max()).item()
        assert err < 2e-2, (j, err)


def test_batch256_graph_decode_equals_eager_with_the_persistent_lm_head():
    """Regression (round 5, profiles/r5/fault/README.md): at batch 256 the
    Llama-3 LM head (256 x 128256 x 4096, 501 tiles) runs on the persistent
    GEMM inside the decode hipGraph. Its ticket slot was reset by a memset node
    that left garbage behind, so graph-replayed steps could skip LM-head tiles
    (or fault). Graph-replayed and eager decode must give the same tokens, and
    the ticket pool must be clean afterwards."""
    from kgs.models.llama import LlamaConfig
    from kgs.ops._lib import tile_queue_check
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    cfg = LlamaConfig(hidden=4096, intermediate=14336, heads=32, kv_heads=8, layers=1, vocab=128256)
    rng = np.random.default_rng(7)
    prompts = [rng.integers(3, cfg.vocab, size=33).tolist() for _ in range(256)]
    p = SamplingParams(max_tokens=5, ignore_eos=True)
    toks = {}
    for graphs in (False, True):
        eng = LLMEngine(cfg, EngineConfig(num_pages=1024, max_batch=256, max_model_len=256, cuda_graphs=graphs),
                        device="cuda", backend="kgs")
        toks[graphs] = [r.output for r in eng.generate(prompts, p)]
        assert eng.stats["decode_steps"] >= 4 and (eng.stats["graph_replays"] > 0) == graphs
        tq = tile_queue_check()
        assert tq["dirty_slots"] == 0, (graphs, tq)
        del eng
        torch.cuda.empty_cache()
    assert toks[True] == toks[False]


@pytest.mark.parametrize("kw", [{}, {"decode_weights": "fp8"}, {"kv_cache_dtype": "fp8"}], ids=["bf16", "fp8w", "fp8kv"])
def test_serving_graphs_hold_no_memset_node(monkeypatch, kw):
    """a memset node (captured hipMemsetAsync) is what left
    garbage in a ticket slot in round 5. Every decode graph the engine captures
    -- all batch / page-width buckets of warmup(), bf16, fp8 weights, fp8 KV --
    is walked node by node through the HIP graph API (kgs.utils.graph_audit,
    child graphs expanded): no memset node, and the kernels are there. The
    audited graphs then serve: the tokens equal the eager engine's."""
    from kgs.serve import SamplingParams

    monkeypatch.setenv("KGS_GRAPH_AUDIT", "1")
    eng = _engine(True, max_batch=16, **kw)
    assert eng.graph_audit
    eng.warmup()
    assert len(eng.graph_audits) >= 5 * 3, sorted(eng.graph_audits)
    for key, a in eng.graph_audits.items():
        assert a["types"].get("kernel", 0) > 10, (key, a["types"])
        assert a["types"].get("memset", 0) == 0 and not a["memsets"], (key, a["memsets"][:3])
    rng = np.random.default_rng(9)
    prompts = [rng.integers(3, 1024, size=n).tolist() for n in (21, 70, 5)]
    p = SamplingParams(max_tokens=6, ignore_eos=True)
    got = [r.output for r in eng.generate(prompts, p)]
    assert eng.stats["graph_replays"] > 0
    monkeypatch.setenv("KGS_GRAPH_AUDIT", "0")
    assert got == [r.output for r in _engine(False, max_batch=16, **kw).generate(prompts, p)]


def test_batch256_serving_graph_with_the_persistent_lm_head_holds_no_memset_node(monkeypatch):
    """The graph that faulted in round 5 (batch 256, Llama-3 LM head on the
    persistent GEMM, a captured ticket slot): its slot is now zeroed by a kernel
    node, and the graph holds no memset node at all."""
    from kgs.models.llama import LlamaConfig
    from kgs.ops._lib import tile_queue_check, tile_queue_stats
    from kgs.serve import EngineConfig, LLMEngine

    monkeypatch.setenv("KGS_GRAPH_AUDIT", "1")
    cfg = LlamaConfig(hidden=4096, intermediate=14336, heads=32, kv_heads=8, layers=1, vocab=128256)
    eng = LLMEngine(cfg, EngineConfig(num_pages=1024, max_batch=256, max_model_len=256, cuda_graphs=True),
                    device="cuda", backend="kgs")
    st0 = tile_queue_stats()
    eng.warmup(batches=[256], widths=[8])
    assert tile_queue_stats()["capture_slots"] > st0["capture_slots"]  # the LM head is the persistent kernel
    a = eng.graph_audits[(256, 8)]
    assert a["types"].get("memset", 0) == 0 and a["types"]["kernel"] > 10, a["types"]
    assert tile_queue_check()["dirty_slots"] == 0
    del eng
    torch.cuda.empty_cache()


def test_nt_loads_and_gate_up_panels_keep_the_tokens(monkeypatch):
    """Round 5 made non-temporal decode weight loads and the SwiGLU gate|up
    tile-panel copies the default (profiles/r5/decode/README.md). Both only
    change how the weights are read -- the nt bit and the weight layout, not the
    K order of the sums -- so batch 128 and 256 decode (the unsplit SwiGLU routes
    of width 128 and 256) must give the same tokens with either switched off."""
    import kgs.ops.decode as D
    from kgs.models.llama import LlamaConfig
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    cfg = LlamaConfig(hidden=4096, intermediate=14336, heads=32, kv_heads=8, layers=2, vocab=32000)
    rng = np.random.default_rng(11)
    p = SamplingParams(max_tokens=4, ignore_eos=True)
    for nb in (128, 256):
        prompts = [rng.integers(3, cfg.vocab, size=21).tolist() for _ in range(nb)]
        toks = {}
        for nt, panels in ((True, True), (False, True), (True, False)):
            monkeypatch.setattr(D, "NT_WEIGHTS", nt)
            eng = LLMEngine(cfg, EngineConfig(num_pages=512, max_batch=nb, max_model_len=128, gate_up_panels=panels),
                            device="cuda", backend="kgs")
            assert (eng.model.gate_up_panels is not None) == panels
            toks[nt, panels] = [r.output for r in eng.generate(prompts, p)]
            del eng
            torch.cuda.empty_cache()
        assert toks[True, True] == toks[False, True] == toks[True, False], nb


@pytest.mark.parametrize("chunked", [0, 512])
def test_overlapped_steps_equal_sequential_steps_on_graphs(chunked):
    """EngineConfig.overlap on the kgs backend with hipGraph decode at batch
    256 (the serving bench's shape, one layer): step t+1 is replayed with its
    input tokens gathered on the device from step t's samples, before the host
    reads them. Tokens equal one-step-at-a-time execution's, with requests of
    different lengths finishing mid-batch (the batch shrinks and the gather is
    not the identity), and the ticket pool is clean."""
    from kgs.models.llama import LlamaConfig
    from kgs.ops._lib import tile_queue_check
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    cfg = LlamaConfig(hidden=4096, intermediate=14336, heads=32, kv_heads=8, layers=1, vocab=128256)
    rng = np.random.default_rng(13)
    # chunked: mixed steps (prompt chunks beside decode rows, eager) between graph-replayed decodes
    n, lo, hi = (256, 20, 60) if not chunked else (64, 100, 700)
    prompts = [rng.integers(3, cfg.vocab, size=int(rng.integers(lo, hi))).tolist() for _ in range(n)]
    ps = [SamplingParams(max_tokens=int(rng.integers(2, 9)), ignore_eos=True) for _ in range(n)]
    toks = {}
    for ov in (False, True):
        eng = LLMEngine(cfg, EngineConfig(num_pages=2048, max_batch=256, max_model_len=1024, overlap=ov,
                                          chunked_prefill=chunked), device="cuda", backend="kgs")
        assert eng.overlap == ov
        toks[ov] = [r.output for r in eng.generate(prompts, ps)]
        assert eng.stats["graph_replays"] >= (7 if not chunked else 1)
        assert not chunked or eng.stats["mixed_steps"] >= 2
        assert tile_queue_check()["dirty_slots"] == 0
        del eng
        torch.cuda.empty_cache()
    assert toks[True] == toks[False]
    assert [len(t) for t in toks[True]] == [p.max_tokens for p in ps]
