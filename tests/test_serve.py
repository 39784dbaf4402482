"""kgs.serve on CPU: the native scheduler's bookkeeping (admission, paging,
preemption, invariants under random traffic) and the engine's paged-KV
generation through the plain-PyTorch reference backend, checked token by token
against a full-recompute forward of the same weights."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
_serve = pytest.importorskip("kgs._native._serve")

from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


def _sched(num_pages=64, max_batch=8, max_model_len=512, max_prefill=1024, chunk_tokens=0):
    c = _serve.SchedulerConfig()
    c.num_pages, c.page_size, c.max_batch = num_pages, 32, max_batch
    c.max_prefill_tokens, c.max_model_len, c.pad_multiple = max_prefill, max_model_len, 128
    c.chunk_tokens = chunk_tokens
    return _serve.Scheduler(c)


def test_allocator_reserves_null_page():
    a = _serve.BlockAllocator(4)
    got = {a.alloc() for _ in range(3)}
    assert got == {1, 2, 3} and a.alloc() == -1
    a.free(0)  # the null page is never freed into the pool
    a.free(2)
    a.free(2)  # double free ignored
    assert a.num_free == 1 and a.alloc() == 2


def test_prefill_then_decode_plan():
    s = _sched()
    assert s.add(10, np.arange(1, 41, dtype=np.int32), 5)
    assert s.add(11, np.arange(1, 71, dtype=np.int32), 5)
    p = s.schedule()
    assert p.kind == 1 and list(p.seq_ids) == [10, 11]
    assert list(p.seq_lens) == [40, 70] and list(p.padded_lens) == [128, 128]
    assert list(p.seq_starts) == [0, 128]
    slots = p.slots
    assert (slots[40:128] == -1).all() and (slots[128 + 70:] == -1).all()
    real = np.concatenate([slots[:40], slots[128:198]])
    assert len(set(real.tolist())) == 110 and (real >= 32).all()  # page 0 never used
    s.update(p.seq_ids, np.array([7, 8], np.int32), np.zeros(2, np.uint8))
    d = s.schedule()
    assert d.kind == 2 and list(d.tokens) == [7, 8]
    assert list(d.positions) == [40, 70] and list(d.ctx_lens) == [41, 71]
    bt = d.block_tables
    assert bt.shape == (2, d.max_pages)
    for row, slot, pos in zip(bt, d.slots, d.positions):
        assert slot == row[pos // 32] * 32 + pos % 32
    assert s.check_invariants() == ""


def test_finish_frees_pages():
    s = _sched(num_pages=16)
    free0 = s.num_free_pages
    s.add(1, np.ones(33, np.int32), 2)
    p = s.schedule()
    s.update(p.seq_ids, np.array([3], np.int32), np.zeros(1, np.uint8))
    p = s.schedule()
    done = s.update(p.seq_ids, np.array([4], np.int32), np.zeros(1, np.uint8))
    assert list(done) == [1] and s.num_free_pages == free0
    assert list(s.tokens(1)[-2:]) == [3, 4]
    s.release(1)
    with pytest.raises(KeyError):
        s.tokens(1)


def test_eos_and_abort():
    s = _sched()
    s.add(1, np.ones(5, np.int32), 100)
    s.add(2, np.ones(5, np.int32), 100)
    p = s.schedule()
    done = s.update(p.seq_ids, np.array([9, 9], np.int32), np.array([1, 0], np.uint8))
    assert list(done) == [1]
    assert s.abort(2) and not s.abort(2)
    assert s.num_running == 0 and s.check_invariants() == ""


def test_rejects_impossible_requests():
    s = _sched(num_pages=4, max_model_len=512)
    assert not s.add(1, np.ones(600, np.int32), 1)      # longer than max_model_len
    assert not s.add(2, np.ones(200, np.int32), 10)     # needs more pages than the cache has
    assert not s.add(3, np.zeros(0, np.int32), 1)
    assert s.add(4, np.ones(10, np.int32), 1) and not s.add(4, np.ones(10, np.int32), 1)  # duplicate id


def test_preemption_recomputes_newest():
    # 7 usable pages: two sequences of 3 pages each (+1% watermark), both growing past a page boundary
    s = _sched(num_pages=8, max_model_len=512)
    assert s.add(1, np.ones(64, np.int32), 120)
    assert s.add(2, np.ones(64, np.int32), 120)
    p = s.schedule()
    assert p.kind == 1 and len(p.seq_ids) == 2
    tok = 5
    preempted = []
    for _ in range(400):
        s.update(p.seq_ids, np.full(len(p.seq_ids), tok, np.int32), np.zeros(len(p.seq_ids), np.uint8))
        p = s.schedule()
        preempted += list(p.preempted)
        assert s.check_invariants() == ""
        if p.kind == 0:
            break
    assert 2 in preempted  # the newest admitted sequence yields its pages
    assert s.info(2)["preemptions"] >= 1


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(1, 300), st.integers(1, 60), st.booleans()), min_size=1, max_size=25),
       st.integers(8, 40), st.integers(1, 6), st.sampled_from([0, 0, 128, 256, 512]))
def test_random_traffic_invariants(reqs, pages, max_batch, chunk):
    """Random traffic through both scheduling modes (whole-prompt prefill and
    chunked prefill): invariants hold every step, every request finishes, no
    page leaks."""
    s = _sched(num_pages=pages, max_batch=max_batch, max_model_len=512, chunk_tokens=chunk)
    live = set()
    for i, (plen, new, _) in enumerate(reqs):
        if s.add(i, np.full(plen, 3, np.int32), new):
            live.add(i)
    rng = np.random.default_rng(0)
    for _ in range(2000):
        p = s.schedule()
        assert s.check_invariants() == "", s.check_invariants()
        if p.kind == 0:
            break
        ids = p.seq_ids
        if p.kind == 3:  # only completed prompts and decodes sample
            ids = np.concatenate([ids[:p.n_prefill][p.last_chunk.astype(bool)], ids[p.n_prefill:]])
        n = len(ids)
        eos = (rng.random(n) < 0.05).astype(np.uint8)
        for d in s.update(ids, np.full(n, 4, np.int32), eos):
            live.discard(int(d))
        if p.kind == 2:
            assert (p.ctx_lens == p.positions + 1).all()
    assert not live and s.num_running == 0 and s.num_waiting == 0
    assert s.num_free_pages == pages - 1


# ---------------------------------------------------------------- engine (ref backend)

def _tiny():
    from kgs.models.llama import LlamaConfig

    return LlamaConfig(hidden=256, intermediate=512, heads=2, kv_heads=1, layers=2, vocab=512)


def _check_against_oracle(eng, prompts, outs):
    oracle = eng.model.oracle
    for prompt, req in zip(prompts, outs):
        seq = list(prompt)
        for tok in req.output:
            logits = oracle.forward(torch.tensor([seq]))[0, -1].float()
            # the engine's token is the oracle's argmax up to bf16 rounding noise
            assert logits[tok] >= logits.max() - 2e-2 * logits.abs().max(), (len(seq), tok, int(logits.argmax()))
            seq.append(tok)


def test_engine_ref_matches_full_recompute():
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=64, max_batch=4, max_model_len=512, cuda_graphs=False),
                    device="cpu", backend="ref")
    rng = np.random.default_rng(1)
    prompts = [rng.integers(3, 512, size=n).tolist() for n in (5, 33, 64, 100, 17)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
    assert all(len(r.output) == 6 and r.finish_reason == "length" for r in outs)
    assert eng.stats["prefill_steps"] >= 2 and eng.stats["decode_steps"] >= 5  # max_batch 4 < 5 prompts
    _check_against_oracle(eng, prompts, outs)


def test_engine_ref_chunked_prefill_matches_full_recompute():
    """Chunked prefill (mixed steps, 256-row budget): long prompts split over
    steps and attend to their own cached chunks; decodes of shorter sequences run
    in the same steps. Generations equal the full-recompute oracle's."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=96, max_batch=4, max_model_len=1024, cuda_graphs=False,
                                          chunked_prefill=256), device="cpu", backend="ref")
    rng = np.random.default_rng(5)
    prompts = [rng.integers(3, 512, size=n).tolist() for n in (40, 700, 300, 129, 5)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=5, ignore_eos=True))
    assert all(len(r.output) == 5 for r in outs)
    assert eng.stats["mixed_steps"] >= 4  # the 700-token prompt alone needs 3 chunks
    assert eng.stats["prefill_tokens"] == sum(len(p) for p in prompts)
    _check_against_oracle(eng, prompts, outs)
    assert eng.sched.check_invariants() == ""


def test_scheduler_chunked_plans():
    """Mixed plans: decode rows after the chunks, non-final chunks whole
    q-blocks, ctx_starts advancing, every prompt token scheduled exactly once."""
    from kgs._native import _serve

    cfg = _serve.SchedulerConfig()
    cfg.num_pages, cfg.page_size, cfg.max_batch, cfg.max_model_len, cfg.pad_multiple = 200, 32, 8, 2048, 128
    cfg.chunk_tokens = 384
    s = _serve.Scheduler(cfg)
    assert s.add(1, list(range(3, 1003)), 4) and s.add(2, [5, 6, 7], 4)
    seen = {1: 0, 2: 0}
    kinds = []
    for _ in range(12):
        p = s.schedule()
        if p.kind == 0:
            break
        kinds.append(p.kind)
        assert s.check_invariants() == ""
        npf = p.n_prefill if p.kind == 3 else 0
        ids = list(p.seq_ids)
        for j in range(npf):
            assert p.ctx_starts[j] == seen[ids[j]] and p.ctx_starts[j] % 128 == 0
            if not p.last_chunk[j]:
                assert p.seq_lens[j] % 128 == 0
            seen[ids[j]] += int(p.seq_lens[j])
        assert len(p.tokens) == sum(p.padded_lens[:npf]) + len(ids) - npf if p.kind == 3 else True
        assert sum(p.padded_lens[:npf]) + len(ids) - npf <= 384 + 128
        sampled = [ids[j] for j in range(npf) if p.last_chunk[j]] + ids[npf:]
        s.update(np.array(sampled, dtype=np.int64), np.full(len(sampled), 9, dtype=np.int32),
                 np.zeros(len(sampled), dtype=np.uint8))
    assert seen == {1: 1000, 2: 3}
    assert 3 in kinds and 2 in kinds  # mixed steps while prompt 1 prefills, then plain decode plans


def test_scheduler_prefix_caching_shares_pages():
    from kgs._native import _serve

    c = _serve.SchedulerConfig()
    c.num_pages, c.page_size, c.max_batch, c.max_model_len, c.pad_multiple = 64, 32, 8, 1024, 128
    c.max_prefill_tokens, c.prefix_caching = 1024, True
    s = _serve.Scheduler(c)
    shared = list(range(10, 10 + 200))  # 6 full pages
    assert s.add(1, shared + [7, 8, 9], 3)
    p = s.schedule()
    assert p.kind == 3 and list(p.ctx_starts) == [0]
    s.update(np.array([1]), np.array([5], np.int32), np.zeros(1, np.uint8))
    assert s.num_cached_pages == 6
    # same 200-token prefix: its 6 full pages are cached and reused (an even
    # count: the chunk context must be a multiple of 64 keys), the rest computed
    assert s.add(2, shared + [1, 2], 3)
    p = s.schedule()
    assert list(p.seq_ids[:p.n_prefill]) == [2] and p.ctx_starts[0] == 192 and p.seq_lens[0] == 202 - 192
    assert s.prefix_hit_tokens == 192 and s.check_invariants() == ""
    bt1, bt2 = s.info(1), s.info(2)
    assert bt1["pages"] >= 7 and bt2["pages"] == 7
    # finishing both releases the shared pages into the evictable cache, no leak
    for _ in range(10):
        p = s.schedule()
        if p.kind == 0:
            break
        ids = p.seq_ids
        if p.kind == 3:
            ids = np.concatenate([ids[:p.n_prefill][p.last_chunk.astype(bool)], ids[p.n_prefill:]])
        s.update(ids, np.full(len(ids), 4, np.int32), np.zeros(len(ids), np.uint8))
        assert s.check_invariants() == ""
    assert s.num_running == 0 and s.num_free_pages == 63 and s.num_cached_pages >= 6
    # eviction: a large prompt reclaims cached pages
    assert s.add(3, list(range(600, 600 + 1000)), 2)
    s.schedule()
    assert s.check_invariants() == ""


def test_prefix_caching_reuses_generated_pages():
    """Multi-turn: the second prompt = first prompt + first answer + more; pages
    filled during decode are registered, so the match extends past the first
    prompt into the generated tokens."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=64, max_batch=2, max_model_len=1024, cuda_graphs=False,
                                          prefix_caching=True, chunked_prefill=256), device="cpu", backend="ref")
    rng = np.random.default_rng(9)
    turn1 = rng.integers(3, 512, size=100).tolist()
    r1 = eng.generate([turn1], SamplingParams(max_tokens=60, ignore_eos=True))[0]
    turn2 = turn1 + r1.output + rng.integers(3, 512, size=20).tolist()  # 180 tokens
    before = eng.sched.prefix_hit_tokens
    r2 = eng.generate([turn2], SamplingParams(max_tokens=4, ignore_eos=True))[0]
    # 5 full pages (160 tokens) of turn 2 are cached, 128 of them reused (even page count);
    # turn 1's prompt alone covers only 3 full pages
    assert eng.sched.prefix_hit_tokens - before == 128
    _check_against_oracle(eng, [turn2], [r2])


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 2), st.integers(1, 200), st.integers(1, 40)), min_size=1, max_size=20),
       st.integers(12, 48), st.integers(1, 6), st.sampled_from([128, 256, 0]))
def test_prefix_caching_random_traffic(reqs, pages, max_batch, chunk):
    """Prompts built on three shared prefixes, random lengths, EOS and cache
    pressure: refcounts match the owners every step, all requests finish, every
    page is free or evictable at the end."""
    c = _serve.SchedulerConfig()
    c.num_pages, c.page_size, c.max_batch, c.max_model_len, c.pad_multiple = pages, 32, max_batch, 512, 128
    c.max_prefill_tokens, c.chunk_tokens, c.prefix_caching = 1024, chunk, True
    s = _serve.Scheduler(c)
    prefixes = [list(range(100 + 300 * k, 100 + 300 * k + 160)) for k in range(3)]
    live = set()
    for i, (k, extra, new) in enumerate(reqs):
        if s.add(i, prefixes[k] + [3] * extra, new):
            live.add(i)
    rng = np.random.default_rng(0)
    for _ in range(3000):
        p = s.schedule()
        assert s.check_invariants() == "", s.check_invariants()
        if p.kind == 0:
            break
        ids = p.seq_ids
        if p.kind == 3:
            ids = np.concatenate([ids[:p.n_prefill][p.last_chunk.astype(bool)], ids[p.n_prefill:]])
        eos = (rng.random(len(ids)) < 0.05).astype(np.uint8)
        for d in s.update(ids, np.full(len(ids), 4, np.int32), eos):
            live.discard(int(d))
    assert not live and s.num_running == 0 and s.num_free_pages == pages - 1


def test_engine_ref_prefix_caching_matches_full_recompute():
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=96, max_batch=4, max_model_len=1024, cuda_graphs=False,
                                          prefix_caching=True, chunked_prefill=256), device="cpu", backend="ref")
    rng = np.random.default_rng(7)
    system = rng.integers(3, 512, size=300).tolist()
    prompts = [system + rng.integers(3, 512, size=n).tolist() for n in (5, 40, 77)]
    first = eng.generate(prompts[:1], SamplingParams(max_tokens=4, ignore_eos=True))
    rest = eng.generate(prompts[1:], SamplingParams(max_tokens=4, ignore_eos=True))
    assert eng.sched.prefix_hit_tokens >= 2 * 256
    _check_against_oracle(eng, prompts, first + rest)


def test_engine_ref_preemption_is_transparent():
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    # 5 usable pages for 3 sequences that grow across page boundaries: forces preemption + recompute
    eng = LLMEngine(_tiny(), EngineConfig(num_pages=6, max_batch=3, max_model_len=256, cuda_graphs=False),
                    device="cpu", backend="ref")
    rng = np.random.default_rng(2)
    prompts = [rng.integers(3, 512, size=n).tolist() for n in (30, 28, 31)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=12, ignore_eos=True))
    assert eng.stats["preemptions"] >= 1
    _check_against_oracle(eng, prompts, outs)


def test_engine_sampling_and_eos():
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False,
                                          eos_token_id=-1), device="cpu", backend="ref")
    outs = eng.generate([[5, 6, 7], [8, 9]], [SamplingParams(max_tokens=4, temperature=1.0, top_k=5),
                                              SamplingParams(max_tokens=3)])
    assert len(outs[0].output) == 4 and len(outs[1].output) == 3
    first = outs[1].output[0]
    eng2 = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False,
                                           eos_token_id=first), device="cpu", backend="ref")
    r = eng2.generate([[8, 9]], SamplingParams(max_tokens=3))[0]
    assert r.output == [first] and r.finish_reason == "stop"


def test_http_api_completions_and_stream():
    from fastapi.testclient import TestClient

    from kgs.serve import EngineConfig, LLMEngine
    from kgs.serve.api import ByteTokenizer, EngineLoop, create_app

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False),
                    device="cpu", backend="ref")
    runner = EngineLoop(eng)
    try:
        client = TestClient(create_app(runner, model_name="tiny"))
        assert client.get("/health").json() == {"status": "ok"}
        assert client.get("/v1/models").json()["data"][0]["id"] == "tiny"
        r = client.post("/v1/completions", json={"prompt": "hello", "max_tokens": 5, "ignore_eos": True}).json()
        ch = r["choices"][0]
        assert len(ch["token_ids"]) == 5 and ch["finish_reason"] == "length"
        assert r["usage"] == {"prompt_tokens": 6, "completion_tokens": 5, "total_tokens": 11}
        # same prompt as token ids gives the same greedy continuation
        r2 = client.post("/v1/completions", json={"prompt": ByteTokenizer().encode("hello"), "max_tokens": 5,
                                                  "ignore_eos": True}).json()
        assert r2["choices"][0]["token_ids"] == ch["token_ids"]
        with client.stream("POST", "/v1/completions",
                           json={"prompt": [5, 6, 7], "max_tokens": 4, "stream": True, "ignore_eos": True}) as s:
            events = [ln for ln in s.iter_lines() if ln.startswith("data: ")]
        assert events[-1] == "data: [DONE]" and len(events) == 5
        bad = client.post("/v1/completions", json={"prompt": [3] * 300, "max_tokens": 4})
        assert bad.status_code == 400
        m = client.get("/metrics").text
        assert "kgs_requests_total 3" in m and "kgs_requests_rejected_total 1" in m
    finally:
        runner.shutdown()


def test_http_api_chat_stop_strings_and_top_p():
    from fastapi.testclient import TestClient

    from kgs.serve import EngineConfig, LLMEngine
    from kgs.serve.api import EngineLoop, create_app, render_chat

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False),
                    device="cpu", backend="ref")
    runner = EngineLoop(eng)
    try:
        client = TestClient(create_app(runner, model_name="tiny"))
        msgs = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "hi"}]
        r = client.post("/v1/chat/completions", json={"messages": msgs, "max_tokens": 6, "ignore_eos": True}).json()
        assert r["object"] == "chat.completion"
        msg = r["choices"][0]["message"]
        assert msg["role"] == "assistant" and r["usage"]["completion_tokens"] == 6
        # the chat endpoint is the completion of the rendered transcript
        from types import SimpleNamespace as NS
        prompt = render_chat([NS(**m) for m in msgs])
        c = client.post("/v1/completions", json={"prompt": prompt, "max_tokens": 6, "ignore_eos": True}).json()
        assert c["choices"][0]["text"] == msg["content"]
        # a stop token id ends generation at its first occurrence (greedy: deterministic)
        ids = c["choices"][0]["token_ids"]
        r3 = client.post("/v1/completions", json={"prompt": prompt, "max_tokens": 6, "stop_token_ids": [ids[2]]}).json()
        assert r3["choices"][0]["token_ids"] == ids[:ids.index(ids[2]) + 1]
        assert r3["choices"][0]["finish_reason"] == "stop"
        # streamed chat: role-tagged deltas, [DONE]
        with client.stream("POST", "/v1/chat/completions",
                           json={"messages": msgs, "max_tokens": 3, "stream": True, "ignore_eos": True}) as s:
            events = [ln for ln in s.iter_lines() if ln.startswith("data: ")]
        assert events[-1] == "data: [DONE]" and len(events) == 4
        import json as _json
        assert _json.loads(events[0][6:])["object"] == "chat.completion.chunk"
        # top_p runs (sampling path) and respects max_tokens
        r4 = client.post("/v1/completions", json={"prompt": "abc", "max_tokens": 4, "temperature": 1.0,
                                                  "top_p": 0.5, "ignore_eos": True}).json()
        assert r4["usage"]["completion_tokens"] == 4
    finally:
        runner.shutdown()


def test_logprobs_engine_and_api():
    from fastapi.testclient import TestClient

    from kgs.serve import EngineConfig, LLMEngine, SamplingParams
    from kgs.serve.api import EngineLoop, create_app

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False),
                    device="cpu", backend="ref")
    prompt = [5, 6, 7, 8]
    r = eng.generate([prompt], SamplingParams(max_tokens=3, ignore_eos=True, logprobs=3))[0]
    assert len(r.logprobs) == 3
    seq = list(prompt)
    for tok, (lp, top) in zip(r.output, r.logprobs):
        ref = torch.log_softmax(eng.model.oracle.forward(torch.tensor([seq]))[0, -1].float(), -1)
        assert abs(lp - float(ref[tok])) < 5e-2 and len(top) == 3
        # greedy: the sampled token is a top-1 (bf16 logits can tie)
        assert abs(top[0][1] - lp) < 1e-6 and top[0][1] >= top[1][1] >= top[2][1]
        seq.append(tok)
    # no logprobs requested: nothing recorded
    r2 = eng.generate([prompt], SamplingParams(max_tokens=2, ignore_eos=True))[0]
    assert r2.logprobs == []
    runner = EngineLoop(eng)
    try:
        client = TestClient(create_app(runner, model_name="tiny"))
        c = client.post("/v1/completions", json={"prompt": prompt, "max_tokens": 3, "ignore_eos": True,
                                                 "logprobs": 2}).json()["choices"][0]
        lp = c["logprobs"]
        assert len(lp["tokens"]) == 3 and len(lp["token_logprobs"]) == 3
        assert all(len(t) <= 2 for t in lp["top_logprobs"]) and all(v <= 0 for v in lp["token_logprobs"])
        ch = client.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "hi"}],
                                                       "max_tokens": 2, "ignore_eos": True, "logprobs": True,
                                                       "top_logprobs": 1}).json()["choices"][0]
        content = ch["logprobs"]["content"]
        assert len(content) == 2 and len(content[0]["top_logprobs"]) == 1
        plain = client.post("/v1/completions", json={"prompt": prompt, "max_tokens": 1}).json()["choices"][0]
        assert "logprobs" not in plain
    finally:
        runner.shutdown()


def test_data_parallel_replicas_cpu():
    """--data-parallel: two engine processes (ref backend on CPU) behind the
    EngineLoop interface; concurrent requests spread over both replicas and each
    generates what one engine generates; the HTTP layer works on top."""
    import asyncio
    import dataclasses

    from fastapi.testclient import TestClient

    from kgs.serve import EngineConfig, LLMEngine, SamplingParams
    from kgs.serve.api import create_app
    from kgs.serve.dp import DPEngineLoop

    ec = EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False)
    runner = DPEngineLoop(2, dataclasses.asdict(_tiny()), ec, device="cpu", backend="ref", start_timeout=300)
    prompts = [[5, 6, 7], [9, 10], [11, 12, 13, 14], [3, 4]]
    p = SamplingParams(max_tokens=4, ignore_eos=True)
    try:
        async def one(prompt):
            q: asyncio.Queue = asyncio.Queue()
            runner.submit(prompt, p, asyncio.get_running_loop(), q)
            kind, _ = await q.get()
            assert kind == "id"
            out = []
            while True:
                _, t, fin, _, _ = await q.get()
                out.append(t)
                if fin:
                    return out

        async def all_():
            return await asyncio.gather(*(one(pr) for pr in prompts))

        got = asyncio.run(all_())
        assert runner.assigned == [2, 2]
        ref = LLMEngine(_tiny(), ec, device="cpu", backend="ref").generate(prompts, p)
        assert got == [r.output for r in ref]
        client = TestClient(create_app(runner, model_name="tiny"))
        r = client.post("/v1/completions", json={"prompt": prompts[0], "max_tokens": 4, "ignore_eos": True}).json()
        assert r["choices"][0]["token_ids"] == got[0]
        assert "kgs_requests_total 5" in client.get("/metrics").text
    finally:
        runner.shutdown()


def test_data_parallel_replica_failure_is_reported():
    import dataclasses

    from kgs.serve import EngineConfig
    from kgs.serve.dp import DPEngineLoop

    bad = dict(dataclasses.asdict(_tiny()), heads=3)  # hidden 256 / 3 heads: engine construction fails
    with pytest.raises(RuntimeError, match="failed to start"):
        DPEngineLoop(1, bad, EngineConfig(num_pages=32, max_batch=2, max_model_len=256, cuda_graphs=False),
                     device="cpu", backend="ref", start_timeout=120)


def test_http_n_samples():
    from fastapi.testclient import TestClient

    from kgs.serve import EngineConfig, LLMEngine
    from kgs.serve.api import EngineLoop, create_app

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=64, max_batch=4, max_model_len=256, cuda_graphs=False,
                                          prefix_caching=True, chunked_prefill=256), device="cpu", backend="ref")
    runner = EngineLoop(eng)
    try:
        client = TestClient(create_app(runner, model_name="tiny"))
        prompt = list(range(3, 3 + 140))
        r = client.post("/v1/completions", json={"prompt": prompt, "max_tokens": 3, "ignore_eos": True,
                                                 "n": 3}).json()
        assert [c["index"] for c in r["choices"]] == [0, 1, 2]
        assert all(c["token_ids"] == r["choices"][0]["token_ids"] for c in r["choices"])  # greedy: identical
        assert r["usage"]["completion_tokens"] == 9
        with client.stream("POST", "/v1/completions", json={"prompt": prompt, "max_tokens": 2, "stream": True,
                                                            "ignore_eos": True, "n": 2}) as s:
            events = [ln for ln in s.iter_lines() if ln.startswith("data: ")]
        import json as _json
        idx = sorted(_json.loads(e[6:])["choices"][0]["index"] for e in events[:-1])
        assert events[-1] == "data: [DONE]" and idx == [0, 0, 1, 1]
        assert eng.sched.prefix_hit_tokens >= 128  # the samples share the prompt's cached pages
    finally:
        runner.shutdown()


def test_sampling_penalties():
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False),
                    device="cpu", backend="ref")
    rid = eng.add_request([5, 6], SamplingParams(max_tokens=1, presence_penalty=1.0, frequency_penalty=0.5,
                                                 repetition_penalty=2.0))
    eng.abort(rid)  # keep it out of the scheduler; drive the sampler by hand
    eng._want_pen.add(rid)
    r = eng.requests[rid]
    r.output = [7, 7, 9]
    logits = torch.zeros(1, 16)
    logits[0, 5], logits[0, 7], logits[0, 9], logits[0, 3] = 4.0, 4.0, -2.0, 1.0
    out = eng._penalize([rid], logits)[0]
    # 7: (4 - 0.5*2 - 1) / 2 = 1; 9: (-2 - 0.5 - 1) * 2 = -7; 5 (prompt): 4 / 2 = 2; 3 untouched
    assert out[7].item() == 1.0 and out[9].item() == -7.0 and out[5].item() == 2.0 and out[3].item() == 1.0
    # greedy with a strong presence penalty never repeats a generated token
    g = eng.generate([[5, 6, 7]], SamplingParams(max_tokens=12, ignore_eos=True, presence_penalty=100.0))[0]
    assert len(set(g.output)) == len(g.output)


def test_seeded_sampling_is_reproducible():
    """A seeded request draws from its own generator: its tokens do not depend on
    the engine-wide generator the unseeded requests beside it consume."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    prompts = [[5, 6, 7], [9, 10], [11, 12, 13]]

    def run(engine_seed, seed):
        eng = LLMEngine(_tiny(), EngineConfig(num_pages=64, max_batch=4, max_model_len=256, cuda_graphs=False),
                        device="cpu", backend="ref")
        eng._gen.manual_seed(engine_seed)  # the engine-wide sampling stream (the weights stay the same)
        ps = [SamplingParams(max_tokens=6, temperature=1.0, seed=seed, ignore_eos=True)] + \
             [SamplingParams(max_tokens=6, temperature=1.0, ignore_eos=True)] * 2
        return [r.output for r in eng.generate(prompts, ps)]

    a, b = run(1, 1234), run(2, 1234)
    assert a[0] == b[0] and a[1:] != b[1:]  # the seeded row repeats, its unseeded mates do not
    assert run(1, 99)[0] != a[0]


def test_stop_text_truncates_and_holds_back():
    from kgs.serve.api import ByteTokenizer, StopText

    tok = ByteTokenizer()
    ids = tok.encode("hello world, bye")[1:]
    st = StopText(tok, ["wor", "xyz"])
    out, hit = "", False
    for i, t in enumerate(ids):
        text, hit = st.push(t, i == len(ids) - 1)
        out += text
        if hit:
            break
    assert hit and out == "hello "
    st2 = StopText(tok, ["zzz"])  # never hits: everything comes out by the final token
    out2 = "".join(st2.push(t, i == len(ids) - 1)[0] for i, t in enumerate(ids))
    assert out2 == "hello world, bye"


def test_top_p_sampling_keeps_nucleus():
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False),
                    device="cpu", backend="ref")
    rid = eng.add_request([5, 6, 7], SamplingParams(max_tokens=1, temperature=1.0, top_p=0.3))
    eng.abort(rid)
    # one dominant token (p ~ 0.9) -> top_p 0.3 always picks it; top_p 1.0 can pick others
    logits = torch.full((2, 64), -5.0)
    logits[:, 7] = 5.0
    eng.requests[rid].params = SamplingParams(temperature=1.0, top_p=0.3)
    rid2 = eng.add_request([5, 6], SamplingParams(max_tokens=1, temperature=1.0, top_p=1.0))
    picks = {int(eng._sample([rid, rid2], logits)[0]) for _ in range(50)}
    assert picks == {7}


def test_online_bench_poisson_cpu():
    """bench --request-rate: Poisson arrivals through the engine loop (ref backend
    on CPU); every request completes and the latency percentiles are ordered."""
    from kgs.serve import bench

    a = bench.main.__globals__["argparse"].Namespace(
        requests=6, input_len=20, output_len=5, max_batch=4, max_model_len=256, max_prefill_tokens=4096,
        layers=2, no_graphs=True, fused_max_batch=0, decode_weights="bf16", kv_cache_dtype="bf16",
        request_rate=200.0)
    r = bench.run_online(a, mc=_tiny(), device="cpu", backend="ref")
    assert r["requests_per_s"] > 0 and r["stats"]["decode_tokens"] + r["stats"]["prefill_steps"] > 0
    for k in ("ttft_ms", "tpot_ms", "itl_ms", "e2e_ms"):
        assert 0 <= r[k]["p50"] <= r[k]["p99"]
    assert r["output_tok_per_s"] > 0 and r["e2e_ms"]["p99"] >= r["ttft_ms"]["p50"]


def test_byte_tokenizer_roundtrip():
    from kgs.serve.api import ByteTokenizer

    t = ByteTokenizer()
    ids = t.encode("héllo ✓")
    assert ids[0] == t.BOS and t.decode(ids) == "héllo ✓"


def test_decode_routing_tables_cpu():
    """The decode GEMM routing/geometry helpers (pure Python, mirrored by decode.hip)."""
    from kgs.ops import decode as D

    for m in (1, 16, 17, 32, 33, 64, 65, 128, 129, 256):
        vs = D.skinny_variants(m)
        assert vs and all(D.SKINNY_VARIANTS[v][1] == D._mt(m) for v in vs)
        for v in vs:
            rps, kpc, mpad = D.skinny_geometry(m, v)
            assert rps % (16 if v in D.KIN_VARIANTS else 64) == 0 and kpc % 32 == 0 and mpad >= m
    for key, val in D.TUNED.items():
        if val is not None:
            v, ks = val
            assert D.SKINNY_VARIANTS[v][1] == key[0]
            _, kpc, _ = D.skinny_geometry(16 * key[0], v)
            assert (key[2] // kpc) % ks == 0, key
    assert D.use_skinny(1, 6144, 4096) and not D.use_skinny(256, 6144, 4096)
    assert D.use_skinny(20, 512, 1024) and not D.use_skinny(40, 512, 1024)
    assert D.skinny_config(16, 4096, 4096) == D.TUNED[(1, 4096, 4096)]
    for fp8, tiny, table in ((False, D.TUNED_TINY, D.TUNED), (True, D.TUNED_TINY_FP8, D.TUNED_FP8)):
        for (n, k), (v, ks, top) in tiny.items():
            assert D.skinny_config(1, n, k, fp8) == (v, ks) and D.skinny_config(top, n, k, fp8) == (v, ks)
            if top < 16:
                assert D.skinny_config(top + 1, n, k, fp8) == table[(1, n, k)]
            _, kpc, _ = D.skinny_geometry(1, v)
            assert (k // kpc) % ks == 0 and n % D.skinny_geometry(1, v)[0] == 0
    pps, ns = D.decode_splits(1, 8, 128)
    assert pps >= 4 and pps * ns >= 128
    # round 3: about two waves per CU -- batch 16 four splits, 32 two, >= 64 one
    # (paired with the kernel's two-page pipeline up to 1024 waves)
    assert [D.decode_splits(b, 8, 64)[1] for b in (16, 32, 64, 128, 256)] == [4, 2, 1, 1, 1]
    assert D.decode_splits(1, 8, 8) == (4, 2)  # >= 4 pages per split


def test_splitk_routing_table_cpu():
    """Every split-K entry is launchable (K slices of whole 128-deep K-tiles) and
    fits the workspace reserved before graph capture."""
    from kgs.ops import decode as D

    for (m, n, k), ns in D.SPLITK_TUNED.items():
        assert m & (m - 1) == 0 and n % 256 == 0, (m, n, k)
        assert k % ns == 0 and (k // ns) % 128 == 0, (m, n, k, ns)
        assert ns * m * n <= D.SPLITK_WS_FLOATS, (m, n, k, ns)
        assert D.splitk_slices(m, n, k) == ns and D.splitk_slices(m // 2 + 1, n, k) == ns
    assert D.splitk_slices(256, 28672, 4096) is None  # gate|up stays on hipBLASLt


def test_fp8_routing_table_cpu():
    from kgs.ops import decode as D

    for key, (v, ks) in D.TUNED_FP8.items():
        assert (v <= 12 or v in D.KIN_VARIANTS) and D.SKINNY_VARIANTS[v][1] == key[0]  # fp8: 1-12, 20-21
        _, kpc, _ = D.skinny_geometry(16 * key[0], v)
        assert (key[2] // kpc) % ks == 0
    assert D.skinny_config(16, 28672, 4096, fp8=True) == D.TUNED_FP8[(1, 28672, 4096)]


def test_w4x_routing_table_cpu():
    """Every four-wave decode route is launchable (tile divides N, K slices of
    whole 128-deep K-tiles, a known tile height) and its fp32 partials fit the
    split-K workspace reserved before graph capture."""
    from kgs.ops import decode as D

    for (m, n, k), r in D.W4X_TUNED.items():
        bn, ns, bm = r[:3]
        st = D.w4x_stages(r)
        assert m in D._W4X_BUCKETS and bn in (128, 256) and bm in (128, 256), (m, n, k)
        assert len(r) in (3, 4) and st in (2, 3, 4) and st * (bm + bn) * 128 <= 160 * 1024, (m, n, k, r)
        assert n % bn == 0 and k % ns == 0 and (k // ns) % 128 == 0, (m, n, k, ns)
        assert ns == 1 or ns * m * n <= D.SPLITK_WS_FLOATS, (m, n, k, ns)
        # 128-row tiles where they pad less (<= 128 rows) or were measured faster (o at 192-256)
        assert bm == 256 or m <= 128 or (n, k) == D._O, (m, bm)
    assert D.w4x_route(D.W4X_MIN_BATCH - 1, 4096, 4096) is None
    assert D.w4x_route(64, 4096, 4096) == D.W4X_TUNED[(64, 4096, 4096)]


def test_rope_packing_cpu():
    """The RoPE-packed qkv order: every q / k head's 16-row tile t holds dims
    8t..8t+7 then 64+8t..64+8t+7 (lane g < 2 and its partner g ^ 2 hold a
    rotate-half pair), v heads untouched; packing round-trips."""
    import torch

    from kgs.ops import decode as D

    heads, hkv = 4, 2
    n = (heads + 2 * hkv) * 128
    rows = D.rope_rows(n, heads, hkv)
    assert sorted(rows.tolist()) == list(range(n))
    for hh in range(heads + hkv):
        for t in range(8):
            tile = rows[hh * 128 + 16 * t: hh * 128 + 16 * t + 16].tolist()
            assert tile[:8] == [hh * 128 + 8 * t + j for j in range(8)]
            assert tile[8:] == [hh * 128 + 64 + 8 * t + j for j in range(8)]
    assert rows[(heads + hkv) * 128:].tolist() == list(range((heads + hkv) * 128, n))
    w = torch.randn(n, 64).bfloat16()
    p = D.PackedWeight(w, rope=(heads, hkv))
    assert torch.equal(p.unpacked(), w)
    with pytest.raises(ValueError):
        D.rope_rows(n + 128, heads, hkv)


def test_w4x_route_override_cpu():
    """KGS_W4X_ROUTES replaces / removes W4X_TUNED entries (same-box routing A/B)
    and rejects malformed specs."""
    import pytest as _pytest

    from kgs.ops import decode as D

    saved = dict(D.W4X_TUNED)
    try:
        D._apply_w4x_override("256,4096,4096=128,4,128,3; 128,6144,4096=none")
        assert D.w4x_route(256, 4096, 4096) == (128, 4, 128, 3) and D.w4x_stages(D.w4x_route(256, 4096, 4096)) == 3
        assert D.w4x_route(128, 6144, 4096) is None
        for bad in ("255,4096,4096=128,4,128", "256,4096=128,4,128", "256,4096,4096=128,4"):
            with _pytest.raises(ValueError):
                D._apply_w4x_override(bad)
    finally:
        D.W4X_TUNED.clear()
        D.W4X_TUNED.update(saved)


def test_engine_checks_every_index_before_the_gpu_sees_it():
    """A corrupted scheduler plan (out-of-range page, position, slot, token or
    a decode slot outside its last page) raises on the host with the values,
    instead of reaching a kernel as an address."""
    import types

    from kgs.serve import EngineConfig, LLMEngine

    eng = LLMEngine(_tiny(), EngineConfig(num_pages=16, max_batch=4, max_model_len=256, cuda_graphs=False),
                    device="cpu", backend="ref")

    def plan(**kw):
        p = dict(kind=2, seq_ids=np.arange(2), tokens=np.array([5, 6]), positions=np.array([40, 7]),
                 slots=np.array([1 * 32 + 8, 3 * 32 + 7]), ctx_lens=np.array([41, 8]),
                 block_tables=np.array([[2, 1], [3, 0]]), n_prefill=0)
        p.update(kw)
        return types.SimpleNamespace(**p)

    eng._check_plan(plan())  # a consistent decode plan passes
    for kw, msg in ((dict(block_tables=np.array([[2, 16], [3, 0]])), "block_tables outside [0, 16)"),
                    (dict(positions=np.array([40, 256])), "positions outside"),
                    (dict(slots=np.array([40, 16 * 32])), "slots outside"),
                    (dict(tokens=np.array([5, 512])), "tokens outside"),
                    (dict(ctx_lens=np.array([41, 0])), "ctx_lens outside"),
                    (dict(slots=np.array([2 * 32 + 8, 3 * 32 + 7])), "not in the last page")):
        with pytest.raises(RuntimeError, match=msg.replace("[", r"\[").replace("(", r"\(").replace(")", r"\)")):
            eng._check_plan(plan(**kw))


def test_step_trace_breadcrumbs(tmp_path):
    """kgs.serve.trace: one begin / end line per engine step, unbuffered, and
    an op line per op with KGS_SYNC_DEBUG (the first op without a line after a
    GPU fault is the faulting one)."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams
    from kgs.serve import trace

    path = tmp_path / "steps.log"
    t = trace.StepTrace(str(path))
    old = trace.TRACE
    import kgs.serve.engine as E

    E.TRACE = t
    try:
        eng = LLMEngine(_tiny(), EngineConfig(num_pages=32, max_batch=4, max_model_len=256, cuda_graphs=False),
                        device="cpu", backend="ref")
        eng.generate([[5, 6, 7], [9, 10]], SamplingParams(max_tokens=3, ignore_eos=True))
    finally:
        E.TRACE = old
    lines = path.read_text().splitlines()
    begins = [ln for ln in lines if ln.endswith(" begin")]
    ends = [ln for ln in lines if ln.endswith(" end")]
    assert len(begins) == len(ends) == eng.stats["prefill_steps"] + eng.stats["decode_steps"] >= 3
    assert "kind=1" in begins[0] and "kind=2" in begins[-1]
    assert not trace.StepTrace(None).on and not trace.StepTrace(None, sync_ops=True).sync_ops


def test_kv_page_budget_counts_the_gate_up_panel_copies(monkeypatch):
    """The SwiGLU gate|up panel copies (one per unsplit decode tile width: 128
    and 256 for Llama-3-8B, 2 x 32 x 235 MB) come out of the KV-page budget:
    with them on, the engine sizes 15 GB fewer pages than with them off."""
    from kgs.models.llama import LlamaConfig
    from kgs.ops.decode import PagedKVCache
    from kgs.serve import EngineConfig, LLMEngine
    from kgs.serve.model import gate_up_panel_widths

    mc = LlamaConfig.named("llama3-8b")
    assert gate_up_panel_widths(2 * mc.intermediate, mc.hidden) == {128, 256}
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (280 << 30, 288 << 30))
    monkeypatch.delenv("KGS_GATEUP_PANELS", raising=False)
    pages = {}
    for on in (True, False):
        eng = object.__new__(LLMEngine)
        eng.device, eng.backend, eng.cfg = torch.device("cuda"), "kgs", EngineConfig(gate_up_panels=on)
        pages[on] = eng._pages_from_memory(mc)
    extra = 2 * mc.layers * 2 * mc.intermediate * mc.hidden * 2
    per_page = PagedKVCache.bytes_per_page(mc.layers, mc.kv_heads, "bf16")
    assert abs((pages[False] - pages[True]) - extra * EngineConfig().kv_fraction / per_page) <= 1


def test_scheduler_two_phase_update():
    """update_pending advances a step's sequences by a pending token (length
    stops apply at once), the next step is scheduled before the values are
    known, and fill_pending writes them in; a late EOS goes through abort."""
    from kgs._native import _serve

    cfg = _serve.SchedulerConfig()
    cfg.num_pages, cfg.page_size, cfg.max_batch, cfg.max_model_len, cfg.pad_multiple = 32, 32, 4, 256, 128
    s = _serve.Scheduler(cfg)
    P = _serve.Scheduler.PENDING
    assert s.add(1, [5, 6, 7], 3) and s.add(2, [8, 9], 1)
    p = s.schedule()
    assert p.kind == 1 and list(p.seq_ids) == [1, 2]
    done = s.update_pending(p.seq_ids)
    assert list(done) == [2]  # max_tokens 1: finished by length before its token is known
    p2 = s.schedule()  # planned while step 1's tokens are in flight
    assert p2.kind == 2 and list(p2.seq_ids) == [1] and list(p2.tokens) == [P] and list(p2.positions) == [3]
    assert s.fill_pending(p.seq_ids, np.array([40, 41], np.int32)) == 2
    assert list(s.tokens(1)) == [5, 6, 7, 40] and list(s.tokens(2)) == [8, 9, 41]
    s.release(2)
    assert list(s.update_pending(p2.seq_ids)) == []
    assert s.fill_pending(np.array([1, 2]), np.array([42, 0], np.int32)) == 1  # 2 is gone: skipped
    assert s.abort(1)  # EOS seen one step late
    assert s.schedule().kind == 0 and s.check_invariants() == ""


@pytest.mark.parametrize("case", ["eos", "preempt", "admission", "chunked", "chunked_preempt"])
def test_overlapped_steps_generate_what_sequential_steps_do(case):
    """EngineConfig.overlap plans step t+1 before step t's tokens are read
    back. With EOS stops (seen one step late), preemption + recompute, and more
    requests than max_batch (prefill steps between decodes), every request's
    tokens and finish reason equal those of one-step-at-a-time execution."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    rng = np.random.default_rng({"eos": 3, "preempt": 4, "admission": 5, "chunked": 6, "chunked_preempt": 7}[case])
    kw = dict(num_pages=64, max_batch=4, max_model_len=256, cuda_graphs=False)
    if case.startswith("chunked"):  # mixed steps: prompt chunks of 128 rows beside the decode rows
        kw.update(chunked_prefill=128, max_model_len=512)
    n = {"eos": 4, "preempt": 3, "admission": 9, "chunked": 6, "chunked_preempt": 3}[case]
    prompts = [rng.integers(3, 512, size=int(rng.integers(5, 40))).tolist() for _ in range(n)]
    params = [SamplingParams(max_tokens=int(rng.integers(2, 14)), ignore_eos=case != "eos") for _ in range(n)]
    if case in ("preempt", "chunked_preempt"):  # 5 usable pages, 3 sequences growing across page boundaries
        kw.update(num_pages=6, max_batch=3)
        prompts = [rng.integers(3, 512, size=m).tolist() for m in (30, 28, 31)]
        params = [SamplingParams(max_tokens=m, ignore_eos=True) for m in (12, 9, 12)]
    if case == "chunked":  # prompts longer than a chunk
        prompts = [rng.integers(3, 512, size=int(rng.integers(100, 300))).tolist() for _ in range(n)]
    eos = -1
    if case == "eos":  # an EOS id that some request samples early on
        probe = LLMEngine(_tiny(), EngineConfig(**kw, overlap=False), device="cpu", backend="ref")
        eos = probe.generate(prompts, [SamplingParams(max_tokens=14, ignore_eos=True)] * n)[1].output[2]
    outs = {}
    for ov in (False, True):
        eng = LLMEngine(_tiny(), EngineConfig(**kw, overlap=ov, eos_token_id=eos), device="cpu", backend="ref")
        assert eng.overlap == ov
        outs[ov] = [(r.output, r.finish_reason) for r in eng.generate(prompts, params)]
        assert eng.sched.check_invariants() == "" and not eng.has_work()
        if case.endswith("preempt"):
            assert eng.stats["preemptions"] >= 1
        if case.startswith("chunked"):
            assert eng.stats["mixed_steps"] >= 1
    assert outs[True] == outs[False]
    if case == "eos":
        assert any(f == "stop" for _, f in outs[True])


def test_overlap_falls_back_for_host_state_sampling():
    """Logprobs, penalties and seeded sampling read per-step host state: a
    batch holding one runs one step at a time (the in-flight step is drained
    first), and its results equal a sequential engine's."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    kw = dict(num_pages=64, max_batch=4, max_model_len=256, cuda_graphs=False)
    prompts = [[5, 6, 7], [8, 9, 10, 11]]
    ps = [SamplingParams(max_tokens=6, ignore_eos=True),
          SamplingParams(max_tokens=6, ignore_eos=True, logprobs=2, frequency_penalty=0.5)]
    res = {}
    for ov in (False, True):
        eng = LLMEngine(_tiny(), EngineConfig(**kw, overlap=ov), device="cpu", backend="ref")
        rid0 = eng.add_request(prompts[0], ps[0])
        eng.step()
        eng.step()  # overlapped: one step in flight
        rid1 = eng.add_request(prompts[1], ps[1])
        while eng.has_work():
            eng.step()
        res[ov] = [(eng.requests[r].output, len(eng.requests[r].logprobs)) for r in (rid0, rid1)]
    assert res[True] == res[False] and res[True][1][1] == 6


def test_abort_while_a_step_is_in_flight():
    """An abort between overlapped steps (the aborted sequence is in the step
    on the GPU): the request gets no more tokens, its pages go back, and the
    other requests generate what a sequential engine gives them."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    kw = dict(num_pages=64, max_batch=4, max_model_len=256, cuda_graphs=False)
    prompts = [[5, 6, 7, 8], [9, 10, 11], [12, 13, 14, 15, 16]]
    p = SamplingParams(max_tokens=8, ignore_eos=True)
    res = {}
    for ov in (False, True):
        eng = LLMEngine(_tiny(), EngineConfig(**kw, overlap=ov), device="cpu", backend="ref")
        rids = [eng.add_request(q, p) for q in prompts]
        for _ in range(3):
            eng.step()
        n_at_abort = len(eng.requests[rids[1]].output)
        eng.abort(rids[1])
        while eng.has_work():
            eng.step()
        r = [eng.requests[i] for i in rids]
        assert r[1].finish_reason == "abort" and len(r[1].output) == n_at_abort
        assert eng.sched.check_invariants() == "" and eng.sched.num_free_pages == 63
        res[ov] = [(x.output, x.finish_reason) for x in (r[0], r[2])]
    assert res[True] == res[False]


def test_overlapped_steps_with_prefix_caching():
    """Prefix caching under overlapped steps: a page completed by a generated
    token that is still pending is registered once fill_pending knows the
    token (its hash needs it). A follow-up turn whose prompt is an earlier
    prompt + its answer hits the generated pages, and every generation equals
    the sequential engine's."""
    from kgs.serve import EngineConfig, LLMEngine, SamplingParams

    rng = np.random.default_rng(17)
    system = rng.integers(3, 512, size=300).tolist()
    prompts = [system + rng.integers(3, 512, size=n).tolist() for n in (5, 40, 77)]
    res = {}
    for ov in (False, True):
        eng = LLMEngine(_tiny(), EngineConfig(num_pages=128, max_batch=4, max_model_len=1024, cuda_graphs=False,
                                              prefix_caching=True, chunked_prefill=256, overlap=ov),
                        device="cpu", backend="ref")
        assert eng.overlap == ov
        p = SamplingParams(max_tokens=40, ignore_eos=True)
        first = eng.generate(prompts, p)
        # second turn: prompt + answer + a new question -> the answer's full pages are cached
        turn2 = [q + r.output + [7, 8, 9] for q, r in zip(prompts, first)]
        hits0 = eng.sched.prefix_hit_tokens
        second = eng.generate(turn2, SamplingParams(max_tokens=6, ignore_eos=True))
        hits = eng.sched.prefix_hit_tokens - hits0
        assert eng.sched.check_invariants() == ""
        res[ov] = ([r.output for r in first], [r.output for r in second], hits)
    assert res[True][0] == res[False][0] and res[True][1] == res[False][1]
    assert res[True][2] == res[False][2] and res[True][2] >= 3 * 320  # system prompt + generated pages


@settings(max_examples=50, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 2), st.integers(1, 200), st.integers(1, 40)), min_size=1, max_size=20),
       st.integers(12, 48), st.integers(1, 6), st.sampled_from([0, 128, 256]), st.booleans())
def test_two_phase_random_traffic(reqs, pages, max_batch, chunk, prefix):
    """The overlapped engine's scheduler protocol under random traffic: step
    t+1 is planned after update_pending(t) and before fill_pending(t); late EOS
    stops go through abort; preemption, chunking and prefix caching as they
    come. Invariants hold every step, no pending token survives a fill, all
    requests finish and no page leaks."""
    c = _serve.SchedulerConfig()
    c.num_pages, c.page_size, c.max_batch, c.max_model_len, c.pad_multiple = pages, 32, max_batch, 512, 128
    c.max_prefill_tokens, c.chunk_tokens, c.prefix_caching = 1024, chunk, prefix
    s = _serve.Scheduler(c)
    P = _serve.Scheduler.PENDING
    prefixes = [list(range(100 + 300 * k, 100 + 300 * k + 160)) for k in range(3)]
    live = set()
    for i, (k, extra, new) in enumerate(reqs):
        if s.add(i, prefixes[k] + [3] * extra, new):
            live.add(i)
    rng = np.random.default_rng(0)
    prev = None
    for _ in range(4000):
        if prev is not None:
            for d in s.update_pending(prev):
                live.discard(int(d))
        p = s.schedule()
        assert s.check_invariants() == "", s.check_invariants()
        if prev is not None:  # step t's tokens arrive after step t+1 was planned
            s.fill_pending(prev, np.full(len(prev), 4, np.int32))
            for j in np.flatnonzero(rng.random(len(prev)) < 0.05):  # EOS seen one step late
                if s.abort(int(prev[j])):
                    live.discard(int(prev[j]))
            for r in prev:
                try:
                    assert P not in s.tokens(int(r))
                except KeyError:
                    pass
        if p.kind == 0:
            prev = None
            if not live:
                break
            continue
        ids = p.seq_ids
        if p.kind == 3:
            ids = np.concatenate([ids[:p.n_prefill][p.last_chunk.astype(bool)], ids[p.n_prefill:]])
        prev = np.asarray(ids, dtype=np.int64)
    assert not live and s.num_running == 0 and s.num_waiting == 0
    assert s.num_free_pages == pages - 1
