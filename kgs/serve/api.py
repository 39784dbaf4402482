"""OpenAI-style HTTP server over :class:`kgs.serve.LLMEngine` -- the kgs
replacement for the vLLM process of ``pods/vllm-rocm-pod.yaml`` (same port
8000, same ``/v1/completions`` request shape; see ``pods/kgs-serve-pod.yaml``).

Endpoints: ``POST /v1/completions`` (prompt as text or token ids; ``stream``
gives server-sent events), ``POST /v1/chat/completions`` (messages rendered by
a plain role-tagged template), ``GET /v1/models``, ``GET /health``,
``GET /metrics`` (Prometheus). Sampling: temperature, top_k, top_p,
stop strings, stop_token_ids, ignore_eos. One background thread owns the engine (it is not thread-safe) and
runs :meth:`LLMEngine.step` whenever there is work; request handlers only talk to
it through a queue.

Tokenizer: byte-level by default (ids 3..258 are the UTF-8 bytes; 1 = BOS,
2 = EOS) because the weights are random-init and no tokenizer can be
downloaded; ``--tokenizer tokenizer.json`` loads a local HF ``tokenizers`` file.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import queue
import threading
import time
import uuid

from pydantic import BaseModel

from .engine import SamplingParams


class _SamplingFields(BaseModel):
    model: str | None = None
    max_tokens: int = 16
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    stop: str | list[str] | None = None
    stop_token_ids: list[int] | None = None
    stream: bool = False
    ignore_eos: bool = False
    n: int = 1  # independent samples of the prompt (choices 0 .. n-1)
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0
    seed: int | None = None

    def n_logprobs(self) -> int | None:
        return None

    def params(self) -> SamplingParams:
        return SamplingParams(max_tokens=self.max_tokens, temperature=self.temperature, top_k=self.top_k,
                              top_p=self.top_p, ignore_eos=self.ignore_eos,
                              stop_token_ids=tuple(self.stop_token_ids or ()), logprobs=self.n_logprobs(),
                              presence_penalty=self.presence_penalty, frequency_penalty=self.frequency_penalty,
                              repetition_penalty=self.repetition_penalty, seed=self.seed)

    def stops(self) -> list[str]:
        return [self.stop] if isinstance(self.stop, str) else [t for t in (self.stop or []) if t]


class CompletionRequest(_SamplingFields):
    prompt: str | list[int]
    logprobs: int | None = None  # OpenAI completions: sampled token + this many alternatives

    def n_logprobs(self) -> int | None:
        return self.logprobs


class ChatMessage(BaseModel):
    role: str
    content: str


class ChatRequest(_SamplingFields):
    messages: list[ChatMessage]
    logprobs: bool = False
    top_logprobs: int = 0

    def n_logprobs(self) -> int | None:
        return self.top_logprobs if self.logprobs else None


def render_chat(messages) -> str:
    """Role-tagged transcript ending with an open assistant turn (the weights are
    random-init, so there is no model-specific chat template to honour)."""
    return "".join(f"<|{m.role}|>\n{m.content}\n" for m in messages) + "<|assistant|>\n"


class StopText:
    """Incremental detokenisation with OpenAI-style stop strings: text is
    released only once it can no longer be the start of a stop string; a match
    truncates the output before the stop string."""

    def __init__(self, tok, stops: list[str]):
        self.tok, self.stops = tok, stops
        self.ids: list[int] = []
        self.sent = 0
        self.hold = max((len(t) for t in stops), default=1) - 1

    def push(self, t: int, final: bool) -> tuple[str, bool]:
        """Add a token; returns (text to emit now, stop string hit)."""
        self.ids.append(t)
        text = self.tok.decode(self.ids)
        if self.stops:
            hits = [i for i in (text.find(st, max(0, self.sent - self.hold)) for st in self.stops) if i >= 0]
            if hits:
                cut = min(hits)
                out, self.sent = text[self.sent:cut], cut
                return out, True
        end = len(text) if final or not self.stops else max(self.sent, len(text) - self.hold)
        out, self.sent = text[self.sent:end], end
        return out, False


class ByteTokenizer:
    BOS, EOS, OFFSET = 1, 2, 3

    def encode(self, text: str) -> list[int]:
        return [self.BOS] + [b + self.OFFSET for b in text.encode("utf-8")]

    def decode(self, ids) -> str:
        return bytes(i - self.OFFSET for i in ids if self.OFFSET <= i < 256 + self.OFFSET).decode("utf-8", "replace")


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(path)

    def encode(self, text: str) -> list[int]:
        return self.tok.encode(text).ids

    def decode(self, ids) -> str:
        return self.tok.decode(list(ids))


class EngineLoop:
    """Runs the engine on its own thread; handlers submit and await token queues."""

    def __init__(self, engine):
        self.engine = engine
        self.inbox: queue.Queue = queue.Queue()
        self.streams: dict = {}
        self.stop = threading.Event()
        self.wake = threading.Event()
        self.counters = {"requests": 0, "rejected": 0, "tokens": 0, "steps": 0}
        self.thread = threading.Thread(target=self._run, name="kgs-engine", daemon=True)
        self.thread.start()

    def submit(self, prompt: list[int], params: SamplingParams, loop, q) -> None:
        self.inbox.put((prompt, params, loop, q))
        self.wake.set()

    def cancel(self, rid: int) -> None:
        self.inbox.put(("abort", rid))
        self.wake.set()

    def shutdown(self) -> None:
        self.stop.set()
        self.wake.set()
        self.thread.join(timeout=10)

    def gauges(self) -> dict:
        eng = self.engine
        return {"running": eng.sched.num_running, "waiting": eng.sched.num_waiting,
                "free_kv_pages": eng.sched.num_free_pages, "preemptions": eng.stats["preemptions"],
                "prefix_hit_tokens": eng.sched.prefix_hit_tokens}

    def _push(self, loop, q, item) -> None:
        loop.call_soon_threadsafe(q.put_nowait, item)

    def _run(self) -> None:
        eng = self.engine
        while not self.stop.is_set():
            while True:
                try:
                    item = self.inbox.get_nowait()
                except queue.Empty:
                    break
                if item[0] == "abort":
                    eng.abort(item[1])
                    self.streams.pop(item[1], None)
                    continue
                prompt, params, loop, q = item
                try:
                    rid = eng.add_request(prompt, params)
                except ValueError as e:
                    self.counters["rejected"] += 1
                    self._push(loop, q, ("error", str(e)))
                    continue
                self.counters["requests"] += 1
                self.streams[rid] = (loop, q)
                self._push(loop, q, ("id", rid))
            if not eng.has_work():
                self.wake.wait(timeout=0.05)
                self.wake.clear()
                continue
            for rid, tok, fin in eng.step():
                self.counters["tokens"] += 1
                st = self.streams.get(rid)
                if st is None:
                    continue
                req = eng.requests[rid]
                reason = req.finish_reason if fin else None
                lp = req.logprobs[-1] if req.params.logprobs is not None and req.logprobs else None
                self._push(st[0], st[1], ("token", tok, fin, reason, lp))
                if fin:
                    self.streams.pop(rid, None)
                    eng.requests.pop(rid, None)
            self.counters["steps"] += 1


def create_app(loop_runner: EngineLoop, tokenizer=None, model_name: str = "meta-llama/Meta-Llama-3-8B"):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import PlainTextResponse, StreamingResponse

    tok = tokenizer or ByteTokenizer()
    app = FastAPI(title="kgs.serve")

    @app.get("/health")
    def health():
        return {"status": "ok"}

    @app.get("/v1/models")
    def models():
        return {"object": "list", "data": [{"id": model_name, "object": "model", "owned_by": "kgs"}]}

    @app.get("/metrics")
    def metrics():
        c = loop_runner.counters
        g = loop_runner.gauges()
        lines = [
            "# TYPE kgs_requests_total counter", f"kgs_requests_total {c['requests']}",
            "# TYPE kgs_requests_rejected_total counter", f"kgs_requests_rejected_total {c['rejected']}",
            "# TYPE kgs_generated_tokens_total counter", f"kgs_generated_tokens_total {c['tokens']}",
            "# TYPE kgs_engine_steps_total counter", f"kgs_engine_steps_total {c['steps']}",
            "# TYPE kgs_running gauge", f"kgs_running {g['running']}",
            "# TYPE kgs_waiting gauge", f"kgs_waiting {g['waiting']}",
            "# TYPE kgs_free_kv_pages gauge", f"kgs_free_kv_pages {g['free_kv_pages']}",
            "# TYPE kgs_preemptions_total counter", f"kgs_preemptions_total {g['preemptions']}",
            "# TYPE kgs_prefix_cache_hit_tokens_total counter", f"kgs_prefix_cache_hit_tokens_total {g['prefix_hit_tokens']}",
        ]
        return PlainTextResponse("\n".join(lines) + "\n")

    async def _start(ids, params):
        if not ids:
            raise HTTPException(400, "empty prompt")
        q: asyncio.Queue = asyncio.Queue()
        loop_runner.submit(ids, params, asyncio.get_running_loop(), q)
        first = await q.get()
        if first[0] == "error":
            raise HTTPException(400, first[1])
        return first[1], q

    async def _tokens(rid, q, stop: StopText):
        """(token id, text, finished, finish reason) until the request ends; a
        stop-string hit aborts the request in the engine."""
        try:
            while True:
                _, t, fin, reason, lp = await q.get()
                text, hit = stop.push(t, fin)
                if hit:
                    loop_runner.cancel(rid)
                    yield t, text, True, "stop", lp
                    return
                yield t, text, fin, reason, lp
                if fin:
                    return
        except asyncio.CancelledError:  # client went away
            loop_runner.cancel(rid)
            raise

    async def _serve(req, ids, chat: bool):
        params = req.params()
        n = max(1, req.n)
        # n samples of one prompt are n engine requests (with prefix caching they
        # share the prompt's KV pages); choice i is request i
        started = []
        try:
            for _ in range(n):
                started.append(await _start(ids, params))
        except HTTPException:
            for rid, _q in started:  # do not leave the samples that did start running
                loop_runner.cancel(rid)
            raise
        cid, created = f"{'chatcmpl' if chat else 'cmpl'}-{uuid.uuid4().hex[:16]}", int(time.time())
        name = req.model or model_name
        obj = "chat.completion" if chat else "text_completion"
        want_lp = params.logprobs is not None

        def logprobs_obj(ids_, lps):
            """OpenAI shapes: completions {tokens, token_logprobs, top_logprobs};
            chat {content: [{token, logprob, top_logprobs: [{token, logprob}]}]}."""
            toks = [tok.decode([t]) for t in ids_]
            if chat:
                return {"content": [{"token": s_, "logprob": lp[0],
                                     "top_logprobs": [{"token": tok.decode([i]), "logprob": v} for i, v in lp[1]]}
                                    for s_, lp in zip(toks, lps)]}
            return {"tokens": toks, "token_logprobs": [lp[0] for lp in lps],
                    "top_logprobs": [{tok.decode([i]): v for i, v in lp[1]} for lp in lps]}

        def choice(i, text, ids_, reason, delta, lps):
            if not chat:
                c = {"index": i, "text": text, "token_ids": ids_, "finish_reason": reason}
            else:
                c = {"index": i, ("delta" if delta else "message"): {"role": "assistant", "content": text},
                     "finish_reason": reason}
            if want_lp:
                c["logprobs"] = logprobs_obj(ids_, lps)
            return c

        if req.stream:
            async def events():
                merged: asyncio.Queue = asyncio.Queue()

                async def feed(i, rid, q):
                    async for item in _tokens(rid, q, StopText(tok, req.stops())):
                        await merged.put((i, item))
                    await merged.put((i, None))

                tasks = [asyncio.ensure_future(feed(i, rid, q)) for i, (rid, q) in enumerate(started)]
                try:
                    live = n
                    while live:
                        i, item = await merged.get()
                        if item is None:
                            live -= 1
                            continue
                        t, text, fin, reason, lp = item
                        chunk = {"id": cid, "object": obj + (".chunk" if chat else ""), "created": created,
                                 "model": name, "choices": [choice(i, text, [t], reason, True, [lp])]}
                        yield f"data: {json.dumps(chunk)}\n\n"
                    yield "data: [DONE]\n\n"
                finally:
                    for tsk in tasks:
                        tsk.cancel()

            return StreamingResponse(events(), media_type="text/event-stream")

        async def collect(rid, q):
            out, parts, lps, reason = [], [], [], None
            async for t, text, fin, reason, lp in _tokens(rid, q, StopText(tok, req.stops())):
                out.append(t)
                parts.append(text)
                lps.append(lp)
            return out, "".join(parts), lps, reason

        results = await asyncio.gather(*(collect(rid, q) for rid, q in started))
        completion = sum(len(r[0]) for r in results)
        return {"id": cid, "object": obj, "created": created, "model": name,
                "choices": [choice(i, text, out, reason, False, lps)
                            for i, (out, text, lps, reason) in enumerate(results)],
                "usage": {"prompt_tokens": len(ids), "completion_tokens": completion,
                          "total_tokens": len(ids) + completion}}

    @app.post("/v1/completions")
    async def completions(req: CompletionRequest):
        ids = tok.encode(req.prompt) if isinstance(req.prompt, str) else list(req.prompt)
        return await _serve(req, ids, chat=False)

    @app.post("/v1/chat/completions")
    async def chat_completions(req: ChatRequest):
        if not req.messages:
            raise HTTPException(400, "no messages")
        return await _serve(req, tok.encode(render_chat(req.messages)), chat=True)

    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m kgs.serve serve", description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--model-name", default="meta-llama/Meta-Llama-3-8B")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--tokenizer", default=None, help="local HF tokenizer.json (default: byte-level)")
    ap.add_argument("--backend", choices=("kgs", "ref"), default="kgs")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--chunked-prefill", type=int, default=2048,
                    help="rows per mixed prompt-chunk + decode step (0 = whole-prompt prefill steps)")
    ap.add_argument("--prefix-caching", action="store_true", help="reuse cached pages of shared prompt prefixes")
    ap.add_argument("--overlap", action=argparse.BooleanOptionalAction, default=False,
                    help="overlapped engine steps: ~7 %% lower TPOT for a few ms more TTFT (a request arriving "
                         "while a step is in flight misses that step; profiles/r5/overlap/README.md)")
    ap.add_argument("--kv-cache-dtype", choices=("bf16", "fp8"), default="bf16")
    ap.add_argument("--decode-weights", choices=("bf16", "fp8"), default="bf16")
    ap.add_argument("--prefill-weights", choices=("bf16", "fp8"), default="bf16",
                    help="fp8: W8A8 projections in prefill and mixed (chunked-prefill) steps")
    ap.add_argument("--data-parallel", type=int, default=1,
                    help="replicas, one engine process per GPU (cuda:0 .. N-1) behind this front end")
    ap.add_argument("--engine-process", action=argparse.BooleanOptionalAction, default=True,
                    help="run the engine in its own process so HTTP/SSE work and engine steps do not share one "
                         "interpreter lock (measured +11%% output tok/s at 64-256 streaming clients; "
                         "--no-engine-process keeps it on a thread of the server)")
    a = ap.parse_args(argv)
    import uvicorn

    from kgs.models.llama import LlamaConfig

    from .engine import EngineConfig, LLMEngine

    mc = LlamaConfig.llama3_8b(layers=a.layers)
    ec = EngineConfig(max_batch=a.max_batch, max_model_len=a.max_model_len, cuda_graphs=not a.no_graphs,
                      chunked_prefill=a.chunked_prefill, prefix_caching=a.prefix_caching,
                      kv_cache_dtype=a.kv_cache_dtype, decode_weights=a.decode_weights,
                      prefill_weights=a.prefill_weights, overlap=a.overlap)
    if a.data_parallel > 1 or a.engine_process:
        import dataclasses

        from .dp import DPEngineLoop

        runner = DPEngineLoop(max(1, a.data_parallel), dataclasses.asdict(mc), ec, device=a.device,
                              backend=a.backend, warmup_widths=[8, 32])
    else:
        eng = LLMEngine(mc, ec, device=a.device, backend=a.backend)
        eng.warmup(widths=[8, 32])
        runner = EngineLoop(eng)
    app = create_app(runner, HFTokenizer(a.tokenizer) if a.tokenizer else None, a.model_name)
    try:
        uvicorn.run(app, host=a.host, port=a.port, log_level="info")
    finally:
        runner.shutdown()
    return 0
