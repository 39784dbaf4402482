"""OpenAI-style HTTP server over :class:`kgs.serve.LLMEngine` -- the kgs
replacement for the vLLM process of ``pods/vllm-rocm-pod.yaml`` (same port
8000, same ``/v1/completions`` request shape; see ``pods/kgs-serve-pod.yaml``).

Endpoints: ``POST /v1/completions`` (prompt as text or token ids; ``stream``
gives server-sent events), ``GET /v1/models``, ``GET /health``, ``GET /metrics``
(Prometheus). One background thread owns the engine (it is not thread-safe) and
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


class CompletionRequest(BaseModel):
    model: str | None = None
    prompt: str | list[int]
    max_tokens: int = 16
    temperature: float = 0.0
    top_k: int = 0
    stream: bool = False
    ignore_eos: bool = False


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
                reason = eng.requests[rid].finish_reason if fin else None
                self._push(st[0], st[1], ("token", tok, fin, reason))
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
        eng = loop_runner.engine
        c = loop_runner.counters
        lines = [
            "# TYPE kgs_requests_total counter", f"kgs_requests_total {c['requests']}",
            "# TYPE kgs_requests_rejected_total counter", f"kgs_requests_rejected_total {c['rejected']}",
            "# TYPE kgs_generated_tokens_total counter", f"kgs_generated_tokens_total {c['tokens']}",
            "# TYPE kgs_engine_steps_total counter", f"kgs_engine_steps_total {c['steps']}",
            "# TYPE kgs_running gauge", f"kgs_running {eng.sched.num_running}",
            "# TYPE kgs_waiting gauge", f"kgs_waiting {eng.sched.num_waiting}",
            "# TYPE kgs_free_kv_pages gauge", f"kgs_free_kv_pages {eng.sched.num_free_pages}",
            "# TYPE kgs_preemptions_total counter", f"kgs_preemptions_total {eng.stats['preemptions']}",
        ]
        return PlainTextResponse("\n".join(lines) + "\n")

    @app.post("/v1/completions")
    async def completions(req: CompletionRequest):
        ids = tok.encode(req.prompt) if isinstance(req.prompt, str) else list(req.prompt)
        if not ids:
            raise HTTPException(400, "empty prompt")
        params = SamplingParams(max_tokens=req.max_tokens, temperature=req.temperature, top_k=req.top_k,
                                ignore_eos=req.ignore_eos)
        q: asyncio.Queue = asyncio.Queue()
        loop_runner.submit(ids, params, asyncio.get_running_loop(), q)
        first = await q.get()
        if first[0] == "error":
            raise HTTPException(400, first[1])
        rid = first[1]
        cid, created = f"cmpl-{uuid.uuid4().hex[:16]}", int(time.time())
        name = req.model or model_name

        if req.stream:
            async def events():
                try:
                    while True:
                        _, t, fin, reason = await q.get()
                        chunk = {"id": cid, "object": "text_completion", "created": created, "model": name,
                                 "choices": [{"index": 0, "text": tok.decode([t]), "token_ids": [t],
                                              "finish_reason": reason}]}
                        yield f"data: {json.dumps(chunk)}\n\n"
                        if fin:
                            break
                    yield "data: [DONE]\n\n"
                except asyncio.CancelledError:  # client went away
                    loop_runner.cancel(rid)
                    raise

            return StreamingResponse(events(), media_type="text/event-stream")

        out, reason = [], None
        while True:
            _, t, fin, reason = await q.get()
            out.append(t)
            if fin:
                break
        return {"id": cid, "object": "text_completion", "created": created, "model": name,
                "choices": [{"index": 0, "text": tok.decode(out), "token_ids": out, "finish_reason": reason}],
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(out),
                          "total_tokens": len(ids) + len(out)}}

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
    a = ap.parse_args(argv)
    import uvicorn

    from kgs.models.llama import LlamaConfig

    from .engine import EngineConfig, LLMEngine

    eng = LLMEngine(LlamaConfig.llama3_8b(layers=a.layers),
                    EngineConfig(max_batch=a.max_batch, max_model_len=a.max_model_len, cuda_graphs=not a.no_graphs),
                    device=a.device, backend=a.backend)
    eng.warmup(widths=[8, 32])
    runner = EngineLoop(eng)
    app = create_app(runner, HFTokenizer(a.tokenizer) if a.tokenizer else None, a.model_name)
    try:
        uvicorn.run(app, host=a.host, port=a.port, log_level="info")
    finally:
        runner.shutdown()
    return 0
