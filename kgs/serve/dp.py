"""Data-parallel serving: one engine process per GPU behind one HTTP front end.

Llama-3-8B needs a fraction of one MI355X (16 GB of 288 GB), so a pod granted
``amd.com/gpu: N`` serves it fastest as N independent replicas: no collective
on the decode critical path, each replica with its own paged KV cache and
hipGraphs. This is the "one process per GPU" layout of the rest of the
framework applied to serving (``kgs.serve serve --data-parallel N``).

:class:`DPEngineLoop` has the interface of :class:`kgs.serve.api.EngineLoop`
(``submit`` / ``cancel`` / ``gauges`` / ``counters`` / ``shutdown``), so the
HTTP layer is unchanged. Each worker process (``spawn``: it initialises only
its own GPU) runs an :class:`~kgs.serve.engine.LLMEngine` on ``cuda:i``; requests
go to the replica with the fewest requests in flight, over a
``multiprocessing`` queue per worker; each worker returns one message per
engine step with all tokens it produced. The front end never touches a GPU.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import queue
import threading


def _worker(index: int, spec: dict, inq, outq) -> None:
    """Replica main: any exception is reported to the front end (which fails
    that replica's requests and stops routing to it) instead of leaving them
    waiting forever."""
    try:
        _serve_replica(index, spec, inq, outq)
    except BaseException:  # noqa: BLE001 -- report everything, then exit
        import traceback

        outq.put(("fatal", index, traceback.format_exc()))


def _serve_replica(index: int, spec: dict, inq, outq) -> None:
    from kgs.models.llama import LlamaConfig

    from .engine import LLMEngine

    device = f"cuda:{index}" if spec["device"] == "cuda" else spec["device"]
    if device.startswith("cuda"):
        import torch

        torch.cuda.set_device(index)
    eng = LLMEngine(LlamaConfig(**spec["model"]), spec["engine"], device=device, backend=spec["backend"])
    if spec.get("warmup_widths"):
        eng.warmup(widths=spec["warmup_widths"])
    outq.put(("ready", index, None))
    gid_of: dict = {}
    rid_of: dict = {}
    while True:
        block = not eng.has_work()
        try:
            msgs = [inq.get(timeout=0.05) if block else inq.get_nowait()]
        except queue.Empty:
            msgs = []
        while True:
            try:
                msgs.append(inq.get_nowait())
            except queue.Empty:
                break
        for m in msgs:
            if m[0] == "stop":
                outq.put(("stopped", index, None))
                return
            if m[0] == "abort":
                rid = rid_of.pop(m[1], None)
                if rid is not None:
                    eng.abort(rid)
                    gid_of.pop(rid, None)
                    eng.requests.pop(rid, None)
                continue
            _, gid, prompt, params = m
            try:
                rid = eng.add_request(prompt, params)
            except ValueError as e:
                outq.put(("error", index, (gid, str(e))))
                continue
            gid_of[rid], rid_of[gid] = gid, rid
            outq.put(("id", index, gid))
        if not eng.has_work():
            continue
        batch = []
        for rid, tok, fin in eng.step():
            gid = gid_of.get(rid)
            if gid is None:
                continue
            req = eng.requests[rid]
            lp = req.logprobs[-1] if req.params.logprobs is not None and req.logprobs else None
            batch.append((gid, tok, fin, req.finish_reason if fin else None, lp))
            if fin:
                gid_of.pop(rid, None)
                rid_of.pop(gid, None)
                eng.requests.pop(rid, None)
        gauges = {"running": eng.sched.num_running, "waiting": eng.sched.num_waiting,
                  "free_kv_pages": eng.sched.num_free_pages, "preemptions": eng.stats["preemptions"],
                  "prefix_hit_tokens": eng.sched.prefix_hit_tokens}
        outq.put(("step", index, (batch, gauges)))


class DPEngineLoop:
    def __init__(self, replicas: int, model: dict, engine, device: str = "cuda", backend: str = "kgs",
                 warmup_widths=None, start_timeout: float = 900.0):
        ctx = mp.get_context("spawn")
        self.n = replicas
        spec = {"model": model, "engine": engine, "device": device, "backend": backend,
                "warmup_widths": warmup_widths}
        self.inqs = [ctx.Queue() for _ in range(replicas)]
        self.outq = ctx.Queue()
        self.procs = [ctx.Process(target=_worker, args=(i, spec, self.inqs[i], self.outq), daemon=True,
                                  name=f"kgs-replica-{i}") for i in range(replicas)]
        for p in self.procs:
            p.start()
        ready = set()
        while len(ready) < replicas:
            try:
                kind, idx, payload = self.outq.get(timeout=start_timeout)
            except queue.Empty:
                self.shutdown()
                raise RuntimeError(f"data-parallel replicas not ready after {start_timeout} s")
            if kind == "ready":
                ready.add(idx)
            elif kind == "fatal":
                self.shutdown()
                raise RuntimeError(f"replica {idx} failed to start:\n{payload}")
        self.counters = {"requests": 0, "rejected": 0, "tokens": 0, "steps": 0}
        self.assigned = [0] * replicas  # requests routed to each replica (tests, logs)
        self._inflight = [0] * replicas
        self._gauges = [{"running": 0, "waiting": 0, "free_kv_pages": 0, "preemptions": 0,
                         "prefix_hit_tokens": 0} for _ in range(replicas)]
        self._streams: dict = {}
        self._dead: set = set()
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._pump, name="kgs-dp-pump", daemon=True)
        self._thread.start()

    # -- EngineLoop interface -------------------------------------------------
    def submit(self, prompt, params, loop, q) -> None:
        with self._lock:
            gid = next(self._ids)
            live = [i for i in range(self.n) if i not in self._dead]
            if not live:
                loop.call_soon_threadsafe(q.put_nowait, ("error", "no live replica"))
                return
            w = min(live, key=lambda i: (self._inflight[i], i))
            self._inflight[w] += 1
            self.assigned[w] += 1
            self._streams[gid] = (loop, q, w)
        self.inqs[w].put(("add", gid, list(prompt), params))

    def cancel(self, gid: int) -> None:
        with self._lock:
            st = self._streams.pop(gid, None)
            if st is not None:
                self._inflight[st[2]] -= 1
        if st is not None:
            self.inqs[st[2]].put(("abort", gid))

    def gauges(self) -> dict:
        with self._lock:
            return {k: sum(g[k] for g in self._gauges) for k in self._gauges[0]}

    def shutdown(self) -> None:
        if hasattr(self, "_stop"):
            self._stop.set()
        for q in self.inqs:
            q.put(("stop",))
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
                p.join(timeout=5)

    # -- token pump -----------------------------------------------------------
    def _push(self, st, item) -> None:
        st[0].call_soon_threadsafe(st[1].put_nowait, item)

    def _pump(self) -> None:
        while not self._stop.is_set():
            try:
                kind, idx, payload = self.outq.get(timeout=0.1)
            except queue.Empty:
                continue
            with self._lock:
                if kind == "id":
                    st = self._streams.get(payload)
                    self.counters["requests"] += 1
                    if st is not None:
                        self._push(st, ("id", payload))
                elif kind == "error":
                    gid, msg = payload
                    st = self._streams.pop(gid, None)
                    self.counters["rejected"] += 1
                    if st is not None:
                        self._inflight[st[2]] -= 1
                        self._push(st, ("error", msg))
                elif kind == "fatal":
                    # the replica died: fail its requests, route around it
                    self._dead.add(idx)
                    for gid, st in list(self._streams.items()):
                        if st[2] == idx:
                            self._streams.pop(gid)
                            self._inflight[idx] -= 1
                            self._push(st, ("error", f"replica {idx} failed"))
                elif kind == "step":
                    batch, gauges = payload
                    self._gauges[idx] = gauges
                    self.counters["steps"] += 1
                    for gid, tok, fin, reason, lp in batch:
                        self.counters["tokens"] += 1
                        st = self._streams.get(gid)
                        if st is None:
                            continue
                        self._push(st, ("token", tok, fin, reason, lp))
                        if fin:
                            self._streams.pop(gid, None)
                            self._inflight[st[2]] -= 1
