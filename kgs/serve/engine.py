"""LLM serving engine: native continuous-batching scheduler + paged-KV model
runner + sampler, with hipGraph-captured decode steps.

One engine step = one scheduler plan (``kgs._native._serve``): a prefill of newly
admitted prompts, or a decode of every running sequence. Decode steps are
padded to a batch bucket (1, 2, 4, ..., max_batch) and a page-table width
bucket and replayed from a captured hipGraph per (batch, width) pair, so the
~260 kernel launches of a Llama-3-8B step cost one graph launch. Padded rows
point at the scheduler's null page 0 and write nothing (slot -1).

:meth:`LLMEngine.generate` is the offline API; :mod:`kgs.serve.api` drives
:meth:`LLMEngine.step` from a background thread for the HTTP server.
"""
from __future__ import annotations

import itertools
import math
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from kgs.models.llama import LlamaConfig
from kgs.ops.decode import PAGE, PagedKVCache

from .model import ServingModel, gate_up_panel_widths
from .trace import TRACE


@dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 0.0   # 0 = greedy
    top_k: int = 0             # 0 = full vocabulary
    top_p: float = 1.0         # nucleus: smallest set of tokens whose probability reaches top_p
    ignore_eos: bool = False
    stop_token_ids: tuple = ()
    logprobs: int | None = None  # None: off; k >= 0: the sampled token's logprob + the k most likely
    presence_penalty: float = 0.0   # OpenAI: minus this once for every token already generated
    frequency_penalty: float = 0.0  # OpenAI: minus this times the token's count in the output
    repetition_penalty: float = 1.0  # CTRL/HF: logits of prompt+output tokens divided (>0) / multiplied (<0)
    seed: int | None = None          # per-request sampling generator (reproducible regardless of batch mates)


@dataclass
class Request:
    id: int
    prompt: list
    params: SamplingParams
    output: list = field(default_factory=list)
    finished: bool = False
    finish_reason: str | None = None
    t_arrival: float = 0.0
    t_first: float | None = None
    t_done: float | None = None
    # per output token, when params.logprobs is set: (logprob, [(token, logprob)] top-k),
    # from the model's distribution before temperature / top-k / top-p
    logprobs: list = field(default_factory=list)
    gen: object = None  # torch.Generator of a seeded request


@dataclass
class EngineConfig:
    num_pages: int | None = None      # None: size from free HBM (kv_fraction)
    kv_fraction: float = 0.85         # of the memory left after weights
    max_batch: int = 256
    max_prefill_tokens: int = 16384
    max_model_len: int = 8192
    eos_token_id: int = 2
    cuda_graphs: bool = True
    fused_max_batch: int = 48         # decode batches up to this use the fused skinny-GEMM layer; above: four-wave GEMMs (measured crossover)
    decode_weights: str = "bf16"      # "fp8": weight-only fp8 decode copies (W8A16)
    kv_cache_dtype: str = "bf16"      # "fp8": e4m3 KV pages
    chunked_prefill: int = 0          # > 0: mixed steps of at most this many rows (prompt chunks + decodes)
    prefix_caching: bool = False      # reuse cached KV pages of shared prompt prefixes (runs on mixed steps)
    packed_decode: bool = True        # prepacked skinny-GEMM decode copies (False: one weight copy, e.g. 70B)
    prefill_weights: str = "bf16"     # "fp8": W8A8 prompt pass (e4m3 weight copies, per-row activation scales)
    fuse_splitk: bool = True          # split-K decode partials reduced inside RoPE/KV-write and add+RMSNorm
    w4x_panels: bool = True           # tile-panel copies of the split-K decode projections (qkv, o, down)
    gate_up_panels: bool = True       # SwiGLU tile-panel copies of gate|up for the unsplit decode routes
    overlap: bool = True              # plan/launch step t+1 before step t's tokens are read back (LLMEngine.step)
    seed: int = 0


def _bucket(n: int, cap: int) -> int:
    b = 1
    while b < n:
        b *= 2
    return min(b, cap)


class LLMEngine:
    def __init__(self, model_cfg: LlamaConfig, cfg: EngineConfig | None = None, device="cuda", backend: str = "kgs"):
        from kgs._native import _serve

        self.cfg = cfg = cfg or EngineConfig()
        self.device = torch.device(device)
        self.backend = backend
        num_pages = cfg.num_pages or self._pages_from_memory(model_cfg)
        self.model = ServingModel(model_cfg, device=device, backend=backend, seed=cfg.seed, num_pages=num_pages,
                                  max_model_len=cfg.max_model_len, fused_max_batch=cfg.fused_max_batch,
                                  decode_weights=cfg.decode_weights, kv_cache_dtype=cfg.kv_cache_dtype,
                                  packed_decode=cfg.packed_decode, prefill_weights=cfg.prefill_weights,
                                  fuse_splitk=cfg.fuse_splitk, w4x_panels=cfg.w4x_panels,
                                  gate_up_panels=cfg.gate_up_panels)
        sc = _serve.SchedulerConfig()
        sc.num_pages, sc.page_size, sc.max_batch = num_pages, PAGE, cfg.max_batch
        sc.max_prefill_tokens, sc.max_model_len, sc.pad_multiple = cfg.max_prefill_tokens, cfg.max_model_len, 128
        sc.chunk_tokens = cfg.chunked_prefill
        sc.prefix_caching = cfg.prefix_caching
        self.sched = _serve.Scheduler(sc)
        self.num_pages = num_pages
        self.requests: dict[int, Request] = {}
        self._ids = itertools.count()
        self._graphs: dict = {}
        self._gen = torch.Generator(device=self.device).manual_seed(cfg.seed)
        self.stats = {"prefill_steps": 0, "decode_steps": 0, "prefill_tokens": 0, "decode_tokens": 0,
                      "mixed_steps": 0, "preemptions": 0, "graph_replays": 0, "graph_captures": 0}
        # per-op synchronisation (fault attribution, kgs.serve.trace) cannot run inside a capture
        self.use_graphs = cfg.cuda_graphs and self.device.type == "cuda" and backend == "kgs" and not TRACE.sync_ops
        self.vocab = model_cfg.vocab
        self.validate = True  # host-side range checks of every step's device inputs (_check_plan)
        # KGS_TQ_CHECK=1: the persistent GEMMs' ticket pool checked after every step (kgs.ops._lib.tile_queue_check)
        self.tq_check = os.environ.get("KGS_TQ_CHECK", "0") == "1" and self.device.type == "cuda"
        # KGS_GRAPH_AUDIT=1: keep each captured hipGraph and record its node types and memset nodes
        # (kgs.utils.graph_audit; a memset node caused the round-5 serving fault)
        from kgs.utils import graph_audit

        self.graph_audit = graph_audit.enabled() and self.device.type == "cuda"
        self.graph_audits: dict = {}
        self._want_lp: set = set()
        self._want_pen: set = set()
        self._seeded: set = set()
        self._watch_eos: set = set()  # requests whose tokens are checked for EOS / stop ids
        # Overlapped steps: step t+1 is planned and launched while step t runs,
        # and step t's tokens are read back after that (see step()). The debug
        # modes synchronise per step: those run one step at a time.
        self.overlap = cfg.overlap and not self.tq_check and not TRACE.sync_ops
        self._inflight: dict | None = None
        self._arrived = False  # add_request since the last plan (see step())
        # KGS_HOST_PHASES=1: per step, the host time of each phase (host_phases()), to find host stalls
        self._phases = [] if os.environ.get("KGS_HOST_PHASES", "0") == "1" else None
        self._pinned = None  # two host buffers the in-flight tokens are copied into, alternately
        self._flip = 0

    def _pages_from_memory(self, mc: LlamaConfig) -> int:
        if self.device.type != "cuda":
            return 256
        free, _ = torch.cuda.mem_get_info(self.device)
        h, i, kvd = mc.hidden, mc.intermediate, mc.kv_heads * mc.head_dim
        per_layer = h * (h + 2 * kvd) + h * h + 2 * h * i + i * h
        weights = 2 * (mc.layers * per_layer + 2 * mc.vocab * h)
        # the kgs backend keeps prefill-order and prepacked decode copies of every projection
        copies = (1.5 if self.cfg.decode_weights == "fp8" else 2) if self.cfg.packed_decode else 1
        copies += 0.5 if self.cfg.prefill_weights == "fp8" else 0
        resident = weights * (copies if self.backend == "kgs" else 1)
        if self.backend == "kgs" and self.cfg.packed_decode and self.cfg.fuse_splitk and self.cfg.w4x_panels:
            resident += 2 * mc.layers * (h * (h + 2 * kvd) + h * h + i * h)  # qkv / o / down panel copies
        if (self.backend == "kgs" and self.cfg.packed_decode and self.cfg.fuse_splitk and self.cfg.gate_up_panels
                and os.environ.get("KGS_GATEUP_PANELS", "1") == "1"):
            resident += 2 * mc.layers * 2 * i * h * len(gate_up_panel_widths(2 * i, h))  # gate|up panel copies
        avail = max(0, (free - resident - (8 << 30)) * self.cfg.kv_fraction)
        return int(max(64, avail // PagedKVCache.bytes_per_page(mc.layers, mc.kv_heads, self.cfg.kv_cache_dtype)))

    # ----------------------------------------------------------------- API
    def add_request(self, prompt: list[int], params: SamplingParams | None = None) -> int:
        params = params or SamplingParams()
        rid = next(self._ids)
        if not self.sched.add(rid, np.asarray(prompt, dtype=np.int32), int(params.max_tokens)):
            raise ValueError(f"request does not fit: prompt {len(prompt)} + max_tokens {params.max_tokens} "
                             f"(max_model_len {self.cfg.max_model_len}, {self.num_pages} pages)")
        self.requests[rid] = Request(rid, list(prompt), params, t_arrival=time.perf_counter())
        # requests that need per-row work after the model step (the common greedy /
        # plain-sampling batch skips those scans entirely)
        if params.logprobs is not None:
            self._want_lp.add(rid)
        if params.presence_penalty or params.frequency_penalty or params.repetition_penalty != 1.0:
            self._want_pen.add(rid)
        if params.seed is not None:
            self._seeded.add(rid)
        if not params.ignore_eos:
            self._watch_eos.add(rid)
        self._arrived = True
        return rid

    def abort(self, rid: int) -> None:
        self._want_lp.discard(rid)
        self._want_pen.discard(rid)
        self._seeded.discard(rid)
        self._watch_eos.discard(rid)
        if self.sched.abort(rid):
            r = self.requests[rid]
            r.finished, r.finish_reason, r.t_done = True, "abort", time.perf_counter()
            self.sched.release(rid)

    def has_work(self) -> bool:
        return self._inflight is not None or self.sched.num_waiting + self.sched.num_running > 0

    def _overlap_now(self) -> bool:
        """Whether the next step may be planned before the current one's tokens
        are known: logprobs, penalties and seeded sampling read per-step host
        state (the output so far, per-request generators), so a batch holding
        any of them runs one step at a time."""
        return self.overlap and not (self._want_lp or self._want_pen or self._seeded)

    def step(self) -> list[tuple[int, int, bool]]:
        """Run one scheduler step; returns [(request id, new token, finished)].

        Overlapped (EngineConfig.overlap, the default): step t+1 is scheduled
        and launched while step t still runs on the GPU, and step t's tokens
        are read back only after that, so the host's share of a step (the
        scheduler, the result loop, staging the next inputs: 2.9 % of a
        batch-256 step, profiles/r5/decode/decode_step_period_b256_o128.txt)
        hides behind the GPU's. The scheduler advances step t's sequences by a
        pending token (Scheduler.update_pending); step t+1 takes their tokens
        straight from step t's sampled tokens on the device, and the values are
        written into the scheduler afterwards (fill_pending). A sequence that
        stops on EOS is seen one step late: it is finished then, and the token
        its extra step computed is dropped. Each call then returns the results
        of the step launched by the call before."""
        ph = self._phases
        t = [time.perf_counter()] if ph is not None else None
        prev = self._inflight
        if prev is not None and (not self._overlap_now() or self._arrived):
            # a request added since the step in flight was planned would only join
            # the step after next (one more step to its first token): finish the
            # step in flight first and plan the next one with it, as the
            # sequential engine does; overlap resumes from there
            self._inflight = None
            self._arrived = False
            return self._complete(prev, advanced=None)
        self._arrived = False
        advanced = self.sched.update_pending(prev["ids"]) if prev is not None else None
        plan = self.sched.schedule()
        if t is not None:
            t.append(time.perf_counter())  # 1: scheduler
        if plan.kind == 0:
            self._inflight = None
            return self._complete(prev, advanced) if prev is not None else []
        self.stats["preemptions"] += len(plan.preempted)
        ids = plan.seq_ids
        if self.validate:
            self._check_plan(plan)
        nstep = sum(self.stats[k] for k in ("prefill_steps", "decode_steps", "mixed_steps"))
        TRACE.mark(f"step {nstep} kind={plan.kind} seqs={len(ids)} rows={len(plan.tokens)} begin")
        if plan.kind == 3:
            logits = self._run_mixed(plan, self._pending_tokens(plan, prev))
            npf = plan.n_prefill
            # only chunks that complete their prompt produce a token
            ids = np.concatenate([ids[:npf][plan.last_chunk.astype(bool)], ids[npf:]])
            self.stats["mixed_steps"] += 1
            self.stats["prefill_tokens"] += int(plan.seq_lens.sum())
            self.stats["decode_tokens"] += len(plan.seq_ids) - npf
            if len(ids) == 0:  # nothing sampled: only the step in flight has results
                self._inflight = None
                return self._complete(prev, advanced) if prev is not None else []
        elif plan.kind == 1:
            logits = self._run_prefill(plan, self._pending_tokens(plan, prev))
            self.stats["prefill_steps"] += 1
            self.stats["prefill_tokens"] += int(plan.seq_lens.sum())
        else:
            tok = self._pending_tokens(plan, prev)
            if t is not None:
                t.append(time.perf_counter())  # 2: plan checks + input tokens
            logits = self._run_decode(plan, tok)
            self.stats["decode_steps"] += 1
            self.stats["decode_tokens"] += len(ids)
        if t is not None:
            t += [time.perf_counter()] * (4 - len(t))  # 3: launch
        toks_dev = self._sample(ids, logits)
        if self._overlap_now():
            self._inflight = self._launch_readback(ids, toks_dev, nstep)
            if t is not None:
                t.append(time.perf_counter())  # 4: sampler + read-back launch
            out = self._complete(prev, advanced, t) if prev is not None else []
            if t is not None:
                ph.append((plan.kind, *[round((b - a) * 1e6, 1) for a, b in zip(t, t[1:])]))
            return out
        lps = self._logprobs(ids, logits, toks_dev)
        toks = toks_dev.cpu().numpy().astype(np.int32)
        TRACE.mark(f"step {nstep} end")
        self._tq_check(nstep, plan.kind)
        eos = self._eos_mask(ids, toks)
        done = set(int(d) for d in self.sched.update(ids, toks, eos))
        return self._emit(ids, toks, eos, done, lps)

    # ------------------------------------------------------- step helpers
    def _launch_readback(self, ids, toks_dev: torch.Tensor, nstep: int) -> dict:
        """Start the copy of an in-flight step's tokens to the host."""
        cur = {"ids": ids, "dev": toks_dev, "nstep": nstep, "event": None}
        if toks_dev.is_cuda:
            if self._pinned is None:
                self._pinned = [torch.empty(self.cfg.max_batch, dtype=torch.int64).pin_memory() for _ in range(2)]
            buf = self._pinned[self._flip][:len(ids)]
            self._flip ^= 1
            buf.copy_(toks_dev, non_blocking=True)
            cur["host"], cur["event"] = buf, torch.cuda.Event()
            cur["event"].record()
        else:
            cur["host"] = toks_dev
        return cur

    def host_phases(self) -> list:
        """KGS_HOST_PHASES=1: per overlapped step (kind, us in the scheduler, the
        plan checks + input tokens, the launch, the sampler + read-back launch,
        the wait for the previous step's tokens, the result loop)."""
        return list(self._phases or [])

    def _complete(self, cur: dict, advanced, t=None) -> list[tuple[int, int, bool]]:
        """Results of an in-flight step. ``advanced``: the ids update_pending
        finished (the scheduler already moved past this step; its tokens are
        filled in and EOS stops applied now), or None (a plain update)."""
        if cur["event"] is not None:
            cur["event"].synchronize()
        if t is not None:
            t.append(time.perf_counter())  # 5: wait for the previous step's tokens
        ids = cur["ids"]
        toks = cur["host"].numpy().astype(np.int32)
        TRACE.mark(f"step {cur['nstep']} end")
        self._tq_check(cur["nstep"], -1)
        eos = self._eos_mask(ids, toks)
        if advanced is None:
            done = set(int(d) for d in self.sched.update(ids, toks, eos))
        else:
            self.sched.fill_pending(ids, toks)
            done = set(int(d) for d in advanced)
            for j in np.flatnonzero(eos):  # EOS seen one step late: the extra step's token is dropped
                rid = int(ids[j])
                if rid not in done and self.sched.abort(rid):
                    done.add(rid)
        out = self._emit(ids, toks, eos, done, None)
        if t is not None:
            t.append(time.perf_counter())  # 6: result loop
        return out

    def _pending_tokens(self, plan, prev) -> torch.Tensor | None:
        """A plan's input tokens on the device when some are still pending in
        the scheduler: those come from the in-flight step's sampled tokens
        (same sequence, on the device), the rest from the plan. A pending token
        is a sequence's last one: a decode row, or the last row of a prompt
        chunk that re-computes a preempted sequence."""
        pend = plan.tokens == self.sched.PENDING
        if prev is None or not pend.any():
            return None
        pids, sid = prev["ids"], self._row_seqs(plan)
        order = np.argsort(pids, kind="stable")
        src = order[np.searchsorted(pids, sid, sorter=order).clip(0, len(pids) - 1)]
        if not np.array_equal(pids[src][pend], sid[pend]):
            raise RuntimeError("overlapped decode: a pending sequence was not in the previous step")
        return self._gather_tokens(prev["dev"], np.where(pend, src, -1), plan.tokens)

    @staticmethod
    def _row_seqs(plan) -> np.ndarray:
        """The sequence id of every input row of a plan."""
        if plan.kind == 2:
            return np.asarray(plan.seq_ids)
        rows = np.full(len(plan.tokens), -1, dtype=np.int64)
        npf = plan.n_prefill if plan.kind == 3 else len(plan.seq_ids)
        for j in range(npf):
            rows[plan.seq_starts[j]:plan.seq_starts[j] + plan.padded_lens[j]] = plan.seq_ids[j]
        nd = len(plan.seq_ids) - npf
        if nd:
            rows[len(rows) - nd:] = plan.seq_ids[npf:]
        return rows

    def _gather_tokens(self, dev: torch.Tensor, src: np.ndarray, tokens: np.ndarray) -> torch.Tensor:
        """tokens[j] = dev[src[j]] where src[j] >= 0, else the host's tokens[j]."""
        if (src >= 0).all() and np.array_equal(src, np.arange(len(src))):
            return dev[:len(src)].to(torch.int32)  # steady state: same sequences, same order
        s = self._dev(src, torch.int64)
        return torch.where(s >= 0, dev.index_select(0, s.clamp(min=0)).to(torch.int32), self._dev(tokens))

    def _eos_mask(self, ids, toks) -> np.ndarray:
        eos = np.zeros(len(ids), dtype=np.uint8)
        if self._watch_eos:
            for j, rid in enumerate(ids):
                rid = int(rid)
                if rid in self._watch_eos:
                    p = self.requests[rid].params
                    t = int(toks[j])
                    if t == self.cfg.eos_token_id or t in p.stop_token_ids:
                        eos[j] = 1
        return eos

    def _emit(self, ids, toks, eos, done: set, lps) -> list[tuple[int, int, bool]]:
        now = time.perf_counter()
        out = []
        for j, rid in enumerate(ids):
            rid = int(rid)
            r = self.requests.get(rid)
            if r is None or r.finished:  # aborted, or finished one step earlier (EOS seen late)
                continue
            r.output.append(int(toks[j]))
            if lps is not None and j in lps:
                r.logprobs.append(lps[j])
            if r.t_first is None:
                r.t_first = now
            fin = rid in done
            if fin:
                r.finished, r.t_done = True, now
                self._want_lp.discard(rid)
                self._want_pen.discard(rid)
                self._seeded.discard(rid)
                self._watch_eos.discard(rid)
                r.finish_reason = "stop" if eos[j] else "length"
                self.sched.release(rid)
            out.append((rid, int(toks[j]), fin))
        return out

    def _tq_check(self, nstep: int, kind: int) -> None:
        if not self.tq_check:
            return
        from kgs.ops._lib import tile_queue_check

        tq = tile_queue_check(self.device.index or 0)
        if tq["dirty_slots"]:
            from kgs.ops._lib import neighbours

            near = neighbours(int(tq["slot_addr"], 16), self.device.index or 0)
            TRACE.mark(f"step {nstep} tile queue dirty {tq} near {near}")
            raise RuntimeError(f"step {nstep} (kind {kind}): persistent-GEMM ticket pool not clean: {tq}; "
                               f"nearest allocator segments: {near}")

    def generate(self, prompts: list[list[int]], params: SamplingParams | list[SamplingParams] | None = None
                 ) -> list[Request]:
        ps = params if isinstance(params, list) else [params or SamplingParams()] * len(prompts)
        rids = [self.add_request(p, q) for p, q in zip(prompts, ps)]
        while self.has_work():
            self.step()
        return [self.requests.pop(r) for r in rids]

    # -------------------------------------------------------------- checks
    def _check_plan(self, plan) -> None:
        """Every index a step's kernels turn into an address, checked on the host
        before it reaches the GPU (microseconds of numpy per step): token ids
        (embedding rows), positions (RoPE table rows), cache slots and block-table
        pages (KV-cache pages) and context lengths. A scheduler bug then raises
        here with the offending values instead of surfacing as an asynchronous
        GPU memory fault with no kernel named."""
        npg, maxpos = self.num_pages, self.cfg.max_model_len
        bad = []

        def rng(name, a, lo, hi):
            a = np.asarray(a)
            if a.size and (a.min() < lo or a.max() >= hi):
                bad.append(f"{name} outside [{lo}, {hi}): min {a.min()} max {a.max()}")

        tok = np.asarray(plan.tokens)
        rng("tokens", tok[tok != self.sched.PENDING], 0, self.vocab)  # pending: the device's own samples
        rng("positions", plan.positions, 0, maxpos)
        rng("slots", plan.slots, -1, npg * PAGE)
        if plan.kind in (2, 3) and len(plan.ctx_lens):
            bt = np.asarray(plan.block_tables)
            ctx = np.asarray(plan.ctx_lens)
            rng("block_tables", bt, 0, npg)
            rng("ctx_lens", ctx, 1, bt.shape[1] * PAGE + 1)
            if not bad and plan.kind == 2:
                # decode: the new token's slot lies in the last page of its context
                last = bt[np.arange(len(ctx)), (ctx - 1) // PAGE]
                sl = np.asarray(plan.slots)
                if np.any((sl >= 0) & (sl // PAGE != last)):
                    bad.append("decode slot not in the last page of its context")
        if plan.kind == 3 and plan.n_prefill:
            rng("pf_block_tables", plan.pf_block_tables, 0, npg)
        if bad:
            raise RuntimeError(f"scheduler plan (kind {plan.kind}, {len(plan.seq_ids)} seqs) failed its checks: "
                               + "; ".join(bad))

    # -------------------------------------------------------------- runners
    def _dev(self, a, dtype=torch.int32):
        t = torch.from_numpy(np.ascontiguousarray(a))
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t.to(dtype)

    def _run_prefill(self, plan, tokens: torch.Tensor | None = None) -> torch.Tensor:
        return self.model.prefill(tokens if tokens is not None else self._dev(plan.tokens),
                                  self._dev(plan.positions), self._dev(plan.slots),
                                  plan.seq_starts.tolist(), plan.seq_lens.tolist(), plan.padded_lens.tolist())

    def _run_mixed(self, plan, tokens: torch.Tensor | None = None) -> torch.Tensor:
        """``tokens``: the input tokens on the device (overlapped steps), else the plan's."""
        npf = plan.n_prefill
        pf_bt = self._dev(plan.pf_block_tables) if npf else None
        chunks = [(int(plan.seq_starts[j]), int(plan.seq_lens[j]), int(plan.padded_lens[j]), int(plan.ctx_starts[j]),
                   pf_bt[j], bool(plan.last_chunk[j])) for j in range(npf)]
        nd = len(plan.seq_ids) - npf
        return self.model.mixed(tokens if tokens is not None else self._dev(plan.tokens), self._dev(plan.positions),
                                self._dev(plan.slots), chunks,
                                self._dev(plan.block_tables) if nd else None,
                                self._dev(plan.ctx_lens) if nd else None)

    def _run_decode(self, plan, tokens: torch.Tensor | None = None) -> torch.Tensor:
        """``tokens``: the input tokens on the device (overlapped steps), else the plan's."""
        b = len(plan.seq_ids)
        if not self.use_graphs:
            return self.model.decode(tokens if tokens is not None else self._dev(plan.tokens),
                                     self._dev(plan.positions), self._dev(plan.slots),
                                     self._dev(plan.block_tables), self._dev(plan.ctx_lens))
        bb = _bucket(b, self.cfg.max_batch)
        wb = _bucket(plan.max_pages, math.ceil(self.cfg.max_model_len / PAGE))
        g = self._graphs.get((bb, wb)) or self._capture(bb, wb)
        io = g["io"]
        # two sets of pinned staging buffers, alternately: with overlapped steps
        # the host fills step t+1's while step t's copies may still be queued
        host, hn = g["host"][g["flip"]], g["host_np"][g["flip"]]  # hn: numpy views of host
        g["flip"] ^= 1
        hn["tokens"][:] = 0
        hn["tokens"][:b] = plan.tokens
        hn["positions"][:] = 0
        hn["positions"][:b] = plan.positions
        hn["slots"][:] = -1
        hn["slots"][:b] = plan.slots
        hn["ctx"][:] = 1
        hn["ctx"][:b] = plan.ctx_lens
        hn["bt"][:] = 0
        hn["bt"][:b, :plan.max_pages] = plan.block_tables
        for k in host:
            io[k].copy_(host[k], non_blocking=True)
        if tokens is not None:
            io["tokens"][:b].copy_(tokens)
        g["graph"].replay()
        self.stats["graph_replays"] += 1
        return g["logits"][:b]

    def _capture(self, bb: int, wb: int):
        """Capture one decode step for batch bucket bb and page-table width wb."""
        def pinned(shape):
            return torch.zeros(shape, dtype=torch.int32).pin_memory()

        host = {"tokens": pinned(bb), "positions": pinned(bb), "slots": pinned(bb), "ctx": pinned(bb),
                "bt": pinned((bb, wb))}
        host["slots"][:] = -1
        host["ctx"][:] = 1
        io = {k: v.to(self.device) for k, v in host.items()}
        run = lambda: self.model.decode(io["tokens"], io["positions"], io["slots"], io["bt"], io["ctx"])  # noqa: E731
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up: workspaces and allocator pools settle before capture
                run()
        torch.cuda.current_stream(self.device).wait_stream(s)
        graph = torch.cuda.CUDAGraph(keep_graph=self.graph_audit)
        with torch.cuda.graph(graph):
            logits = run()
        if self.graph_audit:
            from kgs.utils.graph_audit import audit

            self.graph_audits[(bb, wb)] = audit(graph)
            graph.instantiate()
        host2 = {k: v.clone().pin_memory() for k, v in host.items()}
        g = {"graph": graph, "io": io, "host": [host, host2], "flip": 0,
             "host_np": [{k: v.numpy() for k, v in h.items()} for h in (host, host2)],
             "logits": logits}
        self._graphs[(bb, wb)] = g
        self.stats["graph_captures"] += 1
        return g

    def warmup(self, batches=None, widths=None) -> None:
        """Capture decode graphs ahead of traffic (otherwise captured on first use),
        and run the overlapped steps' token gather once: its first use loads the
        ops' code objects, ~0.1 s the GPU would otherwise spend waiting on the
        first decode after a prefill (profiles/r5/overlap/README.md)."""
        if self.overlap and self.device.type == "cuda":
            dev = torch.zeros(2, dtype=torch.int64, device=self.device)
            self._gather_tokens(dev, np.array([1, -1], np.int64), np.zeros(2, np.int32))
            torch.cuda.synchronize(self.device)
        if not self.use_graphs:
            return
        maxw = math.ceil(self.cfg.max_model_len / PAGE)
        for bb in batches or [1 << i for i in range(int(math.log2(self.cfg.max_batch)) + 1)]:
            for wb in widths or [w for w in (8, 16, 32, 64, 128, 256) if w <= maxw]:
                if (bb, wb) not in self._graphs:
                    self._capture(bb, wb)
        if self.tq_check:  # the captures' eager warm-up runs used the pool too
            from kgs.ops._lib import tile_queue_check

            tq = tile_queue_check(self.device.index or 0)
            TRACE.mark(f"warmup captures done, tile queue {tq}")
            if tq["dirty_slots"]:
                raise RuntimeError(f"after the graph captures: persistent-GEMM ticket pool not clean: {tq}")

    # -------------------------------------------------------------- sampling
    def _logprobs(self, ids, logits: torch.Tensor, toks: torch.Tensor):
        """{row: (logprob of the sampled token, [(token, logprob)] top-k)} for the
        rows whose request asked for logprobs; None when none did."""
        if not self._want_lp:
            return None
        rows = [j for j, r in enumerate(ids) if int(r) in self._want_lp]
        if not rows:
            return None
        sel = torch.as_tensor(rows, device=logits.device)
        lp = torch.log_softmax(logits[sel].float(), dim=-1)
        chosen = lp.gather(1, toks[sel].long()[:, None])[:, 0].cpu().tolist()
        k = max(self.requests[int(ids[j])].params.logprobs for j in rows)
        top_v, top_i = (lp.topk(k, dim=-1) if k > 0 else (lp[:, :0], lp[:, :0].long()))
        top_v, top_i = top_v.cpu().tolist(), top_i.cpu().tolist()
        out = {}
        for n, j in enumerate(rows):
            kj = self.requests[int(ids[j])].params.logprobs
            out[j] = (chosen[n], list(zip(top_i[n][:kj], top_v[n][:kj])))
        return out

    def _penalize(self, ids, logits: torch.Tensor) -> torch.Tensor:
        """Presence / frequency / repetition penalties on the rows that ask for
        them (a per-row token-count vector built from that request's tokens)."""
        if not self._want_pen:
            return logits
        rows = [j for j, r in enumerate(ids) if int(r) in self._want_pen]
        if not rows:
            return logits
        logits = logits.float().clone()
        vocab = logits.shape[1]
        for j in rows:
            r = self.requests[int(ids[j])]
            p = r.params
            if r.output and (p.presence_penalty or p.frequency_penalty):
                cnt = torch.bincount(torch.as_tensor(r.output, device=logits.device), minlength=vocab)[:vocab]
                logits[j] -= p.frequency_penalty * cnt + p.presence_penalty * (cnt > 0)
            if p.repetition_penalty != 1.0:
                seen = torch.as_tensor(sorted(set(r.prompt) | set(r.output)), device=logits.device)
                v = logits[j, seen]
                logits[j, seen] = torch.where(v > 0, v / p.repetition_penalty, v * p.repetition_penalty)
        return logits

    def _sample(self, ids, logits: torch.Tensor) -> torch.Tensor:
        logits = self._penalize(ids, logits)
        ps = [self.requests[int(r)].params for r in ids]
        if all(p.temperature <= 0 for p in ps):
            return self._argmax(logits)
        lf = logits.float()
        temp = torch.tensor([max(p.temperature, 1e-5) for p in ps], device=lf.device)[:, None]
        lf = lf / temp
        ks = [p.top_k for p in ps]
        if any(k > 0 for k in ks):
            kmax = max(ks)
            vals, _ = lf.topk(kmax, dim=-1)
            kth = torch.tensor([k if k > 0 else kmax for k in ks], device=lf.device)[:, None] - 1
            thr = vals.gather(1, kth)
            full = torch.tensor([k <= 0 for k in ks], device=lf.device)[:, None]
            lf = torch.where(full | (lf >= thr), lf, torch.full_like(lf, float("-inf")))
        tp = [p.top_p for p in ps]
        if any(0.0 < t < 1.0 for t in tp):
            # nucleus: keep the highest-probability tokens until their mass reaches
            # top_p (the token that crosses it included); rows with top_p >= 1 keep all
            srt, idx = torch.sort(lf, dim=-1, descending=True)
            cum = torch.softmax(srt, dim=-1).cumsum(dim=-1)
            tpv = torch.tensor([t if 0.0 < t < 1.0 else 1.0 for t in tp], device=lf.device)[:, None]
            drop = (cum - torch.softmax(srt, dim=-1)) >= tpv  # mass before this token already reached top_p
            srt = srt.masked_fill(drop, float("-inf"))
            lf = torch.full_like(lf, float("-inf")).scatter(1, idx, srt)
        probs = torch.softmax(lf, dim=-1)
        sampled = torch.multinomial(probs, 1, generator=self._gen).squeeze(1)
        for j, r in enumerate(ids if self._seeded else ()):  # seeded requests: their own generator
            req = self.requests[int(r)]
            if req.params.seed is not None and req.params.temperature > 0:
                if req.gen is None:
                    req.gen = torch.Generator(device=lf.device).manual_seed(int(req.params.seed))
                sampled[j] = torch.multinomial(probs[j], 1, generator=req.gen)[0]
        greedy = torch.tensor([p.temperature <= 0 for p in ps], device=lf.device)
        return torch.where(greedy, self._argmax(logits), sampled)

    def _argmax(self, logits: torch.Tensor) -> torch.Tensor:
        """Greedy pick: the native row argmax for bf16 GPU logits of the kgs
        backend (torch's generic reduce takes ~40 us for one 128k-vocab row)."""
        if self.backend == "kgs" and logits.is_cuda and logits.dtype == torch.bfloat16 and \
                logits.dim() == 2 and logits.shape[-1] % 8 == 0 and logits.stride(-1) == 1 and \
                logits.stride(0) % 8 == 0 and logits.data_ptr() % 16 == 0:
            from kgs.ops.transformer import argmax_rows

            return argmax_rows(logits)
        return logits.argmax(dim=-1)
