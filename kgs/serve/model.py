"""Paged-KV Llama model runner for :mod:`kgs.serve` (BASELINE config 5 stand-in:
Llama-3-8B bf16, TP=1, one MI355X).

Two step kinds, both driven by the native scheduler's plans
(``native/serve/scheduler.cpp``):

* **prefill** -- the prompts of newly admitted sequences, each padded to a
  multiple of 128 tokens and concatenated: every projection is one
  :func:`kgs.ops.gemm_nt` (256x256 MFMA pipeline), RoPE + the KV-cache scatter
  is one :func:`kgs.ops.decode.rope_cache_` launch, attention is the
  flash-attention forward per sequence, and only the last real token of each
  sequence goes through the LM head;
* **decode** -- one token per running sequence; attention is
  :func:`kgs.ops.decode.paged_decode_attention` over the paged cache. Batches up
  to ``fused_max_batch`` run the FUSED layer: five
  :func:`kgs.ops.decode.skinny_gemm` launches over prepacked weights whose
  epilogues carry the RMSNorms (norm weights folded into the weights, row
  scales from sums of squares the residual-updating GEMMs accumulate), the
  residual adds and SwiGLU -- no elementwise kernels. Larger batches use
  add_rmsnorm/silu_mul and hipBLASLt, with the split-K 256x256 GEMM
  (:func:`kgs.ops.decode.splitk_slices`), the skinny GEMM
  (:func:`kgs.ops.decode.use_skinny`) or the 256x256 GEMM (LM head) where
  those measured faster.

``decode_weights="fp8"``: the decode copies are weight-only fp8 (W8A16, one
scale per output row, dequantised in registers), halving the weight bytes a
decode step streams; prefill and batches above the fused path stay bf16.

``kv_cache_dtype="fp8"``: e4m3 KV pages (scale 1), dequantised in the decode
attention's registers -- half the KV bytes per decode step.

``backend="ref"`` runs the same weights, cache layout and plans through plain
PyTorch (CPU or GPU) -- the numerics reference for tests.

Weights are random-init (no network, no checkpoint) with the same generator
scheme as :class:`kgs.models.llama.LlamaModel`, whose ``forward`` (no cache) is
the full-recompute oracle the tests compare generations against.
"""
from __future__ import annotations

import os

import torch

from kgs.models.llama import LlamaConfig, LlamaModel, _rms_norm
from kgs.ops import decode as D

from .trace import TRACE as T


def gate_up_panel_widths(n: int, k: int) -> set:
    """Tile widths of the unsplit SwiGLU decode routes for a gate|up of shape
    (n, k) (kgs.ops.decode.W4X_TUNED): one tile-panel copy is made per width."""
    return {r[0] for (_, rn, rk), r in D.W4X_TUNED.items() if (rn, rk) == (n, k) and r[1] == 1}


class ServingModel:
    def __init__(self, cfg: LlamaConfig, device="cuda", backend: str = "kgs", seed: int = 0,
                 num_pages: int = 1024, max_model_len: int = 8192, fused_max_batch: int = 48,
                 decode_weights: str = "bf16", kv_cache_dtype: str = "bf16", packed_decode: bool = True,
                 prefill_weights: str = "bf16", fuse_splitk: bool = True, w4x_panels: bool = True,
                 gate_up_panels: bool = True):
        if cfg.head_dim != D.HEAD_DIM:
            raise ValueError(f"head_dim must be {D.HEAD_DIM}")
        self.cfg, self.backend, self.device = cfg, backend, torch.device(device)
        # decode projections on the four-wave kernel fuse into their neighbours:
        # split-K partials go straight to the next op (RoPE + KV write after
        # qkv, residual add + RMSNorm after o and down) instead of a reduce
        # launch, and an unsplit gate|up applies SwiGLU in its epilogue
        self.fuse_splitk = fuse_splitk and backend == "kgs"
        # split-K qkv decode layers: reduce + RoPE + KV write inside the attention
        # launch (KGS_ROPE_ATTN=1). Off by default: measured 2.9 % slower at batch
        # 256 (attention 86 -> 105 us against the 10 us rope_cache it replaces;
        # profiles/r3/decode/README.md, run r3r)
        self.rope_attn = os.environ.get("KGS_ROPE_ATTN", "0") == "1"
        base = LlamaModel(cfg, device=device, backend="torch" if backend == "ref" else "kgs", seed=seed)
        self.oracle = base  # same weights, full-recompute forward (tests)
        self.embed, self.norm = base.embed, base.norm
        self.ln1 = [L["ln1"] for L in base.layers]
        self.ln2 = [L["ln2"] for L in base.layers]
        self.w = [{n: base.layers[i][n].w for n in ("qkv", "o", "gate_up", "down")} for i in range(cfg.layers)]
        self.w_lm = base.lm_head.w
        self.packed = None
        self.fused_max_batch = fused_max_batch
        if decode_weights not in ("bf16", "fp8"):
            raise ValueError(f"decode_weights must be bf16 or fp8, got {decode_weights!r}")
        self.decode_fp8 = decode_weights == "fp8"
        if self.decode_fp8:
            self.fused_max_batch = min(fused_max_batch, 64)  # the W8A16 skinny GEMM covers M <= 64
        if backend == "kgs" and not packed_decode:
            # no prepacked decode copies (e.g. Llama-3-70B: one bf16 copy of the
            # weights is 141 GB): decode runs on the library/split-K GEMMs
            if self.decode_fp8:
                raise ValueError("decode_weights='fp8' needs the packed decode copies")
            self.fused_max_batch = 0
            D.reserve_workspace(self.device)
        elif backend == "kgs":
            f8 = self.decode_fp8
            # decode copies in skinny-GEMM fragment order; the RMSNorm weights
            # in front of qkv / gate|up / lm_head are folded into them (their
            # GEMMs apply the norm in the epilogue), gate|up is SwiGLU-packed,
            # and with bf16 weights and a bf16 cache qkv is RoPE-packed (its
            # epilogue rotates q / k and writes the KV cache)
            rope = None if f8 or kv_cache_dtype != "bf16" else (cfg.heads, cfg.kv_heads)
            self.packed = [{"qkv": D.PackedWeight(lw["qkv"], fold=self.ln1[i], fp8=f8, rope=rope),
                            "o": D.PackedWeight(lw["o"], fp8=f8),
                            "gate_up": D.PackedWeight(lw["gate_up"], swiglu=True, fold=self.ln2[i], fp8=f8),
                            "down": D.PackedWeight(lw["down"], fp8=f8)} for i, lw in enumerate(self.w)]
            self.packed_lm = D.PackedWeight(self.w_lm, fold=self.norm, fp8=f8)
            D.reserve_workspace(self.device)
        # split-K decode projections (qkv, o, down from batch 64 up, kgs.ops.decode
        # W4X_TUNED) read a third copy laid out tile-panel major, so each K-step's
        # weight block is one contiguous HBM run (PACKB): 5-6 % off the down
        # projection at batch 128/256 (profiles/r3/decode/README.md). 6.4 GB for
        # Llama-3-8B; kept only with the other decode copies
        self.w4x_panels = None
        if self.fuse_splitk and packed_decode and w4x_panels:
            from kgs.ops.gemm import pack_w4x_weight

            bns = {n: D.w4x_split_bns(*self.w[0][n].shape) for n in ("qkv", "o", "down")}
            self.w4x_panels = [{(n, bn): pack_w4x_weight(lw[n], bn) for n in bns for bn in bns[n]}
                               for lw in self.w]
        # SwiGLU tile-panel copies of gate|up (235 MB per layer and tile width,
        # 15 GB for Llama-3-8B) for the unsplit decode routes: with non-temporal
        # weight loads they read 4 % faster than row-major at batch 256 (64.9 vs
        # 68.0 us, profiles/r4/decode/README.md); batch-256 serving 18 302 ->
        # 18 442 output tok/s (profiles/r5/decode/README.md). Off:
        # gate_up_panels=False or KGS_GATEUP_PANELS=0.
        self.gate_up_panels = None
        if (self.fuse_splitk and packed_decode and gate_up_panels
                and os.environ.get("KGS_GATEUP_PANELS", "1") == "1"):
            from kgs.ops.gemm import pack_w4x_weight

            gbns = gate_up_panel_widths(*self.w[0]["gate_up"].shape)
            self.gate_up_panels = [{bn: pack_w4x_weight(lw["gate_up"], bn, swiglu=True) for bn in gbns}
                                   for lw in self.w]
        if prefill_weights not in ("bf16", "fp8"):
            raise ValueError(f"prefill_weights must be bf16 or fp8, got {prefill_weights!r}")
        self.prefill_f8 = None
        if prefill_weights == "fp8" and backend == "kgs":
            # W8A8 prefill (e4m3 weights, per-tensor scale; activations quantised per
            # row by the fused norm / SwiGLU producers): ~2x the bf16 GEMM rate on the
            # compute-bound prompt pass; decode and the oracle keep the bf16 weights
            from kgs.ops import Fp8Linear

            self.prefill_f8 = [{n: Fp8Linear(lw[n]) for n in ("qkv", "o", "gate_up", "down")} for lw in self.w]
        self.cache = D.PagedKVCache(cfg.layers, num_pages, cfg.kv_heads, self.device, dtype=kv_cache_dtype)
        self.max_model_len = max_model_len
        from kgs.ops.transformer import rope_tables

        self.cos, self.sin = rope_tables(max_model_len + 256, cfg.head_dim, cfg.rope_theta, self.device)

    # ------------------------------------------------------------------ utils
    def weight_bytes(self) -> int:
        n = sum(w.numel() for lw in self.w for w in lw.values()) + self.w_lm.numel()
        return 2 * n

    def _proj(self, x: torch.Tensor, layer: int | None, name: str, decode: bool) -> torch.Tensor:
        w = self.w_lm if layer is None else self.w[layer][name]
        if self.backend == "ref":
            return (x.float() @ w.float().T).to(torch.bfloat16)
        m = x.shape[0]
        if decode:
            route = D.w4x_route(m, w.shape[0], w.shape[1])
            if route is not None:
                from kgs.ops.gemm import gemm_nt_w4x

                return gemm_nt_w4x(x, w, bn=route[0], nslice=route[1], bm=route[2], stages=D.w4x_stages(route),
                                   nt_weights=D.w4x_nt(route))
        if decode:
            ns = D.splitk_slices(m, w.shape[0], w.shape[1])
            if ns == 1:
                from kgs.ops import gemm_nt

                return gemm_nt(x, w)
            if ns is not None:
                from kgs.ops.gemm import gemm_nt_splitk

                return gemm_nt_splitk(x, w, ns)
        if decode and self.packed is not None and name in ("o", "down") and D.use_skinny(m, w.shape[0], w.shape[1]) and \
                not (self.decode_fp8 and m > 64):
            return D.skinny_gemm(x, self.packed[layer][name])
        # the LM head (N = 128256) from batch 128 up runs faster on the kgs
        # 256x256 GEMM than on hipBLASLt (1.09x at 128, 1.21x at 256,
        # profiles/decode_wide_gemm.jsonl); the other decode shapes do not
        if decode and (layer is not None or m < 128):
            return torch.matmul(x, w.T)
        from kgs.ops import gemm_nt

        return gemm_nt(x, w)

    def _splitk_route(self, m: int, layer: int, name: str):
        """(bn, nslice) when this decode projection runs split-K on the
        four-wave kernel and its reduce can be fused into the consumer."""
        if not self.fuse_splitk:
            return None
        w = self.w[layer][name]
        r = D.w4x_route(m, w.shape[0], w.shape[1])
        if r is None or r[1] < 2:
            return None
        if name in ("o", "down") and self.cfg.hidden % 2048:
            return None
        return r

    def _w4x_weight(self, layer: int, name: str, bn: int):
        """The weight a split-K four-wave projection reads: its tile-panel
        copy when there is one for ``bn``, else the row-major weight."""
        if self.w4x_panels is not None:
            p = self.w4x_panels[layer].get((name, bn))
            if p is not None:
                return p
        return self.w[layer][name]

    def _gate_up_weight(self, layer: int, bn: int):
        """gate|up as the SwiGLU four-wave kernel reads it: the SwiGLU tile-panel
        copy for ``bn`` when ``gate_up_panels`` made one, else row-major."""
        if self.gate_up_panels is not None and bn in self.gate_up_panels[layer]:
            return self.gate_up_panels[layer][bn]
        return self.w[layer]["gate_up"]

    def _swiglu_route(self, m: int):
        """(bn, 1) when the decode gate|up projection runs unsplit on the
        four-wave kernel: SwiGLU then goes into its epilogue."""
        if not self.fuse_splitk:
            return None
        w = self.w[0]["gate_up"]
        r = D.w4x_route(m, w.shape[0], w.shape[1])
        return r if r is not None and r[1] == 1 else None

    def _norm(self, x, d, w):
        """x += d (in place, bf16) and return rmsnorm(x) * w."""
        if self.backend == "ref":
            if d is not None:
                x.copy_((x.float() + d.float()).to(torch.bfloat16))
            return _rms_norm(x, w, self.cfg.eps)
        from kgs.ops.transformer import add_rmsnorm

        return add_rmsnorm(x, d, w, self.cfg.eps)

    def _proj_add_norm(self, a, layer: int, name: str, x, w):
        """Prompt pass: x += a @ W.T, return rmsnorm(x) * w. On kgs with aligned
        operands the residual add runs in the GEMM's store (EPI_ADDC) and the
        norm reads x once: bitwise the GEMM + add_rmsnorm pair, with one
        [rows, hidden] tensor fewer through HBM (profiles/r5/prefill_swiglu)."""
        if self.backend == "kgs":
            from kgs.ops.gemm import addc_ok, gemm_nt_add_

            wt = self.w[layer][name]
            if addc_ok(a, wt, x):
                gemm_nt_add_(a, wt, x)
                return self._norm(x, None, w)
        return self._norm(x, self._proj(a, layer, name, False), w)

    def _gate_up_act(self, y, layer):
        """Prompt-pass SwiGLU MLP input: fused into the GEMM epilogue on kgs."""
        if self.backend == "kgs" and self.fuse_splitk:
            from kgs.ops.gemm import gemm_swiglu

            return gemm_swiglu(y, self.w[layer]["gate_up"])
        return self._silu_mul(self._proj(y, layer, "gate_up", False))

    def _silu_mul(self, gu):
        if self.backend == "ref":
            i = gu.shape[1] // 2
            g, u = gu[:, :i].float(), gu[:, i:].float()
            return (g * torch.sigmoid(g) * u).to(torch.bfloat16)
        from kgs.ops.transformer import silu_mul

        return silu_mul(gu)

    def _rope_cache(self, qkv, layer, positions, slots):
        c = self.cfg
        if self.backend == "ref":
            hq = c.heads + c.kv_heads
            rot = D.ref_rope_rows(qkv, self.cos, self.sin, positions, hq)
            qkv[:, :hq * D.HEAD_DIM] = rot.to(torch.bfloat16)
            k = qkv[:, c.heads * D.HEAD_DIM:hq * D.HEAD_DIM].reshape(-1, c.kv_heads, D.HEAD_DIM)
            v = qkv[:, hq * D.HEAD_DIM:(hq + c.kv_heads) * D.HEAD_DIM].reshape(-1, c.kv_heads, D.HEAD_DIM)
            D.ref_cache_write(self.cache.layer(layer), k, v, slots)
            return
        D.rope_cache_(qkv, self.cos, self.sin, positions, slots, self.cache.layer(layer), c.heads, c.kv_heads)

    # ---------------------------------------------------------------- prefill
    @torch.no_grad()
    def prefill(self, tokens, positions, slots, seq_starts, seq_lens, padded_lens) -> torch.Tensor:
        """Flattened padded prompts -> logits of each sequence's last real token [S, vocab]."""
        c = self.cfg
        h, hd = c.hidden, c.head_dim
        if self.prefill_f8 is not None:
            return self._prefill_fp8(tokens, positions, slots, seq_starts, seq_lens, padded_lens)
        x = self.embed[tokens.long()].reshape(-1, h).contiguous()
        y = self._norm(x, None, self.ln1[0])
        T.op("prefill embed+norm")
        for i in range(c.layers):
            qkv = self._proj(y, i, "qkv", False)
            T.op(f"prefill L{i} qkv")
            self._rope_cache(qkv, i, positions, slots)
            T.op(f"prefill L{i} rope_cache")
            a = self._prefill_attention(qkv, seq_starts, seq_lens, padded_lens)
            T.op(f"prefill L{i} attention")
            y = self._proj_add_norm(a, i, "o", x, self.ln2[i])
            T.op(f"prefill L{i} o+norm")
            act = self._gate_up_act(y, i)
            T.op(f"prefill L{i} gate_up")
            nxt = self.ln1[i + 1] if i + 1 < c.layers else self.norm
            y = self._proj_add_norm(act, i, "down", x, nxt)
            T.op(f"prefill L{i} down+norm")
        last = torch.as_tensor([int(s) + int(n) - 1 for s, n in zip(seq_starts, seq_lens)], device=y.device)
        yl = y[last].contiguous()
        out = self._proj(yl, None, "lm", True)
        T.op("prefill lm_head")
        return out

    def _prefill_fp8(self, tokens, positions, slots, seq_starts, seq_lens, padded_lens) -> torch.Tensor:
        """W8A8 prompt pass: every GEMM input is e4m3 rows with per-row scales from
        its fused producer (add_rmsnorm_fp8, silu_mul_fp8, quantize_rows_fp8);
        attention, RoPE/KV write, the residual stream and the LM head stay bf16."""
        from kgs.ops.transformer import add_rmsnorm, add_rmsnorm_fp8, quantize_rows_fp8, silu_mul_fp8

        c = self.cfg
        x = self.embed[tokens.long()].reshape(-1, c.hidden).contiguous()
        y8, ys = add_rmsnorm_fp8(x, None, self.ln1[0], c.eps)
        y = None
        for i in range(c.layers):
            F = self.prefill_f8[i]
            qkv = F["qkv"].forward_q(y8, ys)
            self._rope_cache(qkv, i, positions, slots)
            a8, as_ = quantize_rows_fp8(self._prefill_attention(qkv, seq_starts, seq_lens, padded_lens))
            y8, ys = add_rmsnorm_fp8(x, F["o"].forward_q(a8, as_), self.ln2[i], c.eps)
            m8, ms = silu_mul_fp8(F["gate_up"].forward_q(y8, ys))
            d = F["down"].forward_q(m8, ms)
            if i + 1 < c.layers:
                y8, ys = add_rmsnorm_fp8(x, d, self.ln1[i + 1], c.eps)
            else:
                y = add_rmsnorm(x, d, self.norm, c.eps)
        last = torch.as_tensor([int(s) + int(n) - 1 for s, n in zip(seq_starts, seq_lens)], device=y.device)
        return self._proj(y[last].contiguous(), None, "lm", True)

    def _prefill_attention(self, qkv, seq_starts, seq_lens, padded_lens):
        c = self.cfg
        hd = c.head_dim
        out = torch.empty((qkv.shape[0], c.heads * hd), dtype=torch.bfloat16, device=qkv.device)
        if self.backend != "ref" and len(set(int(p) for p in padded_lens)) == 1:
            # equal padded lengths, packed back to back: one batched launch
            from kgs.ops.transformer import attention_qkv

            p = int(padded_lens[0])
            attention_qkv(qkv, len(padded_lens), p, c.heads, c.kv_heads, head_dim=hd, causal=True, out=out)
            return out
        for s0, n, p in zip(seq_starts, seq_lens, padded_lens):
            s0, n, p = int(s0), int(n), int(p)
            blk = qkv[s0:s0 + p]
            if self.backend == "ref":
                q = blk[:n, :c.heads * hd].float().reshape(n, c.heads, hd).transpose(0, 1)
                k = blk[:n, c.heads * hd:(c.heads + c.kv_heads) * hd].float().reshape(n, c.kv_heads, hd).transpose(0, 1)
                v = blk[:n, (c.heads + c.kv_heads) * hd:(c.heads + 2 * c.kv_heads) * hd].float().reshape(
                    n, c.kv_heads, hd).transpose(0, 1)
                rep = c.heads // c.kv_heads
                k, v = k.repeat_interleave(rep, 0), v.repeat_interleave(rep, 0)
                o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
                out[s0:s0 + n] = o.transpose(0, 1).reshape(n, c.heads * hd).to(torch.bfloat16)
                out[s0 + n:s0 + p] = 0
            else:
                from kgs.ops.transformer import attention_qkv

                attention_qkv(blk, 1, p, c.heads, c.kv_heads, head_dim=hd, causal=True, out=out[s0:s0 + p])
        return out

    # ------------------------------------------------------------------ mixed
    @torch.no_grad()
    def mixed(self, tokens, positions, slots, chunks, dec_block_tables=None, dec_ctx_lens=None) -> torch.Tensor:
        """Chunked-prefill step: prompt chunks (rows first) plus decode rows in ONE
        pass through the projections. ``chunks``: per prefill sequence
        ``(row0, n, padded, ctx0, pages, last)`` -- rows ``row0 .. row0+padded``
        hold prompt positions ``ctx0 .. ctx0+n-1`` (then padding), ``pages`` its
        block table, ``last`` whether the chunk ends the prompt. Decode rows
        follow. Returns logits for the last row of every ``last`` chunk, then
        for every decode row."""
        c = self.cfg
        hd = c.head_dim
        x = self.embed[tokens.long()].reshape(-1, c.hidden).contiguous()
        n_pf = sum(ch[2] for ch in chunks)
        nd = x.shape[0] - n_pf
        f8 = self.prefill_f8 is not None and n_pf > 0  # W8A8 projections for the whole mixed step
        if f8:
            from kgs.ops.transformer import add_rmsnorm_fp8, quantize_rows_fp8, silu_mul_fp8

            y8, ys = add_rmsnorm_fp8(x, None, self.ln1[0], c.eps)
        else:
            y = self._norm(x, None, self.ln1[0])
        for i in range(c.layers):
            qkv = self.prefill_f8[i]["qkv"].forward_q(y8, ys) if f8 else self._proj(y, i, "qkv", False)
            self._rope_cache(qkv, i, positions, slots)
            a = torch.empty((x.shape[0], c.heads * hd), dtype=torch.bfloat16, device=x.device)
            j = 0
            while j < len(chunks):
                row0, n, p, ctx0, pages, _ = chunks[j]
                # first chunks (no cached context) of equal padded length sit back to
                # back: one batched flash-attention launch for the run
                k = j + 1
                if ctx0 == 0 and self.backend != "ref":
                    while k < len(chunks) and chunks[k][3] == 0 and chunks[k][2] == p:
                        k += 1
                if k - j > 1:
                    from kgs.ops.transformer import attention_qkv

                    attention_qkv(qkv[row0:row0 + p * (k - j)], k - j, p, c.heads, c.kv_heads, head_dim=hd,
                                  causal=True, out=a[row0:row0 + p * (k - j)])
                else:
                    a[row0:row0 + p] = self._chunk_attention(qkv[row0:row0 + p], i, n, p, ctx0, pages)
                j = k
            if nd:
                qd = qkv[n_pf:]
                if self.backend == "ref":
                    a[n_pf:] = D.ref_paged_decode(qd, self.cache.layer(i), dec_block_tables, dec_ctx_lens, c.heads,
                                                  c.kv_heads).to(torch.bfloat16)
                else:
                    D.paged_decode_attention(qd, self.cache.layer(i), dec_block_tables, dec_ctx_lens, c.heads,
                                             c.kv_heads, out=a[n_pf:])
            nxt = self.ln1[i + 1] if i + 1 < c.layers else self.norm
            if f8:
                F = self.prefill_f8[i]
                a8, as_ = quantize_rows_fp8(a)
                y8, ys = add_rmsnorm_fp8(x, F["o"].forward_q(a8, as_), self.ln2[i], c.eps)
                m8, ms = silu_mul_fp8(F["gate_up"].forward_q(y8, ys))
                d = F["down"].forward_q(m8, ms)
                if i + 1 < c.layers:
                    y8, ys = add_rmsnorm_fp8(x, d, nxt, c.eps)
                else:
                    y = self._norm(x, d, nxt)
                continue
            y = self._norm(x, self._proj(a, i, "o", False), self.ln2[i])
            act = self._gate_up_act(y, i)
            y = self._norm(x, self._proj(act, i, "down", False), nxt)
        rows = [row0 + n - 1 for row0, n, _, _, _, last in chunks if last] + list(range(n_pf, n_pf + nd))
        if not rows:
            return torch.empty((0, c.vocab), dtype=torch.bfloat16, device=x.device)
        yl = y[torch.as_tensor(rows, device=y.device)].contiguous()
        return self._proj(yl, None, "lm", True)

    def _chunk_attention(self, blk, layer, n, p, ctx0, pages):
        """Causal attention of one prompt chunk (rows = positions ctx0 .. ctx0+p-1,
        n real) over everything cached before it plus itself; padded rows out 0."""
        c = self.cfg
        hd = c.head_dim
        if ctx0 == 0:  # first chunk: the whole-prompt path
            out = torch.empty((p, c.heads * hd), dtype=torch.bfloat16, device=blk.device)
            if self.backend == "ref":
                return self._prefill_attention(blk, [0], [n], [p])
            from kgs.ops.transformer import attention_qkv

            return attention_qkv(blk, 1, p, c.heads, c.kv_heads, head_dim=hd, causal=True, out=out)
        # keys/values of positions 0 .. ctx0+n-1 (this chunk's rows were just
        # written to the cache by rope_cache), zero-padded to ctx0 + p rows
        if self.backend == "ref":
            from kgs.ops.transformer import ref_attention_chunk

            k, v = D.gather_kv(self.cache.layer(layer), pages, ctx0 + n)
            o = torch.zeros((p, c.heads * hd), dtype=torch.bfloat16, device=blk.device)
            o[:n] = ref_attention_chunk(blk[:n], k, v, c.heads, c.kv_heads, hd).to(torch.bfloat16)
            return o
        from kgs.ops.transformer import attention_chunk

        k, v = D.gather_kv(self.cache.layer(layer), pages, ctx0 + n, rows=ctx0 + p)
        return attention_chunk(blk, k, v, c.heads, c.kv_heads, hd)

    # ----------------------------------------------------------------- decode
    @torch.no_grad()
    def decode(self, tokens, positions, slots, block_tables, ctx_lens, pages_per_split=None) -> torch.Tensor:
        """One token per sequence -> logits [B, vocab]."""
        c = self.cfg
        if self.backend == "kgs" and tokens.shape[0] <= self.fused_max_batch:
            return self._decode_fused(tokens, positions, slots, block_tables, ctx_lens, pages_per_split)
        x = self.embed[tokens.long()].reshape(-1, c.hidden).contiguous()
        y = self._norm(x, None, self.ln1[0])
        m = x.shape[0]
        rq, ro, rd = (self._splitk_route(m, 0, n) for n in ("qkv", "o", "down"))  # same shapes in every layer
        rg = self._swiglu_route(m)
        if rq or ro or rd or rg:
            from kgs.ops.gemm import gemm_nt_w4x_partials, gemm_nt_w4x_swiglu
            from kgs.ops.transformer import splitk_add_rmsnorm
        # split-K qkv with KGS_ROPE_ATTN=1: its reduce + RoPE + KV write run
        # inside the attention launch (one launch per layer fewer)
        fused_attn = bool(rq) and rq[1] in (2, 4, 8) and self.backend == "kgs" and self.rope_attn and \
            c.heads // c.kv_heads <= 6
        for i in range(c.layers):
            if fused_attn:
                part = gemm_nt_w4x_partials(y, self._w4x_weight(i, "qkv", rq[0]), *rq, nt_weights=D.w4x_nt(rq))
                a = D.rope_paged_decode_attention(part, self.cos, self.sin, positions, slots, self.cache.layer(i),
                                                  block_tables, ctx_lens, c.heads, c.kv_heads,
                                                  pages_per_split=pages_per_split)
                T.op(f"decode L{i} qkv+rope+attention")
            elif rq:
                part = gemm_nt_w4x_partials(y, self._w4x_weight(i, "qkv", rq[0]), *rq, nt_weights=D.w4x_nt(rq))
                qkv = torch.empty((m, part.shape[2]), dtype=torch.bfloat16, device=x.device)
                D.rope_cache_(qkv, self.cos, self.sin, positions, slots, self.cache.layer(i), c.heads, c.kv_heads,
                              partials=part)
                T.op(f"decode L{i} qkv+rope_cache")
            else:
                qkv = self._proj(y, i, "qkv", True)
                self._rope_cache(qkv, i, positions, slots)
                T.op(f"decode L{i} qkv+rope_cache")
            if fused_attn:
                pass
            elif self.backend == "ref":
                a = D.ref_paged_decode(qkv, self.cache.layer(i), block_tables, ctx_lens, c.heads,
                                       c.kv_heads).to(torch.bfloat16)
            else:
                a = D.paged_decode_attention(qkv, self.cache.layer(i), block_tables, ctx_lens, c.heads, c.kv_heads,
                                             pages_per_split=pages_per_split)
                T.op(f"decode L{i} attention")
            if ro:
                y = splitk_add_rmsnorm(gemm_nt_w4x_partials(a, self._w4x_weight(i, "o", ro[0]), *ro,
                                                            nt_weights=D.w4x_nt(ro)), x, self.ln2[i], c.eps)
            else:
                y = self._norm(x, self._proj(a, i, "o", True), self.ln2[i])
            T.op(f"decode L{i} o+norm")
            if rg:
                act = gemm_nt_w4x_swiglu(y, self._gate_up_weight(i, rg[0]), bn=rg[0], bm=rg[2],
                                         stages=D.w4x_stages(rg), nt_weights=D.w4x_nt(rg))
            else:
                act = self._silu_mul(self._proj(y, i, "gate_up", True))
            T.op(f"decode L{i} gate_up")
            nxt = self.ln1[i + 1] if i + 1 < c.layers else self.norm
            if rd:
                y = splitk_add_rmsnorm(gemm_nt_w4x_partials(act, self._w4x_weight(i, "down", rd[0]), *rd,
                                                            nt_weights=D.w4x_nt(rd)), x, nxt, c.eps)
            else:
                y = self._norm(x, self._proj(act, i, "down", True), nxt)
            T.op(f"decode L{i} down+norm")
        out = self._proj(y, None, "lm", True)
        T.op("decode lm_head")
        return out

    def _decode_fused(self, tokens, positions, slots, block_tables, ctx_lens, pages_per_split):
        """Decode with every norm / SwiGLU / residual add inside the skinny GEMMs:
        5 GEMMs + RoPE/KV-write + attention per layer, no elementwise launches.
        ss_a / ss_b carry the residual rows' sums of squares between the
        producing GEMM (residual update) and the consuming one (folded RMSNorm)."""
        c = self.cfg
        eps = c.eps
        x = self.embed[tokens.long()].reshape(-1, c.hidden).contiguous()  # residual stream
        ss_b = x.float().pow(2).sum(-1)  # statistic for layer 0's qkv
        ss_a = torch.zeros_like(ss_b)
        for i in range(c.layers):
            P = self.packed[i]
            if P["qkv"].rope:
                qkv = D.skinny_gemm(x, P["qkv"], rms=ss_b, eps=eps,
                                    rope={"cos": self.cos, "sin": self.sin, "positions": positions, "slots": slots,
                                          "cache": self.cache.layer(i)})
            else:
                qkv = D.skinny_gemm(x, P["qkv"], rms=ss_b, eps=eps)
                self._rope_cache(qkv, i, positions, slots)
            T.op(f"decode-fused L{i} qkv+rope")
            a = D.paged_decode_attention(qkv, self.cache.layer(i), block_tables, ctx_lens, c.heads, c.kv_heads,
                                         pages_per_split=pages_per_split)
            T.op(f"decode-fused L{i} attention")
            D.skinny_gemm(a, P["o"], out=x, resid_ss=ss_a, zero=ss_b)
            act = D.skinny_gemm(x, P["gate_up"], rms=ss_a, eps=eps)
            D.skinny_gemm(act, P["down"], out=x, resid_ss=ss_b, zero=ss_a)
            T.op(f"decode-fused L{i} o+mlp")
        out = D.skinny_gemm(x, self.packed_lm, rms=ss_b, eps=eps)
        T.op("decode-fused lm_head")
        return out
