"""Decode-path kernels (native/kernels/decode.hip) against fp32 PyTorch references:
skinny GEMM on prepacked weights (all batch buckets, split-K on/off), the fused
RoPE + paged-KV write, and paged decode attention (context splits, GQA, ragged
contexts, scattered pages)."""
import math

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from kgs.ops import _lib

    _lib.lib()
    torch.manual_seed(0)


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def test_geometry_matches_native():
    import ctypes

    from kgs.ops import _lib
    from kgs.ops.decode import skinny_geometry

    so = _lib.lib()
    for m in (1, 5, 16, 17, 32, 33, 64, 65, 128, 129, 256):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert so.kgs_skinny_geometry(m, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) == 0
        assert (a.value, b.value, c.value) == skinny_geometry(m)


@pytest.mark.parametrize("m", [1, 7, 16, 24, 64, 100, 256])
@pytest.mark.parametrize("n,k", [(256, 1024), (1536, 4096)])
def test_skinny_gemm(m, n, k):
    from kgs.ops.decode import PackedWeight, skinny_gemm

    x = _bf(m, k)
    w = _bf(n, k, scale=k ** -0.5)
    pw = PackedWeight(w)
    ref = x.float() @ w.float().T
    for ks in (None, 1):
        y = skinny_gemm(x, pw, ksplit=ks)
        torch.cuda.synchronize()
        err = (y.float() - ref).abs().max().item()
        assert err <= 2e-2 * ref.abs().max().item() + 1e-3, (ks, err)


def test_skinny_gemm_all_splits_and_strided():
    from kgs.ops.decode import PackedWeight, skinny_gemm, skinny_geometry

    m, n, k = 12, 512, 4096
    x_big = _bf(m, k + 64)
    x = x_big[:, 32:32 + k]
    w = _bf(n, k, scale=0.02)
    pw = PackedWeight(w)
    ref = x.float() @ w.float().T
    _, kpc, _ = skinny_geometry(m)
    nchunks = k // kpc
    out_big = torch.zeros(m, n + 128, dtype=torch.bfloat16, device=DEV)
    for ks in [d for d in range(1, nchunks + 1) if nchunks % d == 0]:
        out = out_big[:, 64:64 + n]
        skinny_gemm(x, pw, out=out, ksplit=ks)
        # repeated calls re-use the ticket counters (re-armed by the reducer)
        skinny_gemm(x, pw, out=out, ksplit=ks)
        torch.cuda.synchronize()
        assert (out.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert out_big[:, :64].abs().max().item() == 0 and out_big[:, 64 + n:].abs().max().item() == 0


def _setup_cache(b, ctxs, hkv, pages_total, seed=0):
    from kgs.ops.decode import PAGE

    g = torch.Generator().manual_seed(seed)
    max_pages = max(math.ceil(c / PAGE) for c in ctxs)
    perm = torch.randperm(pages_total, generator=g)
    bt = torch.zeros(b, max_pages, dtype=torch.int32)
    used = 0
    for i, c in enumerate(ctxs):
        n = math.ceil(c / PAGE)
        bt[i, :n] = perm[used:used + n].int()
        used += n
    return bt


@pytest.mark.parametrize("heads,hkv", [(32, 8), (8, 8), (16, 1)])
def test_rope_cache_and_paged_decode(heads, hkv):
    from kgs.ops.decode import (PAGE, PagedKVCache, paged_decode_attention, ref_cache_write, ref_paged_decode,
                                ref_rope_rows, rope_cache_)
    from kgs.ops.transformer import rope_tables

    b = 5
    ctxs = [1, 31, 32, 77, 300]
    hd = 128
    cache = PagedKVCache(1, 64, hkv, DEV)
    ref_cache = torch.zeros_like(cache.layer(0))
    bt = _setup_cache(b, ctxs, hkv, 64).to(DEV)
    cos, sin = rope_tables(4096, hd, 500000.0, DEV)
    width = (heads + 2 * hkv) * hd
    # fill the whole context of every sequence through the kernel (prefill-like rows)
    rows, pos, slots = [], [], []
    for i, c in enumerate(ctxs):
        for t in range(c):
            pos.append(t)
            slots.append(int(bt[i, t // PAGE]) * PAGE + t % PAGE)
    qkv = _bf(len(pos), width)
    pos_t = torch.tensor(pos, dtype=torch.int32, device=DEV)
    slot_t = torch.tensor(slots, dtype=torch.int32, device=DEV)
    orig = qkv.clone()
    rope_cache_(qkv, cos, sin, pos_t, slot_t, cache.layer(0), heads, hkv)
    torch.cuda.synchronize()
    rot = ref_rope_rows(orig, cos, sin, pos_t, heads + hkv)
    assert (qkv[:, :(heads + hkv) * hd].float() - rot).abs().max().item() < 3e-2
    assert torch.equal(qkv[:, (heads + hkv) * hd:], orig[:, (heads + hkv) * hd:])
    # cache contents == reference scatter of the kernel's own rotated k and v
    k = qkv[:, heads * hd:(heads + hkv) * hd].reshape(-1, hkv, hd)
    v = qkv[:, (heads + hkv) * hd:].reshape(-1, hkv, hd)
    ref_cache_write(ref_cache, k, v, slot_t)
    assert torch.equal(cache.layer(0), ref_cache)
    # decode: the last token of each sequence attends over its whole context
    last = torch.tensor([sum(ctxs[:i + 1]) - 1 for i in range(b)], device=DEV)
    q = qkv[last].contiguous()
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    ref = ref_paged_decode(q, cache.layer(0), bt, ctx_t, heads, hkv)
    for pps in (None, 1, 2, 100):
        o = paged_decode_attention(q, cache.layer(0), bt, ctx_t, heads, hkv, pages_per_split=pps)
        torch.cuda.synchronize()
        err = (o.float() - ref).abs().max().item()
        assert err < 2e-2, (pps, err)


def test_paged_decode_long_context():
    from kgs.ops.decode import PagedKVCache, paged_decode_attention, ref_cache_write, ref_paged_decode

    heads, hkv, b = 32, 8, 3
    ctxs = [4096, 1000, 2500]
    cache = PagedKVCache(1, 300, hkv, DEV)
    bt = _setup_cache(b, ctxs, hkv, 300, seed=1).to(DEV)
    for i, c in enumerate(ctxs):
        pos = torch.arange(c, device=DEV)
        slots = (bt[i, pos // 32].long() * 32 + pos % 32).int()
        ref_cache_write(cache.layer(0), _bf(c, hkv, 128), _bf(c, hkv, 128), slots)
    q = _bf(b, heads * 128, scale=3.0)  # peaky softmax
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    ref = ref_paged_decode(q, cache.layer(0), bt, ctx_t, heads, hkv)
    o = paged_decode_attention(q, cache.layer(0), bt, ctx_t, heads, hkv)
    torch.cuda.synchronize()
    assert (o.float() - ref).abs().max().item() < 2e-2
