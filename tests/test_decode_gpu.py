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
    from kgs.ops.decode import SKINNY_VARIANTS, skinny_geometry, skinny_variants

    so = _lib.lib()
    for m in (1, 5, 16, 17, 32, 33, 64, 65, 128, 129, 256):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert so.kgs_skinny_geometry(m, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) == 0
        assert (a.value, b.value, c.value) == skinny_geometry(m)
        for v in SKINNY_VARIANTS:
            rc = so.kgs_skinny_variant_geometry(v, m, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
            if v in skinny_variants(m):
                assert rc == 0 and (a.value, b.value, c.value) == skinny_geometry(m, v)
            else:
                assert rc == -3


@pytest.mark.parametrize("m", [9, 30, 64, 128, 200])
def test_skinny_gemm_every_variant(m):
    from kgs.ops.decode import PackedWeight, choose_ksplit, skinny_gemm, skinny_variants

    n, k = 512, 1024
    x = _bf(m, k)
    w = _bf(n, k, scale=k ** -0.5)
    pw = PackedWeight(w)
    ref = x.float() @ w.float().T
    for v in skinny_variants(m):
        for ks in sorted({1, choose_ksplit(m, n, k, variant=v)}):
            y = skinny_gemm(x, pw, ksplit=ks, variant=v)
            torch.cuda.synchronize()
            err = (y.float() - ref).abs().max().item()
            assert err <= 2e-2 * ref.abs().max().item() + 1e-3, (v, ks, err)


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


@pytest.mark.parametrize("m", [1, 20, 64, 150])
def test_skinny_swiglu_epilogue(m):
    from kgs.ops.decode import PackedWeight, choose_ksplit, skinny_gemm, skinny_variants

    inter, k = 512, 1024
    x = _bf(m, k)
    w = _bf(2 * inter, k, scale=k ** -0.5)  # fused gate|up, gate rows first
    pw = PackedWeight(w, swiglu=True)
    g = x.float() @ w[:inter].float().T
    u = x.float() @ w[inter:].float().T
    ref = g * torch.sigmoid(g) * u
    for v in skinny_variants(m):
        for ks in sorted({1, choose_ksplit(m, 2 * inter, k, variant=v)}):
            y = skinny_gemm(x, pw, ksplit=ks, variant=v)
            torch.cuda.synchronize()
            assert y.shape == (m, inter)
            assert (y.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-3, (v, ks)


@pytest.mark.parametrize("m", [3, 32, 64])
def test_skinny_fused_rms_and_residual_epilogues(m):
    """The fused decode layer's GEMMs: RMSNorm folded into W + row scale from a
    sum of squares (qkv / gate|up / lm_head) and the in-place residual update that
    accumulates the next sums of squares (o / down)."""
    from kgs.ops.decode import PackedWeight, skinny_gemm
    from kgs.ops.transformer import ref_add_rmsnorm

    h, n = 1024, 1536
    x = _bf(m, h)
    lnw = (_bf(h, scale=0.2) + 1).contiguous()
    w = _bf(n, h, scale=h ** -0.5)
    # rms: rmsnorm(x) * lnw @ W^T
    ss = x.float().pow(2).sum(-1)
    _, y_ref = ref_add_rmsnorm(x, None, lnw)
    ref = y_ref.float() @ w.float().T
    got = skinny_gemm(x, PackedWeight(w, fold=lnw), rms=ss, eps=1e-5)
    torch.cuda.synchronize()
    assert (got.float() - ref).abs().max().item() <= 3e-2 * ref.abs().max().item()
    # swiglu + rms
    wgu = _bf(2 * n, h, scale=h ** -0.5)
    g, u = y_ref.float() @ wgu[:n].float().T, y_ref.float() @ wgu[n:].float().T
    ref2 = g * torch.sigmoid(g) * u
    got2 = skinny_gemm(x, PackedWeight(wgu, swiglu=True, fold=lnw), rms=ss, eps=1e-5)
    torch.cuda.synchronize()
    assert (got2.float() - ref2).abs().max().item() <= 3e-2 * ref2.abs().max().item()
    # residual: res += a @ Wo^T, ss_out += rowsum(res^2), zero cleared
    wo = _bf(h, n, scale=n ** -0.5)
    a = _bf(m, n)
    for ks in (1, None):
        res = _bf(m, h)
        res0 = res.clone()
        ss_out = torch.full((m,), 0.0, device=DEV)
        junk = torch.full((m,), 7.0, device=DEV)
        skinny_gemm(a, PackedWeight(wo), out=res, resid_ss=ss_out, zero=junk, ksplit=ks)
        torch.cuda.synchronize()
        new_ref = (res0.float() + a.float() @ wo.float().T)
        assert (res.float() - new_ref).abs().max().item() <= 2e-2 * new_ref.abs().max().item()
        assert torch.allclose(ss_out, res.float().pow(2).sum(-1), rtol=1e-4, atol=1e-3)
        assert junk.abs().max().item() == 0


@pytest.mark.parametrize("m", [1, 30, 64])
def test_skinny_fp8_weights(m):
    """W8A16: e4m3 weights with per-row scales, dequantised in registers; with and
    without the fused epilogues, against fp32 math on the dequantised weight."""
    from kgs.ops.decode import PackedWeight, choose_ksplit, skinny_gemm, skinny_variants

    n, k = 768, 2048
    x = _bf(m, k)
    w = _bf(n, k, scale=k ** -0.5)
    pw = PackedWeight(w, fp8=True)
    wd = pw.unpacked().float()
    assert (wd - w.float()).abs().max().item() <= 0.07 * w.float().abs().max().item()
    ref = x.float() @ wd.T
    for v in skinny_variants(m):
        for ks in sorted({1, choose_ksplit(m, n, k, variant=v)}):
            y = skinny_gemm(x, pw, ksplit=ks, variant=v)
            torch.cuda.synchronize()
            assert (y.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-3, (v, ks)
    # SwiGLU + folded RMSNorm on fp8 weights
    lnw = (_bf(k, scale=0.2) + 1).contiguous()
    wgu = _bf(2 * n, k, scale=k ** -0.5)
    pgu = PackedWeight(wgu, swiglu=True, fold=lnw, fp8=True)
    wgd = pgu.unpacked().float()  # folded + dequantised, original row order
    ss = x.float().pow(2).sum(-1)
    xn = x.float() * torch.rsqrt(ss / k + 1e-5)[:, None]
    g, u = xn @ wgd[:n].T, xn @ wgd[n:].T
    ref2 = g * torch.sigmoid(g) * u
    y2 = skinny_gemm(x, pgu, rms=ss)
    torch.cuda.synchronize()
    assert (y2.float() - ref2).abs().max().item() <= 3e-2 * ref2.abs().max().item()


@pytest.mark.parametrize("pps", [None, 1, 100])
def test_fp8_kv_cache(pps):
    """e4m3 KV pages: the fused RoPE/KV write stores what the reference quantiser
    stores, and the attention over them matches fp32 math on the dequantised cache."""
    from kgs.ops.decode import (PAGE, PagedKVCache, paged_decode_attention, ref_cache_write, ref_paged_decode,
                                rope_cache_)
    from kgs.ops.transformer import rope_tables

    heads, hkv, hd = 32, 8, 128
    ctxs = [5, 64, 200]
    b = len(ctxs)
    cache = PagedKVCache(1, 32, hkv, DEV, dtype="fp8")
    ref_cache = torch.zeros_like(cache.layer(0))
    bt = _setup_cache(b, ctxs, hkv, 32, seed=3).to(DEV)
    cos, sin = rope_tables(4096, hd, 500000.0, DEV)
    pos, slots = [], []
    for i, c in enumerate(ctxs):
        for t in range(c):
            pos.append(t)
            slots.append(int(bt[i, t // PAGE]) * PAGE + t % PAGE)
    qkv = _bf(len(pos), (heads + 2 * hkv) * hd)
    pos_t = torch.tensor(pos, dtype=torch.int32, device=DEV)
    slot_t = torch.tensor(slots, dtype=torch.int32, device=DEV)
    rope_cache_(qkv, cos, sin, pos_t, slot_t, cache.layer(0), heads, hkv)
    torch.cuda.synchronize()
    k = qkv[:, heads * hd:(heads + hkv) * hd].reshape(-1, hkv, hd)
    v = qkv[:, (heads + hkv) * hd:].reshape(-1, hkv, hd)
    ref_cache_write(ref_cache, k, v, slot_t)
    assert torch.equal(cache.layer(0).view(torch.uint8), ref_cache.view(torch.uint8))
    last = torch.tensor([sum(ctxs[:i + 1]) - 1 for i in range(b)], device=DEV)
    q = qkv[last].contiguous()
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    ref = ref_paged_decode(q, cache.layer(0), bt, ctx_t, heads, hkv)
    o = paged_decode_attention(q, cache.layer(0), bt, ctx_t, heads, hkv, pages_per_split=pps)
    torch.cuda.synchronize()
    assert (o.float() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("kv_dtype", ["bf16", "fp8"])
def test_rope_cache_from_splitk_partials(kv_dtype):
    """qkv projection handed over as split-K partials: one launch reduces,
    rotates and writes the cache -- bit-identical to reduce + rope_cache_."""
    from kgs.ops.decode import PAGE, PagedKVCache, rope_cache_
    from kgs.ops.gemm import gemm_nt_w4x, gemm_nt_w4x_partials
    from kgs.ops.transformer import rope_tables

    heads, hkv, hd, m, k = 32, 8, 128, 200, 4096
    width = (heads + 2 * hkv) * hd
    x = _bf(m, k)
    w = _bf(width, k, scale=k ** -0.5)
    cos, sin = rope_tables(4096, hd, 500000.0, DEV)
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(64 * PAGE, device=DEV)[:m].int()
    slots[3] = -1  # no cache write for this row
    caches = [PagedKVCache(1, 64, hkv, DEV, dtype=kv_dtype) for _ in range(2)]
    q1 = gemm_nt_w4x(x, w, bn=128, nslice=4)
    rope_cache_(q1, cos, sin, pos, slots, caches[0].layer(0), heads, hkv)
    q2 = torch.empty_like(q1)
    rope_cache_(q2, cos, sin, pos, slots, caches[1].layer(0), heads, hkv,
                partials=gemm_nt_w4x_partials(x, w, 128, 4))
    torch.cuda.synchronize()
    assert torch.equal(q1, q2)
    assert torch.equal(caches[0].layer(0).view(torch.uint8), caches[1].layer(0).view(torch.uint8))


@pytest.mark.parametrize("b,kv_dtype,pps", [(4, "bf16", 2), (64, "bf16", None), (256, "bf16", None),
                                             (256, "fp8", None), (20, "fp8", 3)])
def test_rope_paged_decode_matches_two_launches(b, kv_dtype, pps):
    """rope_cache (split-K partials) + paged decode attention folded into one
    launch (kgs_paged_decode_rope_bf16): the same KV cache bytes and the same
    attention output as the two launches, across one-split / split-with-merge /
    split-with-reduce grids, the pipelined and the large-grid kernel, bf16 and
    e4m3 caches, ragged contexts and scattered pages."""
    from kgs.ops.decode import (PAGE, PagedKVCache, paged_decode_attention, rope_cache_,
                                rope_paged_decode_attention)
    from kgs.ops.transformer import rope_tables

    heads, hkv, hd, nslice = 32, 8, 128, 4
    nh = heads + 2 * hkv
    g = torch.Generator(device=DEV).manual_seed(b)
    ctxs = torch.randint(1, 300, (b,), generator=g, device=DEV).int()
    max_pages = int((ctxs.max().item() + PAGE - 1) // PAGE)
    npages = b * max_pages + 4
    perm = torch.randperm(npages, generator=g, device=DEV).int()
    bt = perm[: b * max_pages].view(b, max_pages).contiguous()
    last = ctxs.long() - 1
    slots = (bt.gather(1, (last // PAGE).view(-1, 1)).view(-1).long() * PAGE + last % PAGE).int().contiguous()
    pos = last.int().contiguous()
    cos, sin = rope_tables(4096, hd, 500000.0, DEV)
    parts = (torch.randn(nslice, b, nh * hd, generator=g, device=DEV) * 0.5).contiguous()
    caches = [PagedKVCache(1, npages, hkv, DEV, dtype=kv_dtype) for _ in range(2)]
    fill = (torch.randn(caches[0].layer(0).shape, generator=g, device=DEV) * 0.5).to(caches[0].layer(0).dtype)
    for c in caches:
        c.layer(0).copy_(fill)
    qkv = torch.empty((b, nh * hd), dtype=torch.bfloat16, device=DEV)
    rope_cache_(qkv, cos, sin, pos, slots, caches[0].layer(0), heads, hkv, partials=parts)
    ref = paged_decode_attention(qkv, caches[0].layer(0), bt, ctxs, heads, hkv, pages_per_split=pps)
    out = rope_paged_decode_attention(parts, cos, sin, pos, slots, caches[1].layer(0), bt, ctxs, heads, hkv,
                                      pages_per_split=pps)
    torch.cuda.synchronize()
    c0, c1 = caches[0].layer(0).view(torch.uint8), caches[1].layer(0).view(torch.uint8)
    assert torch.equal(c0, c1), int((c0 != c1).sum())
    err = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
    assert torch.equal(out, ref) or err < 1e-2, err


@pytest.mark.parametrize("m,cols,nslice", [(256, 4096, 8), (200, 4096, 4), (130, 8192, 2)])
def test_splitk_add_rmsnorm_matches_unfused(m, cols, nslice):
    """o / down projection partials reduced inside the residual add + RMSNorm:
    the residual stream is bit-identical to reduce + add_rmsnorm, the normed
    output agrees to bf16 rounding (the row sum of squares is added in another
    order) and with fp32 torch."""
    from kgs.ops.gemm import gemm_nt_w4x, gemm_nt_w4x_partials
    from kgs.ops.transformer import add_rmsnorm, splitk_add_rmsnorm

    k = 4096
    a = _bf(m, k)
    wt = _bf(cols, k, scale=k ** -0.5)
    lnw = (1 + 0.1 * torch.randn(cols, device=DEV)).bfloat16()
    x0 = _bf(m, cols)
    x1, x2 = x0.clone(), x0.clone()
    d = gemm_nt_w4x(a, wt, bn=128, nslice=nslice)
    y1 = add_rmsnorm(x1, d, lnw, 1e-5)
    y2 = splitk_add_rmsnorm(gemm_nt_w4x_partials(a, wt, 128, nslice), x2, lnw, 1e-5)
    torch.cuda.synchronize()
    assert torch.equal(x1, x2)
    diff = (y1.float() - y2.float()).abs()
    assert diff.max().item() <= 2 ** -6 * y1.float().abs().max().item()
    xr = x0.float() + (a.float() @ wt.float().T)
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * lnw.float()
    assert ((y2.float() - yr).abs().max() / yr.abs().max()).item() < 2e-2


@pytest.mark.parametrize("b,pps,kv_dtype", [(1, 4, "bf16"), (2, 1, "bf16"), (3, 2, "fp8"), (96, 100, "bf16"),
                                            (80, 4, "fp8")])
def test_paged_decode_small_and_large_grids(b, pps, kv_dtype):
    """Small grids (<= 512 waves) take the in-wave page pipeline and the
    lane-parallel split merge, large ones the one-page-at-a-time loop; both
    against the fp32 reference over ragged contexts and scattered pages."""
    from kgs.ops.decode import PAGE, PagedKVCache, paged_decode_attention, ref_paged_decode

    heads, hkv, hd = 32, 8, 128
    g = torch.Generator(device=DEV).manual_seed(b)
    ctxs = [int(x) for x in torch.randint(1, 33 * PAGE, (b,), generator=g, device=DEV)]
    max_pages = max(math.ceil(c / PAGE) for c in ctxs) + 3
    npages = b * max_pages + 4
    cache = PagedKVCache(1, npages, hkv, DEV, dtype=kv_dtype)
    lay = cache.layer(0)
    lay.copy_((torch.randn(lay.shape, generator=g, device=DEV) * 0.7).to(lay.dtype))
    bt = torch.randperm(npages, generator=g, device=DEV)[:b * max_pages].view(b, max_pages).int().contiguous()
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    q = _bf(b, heads * hd)
    ref = ref_paged_decode(q, lay, bt, ctx_t, heads, hkv)
    o = paged_decode_attention(q, lay, bt, ctx_t, heads, hkv, pages_per_split=pps)
    o2 = paged_decode_attention(q, lay, bt, ctx_t, heads, hkv, pages_per_split=pps)
    torch.cuda.synchronize()
    assert (o.float() - ref).abs().max().item() < 2e-2
    assert torch.equal(o, o2)  # the merge re-arms its tickets: a second call is identical


@pytest.mark.parametrize("m,heads,hkv", [(1, 32, 8), (16, 32, 8), (40, 8, 8), (7, 16, 1)])
def test_skinny_rope_epilogue_matches_rope_cache(m, heads, hkv):
    """The fused qkv skinny GEMM with RoPE + KV-cache write in its epilogue
    (rope-packed weight) == skinny GEMM + rope_cache_, bit for bit (qkv rows and
    cache pages), with the RMSNorm folded in and a skipped slot."""
    from kgs.ops.decode import PAGE, PackedWeight, PagedKVCache, rope_cache_, skinny_gemm
    from kgs.ops.transformer import rope_tables

    k = 1024
    n = (heads + 2 * hkv) * 128
    w = _bf(n, k, scale=k ** -0.5)
    lnw = (1 + 0.1 * torch.randn(k, device=DEV)).bfloat16()
    x = _bf(m, k)
    ss = x.float().pow(2).sum(-1).contiguous()
    cos, sin = rope_tables(4096, 128, 500000.0, DEV)
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(16 * PAGE, device=DEV)[:m].int()
    if m > 3:
        slots[3] = -1
    caches = [PagedKVCache(1, 16, hkv, DEV) for _ in range(2)]
    plain = PackedWeight(w, fold=lnw)
    roped = PackedWeight(w, fold=lnw, rope=(heads, hkv))
    assert torch.equal(roped.unpacked(), plain.unpacked())
    q1 = skinny_gemm(x, plain, rms=ss, eps=1e-5)
    rope_cache_(q1, cos, sin, pos, slots, caches[0].layer(0), heads, hkv)
    q2 = skinny_gemm(x, roped, rms=ss, eps=1e-5,
                     rope={"cos": cos, "sin": sin, "positions": pos, "slots": slots, "cache": caches[1].layer(0)})
    torch.cuda.synchronize()
    assert torch.equal(q1, q2)
    assert torch.equal(caches[0].layer(0), caches[1].layer(0))


@pytest.mark.parametrize("m", [1, 5, 16])
@pytest.mark.parametrize("v", [20, 21])
def test_skinny_kin_variants(m, v):
    """In-workgroup K split (variants 20 / 21): every split-K factor, fp8
    weights, and the fused decode epilogues (RMS, SwiGLU, residual + sum of
    squares, RoPE + KV write) against fp32 references / the default variant."""
    from kgs.ops.decode import (PAGE, PackedWeight, PagedKVCache, rope_cache_, skinny_gemm,
                                skinny_geometry)
    from kgs.ops.transformer import rope_tables

    n, k = 1024, 4096
    rps, kpc, _ = skinny_geometry(m, v)
    assert (rps, kpc) == ((16, 1024) if v == 20 else (32, 1024))
    x = _bf(m, k)
    w = _bf(n, k, scale=k ** -0.5)
    ref = x.float() @ w.float().T
    tol = 2e-2 * ref.abs().max().item() + 1e-3
    pw = PackedWeight(w)
    for ks in (1, 2, 4):
        y = skinny_gemm(x, pw, ksplit=ks, variant=v)
        torch.cuda.synchronize()
        assert (y.float() - ref).abs().max().item() <= tol, ks
    y8 = skinny_gemm(x, PackedWeight(w, fp8=True), ksplit=2, variant=v)
    torch.cuda.synchronize()
    assert (y8.float() - ref).abs().max().item() <= 8 * tol
    # rms + swiglu
    lnw = (_bf(k, scale=0.2) + 1).contiguous()
    ss = x.float().pow(2).sum(-1).contiguous()
    xn = (x.float() * torch.rsqrt(ss / k + 1e-5)[:, None]).bfloat16().float() * lnw.float()
    wgu = _bf(2 * n, k, scale=k ** -0.5)
    g, u = xn @ wgu[:n].float().T, xn @ wgu[n:].float().T
    ref2 = g * torch.sigmoid(g) * u
    got2 = skinny_gemm(x, PackedWeight(wgu, swiglu=True, fold=lnw), rms=ss, eps=1e-5, variant=v, ksplit=2)
    torch.cuda.synchronize()
    assert (got2.float() - ref2).abs().max().item() <= 3e-2 * ref2.abs().max().item()
    # residual update + sums of squares
    for ks in (1, 4):
        res = _bf(m, n)
        res0 = res.clone()
        ss_out = torch.zeros(m, device=DEV)
        skinny_gemm(x, pw, out=res, resid_ss=ss_out, ksplit=ks, variant=v)
        torch.cuda.synchronize()
        new_ref = res0.float() + ref
        assert (res.float() - new_ref).abs().max().item() <= 2e-2 * new_ref.abs().max().item()
        assert torch.allclose(ss_out, res.float().pow(2).sum(-1), rtol=1e-4, atol=1e-3)
    if v != 20:
        return
    # RoPE + KV-cache write: same bits as the variant's plain output + rope_cache_
    heads, hkv = 32, 8
    nq = (heads + 2 * hkv) * 128
    wq = _bf(nq, k, scale=k ** -0.5)
    cos, sin = rope_tables(4096, 128, 500000.0, DEV)
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(16 * PAGE, device=DEV)[:m].int()
    caches = [PagedKVCache(1, 16, hkv, DEV) for _ in range(2)]
    q1 = skinny_gemm(x, PackedWeight(wq, fold=lnw), rms=ss, eps=1e-5, variant=v, ksplit=2)
    rope_cache_(q1, cos, sin, pos, slots, caches[0].layer(0), heads, hkv)
    q2 = skinny_gemm(x, PackedWeight(wq, fold=lnw, rope=(heads, hkv)), rms=ss, eps=1e-5, variant=v, ksplit=2,
                     rope={"cos": cos, "sin": sin, "positions": pos, "slots": slots, "cache": caches[1].layer(0)})
    torch.cuda.synchronize()
    assert torch.equal(q1, q2)
    assert torch.equal(caches[0].layer(0), caches[1].layer(0))


@pytest.mark.parametrize("M", [256, 200])
def test_nt_weight_loads_are_bitwise_the_default_policy(M):
    """Non-temporal weight loads (gemm_w4.h AUX >= 50: the policy on B's loads
    only) change where the bytes are cached, never the result: the SwiGLU,
    plain and split-K decode GEMMs are bitwise those of the default policy."""
    from kgs.ops.gemm import gemm_nt_w4x, gemm_nt_w4x_swiglu

    x = torch.randn(M, 4096, device=DEV).bfloat16()
    w = (torch.randn(2 * 1024, 4096, device=DEV) * 0.02).bfloat16()
    assert torch.equal(gemm_nt_w4x_swiglu(x, w, bn=128, nt_weights=True), gemm_nt_w4x_swiglu(x, w, bn=128))
    assert torch.equal(gemm_nt_w4x(x, w, bn=128, nt_weights=True), gemm_nt_w4x(x, w, bn=128))
    assert torch.equal(gemm_nt_w4x(x, w, bn=128, nslice=4, nt_weights=True), gemm_nt_w4x(x, w, bn=128, nslice=4))


def test_prompt_rope_cache_v_page_runs():
    """Round 5: at prompt sizes (>= 1024 rows) the v heads are written by
    v_cache_pages -- whole 16-B chunks of the transposed V page when a 32-token
    run fills one page in order, element by element otherwise. Runs from a
    page boundary, a chunk starting mid-page, padding rows (slot -1) and a tail
    shorter than a page: the cache equals the reference scatter of the
    kernel's own rotated k and v, and the q / k rotation equals the short-input
    (per-token) path's."""
    from kgs.ops.decode import PAGE, PagedKVCache, ref_cache_write, rope_cache_
    from kgs.ops.transformer import rope_tables

    heads, hkv, hd = 32, 8, 128
    width = (heads + 2 * hkv) * hd
    cos, sin = rope_tables(4096, hd, 500000.0, DEV)
    pos, slots = [], []
    page = 1
    for n, start in ((700, 0), (333, 0), (300, 40)):  # (tokens, context already cached)
        off = start % PAGE  # 40: this chunk starts 8 tokens into its first page
        for t in range(n):
            pos.append(start + t)
            slots.append(page * PAGE + off + t)
        page += (off + n + PAGE - 1) // PAGE + 1
        pos += [0] * 5  # padding rows between sequences
        slots += [-1] * 5
    T = len(pos)
    assert T >= 1024
    npages = page + 4
    qkv = _bf(T, width)
    pos_t = torch.tensor(pos, dtype=torch.int32, device=DEV)
    slot_t = torch.tensor(slots, dtype=torch.int32, device=DEV)
    cache = PagedKVCache(1, npages, hkv, DEV)
    orig = qkv.clone()
    rope_cache_(qkv, cos, sin, pos_t, slot_t, cache.layer(0), heads, hkv)
    # the per-token path on the same rows, 1000 at a time (below the prompt threshold)
    q2 = orig.clone()
    cache2 = PagedKVCache(1, npages, hkv, DEV)
    for s0 in range(0, T, 1000):
        rope_cache_(q2[s0:s0 + 1000], cos, sin, pos_t[s0:s0 + 1000], slot_t[s0:s0 + 1000], cache2.layer(0), heads, hkv)
    torch.cuda.synchronize()
    assert torch.equal(qkv, q2)
    assert torch.equal(cache.layer(0), cache2.layer(0))
    ref = torch.zeros_like(cache.layer(0))
    k = qkv[:, heads * hd:(heads + hkv) * hd].reshape(-1, hkv, hd)
    v = qkv[:, (heads + hkv) * hd:].reshape(-1, hkv, hd)
    ref_cache_write(ref, k, v, slot_t)
    assert torch.equal(cache.layer(0), ref)
