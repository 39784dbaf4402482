"""Numerics of the fused decoder-block kernels and the flash-attention forward
(native/kernels/transformer.hip, attention.hip) against fp32 PyTorch references."""
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


@pytest.mark.parametrize("cols", [512, 4096, 8192])
@pytest.mark.parametrize("with_delta", [False, True])
def test_add_rmsnorm(cols, with_delta):
    from kgs.ops.transformer import add_rmsnorm, ref_add_rmsnorm

    rows = 37
    x = _bf(rows, cols)
    d = _bf(rows, cols) if with_delta else None
    w = _bf(cols, scale=0.5) + 1
    xr, yr = ref_add_rmsnorm(x, d, w)
    x2 = x.clone()
    y = add_rmsnorm(x2, d, w)
    torch.cuda.synchronize()
    assert torch.equal(x2, xr)  # residual: one bf16 rounding of x + d, same as the reference
    err = (y.float() - yr.float()).abs().max().item()
    assert err <= 2e-2 * yr.float().abs().max().item(), err


def test_add_rmsnorm_strided_out():
    from kgs.ops.transformer import add_rmsnorm, ref_add_rmsnorm

    x = _bf(16, 1024)
    w = _bf(1024) + 1
    big = torch.zeros(16, 2048, dtype=torch.bfloat16, device=DEV)
    add_rmsnorm(x, None, w, out=big[:, 512:1536])
    _, yr = ref_add_rmsnorm(x, None, w)
    assert (big[:, 512:1536].float() - yr.float()).abs().max().item() < 0.05
    assert big[:, :512].abs().max().item() == 0 and big[:, 1536:].abs().max().item() == 0


def test_rope_qkv():
    from kgs.ops.transformer import ref_rope_qkv, rope_qkv_, rope_tables

    b, s, nh, nkv, hd = 2, 64, 4, 2, 128
    qkv = _bf(b * s, (nh + 2 * nkv) * hd)
    cos, sin = rope_tables(s, hd, 500000.0, DEV)
    ref = ref_rope_qkv(qkv, cos, sin, nh + nkv, hd, s)
    got = rope_qkv_(qkv.clone(), cos, sin, nh + nkv, hd, s)
    torch.cuda.synchronize()
    # v heads untouched, rotated heads within one bf16 rounding
    assert torch.equal(got[:, (nh + nkv) * hd:], ref[:, (nh + nkv) * hd:])
    assert (got.float() - ref.float()).abs().max().item() < 3e-2


def test_rope_positions():
    from kgs.ops.transformer import ref_rope_qkv, rope_qkv_, rope_tables

    hd, s = 128, 32
    qkv = _bf(s, 3 * hd)
    cos, sin = rope_tables(4096, hd, 10000.0, DEV)
    pos = torch.arange(s, device=DEV, dtype=torch.int32)
    a = rope_qkv_(qkv.clone(), cos, sin, 2, hd, s, positions=pos)
    b = rope_qkv_(qkv.clone(), cos, sin, 2, hd, s)
    assert torch.equal(a, b)
    ref = ref_rope_qkv(qkv, cos[:s].contiguous(), sin[:s].contiguous(), 2, hd, s)
    assert (a.float() - ref.float()).abs().max().item() < 3e-2


def test_silu_mul():
    from kgs.ops.transformer import ref_silu_mul, silu_mul

    gu = _bf(100, 2 * 1024, scale=3.0)
    got = silu_mul(gu)
    ref = ref_silu_mul(gu)
    err = ((got.float() - ref.float()).abs() / (ref.float().abs() + 1e-2)).max().item()
    assert err < 1.6e-2, err


def _attn_case(b, s, nh, nkv, causal, qscale=1.0, seed=0):
    from kgs.ops.transformer import attention_qkv, ref_attention_qkv

    g = torch.Generator(device=DEV).manual_seed(seed)
    hd = 128
    qkv = torch.randn(b * s, (nh + 2 * nkv) * hd, device=DEV, generator=g)
    qkv[:, :nh * hd] *= qscale
    qkv = qkv.to(torch.bfloat16)
    got = attention_qkv(qkv, b, s, nh, nkv, causal=causal)
    ref = ref_attention_qkv(qkv, b, s, nh, nkv, causal=causal)
    torch.cuda.synchronize()
    assert torch.isfinite(got.float()).all()
    return (got.float() - ref).abs().max().item(), ref.abs().max().item()


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("b,s,nh,nkv", [(1, 128, 4, 4), (2, 256, 8, 2), (1, 1024, 32, 8)])
def test_attention_matches_sdpa(b, s, nh, nkv, causal):
    err, mag = _attn_case(b, s, nh, nkv, causal)
    assert err < 2e-2, (err, mag)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("b,s,nh,nkv,qscale", [(1, 256, 4, 4, 1.0), (2, 512, 8, 2, 1.0), (1, 1024, 32, 8, 1.0),
                                               (2, 512, 8, 2, 6.0)])
def test_attention_w4_matches_reference(b, s, nh, nkv, qscale, causal):
    """The one-wave-per-SIMD named-register kernel (attention_w4.h, via the
    experiments library) against the fp32 reference, including peaky scores
    (qscale 6: the deferred rescale of the AGPR-resident O runs), and against
    the production kernel."""
    from kgs.ops import experiments
    from kgs.ops.transformer import attention_qkv, ref_attention_qkv

    g = torch.Generator(device=DEV).manual_seed(11)
    hd = 128
    qkv = torch.randn(b * s, (nh + 2 * nkv) * hd, device=DEV, generator=g)
    qkv[:, :nh * hd] *= qscale
    qkv = qkv.to(torch.bfloat16)
    got = experiments.attention_qkv_w4(qkv, b, s, nh, nkv, causal=causal)
    ref = ref_attention_qkv(qkv, b, s, nh, nkv, causal=causal)
    prod = attention_qkv(qkv, b, s, nh, nkv, causal=causal)
    torch.cuda.synchronize()
    assert torch.isfinite(got.float()).all()
    mag = ref.abs().max().item()
    assert (got.float() - ref).abs().max().item() < 2e-2 * max(1.0, mag)
    assert (got.float() - prod.float()).abs().max().item() < 2e-2 * max(1.0, mag)
    # deterministic: a second run gives the same bits
    assert torch.equal(got, experiments.attention_qkv_w4(qkv, b, s, nh, nkv, causal=causal))


def test_attention_peaky_softmax_rescales():
    # large scores: the running max moves by a lot between tiles, so the
    # online-softmax rescale of O and l is exercised on every row
    err, mag = _attn_case(2, 512, 8, 2, True, qscale=6.0, seed=3)
    assert err < 4e-2 * max(1.0, mag), (err, mag)


def test_attention_max_grows_along_keys():
    from kgs.ops.transformer import attention_qkv, ref_attention_qkv

    # scores increase with the key index: each new tile holds the new row max
    b, s, nh, nkv, hd = 1, 512, 2, 1, 128
    qkv = torch.zeros(b * s, (nh + 2 * nkv) * hd, device=DEV)
    qkv[:, :nh * hd] = 0.05
    ramp = torch.linspace(0, 4, s, device=DEV)
    qkv[:, nh * hd:(nh + 1) * hd] = ramp[:, None]
    qkv[:, (nh + 1) * hd:] = torch.randn(s, hd, device=DEV)
    qkv = qkv.to(torch.bfloat16)
    got = attention_qkv(qkv, b, s, nh, nkv, causal=True)
    ref = ref_attention_qkv(qkv, b, s, nh, nkv, causal=True)
    assert (got.float() - ref).abs().max().item() < 3e-2


def test_attention_first_row_is_v0():
    from kgs.ops.transformer import attention_qkv

    # causal row 0 attends to key 0 only: O[0] == V[0] exactly (after rounding)
    b, s, nh, nkv, hd = 2, 128, 4, 2, 128
    qkv = _bf(b * s, (nh + 2 * nkv) * hd)
    o = attention_qkv(qkv, b, s, nh, nkv, causal=True)
    for bi in range(b):
        for h in range(nh):
            v0 = qkv[bi * s, (nh + nkv + h // (nh // nkv)) * hd:(nh + nkv + h // (nh // nkv) + 1) * hd]
            assert torch.allclose(o[bi * s, h * hd:(h + 1) * hd].float(), v0.float(), atol=1e-2)


def test_attention_rejects_bad_shapes():
    from kgs.ops import KernelError
    from kgs.ops.transformer import attention_qkv

    qkv = _bf(100, 3 * 128)
    with pytest.raises(KernelError):
        attention_qkv(qkv, 1, 100, 1, 1)  # seq % 128 != 0


def _deq(y8, ys):
    return y8.float() * ys[:, None]


def _close_fp8(deq, ref):
    # e4m3: 3 mantissa bits -> <= 2^-4 relative per element, plus the subnormal
    # floor relative to the row amax
    tol = 0.0625 * ref.abs() + 2e-3 * ref.abs().amax(dim=1, keepdim=True)
    return bool(((deq - ref).abs() <= tol + 1e-6).all())


@pytest.mark.parametrize("with_delta", [False, True])
def test_add_rmsnorm_fp8(with_delta):
    from kgs.ops.transformer import add_rmsnorm_fp8, ref_add_rmsnorm

    x = _bf(64, 4096)
    d = _bf(64, 4096) if with_delta else None
    w = _bf(4096, scale=0.5) + 1
    xr, _ = ref_add_rmsnorm(x, d, w)
    xf = xr.float()
    yref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    x2 = x.clone()
    y8, ys = add_rmsnorm_fp8(x2, d, w)
    torch.cuda.synchronize()
    assert torch.equal(x2, xr)
    assert _close_fp8(_deq(y8, ys), yref)
    # per-row scale = row amax / 448 (the largest element maps to e4m3's max)
    assert torch.allclose(ys, yref.abs().amax(dim=1) / 448, rtol=1e-5)


def test_quantize_rows_fp8():
    from kgs.ops.transformer import quantize_rows_fp8

    x = _bf(33, 1024, scale=3.0)
    x[5] = 0  # an all-zero row must not produce NaN
    y8, ys = quantize_rows_fp8(x)
    deq = _deq(y8, ys)
    assert torch.isfinite(deq).all() and deq[5].abs().max().item() == 0
    assert _close_fp8(deq, x.float())


def test_silu_mul_fp8():
    from kgs.ops.transformer import ref_silu_mul, silu_mul_fp8

    gu = _bf(48, 2 * 14336, scale=2.0)
    a8, s = silu_mul_fp8(gu)
    assert _close_fp8(_deq(a8, s), ref_silu_mul(gu).float())


@pytest.mark.parametrize("m,n,k", [(512, 768, 1024), (300, 520, 272)])
def test_gemm_fp8_rows(m, n, k):
    from kgs.ops.gemm import gemm_fp8_rows, quantize_fp8
    from kgs.ops.transformer import quantize_rows_fp8

    a = _bf(m, k) if k % 512 == 0 else None
    if a is not None:
        a8, sa = quantize_rows_fp8(a)
    else:  # odd K: build the per-row-scaled operand on the host side
        af = torch.randn(m, k, device=DEV)
        sa = af.abs().amax(dim=1) / 448
        a8 = (af / sa[:, None]).to(torch.float8_e4m3fn)
    b8, sb = quantize_fp8(torch.randn(n, k, device=DEV))
    bias = _bf(n)
    got = gemm_fp8_rows(a8, sa.contiguous(), b8, sb, bias=bias)
    ref = (a8.float() * sa[:, None]) @ (b8.float() * sb).T + bias.float()
    rel = ((got.float() - ref).abs().max() / ref.abs().max()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("rows,cols", [(1, 128256), (7, 1024), (256, 128256), (3, 8)])
def test_argmax_rows_matches_torch(rows, cols):
    """Native greedy pick == torch.argmax: first index of the maximum (ties are
    planted), NaN counts as the maximum."""
    from kgs.ops.transformer import argmax_rows

    x = torch.randn(rows, cols, device="cuda").bfloat16()
    x[0, cols // 3] = x[0, cols - 1] = 40.0  # tie: the first index wins
    if rows > 2:
        x[2, cols // 2] = float("nan")
        x[2, cols // 4] = 50.0
    got = argmax_rows(x)
    assert got.dtype == torch.int64
    assert torch.equal(got, x.argmax(dim=-1))
    assert int(got[0]) == cols // 3
