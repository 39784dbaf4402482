"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references.

GEMM checks follow cdna_hip_programming.md §3: an ASYMMETRIC B (so a swapped
C-write cannot pass), A = I, random operands over several shapes, both kernel
variants, every fused epilogue, and a backward pass through ``kgs.ops.Linear``.
"""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ref_nt(a, b, bias=None, act=None):
    y = a.float() @ b.float().T
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = torch.nn.functional.gelu(y, approximate="tanh")
    elif act == "relu":
        y = torch.relu(y)
    elif act == "silu":
        y = torch.nn.functional.silu(y)
    return y


def _rel_err(got, ref):
    return ((got.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()


@pytest.fixture(scope="module", autouse=True)
def _native():
    from kgs.ops import _lib

    _lib.lib()  # fail loudly if the HIP library is missing on a GPU box
    torch.manual_seed(0)


def test_vector_add_f32_and_bf16():
    from kgs.ops import vector_add

    for n in (1, 7, 4096, (1 << 20) + 3):
        a = torch.randn(n, device=DEV)
        b = torch.randn(n, device=DEV)
        torch.testing.assert_close(vector_add(a, b), a + b)
        ab, bb = a.bfloat16(), b.bfloat16()
        ref = (ab.float() + bb.float()).bfloat16()
        torch.testing.assert_close(vector_add(ab, bb), ref)


def test_transpose():
    from kgs.ops import transpose_bf16

    for r, c in ((1, 1), (64, 64), (100, 37), (257, 1031)):
        x = torch.randn(r, c, device=DEV).bfloat16()
        torch.testing.assert_close(transpose_bf16(x), x.T.contiguous(), rtol=0, atol=0)


def test_checksum():
    from kgs.ops import checksum

    x = torch.randn(1 << 16, device=DEV).bfloat16()
    got = checksum(x)
    ref = torch.stack([x.float().sum(), x.float().abs().sum()])
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-2)


def _gemm_v(a, b, variant, **kw):
    """Production variants via kgs.ops.gemm_nt; measured alternatives via the
    opt-in experiments library (kept correct, so they stay tested)."""
    from kgs.ops import experiments, gemm_nt
    from kgs.ops.gemm import VARIANTS

    if variant in VARIANTS:
        return gemm_nt(a, b, variant=variant, **kw)
    return experiments.gemm_nt(a, b, variant, **kw)


@pytest.mark.parametrize("variant", ["generic", "fast", "pingpong", "w4_bk32", "p32", "w4h_1_20_24_1_320000"])
def test_gemm_identity_asymmetric(variant):

    n = 256
    a = torch.eye(n, device=DEV).bfloat16()
    # B[n][k] asymmetric; C = A . B^T = B^T
    idx = torch.arange(n, device=DEV)
    b = ((idx[:, None] * 3 + idx[None, :] * 7) % 61 - 30).float().bfloat16()
    k = 256
    a2 = torch.zeros(n, k, device=DEV).bfloat16()
    a2[:, :n] = a
    c = _gemm_v(a2, b, variant)
    torch.testing.assert_close(c.float(), b.float().T, rtol=0, atol=0)


@pytest.mark.parametrize(
    "M,N,K",
    [(256, 256, 128), (512, 768, 256), (256, 512, 1024), (1024, 1024, 1024), (768, 256, 384), (2048, 1280, 640)],
)
@pytest.mark.parametrize("variant", ["fast", "pingpong", "w4_bk32", "p32"])
def test_gemm_fast_random(M, N, K, variant):
    from kgs.ops import fast_path_ok, gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    assert fast_path_ok(a, b)
    c = _gemm_v(a, b, variant)
    ref = _ref_nt(a, b)
    assert _rel_err(c, ref) < 1e-2
    # the two variants agree (same fp32 accumulation, possibly different order)
    g = gemm_nt(a, b, variant="generic")
    assert _rel_err(c, g.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (17, 33, 65), (100, 300, 70), (255, 129, 31), (1000, 24, 8)])
def test_gemm_generic_ragged(M, N, K):
    from kgs.ops import gemm_nt

    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    c = gemm_nt(a, b)
    assert _rel_err(c, _ref_nt(a, b)) < 1e-2


@pytest.mark.parametrize("variant", ["fast", "pingpong", "w4_bk32", "p32"])
def test_gemm_strided_operands(variant):
    from kgs.ops import gemm_nt

    big_a = torch.randn(512, 1024, device=DEV).bfloat16()
    big_b = torch.randn(512, 1024, device=DEV).bfloat16()
    a = big_a[:, 128:384]  # ld = 1024, K = 256
    b = big_b[:256, 256:512]
    c = _gemm_v(a, b, variant)
    assert _rel_err(c, _ref_nt(a, b)) < 1e-2


@pytest.mark.parametrize("act", ["bias", "gelu", "relu", "silu"])
@pytest.mark.parametrize("variant", ["fast", "w4_oneshot", "pingpong", "generic", "w4_bk32", "p32"])
def test_gemm_epilogues(act, variant):
    from kgs.ops import gemm_nt

    M, N, K = 512, 512, 256
    a = (torch.rand(M, K, device=DEV) - 0.5).bfloat16()
    b = (torch.rand(N, K, device=DEV) - 0.5).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    c = _gemm_v(a, b, variant, bias=bias, act=act)
    ref = _ref_nt(a, b, bias, None if act == "bias" else act)
    torch.testing.assert_close(c.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("variant", ["fast", "pingpong", "w4_bk32", "p32"])
def test_gemm_repeatable_large(variant):
    """Race screen: the pipelined kernels must be bitwise deterministic, and the
    two pipelined variants must agree bitwise (same K order per accumulator)."""
    from kgs.ops import gemm_nt

    for M, N, K in ((2048, 2048, 2048), (1024, 3072, 4096), (4096, 512, 640)):
        a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
        c0 = _gemm_v(a, b, variant)
        assert _rel_err(c0, _ref_nt(a, b)) < 1e-2
        for _ in range(10):
            assert torch.equal(_gemm_v(a, b, variant), c0)
        # same per-accumulator K order as production -> bitwise equal
        assert torch.equal(gemm_nt(a, b, variant="fast"), c0)


@pytest.mark.parametrize("M,N,K", [(1000, 1000, 1000), (300, 520, 72), (257, 264, 8), (4113, 1016, 4104),
                                   (256, 256, 136), (2048, 768, 2048)])
def test_gemm_bounded_ragged(M, N, K):
    """Variant 16: the pipelined kernel on ragged M/N/K (buffer-resource zero fill)."""
    from kgs.ops import gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    c = gemm_nt(a, b, variant="bounded")
    assert _rel_err(c, _ref_nt(a, b)) < 1e-2
    assert torch.equal(gemm_nt(a, b), c)  # auto picks the bounded kernel here
    for _ in range(3):
        assert torch.equal(gemm_nt(a, b, variant="bounded"), c)


@pytest.mark.parametrize("M,N,K,nslice", [(256, 1024, 4096, 1), (256, 1024, 4096, 4), (256, 768, 14336, 14),
                                          (128, 512, 4096, 8), (200, 264, 2048, 2), (64, 4096, 1024, 8)])
def test_gemm_splitk(M, N, K, nslice):
    """Split-K 256x256 pipeline (fp32 partial tiles + reduce) against fp32 torch;
    an asymmetric B and a strided A view catch swapped or shifted slices."""
    from kgs.ops.gemm import gemm_nt_splitk

    a_full = (torch.rand(M, K + 64, device=DEV) * 2 - 1).bfloat16()
    a = a_full[:, 32:32 + K]  # row stride K + 64, 64-B offset
    b = ((torch.rand(N, K, device=DEV) * 2 - 1) * torch.linspace(0.5, 1.5, K, device=DEV)).bfloat16()
    c = gemm_nt_splitk(a, b, nslice)
    ref = _ref_nt(a, b)
    assert _rel_err(c, ref) < 1e-2
    # slices are summed in a fixed order: repeatable bit for bit
    assert torch.equal(gemm_nt_splitk(a, b, nslice), c)


@pytest.mark.parametrize("M,N,K,bn,nslice,bm", [(256, 1024, 4096, 128, 1, 256), (200, 768, 4096, 128, 4, 256),
                                                (256, 512, 14336, 128, 8, 256), (96, 1024, 1024, 256, 2, 256),
                                                (384, 256, 2048, 256, 1, 256), (130, 384, 640, 128, 5, 256),
                                                (128, 1024, 4096, 256, 2, 128), (64, 512, 2048, 128, 4, 128),
                                                (100, 768, 1024, 256, 1, 128), (200, 256, 640, 128, 5, 128)])
def test_gemm_w4x_decode_shapes(M, N, K, bn, nslice, bm):
    """The four-wave decode GEMM (any M, 256x128 / 256x256 tiles, K slices)
    against fp32 torch; slices are summed in a fixed order (repeatable bits)."""
    from kgs.ops.gemm import gemm_nt_w4x

    a_full = (torch.rand(M, K + 64, device=DEV) * 2 - 1).bfloat16()
    a = a_full[:, 32:32 + K]
    b = ((torch.rand(N, K, device=DEV) * 2 - 1) * torch.linspace(0.5, 1.5, K, device=DEV)).bfloat16()
    c = gemm_nt_w4x(a, b, bn=bn, nslice=nslice, bm=bm)
    assert _rel_err(c, _ref_nt(a, b)) < 1e-2
    assert torch.equal(gemm_nt_w4x(a, b, bn=bn, nslice=nslice, bm=bm), c)
    if bm == 128:  # same MFMA order along K as the 256-row tile: same bits
        assert torch.equal(gemm_nt_w4x(a, b, bn=bn, nslice=nslice), c)


def test_splitk_workspace_is_stable_for_graphs():
    """The partial-tile buffer reserved under torch.device("cuda") is the one
    calls on "cuda:0" use (no silent second allocation), and a growth retires the
    old buffer instead of freeing it (hipGraphs captured earlier point at it)."""
    from kgs.ops import decode as D
    from kgs.ops.gemm import gemm_nt_splitk, reserve_splitk_workspace

    ws = reserve_splitk_workspace(torch.device("cuda"), D.SPLITK_WS_FLOATS)
    a = (torch.rand(256, 4096, device="cuda:0") * 2 - 1).bfloat16()
    for n, ns in ((4096, 8), (6144, 8), (4096, 16)):
        b = (torch.rand(n, 4096, device=DEV) * 2 - 1).bfloat16()
        gemm_nt_splitk(a, b, ns)
        assert reserve_splitk_workspace(torch.device("cuda", 0), 1).data_ptr() == ws.data_ptr()
    big = reserve_splitk_workspace(torch.device("cuda"), ws.numel() + 1024)
    assert big.data_ptr() != ws.data_ptr() and any(r is ws for r in D._RETIRED)


def test_gemm_bounded_matches_fast_on_aligned():
    from kgs.ops import gemm_nt

    a = (torch.rand(1024, 2048, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(768, 2048, device=DEV) * 2 - 1).bfloat16()
    assert torch.equal(gemm_nt(a, b, variant="bounded"), gemm_nt(a, b, variant="fast"))
    assert torch.equal(gemm_nt(a, b, variant="pingpong"), gemm_nt(a, b, variant="fast"))


def test_gemm_auto_routes_aligned_to_four_wave_kernel():
    """auto == the four-wave kernel on aligned shapes; its knob variants (the
    experiments library) compute the identical image."""
    from kgs.ops import experiments, gemm_nt

    # K = 1280: 20 K-steps, enough for every variant's peeled ones (w4pq16x1n: 18 + 2)
    a = (torch.rand(2048, 1280, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(1536, 1280, device=DEV) * 2 - 1).bfloat16()
    c = gemm_nt(a, b, variant="w4")
    assert _rel_err(c, _ref_nt(a, b)) < 1e-2
    assert torch.equal(gemm_nt(a, b), c)
    for name in experiments.W4H:
        if name in experiments.NO_OUTPUT:  # measurement builds that do not write C
            continue
        assert torch.equal(experiments.gemm_nt(a, b, name), c), name


@pytest.mark.parametrize("act", ["bias", "gelu"])
def test_gemm_bounded_partial_columns_and_epilogue(act):
    """N % 8 != 0 inside a padded output (ldc % 8 == 0): the predicated store tail."""
    from kgs.ops import gemm_nt

    M, N, K = 300, 251, 96
    a = (torch.rand(M, K, device=DEV) - 0.5).bfloat16()
    b = (torch.rand(N, K, device=DEV) - 0.5).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    big = torch.full((M, 256), 7.0, device=DEV, dtype=torch.bfloat16)
    out = big[:, :N]
    gemm_nt(a, b, bias=bias, act=act, out=out, variant="bounded")
    torch.testing.assert_close(out.float(), _ref_nt(a, b, bias, None if act == "bias" else act), rtol=2e-2,
                               atol=2e-2)
    assert torch.all(big[:, N:] == 7.0)  # nothing written past N


def test_gemm_wide_store_tail_matches_narrow():
    """The permlane16-swap 16-B store tail writes exactly the image of the 8-B one."""
    from kgs.ops import gemm_nt

    for M, N, K in ((512, 768, 256), (2048, 2048, 2048)):
        a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
        assert torch.equal(gemm_nt(a, b, variant="fast"), _gemm_v(a, b, "narrow_store"))


def test_gemm_misaligned_out_and_bias_fall_back():
    from kgs.ops import gemm_nt
    from kgs.ops._lib import KernelError
    from kgs.ops.gemm import fast_path_ok

    M, N, K = 512, 512, 256
    a = (torch.rand(M, K, device=DEV) - 0.5).bfloat16()
    b = (torch.rand(N, K, device=DEV) - 0.5).bfloat16()
    big = torch.zeros(M, N + 8, device=DEV, dtype=torch.bfloat16)
    out = big[:, 4:4 + N]  # 8-B aligned rows: too narrow for the 16-B store tail
    assert not fast_path_ok(a, b, out)
    gemm_nt(a, b, out=out)
    assert _rel_err(out, _ref_nt(a, b)) < 1e-2
    with pytest.raises(KernelError):
        gemm_nt(a, b, out=out, variant="fast")
    bias_store = torch.randn(N + 1, device=DEV).bfloat16()
    bias = bias_store[1:]  # 2-B aligned
    c = gemm_nt(a, b, bias=bias, act="relu")
    torch.testing.assert_close(c.float(), _ref_nt(a, b, bias, "relu"), rtol=2e-2, atol=2e-2)


def test_matmul_and_linear_backward():
    from kgs.ops import Linear, matmul

    a = torch.randn(256, 512, device=DEV).bfloat16()
    b = torch.randn(512, 384, device=DEV).bfloat16()
    assert _rel_err(matmul(a, b), a.float() @ b.float()) < 1e-2

    torch.manual_seed(1)
    lin = Linear(512, 256, act="gelu", device=DEV)
    x = torch.randn(128, 512, device=DEV).bfloat16().requires_grad_(True)
    y = lin(x)
    gy = torch.randn_like(y)
    y.backward(gy)

    xr = x.detach().float().requires_grad_(True)
    wr = lin.weight.detach().float().requires_grad_(True)
    br = lin.bias.detach().float().requires_grad_(True)
    yr = torch.nn.functional.gelu(xr @ wr.T + br, approximate="tanh")
    yr.backward(gy.float())
    assert _rel_err(y, yr) < 2e-2
    assert _rel_err(x.grad, xr.grad) < 3e-2
    assert _rel_err(lin.weight.grad, wr.grad) < 3e-2
    assert _rel_err(lin.bias.grad, br.grad) < 3e-2


# ----------------------------------------------------------------- fp8 GEMM --
def _fp8_pair(M, N, K, seed=0):
    from kgs.ops import quantize_fp8

    g = torch.Generator(device=DEV).manual_seed(seed)
    a = torch.randn(M, K, device=DEV, generator=g)
    b = torch.randn(N, K, device=DEV, generator=g)
    qa, sa = quantize_fp8(a)
    qb, sb = quantize_fp8(b)
    return qa, sa, qb, sb


def _fp8_ref(qa, sa, qb, sb, bias=None, act=None):
    y = (qa.float() * sa) @ (qb.float() * sb).T
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = torch.nn.functional.gelu(y, approximate="tanh")
    return y


def test_gemm_fp8_identity_asymmetric():
    """A = I, B with distinct small integers (exact in e4m3): C must equal B
    exactly, so a transposed or mis-paired K layout cannot pass."""
    from kgs.ops import gemm_fp8_nt

    K = 256
    a = torch.eye(K, device=DEV).to(torch.float8_e4m3fn)
    bf = ((torch.arange(256 * K, device=DEV) * 7 % 31) - 15).float().reshape(256, K)
    b = bf.to(torch.float8_e4m3fn)
    c = gemm_fp8_nt(a, b)
    assert torch.equal(c.float(), bf.T)


@pytest.mark.parametrize("M,N,K,variant", [(512, 512, 512, "fast"), (1024, 768, 2048, "fast"),
                                           (300, 520, 144, "bounded"), (257, 264, 16, "bounded"),
                                           (2048, 1024, 4096, "auto")])
def test_gemm_fp8_random(M, N, K, variant):
    from kgs.ops import gemm_fp8_nt

    qa, sa, qb, sb = _fp8_pair(M, N, K)
    c = gemm_fp8_nt(qa, qb, sa, sb, variant=variant)
    assert _rel_err(c, _fp8_ref(qa, sa, qb, sb)) < 1e-2
    for _ in range(3):
        assert torch.equal(gemm_fp8_nt(qa, qb, sa, sb, variant=variant), c)


def test_gemm_fp8_epilogue_and_bounded_equals_fast():
    from kgs.ops import gemm_fp8_nt

    qa, sa, qb, sb = _fp8_pair(512, 768, 1024, seed=3)
    bias = torch.randn(768, device=DEV).bfloat16()
    c = gemm_fp8_nt(qa, qb, sa, sb, bias=bias, act="gelu")
    torch.testing.assert_close(c.float(), _fp8_ref(qa, sa, qb, sb, bias, "gelu"), rtol=2e-2, atol=2e-2)
    assert torch.equal(gemm_fp8_nt(qa, qb, sa, sb, variant="bounded"), gemm_fp8_nt(qa, qb, sa, sb, variant="fast"))


# ------------------------------------------------- transposed-read layouts --
@pytest.mark.parametrize("force_tr", [True, False])
@pytest.mark.parametrize("trans_a,trans_b", [(False, False), (True, False), (True, True), (False, True)])
@pytest.mark.parametrize("M,N,K", [(256, 512, 128), (1024, 768, 2048), (512, 512, 384)])
def test_gemm_layouts_bitwise_vs_nt(trans_a, trans_b, M, N, K, force_tr, monkeypatch):
    """Every layout, through the tr-read path (forced) and through the measured
    default routing, must equal the NT kernel on the explicitly transposed
    operands bit for bit (same K order per accumulator)."""
    import kgs.ops.gemm as gm
    from kgs.ops import gemm_bf16 as gemm
    from kgs.ops import gemm_nt

    if force_tr:
        monkeypatch.setattr(gm, "TR_READ_A", True)
        monkeypatch.setattr(gm, "TR_READ_B_MAX_M", 1 << 30)

    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a_mk = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).bfloat16()
    b_nk = (torch.rand(N, K, device=DEV, generator=g) * 2 - 1).bfloat16()
    a = a_mk.t().contiguous() if trans_a else a_mk
    b = b_nk if trans_b else b_nk.t().contiguous()
    c = gemm(a, b, trans_a=trans_a, trans_b=trans_b)
    ref = gemm_nt(a_mk, b_nk)
    assert torch.equal(c, ref)
    assert _rel_err(c, _ref_nt(a_mk, b_nk)) < 1e-2


def test_gemm_layout_asymmetric_identity(monkeypatch):
    """A = I stored K-major, B asymmetric stored K-major: C must be B exactly
    (tr-read path forced for both operands)."""
    import kgs.ops.gemm as gm
    from kgs.ops import gemm_bf16 as gemm

    monkeypatch.setattr(gm, "TR_READ_A", True)
    monkeypatch.setattr(gm, "TR_READ_B_MAX_M", 1 << 30)

    M = K = 256
    N = 512
    eye = torch.eye(K, device=DEV).bfloat16()
    b_kn = ((torch.arange(K * N, device=DEV) % 97) - 48).float().reshape(K, N).bfloat16()
    c = gemm(eye, b_kn, trans_a=True)  # A stored [K][M]; B stored [K][N]
    assert torch.equal(c, b_kn)


def test_gemm_layout_epilogue_and_fallback():
    from kgs.ops import gemm_bf16 as gemm

    a = (torch.rand(300, 96, device=DEV) - 0.5).bfloat16()   # ragged: falls back to transpose + NT
    b = (torch.rand(96, 200, device=DEV) - 0.5).bfloat16()
    torch.testing.assert_close(gemm(a, b).float(), a.float() @ b.float(), rtol=2e-2, atol=2e-2)
    a = (torch.rand(512, 256, device=DEV) - 0.5).bfloat16()
    b = (torch.rand(256, 768, device=DEV) - 0.5).bfloat16()
    bias = torch.randn(768, device=DEV).bfloat16()
    ref = torch.nn.functional.gelu(a.float() @ b.float() + bias.float(), approximate="tanh")
    torch.testing.assert_close(gemm(a, b, bias=bias, act="gelu").float(), ref, rtol=2e-2, atol=2e-2)


# ------------------------------------------------------ fp8 quant + W8A8 --
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_quantize_fp8_dev_matches_reference(dtype):
    from kgs.ops import quantize_fp8_dev

    x = (torch.randn(4096, 1024, device=DEV) * 3).to(dtype)
    q, s = quantize_fp8_dev(x)
    amax = x.float().abs().max()
    torch.testing.assert_close(s, (amax / 448).reshape(1), rtol=1e-6, atol=0)
    ref = (x.float() * (1.0 / s)).clamp(-448, 448).to(torch.float8_e4m3fn)
    same = (q.view(torch.uint8) == ref.view(torch.uint8)).float().mean().item()
    assert same > 0.999, same  # rounding of x * (1/scale) may differ in the last bit
    deq = q.float() * s
    assert torch.all((deq - x.float()).abs() <= 0.0625 * x.float().abs() + 2 * s * 2 ** -9)


def test_gemm_fp8_device_scale_and_fp8_linear():
    from kgs.ops import Fp8Linear, Linear, gemm_fp8_nt, quantize_fp8, quantize_fp8_dev

    torch.manual_seed(0)
    x = torch.randn(1024, 2048, device=DEV).bfloat16()
    w = torch.randn(768, 2048, device=DEV).bfloat16() * 0.02
    qx, sx = quantize_fp8_dev(x)
    qw, sw = quantize_fp8(w)
    dev = gemm_fp8_nt(qx, qw, sx, sw)
    host = gemm_fp8_nt(qx, qw, float(sx.item()), sw)
    torch.testing.assert_close(dev.float(), host.float(), rtol=1e-2, atol=1e-3)

    lin = Linear(2048, 768, bias=True, act="gelu", device=DEV)
    with torch.no_grad():
        lin.weight.copy_(w)
        lin.bias.copy_(torch.randn(768, device=DEV).bfloat16() * 0.1)
    f8 = Fp8Linear.from_linear(lin)
    with torch.no_grad():
        ref = lin(x).float()
        got = f8(x).float()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 0.05, rel

    # the W8A8 forward has no host sync: capture it and replay on new data
    xs = torch.zeros_like(x)
    f8(xs)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ys = f8(xs)
    xs.copy_(x)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(ys, f8(x))


def test_timing_probes_refuse_without_opt_in():
    from kgs.ops import experiments

    a = (torch.rand(256, 256, device=DEV) * 2 - 1).bfloat16()
    with pytest.raises(ValueError):
        experiments.gemm_nt(a, a, "probe_l2")
    experiments.gemm_nt(a, a, "probe_l2", allow_wrong=True)  # runs, result undefined
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,I,K,bn,bm", [(256, 1024, 4096, 128, 256), (200, 768, 1024, 128, 256),
                                         (512, 1024, 2048, 256, 256), (130, 512, 640, 256, 256),
                                         (128, 1024, 2048, 256, 128), (72, 512, 1024, 128, 128)])
def test_gemm_w4x_swiglu_epilogue(M, I, K, bn, bm):
    """SwiGLU in the four-wave kernel's epilogue == the gate|up GEMM followed by
    silu_mul, bit for bit (same roundings), and close to fp32 torch."""
    from kgs.ops.gemm import gemm_nt_w4x, gemm_nt_w4x_swiglu
    from kgs.ops.transformer import silu_mul

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(2 * I, K, device=DEV) * 2 - 1) * K ** -0.5 *
         torch.linspace(0.5, 1.5, K, device=DEV)).bfloat16()
    fused = gemm_nt_w4x_swiglu(a, w, bn=bn, bm=bm)
    assert fused.shape == (M, I)
    ref = silu_mul(gemm_nt_w4x(a, w, bn=bn, nslice=1))
    assert torch.equal(fused, ref)
    gu = a.float() @ w.float().T
    r32 = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
    assert ((fused.float() - r32).abs().max() / r32.abs().max()).item() < 2e-2


@pytest.mark.parametrize("M,N,K", [(8192, 4096, 4096), (4096, 8192, 1024), (4096, 4096, 4096), (2048, 1024, 4096),
                                   (1024, 512, 768), (16384, 4096, 1024),
                                   # the long-K persistent instances (tile groups of 8), tall and wide --
                                   # Llama-8B's prompt-pass down projection is 8192 x 4096 x 14336
                                   (8192, 4096, 14336), (4096, 8192, 14336)])
def test_residual_add_epilogue_is_bitwise_gemm_then_add(M, N, K):
    """Round 5: the prompt pass's o / down GEMM with the residual add in its
    store (EPI_ADDC; persistent and one-shot grids, tall and wide) leaves x
    bitwise where gemm_nt + add_rmsnorm's add leaves it, and the plain rmsnorm
    after it gives add_rmsnorm's normalised rows. With more tiles than CUs the
    launch is the persistent kernel: on a fresh stream it takes a ticket slot."""
    from kgs.ops import gemm_nt
    from kgs.ops._lib import tile_queue_check, tile_queue_stats
    from kgs.ops.gemm import addc_ok, gemm_nt_add_
    from kgs.ops.transformer import add_rmsnorm

    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).bfloat16()
    b = ((torch.rand(N, K, device=DEV, generator=g) * 2 - 1) * K ** -0.5).bfloat16()
    x0 = (torch.rand(M, N, device=DEV, generator=g) * 4 - 2).bfloat16()
    w = (torch.rand(N, device=DEV, generator=g) + 0.5).bfloat16()
    x_ref = x0.clone()
    y_ref = add_rmsnorm(x_ref, gemm_nt(a, b), w)
    x = x0.clone()
    assert addc_ok(a, b, x)
    torch.cuda.synchronize()
    st0 = tile_queue_stats()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        gemm_nt_add_(a, b, x)
    torch.cuda.synchronize()
    persistent = (M // 256) * (N // 256) > torch.cuda.get_device_properties(DEV).multi_processor_count
    assert tile_queue_stats()["stream_slots"] == st0["stream_slots"] + int(persistent)
    assert torch.equal(x, x_ref)
    assert torch.equal(add_rmsnorm(x, None, w), y_ref)
    assert not addc_ok(a[: M - 8], b, x[: M - 8])  # unaligned rows: the caller keeps the unfused pair
    assert tile_queue_check()["dirty_slots"] == 0


def test_residual_add_epilogue_in_a_graph_takes_no_ticket_slot():
    """a captured EPI_ADDC launch runs the one-shot grid (a graph
    exec replayed concurrently with itself may compute a persistent tile twice,
    and C += A.B^T would add twice): no capture slot is taken, and one replay
    adds exactly once, bitwise the eager launch."""
    from kgs.ops._lib import tile_queue_stats
    from kgs.ops.gemm import gemm_nt_add_

    M, N, K = 8192, 4096, 4096
    g = torch.Generator(device=DEV).manual_seed(11)
    a = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).bfloat16()
    b = ((torch.rand(N, K, device=DEV, generator=g) * 2 - 1) * K ** -0.5).bfloat16()
    x0 = (torch.rand(M, N, device=DEV, generator=g) * 4 - 2).bfloat16()
    want = gemm_nt_add_(a, b, x0.clone())
    x = x0.clone()
    st0 = tile_queue_stats()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gemm_nt_add_(a, b, x)
    assert tile_queue_stats()["capture_slots"] == st0["capture_slots"]
    x.copy_(x0)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(x, want)
    del graph


@pytest.mark.parametrize("M,I,K", [(2048, 8192, 1024), (1024, 14336, 4096), (4096, 4096, 768)])
def test_prompt_swiglu_on_the_persistent_kernel(M, I, K):
    """Round 5: the prompt pass's gate|up (256 x 256 tiles, aligned M, more tiles
    than CUs) runs on the persistent kernel with the SwiGLU epilogue. It equals
    the plain GEMM + silu_mul bit for bit, and a captured launch takes a ticket
    slot of its own (i.e. it IS the persistent kernel), bitwise the eager result."""
    from kgs.ops._lib import tile_queue_check, tile_queue_stats
    from kgs.ops.gemm import gemm_nt_w4x, gemm_nt_w4x_swiglu
    from kgs.ops.transformer import silu_mul

    g = torch.Generator(device=DEV).manual_seed(M + I)
    a = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(2 * I, K, device=DEV, generator=g) * 2 - 1) * K ** -0.5).bfloat16()
    fused = gemm_nt_w4x_swiglu(a, w, bn=256, bm=256)
    ref = silu_mul(gemm_nt_w4x(a, w, bn=256, nslice=1))
    assert torch.equal(fused, ref)
    gu = a[:256].float() @ w.float().T
    r32 = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
    assert ((fused[:256].float() - r32).abs().max() / r32.abs().max()).item() < 2e-2
    st0 = tile_queue_stats()
    out = torch.zeros_like(fused)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gemm_nt_w4x_swiglu(a, w, bn=256, bm=256, out=out)
    st1 = tile_queue_stats()
    assert st1["capture_slots"] == st0["capture_slots"] + 1 and st1["fallbacks"] == st0["fallbacks"], (st0, st1)
    for _ in range(2):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, fused)
        assert tile_queue_check()["dirty_slots"] == 0
    del graph


@pytest.mark.parametrize("M,N,K", [(4096, 512, 640), (2048, 256, 1024), (768, 256, 384)])
def test_gemm_tall_mirrored_schedule_is_bitwise_the_default(M, N, K):
    """M > N runs the mirrored schedule (GROUP_N order, B's DMAs first, round 3):
    only tile order and DMA issue order differ, so the result must be bitwise
    the default schedule's (experiment w4h_1_24_20_1_0) and match fp32."""
    from kgs.ops import gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    fast = gemm_nt(a, b, variant="fast")
    default = _gemm_v(a, b, "w4h_1_24_20_1_0")
    assert torch.equal(fast, default)
    assert _rel_err(fast, _ref_nt(a, b)) < 1e-2
    # an asymmetric exact check: B^T stacked under itself, A = [I; I]
    a2 = torch.zeros(M, K, device=DEV).bfloat16()
    idx = torch.arange(M, device=DEV)
    a2[idx, idx % min(N, K)] = 1.0
    b2 = ((torch.arange(N, device=DEV)[:, None] * 3 + torch.arange(K, device=DEV)[None, :] * 7) % 61 - 30).float()
    c = gemm_nt(a2, b2.bfloat16(), variant="fast")
    ref = b2.T[idx % min(N, K)]  # row i of C = row (i mod min(N,K)) of B^T
    torch.testing.assert_close(c.float(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("M,I,K,bn,nslice", [(256, 1024, 4096, 256, 2), (200, 768, 1024, 128, 4), (64, 512, 3072, 256, 3)])
def test_gemm_splitk_swiglu_matches_gemm_then_silu_mul(M, I, K, bn, nslice):
    """Split-K gate|up + the fused reduce-and-SwiGLU pass: the roundings of
    gemm_nt + silu_mul (products rounded to bf16 first), close to fp32."""
    from kgs.ops.gemm import gemm_nt_w4x, gemm_nt_w4x_splitk_swiglu
    from kgs.ops.transformer import silu_mul

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(2 * I, K, device=DEV) * 2 - 1) * 0.05).bfloat16()
    got = gemm_nt_w4x_splitk_swiglu(a, w, bn=bn, nslice=nslice)
    # same partials reduced by the plain split-K path, then silu_mul: bitwise
    want = silu_mul(gemm_nt_w4x(a, w, bn=bn, nslice=nslice))
    assert torch.equal(got, want)
    ref = a.float() @ w.float().T
    ref = torch.nn.functional.silu(ref[:, :I]) * ref[:, I:]
    assert _rel_err(got, ref) < 2e-2


@pytest.mark.parametrize("M,N,K,bn,bm,nslice", [(256, 1024, 4096, 256, 256, 1), (200, 768, 1024, 128, 256, 1),
                                                (72, 512, 1024, 128, 128, 1), (64, 1024, 2048, 256, 256, 2),
                                                (130, 512, 3072, 128, 256, 3)])
def test_gemm_w4x_packed_weight_is_bitwise_the_unpacked(M, N, K, bn, bm, nslice):
    """PACKB (round 3): a weight packed tile-panel major gives the same bits as
    the row-major weight (only the B addresses change), incl. split-K slices."""
    from kgs.ops.gemm import gemm_nt_w4x, pack_w4x_weight

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=DEV) * 2 - 1) * 0.05).bfloat16()
    pw = pack_w4x_weight(w, bn)
    got = gemm_nt_w4x(a, pw, bn=bn, nslice=nslice, bm=bm)
    assert torch.equal(got, gemm_nt_w4x(a, w, bn=bn, nslice=nslice, bm=bm))
    assert _rel_err(got, _ref_nt(a, w)) < 1e-2
    with pytest.raises(ValueError):
        gemm_nt_w4x(a, pw, bn=384 - bn, nslice=nslice, bm=bm)


@pytest.mark.parametrize("M,I,K,bn,bm", [(256, 1024, 4096, 128, 256), (200, 768, 1024, 128, 256),
                                         (512, 1024, 2048, 256, 256), (72, 512, 1024, 128, 128)])
def test_gemm_w4x_swiglu_packed_weight_is_bitwise_the_unpacked(M, I, K, bn, bm):
    from kgs.ops.gemm import gemm_nt_w4x_swiglu, pack_w4x_weight

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(2 * I, K, device=DEV) * 2 - 1) * K ** -0.5).bfloat16()
    got = gemm_nt_w4x_swiglu(a, pack_w4x_weight(w, bn, swiglu=True), bn=bn, bm=bm)
    assert torch.equal(got, gemm_nt_w4x_swiglu(a, w, bn=bn, bm=bm))


@pytest.mark.parametrize("M,N,K,bn,bm,nslice,stages", [
    (256, 1024, 640, 128, 256, 1, 3), (200, 768, 1024, 128, 256, 2, 3), (72, 512, 1152, 128, 128, 1, 4),
    (128, 1024, 2048, 128, 128, 4, 4), (130, 512, 1152, 256, 128, 1, 3), (256, 512, 768, 128, 128, 3, 3)])
def test_gemm_w4x_lds_stages_are_bitwise_two_stage(M, N, K, bn, bm, nslice, stages):
    """3 / 4 LDS stages (more K-tiles in flight) change only when tiles are
    loaded: bitwise the two-stage result, incl. K-tile counts that are not a
    multiple of the stage count, split-K and packed weights."""
    from kgs.ops.gemm import gemm_nt_w4x, pack_w4x_weight

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=DEV) * 2 - 1) * 0.05).bfloat16()
    want = gemm_nt_w4x(a, w, bn=bn, nslice=nslice, bm=bm)
    assert torch.equal(gemm_nt_w4x(a, w, bn=bn, nslice=nslice, bm=bm, stages=stages), want)
    pw = pack_w4x_weight(w, bn)
    assert torch.equal(gemm_nt_w4x(a, pw, bn=bn, nslice=nslice, bm=bm, stages=stages), want)
    assert _rel_err(want, _ref_nt(a, w)) < 1e-2


@pytest.mark.parametrize("M,I,K,bn,bm,stages", [(256, 1024, 640, 128, 256, 3), (72, 512, 1024, 128, 128, 4),
                                                (200, 768, 1152, 128, 128, 3)])
def test_gemm_w4x_swiglu_lds_stages_are_bitwise_two_stage(M, I, K, bn, bm, stages):
    from kgs.ops.gemm import gemm_nt_w4x_swiglu

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(2 * I, K, device=DEV) * 2 - 1) * K ** -0.5).bfloat16()
    assert torch.equal(gemm_nt_w4x_swiglu(a, w, bn=bn, bm=bm, stages=stages), gemm_nt_w4x_swiglu(a, w, bn=bn, bm=bm))


def test_gemm_w4x_stages_that_do_not_fit_are_refused():
    from kgs.ops.gemm import gemm_nt_w4x

    a = torch.zeros(256, 256, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        gemm_nt_w4x(a, a, bn=256, bm=256, stages=3)  # 3 x 64 KiB > 160 KiB


@pytest.mark.parametrize("M,N,K", [(2048, 1024, 1024), (1024, 2048, 512), (512, 512, 768), (4096, 2048, 256),
                                   (2048, 4096, 512), (768, 2048, 1280)])
def test_gemm_small_grid_routing_is_bitwise_the_256_tile(M, N, K):
    """Auto routes grids of <= 128 256x256 tiles to 256x128 / 128x256 / 128x128
    four-wave tiles (round 3): same per-element MFMA chain, so bitwise the
    forced 256x256 result, and close to fp32."""
    from kgs.ops import gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    auto = gemm_nt(a, b)
    assert torch.equal(auto, gemm_nt(a, b, variant="fast"))
    assert _rel_err(auto, _ref_nt(a, b)) < 1e-2


@pytest.mark.parametrize("M,N,K,variant", [(8192, 8192, 384, "w4p_0"), (4608, 4096, 384, "w4p_0"),
                                           (8192, 2304, 512, "w4p_140000000"), (1024, 768, 1024, "w4p_0"),
                                           (4608, 4096, 384, "w4pn_0"), (8192, 2304, 9216, "w4pn_140000008"),
                                           # round 4: LDS layout 1 and the MFMA-order knobs
                                           (4608, 4096, 384, "w4pl_0"), (8192, 2304, 9216, "w4pl_140000008"),
                                           (8192, 2304, 512, "w4pl_140000000"), (4096, 4608, 8320, "w4pl_8"),
                                           (4608, 4096, 384, "w4po0_0"), (4608, 4096, 384, "w4po2_0"),
                                           (8192, 2304, 9216, "w4po2_140000008"),
                                           # round 5: drain after each tile's stores (measurement build)
                                           (8192, 8192, 384, "w4pd_0"), (8192, 8192, 384, "w4pw_0"),
                                           (8192, 2304, 9216, "w4pw_0"), (4608, 4096, 384, "w4pw_0"),
                                           # round 6: deferred C stores (gemm_w4p.h DD, SPS)
                                           (8192, 8192, 1024, "w4pq8x2n_0"), (4608, 4096, 768, "w4pq8x2n_0"),
                                           (1024, 768, 1024, "w4pq8x2n_0"), (8192, 8192, 2048, "w4pq4x4n_0"),
                                           (8192, 8192, 1024, "w4pq8x1n_0"), (8192, 8192, 1024, "w4pq10x2n_0"),
                                           (8192, 8192, 1280, "w4pq16x1n_0"), (8192, 8192, 1024, "w4pq12x1n_0"),
                                           (8192, 8192, 1024, "w4pq8x2_0"), (8192, 2304, 9216, "w4pq8x2_140000008"),
                                           (8192, 2304, 9216, "w4pq8x2n_140000008"), (4096, 4608, 8320, "w4pq8x2n_8"),
                                           (8192, 8192, 1024, "w4pq1x16n_0"), (8192, 8192, 1024, "w4pq2x8n_0"),
                                           (8192, 8192, 1024, "w4pq3x6n_0"), (8192, 8192, 1024, "w4pq2x10n_0"),
                                           (8192, 8192, 1024, "w4pq4x5n_0"), (8192, 2304, 9216, "w4pq4x4_140000008"),
                                           (8192, 2304, 9216, "w4pq4x4n_140000008"), (8192, 8192, 1024, "w4pq4x4_0"),
                                           (4096, 4608, 8320, "w4pq4x4_8"), (8192, 2304, 9216, "w4pq2x8_140000008"),
                                           (8192, 8192, 1024, "w4pq2x8_0"), (1024, 768, 1024, "w4pq1x16n_0"),
                                           # round 6: one barrier per K-step
                                           (8192, 8192, 1024, "w4pb_0"), (4608, 4096, 384, "w4pb_0"),
                                           (1024, 768, 1024, "w4pb_0"), (8192, 8192, 1024, "w4pbw48_0"),
                                           (8192, 8192, 1024, "w4pbw32_0"), (8192, 8192, 1024, "w4pbq4x4_0"),
                                           (8192, 2304, 9216, "w4pbt_140000008"), (4096, 4608, 8320, "w4pbt_8"),
                                           (8192, 8192, 1024, "w4pbt_0"), (8192, 8192, 1024, "w4pbw64_0"),
                                           # round 6: K-step schedule (barrier 1 / barrier 2 placement)
                                           (8192, 8192, 1024, "w4pk20r20q4x4n_0"),
                                           (8192, 8192, 1024, "w4pk24r16q4x4n_0"),
                                           (8192, 8192, 1024, "w4pk20r16q4x4n_0"),
                                           (8192, 8192, 1024, "w4pk18r16q4x4n_0"),
                                           (4608, 4096, 768, "w4pk18r16q4x4n_0"),
                                           (8192, 2304, 9216, "w4pk24r16_140000008"),
                                           (8192, 2304, 9216, "w4pk20r16_140000008"),
                                           (8192, 8192, 1024, "w4pk20r24q4x4n_0"),
                                           (8192, 8192, 1024, "w4pk18r24q4x4n_0"),
                                           (8192, 8192, 1024, "w4pk24r24q4x4n_0"),
                                           (8192, 2304, 9216, "w4pk20r24_140000008")])
def test_gemm_persistent_is_bitwise_the_one_shot_kernel(M, N, K, variant):
    """The persistent four-wave kernel (gemm_w4p.h: one workgroup per CU walking
    tiles, named accumulator AGPRs, the next tile's K-tiles loaded by the last
    K-steps) runs gemm_w4.h's K-step, so it must reproduce the one-shot kernel
    bit for bit -- with several tiles per workgroup (1024 / 288 / 288 tiles on
    256 CUs: 4 each, 1-2 each, 1-2 in the mirrored tall order) and with fewer
    tiles than CUs (12)."""
    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    one_shot = _gemm_v(a, b, "w4h_1_24_20_1_0")
    pers = _gemm_v(a, b, variant)
    assert torch.equal(pers, one_shot)
    assert _rel_err(pers, _ref_nt(a, b)) < 1e-2
    # run twice more on other data: nothing carried over between launches/tiles
    a2 = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    assert torch.equal(_gemm_v(a2, b, variant), _gemm_v(a2, b, "w4h_1_24_20_1_0"))


@pytest.mark.parametrize("M,N,K", [(8192, 8192, 384), (8192, 12288, 512), (8192, 8192, 2048), (12288, 8192, 4096),
                                   (8192, 8192, 8192)])
def test_gemm_auto_nt_store_route_is_bitwise_the_one_shot_kernel(M, N, K):
    """3-8 tiles per CU, plain C, not tall, K <= 8192: production stores C
    non-temporally, half of it deferred into the next tile's first K-steps
    from K = 512 (gemm_persistent.hip); the image is the one-shot kernel's, and
    repeated launches keep it (the deferred stores' counted waits)."""
    from kgs.ops import gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    one_shot = _gemm_v(a, b, "w4h_1_24_20_1_0")
    for _ in range(3):
        assert torch.equal(gemm_nt(a, b), one_shot)
    assert torch.equal(gemm_nt(a, b), _gemm_v(a, b, "w4pn_0" if K < 512 else "w4pq4x4n_0"))


def test_deferred_store_route_with_a_strided_output():
    """The deferred C units are stored through a buffer resource on the previous
    tile's rows at stride ldc: with C a column slice of a wider matrix (ldc > N)
    the image is the one-shot kernel's, and the columns outside the slice are
    untouched (the resource's range covers only the tile's rows)."""
    from kgs.ops import gemm_nt

    M, N, K = 8192, 8192, 1024
    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    wide = torch.full((M, N + 512), 7.0, device=DEV, dtype=torch.bfloat16)
    out = wide[:, 256:256 + N]
    assert out.stride(0) == N + 512
    gemm_nt(a, b, out=out)
    assert torch.equal(out, gemm_nt(a, b, variant="w4_oneshot"))
    assert bool((wide[:, :256] == 7.0).all()) and bool((wide[:, 256 + N:] == 7.0).all())


@pytest.mark.parametrize("M,N,K", [(8192, 8192, 8192), (8192, 4096, 14336), (16384, 16384, 8192)])
def test_production_route_at_the_bench_shapes_in_full(M, N, K):
    """gemm_nt's default route at the headline shapes (8192^3:
    persistent, non-temporal C; 8192 x 4096 x 14336: tall, long-K mirrored
    tile-group-8 map; 16384^2 x 8192: persistent, 16 tiles per CU) against an
    fp32 reference over the WHOLE output, and bitwise the one-shot grid of the
    same K-step. The route is the persistent kernel: on a fresh stream the
    launch takes a ticket slot."""
    from kgs.ops import gemm_nt
    from kgs.ops._lib import tile_queue_check, tile_queue_stats

    g = torch.Generator(device=DEV).manual_seed(M + 3 * N + 7 * K)
    a = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV, generator=g) * 2 - 1).bfloat16()
    torch.cuda.synchronize()
    st0 = tile_queue_stats()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        c = gemm_nt(a, b)
    torch.cuda.synchronize()
    assert tile_queue_stats()["stream_slots"] == st0["stream_slots"] + 1
    assert tile_queue_check()["dirty_slots"] == 0
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        bf, err, amax = b.float(), 0.0, 0.0
        for r0 in range(0, M, 2048):
            ref = a[r0:r0 + 2048].float() @ bf.T
            err = max(err, (c[r0:r0 + 2048].float() - ref).abs().max().item())
            amax = max(amax, ref.abs().max().item())
            del ref
    finally:
        torch.backends.cuda.matmul.allow_tf32 = prev
    assert err / amax < 1e-2, err / amax
    assert torch.equal(c, gemm_nt(a, b, variant="w4_oneshot"))


def test_gemm_persistent_counted_store_wait_repeats_bitwise():
    """w4pw (gemm_w4p.h CST 3): K-step 0 after an epilogue waits vmcnt(ND + the
    epilogue's stores), i.e. only for the next tile's K-tile-1 DMAs. If vmcnt did
    not complete in issue order, a tile would read a K-tile still in flight and
    the image would differ: 24 launches (4 tiles per CU, 3 epilogue-to-K-step-0
    changes each), every one bitwise the one-shot kernel."""
    a = (torch.rand(8192, 1024, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(8192, 1024, device=DEV) * 2 - 1).bfloat16()
    one_shot = _gemm_v(a, b, "w4h_1_24_20_1_0")
    for i in range(24):
        assert torch.equal(_gemm_v(a, b, "w4pw_0"), one_shot), i


def test_gemm_persistent_deferred_stores_repeat_bitwise_and_refuse_short_k():
    """w4pq (gemm_w4p.h DD > 0): the next tile's K-steps 0 .. DD - 1 store the
    previous tile's deferred C units and the K-step after each waits
    vmcnt(ND + SPS), counting those stores as younger than the DMA it waits for.
    If vmcnt did not complete in issue order, or a first tile's dropped stores
    (zero-size buffer) were not counted, a K-step would read a K-tile still in
    flight: 24 launches at 4 tiles per CU, every one bitwise the one-shot
    kernel. K-steps fewer than the peeled ones + 2 are refused, not run."""
    from kgs.ops import experiments as ex

    a = (torch.rand(8192, 1024, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(8192, 1024, device=DEV) * 2 - 1).bfloat16()
    one_shot = _gemm_v(a, b, "w4h_1_24_20_1_0")
    for i in range(24):
        assert torch.equal(_gemm_v(a, b, "w4pq8x2n_0" if i % 2 else "w4pq4x4n_0"), one_shot), i
    short = (torch.rand(8192, 640, device=DEV) * 2 - 1).bfloat16()  # 10 K-steps < 10 peeled + 2
    with pytest.raises(RuntimeError):
        ex.gemm_nt(short, short, "w4pq8x2n_0")


@pytest.mark.parametrize("M,N,K,variant", [(8192, 8192, 1024, 0), (8192, 8192, 1024, 1), (8192, 2304, 9216, 2),
                                           (4096, 4608, 768, 3)])
def test_gemm_persistent_wait_stamp_build(M, N, K, variant):
    """bench/gemm_waits.py's source (gemm_w4p.h WSB): the wait-stamp build computes
    the production image, and every wave reports each category's waits, a start
    before its end and its tiles (which add up to the tile grid, 4 waves each)."""
    from kgs.ops import experiments as ex
    from kgs.ops import gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    ref = gemm_nt(a, b, variant="w4_oneshot")
    out = torch.empty_like(ref)
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    st = torch.zeros((cus, 4, 16), dtype=torch.int64, device=DEV)
    grid = ex.gemm_w4p_waits(a, b, out, st, variant)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    s = st[:grid].cpu()
    assert int(s[:, :, 14].sum()) == 4 * (M // 256) * (N // 256)
    assert bool((s[:, :, 13] > s[:, :, 12]).all()) and bool((s[:, :, :12] >= 0).all())
    assert bool((s[:, :, 4:8].sum(-1) > 0).all())  # the steady loop's waits were stamped on every wave
    total = (s[:, :, 13] - s[:, :, 12]).sum()
    assert int(s[:, :, :12].sum()) < int(total)


@pytest.mark.parametrize("M,N,K", [(8192, 8192, 512), (8192, 2304, 9216), (1024, 768, 1024)])
def test_gemm_persistent_timing_build_stamps(M, N, K):
    """bench/gemm_tail.py's source: the timing build (gemm_w4p.h TS) computes
    production's bits, every workgroup stamps a start, its tiles' ends in
    order and an exit after its last tile, and the tile counts add up to the
    tile grid (the per-XCD queue hands out every tile exactly once)."""
    from kgs.ops import experiments as ex
    from kgs.ops import gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    ref = gemm_nt(a, b)
    out = torch.empty_like(ref)
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    st = torch.zeros((cus, 16), dtype=torch.int64, device=DEV)
    grid = ex.gemm_w4p_stamps(a, b, out, st, ex.production_map(M, N, K))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    s = st[:grid].cpu()
    tiles = (M // 256) * (N // 256)
    assert grid == min(tiles, cus)
    assert int(s[:, 15].sum()) == tiles and int(s[:, 15].min()) >= 1
    assert bool((s[:, 0] > 0).all()) and bool((s[:, 14] >= s[:, 0]).all()) and bool((s[:, 13] >= s[:, 14]).all())
    for row in s.tolist():
        n = min(row[15], 11)
        ends = [row[0]] + row[2:2 + n]
        assert ends == sorted(ends), row
        assert (row[1] >> 32) & 0xF < 8  # XCC id


@pytest.mark.parametrize("act", [None, "bias", "gelu", "silu"])
@pytest.mark.parametrize("M,N,K", [(4096, 4608, 512), (8192, 2560, 384), (4608, 4096, 8320), (8192, 2304, 8448)])
def test_gemm_fast_persistent_is_bitwise_the_one_shot_grid(M, N, K, act):
    """Production "fast" launches the persistent grid (K >= 384, more tiles than CUs); "w4_oneshot" the
    one-workgroup-per-tile grid of the same K-step: bitwise equal with every
    epilogue, more tiles than CUs (288 / 320 / 288 / 288), tall and wide, and
    the long-K (> 8192) tile-group-8 maps."""
    from kgs.ops import gemm_nt

    a = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device=DEV) * 2 - 1).bfloat16()
    kw = {} if act is None else {"bias": torch.randn(N, device=DEV).bfloat16(),
                                 "act": None if act == "bias" else act}
    fast = gemm_nt(a, b, variant="fast", **kw)
    assert torch.equal(fast, gemm_nt(a, b, variant="w4_oneshot", **kw))
    ref = _ref_nt(a, b, kw.get("bias"), kw.get("act"))
    torch.testing.assert_close(fast.float(), ref, rtol=2e-2, atol=2e-2)


def test_gemm_persistent_with_cus_held_by_another_kernel():
    """A side-stream kernel whose workgroups need a CU each (the RCCL all-reduce
    of the bench step, here the comm stand-in with 64 KiB of LDS) launched just
    before the persistent GEMM: the GEMM's late workgroups find their tiles
    taken by the others (per-XCD ticket queue), the result is exact, and the
    queue is reset for the next launches on both streams."""
    from kgs.ops import gemm_nt
    from kgs.ops.elementwise import comm_standin

    a = (torch.rand(4096, 2048, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(4608, 2048, device=DEV) * 2 - 1).bfloat16()
    ref = gemm_nt(a, b, variant="w4_oneshot")
    dst = torch.zeros(1 << 22, device=DEV)
    src = torch.ones(1 << 22, device=DEV)
    side = torch.cuda.Stream(device=DEV)
    main = torch.cuda.current_stream(DEV)
    outs = []
    for _ in range(3):
        side.wait_stream(main)
        with torch.cuda.stream(side):
            comm_standin(dst, src, blocks=48, passes=4, lds_kb=64)
        outs.append(gemm_nt(a, b, variant="fast"))
        with torch.cuda.stream(side):  # a persistent GEMM on the side stream too (its own ticket slot)
            outs.append(gemm_nt(a, b, variant="fast"))
        main.wait_stream(side)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)
    assert torch.equal(dst, torch.full_like(dst, 12.0))


def test_gemm_persistent_in_a_hip_graph_replays():
    """The persistent GEMM captured into a hipGraph (the serving engine captures
    its decode step, LM head included): its ticket slot is baked into the graph
    and reset by the kernel itself, so every replay computes the full product."""
    from kgs.ops import gemm_nt

    a = (torch.rand(2304, 1024, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(8192, 1024, device=DEV) * 2 - 1).bfloat16()  # 9 x 32 = 288 tiles
    ref = gemm_nt(a, b, variant="w4_oneshot")
    out = torch.empty_like(ref)
    gemm_nt(a, b, out=out)  # warm-up outside capture (allocates the ticket pool)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gemm_nt(a, b, out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)


@pytest.mark.parametrize("act", [None, "bias", "gelu"])
@pytest.mark.parametrize("M,N,K", [(4096, 4608, 1024), (4608, 4096, 768), (2048, 1024, 4096)])
def test_gemm_fp8_four_wave_persistent_equals_eight_wave(M, N, K, act):
    """The four-wave persistent fp8 kernel (gemm_w4f8.h: one 16x16x128 MFMA per
    accumulator and K-tile, the K-step split by A rows) accumulates each output
    over the same K-tiles in the same order as the 8-wave kernel: bitwise equal,
    with epilogues, more tiles than CUs (288) and fewer (32), and the device
    activation scale."""
    from kgs.ops import gemm_fp8_nt

    qa, sa, qb, sb = _fp8_pair(M, N, K, seed=5)
    kw = {} if act is None else {"bias": torch.randn(N, device=DEV).bfloat16(), "act": None if act == "bias" else act}
    ref8 = gemm_fp8_nt(qa, qb, sa, sb, variant="fast", **kw)
    c = gemm_fp8_nt(qa, qb, sa, sb, variant="w4p", **kw)
    assert torch.equal(c, ref8)
    assert torch.equal(gemm_fp8_nt(qa, qb, sa, sb, **kw), ref8)  # auto
    torch.testing.assert_close(c.float(), _fp8_ref(qa, sa, qb, sb, kw.get("bias"), kw.get("act")),
                               rtol=2e-2, atol=2e-2)
    dev_scale = torch.tensor([sa], device=DEV, dtype=torch.float32)
    assert torch.equal(gemm_fp8_nt(qa, qb, dev_scale, sb, variant="w4p", **kw),
                       gemm_fp8_nt(qa, qb, dev_scale, sb, variant="fast", **kw))


# --- ticket-queue ownership under any stream / graph use
_QM, _QN, _QK = 4608, 4096, 1024  # 18 x 16 = 288 tiles > 256 CUs: the persistent grid


def _queue_operands(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    b = (torch.rand(_QN, _QK, device=DEV, generator=g) * 2 - 1).bfloat16()
    As = [(torch.rand(_QM, _QK, device=DEV, generator=g) * 2 - 1).bfloat16() for _ in range(n)]
    return As, b


def _hip_streams(n):
    """n distinct HIP streams (torch's pool recycles 32 per priority), as
    torch ExternalStreams, plus a destroyer."""
    import ctypes

    # the HIP runtime torch already loaded (one runtime per process)
    hip = ctypes.CDLL([ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln][0])
    handles = []
    for _ in range(n):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1)) == 0  # non-blocking
        handles.append(s)

    def destroy():
        for s in handles:
            hip.hipStreamDestroy(s)

    return [torch.cuda.ExternalStream(s.value, device=DEV) for s in handles], destroy


def test_persistent_graph_replayed_on_another_stream_while_eager_gemms_run_on_the_capture_stream():
    """A graph captured on stream S replayed on S2 at the same time as eager
    persistent GEMMs on S: the graph's kernel owns a slot of its own (not S's),
    so every output is bitwise the one-shot kernel's."""
    from kgs.ops import gemm_nt
    from kgs.ops._lib import tile_queue_stats

    As, b = _queue_operands(4, seed=11)
    refs = [gemm_nt(a, b, variant="w4_oneshot") for a in As]
    S, S2 = torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV, priority=-1)
    gout = torch.empty_like(refs[0])
    with torch.cuda.stream(S):
        gemm_nt(As[0], b, out=gout)  # eager on S first: S owns a slot, the pool exists
    torch.cuda.synchronize()
    st0 = tile_queue_stats()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=S):
        gemm_nt(As[0], b, out=gout)
    st1 = tile_queue_stats()
    assert st1["capture_slots"] == st0["capture_slots"] + 1 and st1["fallbacks"] == st0["fallbacks"], (st0, st1)
    eager = [torch.empty_like(refs[0]) for _ in range(3)]
    for it in range(10):
        gout.zero_()
        for e in eager:
            e.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(S2):
            g.replay()
        with torch.cuda.stream(S):
            for i, e in enumerate(eager):
                gemm_nt(As[1 + i], b, out=e)
        torch.cuda.synchronize()
        assert torch.equal(gout, refs[0]), it
        for i, e in enumerate(eager):
            assert torch.equal(e, refs[1 + i]), (it, i)


def test_two_persistent_graphs_from_one_capture_stream_replayed_concurrently():
    """Two graphs captured on the same stream (each with its own persistent GEMM)
    replayed at the same time on two streams, and one graph replayed
    concurrently with itself: outputs bitwise the one-shot kernel's, every
    time."""
    from kgs.ops import gemm_nt

    As, b = _queue_operands(2, seed=12)
    refs = [gemm_nt(a, b, variant="w4_oneshot") for a in As]
    S = torch.cuda.Stream(device=DEV)
    outs = [torch.empty_like(refs[0]) for _ in range(2)]
    with torch.cuda.stream(S):
        gemm_nt(As[0], b, out=outs[0])
    torch.cuda.synchronize()
    graphs = []
    for i in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=S):
            for _ in range(3):  # three launches per replay: longer overlap window
                gemm_nt(As[i], b, out=outs[i])
        graphs.append(g)
    S1, S2 = torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)
    for it in range(10):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(S1):
            graphs[0].replay()
        with torch.cuda.stream(S2):
            graphs[1].replay()
        torch.cuda.synchronize()
        assert torch.equal(outs[0], refs[0]) and torch.equal(outs[1], refs[1]), it
    for it in range(5):  # one exec on two streams at once: the same product, never a skipped tile
        outs[0].zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(S1):
            graphs[0].replay()
        with torch.cuda.stream(S2):
            graphs[0].replay()
        torch.cuda.synchronize()
        assert torch.equal(outs[0], refs[0]), it
    # the self-concurrent replays shared their capture slots, so those may be
    # left with counts (tile_queue.h: the memset node in front of each captured
    # launch is what makes every replay start from zero); one solo replay
    # leaves them clean again (test_tile_queue_pool_is_clean_after_the_concurrency_tests)
    with torch.cuda.stream(S1):
        graphs[0].replay()
    torch.cuda.synchronize()
    assert torch.equal(outs[0], refs[0])
    # and an eager launch on each stream afterwards still starts from a zero queue
    for s in (S, S1, S2):
        with torch.cuda.stream(s):
            o = gemm_nt(As[1], b)
        torch.cuda.synchronize()
        assert torch.equal(o, refs[1])


def test_eighty_streams_each_launch_a_persistent_gemm():
    """80 distinct HIP streams (more than the old pool's 64 slots, which wrapped
    onto live ones), each launching one persistent GEMM at the same time: each
    stream gets a slot of its own (the pool grows) and every output is bitwise
    the one-shot kernel's."""
    from kgs.ops import gemm_nt
    from kgs.ops._lib import tile_queue_stats

    As, b = _queue_operands(8, seed=13)
    refs = [gemm_nt(a, b, variant="w4_oneshot") for a in As]
    streams, destroy = _hip_streams(80)
    try:
        st0 = tile_queue_stats()
        outs = [torch.empty_like(refs[0]) for _ in streams]
        for rnd in range(2):
            for o in outs:
                o.zero_()
            torch.cuda.synchronize()
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    gemm_nt(As[i % len(As)], b, out=outs[i])
            torch.cuda.synchronize()
            bad = [i for i, o in enumerate(outs) if not torch.equal(o, refs[i % len(As)])]
            assert not bad, (rnd, bad)
        st1 = tile_queue_stats()
        assert st1["stream_slots"] == st0["stream_slots"] + 80, (st0, st1)
        assert st1["fallbacks"] == st0["fallbacks"] and st1["slots"] >= st1["stream_slots"] + st1["capture_slots"]
    finally:
        torch.cuda.synchronize()
        destroy()


def test_first_persistent_gemm_on_a_busy_new_stream_returns_without_waiting():
    """the ticket pool used to grow with a
    hipStreamSynchronize of the CALLER's stream, so the first persistent GEMM
    on a new stream blocked the host until everything already queued there had
    run. Now a stream holding a ~50 ms kernel gets its first persistent GEMM --
    with the pool at its capture reserve, so the call itself grows the pool --
    in under 5 ms of host time, and the product is bitwise the one-shot one."""
    import time

    from kgs.ops import gemm_nt
    from kgs.ops._lib import tile_queue_stats
    from kgs.ops.elementwise import cu_hold

    As, b = _queue_operands(1, seed=14)
    ref = gemm_nt(As[0], b, variant="w4_oneshot")
    # the persistent instance launched once before the timed call: the first launch of a kernel loads
    # its code object (lazy loading), which can wait for the device -- not what this test times
    gemm_nt(As[0], b)
    torch.cuda.synchronize()
    reserve = 64  # tile_queue.h TQ_RESERVE

    def free():
        st = tile_queue_stats()
        return st["slots"] - st["stream_slots"] - st["capture_slots"]

    # new streams (each taking one slot) until the pool is down to its reserve;
    # HIP recycles destroyed stream handles, which keep their old slot, so count
    # by the pool's own statistics, not by streams made
    streams, destroys = [], []
    junk = torch.empty_like(ref)
    while free() > reserve and len(streams) < 1024:
        more, d = _hip_streams(max(1, free() - reserve))
        streams += more
        destroys.append(d)
        for s in more:
            with torch.cuda.stream(s):
                gemm_nt(As[0], b, out=junk)
        torch.cuda.synchronize()
    more, d = _hip_streams(1)
    destroys.append(d)
    streams += more
    try:
        st0 = tile_queue_stats()
        assert st0["slots"] == 0 or free() <= reserve, st0
        busy = streams[-1]
        out = torch.zeros_like(ref)
        torch.cuda.synchronize()
        with torch.cuda.stream(busy):
            cu_hold(256, 50000.0, lds_kb=0)
            t0 = time.perf_counter()
            gemm_nt(As[0], b, out=out)
            host_ms = (time.perf_counter() - t0) * 1e3
        st1 = tile_queue_stats()
        assert st1["slots"] > st0["slots"] and st1["stream_slots"] == st0["stream_slots"] + 1, (st0, st1)
        assert st1["fallbacks"] == st0["fallbacks"]
        assert host_ms < 5.0, host_ms
        busy.synchronize()
        assert torch.equal(out, ref)
    finally:
        torch.cuda.synchronize()
        for d in destroys:
            d()


def test_captured_persistent_gemm_slot_is_zero_after_every_replay():
    """Regression (round 5, profiles/r5/fault/README.md): a persistent GEMM
    captured into a hipGraph zeroes its ticket slot in front of the GEMM node.
    With a captured hipMemsetAsync (a memset node) the slot held 64 bytes of
    host-pointer-like garbage after the serving decode graph's first replay --
    garbage tickets, and with a negative one an illegal-address fault. The
    zeroing is now a kernel node: after every replay the whole pool is zero
    again and the product is bitwise the one-shot kernel's."""
    from kgs.ops import gemm_nt
    from kgs.ops._lib import tile_queue_check, tile_queue_stats

    As, b = _queue_operands(2, seed=21)
    refs = [gemm_nt(a, b, variant="w4_oneshot") for a in As]
    S = torch.cuda.Stream(device=DEV)
    outs = [torch.empty_like(refs[0]) for _ in range(2)]
    with torch.cuda.stream(S):
        gemm_nt(As[0], b, out=outs[0])
    torch.cuda.synchronize()
    st0 = tile_queue_stats()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=S):
        for i in range(2):
            gemm_nt(As[i], b, out=outs[i])
    assert tile_queue_stats()["capture_slots"] == st0["capture_slots"] + 2
    assert tile_queue_check()["dirty_slots"] == 0
    for it in range(8):
        for o in outs:
            o.zero_()
        g.replay()  # on the current stream, alone: nothing shares its slots
        tq = tile_queue_check()
        assert tq["dirty_slots"] == 0, (it, tq)
        assert torch.equal(outs[0], refs[0]) and torch.equal(outs[1], refs[1]), it


def test_tile_queue_pool_is_clean_after_the_concurrency_tests():
    """The pool's quiescent invariant (tile_queue.h tile_queue_check) after the
    graph / multi-stream / busy-stream tests above: every ticket, exit counter
    and padding word back at zero."""
    from kgs.ops._lib import tile_queue_check, tile_queue_stats

    assert tile_queue_stats()["slots"] > 0
    tq = tile_queue_check()
    assert tq == {"dirty_slots": 0, "dirty_words": 0, "first_value": 0, "first_word": -1, "error_slots": 0}, tq


def test_corrupted_ticket_slot_is_reported_not_faulted_or_silent():
    """a slot whose tickets hold garbage (as the round-5 memset node
    left one) must neither become an address nor pass silently. Tickets
    0x40000000 (no launch could issue them) are written into a stream's slot;
    the persistent GEMM on that stream ends cleanly, its workgroups stop at
    their first queued ticket, and the slot's sticky error word reports it
    (tile_queue_check error_slots). The slot is then repaired and the next
    launch is exact again."""
    import ctypes

    from kgs.ops import gemm_nt
    from kgs.ops import _lib
    from kgs.utils.graph_audit import hip_runtime

    a = (torch.rand(8192, 1024, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(8192, 1024, device=DEV) * 2 - 1).bfloat16()
    ref = gemm_nt(a, b, variant="w4_oneshot")
    s = torch.cuda.Stream()
    slot = ctypes.c_void_p()
    _lib.check(_lib.lib().kgs_tile_queue_slot(s.cuda_stream, ctypes.byref(slot)), "kgs_tile_queue_slot")
    torch.cuda.synchronize()
    hip = hip_runtime()
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipMemcpy.restype = ctypes.c_int
    words = (ctypes.c_int * 16)(*([0x40000000] * 8 + [0] * 8))
    assert hip.hipMemcpy(slot, words, 64, 1) == 0  # host to device
    assert _lib.tile_queue_check()["error_slots"] == 0
    out = torch.zeros_like(ref)
    with torch.cuda.stream(s):
        gemm_nt(a, b, out=out)
    torch.cuda.synchronize()
    tq = _lib.tile_queue_check()
    assert tq["error_slots"] == 1 and tq["dirty_slots"] == 1, tq
    # each workgroup computed its static first tile and stopped at its first queued ticket
    same = (out.view(32, 256, 32, 256) == ref.view(32, 256, 32, 256)).all(dim=3).all(dim=1)
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    assert int(same.sum()) == cus, int(same.sum())
    zero = (ctypes.c_int * 16)()
    assert hip.hipMemcpy(slot, zero, 64, 1) == 0
    assert _lib.tile_queue_check() == {"dirty_slots": 0, "dirty_words": 0, "first_value": 0, "first_word": -1,
                                       "error_slots": 0}
    with torch.cuda.stream(s):
        gemm_nt(a, b, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("grid", [0, 224, 100])
def test_persistent_first_ticket_modes_and_reserved_grids_are_exact(mode, grid):
    """The persistent kernel with the static first ticket (1, production) and
    with every ticket from the queue (2), on one workgroup per CU and on fewer
    (CUs left to a collective): bitwise the one-shot kernel, and a CU held by
    another kernel while it starts does not change that."""
    from kgs.ops import gemm_nt
    from kgs.ops.elementwise import cu_hold
    from kgs.ops.experiments import gemm_w4p_grid

    a = (torch.rand(4608, 2048, device=DEV) * 2 - 1).bfloat16()
    b = (torch.rand(4096, 2048, device=DEV) * 2 - 1).bfloat16()
    ref = gemm_nt(a, b, variant="w4_oneshot")
    side = torch.cuda.Stream(device=DEV)
    for held in (0, 48):
        out = torch.zeros_like(ref)
        if held:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                cu_hold(held, 200.0, lds_kb=64)
        gemm_w4p_grid(a, b, out, mode=mode, grid=grid)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (mode, grid, held)
