"""kgs.ops.gemm.pack_w4x_weight: the PACKB layout, checked on the CPU against
the index formula the four-wave kernel reads with (native/kernels/gemm_w4.h,
PACKB: panel tn, K-tile kt, row r, column c at ((tn * K/64 + kt) * bn + r) * 64 + c;
SwiGLU panels stage 32-row groups alternating gate / up)."""
import pytest
import torch

from kgs.ops.gemm import pack_w4x_weight


def _flat(p):
    return p.data.reshape(-1)


@pytest.mark.parametrize("N,K,bn", [(256, 128, 128), (512, 192, 256), (384, 64, 128)])
def test_pack_plain_layout(N, K, bn):
    w = torch.randn(N, K).bfloat16()
    p = pack_w4x_weight(w, bn)
    f = _flat(p)
    kt_n = K // 64
    for n in (0, 1, 31, 32, bn - 1, bn, N - 1):
        for k in sorted({0, 1, 63, min(64, K - 1), K - 1}):
            tn, r, kt, c = n // bn, n % bn, k // 64, k % 64
            assert f[((tn * kt_n + kt) * bn + r) * 64 + c] == w[n, k]


@pytest.mark.parametrize("I,K,bn", [(256, 128, 128), (512, 64, 256), (192, 128, 128)])
def test_pack_swiglu_layout(I, K, bn):
    w = torch.randn(2 * I, K).bfloat16()
    p = pack_w4x_weight(w, bn, swiglu=True)
    f = _flat(p)
    h, kt_n = bn // 2, K // 64
    for tn in range(2 * I // bn):
        for j in range(bn // 32):
            for r in (0, 17, 31):
                src = (I if j & 1 else 0) + tn * h + (j >> 1) * 32 + r
                for k in (0, 5, K - 1):
                    kt, c = k // 64, k % 64
                    assert f[((tn * kt_n + kt) * bn + 32 * j + r) * 64 + c] == w[src, k]


def test_pack_rejects_bad_shapes():
    with pytest.raises(ValueError):
        pack_w4x_weight(torch.zeros(200, 128).bfloat16(), 128)
    with pytest.raises(ValueError):
        pack_w4x_weight(torch.zeros(256, 100).bfloat16(), 128)
    with pytest.raises(ValueError):
        pack_w4x_weight(torch.zeros(256, 128), 128)
