"""CPU checks of the Llama stand-in's PyTorch path (the numerics reference the
GPU kernels are tested against) -- config, parameter count, RoPE convention."""
import pytest

torch = pytest.importorskip("torch")


def test_llama3_8b_config_param_count():
    from kgs.models.llama import LlamaConfig

    cfg = LlamaConfig.llama3_8b()
    assert cfg.head_dim == 128 and cfg.kv_heads == 8
    assert abs(cfg.params() / 1e9 - 8.03) < 0.01  # Llama-3-8B: 8.03 B parameters


def test_torch_rope_matches_kernel_reference():
    from kgs.models.llama import _rope_torch
    from kgs.ops.transformer import ref_rope_qkv, rope_tables

    b, s, nh, nkv, hd = 2, 16, 2, 1, 128
    qkv = torch.randn(b * s, (nh + 2 * nkv) * hd).to(torch.bfloat16)
    cos, sin = rope_tables(s, hd, 500000.0, "cpu")
    ref = ref_rope_qkv(qkv, cos, sin, nh + nkv, hd, s)
    q = qkv[:, :nh * hd].reshape(b, s, nh, hd).transpose(1, 2)
    k = qkv[:, nh * hd:(nh + nkv) * hd].reshape(b, s, nkv, hd).transpose(1, 2)
    q2, k2 = _rope_torch(q, k, cos, sin)
    assert torch.equal(q2.transpose(1, 2).reshape(b * s, nh * hd), ref[:, :nh * hd])
    assert torch.equal(k2.transpose(1, 2).reshape(b * s, nkv * hd), ref[:, nh * hd:(nh + nkv) * hd])


def test_torch_backend_forward_cpu():
    from kgs.models.llama import LlamaConfig, LlamaModel

    cfg = LlamaConfig(hidden=256, intermediate=512, heads=2, kv_heads=1, layers=2, vocab=300)
    m = LlamaModel(cfg, device="cpu", backend="torch")
    tokens = torch.randint(0, cfg.vocab, (2, 8))
    out = m.forward(tokens)
    assert out.shape == (2, 8, cfg.vocab) and torch.isfinite(out.float()).all()
    # causal: the first 4 positions do not depend on later tokens
    t2 = tokens.clone()
    t2[:, 4:] = (t2[:, 4:] + 1) % cfg.vocab
    out2 = m.forward(t2)
    assert torch.allclose(out[:, :4].float(), out2[:, :4].float())
