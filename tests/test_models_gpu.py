"""The DP MLP (kgs.models.mlp) on the GPU: HIP Linear forward/backward vs
torch.nn.Linear (hipBLASLt) from the same init and data."""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def test_mlp_training_kgs_tracks_torch():
    from kgs.models.mlp import train_dp

    dims = [512, 2048, 2048, 512]
    kw = dict(steps=12, global_batch=2048, lr=0.2, device="cuda", dtype=torch.bfloat16)
    k = train_dp(dims, backend="kgs", **kw)
    t = train_dp(dims, backend="torch", **kw)
    assert k["losses"][-1] < 0.97 * k["losses"][0]
    assert t["losses"][-1] < 0.97 * t["losses"][0]
    # same init, same data, bf16 both ways: the curves agree to bf16 noise
    for a, b in zip(k["losses"], t["losses"]):
        assert abs(a - b) <= 0.05 * max(abs(b), 1e-3)
    assert k["tflops_per_rank"] > 0


def test_llama_block_kgs_matches_torch_and_fp8_close():
    """Llama-3-architecture prefill (tiny config): kgs GEMMs vs torch.matmul on
    the same random weights, and the W8A8 fp8 path within fp8 tolerance."""
    from kgs.models.llama import LlamaConfig, LlamaModel

    cfg = LlamaConfig(hidden=1024, intermediate=2048, heads=8, kv_heads=2, layers=2, vocab=1024)
    tokens = torch.randint(0, cfg.vocab, (2, 128), device="cuda")
    ref = LlamaModel(cfg, backend="torch").forward(tokens).float()
    got = LlamaModel(cfg, backend="kgs").forward(tokens).float()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 2e-2, rel
    f8 = LlamaModel(cfg, backend="fp8").forward(tokens).float()
    rel8 = ((f8 - ref).norm() / ref.norm()).item()
    assert rel8 < 0.15, rel8
