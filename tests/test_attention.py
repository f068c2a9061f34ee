"""CPU side of ops/attention.py: the fp32 reference composition equals SDPA,
the hash dropout mask has the requested keep rate and is a pure function of
(seed, index), and self_attention falls back to SDPA off the GPU."""
import torch
import torch.nn.functional as F

from gaussiank_sgd_amd.ops import attention


def _sdpa_ref(qkv, heads):
    B, T, H3 = qkv.shape
    x = qkv.view(B, T, 3, heads, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, T, heads * 64)


def test_reference_matches_sdpa():
    torch.manual_seed(0)
    qkv = torch.randn(2, 32, 3 * 2 * 64)
    assert torch.allclose(attention.reference_attention(qkv, 2), _sdpa_ref(qkv, 2), atol=1e-5)
    assert torch.allclose(attention.self_attention(qkv, 2, 0.0), _sdpa_ref(qkv, 2), atol=1e-5)


def test_dropout_mask_rate_and_determinism():
    m1 = attention.dropout_mask(2, 2, 64, 0.1, 17, "cpu")
    m2 = attention.dropout_mask(2, 2, 64, 0.1, 17, "cpu")
    m3 = attention.dropout_mask(2, 2, 64, 0.1, 18, "cpu")
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    assert abs(m1.float().mean().item() - 0.9) < 0.01
    assert attention.drop_threshold(0.1) == 6554
    assert abs(attention.drop_scale(0.1) - 1 / (1 - 6554 / 65536)) < 1e-9


def test_reference_dropout_expectation():
    # E[dropout(P)] = P: averaged over seeds the output approaches the p = 0 one
    torch.manual_seed(1)
    qkv = torch.randn(1, 16, 3 * 64)
    base = attention.reference_attention(qkv, 1)
    acc = sum(attention.reference_attention(qkv, 1, 0.3, s) for s in range(200)) / 200
    assert (acc - base).abs().max().item() < 0.15


def test_self_attention_cpu_backward():
    torch.manual_seed(2)
    qkv = torch.randn(1, 16, 3 * 2 * 64, requires_grad=True)
    attention.self_attention(qkv, 2, 0.0).sum().backward()
    assert qkv.grad is not None and torch.isfinite(qkv.grad).all()
