"""Fused softmax cross-entropy (ops/xent.py, csrc/kernels/xent.hip) vs
F.cross_entropy on the fp32 copy of the same bf16 logits."""
import pytest
import torch
import torch.nn.functional as F

from gaussiank_sgd_amd.ops import xent

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,V,ignored", [(64, 30522, 0), (300, 1024, 7), (5, 2, 1)])
def test_fused_xent_matches_torch(cuda, R, V, ignored):
    torch.manual_seed(0)
    logits = (3 * torch.randn(R, V, device=cuda)).to(torch.bfloat16)
    labels = torch.randint(0, V, (R,), device=cuda)
    if ignored:
        labels[torch.randperm(R, device=cuda)[:ignored]] = -100
    assert xent.fused_available(logits)
    a = logits.clone().requires_grad_(True)
    loss = xent.cross_entropy(a, labels)
    loss.backward(torch.tensor(2.0, device=cuda))
    b = logits.float().clone().requires_grad_(True)
    ref = F.cross_entropy(b, labels, ignore_index=-100)
    ref.backward(torch.tensor(2.0, device=cuda))
    torch.testing.assert_close(loss.float(), ref, rtol=2e-5, atol=2e-5)
    assert a.grad.dtype == torch.bfloat16
    torch.testing.assert_close(a.grad.float(), b.grad, rtol=1e-2, atol=1e-6)   # bf16-rounded gradient
    if ignored:
        assert a.grad[labels == -100].abs().sum() == 0
