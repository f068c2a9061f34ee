"""Fused residual add + dropout + LayerNorm (ops/ln.py, csrc/kernels/ln.hip)
vs an fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error


@pytest.mark.parametrize("R,H", [(37, 768), (256, 64), (128, 1024), (9, 4096), (300, 136)])
def test_add_ln_no_dropout(R, H):
    from gaussiank_sgd_amd.ops.ln import add_layernorm
    torch.manual_seed(R + H)
    ln = torch.nn.LayerNorm(H).cuda()
    torch.nn.init.uniform_(ln.weight, 0.5, 1.5)
    torch.nn.init.uniform_(ln.bias, -0.5, 0.5)
    a = torch.randn(R, H, device="cuda").to(torch.bfloat16).requires_grad_(True)
    x = torch.randn(R, H, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = add_layernorm(a, x, ln, 0.0, True)
    dy = torch.randn_like(y)
    y.backward(dy)
    ar = a.detach().float().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    w = ln.weight.detach().clone().requires_grad_(True)
    b = ln.bias.detach().clone().requires_grad_(True)
    yr = F.layer_norm(xr + ar, (H,), w, b, ln.eps)
    yr.backward(dy.float())
    assert (y.float() - yr).abs().max().item() < 3e-2
    assert (x.grad.float() - xr.grad).abs().max().item() < 3e-2 * xr.grad.abs().max().item() + 1e-2
    assert (a.grad.float() - ar.grad).abs().max().item() < 3e-2 * ar.grad.abs().max().item() + 1e-2
    assert (ln.weight.grad - w.grad).abs().max().item() < 1e-2 * w.grad.abs().max().item() + 1e-2
    assert (ln.bias.grad - b.grad).abs().max().item() < 1e-2 * b.grad.abs().max().item() + 1e-2


def test_add_ln_dropout_statistics_and_consistency():
    """Dropout keeps ~(1-p), scales kept by 1/(1-p); the backward regenerates
    the same mask (a-gradient is zero exactly where a was dropped)."""
    from gaussiank_sgd_amd.ops.ln import add_layernorm
    torch.manual_seed(1)
    R, H, p = 512, 768, 0.1
    ln = torch.nn.LayerNorm(H, elementwise_affine=True).cuda()
    a = torch.randn(R, H, device="cuda").to(torch.bfloat16).requires_grad_(True)
    x = torch.zeros(R, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = add_layernorm(a, x, ln, p, True)
    y.backward(torch.randn_like(y))
    dropped = a.grad == 0
    frac = dropped.float().mean().item()
    assert abs(frac - p) < 0.01, frac
    # x-gradient is never masked; a-gradient = x-gradient / (1-p) where kept
    kept = ~dropped
    ratio = (a.grad.float()[kept] / x.grad.float()[kept]).median().item()
    assert abs(ratio - 1 / (1 - p)) < 0.02
