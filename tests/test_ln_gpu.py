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


def test_add_ln_direct_arena_grads():
    """bf16-shadow path: dgamma / dbeta accumulated by the fused backward
    straight into the optimizer's fp32 arena == the autograd path."""
    import copy
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.ops.linear import FastLinear
    from gaussiank_sgd_amd.ops.ln import add_layernorm
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer

    class Blk(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = FastLinear(128, 128)
            self.ln = torch.nn.LayerNorm(128)

        def forward(self, x):
            return add_layernorm(self.lin(x), x, self.ln, 0.1, True)
    comm.init()
    torch.manual_seed(3)
    net = Blk().cuda()
    torch.nn.init.uniform_(net.ln.weight, 0.5, 1.5)
    ref = copy.deepcopy(net)
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), named_parameters=net.named_parameters(),
                               compression=compressors["none"], is_sparse=False, density=1.0)
    install_bf16_shadow(net, opt)
    assert getattr(net.ln, "_gk_direct", None) is not None
    x = torch.randn(300, 128, device="cuda")
    for model in (net, ref):
        from gaussiank_sgd_amd import ops as gops
        gops.seed_generator().manual_seed(7)    # same dropout mask in both runs
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = model(x)
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        err = (p.grad - q.grad).abs().max().item()
        assert err <= 2e-2 * q.grad.abs().max().item() + 1e-4, (n, err)


@pytest.mark.parametrize("R,H", [(37, 768), (256, 64), (128, 1024), (9, 4096), (300, 136)])
def test_add_ln_f32_vs_fp64(R, H):
    """fp32 storage (no autocast, the reference's precision): the fused HIP
    row passes vs an fp64 PyTorch LayerNorm, at fp32 tolerances."""
    from gaussiank_sgd_amd.ops import ln as L_
    from gaussiank_sgd_amd.ops.ln import add_layernorm
    torch.manual_seed(R + H + 1)
    ln = torch.nn.LayerNorm(H).cuda()
    torch.nn.init.uniform_(ln.weight, 0.5, 1.5)
    torch.nn.init.uniform_(ln.bias, -0.5, 0.5)
    a = torch.randn(R, H, device="cuda").requires_grad_(True)
    x = torch.randn(R, H, device="cuda").requires_grad_(True)
    assert L_.fused_available(x)
    y = add_layernorm(a, x, ln, 0.0, True)
    assert y.dtype == torch.float32
    dy = torch.randn_like(y)
    y.backward(dy)
    ar = a.detach().double().requires_grad_(True)
    xr = x.detach().double().requires_grad_(True)
    w = ln.weight.detach().double().requires_grad_(True)
    b = ln.bias.detach().double().requires_grad_(True)
    yr = F.layer_norm(xr + ar, (H,), w, b, ln.eps)
    yr.backward(dy.double())
    tol = lambda r: 2e-5 * r.abs().max().item() + 1e-5  # noqa: E731
    assert (y.double() - yr).abs().max().item() <= tol(yr)
    assert (x.grad.double() - xr.grad).abs().max().item() <= tol(xr.grad)
    assert torch.equal(a.grad, x.grad)                    # no dropout: da == dx
    assert (ln.weight.grad.double() - w.grad).abs().max().item() <= 1e-5 * w.grad.abs().max().item() + 1e-4
    assert (ln.bias.grad.double() - b.grad).abs().max().item() <= 1e-5 * b.grad.abs().max().item() + 1e-4


def test_add_ln_f32_dropout_matches_bf16_mask():
    """fp32 and bf16 storage regenerate the same hash mask for one seed."""
    from gaussiank_sgd_amd.ops.ln import _AddLNFn
    torch.manual_seed(3)
    R, H, p = 64, 768, 0.1
    ln = torch.nn.LayerNorm(H).cuda()
    a = torch.randn(R, H, device="cuda")
    x = torch.randn(R, H, device="cuda")
    dyr = torch.randn(R, H, device="cuda")
    masks = []
    for cd in (torch.float32, torch.bfloat16):
        aa = a.clone().requires_grad_(True)
        y = _AddLNFn.apply(aa, x, ln.weight, ln.bias, ln.eps, p, 1234, None, None, cd)
        (y.float() * dyr).sum().backward()
        masks.append(aa.grad == 0)
    assert torch.equal(masks[0], masks[1])
    assert abs(masks[0].float().mean().item() - p) < 0.02
