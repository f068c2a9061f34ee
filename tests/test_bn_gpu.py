"""Fused BN + residual + ReLU kernels vs nn.BatchNorm2d + add + relu (fp32 reference)."""
import pytest
import torch
import torch.nn.functional as F

from gaussiank_sgd_amd.ops.bn import BNAct

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 256, 7, 7), (2, 2048, 3, 3), (3, 96, 5, 5)])
@pytest.mark.parametrize("relu,res", [(True, True), (True, False), (False, False)])
def test_bnact_matches_torch(cuda, dtype, shape, relu, res):
    torch.manual_seed(0)
    N, C, H, W = shape
    bn = BNAct(C, act="relu" if relu else None).to(cuda)
    ref = torch.nn.BatchNorm2d(C).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    x0 = (torch.randn(shape, device=cuda) * 2 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    r0 = torch.randn(shape, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last) if res else None
    g0 = torch.randn(shape, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    x = x0.clone().requires_grad_(True)
    r = r0.clone().requires_grad_(True) if res else None
    y = bn(x, r)
    y.backward(g0)
    xr = x0.float().clone().requires_grad_(True)
    rr = r0.float().clone().requires_grad_(True) if res else None
    yr = ref(xr)
    if res:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    yr.backward(g0.float())
    tol = dict(atol=2e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-4, rtol=1e-4)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    assert torch.allclose(y.float(), yr, **tol)
    assert torch.allclose(x.grad.float(), xr.grad, **(dict(atol=5e-2, rtol=5e-2) if dtype == torch.bfloat16 else tol))
    if res:
        assert torch.allclose(r.grad.float(), rr.grad, **tol)
    assert torch.allclose(bn.weight.grad, ref.weight.grad, rtol=2e-2 if dtype == torch.bfloat16 else 1e-4,
                          atol=2e-1 if dtype == torch.bfloat16 else 1e-3)
    assert torch.allclose(bn.bias.grad, ref.bias.grad, rtol=2e-2 if dtype == torch.bfloat16 else 1e-4,
                          atol=2e-1 if dtype == torch.bfloat16 else 1e-3)
    assert torch.allclose(bn.running_mean, ref.running_mean, atol=1e-3, rtol=1e-3)
    assert torch.allclose(bn.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    assert int(bn.num_batches_tracked) == 1


def test_resnet50_fused_vs_unfused(cuda):
    """Whole-network gradients: fused (fp32) error vs an fp64 reference must be
    no worse than MIOpen's (fp32) error -- deep BN stacks amplify rounding, so
    the comparison is relative to the vendor path, not absolute."""
    from gaussiank_sgd_amd.models import resnet50
    from gaussiank_sgd_amd.ops.bn import BNAct
    torch.manual_seed(0)
    m1 = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    m2 = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    m3 = resnet50(num_classes=10).to(cuda).double().to(memory_format=torch.channels_last)
    m2.load_state_dict(m1.state_dict())
    m3.load_state_dict(m1.state_dict())
    for m in list(m2.modules()) + list(m3.modules()):
        if isinstance(m, BNAct):
            m.fused = False
    x = torch.randn(8, 3, 96, 96, device=cuda).contiguous(memory_format=torch.channels_last)
    ys = [m1(x), m2(x), m3(x.double())]
    for y in ys:
        y.sum().backward()
    assert torch.allclose(ys[0].double(), ys[2], atol=1e-3, rtol=1e-3)
    for (n, p1), (_, p2), (_, p3) in zip(m1.named_parameters(), m2.named_parameters(), m3.named_parameters()):
        ref = p3.grad
        e_fused = float((p1.grad.double() - ref).norm() / (ref.norm() + 1e-30))
        e_vendor = float((p2.grad.double() - ref).norm() / (ref.norm() + 1e-30))
        assert e_fused <= 3 * e_vendor + 1e-4, (n, e_fused, e_vendor)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,pool", [((2, 64, 32, 32), (3, 2, 1)), ((3, 16, 17, 13), (3, 2, 1)),
                                        ((2, 32, 16, 16), (2, 2, 0)), ((2, 8, 9, 11), (3, 1, 1))])
def test_bn_relu_maxpool_matches_torch(cuda, dtype, shape, pool):
    """Fused BN + ReLU + max-pool (argmax bytes, gathered backward) vs
    BatchNorm2d + relu + max_pool2d in fp32."""
    torch.manual_seed(0)
    N, C, H, W = shape
    bn = BNAct(C, act="relu", pool=pool).to(cuda)
    ref = torch.nn.BatchNorm2d(C).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    x0 = (torch.randn(shape, device=cuda) * 2 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    x = x0.clone().requires_grad_(True)
    y = bn(x)
    g0 = torch.randn(y.shape, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    y.backward(g0)
    xr = x0.float().clone().requires_grad_(True)
    yr = F.max_pool2d(F.relu(ref(xr)), *pool)
    yr.backward(g0.float())
    assert y.shape == yr.shape and y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    if dtype == torch.float32:
        assert torch.allclose(y, yr, atol=1e-4, rtol=1e-4)
        assert torch.allclose(x.grad, xr.grad, atol=1e-4, rtol=1e-4)
        assert torch.allclose(bn.weight.grad, ref.weight.grad, atol=1e-3, rtol=1e-4)
        assert torch.allclose(bn.bias.grad, ref.bias.grad, atol=1e-3, rtol=1e-4)
    else:
        assert torch.allclose(y.float(), yr, atol=3e-2, rtol=2e-2)
        err = float((x.grad.float() - xr.grad).norm() / xr.grad.norm())
        assert err < 3e-2, err
        for a, b in ((bn.weight.grad, ref.weight.grad), (bn.bias.grad, ref.bias.grad)):
            assert float((a - b).norm() / b.norm()) < 3e-2
    assert torch.allclose(bn.running_mean, ref.running_mean, atol=1e-3, rtol=1e-3)
    assert torch.allclose(bn.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    assert int(bn.num_batches_tracked) == 1


@pytest.mark.parametrize("pool", [None, (3, 2, 1)])
def test_bnact_twin_sums_both_gradients(cuda, pool):
    """twin=True: two handles on one output; the fused backward sums dy + dy2."""
    torch.manual_seed(0)
    N, C, H, W = 2, 32, 12, 12
    bn = BNAct(C, act="relu", pool=pool, twin=True).to(cuda)
    ref = BNAct(C, act="relu", pool=pool, twin=True, fused=False).to(cuda)
    x0 = torch.randn(N, C, H, W, device=cuda).contiguous(memory_format=torch.channels_last)
    outs = []
    for m in (bn, ref):
        x = x0.clone().requires_grad_(True)
        a, b = m(x)
        g1 = torch.linspace(-1, 1, a.numel(), device=cuda).view_as(a)
        ((a * g1).sum() + (b * b).sum()).backward()
        outs.append((a.detach(), x.grad, m.weight.grad, m.bias.grad))
    for u, v in zip(*outs):
        assert torch.allclose(u, v, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_in_launch_finalize_matches_separate_launch(cuda, dtype, monkeypatch):
    """The finalize folded into the apply pass (bn_act.hip FinSync: ticketed
    leader workgroups + per-layer flags) gives bit-identical outputs,
    gradients and running statistics to the separate finalize launch, over
    many back-to-back launches of several layers and shapes (the ticket
    counter reset and the per-launch epoch are exercised every iteration)."""
    import gaussiank_sgd_amd.ops.bn as bnmod
    torch.manual_seed(0)
    shapes = [(8, 64, 14, 14), (4, 2048, 3, 3), (3, 96, 5, 5), (16, 256, 7, 7)]
    mods = {}
    for fused in (True, False):
        torch.manual_seed(1)
        mods[fused] = [BNAct(s[1], act="relu").to(cuda) for s in shapes]
    for it in range(12):
        si = it % len(shapes)
        shape = shapes[si]
        x0 = (torch.randn(shape, device=cuda) * 2 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
        r0 = torch.randn(shape, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
        g0 = torch.randn(shape, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
        outs = {}
        for fused in (True, False):
            monkeypatch.setattr(bnmod, "_FIN_FUSE", fused)
            m = mods[fused][si]
            x = x0.clone().requires_grad_(True)
            r = r0.clone().requires_grad_(True)
            y = m(x, r if it % 2 else None)
            y.backward(g0)
            outs[fused] = (y.detach(), x.grad, m.weight.grad.clone(), m.bias.grad.clone(), m.running_mean.clone(),
                           m.running_var.clone())
            m.weight.grad = None
            m.bias.grad = None
        assert getattr(mods[True][si], "_gk_fin", None) is not None
        for a, b in zip(outs[True], outs[False]):
            assert torch.equal(a, b), it
