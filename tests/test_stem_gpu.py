"""ResNet stem convolution (7x7 / s2 / p3, 3 -> 64) on the gfx950 kernels of
csrc/kernels/stem.hip vs an fp32 PyTorch reference: forward (+ the BatchNorm
statistics of its epilogue), grad-weight, and the StemConv module under bf16
autocast (weight gradient into a fresh tensor and through the shadow arena)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error


def _inputs(N, H, W, dtype, seed):
    torch.manual_seed(seed)
    x = torch.randn(N, 3, H, W, device="cuda").to(dtype).contiguous(memory_format=CL)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    return x, w


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,H,W", [(2, 224, 224), (3, 64, 64), (5, 32, 48), (1, 96, 80)])
def test_stem_forward_and_stats(dtype, N, H, W):
    g = torch.ops.gksgd
    x, w = _inputs(N, H, W, dtype, N + H)
    assert g.stem_supported(H, W)
    wp = torch.empty(64, 224, dtype=torch.bfloat16, device="cuda")
    g.stem_pack(w, wp)
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty(N, 64, OH, OW, dtype=torch.bfloat16, device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 256, 64), float("nan"), device="cuda")
    rows = g.stem_fwd(x, wp, y, st)
    torch.cuda.synchronize()
    ref = F.conv2d(x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float(), stride=2, padding=3)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    yf = y.float()
    s1 = st[0, :rows].double().sum(0)
    s2 = st[1, :rows].double().sum(0)
    r1 = yf.double().sum((0, 2, 3))
    r2 = yf.double().square().sum((0, 2, 3))
    assert torch.allclose(s1, r1, rtol=1e-4, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s2, r2, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,H,W,cl_out", [(2, 224, 224, True), (3, 64, 64, False), (4, 32, 48, True)])
def test_stem_wgrad(dtype, N, H, W, cl_out):
    g = torch.ops.gksgd
    x, _ = _inputs(N, H, W, dtype, 7 * N + W)
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dy = torch.randn(N, 64, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    out = torch.full((64, 3, 7, 7), 0.5, device="cuda")
    if cl_out:
        out = out.contiguous(memory_format=CL)
    part = torch.empty(int(g.stem_wgrad_ws(N, H, W)), device="cuda")
    g.stem_wgrad(x, dy, out, part)
    torch.cuda.synchronize()
    xr = x.to(torch.bfloat16).float()
    wr = torch.zeros(64, 3, 7, 7, device="cuda", requires_grad=True)
    F.conv2d(xr, wr, stride=2, padding=3).backward(dy.float())
    ref = wr.grad + 0.5
    err = (out - ref).abs().max().item()
    assert err <= 2e-3 * wr.grad.abs().max().item() + 1e-3, err


def test_stemconv_module_autocast():
    from gaussiank_sgd_amd.ops.stem import StemConv
    torch.manual_seed(3)
    m = StemConv().cuda().to(memory_format=CL)
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=CL)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, st = m.forward_stats(x)
    assert st is not None and y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.to(torch.bfloat16).float()
    wr = m.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=2, padding=3)
    yr.backward(dy.float())
    assert (y.float() - yr).abs().max().item() <= 1e-2 * yr.abs().max().item()
    assert (m.weight.grad - wr.grad).abs().max().item() <= 2e-3 * wr.grad.abs().max().item() + 1e-3


def test_resnet50_stem_bn_stats_match_pass():
    """Stem + fused BN/ReLU/max-pool with the epilogue statistics == with its own
    statistics pass (GKSGD_STEM=0 falls back to MIOpen + the BN stats pass)."""
    from gaussiank_sgd_amd.ops import stem
    from gaussiank_sgd_amd.ops.bn import BNAct
    torch.manual_seed(5)
    conv = stem.StemConv().cuda().to(memory_format=CL)
    bn_a = BNAct(64, act="relu", pool=(3, 2, 1)).cuda()
    bn_b = BNAct(64, act="relu", pool=(3, 2, 1)).cuda()
    x = torch.randn(4, 3, 96, 96, device="cuda").contiguous(memory_format=CL)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, st = conv.forward_stats(x)
        assert st is not None
        out_a = bn_a(y, stats=st)
        out_b = bn_b(y)
    assert (out_a.float() - out_b.float()).abs().max().item() <= 2e-2
    assert torch.allclose(bn_a.running_mean, bn_b.running_mean, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn_a.running_var, bn_b.running_var, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("N", [1, 3])
def test_stem_f32_fwd_stats_wgrad(N):
    """fp32 stem kernels (stem_f32.hip) vs fp64 torch: output, BatchNorm
    statistics partials, grad-weight accumulated into a strided target."""
    import torch.nn.functional as F
    from gaussiank_sgd_amd import ops
    assert ops.load()
    g = torch.ops.gksgd
    torch.manual_seed(N)
    CL = torch.channels_last
    x = torch.randn(N, 3, 224, 224, device="cuda").contiguous(memory_format=CL)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    y = torch.full((N, 64, 112, 112), float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 512, 64), float("nan"), device="cuda")
    rows = g.stem_f32_fwd(x, w, y, st)
    ref = F.conv2d(x.double(), w.double(), stride=2, padding=3)
    bound = F.conv2d(x.double().abs(), w.double().abs(), stride=2, padding=3)
    assert (y.double() - ref).abs().max().item() <= 2e-6 * bound.max().item() + 1e-6
    s = st[:, :rows].double().sum(1)
    yd = ref.permute(0, 2, 3, 1).reshape(-1, 64)
    assert torch.allclose(s[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)
    dy = torch.randn(N, 64, 112, 112, device="cuda").contiguous(memory_format=CL)
    out0 = torch.randn(64, 3, 7, 7, device="cuda").contiguous(memory_format=CL)
    out = out0.clone()
    part = torch.empty(int(g.stem_f32_wgrad_ws(N)), device="cuda")
    g.stem_f32_wgrad(x, dy, out, part)
    gw = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [2, 2], [3, 3], [1, 1], False,
                                             [0, 0], 1, [False, True, False])[1]
    gb = torch.ops.aten.convolution_backward(dy.double().abs(), x.double().abs(), w.double(), None, [2, 2], [3, 3],
                                             [1, 1], False, [0, 0], 1, [False, True, False])[1]
    assert (out.double() - out0.double() - gw).abs().max().item() <= 2e-6 * gb.max().item() + 1e-5


def test_stem_conv_f32_autograd():
    """StemConv at fp32 (no autocast) runs stem_f32 and matches fp64 torch."""
    import torch.nn.functional as F
    from gaussiank_sgd_amd.ops.stem import StemConv
    torch.manual_seed(3)
    CL = torch.channels_last
    conv = StemConv().cuda()
    x = torch.randn(2, 3, 224, 224, device="cuda").contiguous(memory_format=CL)
    assert conv._fast_f32(x)
    y = conv(x)
    assert y.dtype == torch.float32
    dy = torch.randn_like(y)
    y.backward(dy)
    wd = conv.weight.detach().double().requires_grad_(True)
    yd = F.conv2d(x.double(), wd, stride=2, padding=3)
    yd.backward(dy.double())
    assert (y.double() - yd).abs().max().item() <= 1e-5 * yd.abs().max().item() + 1e-5
    assert (conv.weight.grad.double() - wd.grad).abs().max().item() <= 1e-5 * wd.grad.abs().max().item() + 1e-5


def test_resnet50_stem_f32_bn_stats_match_pass():
    """fp32 stem + fused BN/ReLU/max-pool fed by the stem's epilogue statistics
    == the same BN running its own statistics pass."""
    from gaussiank_sgd_amd.ops import stem
    from gaussiank_sgd_amd.ops.bn import BNAct
    torch.manual_seed(6)
    conv = stem.StemConv().cuda().to(memory_format=CL)
    bn_a = BNAct(64, act="relu", pool=(3, 2, 1)).cuda()
    bn_b = BNAct(64, act="relu", pool=(3, 2, 1)).cuda()
    x = torch.randn(2, 3, 224, 224, device="cuda").contiguous(memory_format=CL)
    y, st = conv.forward_stats(x)
    assert st is not None and y.dtype == torch.float32
    out_a = bn_a(y, stats=st)
    out_b = bn_b(y)
    assert (out_a - out_b).abs().max().item() <= 1e-4
    assert torch.allclose(bn_a.running_mean, bn_b.running_mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(bn_a.running_var, bn_b.running_var, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("N", [1, 4])
def test_stem_f32x6_fwd_vs_fp64_and_f32_kernel(N):
    """bf16x6 stem forward (stem_f32.hip stem_f32x6_fwd_kernel: hi/mid/lo bf16
    splits of band and weights, six MFMA products) vs fp64 torch: no less
    accurate than the fp32-MFMA kernel (1.1x its max error), same BatchNorm
    statistics partials."""
    g = torch.ops.gksgd
    torch.manual_seed(11 + N)
    x = torch.randn(N, 3, 224, 224, device="cuda").contiguous(memory_format=CL)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    ref = F.conv2d(x.double(), w.double(), stride=2, padding=3)
    bound = F.conv2d(x.double().abs(), w.double().abs(), stride=2, padding=3).max().item()
    y32 = torch.full((N, 64, 112, 112), float("nan"), device="cuda").contiguous(memory_format=CL)
    st32 = torch.full((2, 512, 64), float("nan"), device="cuda")
    r32 = g.stem_f32_fwd(x, w, y32, st32)
    y6 = torch.full_like(y32, float("nan"))
    st6 = torch.full_like(st32, float("nan"))
    wp3 = torch.empty(int(g.stem_f32x6_wplanes()), dtype=torch.bfloat16, device="cuda")
    r6 = g.stem_f32x6_fwd(x, w, y6, st6, wp3)
    torch.cuda.synchronize()
    assert r6 == r32
    e32 = (y32.double() - ref).abs().max().item()
    e6 = (y6.double() - ref).abs().max().item()
    assert e6 <= 1.1 * e32 + 1e-7 * bound, (e6, e32)
    assert e6 <= 2e-6 * bound + 1e-6
    s = st6[:, :r6].double().sum(1)
    yd = ref.permute(0, 2, 3, 1).reshape(-1, 64)
    assert torch.allclose(s[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N", [1, 3])
def test_stem_f32x6_wgrad_vs_fp64_and_f32_kernel(N):
    """bf16x6 stem grad-weight (stem_f32x6_wgrad_kernel: dY and band values
    split into three bf16 parts, six MFMA products over 32 pixels at a time,
    the half step of the 112-pixel rows zero-padded) vs fp64 torch: no less
    accurate than the fp32-MFMA kernel (1.1x its max error), accumulated into
    a strided target."""
    g = torch.ops.gksgd
    torch.manual_seed(21 + N)
    x = torch.randn(N, 3, 224, 224, device="cuda").contiguous(memory_format=CL)
    dy = torch.randn(N, 64, 112, 112, device="cuda").contiguous(memory_format=CL)
    w = torch.randn(64, 3, 7, 7, device="cuda")
    gw = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [2, 2], [3, 3], [1, 1], False,
                                             [0, 0], 1, [False, True, False])[1]
    gb = torch.ops.aten.convolution_backward(dy.double().abs(), x.double().abs(), w.double(), None, [2, 2], [3, 3],
                                             [1, 1], False, [0, 0], 1, [False, True, False])[1]
    part = torch.empty(int(g.stem_f32_wgrad_ws(N)), device="cuda")
    errs = {}
    for x6 in (False, True):
        out0 = torch.randn(64, 3, 7, 7, device="cuda").contiguous(memory_format=CL)
        out = out0.clone()
        g.stem_f32_wgrad(x, dy, out, part, x6)
        torch.cuda.synchronize()
        errs[x6] = (out.double() - out0.double() - gw).abs().max().item()
    assert errs[True] <= 1.1 * errs[False] + 1e-7 * gb.max().item(), errs
    assert errs[True] <= 2e-6 * gb.max().item() + 1e-5, errs


def test_stem_conv_f32_module_bf16x6_mode():
    """StemConv at fp32 under set_f32_matmul('bf16x6') (bench.py's mode) runs
    the x6 forward and matches fp64; 'native' runs the fp32-MFMA forward."""
    from gaussiank_sgd_amd.ops import conv1x1
    from gaussiank_sgd_amd.ops.stem import StemConv
    torch.manual_seed(4)
    conv = StemConv().cuda()
    x = torch.randn(2, 3, 224, 224, device="cuda").contiguous(memory_format=CL)
    wd = conv.weight.detach().double().requires_grad_(True)
    yd = F.conv2d(x.double(), wd, stride=2, padding=3)
    dy = torch.randn_like(yd)
    yd.backward(dy)
    outs, grads = {}, {}
    for mode in ("bf16x6", "native"):
        prev = conv1x1.set_f32_matmul(mode)
        try:
            conv.weight.grad = None
            y = conv(x)
            y.backward(dy.float())
            outs[mode], grads[mode] = y.detach(), conv.weight.grad.clone()
        finally:
            conv1x1.set_f32_matmul(prev)
    for mode, y in outs.items():
        assert (y.double() - yd).abs().max().item() <= 1e-5 * yd.abs().max().item() + 1e-5, mode
        gr = grads[mode].double()
        assert (gr - wd.grad).abs().max().item() <= 1e-5 * wd.grad.abs().max().item() + 1e-5, mode
    assert not torch.equal(outs["bf16x6"], outs["native"])   # two different kernels ran
    assert not torch.equal(grads["bf16x6"], grads["native"])
