"""Winograd F(2x2, 3x3) fp32 convolution (ops/csrc/kernels/winograd.hip) vs an
fp64 PyTorch reference at fp32 tolerances: forward, grad-input (flipped
filter transform), odd spatial sizes (partial tiles), persistent blocks
walking many tile blocks, the BatchNorm-statistics and BN-backward
epilogues, and the FastConv2d fp32 path choosing it."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module")
def g():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error
    return torch.ops.gksgd


def _case(N, C, H, K, seed):
    torch.manual_seed(seed)
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(K, C, 3, 3, device="cuda") * (9 * C) ** -0.5).contiguous(memory_format=CL)
    return x, w


def _tol(bound):
    # Winograd: the same products summed in a different order plus +-1 / 0.5
    # transform roundings; a few times the direct kernel's 2e-6 relative bound
    return 1e-5 * bound.max().item() + 1e-6


CASES = [(2, 64, 8, 64), (3, 64, 7, 128), (2, 128, 14, 64), (1, 8, 9, 64), (4, 256, 7, 256), (2, 64, 28, 64),
         (1, 512, 7, 512), (8, 64, 56, 64)]


@pytest.mark.parametrize("N,C,H,K", CASES)
@pytest.mark.parametrize("mb", [0, 1, 5])
def test_wino_fwd(g, N, C, H, K, mb):
    x, w = _case(N, C, H, K, N + C + H + K + mb)
    u = torch.empty(16 * K * C, device="cuda")
    g.wino_weights(w, u, False)
    y = torch.full((N, K, H, H), float("nan"), device="cuda").contiguous(memory_format=CL)
    g.wino_conv(x, u, y, mb)
    ref = F.conv2d(x.double(), w.double(), padding=1)
    bound = F.conv2d(x.double().abs(), w.double().abs(), padding=1)
    assert (y.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("N,C,H,K", CASES[:6])
def test_wino_dgrad(g, N, C, H, K):
    """Grad-input = forward conv of dY with the flipped, transposed filter."""
    if C % 64:
        pytest.skip("grad-input output channels = C must be a multiple of 64")
    x, w = _case(N, C, H, K, 3 * N + C + H + K)
    dy = torch.randn(N, K, H, H, device="cuda").contiguous(memory_format=CL)
    u = torch.empty(16 * K * C, device="cuda")
    g.wino_weights(w, u, True)
    dx = torch.full(x.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    g.wino_conv(dy, u, dx, 0)
    ref = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [1, 1], [1, 1], [1, 1],
                                              False, [0, 0], 1, [True, False, False])[0]
    bound = torch.ops.aten.convolution_backward(dy.double().abs(), x.double(), w.double().abs(), None, [1, 1], [1, 1],
                                                [1, 1], False, [0, 0], 1, [True, False, False])[0]
    assert (dx.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("H,mb", [(14, 3), (7, 0), (9, 2)])
def test_wino_stats(g, H, mb):
    N, C, K = 4, 64, 128
    x, w = _case(N, C, H, K, H + mb)
    u = torch.empty(16 * K * C, device="cuda")
    g.wino_weights(w, u, False)
    y = torch.full((N, K, H, H), float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, K), float("nan"), device="cuda")
    rows = g.wino_conv(x, u, y, mb, st)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, K)
    s = st[:, :rows].double().sum(1)
    assert torch.allclose(s[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("twin", [False, True])
@pytest.mark.parametrize("H", [9, 14])
def test_wino_dgrad_bn_epilogue(g, twin, H):
    """dz = mask ? dX + dy2 : 0 with partials sum(dz), sum(dz * h) (fp32 mask:
    one byte per 4 channels) -- the conv_nt BN-backward contract."""
    torch.manual_seed(H * 2 + twin)
    N, C, Co = 2, 64, 128
    dy = torch.randn(N, Co, H, H, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(Co, C, 3, 3, device="cuda") * 0.1).contiguous(memory_format=CL)
    h = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    dy2 = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL) if twin else None
    relu = torch.rand(N, C, H, H, device="cuda") > 0.4
    M = N * H * H
    bits = relu.permute(0, 2, 3, 1).reshape(M, C // 4, 4).to(torch.int32)
    mask = (bits * torch.tensor([1, 2, 4, 8], device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).reshape(-1)
    ref_dx = torch.ops.aten.convolution_backward(dy.double(), h.double(), w.double(), None, [1, 1], [1, 1], [1, 1],
                                                 False, [0, 0], 1, [True, False, False])[0]
    dz_ref = torch.where(relu, ref_dx + (dy2.double() if twin else 0), torch.zeros_like(ref_dx))
    u = torch.empty(16 * Co * C, device="cuda")
    g.wino_weights(w, u, True)
    dz = torch.full(h.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, C), float("nan"), device="cuda")
    rows = g.wino_conv(dy, u, dz, 0, st, h, dy2, mask)
    assert (dz.double() - dz_ref).abs().max().item() <= 1e-5 * dz_ref.abs().max().item() + 1e-5
    s = st[:, :rows].double().sum(1)
    dzc = dz_ref.permute(0, 2, 3, 1).reshape(M, C)
    hc = h.double().permute(0, 2, 3, 1).reshape(M, C)
    assert torch.allclose(s[0], dzc.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[1], (dzc * hc).sum(0), rtol=1e-5, atol=1e-4)


def test_fastconv2d_f32_winograd_autograd(monkeypatch):
    """FastConv2d fp32 3x3 stride-1 with the Winograd candidates forced:
    forward and grad-input run wino_conv and match fp64 torch."""
    from gaussiank_sgd_amd.ops import conv1x1
    monkeypatch.setattr(conv1x1, "_FORCE", "wino")
    monkeypatch.setattr(conv1x1, "_choices", {})
    torch.manual_seed(7)
    conv = conv1x1.FastConv2d(64, 128, 3, stride=1, padding=1, bias=False).cuda().to(memory_format=CL)
    x = torch.randn(4, 64, 14, 14, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    y = conv(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xd = x.detach().double().requires_grad_(True)
    wd = conv.weight.detach().double().requires_grad_(True)
    yd = F.conv2d(xd, wd, padding=1)
    yd.backward(dy.double())
    assert (y.double() - yd).abs().max().item() <= 1e-5 * yd.abs().max().item() + 1e-5
    assert (x.grad.double() - xd.grad).abs().max().item() <= 1e-5 * xd.grad.abs().max().item() + 1e-5
    assert (conv.weight.grad.double() - wd.grad).abs().max().item() <= 1e-5 * wd.grad.abs().max().item() + 1e-5
    used = {v[0] for k, v in conv1x1.tuned_choices().items() if "f32" in k and k[0] in ("fwd", "dgrad")}
    assert "wino" in used, conv1x1.tuned_choices()


@pytest.mark.parametrize("N,C,H,K", [(2, 64, 8, 64), (3, 64, 7, 128), (2, 128, 14, 64), (4, 256, 7, 256),
                                     (2, 64, 28, 64), (1, 512, 7, 512), (8, 64, 56, 64)])
@pytest.mark.parametrize("splits", [0, 3, 64])
def test_wino_wgrad(g, N, C, H, K, splits):
    """out += dW (accumulates into the existing values) vs fp64."""
    x, w = _case(N, C, H, K, 5 * N + C + H + K + splits)
    dy = torch.randn(N, K, H, H, device="cuda").contiguous(memory_format=CL)
    out0 = torch.randn(K, C, 3, 3, device="cuda").contiguous(memory_format=CL)
    out = out0.clone()
    part = torch.empty(int(g.wino_wgrad_ws(N, H, H, C, K, splits)), device="cuda")
    g.wino_wgrad(x, dy, out, part, splits)
    ref = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [1, 1], [1, 1], [1, 1],
                                              False, [0, 0], 1, [False, True, False])[1]
    bound = torch.ops.aten.convolution_backward(dy.double().abs(), x.double().abs(), w.double(), None, [1, 1], [1, 1],
                                                [1, 1], False, [0, 0], 1, [False, True, False])[1]
    err = (out.double() - out0.double() - ref).abs().max().item()
    assert err <= _tol(bound) + 1e-6 * out0.abs().max().item(), err


# non-square spatial sizes (H != W, odd W): the kernels take H and W separately
# and the autotuner offers Winograd for any fp32 3x3 stride-1 shape
RECT = [(2, 64, 7, 9, 64), (2, 64, 14, 8, 128), (1, 128, 5, 11, 64), (3, 64, 9, 4, 64)]


def _rect(N, C, H, W, K, seed):
    torch.manual_seed(seed)
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(K, C, 3, 3, device="cuda") * (9 * C) ** -0.5).contiguous(memory_format=CL)
    return x, w


@pytest.mark.parametrize("N,C,H,W,K", RECT)
@pytest.mark.parametrize("mb", [0, 3])
def test_wino_fwd_nonsquare(g, N, C, H, W, K, mb):
    x, w = _rect(N, C, H, W, K, N + C + H + 3 * W + K + mb)
    u = torch.empty(16 * K * C, device="cuda")
    g.wino_weights(w, u, False)
    y = torch.full((N, K, H, W), float("nan"), device="cuda").contiguous(memory_format=CL)
    g.wino_conv(x, u, y, mb)
    ref = F.conv2d(x.double(), w.double(), padding=1)
    bound = F.conv2d(x.double().abs(), w.double().abs(), padding=1)
    assert (y.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("N,C,H,W,K", RECT)
def test_wino_dgrad_nonsquare(g, N, C, H, W, K):
    x, w = _rect(N, C, H, W, K, 7 * N + C + H + W + K)
    dy = torch.randn(N, K, H, W, device="cuda").contiguous(memory_format=CL)
    u = torch.empty(16 * K * C, device="cuda")
    g.wino_weights(w, u, True)
    dx = torch.full(x.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    g.wino_conv(dy, u, dx, 0)
    ref = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [1, 1], [1, 1], [1, 1],
                                              False, [0, 0], 1, [True, False, False])[0]
    bound = torch.ops.aten.convolution_backward(dy.double().abs(), x.double(), w.double().abs(), None, [1, 1], [1, 1],
                                                [1, 1], False, [0, 0], 1, [True, False, False])[0]
    assert (dx.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("N,C,H,W,K", RECT)
@pytest.mark.parametrize("splits", [0, 3])
def test_wino_wgrad_nonsquare(g, N, C, H, W, K, splits):
    x, w = _rect(N, C, H, W, K, 11 * N + C + H + W + K + splits)
    dy = torch.randn(N, K, H, W, device="cuda").contiguous(memory_format=CL)
    out = torch.zeros(K, C, 3, 3, device="cuda").contiguous(memory_format=CL)
    part = torch.empty(int(g.wino_wgrad_ws(N, H, W, C, K, splits)), device="cuda")
    g.wino_wgrad(x, dy, out, part, splits)
    ref = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [1, 1], [1, 1], [1, 1],
                                              False, [0, 0], 1, [False, True, False])[1]
    bound = torch.ops.aten.convolution_backward(dy.double().abs(), x.double().abs(), w.double(), None, [1, 1], [1, 1],
                                                [1, 1], False, [0, 0], 1, [False, True, False])[1]
    assert (out.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("N,C,H,K,splits", [(4, 512, 7, 512, 4), (2, 256, 14, 256, 2), (3, 64, 9, 128, 2),
                                              (1, 128, 7, 64, 4)])
@pytest.mark.parametrize("mb", [0, 3])
def test_wino_fwd_split_stats(g, N, C, H, K, splits, mb):
    """Input-channel split (small batches): fp32 partial planes summed by the
    reduce pass, which also writes the BatchNorm statistics partials."""
    x, w = _case(N, C, H, K, N + C + H + K + splits)
    u = torch.empty(16 * K * C, device="cuda")
    g.wino_weights(w, u, False)
    y = torch.full((N, K, H, H), float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, K), float("nan"), device="cuda")
    rows = g.wino_conv(x, u, y, mb, st, splits=splits)
    ref = F.conv2d(x.double(), w.double(), padding=1)
    bound = F.conv2d(x.double().abs(), w.double().abs(), padding=1)
    assert (y.double() - ref).abs().max().item() <= _tol(bound)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, K)
    s = st[:, :rows].double().sum(1)
    assert torch.allclose(s[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)
    y2 = torch.full_like(y, float("nan"))
    g.wino_conv(x, u, y2, mb, splits=splits)            # plain epilogue
    assert (y2.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("twin", [False, True])
def test_wino_dgrad_bn_epilogue_split(g, twin):
    torch.manual_seed(31 + twin)
    N, C, Co, H = 2, 128, 256, 7
    dy = torch.randn(N, Co, H, H, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(Co, C, 3, 3, device="cuda") * 0.05).contiguous(memory_format=CL)
    h = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    dy2 = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL) if twin else None
    relu = torch.rand(N, C, H, H, device="cuda") > 0.4
    M = N * H * H
    bits = relu.permute(0, 2, 3, 1).reshape(M, C // 4, 4).to(torch.int32)
    mask = (bits * torch.tensor([1, 2, 4, 8], device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).reshape(-1)
    ref_dx = torch.ops.aten.convolution_backward(dy.double(), h.double(), w.double(), None, [1, 1], [1, 1], [1, 1],
                                                 False, [0, 0], 1, [True, False, False])[0]
    dz_ref = torch.where(relu, ref_dx + (dy2.double() if twin else 0), torch.zeros_like(ref_dx))
    u = torch.empty(16 * Co * C, device="cuda")
    g.wino_weights(w, u, True)
    dz = torch.full(h.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, C), float("nan"), device="cuda")
    rows = g.wino_conv(dy, u, dz, 0, st, h, dy2, mask, splits=4)
    assert (dz.double() - dz_ref).abs().max().item() <= 1e-5 * dz_ref.abs().max().item() + 1e-5
    s = st[:, :rows].double().sum(1)
    dzc = dz_ref.permute(0, 2, 3, 1).reshape(M, C)
    hc = h.double().permute(0, 2, 3, 1).reshape(M, C)
    assert torch.allclose(s[0], dzc.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[1], (dzc * hc).sum(0), rtol=1e-5, atol=1e-4)
