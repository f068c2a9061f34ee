"""bf16x6 Winograd F(2x2, 3x3) (ops/csrc/kernels/wino_x6.hip) vs an fp64
PyTorch reference: forward, grad-input (flipped filter), partial tiles,
persistent blocks over many tile blocks, the BatchNorm-statistics and
BN-backward epilogues -- each no less accurate than the fp32-MFMA Winograd
(winograd.hip) on the same case, plus the batched per-step filter planes
(prep.hip) equal to the standalone transform and the FastConv2d path
choosing the kernel."""
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


def _err(y, ref):
    return (y.double() - ref).abs().max().item()


CASES = [(2, 32, 8, 32), (3, 64, 7, 128), (2, 128, 14, 64), (1, 32, 9, 96), (4, 256, 7, 256), (2, 64, 28, 64),
         (1, 512, 7, 512), (8, 64, 56, 64), (2, 96, 5, 32)]


@pytest.mark.parametrize("N,C,H,K", CASES)
@pytest.mark.parametrize("mb", [0, 1, 5])
def test_wx6_fwd(g, N, C, H, K, mb):
    x, w = _case(N, C, H, K, N + C + H + K + mb)
    u3 = torch.empty(48 * K * C, device="cuda", dtype=torch.bfloat16)
    g.wino_x6_weights(w, u3, False)
    y = torch.full((N, K, H, H), float("nan"), device="cuda").contiguous(memory_format=CL)
    g.wino_x6_conv(x, u3, y, mb)
    ref = F.conv2d(x.double(), w.double(), padding=1)
    bound = F.conv2d(x.double().abs(), w.double().abs(), padding=1)
    e6 = _err(y, ref)
    assert e6 <= 1e-5 * bound.max().item() + 1e-6, e6
    if K % 64 == 0 and C % 8 == 0:
        u = torch.empty(16 * K * C, device="cuda")
        g.wino_weights(w, u, False)
        y32 = torch.empty_like(y)
        g.wino_conv(x, u, y32, mb)
        assert e6 <= 1.1 * _err(y32, ref) + 1e-7, (e6, _err(y32, ref))


@pytest.mark.parametrize("N,C,H,K", CASES[:7])
def test_wx6_dgrad(g, N, C, H, K):
    """Grad-input = forward conv of dY with the flipped, transposed filter."""
    x, w = _case(N, C, H, K, 3 * N + C + H + K)
    dy = torch.randn(N, K, H, H, device="cuda").contiguous(memory_format=CL)
    u3 = torch.empty(48 * K * C, device="cuda", dtype=torch.bfloat16)
    g.wino_x6_weights(w, u3, True)
    dx = torch.full(x.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    g.wino_x6_conv(dy, u3, dx, 0)
    ref = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [1, 1], [1, 1], [1, 1],
                                              False, [0, 0], 1, [True, False, False])[0]
    bound = torch.ops.aten.convolution_backward(dy.double().abs(), x.double(), w.double().abs(), None, [1, 1], [1, 1],
                                                [1, 1], False, [0, 0], 1, [True, False, False])[0]
    assert _err(dx, ref) <= 1e-5 * bound.max().item() + 1e-6


@pytest.mark.parametrize("H,mb", [(14, 3), (7, 0), (9, 2)])
def test_wx6_stats(g, H, mb):
    N, C, K = 4, 64, 128
    x, w = _case(N, C, H, K, H + mb)
    u3 = torch.empty(48 * K * C, device="cuda", dtype=torch.bfloat16)
    g.wino_x6_weights(w, u3, False)
    y = torch.full((N, K, H, H), float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, K), float("nan"), device="cuda")
    rows = g.wino_x6_conv(x, u3, y, mb, st)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, K)
    s = st[:, :rows].double().sum(1)
    assert torch.allclose(s[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("twin", [False, True])
@pytest.mark.parametrize("H", [9, 14])
def test_wx6_dgrad_bn_epilogue(g, twin, H):
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
    u3 = torch.empty(48 * Co * C, device="cuda", dtype=torch.bfloat16)
    g.wino_x6_weights(w, u3, True)
    dz = torch.full(h.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, C), float("nan"), device="cuda")
    rows = g.wino_x6_conv(dy, u3, dz, 0, st, h, dy2, mask)
    assert _err(dz, dz_ref) <= 1e-5 * dz_ref.abs().max().item() + 1e-5
    s = st[:, :rows].double().sum(1)
    dzc = dz_ref.permute(0, 2, 3, 1).reshape(M, C)
    hc = h.double().permute(0, 2, 3, 1).reshape(M, C)
    assert torch.allclose(s[0], dzc.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[1], (dzc * hc).sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("flip", [False, True])
def test_wx6_weight_prep_matches(g, flip):
    """The batched per-step re-layout (prep.hip kind 4 / 5) writes the same
    planes as the standalone filter transform."""
    from gaussiank_sgd_amd.ops import weight_prep
    _, w = _case(1, 64, 4, 96, 7 + flip)
    ref = torch.empty(48 * 96 * 64, device="cuda", dtype=torch.bfloat16)
    g.wino_x6_weights(w, ref, flip)
    wp = weight_prep.WeightPrep()
    with wp.step(torch.device("cuda")):
        u3 = weight_prep.wino_x6_filter(w, flip, True)       # registers + fills directly the first time
    with torch.no_grad():
        w.mul_(1.0)
    u3.fill_(0)
    with wp.step(torch.device("cuda")):                      # the batched launch rebuilds it
        got = weight_prep.wino_x6_filter(w, flip, True)
    torch.cuda.synchronize()
    assert got.data_ptr() == u3.data_ptr()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


def test_fastconv2d_wx6_autograd(monkeypatch):
    """FastConv2d fp32 3x3 stride-1 in the bf16x6 mode with the x6 Winograd
    forced: forward and grad-input run wino_x6_conv and match fp64 torch."""
    from gaussiank_sgd_amd.ops import conv1x1
    from gaussiank_sgd_amd.ops.conv1x1 import Conv3x3
    monkeypatch.setattr(conv1x1, "_FORCE", "wx6")
    monkeypatch.setattr(conv1x1, "_WX6", True)
    prev = conv1x1.set_f32_matmul("bf16x6")
    try:
        torch.manual_seed(0)
        conv = Conv3x3(64, 64).cuda().to(memory_format=CL)
        x = torch.randn(4, 64, 14, 14, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
        y = conv(x)
        gy = torch.randn_like(y)
        y.backward(gy)
        xr = x.detach().double().requires_grad_(True)
        yr = F.conv2d(xr, conv.weight.detach().double(), padding=1)
        yr.backward(gy.double())
        assert (y.double() - yr).abs().max().item() < 1e-4
        assert (x.grad.double() - xr.grad).abs().max().item() < 1e-4
        used = [v[0] for k, v in conv1x1.tuned_choices().items() if k[0] in ("fwd", "dgrad") and "wx6" in k]
        assert "wx6" in used, conv1x1.tuned_choices()
    finally:
        conv1x1.set_f32_matmul(prev)
