"""fp32 MFMA GEMMs / implicit-GEMM convolutions (ops/csrc/kernels/gemm.hip,
v_mfma_f32_16x16x4_f32) vs an fp64 PyTorch reference at fp32 tolerances:
every fp32 tile configuration, resident / streamed weight panels, M tails,
stride-2 grad-input classes, grad-weight splits, the BatchNorm-statistics and
BN-backward epilogues, and the FastConv2d fp32 autograd path."""
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


def _tol(ref_abs):
    # fp32 accumulation of K products: ~K * 2^-24 relative to the sum of |terms|
    return 2e-6 * ref_abs.max().item() + 1e-6


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (777, 128, 192), (2048, 512, 128),
                                   (513, 192, 320), (300, 256, 1024)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 7, 11, 13, 22, 24, 101, 104, 201, 203,
                                 # 32x64 wave tiles (family 1000): every tile, panels and stage counts
                                 1001, 1002, 1003, 1004, 1005, 1006, 1007, 1011, 1022, 1103, 1205, 1217])
def test_gemm_nt_f32(g, M, N, K, cfg):
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    C = torch.full((M, N), float("nan"), device="cuda")
    g.gemm_nt(A, B, C, cfg, 0)
    ref = A.double() @ B.double().t()
    err = (C.double() - ref).abs().max().item()
    assert err <= _tol(A.double().abs() @ B.double().abs().t()), err


@pytest.mark.parametrize("cfg,mb", [(13, 1), (24, 3), (204, 7), (0, 5), (1001, 3), (1105, 2), (1003, 0), (1207, 9)])
def test_gemm_nt_f32_few_blocks_bias_stats(g, cfg, mb):
    """Persistent blocks walking many tiles (partial last tile) with the bias
    and BatchNorm-statistics epilogues."""
    torch.manual_seed(cfg + mb)
    M, N, K = 5000 + 37, 256, 128
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    bias = torch.randn(N, device="cuda")
    C = torch.full((M, N), float("nan"), device="cuda")
    st = torch.full((2, 64, N), float("nan"), device="cuda")
    rows = g.gemm_nt(A, B, C, cfg, mb, st, bias)
    ref = A.double() @ B.double().t() + bias.double()
    assert (C.double() - ref).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 1)
    s = st[:, :rows].double().sum(1)
    Cd = C.double()
    assert torch.allclose(s[0], Cd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (Cd * Cd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (777, 128, 192), (2500, 512, 256),
                                   (130, 64, 128), (5000, 128, 512), (3001, 256, 256)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11, 14, 16])
@pytest.mark.parametrize("splits", [0, 1, 7])
def test_gemm_tn_acc_f32(g, M, N, K, cfg, splits):
    torch.manual_seed(M * 3 + N + K)
    G = torch.randn(M, N, device="cuda")
    X = torch.randn(M, K, device="cuda")
    W0 = torch.randn(N, K, device="cuda")
    W = W0.clone()
    g.gemm_tn_acc(G, X, W, cfg, splits)
    ref = W0.double() + G.double().t() @ X.double()
    err = (W.double() - ref).abs().max().item()
    assert err <= _tol(G.double().abs().t() @ X.double().abs() + 1), err


def _conv_case(N, C, H, Co, k):
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(Co, C, k, k, device="cuda") * (C * k * k) ** -0.5).contiguous(memory_format=CL)
    return x, w


CONV_CASES = [(2, 64, 9, 64, 3, 1, 1), (3, 128, 7, 64, 3, 2, 1), (2, 64, 14, 128, 3, 2, 1),
              (2, 128, 5, 256, 1, 1, 0), (1, 64, 11, 192, 3, 1, 1), (2, 256, 8, 128, 1, 2, 0)]


@pytest.mark.parametrize("N,C,H,Co,k,s,p", CONV_CASES)
@pytest.mark.parametrize("cfg", [0, 1, 3, 22, 104, 7, 204, 21, 1001, 1002, 1104, 1007, 1016])
def test_conv_nt_f32(g, N, C, H, Co, k, s, p, cfg):
    torch.manual_seed(N + C + H + Co)
    x, w = _conv_case(N, C, H, Co, k)
    zero = torch.zeros(64, device="cuda")
    ref = F.conv2d(x.double(), w.double(), stride=s, padding=p)
    bound = F.conv2d(x.double().abs(), w.double().abs(), stride=s, padding=p)
    y = torch.full(ref.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    g.conv_nt(x, w, y, zero, s, p, cfg, 0)
    assert (y.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("N,C,H,Co,k,s,p", [(4, 512, 14, 512, 3, 2, 1), (2, 256, 28, 256, 3, 2, 1),
                                            (3, 128, 9, 64, 3, 1, 1), (4, 1024, 14, 256, 1, 2, 0)])
@pytest.mark.parametrize("cfg", [20004, 41002, 81001, 30004])
def test_conv_nt_f32_splitk_stats(g, N, C, H, Co, k, s, p, cfg):
    """Implicit-GEMM split-K: each plane starts at its own (tap, channel)
    slice (planes cross tap boundaries when the slice count per tap does not
    divide), reduce epilogue with the bias and BatchNorm statistics."""
    S = cfg // 10000
    torch.manual_seed(N + C + H + Co + cfg)
    x, w = _conv_case(N, C, H, Co, k)
    if (k * k * C // 32) % S:
        OH = (H + 2 * p - k) // s + 1
        y = torch.empty(N, Co, OH, OH, device="cuda").contiguous(memory_format=CL)
        with pytest.raises(RuntimeError):
            g.conv_nt(x, w, y, torch.zeros(64, device="cuda"), s, p, cfg, 0)
        return
    bias = torch.randn(Co, device="cuda")
    zero = torch.zeros(64, device="cuda")
    ref = F.conv2d(x.double(), w.double(), bias.double(), stride=s, padding=p)
    bound = F.conv2d(x.double().abs(), w.double().abs(), bias.double().abs(), stride=s, padding=p)
    y = torch.full(ref.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    M = ref.shape[0] * ref.shape[2] * ref.shape[3]
    st = torch.full((2, min(1280, (M + 63) // 64), Co), float("nan"), device="cuda")
    rows = g.conv_nt(x, w, y, zero, s, p, cfg, 0, st, bias)
    assert (y.double() - ref).abs().max().item() <= _tol(bound)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, Co)
    sm = st[:, :rows].double().sum(1)
    assert torch.allclose(sm[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(sm[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,C,H,Co,k,s,p", [c for c in CONV_CASES if c[5] == 2])
@pytest.mark.parametrize("cfg", [0, 1, 4, 13, 1002, 1103])
def test_conv_dgrad_s2_f32(g, N, C, H, Co, k, s, p, cfg):
    torch.manual_seed(N + 5 * C + H + Co)
    x, w = _conv_case(N, C, H, Co, k)
    xr = x.double().requires_grad_(True)
    yr = F.conv2d(xr, w.double(), stride=s, padding=p)
    dy = torch.randn(yr.shape, device="cuda").contiguous(memory_format=CL)
    yr.backward(dy.double())
    dx = torch.full(x.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    g.conv_dgrad_s2(dy, w, dx, torch.zeros(64, device="cuda"), cfg, 0)
    assert (dx.double() - xr.grad).abs().max().item() <= 1e-5 * xr.grad.abs().max().item() + 1e-5


@pytest.mark.parametrize("N,C,H,Co,k,s,p", CONV_CASES)
@pytest.mark.parametrize("cfg,splits", [(0, 0), (1, 3), (4, 0), (2, 7), (7, 0), (8, 2), (14, 0), (9, 0), (13, 5)])
def test_conv_tn_acc_f32(g, N, C, H, Co, k, s, p, cfg, splits):
    torch.manual_seed(N * 7 + C + H + Co)
    x, w = _conv_case(N, C, H, Co, k)
    xr = x.double()
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=p)
    dy = torch.randn(yr.shape, device="cuda").contiguous(memory_format=CL)
    yr.backward(dy.double())
    out = torch.zeros(Co, C, k, k, device="cuda").contiguous(memory_format=CL)
    g.conv_tn_acc(dy, x, out, torch.zeros(64, device="cuda"), s, p, cfg, splits)
    err = (out.double() - wr.grad).abs().max().item()
    assert err <= 1e-5 * wr.grad.abs().max().item() + 1e-5, err


@pytest.mark.parametrize("M,N,K", [(1568, 512, 2048), (6272 + 5, 256, 1024), (100, 64, 512)])
@pytest.mark.parametrize("cfg", [20004, 40001, 81001, 21002, 41003, 80004])
@pytest.mark.parametrize("mb", [0, 1 << 20, 3])
def test_gemm_nt_f32_splitk_bias_stats(g, M, N, K, cfg, mb):
    """Split-K (cfg + 10000 S): S fp32 partial planes over K slices, summed by
    the reduce epilogue with the bias and BatchNorm-statistics partials."""
    S = cfg // 10000
    if K % (64 * S):
        pytest.skip("K not divisible")
    torch.manual_seed(M + N + cfg)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    bias = torch.randn(N, device="cuda")
    C = torch.full((M, N), float("nan"), device="cuda")
    st = torch.full((2, min(1280, (M + 63) // 64), N), float("nan"), device="cuda")
    rows = g.gemm_nt(A, B, C, cfg, mb, st, bias)
    ref = A.double() @ B.double().t() + bias.double()
    assert (C.double() - ref).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 1)
    assert 1 <= rows <= st.shape[1]
    s = st[:, :rows].double().sum(1)
    Cd = C.double()
    assert torch.allclose(s[0], Cd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (Cd * Cd).sum(0), rtol=1e-5, atol=1e-3)
    C2 = torch.full((M, N), float("nan"), device="cuda")
    g.gemm_nt(A, B, C2, cfg, mb)                       # plain epilogue
    assert (C2.double() - (ref - bias.double())).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 1)


def test_gemm_nt_f32_splitk_refuses_bad_k(g):
    A = torch.randn(64, 192, device="cuda")
    B = torch.randn(64, 192, device="cuda")
    C = torch.empty(64, 64, device="cuda")
    with pytest.raises(RuntimeError):
        g.gemm_nt(A, B, C, 40004, 0)                    # K = 192 is not a multiple of 64 * 4


@pytest.mark.parametrize("twin", [False, True])
@pytest.mark.parametrize("cfg", [20004, 41002])
def test_dgrad_bn_epilogue_f32_splitk(g, twin, cfg):
    """Split-K grad-input with the BN-backward epilogue in the reduce pass."""
    torch.manual_seed(7 + twin)
    M, C, Co = 1568 + 3, 256, 1024
    dy = torch.randn(M, Co, device="cuda")
    w = torch.randn(Co, C, device="cuda") * Co ** -0.5
    h = torch.randn(M, C, device="cuda")
    dy2 = torch.randn(M, C, device="cuda") if twin else None
    relu = torch.rand(M, C, device="cuda") > 0.4
    bits = relu.reshape(M, C // 4, 4).to(torch.int32)
    mask = (bits * torch.tensor([1, 2, 4, 8], device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).reshape(-1)
    ref = dy.double() @ w.double() + (dy2.double() if twin else 0)
    ref = torch.where(relu, ref, torch.zeros_like(ref))
    dz = torch.full((M, C), float("nan"), device="cuda")
    st = torch.full((2, 64, C), float("nan"), device="cuda")
    rows = g.gemm_nt(dy, w.t().contiguous(), dz, cfg, 0, st, None, h, dy2, mask)
    assert (dz.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-5
    s = st[:, :rows].double().sum(1)
    assert torch.allclose(s[0], ref.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[1], (ref * h.double()).sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("twin", [False, True])
@pytest.mark.parametrize("cfg", [4, 1002, 1003, 1105])
def test_dgrad_bn_epilogue_f32(g, k, twin, cfg):
    """Grad-input with the BN-backward epilogue: dz = mask ? dX + dy2 : 0 and the
    partials sum(dz), sum(dz * h) -- fp32 operands, fp32 ReLU mask layout."""
    torch.manual_seed(k * 10 + twin)
    N, C, H, Co = 2, 64, 9, 128
    p = k // 2
    dy = torch.randn(N, Co, H, H, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(Co, C, k, k, device="cuda") * 0.1).contiguous(memory_format=CL)
    h = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    dy2 = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL) if twin else None
    relu = torch.rand(N, C, H, H, device="cuda") > 0.4
    M = N * H * H
    # bn_act.hip fp32 mask: one byte per 4 channels, bit i = channel 4j + i
    bits = relu.permute(0, 2, 3, 1).reshape(M, C // 4, 4).to(torch.int32)
    mask = (bits * torch.tensor([1, 2, 4, 8], device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).reshape(-1)
    ref_dx = torch.ops.aten.convolution_backward(dy.double(), h.double(), w.double(), None, [1, 1], [p, p], [1, 1],
                                                 False, [0, 0], 1, [True, False, False])[0]
    dz_ref = ref_dx + (dy2.double() if twin else 0)
    dz_ref = torch.where(relu, dz_ref, torch.zeros_like(dz_ref))
    dz = torch.full(h.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, C), float("nan"), device="cuda")
    zero = torch.zeros(64, device="cuda")
    if k == 1:
        rows = g.gemm_nt(dy.permute(0, 2, 3, 1).reshape(M, Co), w.reshape(Co, C).t().contiguous(),
                         dz.permute(0, 2, 3, 1).reshape(M, C), cfg, 0, st, None,
                         h.permute(0, 2, 3, 1).reshape(M, C),
                         dy2.permute(0, 2, 3, 1).reshape(M, C) if twin else None, mask)
    else:
        wf = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL)
        rows = g.conv_nt(dy, wf, dz, zero, 1, p, cfg, 0, st, None, h, dy2, mask)
    assert (dz.double() - dz_ref).abs().max().item() <= 1e-5 * dz_ref.abs().max().item() + 1e-5
    s = st[:, :rows].double().sum(1)
    dzc = dz_ref.permute(0, 2, 3, 1).reshape(M, C)
    hc = h.double().permute(0, 2, 3, 1).reshape(M, C)
    assert torch.allclose(s[0], dzc.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[1], (dzc * hc).sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("k,s", [(1, 1), (3, 1), (3, 2), (1, 2)])
def test_fastconv2d_f32_autograd(k, s):
    """FastConv2d on fp32 inputs (no autocast) runs the fp32 HIP kernels for
    forward, grad-input and grad-weight and matches fp64 torch."""
    from gaussiank_sgd_amd.ops import conv1x1
    torch.manual_seed(k * 3 + s)
    conv = conv1x1.FastConv2d(64, 128, k, stride=s, padding=k // 2, bias=False).cuda().to(memory_format=CL)
    x = torch.randn(4, 64, 14, 14, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    y = conv(x)
    assert y.dtype == torch.float32
    dy = torch.randn_like(y)
    y.backward(dy)
    xd = x.detach().double().requires_grad_(True)
    wd = conv.weight.detach().double().requires_grad_(True)
    yd = F.conv2d(xd, wd, stride=s, padding=k // 2)
    yd.backward(dy.double())
    assert (y.double() - yd).abs().max().item() <= 1e-5 * yd.abs().max().item() + 1e-5
    assert (x.grad.double() - xd.grad).abs().max().item() <= 1e-5 * xd.grad.abs().max().item() + 1e-5
    assert (conv.weight.grad.double() - wd.grad).abs().max().item() <= 1e-5 * wd.grad.abs().max().item() + 1e-5
    keys = [key for key in conv1x1.tuned_choices() if "f32" in key]
    assert keys, "fp32 path was not taken"
