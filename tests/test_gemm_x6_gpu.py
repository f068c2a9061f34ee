"""bf16x6 fp32 GEMMs (ops/csrc/kernels/gemm_kern.h X6, cfg digit 100000):
fp32 operands split exactly into three bf16 parts, the six part products of
order <= 2 accumulated in fp32 on v_mfma_f32_16x16x32_bf16.  Checked against
an fp64 PyTorch reference at the SAME tolerances as the fp32-MFMA kernels
(tests/test_gemm_f32_gpu.py), and against the fp32-MFMA kernel's own error:
the split must be at least as accurate as the fp32 matrix cores, otherwise it
would not be an fp32 algorithm.  Row GEMMs (every tile family, resident /
streamed panels, M tails, split-K, bias / BatchNorm-statistics / BN-backward
epilogues, the lazy BN operand), implicit-GEMM convolutions, stride-2
grad-input classes and grad-weight (TN) GEMMs."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last
X6 = 100000


@pytest.fixture(scope="module")
def g():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error
    return torch.ops.gksgd


def _tol(ref_abs):
    return 2e-6 * ref_abs.max().item() + 1e-6


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (777, 128, 192), (2048, 512, 128),
                                   (513, 192, 320), (300, 256, 1024)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 7, 13, 22, 104, 201, 1001, 1002, 1003, 1005, 1104])
def test_gemm_nt_x6(g, M, N, K, cfg):
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    C = torch.full((M, N), float("nan"), device="cuda")
    g.gemm_nt(A, B, C, cfg + X6, 0)
    ref = A.double() @ B.double().t()
    err = (C.double() - ref).abs().max().item()
    assert err <= _tol(A.double().abs() @ B.double().abs().t()), err


@pytest.mark.parametrize("M,N,K", [(16384, 768, 3072), (25088, 512, 2048), (100352, 256, 1024)])
def test_x6_at_least_as_accurate_as_fp32_mfma(g, M, N, K):
    """RMS and max error vs fp64 of the bf16x6 kernel <= those of the
    fp32-MFMA kernel (+10% slack for sampling), on BERT / ResNet-50 shapes."""
    torch.manual_seed(K)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    rows = 4096
    ref = A[:rows].double() @ B.double().t()
    errs = {}
    for name, cfg in (("f32", 3), ("x6", 3 + X6)):
        C = torch.empty(M, N, device="cuda")
        g.gemm_nt(A, B, C, cfg, 0)
        d = C[:rows].double() - ref
        errs[name] = ((d.norm() / ref.norm()).item(), d.abs().max().item())
    assert errs["x6"][0] <= 1.1 * errs["f32"][0], errs
    assert errs["x6"][1] <= 1.1 * errs["f32"][1], errs


def test_x6_split_is_exact(g):
    """Values needing all 24 mantissa bits (and tiny / huge magnitudes) come
    through a K = 64 product with one non-zero term exactly: x * 1.0."""
    torch.manual_seed(0)
    M, N, K = 256, 64, 64
    A = torch.zeros(M, K, device="cuda")
    vals = torch.randn(M, device="cuda") * torch.logspace(-30, 30, M, device="cuda")
    vals = vals + vals * 2.0 ** -20     # low mantissa bits set
    A[:, 5] = vals
    B = torch.zeros(N, K, device="cuda")
    B[:, 5] = 1.0
    C = torch.empty(M, N, device="cuda")
    g.gemm_nt(A, B, C, 2 + X6, 0)
    assert torch.equal(C, vals[:, None].expand(M, N))


@pytest.mark.parametrize("cfg,mb", [(13, 1), (24, 3), (204, 7), (0, 5), (1001, 3), (1105, 2), (1003, 0)])
def test_gemm_nt_x6_few_blocks_bias_stats(g, cfg, mb):
    torch.manual_seed(cfg + mb)
    M, N, K = 5000 + 37, 256, 128
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    bias = torch.randn(N, device="cuda")
    C = torch.full((M, N), float("nan"), device="cuda")
    st = torch.full((2, 64, N), float("nan"), device="cuda")
    rows = g.gemm_nt(A, B, C, cfg + X6, mb, st, bias)
    ref = A.double() @ B.double().t() + bias.double()
    assert (C.double() - ref).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 1)
    s = st[:, :rows].double().sum(1)
    Cd = C.double()
    assert torch.allclose(s[0], Cd.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (Cd * Cd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("cfg", [20004, 41002, 81001])
def test_gemm_nt_x6_splitk(g, cfg):
    M, N, K = 1568, 512, 2048
    torch.manual_seed(cfg)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    bias = torch.randn(N, device="cuda")
    C = torch.full((M, N), float("nan"), device="cuda")
    st = torch.full((2, min(1280, (M + 63) // 64), N), float("nan"), device="cuda")
    rows = g.gemm_nt(A, B, C, cfg + X6, 0, st, bias)
    ref = A.double() @ B.double().t() + bias.double()
    assert (C.double() - ref).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 1)
    s = st[:, :rows].double().sum(1)
    assert torch.allclose(s[0], C.double().sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 1001, 1002])
@pytest.mark.parametrize("dy2", [False, True])
def test_gemm_nt_x6_bn_backward_epilogue(g, cfg, dy2):
    """BN-backward epilogue: dz = mask ? (A B^T + dy2) : 0 with partials
    sum(dz), sum(dz * h)."""
    torch.manual_seed(cfg + dy2)
    M, N, K = 3000, 256, 256
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    h = torch.randn(M, N, device="cuda")
    d2 = torch.randn(M, N, device="cuda") if dy2 else None
    keep = torch.rand(M, N // 4, 4, device="cuda") > 0.3
    mask = (keep.to(torch.uint8) * torch.tensor([1, 2, 4, 8], dtype=torch.uint8, device="cuda")).sum(-1).to(torch.uint8)
    C = torch.full((M, N), float("nan"), device="cuda")
    st = torch.full((2, min(1280, (M + 63) // 64), N), float("nan"), device="cuda")
    rows = g.gemm_nt(A, B, C, cfg + X6, 0, st, None, h, d2, mask)
    dx = A.double() @ B.double().t() + (d2.double() if dy2 else 0)
    dz = torch.where(keep.reshape(M, N), dx, torch.zeros_like(dx))
    assert (C.double() - dz).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 4)
    s = st[:, :rows].double().sum(1)
    assert torch.allclose(s[0], dz.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (dz * h.double()).sum(0), rtol=1e-5, atol=1e-3)


CONV_CASES = [(2, 64, 9, 64, 3, 1, 1), (3, 128, 7, 64, 3, 2, 1), (2, 64, 14, 128, 3, 2, 1),
              (2, 128, 5, 256, 1, 1, 0), (1, 64, 11, 192, 3, 1, 1), (2, 256, 8, 128, 1, 2, 0)]


def _conv_case(N, C, H, Co, k):
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(Co, C, k, k, device="cuda") * (C * k * k) ** -0.5).contiguous(memory_format=CL)
    return x, w


@pytest.mark.parametrize("N,C,H,Co,k,s,p", CONV_CASES)
@pytest.mark.parametrize("cfg", [0, 1, 3, 104, 204, 1001, 1002, 20004])
def test_conv_nt_x6(g, N, C, H, Co, k, s, p, cfg):
    torch.manual_seed(N + C + H + Co)
    x, w = _conv_case(N, C, H, Co, k)
    zero = torch.zeros(64, device="cuda")
    ref = F.conv2d(x.double(), w.double(), stride=s, padding=p)
    bound = F.conv2d(x.double().abs(), w.double().abs(), stride=s, padding=p)
    y = torch.full(ref.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    S = cfg // 10000
    if S > 1 and (k * k * C // 32) % S:
        with pytest.raises(RuntimeError):
            g.conv_nt(x, w, y, zero, s, p, cfg + X6, 0)
        return
    g.conv_nt(x, w, y, zero, s, p, cfg + X6, 0)
    assert (y.double() - ref).abs().max().item() <= _tol(bound)


@pytest.mark.parametrize("N,C,H,Co,k,s,p", [c for c in CONV_CASES if c[5] == 2])
@pytest.mark.parametrize("cfg", [0, 4, 1002])
def test_conv_dgrad_s2_x6(g, N, C, H, Co, k, s, p, cfg):
    torch.manual_seed(N + 5 * C + H + Co)
    x, w = _conv_case(N, C, H, Co, k)
    xr = x.double().requires_grad_(True)
    yr = F.conv2d(xr, w.double(), stride=s, padding=p)
    dy = torch.randn(yr.shape, device="cuda").contiguous(memory_format=CL)
    yr.backward(dy.double())
    dx = torch.full(x.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    g.conv_dgrad_s2(dy, w, dx, torch.zeros(64, device="cuda"), cfg + X6, 0)
    assert (dx.double() - xr.grad).abs().max().item() <= 1e-5 * xr.grad.abs().max().item() + 1e-5


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (2500, 512, 256), (130, 64, 128),
                                   (3001, 256, 256)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 4, 7, 9, 11, 14])
@pytest.mark.parametrize("splits", [0, 7])
def test_gemm_tn_acc_x6(g, M, N, K, cfg, splits):
    torch.manual_seed(M * 3 + N + K)
    G = torch.randn(M, N, device="cuda")
    X = torch.randn(M, K, device="cuda")
    W0 = torch.randn(N, K, device="cuda")
    W = W0.clone()
    g.gemm_tn_acc(G, X, W, cfg + X6, splits)
    ref = W0.double() + G.double().t() @ X.double()
    err = (W.double() - ref).abs().max().item()
    assert err <= _tol(G.double().abs().t() @ X.double().abs() + 1), err


@pytest.mark.parametrize("N,C,H,Co,k,s,p", CONV_CASES)
@pytest.mark.parametrize("cfg,splits", [(0, 0), (4, 0), (8, 2), (13, 5)])
def test_conv_tn_acc_x6(g, N, C, H, Co, k, s, p, cfg, splits):
    torch.manual_seed(N * 7 + C + H + Co)
    x, w = _conv_case(N, C, H, Co, k)
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(x.double(), wr, stride=s, padding=p)
    dy = torch.randn(yr.shape, device="cuda").contiguous(memory_format=CL)
    yr.backward(dy.double())
    out = torch.zeros(Co, C, k, k, device="cuda").contiguous(memory_format=CL)
    g.conv_tn_acc(dy, x, out, torch.zeros(64, device="cuda"), s, p, cfg + X6, splits)
    err = (out.double() - wr.grad).abs().max().item()
    assert err <= 1e-5 * wr.grad.abs().max().item() + 1e-5, err


def test_fastconv_autograd_x6_mode(g):
    """FastConv2d fp32 forward + backward with the bf16x6 candidates offered
    to the tuner (set_f32_matmul("bf16x6")) vs fp64 autograd."""
    from gaussiank_sgd_amd.ops import conv1x1
    prev = conv1x1.set_f32_matmul("bf16x6")
    try:
        torch.manual_seed(3)
        for (C, Co, k, s) in [(64, 128, 1, 1), (128, 128, 3, 1), (128, 256, 3, 2), (256, 64, 1, 2)]:
            conv = conv1x1.FastConv2d(C, Co, k, stride=s, padding=k // 2, bias=False).cuda()
            x = torch.randn(4, C, 14, 14, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
            y = conv(x)
            dy = torch.randn_like(y)
            y.backward(dy)
            xr = x.detach().double().requires_grad_(True)
            wr = conv.weight.detach().double().requires_grad_(True)
            yr = F.conv2d(xr, wr, stride=s, padding=k // 2)
            yr.backward(dy.double())
            tol = lambda r: 1e-5 * r.abs().max().item() + 1e-5  # noqa: E731
            assert (y.double() - yr).abs().max().item() <= tol(yr)
            assert (x.grad.double() - xr.grad).abs().max().item() <= tol(xr.grad)
            assert (conv.weight.grad.double() - wr.grad).abs().max().item() <= tol(wr.grad)
    finally:
        conv1x1.set_f32_matmul(prev)


# register-staged bf16x6 (gemm_nt_x62_kernel), tiles 1-7: family 2 splits both
# operands in the kernel, family 3 reads B pre-split by the binding (split3_rows)
X62 = [2 * X6 + t for t in range(1, 8)] + [3 * X6 + t for t in range(1, 8)]


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (777, 128, 192), (2048, 512, 128),
                                   (513, 192, 320), (300, 256, 1024), (5000, 768, 768)])
@pytest.mark.parametrize("cfg", X62)
@pytest.mark.parametrize("mb", [0, 3])
def test_gemm_nt_x62(g, M, N, K, cfg, mb):
    torch.manual_seed(M + N + K + cfg)
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
    C2 = torch.full((M, N), float("nan"), device="cuda")
    g.gemm_nt(A, B, C2, cfg, mb)
    assert (C2.double() - (ref - bias.double())).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 1)


@pytest.mark.parametrize("cfg", X62)
@pytest.mark.parametrize("dy2", [False, True])
def test_gemm_nt_x62_bn_backward_epilogue(g, cfg, dy2):
    torch.manual_seed(cfg + dy2)
    M, N, K = 3000, 256, 256
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * K ** -0.5
    h = torch.randn(M, N, device="cuda")
    d2 = torch.randn(M, N, device="cuda") if dy2 else None
    keep = torch.rand(M, N // 4, 4, device="cuda") > 0.3
    mask = (keep.to(torch.uint8) * torch.tensor([1, 2, 4, 8], dtype=torch.uint8, device="cuda")).sum(-1).to(torch.uint8)
    C = torch.full((M, N), float("nan"), device="cuda")
    st = torch.full((2, min(1280, (M + 63) // 64), N), float("nan"), device="cuda")
    rows = g.gemm_nt(A, B, C, cfg, 0, st, None, h, d2, mask)
    dx = A.double() @ B.double().t() + (d2.double() if dy2 else 0)
    dz = torch.where(keep.reshape(M, N), dx, torch.zeros_like(dx))
    assert (C.double() - dz).abs().max().item() <= _tol(A.double().abs() @ B.double().abs().t() + 4)
    s = st[:, :rows].double().sum(1)
    assert torch.allclose(s[0], dz.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[1], (dz * h.double()).sum(0), rtol=1e-5, atol=1e-3)


def test_x62_refuses_unsupported_calls(g):
    A = torch.randn(1568, 2048, device="cuda")
    B = torch.randn(512, 2048, device="cuda")
    C = torch.empty(1568, 512, device="cuda")
    with pytest.raises(RuntimeError):
        g.gemm_nt(A, B, C, 2 * X6 + 20001, 0)     # split-K
    with pytest.raises(RuntimeError):
        g.gemm_nt(A, B, C, 3 * X6 + 20001, 0)
    with pytest.raises(RuntimeError):
        g.gemm_nt(A.bfloat16(), B.bfloat16(), C.bfloat16(), 3 * X6 + 1, 0)   # pre-split B: fp32 only
    W = torch.zeros(512, 2048, device="cuda")
    with pytest.raises(RuntimeError):
        g.gemm_tn_acc(torch.randn(1568, 512, device="cuda"), A, W, 3 * X6 + 1, 0)   # forward / dgrad kernels only


@pytest.mark.parametrize("R,S,ld", [(64, 768, 768), (192, 256, 320), (1024, 3072, 3072)])
def test_split3_rows_layout(g, R, S, ld):
    """The pre-split B of cfg family 3 equals the kernel-side split: a family-3
    GEMM and a family-2 GEMM over the same operands agree bit for bit."""
    torch.manual_seed(R + S)
    A = torch.randn(300, S, device="cuda")
    Bfull = torch.randn(R, ld, device="cuda") * S ** -0.5
    B = Bfull[:, :S]   # strided rows when ld > S
    C2 = torch.empty(300, R, device="cuda")
    C3 = torch.empty(300, R, device="cuda")
    g.gemm_nt(A, B, C2, 2 * X6 + 1, 0)
    g.gemm_nt(A, B, C3, 3 * X6 + 1, 0)
    assert torch.equal(C2, C3)


@pytest.mark.parametrize("N,C,H,Co,k,s,p", CONV_CASES + [(2, 128, 7, 128, 3, 1, 1), (1, 64, 6, 64, 3, 2, 1)])
@pytest.mark.parametrize("cfg", X62)
def test_conv_nt_x62(g, N, C, H, Co, k, s, p, cfg):
    """Register-staged bf16x6 implicit GEMM: per-pixel tap validity, zero
    padding rows, stride 2, tail tiles; with the BN-statistics epilogue."""
    torch.manual_seed(N + C + H + Co + cfg)
    x, w = _conv_case(N, C, H, Co, k)
    zero = torch.zeros(64, device="cuda")
    ref = F.conv2d(x.double(), w.double(), stride=s, padding=p)
    bound = F.conv2d(x.double().abs(), w.double().abs(), stride=s, padding=p)
    y = torch.full(ref.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    M = ref.shape[0] * ref.shape[2] * ref.shape[3]
    st = torch.full((2, min(1280, (M + 63) // 64), Co), float("nan"), device="cuda")
    rows = g.conv_nt(x, w, y, zero, s, p, cfg, 0, st)
    assert (y.double() - ref).abs().max().item() <= _tol(bound)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, Co)
    sm = st[:, :rows].double().sum(1)
    assert torch.allclose(sm[0], yd.sum(0), rtol=1e-5, atol=1e-3)


TN_X62 = [2 * X6 + t for t in range(1, 9)]   # register-staged bf16x6 grad-weight (gemm_tn_x62_kernel), tiles 1-8


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (2500, 512, 256), (130, 64, 128),
                                   (3001, 256, 256), (777, 128, 512)])
@pytest.mark.parametrize("cfg", TN_X62)
@pytest.mark.parametrize("splits", [0, 1, 7])
def test_gemm_tn_acc_x62(g, M, N, K, cfg, splits):
    torch.manual_seed(M * 3 + N + K + cfg)
    G = torch.randn(M, N, device="cuda")
    X = torch.randn(M, K, device="cuda")
    W0 = torch.randn(N, K, device="cuda")
    W = W0.clone()
    g.gemm_tn_acc(G, X, W, cfg, splits)
    ref = W0.double() + G.double().t() @ X.double()
    err = (W.double() - ref).abs().max().item()
    assert err <= _tol(G.double().abs().t() @ X.double().abs() + 1), err


def test_tn_x62_refuses_implicit_gemm(g):
    x = torch.randn(2, 64, 9, 9, device="cuda").contiguous(memory_format=CL)
    dy = torch.randn(2, 64, 9, 9, device="cuda").contiguous(memory_format=CL)
    out = torch.zeros(64, 64, 3, 3, device="cuda").contiguous(memory_format=CL)
    with pytest.raises(RuntimeError):
        g.conv_tn_acc(dy, x, out, torch.zeros(64, device="cuda"), 1, 1, 2 * X6 + 1, 0)
