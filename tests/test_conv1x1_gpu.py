"""Conv1x1 (ops/conv1x1.py): autotuned MFMA GEMM 1x1 convolution vs an fp32
PyTorch reference (forward, grad-input, grad-weight), plain and through the
bf16-shadow / direct-to-arena path of the DistributedOptimizer."""
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


def _ref(x, w, dy, stride=1, padding=0):
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    y = F.conv2d(xr, wr, stride=stride, padding=padding)
    y.backward(dy.float())
    return y.detach(), xr.grad, wr.grad


@pytest.mark.parametrize("N,C,H,K,k,s", [(4, 64, 14, 64, 3, 1), (3, 128, 9, 128, 3, 2), (2, 64, 10, 256, 1, 2),
                                         (2, 256, 7, 128, 3, 1)])
def test_fastconv_kxk(N, C, H, K, k, s, hip_only):
    from gaussiank_sgd_amd.ops.conv1x1 import FastConv2d
    torch.manual_seed(N * C + K + k)
    m = FastConv2d(C, K, k, stride=s, padding=k // 2, bias=False).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    ry, rdx, rdw = _ref(x, m.weight, dy, s, k // 2)
    assert y.shape == ry.shape
    tol = lambda r: 1e-2 * r.abs().max().item() + 1e-3  # noqa: E731
    assert (y.float() - ry).abs().max().item() <= tol(ry)
    assert (x.grad.float() - rdx).abs().max().item() <= tol(rdx)
    assert (m.weight.grad - rdw).abs().max().item() <= 2e-3 * rdw.abs().max().item() + 1e-3


@pytest.mark.parametrize("N,C,H,K", [(4, 64, 14, 256), (3, 256, 7, 64), (2, 128, 9, 128), (8, 512, 7, 2048)])
def test_conv1x1_plain(N, C, H, K, hip_only):
    from gaussiank_sgd_amd.ops.conv1x1 import Conv1x1
    torch.manual_seed(N * C + K)
    m = Conv1x1(C, K).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(y)
    y.backward(dy)
    ry, rdx, rdw = _ref(x, m.weight, dy)
    tol = lambda r: 1e-2 * r.abs().max().item() + 1e-3  # noqa: E731
    assert (y.float() - ry).abs().max().item() <= tol(ry)
    assert (x.grad.float() - rdx).abs().max().item() <= tol(rdx)
    assert m.weight.grad is not None and m.weight.grad.dtype == torch.float32
    assert (m.weight.grad - rdw).abs().max().item() <= 2e-3 * rdw.abs().max().item() + 1e-3


def test_conv1x1_stride2():
    from gaussiank_sgd_amd.ops.conv1x1 import Conv1x1
    m = Conv1x1(64, 128, stride=2).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(2, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert y.shape == (2, 128, 4, 4)
    ref = F.conv2d(x.to(torch.bfloat16).float(), m.weight.to(torch.bfloat16).float(), stride=2)
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


def test_conv1x1_shadow_arena_grad():
    """Through DistributedOptimizer + install_bf16_shadow the weight gradient is
    accumulated into the fp32 arena by the grad-weight GEMM; compare with the
    same model on the plain autocast path."""
    import copy
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.ops.conv1x1 import Conv1x1
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    comm.init()
    torch.manual_seed(0)
    net = torch.nn.Sequential(Conv1x1(64, 128), torch.nn.ReLU(), Conv1x1(128, 64)).cuda().to(
        memory_format=torch.channels_last)
    ref = copy.deepcopy(net)
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), named_parameters=net.named_parameters(),
                               compression=compressors["none"], is_sparse=False, density=1.0)
    install_bf16_shadow(net, opt)
    x = torch.randn(4, 64, 10, 10, device="cuda").contiguous(memory_format=torch.channels_last)
    for model in (net, ref):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = model(x)
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        err = (p.grad - q.grad).abs().max().item()
        assert err <= 2e-2 * q.grad.abs().max().item() + 1e-4, (n, err)


@pytest.fixture
def hip_only(monkeypatch):
    """Force the HIP kernels (no autotune against MIOpen) for one test."""
    from gaussiank_sgd_amd.ops import conv1x1
    monkeypatch.setattr(conv1x1, "_TUNE", False)
    monkeypatch.setattr(conv1x1, "_choices", {})


@pytest.mark.parametrize("k,s,C,K", [(1, 1, 64, 256), (3, 1, 64, 64), (3, 2, 128, 128), (1, 2, 256, 512)])
def test_conv_epilogue_bn_stats(k, s, C, K, hip_only):
    """BatchNorm statistics reduced in the conv epilogue == the BN pass's own."""
    from gaussiank_sgd_amd.ops.bn import BNAct
    from gaussiank_sgd_amd.ops.conv1x1 import FastConv2d, conv_stats
    torch.manual_seed(k * 100 + C)
    conv = FastConv2d(C, K, k, stride=s, padding=k // 2, bias=False).cuda().to(memory_format=torch.channels_last)
    bn_a = BNAct(K, act="relu").cuda()
    bn_b = BNAct(K, act="relu").cuda()
    x = torch.randn(4, C, 12, 12, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, st = conv_stats(conv, x)
        assert st is not None and st[1] > 0
        out_a = bn_a(y, stats=st)
        out_b = bn_b(y)
    assert (out_a.float() - out_b.float()).abs().max().item() <= 2e-2
    assert torch.allclose(bn_a.running_mean, bn_b.running_mean, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn_a.running_var, bn_b.running_var, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("k,s", [(3, 1), (1, 1), (3, 2)])
def test_fastconv_bias(k, s, hip_only):
    """Conv bias added in the GEMM epilogue; its gradient = sum of dY."""
    from gaussiank_sgd_amd.ops.conv1x1 import FastConv2d
    torch.manual_seed(k + s)
    m = FastConv2d(64, 128, k, stride=s, padding=k // 2, bias=True).cuda().to(memory_format=torch.channels_last)
    torch.nn.init.uniform_(m.bias, -1.0, 1.0)
    x = torch.randn(3, 64, 10, 10, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = m.bias.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, stride=s, padding=k // 2)
    yr.backward(dy.float())
    assert (y.float() - yr).abs().max().item() <= 1e-2 * yr.abs().max().item() + 1e-2
    assert (m.bias.grad - br.grad).abs().max().item() <= 1e-3 * br.grad.abs().max().item() + 1e-3
    assert (x.grad.float() - xr.grad).abs().max().item() <= 1e-2 * xr.grad.abs().max().item() + 1e-3


@pytest.mark.parametrize("cfg", [1, 4, 124, 125])
@pytest.mark.parametrize("N,C,H,W,K,k", [(2, 64, 10, 10, 128, 3), (3, 128, 9, 7, 64, 3), (2, 64, 12, 12, 256, 1),
                                         (2, 128, 9, 11, 128, 1)])
def test_conv_dgrad_s2_parity_classes(cfg, N, C, H, W, K, k):
    """Stride-2 grad-input as four stride-1 parity-class GEMMs (remapped
    epilogue; 1x1: zeros on the untouched parities) == conv_transpose."""
    g = torch.ops.gksgd
    torch.manual_seed(cfg + C + k)
    p = k // 2
    OH, OW = (H + 2 * p - k) // 2 + 1, (W + 2 * p - k) // 2 + 1
    dy = torch.randn(N, K, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, k, k, device="cuda") * 0.1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dx = torch.full((N, C, H, W), float("nan"), device="cuda").to(torch.bfloat16)
    dx = dx.contiguous(memory_format=torch.channels_last)
    z = torch.zeros(256, dtype=torch.bfloat16, device="cuda")
    g.conv_dgrad_s2(dy, w, dx, z, cfg, 0)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.float(), dy.float(), stride=2, padding=p)
    assert not torch.isnan(dx.float()).any()
    assert (dx.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 1e-3


@pytest.mark.parametrize("N,C,H,W,K", [(2, 64, 10, 10, 64), (3, 128, 7, 9, 64), (2, 64, 14, 14, 192),
                                       (1, 64, 30, 12, 128), (2, 128, 5, 40, 128)])
def test_conv3_wgrad_tap_parallel(N, C, H, W, K):
    """Tap-parallel 3x3 grad-weight (wgrad3.hip) == PyTorch's, accumulated into
    a pre-filled fp32 output in either memory format."""
    g = torch.ops.gksgd
    torch.manual_seed(N + C + H + K)
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for cl in (True, False):
        out = torch.full((K, C, 3, 3), 0.25, device="cuda")
        if cl:
            out = out.contiguous(memory_format=torch.channels_last)
        part = torch.empty(int(g.wgrad3_ws(N, H, W, C, K)), device="cuda")
        g.conv3_wgrad(dy, x, out, part, torch.zeros(256, dtype=torch.bfloat16, device=x.device))
        torch.cuda.synchronize()
        ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, 3, 3), dy.float(), padding=1) + 0.25
        err = (out - ref).abs().max().item()
        assert err <= 2e-3 * (ref - 0.25).abs().max().item() + 1e-3, (cl, err)
