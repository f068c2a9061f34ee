"""1x1-convolution MFMA GEMMs (ops/csrc/kernels/gemm.hip) vs an fp32 PyTorch
reference: every tile configuration, resident / streamed weight panels,
M tails, row strides and grad-weight splits."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error
    return torch.ops.gksgd


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (777, 128, 192), (2048, 512, 128),
                                   (513, 192, 320), (300, 256, 1024)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 11, 21, 13, 23, 5, 6, 7, 125, 126, 127, 15, 211, 213, 222, 224])
def test_gemm_nt(g, M, N, K, cfg):
    torch.manual_seed(M + N + K)
    A = _rand(M, K)
    B = _rand(N, K, scale=K ** -0.5)
    C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    g.gemm_nt(A, B, C, cfg, 0)
    ref = A.float() @ B.float().t()
    err = (C.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err


def test_gemm_nt_strided_rows_and_grid(g):
    torch.manual_seed(1)
    A_big = _rand(900, 256)
    A = A_big[:, 64:192]                 # row stride 256, K = 128
    B = _rand(128, 128, scale=0.1)
    C_big = torch.zeros(900, 384, device="cuda", dtype=torch.bfloat16)
    C = C_big[:, 128:256]
    for mb in (1, 3, 0):
        C_big.zero_()
        g.gemm_nt(A, B, C, 0, mb)
        ref = A.float() @ B.float().t()
        assert (C.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
        assert C_big[:, :128].abs().max().item() == 0 and C_big[:, 256:].abs().max().item() == 0


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 256, 64), (777, 128, 192), (2500, 512, 256),
                                   (130, 64, 128), (5000, 128, 512), (3001, 256, 256)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8, 21, 27, 9, 29, 101, 121, 102, 122])
@pytest.mark.parametrize("splits", [0, 1, 7])
def test_gemm_tn_acc(g, M, N, K, cfg, splits):
    torch.manual_seed(M * 3 + N + K)
    G = _rand(M, N)
    X = _rand(M, K)
    W0 = torch.randn(N, K, device="cuda")
    W = W0.clone()
    g.gemm_tn_acc(G, X, W, cfg, splits)
    ref = W0 + G.float().t() @ X.float()
    err = (W - ref).abs().max().item()
    assert err <= 1e-4 * (G.float().abs().t() @ X.float().abs()).max().item() + 1e-4, err


def _conv_case(N, C, H, Co, k, s, p):
    x = _rand(N, C, H, H).contiguous(memory_format=torch.channels_last)
    w = _rand(Co, C, k, k, scale=(C * k * k) ** -0.5).contiguous(memory_format=torch.channels_last)
    return x, w


@pytest.mark.parametrize("N,C,H,Co,k,s,p", [(2, 64, 9, 64, 3, 1, 1), (3, 128, 7, 64, 3, 2, 1), (2, 64, 14, 128, 3, 2, 1),
                                            (2, 128, 5, 256, 1, 1, 0), (1, 64, 11, 192, 3, 1, 1)])
@pytest.mark.parametrize("cfg", [0, 1, 3, 22, 124, 5, 126, 7, 214, 221])
def test_conv_nt(g, N, C, H, Co, k, s, p, cfg):
    import torch.nn.functional as F
    torch.manual_seed(N + C + H + Co)
    x, w = _conv_case(N, C, H, Co, k, s, p)
    zero = torch.zeros(64, device="cuda", dtype=torch.bfloat16)
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=p)
    y = torch.full(ref.shape, float("nan"), device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    g.conv_nt(x, w, y, zero, s, p, cfg, 0)
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 1e-3


@pytest.mark.parametrize("N,C,H,Co,k,s,p", [(2, 64, 9, 64, 3, 1, 1), (3, 128, 7, 64, 3, 2, 1), (2, 64, 14, 128, 3, 2, 1),
                                            (2, 128, 5, 256, 1, 1, 0)])
@pytest.mark.parametrize("cfg,splits", [(0, 0), (1, 3), (4, 0), (25, 0), (2, 7), (7, 0), (8, 2), (23, 0), (29, 0),
                                        (121, 3), (102, 0)])
def test_conv_tn_acc(g, N, C, H, Co, k, s, p, cfg, splits):
    import torch.nn.functional as F
    torch.manual_seed(N * 7 + C + H + Co)
    x, w = _conv_case(N, C, H, Co, k, s, p)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=p)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    zero = torch.zeros(64, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(Co, C, k, k, device="cuda").contiguous(memory_format=torch.channels_last)
    g.conv_tn_acc(dy, x, out, zero, s, p, cfg, splits)
    err = (out - wr.grad).abs().max().item()
    assert err <= 1e-3 * wr.grad.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("cfg", [211, 213, 222, 224, 13, 124])
@pytest.mark.parametrize("mb", [1, 3, 7])
def test_gemm_nt_deep_pipeline_few_blocks(g, cfg, mb):
    """Few persistent blocks walking many tiles: every LDS stage of the 3- and
    4-stage pipelines is reused many times (partial last tile included)."""
    torch.manual_seed(cfg + mb)
    M, N, K = 5000 + 37, 256, 128
    A = _rand(M, K)
    B = _rand(N, K, scale=K ** -0.5)
    C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    g.gemm_nt(A, B, C, cfg, mb)
    ref = A.float() @ B.float().t()
    assert (C.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 1e-3
