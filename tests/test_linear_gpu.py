"""FastLinear (ops/linear.py, csrc/kernels/linear.hip): autotuned MFMA GEMM
linear layers with the bias gradient / GELU backward in one fused HIP column
pass, vs an fp32 PyTorch reference; plain and through the bf16-shadow /
direct-to-arena path of the DistributedOptimizer."""
import copy

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


@pytest.fixture
def hip_only(monkeypatch):
    """Force the HIP GEMM kernels (no autotune against hipBLASLt) for one test."""
    from gaussiank_sgd_amd.ops import conv1x1
    monkeypatch.setattr(conv1x1, "_TUNE", False)
    monkeypatch.setattr(conv1x1, "_choices", {})


@pytest.mark.parametrize("M,N", [(1000, 264), (37, 8), (4096, 768), (257, 3072), (4480, 10000)])
def test_colsum_acc(M, N):
    from gaussiank_sgd_amd.ops.linear import bias_grad_acc_
    torch.manual_seed(M + N)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    db = torch.randn(N, device="cuda")
    ref = db.double() + dy.double().sum(0)
    bias_grad_acc_(db, dy)
    assert (db.double() - ref).abs().max().item() <= 1e-5 * M + 1e-4


@pytest.mark.parametrize("M,N", [(1000, 264), (512, 3072), (3, 64)])
@pytest.mark.parametrize("with_db", [True, False])
def test_gelu_backward_colsum(M, N, with_db):
    from gaussiank_sgd_amd.ops.linear import gelu_backward_
    torch.manual_seed(M + N)
    pre = (torch.randn(M, N, device="cuda") * 2).to(torch.bfloat16)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    db = torch.zeros(N, device="cuda") if with_db else None
    dpre = gelu_backward_(dy, pre, db)
    ref = torch.ops.aten.gelu_backward(dy.float(), pre.float())
    assert dpre.dtype == torch.bfloat16
    assert (dpre.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    if with_db:
        assert (db.double() - dpre.double().sum(0)).abs().max().item() <= 1e-5 * M + 1e-4


def _check_linear(M, K, N, act, bias):
    from gaussiank_sgd_amd.ops.linear import FastLinear
    torch.manual_seed(M + K + N)
    m = FastLinear(K, N, bias=bias).cuda()
    if bias:
        torch.nn.init.uniform_(m.bias, -1.0, 1.0)
    x = torch.randn(3, M, K, device="cuda").to(torch.bfloat16).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x, act=act)
    assert y.dtype == torch.bfloat16 and y.shape == (3, M, N)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = m.bias.detach().float().requires_grad_(True) if bias else None
    yr = F.linear(xr, wr, br)
    if act == "gelu":
        yr = F.gelu(yr)
    yr.backward(dy.float())
    tol = lambda r: 2e-2 * r.abs().max().item() + 1e-3  # noqa: E731
    assert (y.float() - yr).abs().max().item() <= tol(yr)
    assert (x.grad.float() - xr.grad).abs().max().item() <= tol(xr.grad)
    assert m.weight.grad is not None and m.weight.grad.dtype == torch.float32
    assert (m.weight.grad - wr.grad).abs().max().item() <= tol(wr.grad)
    if bias:
        assert (m.bias.grad - br.grad).abs().max().item() <= tol(br.grad)


@pytest.mark.parametrize("M,K,N,act,bias", [(300, 128, 192, None, True), (517, 64, 256, "gelu", True),
                                            (128, 256, 64, None, False), (200, 768, 2304, None, True)])
def test_fastlinear_hip_vs_fp32(M, K, N, act, bias, hip_only):
    _check_linear(M, K, N, act, bias)


@pytest.mark.parametrize("M,K,N,act", [(300, 128, 192, "gelu"), (100, 1500, 1000, None)])
def test_fastlinear_autotuned_vs_fp32(M, K, N, act):
    """Autotune on (HIP kernels vs hipBLASLt), and a non-multiple-of-64 layer
    (hipBLASLt GEMMs + the fused bias pass)."""
    _check_linear(M, K, N, act, True)


def test_fastlinear_shadow_arena_grad():
    """Through DistributedOptimizer + install_bf16_shadow the weight / bias
    gradients go straight into the fp32 arena; compare with the same model
    off the shadow path."""
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.ops.linear import FastLinear
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = FastLinear(128, 256)
            self.b = FastLinear(256, 64)

        def forward(self, x):
            return self.b(self.a(x, act="gelu"))
    comm.init()
    torch.manual_seed(0)
    net = Net().cuda()
    ref = copy.deepcopy(net)
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), named_parameters=net.named_parameters(),
                               compression=compressors["none"], is_sparse=False, density=1.0)
    install_bf16_shadow(net, opt)
    x = torch.randn(200, 128, device="cuda")
    for model in (net, ref):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = model(x)
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        err = (p.grad - q.grad).abs().max().item()
        assert err <= 2e-2 * q.grad.abs().max().item() + 1e-4, (n, err)


def test_bert_tiny_step_bf16(cuda):
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    from gaussiank_sgd_amd.train import DLTrainer
    torch.manual_seed(0)
    comm.init()
    t = DLTrainer(0, 1, dnn="bert_tiny", dataset="wikipedia", batch_size=8, lr=0.05, device="cuda", amp="bf16",
                  learnable_data=True, data_pool=1)
    opt = DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                               compression=compressors["gaussian"], is_sparse=True, density=0.01,
                               compress_single_rank=True, density_warmup=False)
    install_bf16_shadow(t.net, opt)
    t.update_optimizer(opt)
    losses = []
    for _ in range(20):
        opt.zero_grad()
        t.train(1)
        t.update_model()
        losses.append(t.current_loss())
    assert all(v == v for v in losses)
    # the reference's Gaussian-k may select nothing from a tiny bucket on a given
    # step (a 128-element LayerNorm bucket at density 0.01 has k = 2): check
    # that the step as a whole sent gradients
    assert sum(int(b.bufs.record[0]) for b in opt.arena.buckets) > 0
    assert min(losses[-5:]) < losses[0]



# ---- fp32 path (no autocast: the reference's precision) --------------------
@pytest.mark.parametrize("M,N", [(1000, 264), (37, 8), (4096, 768)])
def test_colsum_acc_f32(M, N):
    from gaussiank_sgd_amd.ops.linear import bias_grad_acc_
    torch.manual_seed(M + N)
    dy = torch.randn(M, N, device="cuda")
    db = torch.randn(N, device="cuda")
    ref = db.double() + dy.double().sum(0)
    bias_grad_acc_(db, dy)
    assert (db.double() - ref).abs().max().item() <= 2e-6 * M + 1e-5


@pytest.mark.parametrize("M,N", [(1000, 264), (512, 3072)])
def test_gelu_backward_colsum_f32(M, N):
    from gaussiank_sgd_amd.ops.linear import gelu_backward_
    torch.manual_seed(M + N)
    pre = torch.randn(M, N, device="cuda") * 2
    dy = torch.randn(M, N, device="cuda")
    db = torch.zeros(N, device="cuda")
    dpre = gelu_backward_(dy, pre, db)
    ref = torch.ops.aten.gelu_backward(dy.double(), pre.double())
    assert dpre.dtype == torch.float32
    assert (dpre.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert (db.double() - ref.sum(0)).abs().max().item() <= 2e-6 * M + 1e-5


def _check_linear_f32(M, K, N, act, bias):
    from gaussiank_sgd_amd.ops import conv1x1
    from gaussiank_sgd_amd.ops.linear import FastLinear
    torch.manual_seed(M + K + N)
    m = FastLinear(K, N, bias=bias).cuda()
    if bias:
        torch.nn.init.uniform_(m.bias, -1.0, 1.0)
    x = torch.randn(3, M, K, device="cuda").requires_grad_(True)
    y = m(x, act=act)
    assert y.dtype == torch.float32 and y.shape == (3, M, N)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().double().requires_grad_(True)
    wr = m.weight.detach().double().requires_grad_(True)
    br = m.bias.detach().double().requires_grad_(True) if bias else None
    yr = F.linear(xr, wr, br)
    if act == "gelu":
        yr = F.gelu(yr)
    yr.backward(dy.double())
    tol = lambda r: 1e-5 * r.abs().max().item() + 1e-5  # noqa: E731
    assert (y.double() - yr).abs().max().item() <= tol(yr)
    assert (x.grad.double() - xr.grad).abs().max().item() <= tol(xr.grad)
    assert (m.weight.grad.double() - wr.grad).abs().max().item() <= tol(wr.grad)
    if bias:
        assert (m.bias.grad.double() - br.grad).abs().max().item() <= tol(br.grad)
    keys = [k for k in conv1x1.tuned_choices() if k[0].startswith("lin_") and "f32" in k]
    assert keys, "fp32 linear path not taken"


@pytest.mark.parametrize("M,K,N,act,bias", [(300, 128, 192, None, True), (517, 64, 256, "gelu", True),
                                            (128, 256, 64, None, False), (200, 768, 2304, None, True)])
def test_fastlinear_f32_hip_vs_fp64(M, K, N, act, bias, hip_only):
    _check_linear_f32(M, K, N, act, bias)


def test_fastlinear_f32_autotuned_and_direct_arena():
    """Autotuned fp32 linears; through DistributedOptimizer + install_direct_grads
    the fp32 weight / bias gradients go straight into the arena."""
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.ops.linear import FastLinear
    from gaussiank_sgd_amd.parallel import comm, install_direct_grads
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    _check_linear_f32(300, 128, 192, "gelu", True)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = FastLinear(128, 256)
            self.b = FastLinear(256, 64)

        def forward(self, x):
            return self.b(self.a(x, act="gelu"))
    comm.init()
    torch.manual_seed(0)
    net = Net().cuda()
    ref = copy.deepcopy(net)
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), named_parameters=net.named_parameters(),
                               compression=compressors["none"], is_sparse=False, density=1.0)
    assert install_direct_grads(net, opt) == 4
    x = torch.randn(200, 128, device="cuda")
    for model in (net, ref):
        model(x).square().mean().backward()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        err = (p.grad - q.grad).abs().max().item()
        assert err <= 1e-5 * q.grad.abs().max().item() + 1e-6, (n, err)


@pytest.mark.parametrize("M,K,N", [(448, 1500, 1000), (130, 200, 104), (64, 1536, 10000)])
@pytest.mark.parametrize("bias", [True, False])
def test_fp32_linear_padded_operands_vs_fp64(hip_only, M, K, N, bias):
    """fp32 FastLinear with K / N not multiples of 64 (the LSTM's 1500-unit
    layers and 10k softmax): the HIP kernels on zero-padded operand copies
    (forward, grad-input, grad-weight into a padded scratch) against fp64."""
    from gaussiank_sgd_amd.ops import conv1x1
    from gaussiank_sgd_amd.ops.linear import FastLinear
    torch.manual_seed(M + K + N)
    m = FastLinear(K, N, bias=bias).cuda()
    x = torch.randn(M, K, device="cuda", requires_grad=True)
    y = m(x)
    assert y.shape == (M, N)
    # the padded HIP path ran (its tuner keys carry "pad")
    assert any(k[0] == "lin_fwd" and k[-1] == "pad" for k in conv1x1._choices)
    gy = torch.randn(M, N, device="cuda")
    (y * gy).sum().backward()
    assert any(k[0] == "lin_dgrad" and k[-1] == "pad" for k in conv1x1._choices)
    assert any(k[0] == "lin_wgrad" and k[-1] == "pad" for k in conv1x1._choices)
    xd = x.detach().double().requires_grad_(True)
    wd = m.weight.detach().double().requires_grad_(True)
    bd = m.bias.detach().double().requires_grad_(True) if bias else None
    yd = F.linear(xd, wd, bd)
    (yd * gy.double()).sum().backward()

    def close(a, b):
        return (a.double() - b).abs().max().item() <= 2e-5 * b.abs().max().item() + 1e-6
    assert close(y.detach(), yd.detach())
    assert close(x.grad, xd.grad)
    assert close(m.weight.grad, wd.grad)
    if bias:
        assert close(m.bias.grad, bd.grad)
