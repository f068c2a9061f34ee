"""GkLSTM (ops/lstm.py, csrc/kernels/lstm.hip): the fused HIP LSTM cells vs
their fp32 PyTorch reference, the bf16 layer vs an fp32 nn.LSTM, and the
bf16-shadow / direct-to-arena gradients vs the plain path."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error


@pytest.mark.parametrize("B,H", [(128, 1500), (3, 40)])
def test_lstm_cells_vs_reference(B, H):
    from gaussiank_sgd_amd.ops.lstm import _cell_bwd_ref, _cell_fwd_ref
    g = torch.ops.gksgd
    torch.manual_seed(B + H)
    xg = (torch.randn(B, 4 * H, device="cuda") * 2).to(torch.bfloat16)
    hg = torch.randn(B, 4 * H, device="cuda").to(torch.bfloat16)
    cp = torch.randn(B, H, device="cuda")
    outs = [torch.empty(B, H, device="cuda"), torch.empty(B, H, device="cuda", dtype=torch.bfloat16),
            torch.empty(B, 4 * H, device="cuda")]
    refs = [torch.empty_like(o, dtype=torch.float32) for o in outs]
    g.lstm_cell_fwd(xg, hg, cp, *outs)
    _cell_fwd_ref(xg, hg, cp, *refs)
    for o, r in zip(outs, refs):
        assert (o.float() - r).abs().max().item() <= 1e-2 * r.abs().max().item() + 1e-5
    c, _, gates = refs
    dout = torch.randn(B, H, device="cuda").to(torch.bfloat16)
    dh = torch.randn(B, H, device="cuda").to(torch.bfloat16)
    dcn = torch.randn(B, H, device="cuda")
    dG = torch.empty(B, 4 * H, device="cuda", dtype=torch.bfloat16)
    dcp = torch.empty(B, H, device="cuda")
    rG = torch.empty(B, 4 * H, device="cuda")
    rcp = torch.empty(B, H, device="cuda")
    g.lstm_cell_bwd(dout, dh, dcn, gates, c, cp, dG, dcp)
    _cell_bwd_ref(dout, dh, dcn, gates, c, cp, rG, rcp)
    assert (dG.float() - rG).abs().max().item() <= 1e-2 * rG.abs().max().item()
    assert (dcp - rcp).abs().max().item() <= 1e-5 * rcp.abs().max().item() + 1e-6
    g.lstm_cell_bwd(None, None, None, gates, c, cp, dG, dcp)
    assert dG.float().abs().max().item() == 0.0


def test_gklstm_bf16_vs_fp32_nn_lstm():
    from gaussiank_sgd_amd.ops.lstm import GkLSTM
    torch.manual_seed(0)
    T, B, I, H, L = 35, 16, 256, 320, 2
    ref = torch.nn.LSTM(I, H, num_layers=L).cuda()
    m = GkLSTM(I, H, num_layers=L).cuda()
    m.load_state_dict(ref.state_dict())
    x = torch.randn(T, B, I, device="cuda")
    xa = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, (hn, cn) = m(xa)
    assert y.dtype == torch.bfloat16
    xr = x.clone().requires_grad_(True)
    torch.backends.cudnn.enabled = False     # fp32 native LSTM as the reference
    try:
        yr, (hnr, cnr) = ref(xr)
    finally:
        torch.backends.cudnn.enabled = True
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    tol = lambda r: 3e-2 * r.abs().max().item() + 1e-3  # noqa: E731
    assert (y.float() - yr).abs().max().item() <= tol(yr)
    assert (cn.float() - cnr).abs().max().item() <= tol(cnr)
    assert (xa.grad - xr.grad).abs().max().item() <= tol(xr.grad)
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert (p.grad - q.grad).abs().max().item() <= tol(q.grad), n


def test_gklstm_shadow_arena_grads():
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.ops.lstm import GkLSTM
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    comm.init()
    torch.manual_seed(1)
    net = GkLSTM(128, 192, num_layers=2).cuda()
    ref = copy.deepcopy(net)
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), named_parameters=net.named_parameters(),
                               compression=compressors["none"], is_sparse=False, density=1.0)
    install_bf16_shadow(net, opt)
    assert len(net._gk_shadow) == 8
    x = torch.randn(12, 8, 128, device="cuda")
    for model in (net, ref):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y, _ = model(x)
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        err = (p.grad - q.grad).abs().max().item()
        assert err <= 2e-2 * q.grad.abs().max().item() + 1e-5, (n, err)


def test_ptb_lstm_step_bf16(cuda):
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    from gaussiank_sgd_amd.train import DLTrainer
    torch.manual_seed(0)
    comm.init()
    t = DLTrainer(0, 1, dnn="lstm", dataset="ptb", batch_size=16, lr=1.0, device="cuda", amp="bf16",
                  learnable_data=True, data_pool=1)
    opt = DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                               compression=compressors["gaussian"], is_sparse=True, density=0.01,
                               compress_single_rank=True, density_warmup=False)
    install_bf16_shadow(t.net, opt)
    t.update_optimizer(opt)
    hidden = None
    losses = []
    for _ in range(8):
        opt.zero_grad()
        _, hidden = t.train(1, hidden=hidden)
        opt.synchronize()
        opt.clip_grad_norm_(0.25)
        t.update_model()
        losses.append(t.current_loss())
    assert all(v == v for v in losses) and losses[-1] < losses[0]
    assert not torch.isnan(opt.arena.weights).any()
    # per-tensor buckets: a small bucket may legitimately send nothing in a step
    assert sum(int(b.bufs.record[0]) for b in opt.arena.buckets) > 0
