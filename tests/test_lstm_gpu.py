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
    Hp = (H + 63) // 64 * 64
    # two fp32 K-slice partials whose sum is hg, laid out in 64-padded gate columns
    P = torch.zeros(2, B, 4, Hp, device="cuda")
    P[0, :, :, :H] = hg.float().view(B, 4, H) * 0.25
    P[1, :, :, :H] = hg.float().view(B, 4, H) * 0.75
    P = P.view(2, B, 4 * Hp)
    h_pad = torch.full((B, Hp), 7.0, device="cuda", dtype=torch.bfloat16)
    cp = torch.randn(B, H, device="cuda")
    outs = [torch.empty(B, H, device="cuda"), torch.empty(B, H, device="cuda", dtype=torch.bfloat16),
            torch.empty(B, 4 * H, device="cuda")]
    refs = [torch.empty_like(o, dtype=torch.float32) for o in outs]
    g.lstm_cell_fwd(xg, None, P, 2, cp, outs[0], outs[1], h_pad, outs[2])
    _cell_fwd_ref(xg, hg, cp, *refs)
    for o, r in zip(outs, refs):
        assert (o.float() - r).abs().max().item() <= 1e-2 * r.abs().max().item() + 1e-5
    assert torch.equal(h_pad[:, :H], outs[1])
    assert (h_pad[:, H:].float() == 7.0).all()
    c, _, gates = refs
    dout = torch.randn(B, H, device="cuda").to(torch.bfloat16)
    dh = torch.randn(B, H, device="cuda").to(torch.bfloat16)
    dcn = torch.randn(B, H, device="cuda")
    dG = torch.empty(B, 4 * H, device="cuda", dtype=torch.bfloat16)
    dcp = torch.empty(B, H, device="cuda")
    rG = torch.empty(B, 4 * H, device="cuda")
    rcp = torch.empty(B, H, device="cuda")
    Pb = torch.zeros(3, B, Hp, device="cuda")
    for s in range(3):
        Pb[s, :, :H] = dh.float() / 3
    dG_pad = torch.zeros(B, 4 * Hp, device="cuda", dtype=torch.bfloat16)
    g.lstm_cell_bwd(dout, None, Pb, 3, dcn, gates, c, cp, dG, dG_pad, dcp)
    _cell_bwd_ref(dout, dh, dcn, gates, c, cp, rG, rcp)
    assert (dG.float() - rG).abs().max().item() <= 1e-2 * rG.abs().max().item()
    assert (dcp - rcp).abs().max().item() <= 1e-5 * rcp.abs().max().item() + 1e-6
    assert torch.equal(dG_pad.view(B, 4, Hp)[:, :, :H], dG.view(B, 4, H))
    assert (dG_pad.view(B, 4, Hp)[:, :, H:] == 0).all()
    g.lstm_cell_bwd(None, None, None, 1, None, gates, c, cp, dG, None, dcp)
    assert dG.float().abs().max().item() == 0.0
    # bf16 hg / dh_rec inputs (the hipBLASLt step-GEMM path)
    outs2 = [torch.empty_like(o) for o in outs]
    g.lstm_cell_fwd(xg, hg, None, 0, cp, outs2[0], outs2[1], None, outs2[2])
    for o, r in zip(outs2, refs):
        assert (o.float() - r).abs().max().item() <= 1e-2 * r.abs().max().item() + 1e-5
    g.lstm_cell_bwd(dout, dh, None, 0, dcn, gates, c, cp, dG, None, dcp)
    assert (dG.float() - rG).abs().max().item() <= 1e-2 * rG.abs().max().item()
    assert (dcp - rcp).abs().max().item() <= 1e-5 * rcp.abs().max().item() + 1e-6
    g.lstm_cell_bwd(None, None, None, 0, None, gates, c, cp, dG, None, dcp)
    assert dG.float().abs().max().item() == 0.0


@pytest.mark.parametrize("M,N,K,S", [(128, 6144, 1536, 4), (20, 1536, 6144, 16), (3, 256, 64, 1), (200, 128, 256, 2)])
def test_lstm_rec_gemm_vs_fp32(M, N, K, S):
    g = torch.ops.gksgd
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    Bm = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    P = torch.full((S, M, N), float("nan"), device="cuda")
    g.lstm_rec_gemm(A, Bm, P, S)
    ref = A.float() @ Bm.float().t()
    got = P.sum(0)
    assert (got - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-3
    # every slice is its own K range
    ks = K // S
    ref0 = A[:, :ks].float() @ Bm[:, :ks].float().t()
    assert (P[0] - ref0).abs().max().item() <= 1e-4 * ref0.abs().max().item() + 1e-3


@pytest.mark.parametrize("fwd_max,bwd_max", [(1 << 30, 1 << 30), (0, 0), (0, 1 << 30)],
                         ids=["splitk", "hipblaslt", "mixed"])
def test_gklstm_bf16_vs_fp32_nn_lstm(monkeypatch, fwd_max, bwd_max):
    from gaussiank_sgd_amd.ops import lstm as L_
    from gaussiank_sgd_amd.ops.lstm import GkLSTM
    monkeypatch.setitem(L_.SPLITK_MAX_BATCH, "fwd", fwd_max)
    monkeypatch.setitem(L_.SPLITK_MAX_BATCH, "bwd", bwd_max)
    torch.manual_seed(0)
    T, B, I, H, L = 35, 16, 256, 320, 2
    ref = torch.nn.LSTM(I, H, num_layers=L).cuda()
    m = GkLSTM(I, H, num_layers=L).cuda()
    m.load_state_dict(ref.state_dict())
    x = torch.randn(T, B, I, device="cuda")
    h0 = torch.randn(L, B, H, device="cuda") * 0.5
    c0 = torch.randn(L, B, H, device="cuda") * 0.5
    xa, ha, ca = (t.clone().requires_grad_(True) for t in (x, h0, c0))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, (hn, cn) = m(xa, (ha, ca))
    assert y.dtype == torch.bfloat16
    xr, hr, cr = (t.clone().requires_grad_(True) for t in (x, h0, c0))
    torch.backends.cudnn.enabled = False     # fp32 native LSTM as the reference
    try:
        yr, (hnr, cnr) = ref(xr, (hr, cr))
    finally:
        torch.backends.cudnn.enabled = True
    gy = torch.randn_like(yr)
    ghn = torch.randn_like(hnr)
    (y.float() * gy).sum().add_((hn.float() * ghn).sum()).backward()
    (yr * gy).sum().add_((hnr * ghn).sum()).backward()
    tol = lambda r: 3e-2 * r.abs().max().item() + 1e-3  # noqa: E731
    assert (y.float() - yr).abs().max().item() <= tol(yr)
    assert (cn.float() - cnr).abs().max().item() <= tol(cnr)
    assert (xa.grad - xr.grad).abs().max().item() <= tol(xr.grad)
    assert (ha.grad - hr.grad).abs().max().item() <= tol(hr.grad)
    assert (ca.grad - cr.grad).abs().max().item() <= tol(cr.grad)
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


# ---- fp32 path (no autocast: the reference's precision) --------------------

@pytest.mark.parametrize("B,H", [(128, 1500), (3, 40)])
def test_lstm_cells_f32_vs_reference(B, H):
    """fp32 cell kernels (xg / hg / h / dG in fp32) vs the fp32 PyTorch cells."""
    from gaussiank_sgd_amd.ops.lstm import _cell_bwd_ref, _cell_fwd_ref
    g = torch.ops.gksgd
    torch.manual_seed(B + H + 1)
    xg = torch.randn(B, 4 * H, device="cuda") * 2
    hg = torch.randn(B, 4 * H, device="cuda")
    Hp = (H + 63) // 64 * 64
    P = torch.zeros(2, B, 4, Hp, device="cuda")
    P[0, :, :, :H] = hg.view(B, 4, H) * 0.25
    P[1, :, :, :H] = hg.view(B, 4, H) * 0.75
    P = P.view(2, B, 4 * Hp)
    h_pad = torch.full((B, Hp), 7.0, device="cuda")
    cp = torch.randn(B, H, device="cuda")
    outs = [torch.empty(B, H, device="cuda"), torch.empty(B, H, device="cuda"), torch.empty(B, 4 * H, device="cuda")]
    refs = [torch.empty_like(o) for o in outs]
    g.lstm_cell_fwd(xg, None, P, 2, cp, outs[0], outs[1], h_pad, outs[2])
    _cell_fwd_ref(xg, hg, cp, *refs)
    for o, r in zip(outs, refs):
        assert (o - r).abs().max().item() <= 1e-5 * r.abs().max().item() + 1e-6
    assert torch.equal(h_pad[:, :H], outs[1])
    assert (h_pad[:, H:] == 7.0).all()
    c, _, gates = refs
    dout = torch.randn(B, H, device="cuda")
    dh = torch.randn(B, H, device="cuda")
    dcn = torch.randn(B, H, device="cuda")
    dG = torch.empty(B, 4 * H, device="cuda")
    dcp = torch.empty(B, H, device="cuda")
    rG = torch.empty(B, 4 * H, device="cuda")
    rcp = torch.empty(B, H, device="cuda")
    Pb = torch.zeros(3, B, Hp, device="cuda")
    for s in range(3):
        Pb[s, :, :H] = dh / 3
    dG_pad = torch.zeros(B, 4 * Hp, device="cuda")
    g.lstm_cell_bwd(dout, None, Pb, 3, dcn, gates, c, cp, dG, dG_pad, dcp)
    _cell_bwd_ref(dout, dh, dcn, gates, c, cp, rG, rcp)
    assert (dG - rG).abs().max().item() <= 1e-5 * rG.abs().max().item() + 1e-6
    assert (dcp - rcp).abs().max().item() <= 1e-5 * rcp.abs().max().item() + 1e-6
    assert torch.equal(dG_pad.view(B, 4, Hp)[:, :, :H], dG.view(B, 4, H))
    assert (dG_pad.view(B, 4, Hp)[:, :, H:] == 0).all()
    # fp32 hg / dh_rec inputs (the unpadded step-GEMM path)
    outs2 = [torch.empty_like(o) for o in outs]
    g.lstm_cell_fwd(xg, hg, None, 0, cp, outs2[0], outs2[1], None, outs2[2])
    for o, r in zip(outs2, refs):
        assert (o - r).abs().max().item() <= 1e-5 * r.abs().max().item() + 1e-6
    g.lstm_cell_bwd(dout, dh, None, 0, dcn, gates, c, cp, dG, None, dcp)
    assert (dG - rG).abs().max().item() <= 1e-5 * rG.abs().max().item() + 1e-6
    g.lstm_cell_bwd(None, None, None, 0, None, gates, c, cp, dG, None, dcp)
    assert dG.abs().max().item() == 0.0
    with pytest.raises(RuntimeError):    # mixed storage dtypes are refused
        g.lstm_cell_fwd(xg, hg.to(torch.bfloat16), None, 0, cp, outs2[0], outs2[1], None, outs2[2])


@pytest.mark.parametrize("M,N,K,S", [(128, 6144, 1536, 4), (20, 1536, 6144, 16), (3, 256, 64, 1), (200, 128, 256, 2)])
def test_lstm_rec_gemm_f32_vs_fp64(M, N, K, S):
    g = torch.ops.gksgd
    torch.manual_seed(M + N + K + 1)
    A = torch.randn(M, K, device="cuda")
    Bm = torch.randn(N, K, device="cuda")
    P = torch.full((S, M, N), float("nan"), device="cuda")
    g.lstm_rec_gemm(A, Bm, P, S)
    ref = A.double() @ Bm.double().t()
    scale = (A.double().abs() @ Bm.double().abs().t()).max().item()
    assert (P.double().sum(0) - ref).abs().max().item() <= 2e-6 * scale
    ks = K // S
    ref0 = A[:, :ks].double() @ Bm[:, :ks].double().t()
    assert (P[0].double() - ref0).abs().max().item() <= 2e-6 * scale


@pytest.mark.parametrize("M,N,K,S", [(128, 6144, 1536, 4), (128, 1536, 6144, 16), (20, 6144, 1536, 8),
                                     (20, 1536, 6144, 16), (3, 256, 64, 1), (200, 128, 256, 2)])
def test_lstm_rec_gemm_x6_vs_fp64(M, N, K, S):
    """bf16x6 split-K step GEMM (fp32 A split in registers, B as three exact
    bf16 planes): every K slice against fp64, and no less accurate than the
    fp32-MFMA kernel on the same operands."""
    from gaussiank_sgd_amd.ops.lstm import split3
    g = torch.ops.gksgd
    torch.manual_seed(M + N + K + 7)
    A = torch.randn(M, K, device="cuda")
    Bm = torch.randn(N, K, device="cuda") / K ** 0.5
    B3 = split3(Bm)
    assert torch.equal(B3[0].float() + B3[1].float() + B3[2].float(), Bm)   # the split is exact
    P = torch.full((S, M, N), float("nan"), device="cuda")
    g.lstm_rec_gemm_x6(A, B3, P, S)
    Pf = torch.full((S, M, N), float("nan"), device="cuda")
    g.lstm_rec_gemm(A, Bm, Pf, S)
    ref = A.double() @ Bm.double().t()
    scale = (A.double().abs() @ Bm.double().abs().t()).max().item()
    err = (P.double().sum(0) - ref).abs()
    assert err.max().item() <= 2e-6 * scale
    ks = K // S
    ref0 = A[:, :ks].double() @ Bm[:, :ks].double().t()
    assert (P[0].double() - ref0).abs().max().item() <= 2e-6 * scale
    e_x6 = float((P.double().sum(0) - ref).norm() / ref.norm())
    e_f32 = float((Pf.double().sum(0) - ref).norm() / ref.norm())
    assert e_x6 <= 1.05 * e_f32 + 1e-12, (e_x6, e_f32)


@pytest.mark.parametrize("fwd_max,bwd_max,x6", [(1 << 30, 1 << 30, False), (0, 0, False), (0, 1 << 30, False),
                                                (0, 0, True), (None, None, False)],
                         ids=["splitk", "blas", "mixed", "x6", "tuned"])
def test_gklstm_f32_vs_fp64_nn_lstm(monkeypatch, fwd_max, bwd_max, x6):
    """fp32 GkLSTM (HIP step GEMM -- fp32 MFMA or bf16x6 -- + fp32 cells) vs an fp64 nn.LSTM."""
    from gaussiank_sgd_amd.ops import lstm as L_
    from gaussiank_sgd_amd.ops.lstm import GkLSTM
    monkeypatch.setitem(L_.SPLITK_MAX_BATCH, "fwd", fwd_max)
    monkeypatch.setitem(L_.SPLITK_MAX_BATCH, "bwd", bwd_max)
    monkeypatch.setattr(L_, "_X6", x6)
    torch.manual_seed(0)
    T, B, I, H, L = 35, 16, 256, 320, 2
    ref = torch.nn.LSTM(I, H, num_layers=L).cuda().double()
    m = GkLSTM(I, H, num_layers=L).cuda()
    m.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    x = torch.randn(T, B, I, device="cuda")
    h0 = torch.randn(L, B, H, device="cuda") * 0.5
    c0 = torch.randn(L, B, H, device="cuda") * 0.5
    xa, ha, ca = (t.clone().requires_grad_(True) for t in (x, h0, c0))
    y, (hn, cn) = m(xa, (ha, ca))
    assert y.dtype == torch.float32
    xr, hr, cr = (t.double().requires_grad_(True) for t in (x, h0, c0))
    torch.backends.cudnn.enabled = False
    try:
        yr, (hnr, cnr) = ref(xr, (hr, cr))
    finally:
        torch.backends.cudnn.enabled = True
    gy = torch.randn_like(yr)
    ghn = torch.randn_like(hnr)
    (y.double() * gy).sum().add_((hn.double() * ghn).sum()).backward()
    (yr * gy).sum().add_((hnr * ghn).sum()).backward()
    tol = lambda r: 1e-4 * r.abs().max().item() + 1e-6  # noqa: E731
    assert (y.double() - yr).abs().max().item() <= tol(yr)
    assert (cn.double() - cnr).abs().max().item() <= tol(cnr)
    assert (xa.grad.double() - xr.grad).abs().max().item() <= tol(xr.grad)
    assert (ha.grad.double() - hr.grad).abs().max().item() <= tol(hr.grad)
    assert (ca.grad.double() - cr.grad).abs().max().item() <= tol(cr.grad)
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert (p.grad.double() - q.grad).abs().max().item() <= tol(q.grad), n


def test_gklstm_f32_direct_arena_grads():
    """install_direct_grads: the fp32 GkLSTM backward adds its weight / bias
    gradients straight into the optimizer arena (same values as the plain path)."""
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.ops.lstm import GkLSTM
    from gaussiank_sgd_amd.parallel import comm, install_direct_grads
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    comm.init()
    torch.manual_seed(1)
    net = GkLSTM(128, 192, num_layers=2).cuda()
    ref = copy.deepcopy(net)
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), named_parameters=net.named_parameters(),
                               compression=compressors["none"], is_sparse=False, density=1.0)
    assert install_direct_grads(net, opt) == 8
    x = torch.randn(12, 8, 128, device="cuda")
    for model in (net, ref):
        y, _ = model(x)
        y.square().mean().backward()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        err = (p.grad - q.grad).abs().max().item()
        assert err <= 1e-5 * q.grad.abs().max().item() + 1e-7, (n, err)
