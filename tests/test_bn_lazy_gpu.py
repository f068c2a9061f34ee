"""Lazy BatchNorm backward (ops/bn.py ProducerLink; gemm.hip LazyA / the fp32
TN kernel's lazy G operand; bn_act.hip bn_bwd_finalize_lazy / bn_lazy_apply).

The BN backward's apply pass dx = k1 ((dz - k2) - (x - mu) k4) is folded
into the operand load of the producing convolution's grad-input (NT) and
grad-weight (TN) GEMMs.  Each kernel is checked against an fp64 PyTorch
reference computed from the materialised dx, including padded taps (the
pad rows padz = k2, padx = mu must contribute exactly 0), M tails and split
boundaries; the BN kernels against the non-lazy fused backward; and a whole
fp32 ResNet-50 step against the same step with GKSGD_BN_LAZY=0.
"""
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


def _lazy_operand(shape4d, C):
    """(dz, x, coef, padz, padx, dx_ref fp64) with the channel dim last in memory."""
    dz = torch.randn(shape4d, device="cuda").contiguous(memory_format=CL)
    x = (torch.randn(shape4d, device="cuda") * 2 + 0.5).contiguous(memory_format=CL)
    k1 = torch.rand(C, device="cuda") + 0.5
    k2 = torch.randn(C, device="cuda") * 0.1
    mu = torch.randn(C, device="cuda") * 0.5
    k4 = torch.randn(C, device="cuda") * 0.2
    coef = torch.stack([k1, k2, mu, k4], 1).contiguous()
    c = lambda v: v.double().view(1, C, 1, 1)  # noqa: E731
    dx = c(k1) * ((dz.double() - c(k2)) - (x.double() - c(mu)) * c(k4))
    return dz, x, coef, k2.clone(), mu.clone(), dx


def _rows(t):
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _kw(x, coef, padz, padx, rows=False):
    return dict(lz_x=_rows(x) if rows else x, lz_coef=coef, lz_padz=padz, lz_padx=padx)


def _call(fn, *a, **kw):
    """Run a kernel; a tile whose doubled A stage + coefficient table exceeds
    the 160 KiB LDS refuses the lazy operand (the autotuner skips it)."""
    try:
        return fn(*a, **kw)
    except RuntimeError as e:
        if "does not fit" in str(e):
            pytest.skip("lazy operand does not fit this tile")
        raise


def _close(out, ref, bound):
    err = (out.double() - ref).abs().max().item()
    assert err <= 4e-6 * bound.abs().max().item() + 1e-5, err


@pytest.mark.parametrize("N,H,K,Cout", [(2, 9, 64, 64), (3, 7, 128, 256), (1, 31, 256, 64), (2, 14, 512, 128)])
@pytest.mark.parametrize("cfg,mb", [(1, 0), (3, 0), (4, 3), (13, 0), (22, 0), (104, 1), (204, 0), (2, 2)])
def test_gemm_nt_lazy(g, N, H, K, Cout, cfg, mb):
    """1x1 stride-1 grad-input: C[M, Cout] = dx[M, K] . W^T with dx lazy."""
    torch.manual_seed(N * H + K + cfg)
    dz, x, coef, padz, padx, dx = _lazy_operand((N, K, H, H), K)
    B = torch.randn(Cout, K, device="cuda") * K ** -0.5
    out = torch.full((N * H * H, Cout), float("nan"), device="cuda")
    _call(g.gemm_nt, _rows(dz), B, out, cfg, mb, **_kw(x, coef, padz, padx, rows=True))
    ref = _rows(dx) @ B.double().t()
    _close(out, ref, _rows(dx).abs() @ B.double().abs().t())


@pytest.mark.parametrize("N,H,K,Cout", [(2, 9, 64, 64), (1, 14, 128, 64), (2, 7, 256, 128), (1, 11, 64, 192)])
@pytest.mark.parametrize("cfg", [1, 3, 4, 13, 22, 104, 204])
def test_conv_nt_lazy(g, N, H, K, Cout, cfg):
    """3x3 stride-1 grad-input as a conv of the lazy dx: padded taps give 0."""
    torch.manual_seed(N * H + K + cfg + 1)
    dz, x, coef, padz, padx, dx = _lazy_operand((N, K, H, H), K)
    wf = (torch.randn(Cout, K, 3, 3, device="cuda") * (9 * K) ** -0.5).contiguous(memory_format=CL)
    out = torch.full((N, Cout, H, H), float("nan"), device="cuda").contiguous(memory_format=CL)
    _call(g.conv_nt, dz, wf, out, torch.zeros(64, device="cuda"), 1, 1, cfg, 0, **_kw(x, coef, padz, padx))
    ref = F.conv2d(dx, wf.double(), padding=1)
    _close(out, ref, F.conv2d(dx.abs(), wf.double().abs(), padding=1))


@pytest.mark.parametrize("N,C,H,K,k", [(3, 128, 7, 64, 3), (2, 64, 14, 128, 3), (2, 256, 8, 128, 1),
                                       (2, 64, 13, 64, 3)])
@pytest.mark.parametrize("cfg", [1, 4, 13, 2, 102, 22, 204])
def test_conv_dgrad_s2_lazy(g, N, C, H, K, k, cfg):
    """Stride-2 grad-input: the forward conv's output gradient is lazy."""
    torch.manual_seed(N + C + H + K + cfg)
    p = k // 2
    OH = (H + 2 * p - k) // 2 + 1
    dz, x, coef, padz, padx, dyd = _lazy_operand((N, K, OH, OH), K)
    w = (torch.randn(K, C, k, k, device="cuda") * (C * k * k) ** -0.5).contiguous(memory_format=CL)
    dx = torch.full((N, C, H, H), float("nan"), device="cuda").contiguous(memory_format=CL)
    _call(g.conv_dgrad_s2, dz, w, dx, torch.zeros(64, device="cuda"), cfg, 0, **_kw(x, coef, padz, padx))
    ref = torch.ops.aten.convolution_backward(dyd, torch.zeros(N, C, H, H, device="cuda", dtype=torch.float64),
                                              w.double(), None, [2, 2], [p, p], [1, 1], False, [0, 0], 1,
                                              [True, False, False])[0]
    bound = torch.ops.aten.convolution_backward(dyd.abs(), torch.zeros(N, C, H, H, device="cuda",
                                                                       dtype=torch.float64),
                                                w.double().abs(), None, [2, 2], [p, p], [1, 1], False, [0, 0], 1,
                                                [True, False, False])[0]
    _close(dx, ref, bound)


@pytest.mark.parametrize("N,H,Nc,Kc", [(2, 9, 64, 64), (3, 13, 128, 256), (2, 31, 256, 64), (1, 7, 512, 128)])
@pytest.mark.parametrize("cfg,splits", [(1, 0), (2, 3), (4, 0), (7, 5), (9, 0), (11, 2), (13, 0), (16, 7)])
def test_gemm_tn_lazy(g, N, H, Nc, Kc, cfg, splits):
    """1x1 grad-weight W[Nc, Kc] += dx^T X with dx lazy (rows past a split end
    must contribute 0, not k1 (mu k4 - k2))."""
    torch.manual_seed(N * H + Nc + cfg + splits)
    dz, x, coef, padz, padx, dx = _lazy_operand((N, Nc, H, H), Nc)
    X = torch.randn(N * H * H, Kc, device="cuda")
    W0 = torch.randn(Nc, Kc, device="cuda")
    W = W0.clone()
    _call(g.gemm_tn_acc, _rows(dz), X, W, cfg, splits, **_kw(x, coef, padz, padx, rows=True))
    ref = W0.double() + _rows(dx).t() @ X.double()
    _close(W, ref, _rows(dx).abs().t() @ X.double().abs() + 1)


@pytest.mark.parametrize("N,C,H,Co,k,s", [(2, 64, 9, 64, 3, 1), (3, 128, 7, 64, 3, 2), (2, 64, 14, 128, 3, 2),
                                          (2, 256, 8, 128, 1, 2), (1, 64, 11, 192, 3, 1)])
@pytest.mark.parametrize("cfg,splits", [(1, 0), (4, 3), (8, 0), (13, 5), (9, 0)])
def test_conv_tn_lazy(g, N, C, H, Co, k, s, cfg, splits):
    """Implicit-GEMM grad-weight with the output gradient lazy."""
    torch.manual_seed(N * 7 + C + H + Co + cfg)
    p = k // 2
    OH = (H + 2 * p - k) // s + 1
    dz, x_bn, coef, padz, padx, dyd = _lazy_operand((N, Co, OH, OH), Co)
    xin = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    out = torch.zeros(Co, C, k, k, device="cuda").contiguous(memory_format=CL)
    _call(g.conv_tn_acc, dz, xin, out, torch.zeros(64, device="cuda"), s, p, cfg, splits, **_kw(x_bn, coef, padz, padx))
    wr = torch.ops.aten.convolution_backward(dyd, xin.double(), torch.zeros(Co, C, k, k, device="cuda",
                                                                            dtype=torch.float64),
                                             None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                             [False, True, False])[1]
    bound = torch.ops.aten.convolution_backward(dyd.abs(), xin.double().abs(),
                                                torch.zeros(Co, C, k, k, device="cuda", dtype=torch.float64),
                                                None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                [False, True, False])[1]
    _close(out, wr, bound)


@pytest.mark.parametrize("k", [1, 3])
def test_dgrad_bn_epilogue_lazy(g, k):
    """Both fusions at once: lazy dx operand + BN-backward epilogue (dz of
    the NEXT BN up and its reduction partials)."""
    torch.manual_seed(40 + k)
    N, C, H, Co = 2, 64, 9, 128
    p = k // 2
    dz_in, x_bn, coef, padz, padx, dyd = _lazy_operand((N, Co, H, H), Co)
    w = (torch.randn(Co, C, k, k, device="cuda") * 0.1).contiguous(memory_format=CL)
    h = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
    relu = torch.rand(N, C, H, H, device="cuda") > 0.4
    M = N * H * H
    bits = relu.permute(0, 2, 3, 1).reshape(M, C // 4, 4).to(torch.int32)
    mask = (bits * torch.tensor([1, 2, 4, 8], device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).reshape(-1)
    ref_dx = torch.ops.aten.convolution_backward(dyd, h.double(), w.double(), None, [1, 1], [p, p], [1, 1],
                                                 False, [0, 0], 1, [True, False, False])[0]
    dz_ref = torch.where(relu, ref_dx, torch.zeros_like(ref_dx))
    dz = torch.full(h.shape, float("nan"), device="cuda").contiguous(memory_format=CL)
    st = torch.full((2, 64, C), float("nan"), device="cuda")
    if k == 1:
        rows = g.gemm_nt(_rows(dz_in), w.reshape(Co, C).t().contiguous(), _rows(dz), 4, 0, st, None, _rows(h),
                         None, mask, **_kw(x_bn, coef, padz, padx, rows=True))
    else:
        wf = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL)
        rows = g.conv_nt(dz_in, wf, dz, torch.zeros(64, device="cuda"), 1, p, 4, 0, st, None, h, None, mask,
                         **_kw(x_bn, coef, padz, padx))
    assert (dz.double() - dz_ref).abs().max().item() <= 1e-5 * dz_ref.abs().max().item() + 1e-5
    s = st[:, :rows].double().sum(1)
    dzc = _rows(dz_ref)
    assert torch.allclose(s[0], dzc.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[1], (dzc * _rows(h).double()).sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bnact_lazy_backward_matches_fused(monkeypatch, relu, res):
    """BNAct after a FastConv2d: the lazy backward (dz to the conv, dx formed in
    its GEMMs) gives the same input / weight / BN-parameter gradients as the
    fused non-lazy backward and fp64 torch."""
    from gaussiank_sgd_amd.ops import conv1x1
    from gaussiank_sgd_amd.ops.bn import BNAct

    def run(lazy):
        monkeypatch.setenv("GKSGD_BN_LAZY", "1" if lazy else "0")
        torch.manual_seed(3)
        conv = conv1x1.FastConv2d(64, 128, 3, padding=1, bias=False).cuda().to(memory_format=CL)
        bn = BNAct(128, act="relu" if relu else None).cuda()
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.2, 0.2)
        x = torch.randn(4, 64, 14, 14, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
        r = torch.randn(4, 128, 14, 14, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
        y, st = conv1x1.conv_stats(conv, x)
        out = bn(y, r if res else None, stats=st)
        dy = torch.randn(out.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(9))
        out.backward(dy.contiguous(memory_format=CL))
        return [t.detach().clone() for t in (x.grad, conv.weight.grad, bn.weight.grad, bn.bias.grad)] + \
            ([r.grad.clone()] if res else [])

    lazy, plain = run(True), run(False)
    for a, b in zip(lazy, plain):
        assert (a - b).abs().max().item() <= 1e-4 * b.abs().max().item() + 1e-5
    assert any(key[-1] == "lz" for key in conv1x1.tuned_choices()), "lazy path not taken"


def test_resnet50_step_lazy_matches_plain(monkeypatch):
    """One fp32 ResNet-50 training step (small batch): the lazy BN backward's
    parameter gradients are as close to an fp64 run of the same network as
    the non-lazy fused backward's (fp32 reordering is amplified through 53
    small-batch BatchNorms, so both are compared against fp64, not each
    other)."""
    from gaussiank_sgd_amd.models.resnet_imagenet import resnet50
    from gaussiank_sgd_amd.ops import conv1x1
    # the lazy operands ride on the direct kernels; compare like with like
    monkeypatch.setattr(conv1x1, "_WINO", False)
    torch.manual_seed(0)
    m0 = resnet50(num_classes=10)
    x = torch.randn(8, 3, 96, 96)
    t = torch.randint(0, 10, (8,))

    def run(lazy, dtype=torch.float32):
        monkeypatch.setenv("GKSGD_BN_LAZY", "1" if lazy else "0")
        m = resnet50(num_classes=10)
        m.load_state_dict(m0.state_dict())
        m = m.to(device="cuda", dtype=dtype).to(memory_format=CL)
        xi = x.to(device="cuda", dtype=dtype).contiguous(memory_format=CL)
        F.cross_entropy(m(xi), t.cuda()).backward()
        return {n: p.grad.detach().double() for n, p in m.named_parameters()}

    ref = run(False, torch.float64)
    # the second lazy run replays the autotuned choices without the search
    # (a tile that silently skipped work would only show there)
    lazy, plain, lazy2 = run(True), run(False), run(True)
    # small-batch BatchNorm makes this step chaotic (plain fp32 is ~2% off fp64
    # too, and which parameter is worst changes run to run with the atomic
    # summation order): compare the error over all parameters, and bound the
    # worst single parameter loosely (a skipped tile would be ~100% off)
    worst = 0.0
    tot_plain = tot_lazy = 0.0
    for n in ref:
        scale = ref[n].abs().max().item() + 1e-12
        e_plain = (plain[n] - ref[n]).abs().max().item() / scale
        tot_plain += e_plain
        for got in (lazy, lazy2):
            e_lazy = (got[n] - ref[n]).abs().max().item() / scale
            tot_lazy += 0.5 * e_lazy
            worst = max(worst, e_lazy)
    assert tot_lazy <= 2 * tot_plain + 1e-2 * len(ref), (tot_lazy, tot_plain)
    assert worst < 0.3, worst
