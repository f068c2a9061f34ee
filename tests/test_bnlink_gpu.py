"""BatchNorm-backward reduction fused into the consuming convolution's
grad-input GEMM epilogue (csrc/kernels/gemm.hip ``BnBwd``, ops/bn.py
``BnLink``, ops/conv1x1.py ``_dgrad_bn``).

Kernel level: the epilogue's dz = mask ? bf16(acc) + dy2 : 0 and its partials
sum(dz), sum(dz * h) against an fp32 PyTorch reference.  Network level: a
ResNet-50 training step with the fusion on and off gives the same gradients,
and the fused path really runs (BN reduction kernels skipped)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error


def _bits(mask_bytes, M, N):
    """[M, N/8] uint8 -> [M, N] bool (bit j of byte c = channel 8c + j)."""
    b = mask_bytes.view(M, N // 8).to(torch.int32)
    sh = torch.arange(8, device=b.device, dtype=torch.int32)
    return ((b[:, :, None] >> sh) & 1).reshape(M, N).bool()


def _check(dz, part, rows, y_bf16, dy2, keep, h):
    M, N = y_bf16.shape
    ref = y_bf16.float() + (dy2.float() if dy2 is not None else 0.0)
    ref = torch.where(keep, ref, torch.zeros_like(ref))
    scale = ref.abs().max().item() + 1e-6
    assert (dz.float() - ref).abs().max().item() <= 1e-2 * scale
    s1 = part[0, :rows].double().sum(0)
    s2 = part[1, :rows].double().sum(0)
    r1 = ref.double().sum(0)
    r2 = (ref.double() * h.double()).sum(0)
    assert (s1 - r1).abs().max().item() <= 1e-2 * r1.abs().max().item() + 1e-3 * scale
    assert (s2 - r2).abs().max().item() <= 1e-2 * r2.abs().max().item() + 1e-3 * scale


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 21, 113, 124])
@pytest.mark.parametrize("M,N,K,twin", [(1000 + 37, 256, 64, True), (777, 128, 192, False), (4096, 64, 256, True)])
def test_gemm_nt_bn_epilogue(cfg, M, N, K, twin):
    torch.manual_seed(cfg + M)
    g = torch.ops.gksgd
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    h = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    dy2 = torch.randn(M, N, device="cuda").to(torch.bfloat16) if twin else None
    mask = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    part = torch.full((2, 1280, N), float("nan"), device="cuda")
    rows = g.gemm_nt(A, B, C, cfg, 0, part, None, h, dy2, mask)
    torch.cuda.synchronize()
    y = (A.float() @ B.float().t()).to(torch.bfloat16)
    _check(C, part, rows, y, dy2, _bits(mask, M, N), h.float())


@pytest.mark.parametrize("cfg", [1, 4, 121])
@pytest.mark.parametrize("Nb,C,H,K", [(2, 64, 14, 64), (3, 128, 9, 256)])
def test_conv_nt_bn_epilogue(cfg, Nb, C, H, K):
    torch.manual_seed(cfg + C)
    g = torch.ops.gksgd
    x = torch.randn(Nb, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(K, C, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    h = torch.randn(Nb, K, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    dy2 = torch.randn(Nb, K, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    M = Nb * H * H
    mask = torch.randint(0, 256, (M * K // 8,), device="cuda", dtype=torch.uint8)
    y = torch.empty(Nb, K, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=CL)
    z = torch.zeros(256, device="cuda", dtype=torch.bfloat16)
    part = torch.empty(2, 1280, K, device="cuda")
    rows = g.conv_nt(x, w, y, z, 1, 1, cfg, 0, part, None, h, dy2, mask)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.float(), padding=1).to(torch.bfloat16)
    rows2d = lambda t: t.permute(0, 2, 3, 1).reshape(M, -1)  # noqa: E731
    _check(rows2d(y), part, rows, rows2d(ref), rows2d(dy2), _bits(mask, M, K), rows2d(h).float())


def _step(model, x, amp=True):
    model.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        out = model(x)
    out.float().square().mean().backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().double().clone() for n, p in model.named_parameters()}


def test_resnet50_bn_link_matches_unfused(monkeypatch):
    """One bf16 training step with the BN-backward fusion on and off, each
    against the fp32 step of the same network: the fused path's error must be
    no worse than the unfused one's (deep BN stacks amplify bf16 rounding, so
    the comparison is relative to the unfused bf16 path, not absolute), and
    the fused grad-input must actually run for every linked BN."""
    from gaussiank_sgd_amd.models import resnet50
    from gaussiank_sgd_amd.ops import conv1x1
    monkeypatch.setattr(conv1x1, "_TUNE", False)
    monkeypatch.setattr(conv1x1, "_choices", {})
    calls = []
    orig = conv1x1._dgrad_bn

    def counting(*a, **k):
        calls.append(a[0].shape)
        return orig(*a, **k)
    monkeypatch.setattr(conv1x1, "_dgrad_bn", counting)
    torch.manual_seed(0)
    m = resnet50(num_classes=16).cuda().to(memory_format=CL)
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=CL)
    ref = _step(m, x, amp=False)
    # the fp32 reference step runs the fp32 MFMA kernels, BN-backward fusion included
    assert len(calls) == 13 + 16 + 12, len(calls)
    calls.clear()
    monkeypatch.setenv("GKSGD_BN_LINK", "0")
    g0 = _step(m, x)
    assert not calls
    monkeypatch.setenv("GKSGD_BN_LINK", "1")
    g1 = _step(m, x)
    # bn1 -> conv2 (13 stride-1 conv2), bn2 -> conv3 (16), block outputs -> next conv1 (12)
    assert len(calls) == 13 + 16 + 12, len(calls)
    worse = []
    for n in ref:
        r = ref[n]
        e0 = float((g0[n] - r).norm() / (r.norm() + 1e-30))
        e1 = float((g1[n] - r).norm() / (r.norm() + 1e-30))
        if e1 > 1.5 * e0 + 2e-3:
            worse.append((n, e1, e0))
    assert not worse, worse
