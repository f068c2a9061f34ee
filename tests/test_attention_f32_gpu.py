"""fp32 fused self-attention (csrc/kernels/attn_f32.hip) vs an fp64 PyTorch
reference of the same op (the kernels' own dropout mask): forward output and
log-sum-exp, dQ / dK / dV at fp32 tolerances, determinism, and the fp32 BERT
layer taking the fused path."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from gaussiank_sgd_amd import ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load(), ops._load_error


def _qkv(B, T, heads, seed, qscale=1.0):
    torch.manual_seed(seed)
    x = torch.randn(B, T, 3, heads, 64, device="cuda")
    x[:, :, 0] *= qscale
    return x.reshape(B, T, 3 * heads * 64).contiguous()


def _ref64(qkv, heads, p, seed):
    """fp64 attention with the kernels' keep mask (autograd-able)."""
    from gaussiank_sgd_amd.ops import attention
    B, T, _ = qkv.shape
    x = qkv.view(B, T, 3, heads, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = torch.matmul(q, k.transpose(-1, -2)) / 8.0
    a = torch.softmax(s, dim=-1)
    if p > 0:
        keep = attention.dropout_mask(B, heads, T, p, seed, qkv.device)
        a = a * keep.to(a.dtype) * attention.drop_scale(p)
    return torch.matmul(a, v).transpose(1, 2).reshape(B, T, heads * 64), s


@pytest.mark.parametrize("B,T,heads,qscale", [(2, 128, 3, 1.0), (1, 256, 2, 3.0), (2, 512, 2, 1.0), (1, 384, 1, 6.0)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_f32_forward(B, T, heads, qscale, p):
    qkv = _qkv(B, T, heads, T + heads, qscale)
    seed = 4321 + T
    out = torch.full((B, T, heads * 64), float("nan"), device="cuda")
    lse = torch.empty(B * heads * T, device="cuda")
    torch.ops.gksgd.attn_f32_fwd(qkv, out, lse, heads, p, seed)
    ref, s = _ref64(qkv.double(), heads, p, seed)
    err = (out.double() - ref).abs().max().item()
    assert err <= 2e-5 * max(1.0, ref.abs().max().item()), err
    lse_ref = (torch.logsumexp(s, dim=-1) / math.log(2.0)).reshape(-1)
    assert (lse.double() - lse_ref).abs().max().item() <= 1e-4 * max(1.0, qscale) ** 2


@pytest.mark.parametrize("B,T,heads,qscale", [(2, 128, 3, 1.0), (1, 256, 2, 3.0), (2, 512, 2, 1.0)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_f32_backward(B, T, heads, qscale, p):
    from gaussiank_sgd_amd.ops import attention
    qkv = _qkv(B, T, heads, 7 * T + heads, qscale)
    torch.manual_seed(99)
    dout = torch.randn(B, T, heads * 64, device="cuda")
    seed = 77 + T
    qkv_a = qkv.clone().requires_grad_(True)
    out = attention._FlashAttnF32Fn.apply(qkv_a, heads, p, seed)
    out.backward(dout)
    qkv_r = qkv.double().requires_grad_(True)
    ref, _ = _ref64(qkv_r, heads, p, seed)
    ref.backward(dout.double())
    assert (out.double() - ref).abs().max().item() <= 2e-5 * max(1.0, ref.abs().max().item())
    g = qkv_a.grad.double().view(B, T, 3, heads, 64)
    gr = qkv_r.grad.view(B, T, 3, heads, 64)
    for i, name in enumerate("qkv"):
        e = (g[:, :, i] - gr[:, :, i]).abs().max().item()
        scale = gr[:, :, i].abs().max().item()
        assert e <= 1e-4 * scale + 1e-5, (name, e, scale)


def test_attn_f32_deterministic():
    qkv = _qkv(2, 256, 2, 3)
    outs = []
    for _ in range(2):
        out = torch.empty(2, 256, 128, device="cuda")
        lse = torch.empty(2 * 2 * 256, device="cuda")
        torch.ops.gksgd.attn_f32_fwd(qkv, out, lse, 2, 0.1, 42)
        dq = torch.empty_like(qkv)
        torch.ops.gksgd.attn_f32_bwd(qkv, out, out, lse, torch.empty_like(lse), dq, 2, 0.1, 42)
        outs.append((out, dq))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_bert_layer_f32_fused_matches_sdpa():
    """fp32 (no autocast) BERT layer: the fused fp32 kernels vs the SDPA path."""
    from gaussiank_sgd_amd.models.bert import BertConfig, BertLayer
    from gaussiank_sgd_amd.ops import attention
    torch.manual_seed(0)
    c = BertConfig(hidden=256, heads=4, intermediate=512, dropout=0.0)
    layer = BertLayer(c).cuda().eval()
    x = torch.randn(2, 256, 256, device="cuda")
    assert attention.fused_available(layer.qkv(x), 4)
    y = layer(x)
    mask = torch.zeros(2, 1, 256, 256, device="cuda")
    y2 = layer(x, attn_mask=mask)
    assert (y - y2).abs().max().item() <= 1e-4
