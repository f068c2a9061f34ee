"""Fused self-attention (csrc/kernels/attn.hip) vs an fp32 PyTorch reference of
the same op (ops.attention.reference_attention, with the kernels' own dropout
mask): forward output and log-sum-exp, dQ / dK / dV, the mask kernel vs its
CPU mirror, and the BERT layer on the fused path vs the SDPA path."""
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
    return x.reshape(B, T, 3 * heads * 64).to(torch.bfloat16).contiguous()


@pytest.mark.parametrize("B,T,heads,qscale", [(2, 128, 3, 1.0), (1, 256, 2, 3.0), (2, 512, 2, 1.0), (1, 384, 1, 6.0)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_forward(B, T, heads, qscale, p):
    from gaussiank_sgd_amd.ops import attention
    qkv = _qkv(B, T, heads, T + heads, qscale)
    seed = 1234 + T
    out = torch.empty(B, T, heads * 64, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B * heads * T, device="cuda")
    torch.ops.gksgd.attn_fwd(qkv, out, lse, heads, p, seed)
    ref = attention.reference_attention(qkv, heads, p, seed)
    err = (out.float() - ref).abs().max().item()
    assert err <= 2e-2 * max(1.0, ref.abs().max().item()), err
    x = qkv.float().view(B, T, 3, heads, 64)
    s = torch.einsum("bqhd,bkhd->bhqk", x[:, :, 0], x[:, :, 1]) / 8.0
    lse_ref = (torch.logsumexp(s, dim=-1) / math.log(2.0)).reshape(-1)
    # the kernels pre-scale q by log2(e)/8 in bf16 (one more operand rounding):
    # the score error grows with |q|, so the bound does too
    dl = (lse - lse_ref).abs()
    assert dl.max().item() <= 4e-3 * max(1.0, qscale) ** 2, (dl.max().item(), int(dl.argmax()), dl.mean().item())


@pytest.mark.parametrize("B,T,heads,qscale", [(2, 128, 3, 1.0), (1, 256, 2, 3.0), (2, 512, 2, 1.0)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_backward(B, T, heads, qscale, p):
    from gaussiank_sgd_amd.ops import attention
    qkv = _qkv(B, T, heads, 7 * T + heads, qscale)
    torch.manual_seed(99)
    dout = torch.randn(B, T, heads * 64, device="cuda").to(torch.bfloat16)
    seed = 77 + T
    qkv_a = qkv.clone().requires_grad_(True)
    out = attention._FlashAttnFn.apply(qkv_a, heads, p, seed)
    out.backward(dout)
    qkv_r = qkv.float().requires_grad_(True)
    ref = attention.reference_attention(qkv_r, heads, p, seed)
    ref.backward(dout.float())
    assert (out.float() - ref).abs().max().item() <= 2e-2 * max(1.0, ref.abs().max().item())
    g = qkv_a.grad.float().view(B, T, 3, heads, 64)
    gr = qkv_r.grad.view(B, T, 3, heads, 64)
    for i, name in enumerate("qkv"):
        e = (g[:, :, i] - gr[:, :, i]).abs().max().item()
        scale = gr[:, :, i].abs().max().item()
        assert e <= 2.5e-2 * scale + 1e-3, (name, e, scale)


def test_attn_dropout_mask_matches_cpu_mirror():
    from gaussiank_sgd_amd.ops import attention
    for p, seed in [(0.1, 5), (0.5, 123456)]:
        g = attention.dropout_mask(2, 3, 128, p, seed, "cuda").cpu()
        c = attention.dropout_mask(2, 3, 128, p, seed, "cpu")
        assert torch.equal(g, c)
        assert abs(g.float().mean().item() - (1 - p)) < 0.01


def test_attn_deterministic():
    qkv = _qkv(2, 256, 2, 3)
    outs = []
    for _ in range(2):
        out = torch.empty(2, 256, 128, dtype=torch.bfloat16, device="cuda")
        lse = torch.empty(2 * 2 * 256, device="cuda")
        torch.ops.gksgd.attn_fwd(qkv, out, lse, 2, 0.1, 42)
        dq = torch.empty_like(qkv)
        torch.ops.gksgd.attn_bwd(qkv, out, out, lse, torch.empty_like(lse), dq, 2, 0.1, 42)
        outs.append((out, dq))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_bert_layer_fused_matches_sdpa():
    from gaussiank_sgd_amd.models.bert import BertConfig, BertLayer
    from gaussiank_sgd_amd.ops import attention
    torch.manual_seed(0)
    c = BertConfig(hidden=256, heads=4, intermediate=512, dropout=0.0)
    layer = BertLayer(c).cuda().eval()
    x = torch.randn(2, 256, 256, device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = layer(x)
    # the SDPA path: an all-zero additive mask disables the fused kernel
    mask = torch.zeros(2, 1, 256, 256, device="cuda", dtype=torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert attention.fused_available(layer.qkv(x), 4)
        y2 = layer(x, attn_mask=mask)
    assert (y.float() - y2.float()).abs().max().item() <= 5e-2
