"""Fused BERT input embedding (ops/embedding.py, csrc/kernels/embed.hip) vs the
plain fp32 PyTorch composition word(ids) + pos(arange(T)) + type(tt)."""
import pytest
import torch
import torch.nn as nn

from gaussiank_sgd_amd.ops import embedding as emb

pytestmark = pytest.mark.gpu


def _mods(V, P, NT, H, dev):
    torch.manual_seed(0)
    return [nn.Embedding(n, H).to(dev) for n in (V, P, NT)]


def _grads(mods):
    return [m.weight.grad.detach().clone() for m in mods]


@pytest.mark.parametrize("B,T,V,P,H,with_tt", [(2, 16, 100, 32, 64, True), (4, 128, 30522, 512, 768, True),
                                               (3, 7, 50, 7, 12, False)])
def test_fused_embedding_matches_torch(cuda, B, T, V, P, H, with_tt):
    mods = _mods(V, P, 2, H, cuda)
    ids = torch.randint(0, V, (B, T), device=cuda)
    ids[0, :3] = 5                      # an id seen a few times: ranked (ascending token) sum
    if T >= 100:
        ids[:, :100] = 7                    # an id seen > 64 times: slot-order sum
    tt = torch.randint(0, 2, (B, T), device=cuda) if with_tt else None
    assert emb.fused_available(ids, *mods)
    dy = torch.randn(B, T, H, device=cuda)

    out = emb.bert_embeddings(ids, tt, *mods)
    out.backward(dy)
    g_fused = _grads(mods)
    for m in mods:
        m.weight.grad = None

    pos = torch.arange(T, device=cuda).unsqueeze(0)
    ref = mods[0](ids) + mods[1](pos) + mods[2](tt if tt is not None else torch.zeros_like(ids))
    ref.backward(dy)
    g_ref = _grads(mods)

    assert out.dtype == torch.float32
    assert torch.equal(out, ref)        # same gathers, same add order
    for a, b in zip(g_fused, g_ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_fused_embedding_bert_autocast(cuda):
    from gaussiank_sgd_amd.models.bert import bert_tiny
    torch.manual_seed(0)
    m = bert_tiny().to(cuda)
    ids = torch.randint(0, 1024, (2, 64), device=cuda)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(ids)
    out.float().square().mean().backward()
    g = m.word_embeddings.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0
    assert m.position_embeddings.weight.grad[64:].abs().sum() == 0     # rows past T get no gradient


def test_fused_embedding_backward_deterministic(cuda):
    B, T, V, P, H = 8, 512, 30522, 512, 768
    mods = _mods(V, P, 2, H, cuda)
    ids = torch.randint(5, V, (B, T), device=cuda)
    ids[:, ::7] = 4                     # a [MASK]-like id: 586 tokens, ten 64-token chunks
    tt = torch.randint(0, 2, (B, T), device=cuda)
    dy = torch.randn(B, T, H, device=cuda)
    runs = []
    for _ in range(2):
        for m in mods:
            m.weight.grad = None
        emb.bert_embeddings(ids, tt, *mods).backward(dy)
        runs.append(_grads(mods))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    ref = torch.zeros(V, H, device=cuda, dtype=torch.float64).index_add_(0, ids.view(-1), dy.view(-1, H).double())
    torch.testing.assert_close(runs[0][0].double(), ref, rtol=1e-5, atol=1e-4)
