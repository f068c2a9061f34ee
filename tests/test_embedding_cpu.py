"""ops/embedding.py off the GPU: the plain composition, same semantics as the
BERT model's three nn.Embedding lookups (the HIP path is tests/test_embedding_gpu.py)."""
import torch
import torch.nn as nn

from gaussiank_sgd_amd.models.bert import bert_tiny
from gaussiank_sgd_amd.ops import embedding as emb


def test_cpu_fallback_matches_composition():
    torch.manual_seed(0)
    word, pos, tt_emb = nn.Embedding(50, 8), nn.Embedding(16, 8), nn.Embedding(2, 8)
    ids = torch.randint(0, 50, (3, 10))
    tt = torch.randint(0, 2, (3, 10))
    assert not emb.fused_available(ids, word, pos, tt_emb)
    out = emb.bert_embeddings(ids, tt, word, pos, tt_emb)
    ref = word(ids) + pos(torch.arange(10).unsqueeze(0)) + tt_emb(tt)
    assert torch.equal(out, ref)
    out0 = emb.bert_embeddings(ids, None, word, pos, tt_emb)
    assert torch.equal(out0, word(ids) + pos(torch.arange(10).unsqueeze(0)) + tt_emb(torch.zeros_like(ids)))


def test_bert_embedding_gradients_cpu():
    torch.manual_seed(0)
    m = bert_tiny()
    ids = torch.randint(0, 1024, (2, 32))
    m(ids).float().sum().backward()
    g = m.position_embeddings.weight.grad
    assert g[:32].abs().sum() > 0 and g[32:].abs().sum() == 0
    assert m.token_type_embeddings.weight.grad[1].abs().sum() == 0   # type 1 never used
