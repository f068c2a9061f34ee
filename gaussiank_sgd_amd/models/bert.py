"""BERT-base masked-language model (BASELINE config 5; not in the reference).

Standard BERT-base: vocab 30522, hidden 768, 12 layers, 12 heads, FFN 3072,
512 positions, GELU, post-LN, MLM head tied to the word embeddings
(~110M parameters).  On the GPU, attention is the flash-style HIP kernel of
ops/attention.py on the packed QKV projection (no head split / merge copies);
with an attention mask or on the CPU it is ``F.scaled_dot_product_attention``.
Run under bf16 autocast.  Every encoder / MLM-head
linear is a ``FastLinear`` (ops/linear.py: autotuned MFMA GEMMs, GELU backward
and bias gradient in one fused pass into the fp32 gradient arena).  Gradients stay fp32 in
the flat arena, so compression is unaffected by the compute dtype.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import attention, xent
from ..ops.embedding import bert_embeddings
from ..ops.linear import FastLinear
from ..ops.ln import add_layernorm


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    dropout: float = 0.1
    ln_eps: float = 1e-12


class _SplitHeads(torch.autograd.Function):
    """[B, T, 3*H] projection -> q, k, v as [B, heads, T, d] strided views (no
    copy).  The backward writes dq, dk, dv straight into ONE [B, T, 3, heads, d]
    gradient -- three strided copies, instead of autograd's stack of the three
    (a 75 MB CatArrayBatchedCopy per BERT-base layer at ~1.5 TB/s) followed by
    the permute's reshape copy."""

    @staticmethod
    def forward(ctx, y, heads):
        B, T, H3 = y.shape
        d = H3 // (3 * heads)
        ctx.dims = (B, T, heads, d)
        v5 = y.view(B, T, 3, heads, d)
        return v5[:, :, 0].transpose(1, 2), v5[:, :, 1].transpose(1, 2), v5[:, :, 2].transpose(1, 2)

    @staticmethod
    def backward(ctx, dq, dk, dv):
        B, T, h, d = ctx.dims
        ref = next(g for g in (dq, dk, dv) if g is not None)
        g5 = torch.empty(B, T, 3, h, d, dtype=ref.dtype, device=ref.device)
        for i, gi in enumerate((dq, dk, dv)):
            if gi is None:
                g5[:, :, i].zero_()
            else:
                g5[:, :, i].copy_(gi.transpose(1, 2))
        return g5.view(B, T, 3 * h * d), None


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.heads = c.heads
        self.qkv = FastLinear(c.hidden, 3 * c.hidden)
        self.attn_out = FastLinear(c.hidden, c.hidden)
        self.ln1 = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.ffn_in = FastLinear(c.hidden, c.intermediate)
        self.ffn_out = FastLinear(c.intermediate, c.hidden)
        self.ln2 = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.drop = nn.Dropout(c.dropout)
        self.p = c.dropout

    def forward(self, x, attn_mask=None):
        B, T, H = x.shape
        y = self.qkv(x)
        if attn_mask is None and attention.fused_available(y, self.heads):
            # flash-style HIP attention straight on the packed projection (ops/attention.py)
            a = attention.self_attention(y, self.heads, self.p, self.training)
        else:
            q, k, v = _SplitHeads.apply(y, self.heads)
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask,
                                               dropout_p=self.p if self.training else 0.0)
            a = a.transpose(1, 2).reshape(B, T, H)
        # ln(x + drop(y)) as one fused HIP pass each way on the GPU (ops/ln.py)
        x = add_layernorm(self.attn_out(a), x, self.ln1, self.p, self.training)
        h = self.ffn_out(self.ffn_in(x, act="gelu"))
        return add_layernorm(h, x, self.ln2, self.p, self.training)


class BertForMaskedLM(nn.Module):
    def __init__(self, c: BertConfig = None):
        super().__init__()
        c = c or BertConfig()
        self.config = c
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden)
        self.position_embeddings = nn.Embedding(c.max_position, c.hidden)
        self.token_type_embeddings = nn.Embedding(c.type_vocab, c.hidden)
        self.emb_ln = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.emb_drop = nn.Dropout(c.dropout)
        self.encoder = nn.ModuleList([BertLayer(c) for _ in range(c.layers)])
        self.mlm_dense = FastLinear(c.hidden, c.hidden)
        self.mlm_ln = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.mlm_bias = nn.Parameter(torch.zeros(c.vocab_size))
        self.name = "bert"
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)
        if isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_positions=None):
        """Logits [B, T, V], or [B, P, V] at ``masked_positions`` ([B, P]
        indices, the Google-BERT pre-training format): the MLM head and the
        vocabulary projection then run on the masked rows only."""
        # word + position + token-type lookups: one fused HIP pass each way on the GPU (ops/embedding.py)
        x = bert_embeddings(input_ids, token_type_ids, self.word_embeddings, self.position_embeddings,
                            self.token_type_embeddings)
        x = self.emb_drop(self.emb_ln(x))
        mask = None
        if attention_mask is not None:
            mask = attention_mask[:, None, None, :].to(torch.bool)
        for layer in self.encoder:
            x = layer(x, mask)
        if masked_positions is not None:
            x = x.gather(1, masked_positions.unsqueeze(-1).expand(-1, -1, x.shape[-1]))
        h = self.mlm_ln(self.mlm_dense(x, act="gelu"))
        return vocab_projection(h, self.word_embeddings.weight, self.mlm_bias)


def vocab_projection(h: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """Logits = h W_emb^T + b with the (tied) word-embedding matrix.  fp32 on
    the GPU (the headline precision): the autotuned GEMMs of ops/linear.py,
    which offer the HIP kernels on zero-padded operands for the 30,522-word
    vocabulary (not a multiple of 64) against hipBLASLt; the gradients flow
    to the tied parameter through autograd as with F.linear."""
    dev = h.device.type
    if (h.is_cuda and h.dtype == torch.float32 and weight.dtype == torch.float32 and
            not torch.is_autocast_enabled(dev)):
        from ..ops import load
        from ..ops.linear import _LinearFn
        if load():
            return _LinearFn.apply(h, weight, None, None, bias, None, False, None, torch.float32)
    return F.linear(h, weight, bias)


class MaskedLMLoss(nn.Module):
    """Cross entropy over masked positions (labels == -100 ignored)."""

    def forward(self, logits, labels):
        # one fused HIP pass each way on bf16 logits on the GPU (ops/xent.py)
        return xent.cross_entropy(logits, labels, ignore_index=-100)


def bert_base(**kw):
    return BertForMaskedLM(BertConfig(**kw))


def bert_tiny(**kw):
    d = dict(vocab_size=1024, hidden=64, layers=2, heads=2, intermediate=128, max_position=128)
    d.update(kw)
    return BertForMaskedLM(BertConfig(**d))
