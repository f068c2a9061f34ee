"""2-layer LSTM language model for PTB-shaped data.

Parity: reference models/lstm.py:5-47 -- embedding 1500, 2 x LSTM(1500),
35 unrolled steps, dropout 1 - 0.35 = 0.65, vocab 10k, uniform(-0.1, 0.1)
init of embedding and softmax weights; 66,034,000 parameters in 11 tensors.
``forward(inputs[T,B], hidden) -> (logits[T,B,V], hidden)``.  The LSTM is
``ops/lstm.py GkLSTM`` (same parameters as ``nn.LSTM``): bf16 hipBLASLt GEMMs
and one fused HIP cell kernel per step -- nn.LSTM on ROCm (MIOpen) would
compute in fp16 under bf16 autocast.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.linear import FastLinear
from ..ops.lstm import GkLSTM


class PTBLSTM(nn.Module):
    def __init__(self, vocab_size: int = 10000, embedding_dim: int = 1500, num_steps: int = 35,
                 batch_size: int = 20, num_layers: int = 2, dp_keep_prob: float = 0.35):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.num_steps = num_steps
        self.batch_size = batch_size
        self.vocab_size = vocab_size
        self.dp_keep_prob = dp_keep_prob
        self.num_layers = num_layers
        self.dropout = nn.Dropout(1 - dp_keep_prob)
        self.word_embeddings = nn.Embedding(vocab_size, embedding_dim)
        # drop-in nn.LSTM (same parameter names): bf16 GEMMs + fused HIP cells (ops/lstm.py)
        self.lstm = GkLSTM(input_size=embedding_dim, hidden_size=embedding_dim, num_layers=num_layers,
                           dropout=1 - dp_keep_prob)
        self.sm_fc = FastLinear(embedding_dim, vocab_size)   # fused bias-gradient pass on the GPU
        self.name = "lstm"
        self.init_weights()

    def init_weights(self):
        r = 0.1
        self.word_embeddings.weight.data.uniform_(-r, r)
        self.sm_fc.bias.data.fill_(0.0)
        self.sm_fc.weight.data.uniform_(-r, r)

    def init_hidden(self, batch_size: int = None):
        b = self.batch_size if batch_size is None else batch_size
        w = next(self.parameters())
        z = w.new_zeros(self.num_layers, b, self.embedding_dim)
        return (z, z.clone())

    def forward(self, inputs, hidden):
        embeds = self.dropout(self.word_embeddings(inputs))
        out, hidden = self.lstm(embeds, hidden)
        out = self.dropout(out)
        logits = self.sm_fc(out.reshape(-1, self.embedding_dim))
        return logits.view(inputs.shape[0], inputs.shape[1], self.vocab_size), hidden


def repackage_hidden(h):
    """Detach hidden states from their history (reference models/lstm.py:44-47)."""
    if isinstance(h, torch.Tensor):
        return h.detach()
    return tuple(repackage_hidden(v) for v in h)


def lstm(vocab_size=10000, batch_size=20, **kw):
    return PTBLSTM(vocab_size=vocab_size, batch_size=batch_size, **kw)
