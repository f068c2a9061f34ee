"""Fused BERT input embedding (``csrc/kernels/embed.hip``).

``bert_embeddings(ids, tt, word, pos, ttype)`` = ``word(ids) + pos(arange(T))
+ ttype(tt)`` -- the three ``nn.Embedding`` lookups of the BERT input layer
(fp32 [B, T, H]).  On the GPU it is one HIP pass forward and, backward, a
bucketed row gather (word table), a batch sum (positions) and a fixed-order
per-type reduction (token types) instead of PyTorch's three sort-based
``embedding_dense_backward`` passes.  The word-table gradient is a stable
sort of the ids plus gather-sums (64-token chunks for frequent ids, then one
wave per vocabulary row), in ascending token order: deterministic;
``torch.use_deterministic_algorithms(True)`` or ``GKSGD_FUSED_EMB=0`` keeps
the PyTorch path.  Elsewhere (CPU, no
extension, non-fp32 tables, padding_idx / max_norm) it is the plain
composition.  The ``nn.Embedding`` modules and their state_dict keys are
untouched.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import load

_ENABLED = os.environ.get("GKSGD_FUSED_EMB", "1") != "0"


def _ops():
    return torch.ops.gksgd


class _EmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, Ww, Wp, Wt):
        B, T = ids.shape
        H = Ww.shape[1]
        out = torch.empty(B, T, H, dtype=torch.float32, device=ids.device)
        _ops().emb_forward(ids, tt, Ww.detach(), Wp.detach(), Wt.detach(), out)
        ctx.save_for_backward(ids, tt if tt is not None else torch.empty(0, dtype=torch.long, device=ids.device))
        ctx.has_tt = tt is not None
        ctx.shapes = (Ww.shape, Wp.shape, Wt.shape)
        return out

    @staticmethod
    def backward(ctx, dx):
        ids, tt = ctx.saved_tensors
        tt = tt if ctx.has_tt else None
        sw, sp, st = ctx.shapes
        dev = dx.device
        dx = dx.float().contiguous()
        # every row of dWw is written by the counting-sort gather (no zero fill)
        dWw = torch.empty(sw, dtype=torch.float32, device=dev) if ctx.needs_input_grad[2] else None
        dWp = torch.empty(sp, dtype=torch.float32, device=dev) if ctx.needs_input_grad[3] else None
        dWt = torch.empty(st, dtype=torch.float32, device=dev) if ctx.needs_input_grad[4] else None
        part = torch.empty(_ops().emb_part_floats(sw[1]), dtype=torch.float32, device=dev)
        M = ids.numel()
        if dWw is not None:
            sid, order = torch.sort(ids.reshape(-1), stable=True)   # rocprim radix sort: ids bucketed, positions ascending
        else:
            sid = order = ids.reshape(-1)
        wws = torch.empty(_ops().emb_word_ws_ints(sw[0], M), dtype=torch.int32, device=dev)
        wpart = torch.empty(_ops().emb_word_part_floats(M, sw[1]), dtype=torch.float32, device=dev)
        _ops().emb_backward(ids, tt, dx, dWw, dWp, dWt, part, sid, order, wws, wpart)
        return None, None, dWw, dWp, dWt


def _plain(m: nn.Embedding) -> bool:
    return (m.padding_idx is None and m.max_norm is None and not m.scale_grad_by_freq and not m.sparse and
            m.weight.dtype == torch.float32)


def fused_available(ids: torch.Tensor, word: nn.Embedding, pos: nn.Embedding, ttype: nn.Embedding) -> bool:
    if not (_ENABLED and ids.is_cuda and ids.dim() == 2 and load()):
        return False
    if torch.are_deterministic_algorithms_enabled():
        return False
    if not all(_plain(m) for m in (word, pos, ttype)):
        return False
    H = word.weight.shape[1]
    if not (pos.weight.shape[1] == H and ttype.weight.shape[1] == H and ids.shape[1] <= pos.weight.shape[0]):
        return False
    try:
        return bool(_ops().emb_supported(H, ttype.weight.shape[0]))
    except (AttributeError, RuntimeError):   # an extension built before embed.hip
        return False


def bert_embeddings(ids: torch.Tensor, tt, word: nn.Embedding, pos: nn.Embedding, ttype: nn.Embedding) -> torch.Tensor:
    """word(ids) + pos(arange(T)) + ttype(tt) (tt None: type 0 everywhere)."""
    if fused_available(ids, word, pos, ttype):
        ids_c = ids.contiguous().long()
        tt_c = tt.contiguous().long() if tt is not None else None
        return _EmbFn.apply(ids_c, tt_c, word.weight, pos.weight, ttype.weight)
    T = ids.shape[1]
    p = torch.arange(T, device=ids.device).unsqueeze(0)
    t = tt if tt is not None else torch.zeros_like(ids)
    return word(ids) + pos(p) + ttype(t)
