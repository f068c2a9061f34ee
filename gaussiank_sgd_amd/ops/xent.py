"""Fused softmax cross-entropy on bf16 logits (``csrc/kernels/xent.hip``).

``cross_entropy(logits, labels, ignore_index=-100)`` == ``F.cross_entropy(
logits.float(), labels, ignore_index=ignore_index)`` (mean over the counted
rows).  On the GPU with bf16 logits it is one HIP row pass forward (max,
sum of exp, the row's log-sum-exp kept) and one backward that writes the bf16
logit gradient ``(softmax - onehot) / count`` directly -- no fp32 copy of the
logits, no separate log_softmax / nll / cast kernels.  Elsewhere it is the
PyTorch call.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import load

_ENABLED = os.environ.get("GKSGD_FUSED_XENT", "1") != "0"


def _ops():
    return torch.ops.gksgd


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore):
        R = logits.shape[0]
        lse = torch.empty(R, dtype=torch.float32, device=logits.device)
        loss_r = torch.empty(R, dtype=torch.float32, device=logits.device)
        _ops().xent_forward(logits, labels, lse, loss_r, int(ignore))
        count = (labels != ignore).sum().clamp_(min=1).float()
        ctx.save_for_backward(logits, labels, lse, count)
        ctx.ignore = int(ignore)
        return loss_r.sum() / count

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, count = ctx.saved_tensors
        scale = (g.float() / count).reshape(1)   # device scalar: no host sync
        grad = torch.empty_like(logits)
        _ops().xent_backward(logits, labels, lse, scale, grad, ctx.ignore)
        return grad, None, None


def fused_available(logits: torch.Tensor) -> bool:
    if not (_ENABLED and logits.is_cuda and logits.dtype == torch.bfloat16 and load()):
        return False
    try:
        return bool(_ops().xent_supported(logits.shape[-1]))
    except (AttributeError, RuntimeError):   # an extension built before xent.hip
        return False


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    V = logits.shape[-1]
    if fused_available(logits):
        return _XentFn.apply(logits.reshape(-1, V).contiguous(), labels.reshape(-1).long().contiguous(), ignore_index)
    return F.cross_entropy(logits.reshape(-1, V).float(), labels.reshape(-1), ignore_index=ignore_index)
