"""Optimizers: LARS (lars.py parity) and the SGD parameter-group helper of the
reference trainer (dl_trainer.py:212-228)."""
from __future__ import annotations

from typing import List

import torch

from .lars import LARS


def sgd_param_groups(net: torch.nn.Module, weight_decay: float) -> List[dict]:
    """No weight decay on 1-D tensors, batch-norm and bias parameters."""
    decay, no_decay = [], []
    for name, param in net.named_parameters():
        if not param.requires_grad:
            continue
        if len(param.shape) == 1 or "bn" in name or "bias" in name:
            no_decay.append(param)
        else:
            decay.append(param)
    return [{"params": no_decay, "weight_decay": 0.0}, {"params": decay, "weight_decay": weight_decay}]


__all__ = ["LARS", "sgd_param_groups"]
