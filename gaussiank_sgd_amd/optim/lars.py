"""Layer-wise adaptive rate scaling (You, Gitman & Ginsburg, 2017).

Parity: reference ``lars.py:6-134`` -- trust ratio
``eeta*||w|| / (||g|| + wd*||w|| + eps)`` (1 when either norm is 0) clamped to
[0, 50]; decayed gradient ``g + wd*w`` clamped to +-10; the acceleration
buffer starts at ONES (lars.py:116-118); update ``w -= acc`` with
``acc = momentum*acc + lr*trust*d``.

``step()`` below is the portable per-tensor implementation; wrapped by
``DistributedOptimizer`` on a GPU the whole model is updated by two fused HIP
launches instead (segmented norms + fused update, ``ops.fused_lars_``).
"""
from __future__ import annotations

import torch
from torch.optim.optimizer import Optimizer


class LARS(Optimizer):
    def __init__(self, params, lr=0.1, momentum=0.9, weight_decay=0.0005, eeta=0.0001, epsilon=1e-5,
                 max_epoch=200):
        if lr < 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if momentum < 0.0:
            raise ValueError("Invalid momentum value: {}".format(momentum))
        if weight_decay < 0.0:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        if eeta < 0.0:
            raise ValueError("Invalid LARS coefficient value: {}".format(eeta))
        defaults = dict(lr=lr, momentum=momentum, weight_decay=weight_decay, eeta=eeta, epsilon=epsilon,
                        max_epoch=max_epoch)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr = group["lr"]
            momentum = group["momentum"]
            wd = group["weight_decay"]
            eeta = group["eeta"]
            eps = group["epsilon"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                w = p.data
                g = p.grad.data
                wn = torch.linalg.vector_norm(w)
                gn = torch.linalg.vector_norm(g)
                one = torch.ones_like(wn)
                trust = torch.where(wn > 0, torch.where(gn > 0, eeta * wn / (gn + wd * wn + eps), one), one)
                trust = trust.clamp(0.0, 50.0)
                d = (g + wd * w).clamp_(-10.0, 10.0)
                st = self.state[p]
                if "acceleration" not in st:
                    st["acceleration"] = torch.ones_like(w)
                acc = st["acceleration"]
                acc.mul_(momentum).add_(d * (lr * trust))
                w.sub_(acc)
        return loss
