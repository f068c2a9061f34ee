"""Fused BatchNorm2d (+ residual add) (+ ReLU) for channels-last activations.

``BNAct`` is a drop-in ``nn.BatchNorm2d`` (same parameters, buffers and
state_dict keys) whose ``forward(x, residual=None)`` computes
``act(bn(x) + residual)``.  In training mode on the GPU, with a
channels-last bf16/fp32 input, it runs the gfx950 kernels of
``csrc/kernels/bn_act.hip`` (3 launches forward, 3 backward, ReLU mask and
residual gradient folded into the BN passes; the ReLU mask is kept as one
bit per element instead of saving the output).  Everywhere else (CPU, eval,
NCHW input) it falls back to ``F.batch_norm`` + add + relu with identical
semantics, so models built with it run anywhere.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import load, require_native

_CL = torch.channels_last


def _ops():
    return torch.ops.gksgd


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, momentum, eps, relu, direct=None):
        # direct = (gw_view, gb_view): weight/bias gradients are accumulated
        # straight into the optimizer's fp32 arena by the backward kernel and
        # None is returned for them, so AccumulateGrad launches nothing (its
        # post-accumulate hook still fires and reports readiness).
        ctx.direct = direct
        C = x.shape[1]
        M = x.numel() // C
        eb = x.element_size()
        y = torch.empty_like(x, memory_format=_CL)
        stats = torch.empty(4, C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, eb)), dtype=torch.float32, device=x.device)
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        if residual is not None and not residual.is_contiguous(memory_format=_CL):
            residual = residual.contiguous(memory_format=_CL)
        mask = None
        if relu:
            mask = torch.empty(int(_ops().bn_mask_bytes(M, C, eb)), dtype=torch.uint8, device=x.device)
        _ops().bn_act_forward(x, residual, y, mask, weight, bias, running_mean, running_var, stats[0], stats[1],
                              stats[2], stats[3], ws, float(eps), float(momentum), bool(relu))
        ctx.relu = bool(relu)
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, mask, weight, stats[0], stats[1])
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd = ctx.saved_tensors
        C = x.shape[1]
        M = x.numel() // C
        dy = dy.contiguous(memory_format=_CL)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        dx = torch.empty_like(x, memory_format=_CL)
        dres = torch.empty_like(x, memory_format=_CL) if ctx.has_res else None
        g = torch.empty(2, C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, x.element_size())), dtype=torch.float32,
                         device=x.device)
        if ctx.direct is not None:
            gw, gb = ctx.direct
            _ops().bn_act_backward(dy, mask, x, dx, dres, weight, mean, invstd, g[0], g[1], ws, ctx.relu, gw, gb)
            return dx, dres, None, None, None, None, None, None, None, None
        _ops().bn_act_backward(dy, mask, x, dx, dres, weight, mean, invstd, g[0], g[1], ws, ctx.relu)
        dgamma = g[0] if weight is not None and ctx.needs_input_grad[2] else None
        dbeta = g[1] if ctx.needs_input_grad[3] else None
        return dx, dres, dgamma, dbeta, None, None, None, None, None, None


_supported_cache = {}


def fused_bn_available(x: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32)):
        return False
    if not x.is_contiguous(memory_format=_CL):
        return False
    key = (x.shape[1], x.element_size())
    ok = _supported_cache.get(key)
    if ok is None:
        if not load():
            require_native(x)
        ok = bool(_ops().bn_supported(x.shape[1], x.element_size()))
        _supported_cache[key] = ok
    return ok


class BNAct(nn.BatchNorm2d):
    """BatchNorm2d with optional fused residual add and ReLU."""

    def __init__(self, num_features: int, act: Optional[str] = None, eps: float = 1e-5, momentum: float = 0.1,
                 affine: bool = True, track_running_stats: bool = True, fused: bool = True):
        super().__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                         track_running_stats=track_running_stats)
        assert act in (None, "relu")
        self.act = act
        self.fused = fused

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        relu = self.act == "relu"
        if self.training and self.fused and self.track_running_stats and fused_bn_available(x):
            if self.num_batches_tracked is not None:
                self.num_batches_tracked.add_(1)
            if self.momentum is None:
                mom = 1.0 / float(self.num_batches_tracked)
            else:
                mom = self.momentum
            direct = getattr(self, "_gk_direct", None)
            return _BNActFn.apply(x, residual, self.weight, self.bias, self.running_mean, self.running_var, mom,
                                  self.eps, relu, direct)
        out = super().forward(x)
        if residual is not None:
            out = out + residual
        if relu:
            out = F.relu(out)
        return out

    def extra_repr(self) -> str:
        return super().extra_repr() + ", act=%s" % self.act
