"""Fused residual add + dropout + LayerNorm (``csrc/kernels/ln.hip``).

``add_layernorm(a, x, ln, p)`` computes ``ln(x + dropout_p(a))`` -- the
post-LN transformer sub-layer output (BERT: ``LN(x + drop(attn_out))`` and
``LN(x + drop(ffn_out))``).  On a GPU it is one HIP row pass forward and one
backward (plus a small dgamma / dbeta finalize), with bf16 row tensors under
autocast and fp32 ones at the reference's precision (``GKSGD_LN_F32=0``
keeps PyTorch there); the dropout mask is a hash of (seed, row, column),
regenerated in the backward instead of stored.  Elsewhere (CPU) it is the
plain PyTorch composition with identical semantics.  ``ln`` is an ordinary
``nn.LayerNorm`` (its parameters / state_dict keys are untouched).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import capture_seed_word, load, seed_generator


def _ops():
    return torch.ops.gksgd


class _AddLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, x, gamma, beta, eps, p, seed, direct=None, seed_dev=None, cd=torch.bfloat16):
        # direct = (dgamma_view, dbeta_view): fp32 gradient-arena views the
        # backward kernel accumulates into (bf16-shadow path); None is then
        # returned for gamma / beta, so AccumulateGrad launches nothing.
        # cd: storage dtype of the row tensors -- bf16 under autocast, fp32 at
        # the reference's precision (same kernels, fp32 math either way)
        H = x.shape[-1]
        a = a.to(cd).contiguous()
        x = x.to(cd).contiguous()
        R = x.numel() // H
        y = torch.empty_like(x)
        h = torch.empty_like(x)
        mean = torch.empty(R, dtype=torch.float32, device=x.device)
        rstd = torch.empty(R, dtype=torch.float32, device=x.device)
        g = gamma.detach().float().contiguous() if gamma is not None else None
        b = beta.detach().float().contiguous() if beta is not None else None
        _ops().add_ln_forward(a, x, g, b, y, h, mean, rstd, float(eps), float(p), int(seed), seed_dev)
        ctx.save_for_backward(h, mean, rstd, g if g is not None else torch.empty(0, device=x.device))
        ctx.p, ctx.seed, ctx.seed_dev = float(p), int(seed), seed_dev
        ctx.has_g, ctx.has_b = gamma is not None, beta is not None
        ctx.gdtype = gamma.dtype if gamma is not None else torch.float32
        ctx.direct = direct
        return y

    @staticmethod
    def backward(ctx, dy):
        h, mean, rstd, g = ctx.saved_tensors
        H = h.shape[-1]
        R = h.numel() // H
        dy = dy.to(h.dtype).contiguous()
        dx = torch.empty_like(h)
        da = torch.empty_like(h) if ctx.p > 0 else None
        direct = ctx.direct
        if direct is not None:
            dg, db = direct
        else:
            dg = torch.empty(H, dtype=torch.float32, device=h.device) if ctx.has_g and ctx.needs_input_grad[2] else None
            db = torch.empty(H, dtype=torch.float32, device=h.device) if ctx.has_b and ctx.needs_input_grad[3] else None
        ws = torch.empty(int(_ops().add_ln_ws_floats(R, H)), dtype=torch.float32, device=h.device)
        _ops().add_ln_backward(dy, h, mean, rstd, g if ctx.has_g else None, dx, da, dg, db, direct is not None, ws,
                               ctx.p, ctx.seed, ctx.seed_dev)
        if da is None:
            da = dx
        if direct is not None:
            return da, dx, None, None, None, None, None, None, None, None
        return (da, dx, dg.to(ctx.gdtype) if dg is not None else None,
                db.to(ctx.gdtype) if db is not None else None, None, None, None, None, None, None)


def _compute_dtype(x: torch.Tensor):
    """Storage dtype of the fused path for ``x`` (None: PyTorch composition)."""
    dev = x.device.type
    if x.dtype == torch.bfloat16 or (torch.is_autocast_enabled(dev) and
                                     torch.get_autocast_dtype(dev) == torch.bfloat16):
        return torch.bfloat16
    if x.dtype == torch.float32 and not torch.is_autocast_enabled(dev) and os.environ.get("GKSGD_LN_F32", "1") != "0":
        return torch.float32
    return None


def fused_available(x: torch.Tensor) -> bool:
    if not x.is_cuda or _compute_dtype(x) is None:
        return False
    return load() and bool(_ops().add_ln_supported(x.shape[-1]))


def add_layernorm(a: torch.Tensor, x: torch.Tensor, ln: nn.LayerNorm, p: float = 0.0,
                  training: bool = True) -> torch.Tensor:
    """``ln(x + dropout_p(a))`` (dropout only when ``training``)."""
    p = float(p) if training else 0.0
    if (fused_available(x) and ln.elementwise_affine and len(ln.normalized_shape) == 1 and
            a.shape == x.shape):
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,), generator=seed_generator())) if p > 0 else 0
        direct = getattr(ln, "_gk_direct", None)
        if direct is not None and not (torch.is_grad_enabled() and ln.weight.requires_grad and ln.bias.requires_grad):
            direct = None
        return _AddLNFn.apply(a, x, ln.weight, ln.bias, ln.eps, p, seed, direct,
                              capture_seed_word(x.device) if p > 0 else None, _compute_dtype(x))
    return ln(x + F.dropout(a, p, training=p > 0))
