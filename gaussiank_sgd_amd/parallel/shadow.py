"""bf16 shadow weights + direct-to-arena gradients (mixed precision "O2" on MI355X).

Under bf16 autocast, every step PyTorch (a) casts each fp32 conv/linear
weight to bf16 in forward, (b) casts each bf16 weight gradient back to fp32
in backward and (c) adds it into ``p.grad`` with a separate AccumulateGrad
kernel -- three small launches per parameter, ~1.5 ms per ResNet-50 step on
MI355X (profiles/r01_resnet50_bs256_fusedbn_kernel_stats.csv).

``install_bf16_shadow`` removes all three:
  * the fused SGD kernel writes a bf16 copy of the new weights ("shadow
    arena") in the same pass that updates the fp32 master weights, and
    conv/linear modules compute with views of that shadow arena;
  * the shadow view's backward accumulates the bf16 gradient straight into
    the fp32 gradient arena (one fused cast+add kernel) and returns None for
    the fp32 parameter, so AccumulateGrad launches nothing; its
    post-accumulate hook still fires afterwards and reports the parameter
    ready to the bucket engine exactly as on the plain path;
  * ``BNAct`` modules get the same direct path for gamma/beta: the BN backward
    kernel adds them into the arena; so do LayerNorms used through
    ``ops/ln.py add_layernorm`` (the fused add+LN backward accumulates them).
Outside bf16 autocast modules fall back to their fp32 parameters, so the
model stays usable for fp32 evaluation.  (CPU autocast works too -- the ops
have PyTorch fallbacks -- which is how the CPU tests check the wiring.)
"""
from __future__ import annotations

import types

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.bn import BNAct
from ..ops.conv1x1 import FastConv2d
from ..ops.linear import FastLinear
from ..ops.lstm import GkLSTM
from ..ops.stem import StemConv


class _ShadowWeight(torch.autograd.Function):
    @staticmethod
    def forward(ctx, param, shadow, sink):
        ctx.sink = sink
        return shadow.view_as(shadow)

    @staticmethod
    def backward(ctx, grad):
        ctx.sink(grad)
        return None, None, None


def _shadow(module: nn.Module, name: str, x: torch.Tensor):
    info = module._gk_shadow.get(name)
    p = getattr(module, name)
    dev = x.device.type
    if info is None or not torch.is_autocast_enabled(dev) or torch.get_autocast_dtype(dev) != torch.bfloat16:
        return p
    shadow, sink = info
    if torch.is_grad_enabled() and p.requires_grad:
        return _ShadowWeight.apply(p, shadow, sink)
    return shadow


def _conv_forward(self, x):
    w = _shadow(self, "weight", x)
    b = _shadow(self, "bias", x) if self.bias is not None else None
    return self._conv_forward(x, w, b)


def _linear_forward(self, x):
    w = _shadow(self, "weight", x)
    b = _shadow(self, "bias", x) if self.bias is not None else None
    return F.linear(x, w, b)


def _mark_shared_sinks(model: nn.Module) -> None:
    """A parameter that several modules hold (tied weights) has its gradient
    accumulated by each of them into the same arena view: such sinks are
    flagged ``shared`` so their grad-weight is never forked onto the side
    stream (ops/streams.py), where it could race the other module's
    accumulation on the main stream."""
    uses = {}
    for m in model.modules():
        for p in m.parameters(recurse=False):
            uses[id(p)] = uses.get(id(p), 0) + 1
    for m in model.modules():
        for attr in ("_gk_shadow", "_gk_direct_grads"):
            table = getattr(m, attr, None)
            if not table:
                continue
            for pname, entry in table.items():
                sink = entry[1] if isinstance(entry, tuple) else entry
                p = getattr(m, pname, None)
                sink.shared = p is not None and uses.get(id(p), 0) > 1


def install_bf16_shadow(model: nn.Module, opt) -> int:
    """Attach the shadow path to ``model``'s Conv2d / Linear / BNAct modules.

    ``opt`` is the DistributedOptimizer owning the arenas.  Returns the number
    of parameters that now bypass AccumulateGrad.
    """
    arena = opt.arena
    shadow = opt._ensure_shadow()
    names = opt._parameter_names
    count = 0
    for mod in model.modules():
        if isinstance(mod, (FastConv2d, FastLinear, StemConv)):
            # its own forward reads the shadow view and (GEMM path) adds the fp32
            # weight / bias gradients straight into the arena; unsupported
            # shapes fall back to the plain shadow conv / linear
            table = {}
            for pname in ("weight", "bias"):
                p = getattr(mod, pname, None)
                if p is not None and p in names:
                    key = names[p]
                    table[pname] = (arena.view_of(shadow, key), opt._make_sink(key))
                    count += 1
            if table:
                mod._gk_shadow = table
                mod._gk_slow = types.MethodType(_conv_forward if isinstance(mod, nn.Conv2d) else _linear_forward,
                                                mod)
        elif isinstance(mod, (nn.Conv2d, nn.Linear)) and type(mod).forward in (nn.Conv2d.forward, nn.Linear.forward):
            table = {}
            for pname in ("weight", "bias"):
                p = getattr(mod, pname, None)
                if p is None or p not in names:
                    continue
                key = names[p]
                table[pname] = (arena.view_of(shadow, key), opt._make_sink(key))
                count += 1
            if table:
                mod._gk_shadow = table
                mod.forward = types.MethodType(_conv_forward if isinstance(mod, nn.Conv2d) else _linear_forward, mod)
        elif isinstance(mod, GkLSTM):
            # bf16 weight views for its GEMMs; its backward adds every weight /
            # bias gradient straight into the arena
            table = {}
            for pname, p in mod.named_parameters(recurse=False):
                if p in names:
                    key = names[p]
                    table[pname] = (arena.view_of(shadow, key), opt._make_sink(key))
                    count += 1
            if table:
                mod._gk_shadow = table
        elif isinstance(mod, nn.LayerNorm) and mod.elementwise_affine and mod.bias is not None:
            # ops/ln.py add_layernorm: the fused backward accumulates dgamma /
            # dbeta straight into the arena (plain ln(x) calls ignore this)
            if mod.weight in names and mod.bias in names:
                mod._gk_direct = (arena.grad_views[names[mod.weight]], arena.grad_views[names[mod.bias]])
                count += 2
        elif isinstance(mod, BNAct) and mod.affine:
            if mod.weight in names and mod.bias in names:
                kw, kb = names[mod.weight], names[mod.bias]
                mod._gk_direct = (arena.grad_views[kw], arena.grad_views[kb])
                count += 2
    _mark_shared_sinks(model)
    opt.refresh_shadow()
    if not getattr(model, "_gk_shadow_hooked", False):
        # model.load_state_dict copies into the fp32 arena: keep the shadow in sync
        model.register_load_state_dict_post_hook(lambda m, keys: opt.refresh_shadow())
        model._gk_shadow_hooked = True
    return count


def install_direct_grads(model: nn.Module, opt) -> int:
    """fp32 counterpart of ``install_bf16_shadow`` (the reference's precision:
    fp32 weights, activations and gradients, settings.py:28): no shadow
    weights, but the hand-written kernels add their weight gradients straight
    into the optimizer's fp32 gradient arena -- FastConv2d's grad-weight GEMM
    (ops/conv1x1.py fp32 path), FastLinear's (ops/linear.py fp32 path), the
    fp32 stem (ops/stem.py), the LSTM (ops/lstm.py), the fused add + LayerNorm
    (ops/ln.py) and BNAct's backward (gamma / beta) -- so
    AccumulateGrad launches nothing for them.  Returns the number of
    parameters on the direct path."""
    arena = opt.arena
    names = opt._parameter_names
    count = 0
    for mod in model.modules():
        if isinstance(mod, (FastConv2d, StemConv, FastLinear)):
            table = {}
            for pname in ("weight", "bias"):
                p = getattr(mod, pname, None)
                if p is not None and p in names:
                    table[pname] = opt._make_sink(names[p])
                    count += 1
            if table:
                mod._gk_direct_grads = table
        elif isinstance(mod, BNAct) and mod.affine:
            if mod.weight in names and mod.bias in names:
                mod._gk_direct = (arena.grad_views[names[mod.weight]], arena.grad_views[names[mod.bias]])
                count += 2
        elif isinstance(mod, nn.LayerNorm) and mod.elementwise_affine and mod.bias is not None:
            # fp32 fused add + LayerNorm (ops/ln.py): dgamma / dbeta into the arena
            if mod.weight in names and mod.bias in names:
                mod._gk_direct = (arena.grad_views[names[mod.weight]], arena.grad_views[names[mod.bias]])
                count += 2
        elif isinstance(mod, GkLSTM):
            # fp32 GkLSTM (ops/lstm.py): its backward adds every weight / bias
            # gradient straight into the arena
            table = {}
            for pname, p in mod.named_parameters(recurse=False):
                if p in names:
                    table[pname] = opt._make_sink(names[p])
                    count += 1
            if table:
                mod._gk_direct_grads = table
    _mark_shared_sinks(model)
    return count
