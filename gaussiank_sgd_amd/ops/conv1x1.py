"""Stride-1 1x1 convolution on channels-last bf16 activations through the
MFMA GEMMs of ``csrc/kernels/gemm.hip``, autotuned per shape against MIOpen.

A 1x1 convolution over NHWC data is a GEMM over the ``M = N*H*W`` pixel rows
(forward ``Y = X W^T``, grad-input ``dX = dY W``, grad-weight
``dW += dY^T X``).  For every distinct (direction, M, Cin, Cout) the first
call times a small set of kernel configurations *and* the MIOpen
convolution with HIP events and keeps the fastest (``GKSGD_GEMM_TUNE=0``
skips the search and uses the heuristic default of the HIP kernel).  The
grad-weight kernel adds its fp32 result straight into the optimizer's
gradient arena (float atomics) when the module is on the bf16-shadow path
(``parallel/shadow.py``), so no bf16 weight gradient is materialised.

Reference parity: the reference's ResNets use ``nn.Conv2d(k=1)``
(models/resnet.py / torchvision Bottleneck); ``Conv1x1`` is a drop-in
``nn.Conv2d`` subclass with identical parameters and state_dict keys.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import load

_CL = torch.channels_last
_TUNE = os.environ.get("GKSGD_GEMM_TUNE", "1") != "0"
_choices: Dict[tuple, tuple] = {}
# candidate kernel configurations (see gemm.hip: cfg digits = tile + 10*panel + 100*stages)
_NT_CFGS = [0, 1, 2, 3, 4, 11, 13, 21, 22, 23, 24, 111, 113, 121, 122, 123, 124]
_TN_CFGS = [(c, s) for c in (0, 1, 2, 3, 4, 5, 6, 21, 24, 25) for s in (0, 64, 256)]


def _g():
    return torch.ops.gksgd


def _time(fn: Callable[[], None], reps: int = 5) -> float:
    fn()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def _pick(key: tuple, cands: List[Tuple[tuple, Callable[[], None]]]) -> tuple:
    """Fastest candidate for ``key`` (timed once per process, then cached)."""
    got = _choices.get(key)
    if got is not None:
        return got
    if not _TUNE or len(cands) == 1:
        _choices[key] = cands[0][0]
        return cands[0][0]
    best, best_t = None, float("inf")
    for tag, fn in cands:
        try:
            t = _time(fn)
        except RuntimeError:
            continue
        if t < best_t:
            best, best_t = tag, t
    _choices[key] = best
    return best


def tuned_choices() -> Dict[tuple, tuple]:
    """(direction, M, Cin, Cout) -> chosen (impl, cfg, grid/splits)."""
    return dict(_choices)


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and conv.stride == (1, 1) and conv.padding == (0, 0)
            and conv.groups == 1 and conv.bias is None and x.is_contiguous(memory_format=_CL)
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0 and x.shape[0] * x.shape[2] * x.shape[3] > 0)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels-last -> [N*H*W, C] view."""
    N, C, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(N * H * W, C)


def _fwd(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    N, C, H, W = x.shape
    K = w.shape[0]
    M = N * H * W
    y = torch.empty((N, K, H, W), dtype=torch.bfloat16, device=x.device, memory_format=_CL)
    X, Y, Wm = _rows(x), _rows(y), w.reshape(K, C)
    g = _g()
    cands = [(("hip", c, 0), (lambda c=c: g.gemm_nt(X, Wm, Y, c, 0))) for c in _NT_CFGS]
    cands.append((("miopen", 0, 0), lambda: F.conv2d(x, w)))
    ch = _pick(("fwd", M, C, K), cands)
    if ch[0] == "miopen":
        return F.conv2d(x, w).contiguous(memory_format=_CL)
    g.gemm_nt(X, Wm, Y, ch[1], ch[2])
    return y


def _dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape) -> torch.Tensor:
    N, C, H, W = x_shape
    K = w.shape[0]
    M = N * H * W
    dx = torch.empty((N, C, H, W), dtype=torch.bfloat16, device=dy.device, memory_format=_CL)
    DY, DX = _rows(dy), _rows(dx)
    Wt = w.reshape(K, C).t().contiguous()
    g = _g()

    def miopen():
        return torch.ops.aten.convolution_backward(dy, dx, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                   [True, False, False])[0]
    cands = [(("hip", c, 0), (lambda c=c: g.gemm_nt(DY, Wt, DX, c, 0))) for c in _NT_CFGS]
    cands.append((("miopen", 0, 0), miopen))
    ch = _pick(("dgrad", M, C, K), cands)
    if ch[0] == "miopen":
        return miopen().contiguous(memory_format=_CL)
    g.gemm_nt(DY, Wt, DX, ch[1], ch[2])
    return dx


def _wgrad_into(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, out_f32: torch.Tensor) -> None:
    """out_f32[K, C] += dW (fp32)."""
    N, C, H, W = x.shape
    K = w.shape[0]
    M = N * H * W
    DY, X = _rows(dy), _rows(x)
    g = _g()
    scratch = torch.zeros(K, C, dtype=torch.float32, device=x.device)

    def miopen():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                   [False, True, False])[1]
    cands = [(("hip", c, s), (lambda c=c, s=s: g.gemm_tn_acc(DY, X, scratch, c, s))) for c, s in _TN_CFGS]
    cands.append((("miopen", 0, 0), miopen))
    ch = _pick(("wgrad", M, C, K), cands)
    if ch[0] == "miopen":
        from . import accum_grad_
        accum_grad_(out_f32, miopen().reshape(K, C))
        return
    g.gemm_tn_acc(DY, X, out_f32, ch[1], ch[2])


class _Conv1x1Fn(torch.autograd.Function):
    """y = conv1x1(x, w_bf16).  ``param`` is the fp32 master weight; with a
    ``sink`` (bf16-shadow path) its gradient is added into the optimizer's
    fp32 arena in the backward and None is returned for it."""

    @staticmethod
    def forward(ctx, x, param, w_bf16, sink):
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        x = x.contiguous(memory_format=_CL)
        w = w_bf16 if w_bf16 is not None else param.detach().to(torch.bfloat16)
        w = w.contiguous(memory_format=_CL)
        y = _fwd(x, w)
        ctx.sink = sink
        ctx.param_dtype = param.dtype
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=_CL)
        dx = _dgrad(dy, w, x.shape) if ctx.needs_input_grad[0] else None
        gparam = None
        if ctx.needs_input_grad[1]:
            K, C = w.shape[0], w.shape[1]
            sink = ctx.sink
            if sink is not None and getattr(sink, "grad_view", None) is not None:
                sink.check()
                _wgrad_into(dy, x, w, sink.grad_view.view(K, C))
            else:
                out = torch.zeros(K, C, dtype=torch.float32, device=x.device)
                _wgrad_into(dy, x, w, out)
                gparam = out.view(K, C, 1, 1).to(ctx.param_dtype)
        return dx, gparam, None, None


class Conv1x1(nn.Conv2d):
    """``nn.Conv2d(in, out, 1, stride, bias=False)`` whose stride-1 training
    path on a GPU runs the autotuned MFMA GEMMs (bf16 compute, as autocast)."""

    def __init__(self, inp: int, out: int, stride: int = 1):
        super().__init__(inp, out, 1, stride=stride, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        dev = x.device.type
        bf16 = x.dtype == torch.bfloat16 or (torch.is_autocast_enabled(dev) and
                                             torch.get_autocast_dtype(dev) == torch.bfloat16)
        if bf16 and supported(x, self) and load():
            table = getattr(self, "_gk_shadow", None)
            info = table.get("weight") if table else None
            use_shadow = info is not None and torch.is_autocast_enabled(dev)
            w_bf16, sink = (info[0], info[1]) if use_shadow else (None, None)
            if not torch.is_grad_enabled() or not self.weight.requires_grad:
                sink = None
            return _Conv1x1Fn.apply(x, self.weight, w_bf16, sink)
        slow = getattr(self, "_gk_slow", None)
        return slow(x) if slow is not None else super().forward(x)
