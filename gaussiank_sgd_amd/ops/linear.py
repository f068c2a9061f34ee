"""Linear layers on bf16 activations through the MFMA GEMMs of
``csrc/kernels/gemm.hip`` (autotuned per shape against hipBLASLt), with the
bias gradient -- and, for ``act="gelu"``, the GELU backward -- in ONE fused
HIP column pass (``csrc/kernels/linear.hip``) that adds straight into the
optimizer's fp32 gradient arena.

A linear layer over the M = prod(x.shape[:-1]) rows is the GEMM of a 1x1
convolution over NHWC pixel rows (ops/conv1x1.py):

  forward      y[M, N]  = x[M, K] . W[N, K]^T (+ b in the epilogue)   gemm_nt
  grad-input   dx[M, K] = dy[M, N] . Wt[K, N]^T                       gemm_nt (Wt = W^T)
  grad-weight  dW[N, K] += dy[M, N]^T . x[M, K]  (fp32 atomics)       gemm_tn_acc
  grad-bias    db[N]   += sum_m dy[m, :]                             colsum_acc

Each (direction, M, K, N) times the HIP kernel configurations and
``torch.addmm`` / ``torch.mm`` (hipBLASLt) once per process and keeps the
fastest (cache and switches shared with the convolutions: ``GKSGD_GEMM_TUNE``,
``tuning/gemm_choices.json``; ``GKSGD_FASTLINEAR=0`` disables the path).
Dimensions that are not multiples of 64 (the LSTM's 1500 -> 10000 softmax
layer, BERT's vocabulary) also offer the HIP kernels on zero-padded operands
(timed with their copies against hipBLASLt, ``_fwd_padded``).
``FastLinear`` is a drop-in ``nn.Linear`` (same parameters and state_dict
keys).  fp32 inputs without autocast (the reference's precision) take the same
path on the fp32 MFMA kernels (``v_mfma_f32_16x16x4_f32``) and the fp32 column
pass; off the GPU it is the stock layer (+ ``F.gelu``).

Reference parity: the reference's models use ``nn.Linear`` (models/fcn.py,
models/lstm.py:29); BERT is not in the reference (BASELINE config 5).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import accum_grad_, load, require_native
from . import conv1x1 as _cv
from . import streams

_ENABLED = os.environ.get("GKSGD_FASTLINEAR", "1") != "0"


def _g():
    return torch.ops.gksgd


def _colsum_ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.dim() == 2 and t.is_contiguous() and
            t.shape[1] % 8 == 0 and t.data_ptr() % 16 == 0)


def bias_grad_acc_(db: torch.Tensor, dy: torch.Tensor) -> None:
    """db (fp32 [N]) += dy.sum(0) for a 2-D [M, N] gradient."""
    if _colsum_ok(dy) and db.dtype == torch.float32 and db.is_contiguous():
        require_native(dy)
        _g().colsum_acc(dy, db)
    else:
        db.add_(dy.float().sum(0))


def gelu_backward_(dy: torch.Tensor, pre: torch.Tensor, db: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dpre = dy * gelu'(pre) (erf GELU) in pre's dtype; with ``db`` (fp32 [N])
    also db += dpre.sum(0) -- one pass on the GPU."""
    if _colsum_ok(dy) and _colsum_ok(pre) and dy.shape == pre.shape and dy.dtype == pre.dtype and \
            (db is None or (db.dtype == torch.float32 and db.is_contiguous())):
        require_native(dy)
        dpre = torch.empty_like(pre)
        _g().gelu_bwd_colsum(dy, pre, dpre, db)
        return dpre
    dpre = torch.ops.aten.gelu_backward(dy.float(), pre.float()).to(pre.dtype)
    if db is not None:
        db.add_(dpre.float().sum(0))
    return dpre


def _hip_gemm_ok(K: int, N: int) -> bool:
    return K % 64 == 0 and N % 64 == 0


# Dimensions that are not multiples of 64 (the LSTM's 1500 hidden units and
# 10,000-word softmax, BERT's 30,522-word vocabulary) can still run the HIP
# kernels on zero-padded copies of the operands: K and N are padded to the
# next multiple of 64 (zero columns add nothing to the products), the output
# is the [:, :N] view of the padded result.  The padded candidates are timed
# WITH their copies against hipBLASLt, so the tuner keeps whichever is faster
# per shape; GKSGD_LINEAR_PAD=0 restores hipBLASLt-only for these shapes.
_PAD = os.environ.get("GKSGD_LINEAR_PAD", "1") != "0"


def _p64(n: int) -> int:
    return (n + 63) // 64 * 64


_PAD_SHARE = os.environ.get("GKSGD_LINEAR_PAD_SHARE", "1") == "1"


def _pad2(t: torch.Tensor, rows: int, cols: int, cache: Optional[dict] = None) -> torch.Tensor:
    """Zero-padded contiguous copy of a 2-D tensor to [rows, cols] (one kernel).
    ``cache``: a dict scoped to one backward call (the tensor is not modified
    inside it), so the grad-input and grad-weight GEMMs share one padded copy
    of the output gradient."""
    r, c = t.shape
    if r == rows and c == cols and t.is_contiguous():
        return t
    if cache is not None:
        key = (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype, rows, cols)
        got = cache.get(key)
        if got is None:
            got = cache[key] = F.pad(t, (0, cols - c, 0, rows - r))
        return got
    return F.pad(t, (0, cols - c, 0, rows - r))


def _pad_ok(t: torch.Tensor) -> bool:
    return _PAD and t.is_cuda


def _fwd(x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor],
         b16: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x2 . w^T (+ bias) in x2's dtype (bf16, or fp32: the fp32 MFMA
    kernels).  ``b16``: the bias already in bf16 (the shadow arena's view) --
    hipBLASLt then needs no per-call cast."""
    M, K = x2.shape
    N = w.shape[0]
    dt = x2.dtype
    if b16 is None and bias is not None:
        b16 = bias.to(dt)

    def blas():
        return torch.addmm(b16, x2, w.t()) if b16 is not None else torch.mm(x2, w.t())
    if not _hip_gemm_ok(K, N):
        if not _pad_ok(x2):
            return blas()
        return _fwd_padded(x2, w, bias, blas)
    g = _g()
    y = torch.empty(M, N, dtype=dt, device=x2.device)
    cands = [(("hip", c, mb), (lambda c=c, mb=mb: g.gemm_nt(x2, w, y, c, mb, None, bias)))
             for c in _cv._nt_cfgs(dt) for mb in _cv._NT_GRIDS]
    cands.append((("blas", 0, 0), blas))
    ch = _cv._pick(("lin_fwd", M, K, N, bias is not None) + _cv._dkey(dt), cands)
    if ch[0] == "blas":
        return blas()
    g.gemm_nt(x2, w, y, ch[1], ch[2], None, bias)
    return y


def _fwd_padded(x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], blas) -> torch.Tensor:
    """y = x2 . w^T (+ bias) with K / N not multiples of 64: the HIP kernels on
    zero-padded operands (the copies timed with them) vs hipBLASLt."""
    M, K = x2.shape
    N = w.shape[0]
    Kp, Np = _p64(K), _p64(N)
    dt = x2.dtype
    g = _g()

    def padded(c, mb):
        xp = _pad2(x2, M, Kp)
        wp = _pad2(w, Np, Kp)
        bp = F.pad(bias, (0, Np - N)) if bias is not None else None
        yp = torch.empty(M, Np, dtype=dt, device=x2.device)
        g.gemm_nt(xp, wp, yp, c, mb, None, bp)
        return yp[:, :N]
    key = ("lin_fwd", M, K, N, bias is not None) + _cv._dkey(dt) + ("pad",)
    got = _cv._choices.get(key)
    if got is not None and got[0] == "blas":
        return blas()
    cands = [(("hip", c, mb), (lambda c=c, mb=mb: padded(c, mb))) for c in _cv._nt_cfgs(dt) for mb in _cv._NT_GRIDS]
    cands.append((("blas", 0, 0), blas))
    ch = _cv._pick(key, cands)
    if ch[0] == "blas":
        return blas()
    return padded(ch[1], ch[2])


def _dgrad_padded(dy2: torch.Tensor, w: torch.Tensor, pads: Optional[dict] = None) -> torch.Tensor:
    """dx = dy2 . w with K / N not multiples of 64 (see _fwd_padded)."""
    M, N = dy2.shape
    K = w.shape[1]
    Kp, Np = _p64(K), _p64(N)
    dt = dy2.dtype
    g = _g()
    key = ("lin_dgrad", M, K, N) + _cv._dkey(dt) + ("pad",)
    got = _cv._choices.get(key)
    if got is not None and got[0] == "blas":
        return torch.mm(dy2, w)

    def padded(c, mb, cache=None):
        dyp = _pad2(dy2, M, Np, cache)
        wtp = _pad2(w.t(), Kp, Np)
        dxp = torch.empty(M, Kp, dtype=dt, device=dy2.device)
        g.gemm_nt(dyp, wtp, dxp, c, mb)
        return dxp[:, :K]
    cands = [(("hip", c, mb), (lambda c=c, mb=mb: padded(c, mb))) for c in _cv._nt_cfgs(dt) for mb in _cv._NT_GRIDS]
    cands.append((("blas", 0, 0), lambda: torch.mm(dy2, w)))
    ch = _cv._pick(key, cands)
    if ch[0] == "blas":
        return torch.mm(dy2, w)
    return padded(ch[1], ch[2], pads)


def _dgrad(dy2: torch.Tensor, w: torch.Tensor, pads: Optional[dict] = None) -> torch.Tensor:
    """dx = dy2 . w in dy2's dtype.  ``pads``: see _pad2."""
    M, N = dy2.shape
    K = w.shape[1]
    dt = dy2.dtype
    key = ("lin_dgrad", M, K, N) + _cv._dkey(dt)
    got = _cv._choices.get(key)
    if not _hip_gemm_ok(K, N) and _pad_ok(dy2):
        return _dgrad_padded(dy2, w, pads)
    if not _hip_gemm_ok(K, N) or (got is not None and got[0] == "blas"):
        return torch.mm(dy2, w)
    g = _g()
    dx = torch.empty(M, K, dtype=dt, device=dy2.device)
    wt = w.t().contiguous()
    cands = [(("hip", c, mb), (lambda c=c, mb=mb: g.gemm_nt(dy2, wt, dx, c, mb)))
             for c in _cv._nt_cfgs(dt) for mb in _cv._NT_GRIDS]
    cands.append((("blas", 0, 0), lambda: torch.mm(dy2, w)))
    ch = _cv._pick(key, cands)
    if ch[0] == "blas":
        return torch.mm(dy2, w)
    g.gemm_nt(dy2, wt, dx, ch[1], ch[2])
    return dx


def _wgrad_into(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor, pads: Optional[dict] = None) -> None:
    """out (fp32 [N, K]) += dy2^T . x2.  ``pads``: see _pad2."""
    M, N = dy2.shape
    K = x2.shape[1]

    def blas(o):
        accum_grad_(o, torch.mm(dy2.t(), x2))

    f32 = dy2.dtype == torch.float32

    def blas32(o):   # hipBLASLt -> fp32 with beta = 1, straight into the arena view
        if f32:
            torch.addmm(o, dy2.t(), x2, out=o)
        else:
            torch.addmm(o, dy2.t(), x2, out_dtype=torch.float32, out=o)
    if not dy2.is_cuda:
        blas(out)
        return
    g = _g()
    key = ("lin_wgrad", M, K, N) + _cv._dkey(dy2.dtype)
    scratch = torch.zeros_like(out) if key not in _cv._choices else None
    cands = []
    padded = None
    if _hip_gemm_ok(K, N):
        cands = [(("hip", c, sp), (lambda c=c, sp=sp: g.gemm_tn_acc(dy2, x2, scratch, c, sp)))
                 for c, sp in _cv._tn_cfgs(torch.float32 if f32 else torch.bfloat16)]
    elif _pad_ok(dy2):
        # zero-padded operands into a padded fp32 scratch, then one add of its
        # [:N, :K] block into the target (see _fwd_padded)
        key = key + ("pad",)
        Kp, Np = _p64(K), _p64(N)

        def padded(o, c, sp, cache=None):
            dyp = _pad2(dy2, M, Np, cache)
            xp = _pad2(x2, M, Kp)
            op = torch.zeros(Np, Kp, dtype=torch.float32, device=dy2.device)
            g.gemm_tn_acc(dyp, xp, op, c, sp)
            o.add_(op[:N, :K])
        scratch = torch.zeros_like(out) if key not in _cv._choices else None
        cands = [(("hip", c, sp), (lambda c=c, sp=sp: padded(scratch, c, sp)))
                 for c, sp in _cv._tn_cfgs(torch.float32 if f32 else torch.bfloat16)]
    cands.append((("blas32", 0, 0), lambda: blas32(scratch)))
    cands.append((("blas", 0, 0), lambda: blas(scratch)))
    ch = _cv._pick(key, cands)
    if ch[0] == "blas":
        blas(out)
    elif ch[0] == "blas32":
        blas32(out)
    elif padded is not None:
        padded(out, ch[1], ch[2], pads)
    else:
        g.gemm_tn_acc(dy2, x2, out, ch[1], ch[2])


def _wgrad_forkable(dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    """Is this grad-weight's tuned choice a HIP kernel (direct or padded), so it
    may run on the side stream (ops/streams.py)?  hipBLASLt choices stay on the
    stream their handle / workspace belong to, untuned keys are timed inline."""
    M, N = dy2.shape
    K = x2.shape[1]
    if not streams.worth(dy2.device, 2.0 * M * N * K):
        return False
    key = ("lin_wgrad", M, K, N) + _cv._dkey(dy2.dtype)
    if not _hip_gemm_ok(K, N):
        key = key + ("pad",)
    ch = _cv._choices.get(key)
    return ch is not None and ch[0] == "hip"


def _target(sink) -> Optional[torch.Tensor]:
    """The fp32 arena gradient view a shadow sink accumulates into (None: no direct path)."""
    if sink is None:
        return None
    gv = getattr(sink, "grad_view", None)
    if gv is None or not gv.is_contiguous():
        return None
    sink.check()
    return gv


class _LinearFn(torch.autograd.Function):
    """y = act(x . W^T + b) with bf16 operands (``dt`` bf16) or fp32 operands
    (``dt`` fp32: the reference's precision, fp32 MFMA kernels).  ``weight`` /
    ``bias`` are the fp32 master parameters; with sinks (bf16-shadow path or
    fp32 direct-gradient path, parallel/shadow.py) their gradients are added
    into the optimizer's fp32 arena in the backward and None is returned for
    them, so AccumulateGrad launches nothing (its post-accumulate hook still
    reports the parameter ready)."""

    @staticmethod
    def forward(ctx, x, weight, w_bf16, wsink, bias, bsink, gelu, b_bf16=None, dt=torch.bfloat16):
        shape = x.shape
        K = shape[-1]
        x2 = x.reshape(-1, K)
        if x2.dtype != dt:
            x2 = x2.to(dt)
        x2 = x2.contiguous()
        w = w_bf16 if w_bf16 is not None else weight.detach().to(dt)
        w = w.contiguous()
        b = bias.detach().float().contiguous() if bias is not None else None
        y = _fwd(x2, w, b, b_bf16)
        pre = None
        if gelu:
            pre, y = y, F.gelu(y)
        ctx.save_for_backward(x2, w, pre)
        ctx.wsink, ctx.bsink, ctx.gelu = wsink, bsink, gelu
        ctx.has_bias = bias is not None
        ctx.in_shape = shape
        ctx.wdtype = weight.dtype
        ctx.bdtype = bias.dtype if bias is not None else None
        return y.view(*shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, w, pre = ctx.saved_tensors
        N, K = w.shape
        dy2 = dy.reshape(-1, N)
        if dy2.dtype != x2.dtype:
            dy2 = dy2.to(x2.dtype)
        dy2 = dy2.contiguous()
        db = gbias = None
        if ctx.has_bias and ctx.needs_input_grad[4]:
            db = _target(ctx.bsink)
            if db is None:
                db = gbias = torch.zeros(N, dtype=torch.float32, device=dy2.device)
        if ctx.gelu:
            dpre = gelu_backward_(dy2, pre, db)
        else:
            dpre = dy2
            if db is not None:
                bias_grad_acc_(db, dpre)
        # one zero-padded copy of dpre for both GEMMs (K / N not multiples of 64)
        pads = {} if _PAD_SHARE else None
        dx = _dgrad(dpre, w, pads).view(ctx.in_shape) if ctx.needs_input_grad[0] else None
        gweight = None
        if ctx.needs_input_grad[1]:
            gw = _target(ctx.wsink)
            if gw is not None and not getattr(ctx.wsink, "shared", False) and _wgrad_forkable(dpre, x2):
                # off the critical path: the grad-weight only feeds the optimizer
                side = streams.fork(dpre.device)
                with torch.cuda.stream(side):
                    _wgrad_into(dpre, x2, gw, pads)
                streams.hold(dpre.device, dpre, x2, *(pads.values() if pads else ()))
            elif gw is not None:
                _wgrad_into(dpre, x2, gw, pads)
            else:
                gw = torch.zeros(N, K, dtype=torch.float32, device=dy2.device)
                _wgrad_into(dpre, x2, gw, pads)
                if ctx.wsink is not None:
                    ctx.wsink(gw)
                else:
                    gweight = gw.to(ctx.wdtype)
        if gbias is not None:
            if ctx.bsink is not None:
                ctx.bsink(gbias)
                gbias = None
            else:
                gbias = gbias.to(ctx.bdtype)
        return dx, gweight, None, None, gbias, None, None, None, None


def _supported(x: torch.Tensor, mod: nn.Linear) -> bool:
    return (_ENABLED and x.is_cuda and x.dim() >= 1 and x.shape[-1] == mod.in_features and x.numel() > 0 and
            mod.weight.dtype == torch.float32 and mod.out_features % 8 == 0)


class FastLinear(nn.Linear):
    """``nn.Linear`` whose bf16 training path on a GPU runs the autotuned MFMA
    kernels and the fused bias-gradient pass; ``forward(x, act="gelu")``
    applies GELU with its backward fused into that pass.  Everywhere else it
    is the stock layer (+ ``F.gelu``)."""

    def forward(self, x: torch.Tensor, act: Optional[str] = None) -> torch.Tensor:
        if act not in (None, "gelu"):
            raise ValueError("FastLinear act must be None or 'gelu', got %r" % (act,))
        dev = x.device.type
        autocast = torch.is_autocast_enabled(dev)
        bf16 = x.dtype == torch.bfloat16 or (autocast and torch.get_autocast_dtype(dev) == torch.bfloat16)
        f32 = not autocast and x.dtype == torch.float32 and os.environ.get("GKSGD_FASTLINEAR_F32", "1") != "0"
        if f32 and _supported(x, self) and load():
            # fp32 (the reference's precision): fp32 MFMA GEMMs, weight / bias
            # gradients straight into the fp32 arena (install_direct_grads)
            table = getattr(self, "_gk_direct_grads", None) or {}
            wsink, bsink = table.get("weight"), table.get("bias")
            if not torch.is_grad_enabled() or not self.weight.requires_grad:
                wsink = None
            if not torch.is_grad_enabled() or self.bias is None or not self.bias.requires_grad:
                bsink = None
            return _LinearFn.apply(x, self.weight, None, wsink, self.bias, bsink, act == "gelu", None,
                                   torch.float32)
        if bf16 and _supported(x, self) and load():
            table = getattr(self, "_gk_shadow", None)
            winfo = table.get("weight") if table else None
            binfo = table.get("bias") if table else None
            use_shadow = winfo is not None and torch.is_autocast_enabled(dev)
            w_bf16, wsink = (winfo[0], winfo[1]) if use_shadow else (None, None)
            bsink = binfo[1] if (use_shadow and binfo is not None) else None
            b_bf16 = binfo[0] if (use_shadow and binfo is not None) else None
            if not torch.is_grad_enabled() or not self.weight.requires_grad:
                wsink = None
            if not torch.is_grad_enabled() or self.bias is None or not self.bias.requires_grad:
                bsink = None
            return _LinearFn.apply(x, self.weight, w_bf16, wsink, self.bias, bsink, act == "gelu", b_bf16)
        slow = getattr(self, "_gk_slow", None)
        y = slow(x) if slow is not None else super().forward(x)
        return F.gelu(y) if act == "gelu" else y
