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

import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import load, require_native

_CL = torch.channels_last
# In-launch finalize (bn_act.hip FinSync) is opt-in: measured on ResNet-50 bs32
# fp32 (r5c2) the fused apply passes ran 35 us per call against 17 + 5 for
# finalize + apply as two launches -- ~1000 workgroups polling the leaders'
# flags slow the leaders' partial reductions -- 14.38 vs 12.99 ms per step.
_FIN_FUSE = os.environ.get("GKSGD_BN_FIN_FUSE", "0") == "1"


def _ops():
    return torch.ops.gksgd


def _grad_pair(grads, like):
    """(dy, dy2) from the output gradients of a (possibly twin-output) Function."""
    gs = [g for g in grads if g is not None]
    out = []
    for g in gs:
        g = g.contiguous(memory_format=_CL)
        if g.dtype != like.dtype:
            g = g.to(like.dtype)
        out.append(g)
    return (out + [None, None])[:2]


class BnLink:
    """Hand-off between a fused BN and the convolution that consumes its output
    (its only consumer, guaranteed by the model wiring, ``BNAct.bwd_link``).

    The consumer's grad-input GEMM runs the BN-backward epilogue
    (csrc/kernels/gemm.hip ``BnBwd``): it writes ``dz`` = ReLU-masked
    (dy + dy2) instead of dy and the per-channel partials of sum(dz) and
    sum(dz * h), so the BN backward skips its reduction pass and only
    finalizes + applies (``bn_act_backward_pre``).  For a twin output (ResNet
    block output: next conv1 + shortcut) the shortcut's gradient dy2 must be
    known when the conv1 grad-input runs: the residual consumer (the next
    block's last BN, which runs its backward first) stores it here.
    """

    __slots__ = ("h", "mask", "twin", "dy2", "dz", "part")

    def __init__(self):
        self.h = self.mask = self.dy2 = self.dz = self.part = None
        self.twin = False

    def ready(self) -> bool:
        """Can the consumer's grad-input fuse the BN-backward reduction now?"""
        return self.h is not None and (not self.twin or self.dy2 is not None)

    def clear(self) -> None:
        self.h = self.mask = self.dy2 = self.dz = self.part = None


class ProducerLink:
    """Hand-off between a fused BN and the convolution that PRODUCED its input
    (fp32 path; ops/conv1x1.py attaches one to its output).

    Lazy BN backward: instead of materialising dx = dL/d(conv output) with an
    apply pass, the BN backward stores dz (ReLU-masked, twin-summed gradient),
    its input x and the per-channel coefficients here, and returns dz itself
    to autograd; the producer's grad-input and grad-weight GEMMs recognise it
    (same storage) and compute dx = k1 ((dz - k2) - (x - mu) k4) on the fly
    (gemm.hip LazyA).  ``materialize()`` runs the apply kernel for a consumer
    without the lazy path (MIOpen choice, bf16).

    Opt-in (``GKSGD_BN_LAZY=1``).  Measured on MI355X at ResNet-50 bs512 fp32
    (gpurun_out tune dump summarised in profiles/r03_bn_lazy_tuning.txt): the
    lazy NT / TN GEMMs run 1.3-2.4x the time of the plain GEMM on every shape
    -- the dz and x tiles double the A-side LDS-DMA stages and the coefficient
    reads double the fragment reads, which costs the deep stage pipeline the
    fp32 kernels rely on at one wave per SIMD -- so the autotuner picks
    "materialise + plain GEMM" everywhere and the step is 1 ms slower (148.4
    vs 147.4 ms).  The kernels stay tested (tests/test_bn_lazy_gpu.py) for
    the cases where the GEMM is not the bound.
    """

    __slots__ = ("lazy", "dx")

    def __init__(self):
        self.lazy = None    # (dz, x, coef, padz, padx)
        self.dx = None      # materialised dx (cached: grad-input and grad-weight may both ask)

    def matches(self, dy: torch.Tensor) -> bool:
        return self.lazy is not None and dy.data_ptr() == self.lazy[0].data_ptr() and dy.shape == self.lazy[0].shape

    def materialize(self) -> torch.Tensor:
        if self.dx is None:
            dz, x, coef, _, _ = self.lazy
            self.dx = torch.empty_like(x, memory_format=_CL)
            _ops().bn_lazy_apply(dz, x, self.dx, coef)
        return self.dx

    def clear(self) -> None:
        self.lazy = self.dx = None


def _lazy_buffers(x: torch.Tensor):
    C = x.shape[1]
    coef = torch.empty(C, 4, dtype=torch.float32, device=x.device)
    padz = torch.empty(C, dtype=x.dtype, device=x.device)
    padx = torch.empty(C, dtype=x.dtype, device=x.device)
    return coef, padz, padx


def _lazy_ok(x: torch.Tensor, plink) -> bool:
    import os
    return (plink is not None and x.dtype == torch.float32 and x.shape[1] % 64 == 0 and
            os.environ.get("GKSGD_BN_LAZY", "0") != "0")


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, momentum, eps, relu, direct=None,
                nbt=None, twin=False, pre=None, link=None, res_link=None, plink=None, fin=None, rbn=None):
        # direct = (gw_view, gb_view): weight/bias gradients are accumulated
        # straight into the optimizer's fp32 arena by the backward kernel and
        # None is returned for them, so AccumulateGrad launches nothing (its
        # post-accumulate hook still fires and reports readiness).
        # twin: return the output twice (ResNet: next block's conv1 input and
        # its shortcut); the backward sums both gradients inside the BN passes.
        ctx.direct = direct
        ctx.set_materialize_grads(False)
        C = x.shape[1]
        M = x.numel() // C
        eb = x.element_size()
        y = torch.empty_like(x, memory_format=_CL)
        stats = torch.empty(4, C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, eb)), dtype=torch.float32, device=x.device)
        # a deferred residual BN (_BNDeferFn): residual = r * rscale + rshift formed on load
        rscale, rshift, dlink = rbn if rbn is not None else (None, None, None)
        ctx.dlink = dlink
        if rbn is not None and (residual.dtype != x.dtype or not residual.is_contiguous(memory_format=_CL)):
            raise RuntimeError("deferred residual BN: the pending tensor must match x (dtype, channels-last)")
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        if residual is not None and not residual.is_contiguous(memory_format=_CL):
            residual = residual.contiguous(memory_format=_CL)
        mask = None
        if relu:
            mask = torch.empty(int(_ops().bn_mask_bytes(M, C, eb)), dtype=torch.uint8, device=x.device)
        # pre = (partials [2, rows, C], rows): batch statistics already reduced by
        # the producing convolution's epilogue (ops/conv1x1.py) -- no stats pass
        pre_t, pre_rows = pre if pre is not None else (None, 0)
        _ops().bn_act_forward(x, residual, y, mask, weight, bias, running_mean, running_var, stats[0], stats[1],
                              stats[2], stats[3], ws, float(eps), float(momentum), bool(relu), nbt, pre_t, pre_rows,
                              fin, rscale, rshift)
        ctx.fin = fin
        ctx.relu = bool(relu)
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, mask, weight, stats[0], stats[1])
        # link: this BN's output feeds one conv that may fuse our backward
        # reduction; res_link: our residual came from a linked twin BN, which
        # needs our residual gradient before its consumer's grad-input runs
        ctx.link = link
        ctx.res_link = res_link
        ctx.plink = plink
        if link is not None:
            link.h, link.mask, link.twin = x, mask, bool(twin)
        return (y, y.view_as(y)) if twin else y

    @staticmethod
    def backward(ctx, *grads):
        x, mask, weight, mean, invstd = ctx.saved_tensors
        link, res_link, plink, dlink = ctx.link, ctx.res_link, ctx.plink, ctx.dlink
        ctx.link = ctx.res_link = ctx.plink = ctx.dlink = None
        gw, gb = ctx.direct if ctx.direct is not None else (None, None)
        lazy = _lazy_ok(x, plink) and ctx.needs_input_grad[0]
        if link is not None and link.part is not None:
            # the consumer conv's grad-input epilogue produced dz (masked, twin-summed)
            # and its reduction partials: finalize + apply only
            dz = grads[0]
            if dz is None or dz.data_ptr() != link.dz.data_ptr():
                raise RuntimeError("BNAct bwd_link: the linked output had another consumer")
            part, rows = link.part
            link.clear()
            g = torch.empty(2, x.shape[1], dtype=torch.float32, device=x.device)
            if lazy:
                # finalize only; the producing conv's GEMMs apply the BN backward themselves
                coef, padz, padx = _lazy_buffers(x)
                _ops().bn_bwd_lazy_pre(x, part, rows, weight, mean, invstd, g[0], g[1], coef, padz, padx, gw, gb)
                plink.lazy = (dz, x, coef, padz, padx)
                dx = dz
            elif dlink is not None and ctx.needs_input_grad[1]:
                # residual = a deferred BN: its backward in this apply pass too
                dx = torch.empty_like(x, memory_format=_CL)
                x2 = dlink.x
                dx2 = torch.empty_like(x2, memory_format=_CL)
                g2 = torch.empty(2, x2.shape[1], dtype=torch.float32, device=x.device)
                ws2 = torch.empty(int(_ops().bn_workspace_floats(x2.numel() // x2.shape[1], x2.shape[1],
                                                                 x2.element_size())),
                                  dtype=torch.float32, device=x.device)
                gw2, gb2 = dlink.direct if dlink.direct is not None else (None, None)
                _ops().bn_act_backward_pre_dual(dz, x, dx, weight, mean, invstd, g[0], g[1], part, rows, gw, gb, x2,
                                                dx2, dlink.weight, dlink.mean, dlink.invstd, g2[0], g2[1], ws2, gw2,
                                                gb2)
                dlink.dz, dlink.dx, dlink.g = dz, dx2, g2
            else:
                dx = torch.empty_like(x, memory_format=_CL)
                _ops().bn_act_backward_pre(dz, x, dx, weight, mean, invstd, g[0], g[1], part, rows, gw, gb, ctx.fin)
            dres = dz if ctx.has_res and ctx.needs_input_grad[1] else None
            if res_link is not None and dres is not None:
                res_link.dy2 = dres
            if ctx.direct is not None:
                return (dx, dres) + (None,) * 16
            dgamma = g[0] if weight is not None and ctx.needs_input_grad[2] else None
            dbeta = g[1] if ctx.needs_input_grad[3] else None
            return (dx, dres, dgamma, dbeta) + (None,) * 14
        if link is not None:
            link.clear()
        dy, dy2 = _grad_pair(grads, x)
        if dy is None:
            return (None,) * 18
        C = x.shape[1]
        M = x.numel() // C
        g = torch.empty(2, C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, x.element_size())), dtype=torch.float32,
                         device=x.device)
        if lazy:
            # the reduce pass writes dz (= the residual gradient); no apply pass
            dz = torch.empty_like(x, memory_format=_CL)
            coef, padz, padx = _lazy_buffers(x)
            _ops().bn_act_backward_lazy(dy, dy2, mask, x, dz, weight, mean, invstd, g[0], g[1], ws, ctx.relu, coef,
                                        padz, padx, gw, gb)
            plink.lazy = (dz, x, coef, padz, padx)
            dx = dz
            dres = dz if ctx.has_res and ctx.needs_input_grad[1] else None
        else:
            dx = torch.empty_like(x, memory_format=_CL)
            dres = torch.empty_like(x, memory_format=_CL) if ctx.has_res and ctx.needs_input_grad[1] else None
            _ops().bn_act_backward(dy, mask, x, dx, dres, weight, mean, invstd, g[0], g[1], ws, ctx.relu, gw, gb,
                                   dy2, ctx.fin)
        if res_link is not None and dres is not None:
            res_link.dy2 = dres
        if ctx.direct is not None:
            return (dx, dres) + (None,) * 16
        dgamma = g[0] if weight is not None and ctx.needs_input_grad[2] else None
        dbeta = g[1] if ctx.needs_input_grad[3] else None
        return (dx, dres, dgamma, dbeta) + (None,) * 14


class DeferLink:
    """Backward hand-off between a deferred BN (``_BNDeferFn``) and the fused BN
    that applied it as its residual: when that BN's backward is linked (dz and
    its partials from the consumer conv's GEMM epilogue) it also runs the
    deferred BN's reduce + finalize and writes its dx in the SAME apply pass
    (``bn_act_backward_pre_dual``: dz read once), leaving dx and the parameter
    gradients here; the deferred BN's backward then returns them when its
    incoming gradient is that dz."""

    __slots__ = ("x", "weight", "mean", "invstd", "direct", "dz", "dx", "g")

    def __init__(self, x, weight, mean, invstd, direct):
        self.x, self.weight, self.mean, self.invstd, self.direct = x, weight, mean, invstd, direct
        self.dz = self.dx = self.g = None


class _BNDeferFn(torch.autograd.Function):
    """A plain BN (no ReLU, no residual) whose apply pass is deferred into its
    only consumer: the forward runs the statistics + finalize (running stats,
    saved mean / invstd, per-channel scale / shift) and returns a view of the
    UN-normalised input tagged ``_gk_pending_bn = (scale, shift, DeferLink)``; the
    consumer -- the block's last fused BN, which takes it as its residual --
    adds ``x * scale + shift`` on load (bn_act.hip ``bn_apply_kernel`` RBN).
    The BN output is never written: one streaming pass (read x, write y) less
    per ResNet downsample shortcut.  The backward is the plain BN backward of
    the gradient the consumer hands back for its residual (d out / d residual
    = the consumer's dz), so it is unchanged.

    The handle is only valid as the residual of a fused BNAct; model code that
    wires it (models/resnet_imagenet.py Bottleneck) guarantees that."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, stats, direct=None, nbt=None,
                pre=None, dlink=None):
        # stats: fp32 [4, C] (mean, invstd, scale, shift), allocated by the caller, which
        # tags the returned handle with its scale / shift rows
        ctx.direct = direct
        ctx.set_materialize_grads(False)
        C = x.shape[1]
        M = x.numel() // C
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, x.element_size())), dtype=torch.float32,
                         device=x.device)
        pre_t, pre_rows = pre if pre is not None else (None, 0)
        _ops().bn_act_finalize(x, weight, bias, running_mean, running_var, stats[0], stats[1], stats[2], stats[3], ws,
                               float(eps), float(momentum), nbt, pre_t, pre_rows)
        ctx.save_for_backward(x, weight, stats[0], stats[1])
        ctx.dlink = dlink
        return x.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, invstd = ctx.saved_tensors
        dl, ctx.dlink = ctx.dlink, None
        if dy is None:
            return (None,) * 12
        if dl is not None and dl.dx is not None and dl.dz is not None and dy.data_ptr() == dl.dz.data_ptr():
            # computed by the consumer BN's dual apply pass
            dx, g = dl.dx, dl.g
            dl.dz = dl.dx = dl.g = None
            if ctx.direct is not None:
                return (dx,) + (None,) * 11
            dgamma = g[0] if weight is not None and ctx.needs_input_grad[1] else None
            dbeta = g[1] if ctx.needs_input_grad[2] else None
            return (dx, dgamma, dbeta) + (None,) * 9
        if dl is not None and dl.dx is not None:
            # the dual pass already ran (and may have accumulated into the arena)
            raise RuntimeError("deferred BN: the consumer's gradient reached the shortcut BN as another tensor")
        dy = dy.contiguous(memory_format=_CL)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        C = x.shape[1]
        M = x.numel() // C
        g = torch.empty(2, C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, x.element_size())), dtype=torch.float32,
                         device=x.device)
        gw, gb = ctx.direct if ctx.direct is not None else (None, None)
        dx = torch.empty_like(x, memory_format=_CL)
        _ops().bn_act_backward(dy, None, x, dx, None, weight, mean, invstd, g[0], g[1], ws, False, gw, gb, None, None)
        if ctx.direct is not None:
            return (dx,) + (None,) * 11
        dgamma = g[0] if weight is not None and ctx.needs_input_grad[1] else None
        dbeta = g[1] if ctx.needs_input_grad[2] else None
        return (dx, dgamma, dbeta) + (None,) * 9


_DEFER = os.environ.get("GKSGD_BN_DEFER", "1") != "0"
# the deferred BN's backward in the consumer's linked apply pass (bn_act_backward_pre_dual)
_DEFER_BWD = os.environ.get("GKSGD_BN_DEFER_BWD", "1") != "0"


class _BNReLUPoolFn(torch.autograd.Function):
    """maxpool(relu(bn(x))) with the pool folded into the BN passes (bn_act.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, pool, direct=None, nbt=None,
                twin=False, pre=None):
        ctx.set_materialize_grads(False)
        k, st, pad = pool
        N, C, H, W = x.shape
        OH = (H + 2 * pad - k) // st + 1
        OW = (W + 2 * pad - k) // st + 1
        y = torch.empty((N, C, OH, OW), dtype=x.dtype, device=x.device, memory_format=_CL)
        amax = torch.empty(N * C * OH * OW, dtype=torch.uint8, device=x.device)
        stats = torch.empty(4, C, dtype=torch.float32, device=x.device)
        M = N * H * W
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, x.element_size())), dtype=torch.float32,
                         device=x.device)
        # pre = (partials [2, rows, C], rows): statistics from the stem conv's epilogue
        pre_t, pre_rows = pre if pre is not None else (None, 0)
        _ops().bn_relu_pool_forward(x, y, amax, weight, bias, running_mean, running_var, stats[0], stats[1],
                                    stats[2], stats[3], ws, float(eps), float(momentum), k, st, pad, nbt, pre_t,
                                    pre_rows)
        ctx.pool = (k, st, pad)
        ctx.direct = direct
        ctx.save_for_backward(x, amax, weight, stats[0], stats[1])
        return (y, y.view_as(y)) if twin else y

    @staticmethod
    def backward(ctx, *grads):
        x, amax, weight, mean, invstd = ctx.saved_tensors
        dy, dy2 = _grad_pair(grads, x)
        if dy is None:
            return (None,) * 12
        k, st, pad = ctx.pool
        C = x.shape[1]
        M = x.numel() // C
        dx = torch.empty_like(x, memory_format=_CL)
        g = torch.empty(2, C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(_ops().bn_workspace_floats(M, C, x.element_size())), dtype=torch.float32,
                         device=x.device)
        gw, gb = ctx.direct if ctx.direct is not None else (None, None)
        _ops().bn_relu_pool_backward(dy, amax, x, dx, weight, mean, invstd, g[0], g[1], ws, k, st, pad, gw, gb, dy2)
        if ctx.direct is not None:
            return (dx,) + (None,) * 11
        dgamma = g[0] if weight is not None and ctx.needs_input_grad[1] else None
        dbeta = g[1] if ctx.needs_input_grad[2] else None
        return (dx, dgamma, dbeta) + (None,) * 9


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
    """BatchNorm2d with optional fused residual add, ReLU and trailing max-pool.

    ``pool=(k, s, p)`` (requires ``act="relu"``) appends ``max_pool2d(k, s, p)``:
    the fused path never writes the full-resolution activation and gathers the
    pool gradient inside the BN backward (the ResNet stem).
    """

    def __init__(self, num_features: int, act: Optional[str] = None, eps: float = 1e-5, momentum: float = 0.1,
                 affine: bool = True, track_running_stats: bool = True, fused: bool = True,
                 pool: Optional[tuple] = None, twin: bool = False, bwd_link: bool = False):
        super().__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                         track_running_stats=track_running_stats)
        assert act in (None, "relu")
        assert pool is None or (act == "relu" and len(pool) == 3)
        self.act = act
        self.fused = fused
        self.pool = tuple(pool) if pool is not None else None
        # twin: forward returns (out, out) -- two handles on one output whose
        # gradients the fused backward sums on load (ResNet block outputs feed
        # both the next conv1 and the next shortcut).
        self.twin = twin
        # bwd_link: the (main) output is consumed by exactly one FastConv2d, which
        # may fuse this BN's backward reduction into its grad-input GEMM (BnLink);
        # set by model code that guarantees the single consumer.
        self.bwd_link = bwd_link

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, stats=None) -> torch.Tensor:
        """``stats``: optional (partials, rows) of x's batch statistics reduced
        by the producing convolution (ops/conv1x1.py conv_stats); used only on
        the fused training path."""
        relu = self.act == "relu"
        pool = self.pool
        if self.training and self.fused and self.track_running_stats and fused_bn_available(x) and \
                (pool is None or (residual is None and x.numel() // x.shape[1] < 2 ** 32)):
            nbt = self.num_batches_tracked
            if self.momentum is None:
                nbt.add_(1)
                mom = 1.0 / float(nbt)  # host sync, as in nn.BatchNorm2d's cumulative mode
                nbt = None
            else:
                mom = self.momentum     # the finalize kernel increments num_batches_tracked
            direct = getattr(self, "_gk_direct", None)
            if pool is not None:
                pre = stats if (stats is not None and stats[0].shape[2] == x.shape[1]) else None
                return _BNReLUPoolFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var, mom,
                                           self.eps, pool, direct, nbt, self.twin, pre)
            if stats is not None and stats[0].shape[2] != x.shape[1]:
                stats = None
            link = BnLink() if self.bwd_link and torch.is_grad_enabled() else None
            res_link = getattr(residual, "_gk_res_link", None) if residual is not None else None
            plink = getattr(x, "_gk_plink", None) if torch.is_grad_enabled() else None
            rbn = getattr(residual, "_gk_pending_bn", None) if residual is not None else None
            out = _BNActFn.apply(x, residual, self.weight, self.bias, self.running_mean, self.running_var, mom,
                                 self.eps, relu, direct, nbt, self.twin, stats, link, res_link, plink,
                                 self._fin_state(x), rbn)
            if link is not None:
                main = out[0] if self.twin else out
                main._gk_bn_link = link
                if self.twin:
                    out[1]._gk_res_link = link
            return out
        out = super().forward(x)
        if residual is not None:
            pend = getattr(residual, "_gk_pending_bn", None)
            if pend is not None:   # a deferred BN output (BNAct.deferred): apply it here
                C = residual.shape[1]
                residual = residual * pend[0].view(1, C, 1, 1).to(residual.dtype) + \
                    pend[1].view(1, C, 1, 1).to(residual.dtype)
            out = out + residual
        if relu:
            out = F.relu(out)
        if pool is not None:
            out = F.max_pool2d(out, pool[0], pool[1], pool[2])
        return (out, out) if self.twin else out

    def fused_ok(self, x: torch.Tensor) -> bool:
        """Will ``forward(x)`` take the fused training path?"""
        return bool(self.training and self.fused and self.track_running_stats and fused_bn_available(x))

    def deferred(self, x: torch.Tensor, stats=None) -> Optional[torch.Tensor]:
        """BN of ``x`` with the apply pass deferred into the consumer (see
        ``_BNDeferFn``): returns the pending handle, or None when this BN
        cannot defer (then call ``forward``).  Only for a plain BN (no act,
        pool or twin) whose output is the residual of a fused BNAct."""
        if not (_DEFER and self.act is None and self.pool is None and not self.twin and self.fused_ok(x)):
            return None
        nbt = self.num_batches_tracked
        if self.momentum is None:
            nbt.add_(1)
            mom = 1.0 / float(nbt)
            nbt = None
        else:
            mom = self.momentum
        if stats is not None and stats[0].shape[2] != x.shape[1]:
            stats = None
        st = torch.empty(4, x.shape[1], dtype=torch.float32, device=x.device)
        direct = getattr(self, "_gk_direct", None)
        dlink = DeferLink(x, self.weight, st[0], st[1], direct) if _DEFER_BWD and torch.is_grad_enabled() else None
        out = _BNDeferFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var, mom, self.eps, st,
                               direct, nbt, stats, dlink)
        out._gk_pending_bn = (st[2], st[3], dlink)
        return out

    def _fin_state(self, x: torch.Tensor) -> Optional[torch.Tensor]:
        """Per-layer state of the in-launch finalize (bn_act.hip FinSync: a
        ticket counter and one flag per 16-channel group, zeroed ONCE): the
        statistics finalize runs inside the apply pass instead of as its own
        launch (2 launches per BN and step fewer; opt-in: GKSGD_BN_FIN_FUSE=1)."""
        if not _FIN_FUSE:
            return None
        st = getattr(self, "_gk_fin", None)
        if st is None or st.device != x.device:
            n = int(_ops().bn_fin_state_bytes(self.num_features))
            st = torch.zeros((n + 15) // 16 * 16, dtype=torch.uint8, device=x.device)
            self._gk_fin = st
        return st

    def extra_repr(self) -> str:
        return super().extra_repr() + ", act=%s" % self.act + (", pool=%s" % (self.pool,) if self.pool else "")


class _GlobalAvgPoolCL(torch.autograd.Function):
    """mean over H, W whose backward writes a channels-last gradient directly
    (the generic adaptive_avg_pool2d backward yields NCHW, and the fused BN
    backward that consumes it would need a transposing copy)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x.mean(dim=(2, 3))

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        return (g / (H * W))[:, :, None, None].expand(N, C, H, W).contiguous(memory_format=_CL)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] -> [N, C]; channels-last aware backward."""
    if x.dim() == 4 and x.is_contiguous(memory_format=_CL) and x.requires_grad:
        return _GlobalAvgPoolCL.apply(x)
    return x.mean(dim=(2, 3))
