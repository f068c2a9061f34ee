"""ImageNet-ResNet stem convolution (7x7, stride 2, padding 3, 3 -> 64
channels) on the hand-written gfx950 kernels of ``csrc/kernels/stem.hip``.

``StemConv`` is a drop-in ``nn.Conv2d(3, 64, 7, 2, 3, bias=False)`` (same
parameter, same state_dict key).  In training on a GPU with a channels-last
fp32 / bf16 image batch and bf16 autocast it runs:

* forward: the MFMA kernel reads the fp32 batch directly (no cast pass),
  writes the bf16 NHWC output and reduces the following BatchNorm's batch
  statistics in its epilogue (``forward_stats`` -> ``BNAct(stats=...)``);
* backward: grad-weight only (the image needs no gradient) -- added into the
  optimizer's fp32 gradient arena on the bf16-shadow path, like FastConv2d.

Without autocast (fp32 compute, the reference's precision) the fp32 kernels of
``csrc/kernels/stem_f32.hip`` run instead (fp32 output and statistics).

MIOpen's implicit GEMM handles the 3-channel input badly (0.7 ms per
direction at bs512, profiles/r01_resnet50_conv_roofline_bs512.txt).
Reference parity: the reference's ResNet-50 is torchvision's
(dl_trainer.py:88-90), whose ``conv1`` this replaces one-for-one.
Everything else (CPU, eval, other dtypes/layouts) is the stock convolution.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import load

_CL = torch.channels_last
_ENABLED = os.environ.get("GKSGD_STEM", "1") != "0"
_F32 = os.environ.get("GKSGD_STEM_F32", "1") != "0"   # fp32 stem kernels (else MIOpen at fp32)
# fp32 stem forward on the bf16x6 kernel when the fp32 GEMM family is bf16x6
# (ops/conv1x1.py set_f32_matmul; GKSGD_STEM_X6=0 keeps the fp32-MFMA kernel)
_X6 = os.environ.get("GKSGD_STEM_X6", "1") != "0"


from . import conv1x1 as _cv  # noqa: E402


def _g():
    return torch.ops.gksgd


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, param, sink, stats_box):
        g = _g()
        N, _, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        wp = torch.empty(64, 224, dtype=torch.bfloat16, device=x.device)
        g.stem_pack(param.detach().float(), wp)
        y = torch.empty((N, 64, OH, OW), dtype=torch.bfloat16, device=x.device, memory_format=_CL)
        st = None
        if stats_box is not None:
            st = torch.empty(2, 256, 64, dtype=torch.float32, device=x.device)
        rows = g.stem_fwd(x, wp, y, st)
        if st is not None:
            stats_box.append((st, int(rows)))
        ctx.sink = sink
        ctx.param_dtype = param.dtype
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        g = _g()
        dy = dy.to(torch.bfloat16).contiguous(memory_format=_CL)
        gparam = None
        if ctx.needs_input_grad[1]:
            N, _, H, W = x.shape
            part = torch.empty(int(g.stem_wgrad_ws(N, H, W)), dtype=torch.float32, device=x.device)
            sink = ctx.sink
            if sink is not None and getattr(sink, "grad_view", None) is not None:
                sink.check()
                g.stem_wgrad(x, dy, sink.grad_view, part)
            else:
                out = torch.zeros(64, 3, 7, 7, dtype=torch.float32, device=x.device)
                g.stem_wgrad(x, dy, out, part)
                if sink is not None:
                    sink(out)
                else:
                    gparam = out.to(ctx.param_dtype)
        return None, gparam, None, None


class _StemF32Fn(torch.autograd.Function):
    """fp32 stem (csrc/kernels/stem_f32.hip): fp32 products and sums, the
    reference's precision; grad-weight into the fp32 direct-gradient arena
    when the model is on that path (parallel/shadow.py install_direct_grads)."""

    @staticmethod
    def forward(ctx, x, param, sink, stats_box):
        g = _g()
        N = x.shape[0]
        y = torch.empty((N, 64, 112, 112), dtype=torch.float32, device=x.device, memory_format=_CL)
        st = None
        if stats_box is not None:
            st = torch.empty(2, 512, 64, dtype=torch.float32, device=x.device)
        x6 = _X6 and _cv.f32_matmul() == "bf16x6"
        if x6:
            # bf16x6 products (fp32-accurate, stem_f32.hip stem_f32x6_fwd_kernel):
            # the weight planes are split into a per-call workspace
            wp3 = torch.empty(int(g.stem_f32x6_wplanes()), dtype=torch.bfloat16, device=x.device)
            rows = g.stem_f32x6_fwd(x, param.detach(), y, st, wp3)
        else:
            rows = g.stem_f32_fwd(x, param.detach(), y, st)
        if st is not None:
            stats_box.append((st, int(rows)))
        ctx.sink = sink
        ctx.x6 = x6     # the grad-weight runs the same family (stem_f32x6_wgrad_kernel)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        g = _g()
        dy = dy.float().contiguous(memory_format=_CL)
        gparam = None
        if ctx.needs_input_grad[1]:
            part = torch.empty(int(g.stem_f32_wgrad_ws(x.shape[0])), dtype=torch.float32, device=x.device)
            sink = ctx.sink
            if sink is not None and getattr(sink, "grad_view", None) is not None:
                sink.check()
                g.stem_f32_wgrad(x, dy, sink.grad_view, part, ctx.x6)
            else:
                out = torch.zeros(64, 3, 7, 7, dtype=torch.float32, device=x.device)
                g.stem_f32_wgrad(x, dy, out, part, ctx.x6)
                if sink is not None:
                    sink(out)
                else:
                    gparam = out
        return None, gparam, None, None


class StemConv(nn.Conv2d):
    """``nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)`` with the
    gfx950 stem kernels on the training path."""

    def __init__(self, in_channels: int = 3, out_channels: int = 64):
        super().__init__(in_channels, out_channels, 7, stride=2, padding=3, bias=False)

    def _fast(self, x: torch.Tensor) -> bool:
        dev = x.device.type
        return (_ENABLED and x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and self.out_channels == 64 and
                x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous(memory_format=_CL) and
                torch.is_autocast_enabled(dev) and torch.get_autocast_dtype(dev) == torch.bfloat16 and
                not (torch.is_grad_enabled() and x.requires_grad) and load() and
                bool(_g().stem_supported(x.shape[2], x.shape[3])))

    def _fast_f32(self, x: torch.Tensor) -> bool:
        dev = x.device.type
        return (_ENABLED and _F32 and x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and self.out_channels == 64 and
                x.dtype == torch.float32 and self.weight.dtype == torch.float32 and
                x.is_contiguous(memory_format=_CL) and x.data_ptr() % 16 == 0 and
                not torch.is_autocast_enabled(dev) and not (torch.is_grad_enabled() and x.requires_grad) and
                load() and bool(_g().stem_f32_supported(x.shape[2], x.shape[3])))

    def _run(self, x: torch.Tensor, box):
        if self._fast_f32(x):
            table = getattr(self, "_gk_direct_grads", None) or {}
            sink = table.get("weight")
            if not torch.is_grad_enabled() or not self.weight.requires_grad:
                sink = None
            return _StemF32Fn.apply(x, self.weight, sink, box)
        if self._fast(x):
            table = getattr(self, "_gk_shadow", None)
            info = table.get("weight") if table else None
            sink = info[1] if info is not None else None
            if not torch.is_grad_enabled() or not self.weight.requires_grad:
                sink = None
            return _StemFn.apply(x, self.weight, sink, box)
        slow = getattr(self, "_gk_slow", None)
        return slow(x) if slow is not None else super().forward(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self._run(x, None)

    def forward_stats(self, x: torch.Tensor):
        """(y, stats) -- see FastConv2d.forward_stats."""
        box = []
        y = self._run(x, box)
        return y, (box[0] if box else None)
