"""bf16 LSTM layers: hipBLASLt GEMMs + one fused HIP cell kernel per step.

``GkLSTM`` is a drop-in ``nn.LSTM`` (sequence-first, same parameter names
``weight_ih_l{k}`` / ``weight_hh_l{k}`` / ``bias_ih_l{k}`` / ``bias_hh_l{k}``,
PyTorch gate order i, f, g, o, dropout between layers) for the PTB language
model (BASELINE config 4; reference models/lstm.py:5-47).  On ROCm
``nn.LSTM`` dispatches to MIOpen's RNN, which computes in **fp16** even under
bf16 autocast and runs each step as a poorly tiled GEMM plus two hidden-update
kernels (profiles/r01_lstm_kernel_stats.csv).  Per layer this module runs

  forward : xg = x W_ih^T + (b_ih + b_hh)          one GEMM over all T steps
            per step: hg = h W_hh^T (GEMM); lstm_cell_fwd(xg[t], hg, c) -> h, c, gates
  backward: per step: lstm_cell_bwd(dout[t], dh_rec, dc) -> dG[t], dc;
                      dh_rec = dG[t] W_hh (GEMM)
            dW_ih += dG^T x, dW_hh += dG^T h_prev, db += colsum(dG), dx = dG W_ih
            -- four GEMMs over all T steps; with the bf16 shadow
            (parallel/shadow.py) the weight / bias gradients go straight into
            the optimizer's fp32 arena (fp32-output GEMM, fused column pass).

in bf16 with fp32 cell state.  Off the GPU (or outside bf16 autocast) the
same recurrence runs in fp32 with PyTorch ops, so CPU tests compare it with
``nn.LSTM`` exactly.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import load, require_native
from .linear import _target, _wgrad_into, bias_grad_acc_


def _g():
    return torch.ops.gksgd


def _cell_fwd_ref(xg, hg, c_prev, c_out, h_out, gates_out):
    a = xg.float() + hg.float()
    i, f, g, o = a.chunk(4, dim=1)
    i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
    c = f * c_prev + i * g
    c_out.copy_(c)
    h_out.copy_(o * torch.tanh(c))
    gates_out.copy_(torch.cat([i, f, g, o], dim=1))


def _cell_bwd_ref(dout, dh_rec, dc_next, gates, c, c_prev, dG_out, dc_prev_out):
    i, f, g, o = gates.chunk(4, dim=1)
    dh = torch.zeros_like(c)
    if dout is not None:
        dh = dh + dout.float()
    if dh_rec is not None:
        dh = dh + dh_rec.float()
    tc = torch.tanh(c)
    dc = dh * o * (1 - tc * tc)
    if dc_next is not None:
        dc = dc + dc_next
    dG_out.copy_(torch.cat([dc * g * i * (1 - i), dc * c_prev * f * (1 - f), dc * i * (1 - g * g),
                            dh * tc * o * (1 - o)], dim=1))
    dc_prev_out.copy_(dc * f)


class _LSTMLayerFn(torch.autograd.Function):
    """One LSTM layer over a whole sequence (one autograd node: the step loop
    lives inside forward / backward)."""

    @staticmethod
    def forward(ctx, x, h0, c0, w_ih, w_hh, b_ih, b_hh, shadows, sinks, fast):
        T, B, _ = x.shape
        H = w_hh.shape[1]
        cd = torch.bfloat16 if fast else torch.float32
        dev = x.device
        wih = shadows[0] if shadows[0] is not None else w_ih.detach().to(cd)
        whh = shadows[1] if shadows[1] is not None else w_hh.detach().to(cd)
        x2 = x.reshape(T * B, -1).to(cd).contiguous()
        bias = (b_ih.detach().float() + b_hh.detach().float()).to(cd)
        xg = torch.addmm(bias, x2, wih.t()).view(T, B, 4 * H)
        out = torch.empty(T, B, H, dtype=cd, device=dev)
        c_all = torch.empty(T + 1, B, H, dtype=torch.float32, device=dev)
        c_all[0].copy_(c0)
        gates = torch.empty(T, B, 4 * H, dtype=torch.float32, device=dev)
        h = h0.to(cd).contiguous()
        h0c = h
        ops = _g() if fast else None
        whh_t = whh.t()
        for t in range(T):
            hg = torch.mm(h, whh_t)
            if fast:
                ops.lstm_cell_fwd(xg[t], hg, c_all[t], c_all[t + 1], out[t], gates[t])
            else:
                _cell_fwd_ref(xg[t], hg, c_all[t], c_all[t + 1], out[t], gates[t])
            h = out[t]
        ctx.save_for_backward(x2, h0c, out, c_all, gates, wih, whh)
        ctx.sinks, ctx.fast, ctx.cd = sinks, fast, cd
        ctx.dtypes = (x.dtype, h0.dtype, c0.dtype, w_ih.dtype)
        ctx.in_shape = x.shape
        return out, out[T - 1].clone(), c_all[T].clone()

    @staticmethod
    def backward(ctx, dout, dh_n, dc_n):
        x2, h0c, out, c_all, gates, wih, whh = ctx.saved_tensors
        T, B, H = out.shape
        cd, fast = ctx.cd, ctx.fast
        dev = out.device
        ops = _g() if fast else None
        dG = torch.empty(T, B, 4 * H, dtype=cd, device=dev)
        if dout is not None:
            dout = dout.to(cd).contiguous()
        dh_rec = dh_n.to(cd).contiguous() if dh_n is not None else None
        dc = dc_n.float().contiguous() if dc_n is not None else None
        bufs = [torch.empty(B, H, dtype=torch.float32, device=dev) for _ in range(2)]
        for t in range(T - 1, -1, -1):
            dc_prev = bufs[t & 1]
            do_t = dout[t] if dout is not None else None
            if fast:
                ops.lstm_cell_bwd(do_t, dh_rec, dc, gates[t], c_all[t + 1], c_all[t], dG[t], dc_prev)
            else:
                _cell_bwd_ref(do_t, dh_rec, dc, gates[t], c_all[t + 1], c_all[t], dG[t], dc_prev)
            dc = dc_prev
            dh_rec = torch.mm(dG[t], whh)
        dG2 = dG.view(T * B, 4 * H)
        xdt, hdt, cdt, wdt = ctx.dtypes
        dx = torch.mm(dG2, wih).view(ctx.in_shape) if ctx.needs_input_grad[0] else None
        dh0 = dh_rec if ctx.needs_input_grad[1] else None
        dc0 = dc if ctx.needs_input_grad[2] else None
        grads: List[Optional[torch.Tensor]] = [None, None, None, None]
        wsinks = ctx.sinks
        h_prev = None
        for k, need in enumerate(ctx.needs_input_grad[3:7]):
            if not need:
                continue
            sink = wsinks[k]
            tgt = _target(sink)
            own = tgt is None
            if own:
                shape = (4 * H, x2.shape[1]) if k == 0 else ((4 * H, H) if k == 1 else (4 * H,))
                tgt = torch.zeros(shape, dtype=torch.float32, device=dev)
            if k == 0:
                _wgrad_into(dG2, x2, tgt)
            elif k == 1:
                if h_prev is None:
                    h_prev = torch.cat([h0c.unsqueeze(0), out[:-1]]).view(T * B, H)
                _wgrad_into(dG2, h_prev, tgt)
            else:
                bias_grad_acc_(tgt, dG2)
            if own:
                if sink is not None:
                    sink(tgt)
                else:
                    grads[k] = tgt.to(wdt)
        return (dx, dh0, dc0, grads[0], grads[1], grads[2], grads[3], None, None, None)


class GkLSTM(nn.Module):
    """``nn.LSTM(input_size, hidden_size, num_layers, dropout)`` (sequence-first,
    biases on, unidirectional) on bf16 GEMMs + fused HIP cells."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1, dropout: float = 0.0):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers, self.dropout = input_size, hidden_size, num_layers, dropout
        for k in range(num_layers):
            inp = input_size if k == 0 else hidden_size
            setattr(self, "weight_ih_l%d" % k, nn.Parameter(torch.empty(4 * hidden_size, inp)))
            setattr(self, "weight_hh_l%d" % k, nn.Parameter(torch.empty(4 * hidden_size, hidden_size)))
            setattr(self, "bias_ih_l%d" % k, nn.Parameter(torch.empty(4 * hidden_size)))
            setattr(self, "bias_hh_l%d" % k, nn.Parameter(torch.empty(4 * hidden_size)))
        self.reset_parameters()

    def reset_parameters(self) -> None:   # nn.LSTM's init
        std = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -std, std)

    @staticmethod
    def _layer_names(k: int):
        return [n % k for n in ("weight_ih_l%d", "weight_hh_l%d", "bias_ih_l%d", "bias_hh_l%d")]

    def forward(self, x: torch.Tensor, hx: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        T, B, _ = x.shape
        L, H = self.num_layers, self.hidden_size
        if hx is None:
            z = torch.zeros(L, B, H, dtype=torch.float32, device=x.device)
            hx = (z, z)
        h0, c0 = hx
        dev = x.device.type
        fast = (x.is_cuda and torch.is_autocast_enabled(dev) and torch.get_autocast_dtype(dev) == torch.bfloat16
                and load())
        if x.is_cuda and fast:
            require_native(x)
        table = getattr(self, "_gk_shadow", None) if fast else None
        grad_on = torch.is_grad_enabled()
        hn, cn = [], []
        y = x
        for k in range(L):
            names = self._layer_names(k)
            params = [getattr(self, n) for n in names]
            shadows, sinks = [None, None], [None, None, None, None]
            if table:
                for j, (n, p) in enumerate(zip(names, params)):
                    info = table.get(n)
                    if info is None:
                        continue
                    if j < 2:
                        shadows[j] = info[0]
                    if grad_on and p.requires_grad:
                        sinks[j] = info[1]
            with torch.autocast(dev, enabled=False):
                y, h_k, c_k = _LSTMLayerFn.apply(y, h0[k], c0[k], *params, tuple(shadows), tuple(sinks), fast)
            hn.append(h_k)
            cn.append(c_k)
            if k < L - 1 and self.dropout > 0 and self.training:
                y = F.dropout(y, self.dropout, training=True)
        return y, (torch.stack(hn), torch.stack(cn))

    def extra_repr(self) -> str:
        return "%d, %d, num_layers=%d, dropout=%s" % (self.input_size, self.hidden_size, self.num_layers, self.dropout)
