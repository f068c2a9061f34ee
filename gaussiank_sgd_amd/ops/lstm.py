"""LSTM layers: a split-K MFMA step GEMM + one fused HIP cell kernel per step
(bf16 under autocast, fp32 at the reference's precision).

``GkLSTM`` is a drop-in ``nn.LSTM`` (sequence-first, same parameter names
``weight_ih_l{k}`` / ``weight_hh_l{k}`` / ``bias_ih_l{k}`` / ``bias_hh_l{k}``,
PyTorch gate order i, f, g, o, dropout between layers) for the PTB language
model (BASELINE config 4; reference models/lstm.py:5-47).  On ROCm
``nn.LSTM`` dispatches to MIOpen's RNN, which computes in **fp16** even under
bf16 autocast and runs each step as a poorly tiled GEMM plus two hidden-update
kernels (profiles/r01_lstm_kernel_stats.csv).  Per layer this module runs

  forward : xg = x W_ih^T + (b_ih + b_hh)          one GEMM over all T steps
            per step: P = h W_hh^T (lstm_rec_gemm, fp32 K-slice partials);
                      lstm_cell_fwd(xg[t], P, c) -> h, c, gates
  backward: per step: lstm_cell_bwd(dout[t], P, dc) -> dG[t], dc;
                      P = dG[t] W_hh (lstm_rec_gemm)
            dW_ih += dG^T x, dW_hh += dG^T h_prev, db += colsum(dG), dx = dG W_ih
            -- four GEMMs over all T steps; with the bf16 shadow
            (parallel/shadow.py) the weight / bias gradients go straight into
            the optimizer's fp32 arena (fp32-output GEMM, fused column pass).

in bf16 with fp32 cell state.  The step GEMM is tiny (M = batch, K = H) and
latency-bound as one GEMM (~20-35 us for H = 1500 on hipBLASLt,
bench/lstm_gemm_probe.py); split over S K-slices into a few hundred
workgroups it runs a handful of MFMA steps per wave, and the cell kernel sums
the fp32 slices on load (no atomics, no extra reduction launch).  Its
operands are 64-padded (h_pad / dG_pad written by the cell kernels, W_hh
padded once per forward).  fp32 inputs without autocast (the reference's
precision) run the same kernels on fp32 operands (``v_mfma_f32_16x16x4_f32``
step GEMM, fp32 h / dG).  Off the GPU the same recurrence runs in fp32 with
PyTorch ops, so CPU tests compare it with ``nn.LSTM`` exactly.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import load, require_native
from .linear import _dgrad as _lin_dgrad
from .linear import _fwd as _lin_fwd
from .linear import _target, _wgrad_forkable, _wgrad_into, bias_grad_acc_
from . import streams


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


def _pad64(n: int) -> int:
    return (n + 63) // 64 * 64


def _cdiv(a: int, b: int) -> int:
    return (a + b - 1) // b


# Step GEMM per direction: None = autotuned once per (direction, dtype, batch,
# H) among hipBLASLt and the split-K kernel at every K-slice count S (cached
# with the other GEMM choices, ops/conv1x1.py _pick).  An int forces the
# round-5 rule instead: split-K with the default S up to that batch, hipBLASLt
# above.  Measured on MI355X (bench/lstm_x6_probe.py, profiles/r06_lstm_step_probe.json),
# fp32 H = 1500: B = 20 forward split-K S = 8 11.9 us vs the rule's S = 4 18.5,
# backward S = 24 14.2 vs S = 8 33.6 (hipBLASLt 19 / 22); B = 128 hipBLASLt
# 29 / 28.5 vs split-K 34 / 39.5 -- no single rule is right for every shape.
# GKSGD_LSTM_SPLITK="fwd:<maxB>,bwd:<maxB>" forces the rule.
SPLITK_MAX_BATCH = {"fwd": None, "bwd": None}
for _kv in os.environ.get("GKSGD_LSTM_SPLITK", "").split(","):
    if ":" in _kv:
        _k, _v = _kv.split(":", 1)
        SPLITK_MAX_BATCH[_k.strip()] = int(_v)


def _splits(kblocks: int, nblocks: int, target: int = 512) -> int:
    """K-slice count S for the split-K step GEMM: the largest divisor of the
    64-deep K-block count keeping S * nblocks <= target workgroups (two per
    CU) and every slice >= two K-blocks deep."""
    best = 1
    for d in range(2, kblocks + 1):
        if kblocks % d == 0 and d * nblocks <= target and kblocks // d >= 2:
            best = d
    return best


def _step_plan(direction: str, cd: torch.dtype, B: int, H: int, dev) -> Tuple[str, int]:
    """("hip", S): the split-K kernel with S K-slices on the 64-padded
    operands; ("blas", 0): hipBLASLt on the unpadded ones."""
    Hp = _pad64(H)
    fwd = direction == "fwd"
    kb, nb = (Hp // 64, 4 * Hp // 64) if fwd else (4 * Hp // 64, Hp // 64)
    mb = _cdiv(B, 128)
    mx = SPLITK_MAX_BATCH[direction]
    if mx is not None:
        if B > mx:
            return ("blas", 0)
        return ("hip", _splits(kb, nb * mb, target=512 if fwd else 256))
    from . import conv1x1 as _cv
    key = ("lstm_step", direction, B, H, "f32" if cd == torch.float32 else "bf16")
    got = _cv._choices.get(key)
    if got is not None:
        return (got[0], int(got[1]))
    g = _g()
    M, N, K = (B, 4 * Hp, Hp) if fwd else (B, Hp, 4 * Hp)
    a = torch.zeros(M, K, dtype=cd, device=dev)
    w = torch.zeros(N, K, dtype=cd, device=dev)
    cands = []
    for S in range(1, kb + 1):
        if kb % S or (S > 1 and kb // S < 2) or S * nb * mb > 2048:
            continue
        P = torch.empty(S, M, N, dtype=torch.float32, device=dev)
        cands.append((("hip", S, 0), (lambda S=S, P=P: g.lstm_rec_gemm(a, w, P, S))))
    ab = torch.zeros(B, H if fwd else 4 * H, dtype=cd, device=dev)
    wb = torch.zeros(4 * H, H, dtype=cd, device=dev)
    cands.append((("blas", 0, 0), (lambda: torch.mm(ab, wb.t())) if fwd else (lambda: torch.mm(ab, wb))))
    ch = _cv._pick(key, cands)
    return (ch[0], int(ch[1]))


# fp32 step GEMM on the bf16x6 split-K kernel (lstm.hip rec_gemm_x6_kernel:
# fp32-accurate on the bf16 matrix cores, W_hh split once into three bf16
# planes).  Opt-in (GKSGD_LSTM_X6=1): the step GEMM is bound by its operand
# loads, not by the matrix pipe, and the three planes are 1.5x the bytes of
# fp32 -- measured 37 / 47 us (B = 128 forward / backward, best S) against
# 34 / 39.5 for the fp32-MFMA kernel and 29 / 28.5 for hipBLASLt, and the
# LSTM step 20.9 vs 16.3 ms (r6c4, profiles/r06_lstm_step_probe.json).
_X6 = os.environ.get("GKSGD_LSTM_X6", "0") == "1"


def split3(w: torch.Tensor) -> torch.Tensor:
    """Exact fp32 -> three bf16 planes [3, *w.shape] with w = hi + mid + lo
    (round-to-nearest-even at each step, as mfma_util.h split3x8: every
    residual is exact in fp32, so the three parts hold all 24 mantissa bits)."""
    hi = w.to(torch.bfloat16)
    r = w - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return torch.stack([hi, mid, lo]).contiguous()


def _splits(kblocks: int, nblocks: int, target: int = 512) -> int:
    """K-slice count S for the split-K step GEMM: the largest divisor of the
    64-deep K-block count keeping S * nblocks <= target workgroups (two per
    CU) and every slice >= two K-blocks deep."""
    best = 1
    for d in range(2, kblocks + 1):
        if kblocks % d == 0 and d * nblocks <= target and kblocks // d >= 2:
            best = d
    return best


class _LSTMLayerFn(torch.autograd.Function):
    """One LSTM layer over a whole sequence (one autograd node: the step loop
    lives inside forward / backward)."""

    @staticmethod
    def forward(ctx, x, h0, c0, w_ih, w_hh, b_ih, b_hh, shadows, sinks, fast, cd=torch.bfloat16):
        # fast: the HIP kernels (split-K step GEMM + fused cells) in the compute
        # dtype cd -- bf16 under autocast, fp32 otherwise (the reference's precision)
        T, B, _ = x.shape
        H = w_hh.shape[1]
        cd = cd if fast else torch.float32
        dev = x.device
        wih = shadows[0] if shadows[0] is not None else w_ih.detach().to(cd)
        whh = shadows[1] if shadows[1] is not None else w_hh.detach().to(cd)
        x2 = x.reshape(T * B, -1).to(cd).contiguous()
        if fast:
            # the autotuned GEMM of ops/linear.py: HIP kernels on zero-padded
            # operands (H = 1500 is not a multiple of 64) or hipBLASLt, whichever
            # is faster for the shape; the bias in its epilogue
            bias32 = (b_ih.detach().float() + b_hh.detach().float()).contiguous()
            xg = _lin_fwd(x2, wih.contiguous(), bias32).contiguous().view(T, B, 4 * H)
        else:
            bias = (b_ih.detach().float() + b_hh.detach().float()).to(cd)
            xg = torch.addmm(bias, x2, wih.t()).view(T, B, 4 * H)
        out = torch.empty(T, B, H, dtype=cd, device=dev)
        c_all = torch.empty(T + 1, B, H, dtype=torch.float32, device=dev)
        c_all[0].copy_(c0)
        gates = torch.empty(T, B, 4 * H, dtype=torch.float32, device=dev)
        h = h0.to(cd).contiguous()
        h0c = h
        x6 = fast and cd == torch.float32 and _X6
        plan = _step_plan("fwd", cd, B, H, dev) if fast else ("blas", 0)
        if fast and (x6 or plan[0] == "hip"):
            # split-K step GEMM over 64-padded operands (lstm.hip rec_gemm_kernel;
            # fp32: rec_gemm_x6_kernel on the three bf16 planes of W_hh)
            ops = _g()
            Hp = _pad64(H)
            wpf = torch.zeros(4, Hp, Hp, dtype=cd, device=dev)
            wpf[:, :H, :H] = whh.view(4, H, H)
            wpf = wpf.view(4 * Hp, Hp)
            wpf3 = split3(wpf) if x6 else None
            S = _splits(Hp // 64, (4 * Hp // 64) * _cdiv(B, 128)) if x6 else plan[1]
            P = torch.empty(S, B, 4 * Hp, dtype=torch.float32, device=dev)
            h_pad = torch.zeros(B, Hp, dtype=cd, device=dev)
            h_pad[:, :H] = h
            for t in range(T):
                if x6:
                    ops.lstm_rec_gemm_x6(h_pad, wpf3, P, S)
                else:
                    ops.lstm_rec_gemm(h_pad, wpf, P, S)
                ops.lstm_cell_fwd(xg[t], None, P, S, c_all[t], c_all[t + 1], out[t], h_pad, gates[t])
        else:
            whh_t = whh.t()
            for t in range(T):
                if fast:
                    _g().lstm_cell_fwd(xg[t], torch.mm(h, whh_t), None, 0, c_all[t], c_all[t + 1], out[t], None,
                                       gates[t])
                else:
                    _cell_fwd_ref(xg[t], torch.mm(h, whh_t), c_all[t], c_all[t + 1], out[t], gates[t])
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
        dG = torch.empty(T, B, 4 * H, dtype=cd, device=dev)
        if dout is not None:
            dout = dout.to(cd).contiguous()
        dc = dc_n.float().contiguous() if dc_n is not None else None
        bufs = [torch.empty(B, H, dtype=torch.float32, device=dev) for _ in range(2)]
        need_dh0 = ctx.needs_input_grad[1]
        x6 = fast and cd == torch.float32 and _X6
        plan = _step_plan("bwd", cd, B, H, dev) if fast else ("blas", 0)
        if fast and (x6 or plan[0] == "hip"):
            ops = _g()
            Hp = _pad64(H)
            # wpb[j'][k Hp + j] = W_hh[k H + j][j']: dh = dG_pad wpb^T
            wpb = torch.zeros(Hp, 4, Hp, dtype=cd, device=dev)
            wpb[:H, :, :H] = whh.view(4, H, H).permute(2, 0, 1)
            wpb = wpb.view(Hp, 4 * Hp)
            wpb3 = split3(wpb) if x6 else None
            S = _splits(4 * Hp // 64, (Hp // 64) * _cdiv(B, 128), target=256) if x6 else plan[1]
            P = torch.empty(S, B, Hp, dtype=torch.float32, device=dev)
            dG_pad = torch.zeros(B, 4 * Hp, dtype=cd, device=dev)
            for t in range(T - 1, -1, -1):
                dc_prev = bufs[t & 1]
                do_t = dout[t] if dout is not None else None
                if t == T - 1 and dh_n is not None:
                    do_t = (dh_n.float() if do_t is None else do_t.float() + dh_n.float()).to(cd)
                ops.lstm_cell_bwd(do_t, None, P if t < T - 1 else None, S, dc, gates[t], c_all[t + 1], c_all[t],
                                  dG[t], dG_pad, dc_prev)
                dc = dc_prev
                if t > 0 or need_dh0:
                    if x6:
                        ops.lstm_rec_gemm_x6(dG_pad, wpb3, P, S)
                    else:
                        ops.lstm_rec_gemm(dG_pad, wpb, P, S)
            dh_rec = P.sum(0)[:, :H] if need_dh0 else None
        else:
            dh_rec = dh_n.to(cd).contiguous() if dh_n is not None else None
            for t in range(T - 1, -1, -1):
                dc_prev = bufs[t & 1]
                do_t = dout[t] if dout is not None else None
                if fast:
                    _g().lstm_cell_bwd(do_t, dh_rec, None, 0, dc, gates[t], c_all[t + 1], c_all[t], dG[t], None,
                                       dc_prev)
                else:
                    _cell_bwd_ref(do_t, dh_rec, dc, gates[t], c_all[t + 1], c_all[t], dG[t], dc_prev)
                dc = dc_prev
                dh_rec = torch.mm(dG[t], whh)
        dG2 = dG.view(T * B, 4 * H)
        xdt, hdt, cdt, wdt = ctx.dtypes
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (_lin_dgrad(dG2, wih.contiguous()) if fast else torch.mm(dG2, wih)).view(ctx.in_shape)
        dh0 = dh_rec.to(hdt) if need_dh0 else None
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
            if k < 2:
                if k == 1 and h_prev is None:
                    h_prev = torch.cat([h0c.unsqueeze(0), out[:-1]]).view(T * B, H)
                xk = x2 if k == 0 else h_prev
                if not own and fast and not getattr(sink, "shared", False) and _wgrad_forkable(dG2, xk):
                    # on the side stream: overlaps the next layer's serial recurrence
                    side = streams.fork(dev)
                    with torch.cuda.stream(side):
                        _wgrad_into(dG2, xk, tgt)
                    streams.hold(dev, dG2, xk)
                else:
                    _wgrad_into(dG2, xk, tgt)
            else:
                bias_grad_acc_(tgt, dG2)
            if own:
                if sink is not None:
                    sink(tgt)
                else:
                    grads[k] = tgt.to(wdt)
        return (dx, dh0, dc0, grads[0], grads[1], grads[2], grads[3], None, None, None, None)


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
        bf16 = x.is_cuda and torch.is_autocast_enabled(dev) and torch.get_autocast_dtype(dev) == torch.bfloat16
        # fp32 (no autocast, the reference's precision) runs the same HIP step
        # GEMM and cell kernels on fp32 operands (GKSGD_LSTM_F32=0: PyTorch ops)
        f32 = (x.is_cuda and not torch.is_autocast_enabled(dev) and x.dtype == torch.float32 and
               os.environ.get("GKSGD_LSTM_F32", "1") != "0")
        fast = (bf16 or f32) and load()
        if x.is_cuda and fast:
            require_native(x)
        cd = torch.bfloat16 if bf16 else torch.float32
        table = getattr(self, "_gk_shadow", None) if (fast and bf16) else None
        direct = getattr(self, "_gk_direct_grads", None) if (fast and not bf16) else None
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
            elif direct:
                for j, (n, p) in enumerate(zip(names, params)):
                    if n in direct and grad_on and p.requires_grad:
                        sinks[j] = direct[n]
            with torch.autocast(dev, enabled=False):
                y, h_k, c_k = _LSTMLayerFn.apply(y, h0[k], c0[k], *params, tuple(shadows), tuple(sinks), fast, cd)
            hn.append(h_k)
            cn.append(c_k)
            if k < L - 1 and self.dropout > 0 and self.training:
                y = F.dropout(y, self.dropout, training=True)
        return y, (torch.stack(hn), torch.stack(cn))

    def extra_repr(self) -> str:
        return "%d, %d, num_layers=%d, dropout=%s" % (self.input_size, self.hidden_size, self.num_layers, self.dropout)
