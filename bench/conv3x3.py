#!/usr/bin/env python3
"""Implicit-GEMM KxK convolution kernels (gemm.hip conv_nt / conv_tn_acc) vs
MIOpen on the ResNet-50 3x3 shapes: best kernel configuration per shape and
direction (forward; grad-input for stride 1 = forward of dY with the flipped,
transposed weight; grad-weight), efficiency against the MFMA/HBM roofline.

Usage (GPU): python bench/conv3x3.py [--batch 512] [--json-out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_HERE, "tuning", "miopen"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

PEAK = 2.5e15
HBM = 6.3e12
# (Cin=Cout, H_in, stride, count) of ResNet-50's 3x3 convolutions
SHAPES = [(64, 56, 1, 3), (128, 56, 2, 1), (128, 28, 1, 3), (256, 28, 2, 1), (256, 14, 1, 5), (512, 14, 2, 1),
          (512, 7, 1, 2)]
NT_CFGS = [1, 2, 3, 4, 21, 22, 23, 24, 121, 122, 123, 124, 25, 26, 27, 125, 126, 127]
TN_CFGS = [(c, sp) for c in (1, 2, 3, 4, 5, 6, 7, 8, 21, 22, 23, 24, 27) for sp in (0, 128)]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    from gaussiank_sgd_amd import ops
    assert ops.load(), ops._load_error
    g = torch.ops.gksgd
    dev = torch.device("cuda", 0)
    zero = torch.zeros(64, device=dev, dtype=torch.bfloat16)
    rows = []
    tot = {k: [0.0, 0.0, 0.0] for k in ("fwd", "dgrad", "wgrad")}
    for (C, H, s, cnt) in SHAPES:
        N = args.batch
        x = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=s, padding=1)
        dy = torch.randn_like(y)
        OH = y.shape[2]
        M = N * OH * OH
        flops = 2.0 * M * C * C * 9
        nbytes = (x.numel() + y.numel() + w.numel()) * 2
        roof = max(flops / PEAK, nbytes / HBM)
        yo = torch.empty_like(y)
        dxo = torch.empty_like(x)
        wflip = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        dwo = torch.zeros(C, C, 3, 3, device=dev).contiguous(memory_format=torch.channels_last)
        xg = x.detach().requires_grad_(True)
        wg = w.detach().requires_grad_(True)
        yg = F.conv2d(xg, wg, stride=s, padding=1)
        theirs = {"fwd": lambda: F.conv2d(x, w, stride=s, padding=1),
                  "dgrad": lambda: torch.autograd.grad(yg, xg, dy, retain_graph=True),
                  "wgrad": lambda: torch.autograd.grad(yg, wg, dy, retain_graph=True)}
        ours = {"fwd": [(c, lambda c=c: g.conv_nt(x, w, yo, zero, s, 1, c, 0)) for c in NT_CFGS],
                "dgrad": ([(c, lambda c=c: g.conv_nt(dy, wflip, dxo, zero, 1, 1, c, 0)) for c in NT_CFGS]
                          if s == 1 else []),
                "wgrad": [(cs, lambda cs=cs: g.conv_tn_acc(dy, x, dwo, zero, s, 1, cs[0], cs[1])) for cs in TN_CFGS]}
        # numerics
        ref = F.conv2d(x.float()[:8], w.float(), stride=s, padding=1)
        g.conv_nt(x, w, yo, zero, s, 1, 0, 0)
        e_f = float((yo[:8].float() - ref).abs().max() / ref.abs().max())
        e_d = None
        if s == 1:
            g.conv_nt(dy, wflip, dxo, zero, 1, 1, 0, 0)
            rd = torch.nn.grad.conv2d_input(x[:8].shape, w.float(), dy[:8].float(), stride=1, padding=1)
            e_d = float((dxo[:8].float() - rd).abs().max() / rd.abs().max())
        dwo.zero_()
        g.conv_tn_acc(dy[:8], x[:8], dwo, zero, s, 1, 0, 0)
        rw = torch.nn.grad.conv2d_weight(x[:8].float(), w.shape, dy[:8].float(), stride=s, padding=1)
        e_w = float((dwo - rw).abs().max() / rw.abs().max())
        errs = {"fwd": e_f, "dgrad": e_d, "wgrad": e_w}
        for name in ("fwd", "dgrad", "wgrad"):
            t_m = timeit(theirs[name])
            best, best_t = None, float("inf")
            for c, fn in ours[name]:
                t = timeit(fn)
                if t < best_t:
                    best, best_t = c, t
            tot[name][0] += min(best_t, t_m) * cnt
            tot[name][1] += t_m * cnt
            tot[name][2] += roof * cnt
            r = dict(op=name, C=C, H=H, stride=s, count=cnt, M=M, best_cfg=best,
                     ours_us=round(best_t * 1e6, 1) if best is not None else None, miopen_us=round(t_m * 1e6, 1),
                     roofline_us=round(roof * 1e6, 1), eff=round(roof / best_t, 3) if best is not None else None,
                     speedup=round(t_m / best_t, 2) if best is not None else None, rel_err=errs[name])
            rows.append(r)
            print(json.dumps(r), flush=True)
        del x, w, y, dy, yo, dxo, wflip, dwo, xg, wg, yg
    for name, (a, b, c) in tot.items():
        print("TOTAL %-5s best-of %.2f ms  miopen %.2f ms  roofline %.2f ms" % (name, a * 1e3, b * 1e3, c * 1e3))
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump({"rows": rows, "totals_ms": {k: [v[0] * 1e3, v[1] * 1e3, v[2] * 1e3] for k, v in tot.items()}},
                      f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
