#!/usr/bin/env python3
"""1x1-convolution GEMM kernels (ops/csrc/kernels/gemm.hip) vs MIOpen on the
ResNet-50 stride-1 1x1 shapes: forward / grad-input / grad-weight time,
efficiency against the HBM / MFMA roofline, and max error against an fp32
torch reference.

Usage (GPU): python bench/gemm1x1.py [--batch 512] [--json-out FILE] [--cfg N]
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

# (Cin, H, Cout, count) of the stride-1 1x1 convolutions of ResNet-50
SHAPES = [(64, 56, 64, 1), (64, 56, 256, 4), (256, 56, 64, 2), (256, 56, 128, 1), (128, 28, 512, 4),
          (512, 28, 128, 3), (512, 28, 256, 1), (256, 14, 1024, 6), (1024, 14, 256, 5), (1024, 14, 512, 1),
          (512, 7, 2048, 3), (2048, 7, 512, 2)]


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--tn-cfg", type=int, default=0)
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--max-blocks", type=int, default=0)
    args = ap.parse_args()
    from gaussiank_sgd_amd import ops
    assert ops.load(), ops._load_error
    g = torch.ops.gksgd
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rows = []
    tot = {k: [0.0, 0.0, 0.0] for k in ("fwd", "dgrad", "wgrad")}   # ours, miopen, roofline
    for (C, H, K, cnt) in SHAPES:
        N = args.batch
        M = N * H * H
        x = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, 1, 1, device=dev, dtype=torch.bfloat16) / C ** 0.5).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(N, K, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        X = x.permute(0, 2, 3, 1).reshape(M, C)
        Wm = w.reshape(K, C)
        Wt = Wm.t().contiguous()
        DY = dy.permute(0, 2, 3, 1).reshape(M, K)
        Y = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        DX = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        DW = torch.zeros(K, C, device=dev, dtype=torch.float32)
        flops = 2.0 * M * K * C
        nbytes = (M * C + M * K + K * C) * 2
        roof = max(flops / PEAK, nbytes / HBM)
        ours = {
            "fwd": lambda: g.gemm_nt(X, Wm, Y, args.cfg, args.max_blocks),
            "dgrad": lambda: g.gemm_nt(DY, Wt, DX, args.cfg, args.max_blocks),
            "wgrad": lambda: g.gemm_tn_acc(DY, X, DW, args.tn_cfg, args.splits),
        }
        xg = x.detach().requires_grad_(True)
        wg = w.detach().requires_grad_(True)
        yg = F.conv2d(xg, wg)
        theirs = {
            "fwd": lambda: F.conv2d(x, w),
            "dgrad": lambda: torch.autograd.grad(yg, xg, dy, retain_graph=True),
            "wgrad": lambda: torch.autograd.grad(yg, wg, dy, retain_graph=True),
        }
        # numerics vs fp32 on a row subset (full M for the reduction)
        ours["fwd"]()
        ours["dgrad"]()
        DW.zero_()
        ours["wgrad"]()
        torch.cuda.synchronize()
        sub = slice(0, min(M, 65536))
        ref_y = X[sub].float() @ Wm.float().t()
        ref_dx = DY[sub].float() @ Wm.float()
        ref_dw = DY.float().t() @ X.float()
        err = {
            "fwd": float((Y[sub].float() - ref_y).abs().max() / ref_y.abs().max()),
            "dgrad": float((DX[sub].float() - ref_dx).abs().max() / ref_dx.abs().max()),
            "wgrad": float((DW - ref_dw).abs().max() / ref_dw.abs().max()),
        }
        del ref_y, ref_dx, ref_dw
        for name in ("fwd", "dgrad", "wgrad"):
            t_o = timeit(ours[name])
            t_m = timeit(theirs[name])
            tot[name][0] += t_o * cnt
            tot[name][1] += t_m * cnt
            tot[name][2] += roof * cnt
            r = dict(op=name, M=M, Cin=C, Cout=K, H=H, count=cnt, ours_us=round(t_o * 1e6, 1),
                     miopen_us=round(t_m * 1e6, 1), roofline_us=round(roof * 1e6, 1), eff=round(roof / t_o, 3),
                     speedup=round(t_m / t_o, 2), rel_err=err[name])
            rows.append(r)
            print(json.dumps(r), flush=True)
        del x, w, dy, X, Wm, Wt, DY, Y, DX, DW, xg, wg, yg
    for name, (a, b, c) in tot.items():
        print("TOTAL %-5s ours %.2f ms  miopen %.2f ms  roofline %.2f ms  (ours %.0f%% of roofline, %.2fx)" % (
            name, a * 1e3, b * 1e3, c * 1e3, 100 * c / a, b / a))
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump({"rows": rows, "totals_ms": {k: [v[0] * 1e3, v[1] * 1e3, v[2] * 1e3] for k, v in tot.items()}},
                      f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
