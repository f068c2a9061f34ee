#!/usr/bin/env python3
"""Per-convolution roofline report for ResNet-50 at the bench batch size.

For every distinct convolution of ResNet-50 (bf16, channels-last, MIOpen via
torch) this times forward, backward-data and backward-weight and compares
each against its roofline: max(FLOPs / 2.5 PFLOP/s dense bf16,
compulsory bytes / 6.3 TB/s achievable HBM).  Shows where the vendor
convolutions leave time on the table (the input to custom-kernel work).

Usage (GPU): python bench/convs.py [--batch 512] [--json-out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_HERE, "tuning", "miopen"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

PEAK = 2.5e15
HBM = 6.3e12


def resnet50_convs(batch: int):
    """(N, Cin, H, W, Cout, k, stride, pad) with multiplicity -- ResNet-50 v1.5
    (stride on the 3x3; models/resnet_imagenet.py), enumerated from the
    architecture (the fused blocks call their convolutions through
    forward_stats, which bypasses module forward hooks)."""
    shapes = Counter()
    shapes[(batch, 3, 224, 224, 64, 7, 2, 3)] += 1
    cin, H = 64, 56
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        out = planes * 4
        for b in range(blocks):
            s = stride if b == 0 else 1
            shapes[(batch, cin, H, H, planes, 1, 1, 0)] += 1
            shapes[(batch, planes, H, H, planes, 3, s, 1)] += 1
            Ho = H // s
            shapes[(batch, planes, Ho, Ho, out, 1, 1, 0)] += 1
            if b == 0:
                shapes[(batch, cin, H, H, out, 1, s, 0)] += 1
            cin, H = out, Ho
    return shapes


def timeit(fn, iters=10):
    for _ in range(2):
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
    ap.add_argument("--gemm", action="store_true",
                    help="also time the stride-1 1x1 convs as plain torch.mm (hipBLASLt) GEMMs")
    ap.add_argument("--ours", action="store_true",
                    help="time the production path (ops/conv1x1.py: autotuned MFMA kernels vs MIOpen, "
                         "tuning/gemm_choices.json) and report which implementation each direction uses")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.ours:
        from gaussiank_sgd_amd import ops
        assert ops.load(), "native extension not built"
    rows = []
    tot = {"fwd": [0.0, 0.0], "dgrad": [0.0, 0.0], "wgrad": [0.0, 0.0]}
    for (N, C, H, W, K, k, s, p), mult in sorted(resnet50_convs(args.batch).items()):
        x = torch.randn(N, C, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(K, C, k, k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=s, padding=p)
        OH, OW = y.shape[2], y.shape[3]
        dy = torch.randn_like(y)
        flops = 2.0 * N * OH * OW * K * C * k * k
        bx, bw, by = x.numel() * 2, w.numel() * 2, y.numel() * 2
        xg = x.detach().requires_grad_(True)
        wg = w.detach().requires_grad_(True)
        yg = F.conv2d(xg, wg, stride=s, padding=p)
        cases = {
            "fwd": (lambda: F.conv2d(x, w, stride=s, padding=p), bx + bw + by),
            "dgrad": (lambda: torch.autograd.grad(yg, xg, dy, retain_graph=True), by + bw + bx),
            "wgrad": (lambda: torch.autograd.grad(yg, wg, dy, retain_graph=True), by + bx + bw),
        }
        impl = {}
        if args.ours and C % 64 == 0 and K % 64 == 0:
            from gaussiank_sgd_amd.ops import conv1x1 as cv
            wo = torch.zeros(K, C, k, k, device=dev, dtype=torch.float32).contiguous(memory_format=torch.channels_last)
            cases = {
                "fwd": (lambda: cv._fwd(x, w, s, []), bx + bw + by),   # production: BN stats epilogue
                "dgrad": (lambda: cv._dgrad(dy, w, x.shape, s), by + bw + bx),
                "wgrad": (lambda: cv._wgrad_into(dy, x, w, s, wo), by + bx + bw),
            }
            for name, (fn, _) in cases.items():
                fn()
            geo = (N, C, H, W, K, k, s)
            impl = {"fwd": cv._choices.get(("fwd",) + geo + (True,)), "dgrad": cv._choices.get(("dgrad",) + geo),
                    "wgrad": cv._choices.get(("wgrad",) + geo)}
        if C == 3:
            del cases["dgrad"]   # the stem's input (the image batch) needs no gradient in training
        for name, (fn, nbytes) in cases.items():
            t = timeit(fn)
            roof = max(flops / PEAK, nbytes / HBM)
            tot[name][0] += t * mult
            tot[name][1] += roof * mult
            r = dict(op=name, N=N, Cin=C, H=H, W=W, Cout=K, k=k, stride=s, count=mult, us=round(t * 1e6, 1),
                     roofline_us=round(roof * 1e6, 1), eff=round(roof / t, 3),
                     tflops=round(flops / t / 1e12, 1), bound="compute" if flops / PEAK > nbytes / HBM else "memory")
            if impl.get(name) is not None:
                r["impl"] = list(impl[name])
            rows.append(r)
            print(json.dumps(r), flush=True)
        if args.gemm and k == 1 and s == 1:
            M = N * H * W
            X = x.permute(0, 2, 3, 1).reshape(M, C)
            Wm = w.reshape(K, C)
            DY = dy.permute(0, 2, 3, 1).reshape(M, K)
            for name, fn, nbytes in (("mm_fwd", lambda: X @ Wm.t(), bx + bw + by),
                                     ("mm_dgrad", lambda: DY @ Wm, bx + bw + by),
                                     ("mm_wgrad", lambda: DY.t() @ X, bx + bw + by)):
                t = timeit(fn)
                roof = max(flops / PEAK, nbytes / HBM)
                r = dict(op=name, N=N, Cin=C, H=H, W=W, Cout=K, k=k, stride=s, count=mult, us=round(t * 1e6, 1),
                         roofline_us=round(roof * 1e6, 1), eff=round(roof / t, 3))
                rows.append(r)
                print(json.dumps(r), flush=True)
        del x, w, y, dy, xg, wg, yg
    for name, (t, roof) in tot.items():
        print("TOTAL %-5s %.2f ms per step (roofline %.2f ms, efficiency %.0f%%)" % (name, t * 1e3, roof * 1e3,
                                                                                   100 * roof / max(t, 1e-12)))
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump({"rows": rows, "totals_ms": {k: [v[0] * 1e3, v[1] * 1e3] for k, v in tot.items()}}, f,
                      indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
