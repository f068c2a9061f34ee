#!/usr/bin/env python3
"""Tap-parallel 3x3 grad-weight (csrc/kernels/wgrad3.hip) on the ResNet-50
bs512 stride-1 3x3 shapes: time per call and % of the 2.5 PF bf16 peak.

Usage (GPU): python bench/w3_probe.py [--shapes 0,1,2,3] [--json-out FILE]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [(512, 64, 56, 64), (512, 128, 28, 128), (512, 256, 14, 256), (512, 512, 7, 512)]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="0,1,2,3")
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    from gaussiank_sgd_amd import ops
    assert ops.load()
    g = torch.ops.gksgd
    rows = []
    for i in [int(v) for v in args.shapes.split(",")]:
        N, C, H, K = SHAPES[i]
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, K, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        out = torch.zeros(K, C, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
        part = torch.empty(int(g.wgrad3_ws(N, H, H, C, K)), device="cuda")
        t = timeit(lambda: g.conv3_wgrad(dy, x, out, part, torch.zeros(256, dtype=torch.bfloat16, device=x.device)))
        flops = 2.0 * N * H * H * C * K * 9
        r = {"shape": "N=%d C=%d H=%d K=%d" % (N, C, H, K), "us": round(t * 1e6, 1),
             "pct_peak": round(100 * flops / t / 2.5e15, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
