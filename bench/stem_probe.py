#!/usr/bin/env python3
"""ResNet stem (7x7/s2, 3 -> 64) kernels (csrc/kernels/stem.hip) vs MIOpen at
the bench batch: forward (+ BN statistics epilogue) and grad-weight, with the
achieved HBM bandwidth of the compulsory traffic.

Usage (GPU): python bench/stem_probe.py [--batch 512] [--json-out FILE]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


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
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    from gaussiank_sgd_amd import ops
    assert ops.load()
    g = torch.ops.gksgd
    N, H = args.batch, 224
    x = torch.randn(N, 3, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    xb = x.to(torch.bfloat16)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    wb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wp = torch.empty(64, 224, dtype=torch.bfloat16, device="cuda")
    g.stem_pack(w, wp)
    y = torch.empty(N, 64, 112, 112, dtype=torch.bfloat16, device="cuda").contiguous(memory_format=torch.channels_last)
    st = torch.empty(2, 256, 64, device="cuda")
    dy = torch.randn_like(y)
    out = torch.zeros(64, 3, 7, 7, device="cuda").contiguous(memory_format=torch.channels_last)
    part = torch.empty(int(g.stem_wgrad_ws(N, H, H)), device="cuda")
    rows = []
    xbytes, ybytes = x.numel() * 4, y.numel() * 2
    cases = [
        ("fwd hip (fp32 x, stats)", lambda: g.stem_fwd(x, wp, y, st), xbytes + ybytes),
        ("fwd hip (bf16 x, stats)", lambda: g.stem_fwd(xb, wp, y, st), xbytes // 2 + ybytes),
        ("fwd miopen (bf16 x)", lambda: F.conv2d(xb, wb, stride=2, padding=3), xbytes // 2 + ybytes),
        ("wgrad hip (fp32 x)", lambda: g.stem_wgrad(x, dy, out, part), xbytes + ybytes),
        ("wgrad hip (bf16 x)", lambda: g.stem_wgrad(xb, dy, out, part), xbytes // 2 + ybytes),
        ("wgrad miopen (bf16 x)", lambda: torch.ops.aten.convolution_backward(
            dy, xb, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]), xbytes // 2 + ybytes),
    ]
    for name, fn, nbytes in cases:
        t = timeit(fn)
        r = {"case": name, "us": round(t * 1e6, 1), "GB/s": round(nbytes / t / 1e9, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
