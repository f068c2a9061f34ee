"""Implicit-GEMM 3x3 forward (gemm.hip conv_nt) at ResNet-50 bs512 shapes:
microseconds and TFLOP/s per kernel configuration, to A/B two builds of the
extension (GKSGD_EXT=variants/<name>/_C.so loads another build).

    python bench/nt_probe.py [--cfgs 124,125,126,24] [--json-out FILE]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussiank_sgd_amd import ops  # noqa: E402

# (Cin, Cout, H_in, stride)
SHAPES = [(64, 64, 56, 1), (128, 128, 28, 1), (256, 256, 14, 1), (512, 512, 7, 1), (128, 128, 56, 2)]


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--cfgs", default="124,125,126,24,4,121")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    assert ops.load(), ops._load_error
    g = torch.ops.gksgd
    dev = torch.device("cuda", 0)
    z = torch.zeros(256, device=dev, dtype=torch.bfloat16)
    out = []
    for C, K, H, s in SHAPES:
        x = torch.randn(a.batch, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (0.05 * torch.randn(K, C, 3, 3, device=dev)).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        OH = (H + 2 - 3) // s + 1
        y = torch.empty(a.batch, K, OH, OH, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        flop = 2.0 * a.batch * OH * OH * K * C * 9
        ref = torch.nn.functional.conv2d(x.float(), w.float(), stride=s, padding=1)
        row = {"C": C, "K": K, "H": H, "s": s}
        for cfg in [int(c) for c in a.cfgs.split(",")]:
            try:
                fn = lambda: g.conv_nt(x, w, y, z, s, 1, cfg, 0)  # noqa: E731
                us = timeit(fn)
                err = float((y.float() - ref).abs().max() / ref.abs().max())
                row[str(cfg)] = [round(us, 1), round(flop / us / 1e6, 1), round(err, 4)]
            except RuntimeError as e:
                row[str(cfg)] = str(e).splitlines()[0][:80]
        out.append(row)
        print(json.dumps(row), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
