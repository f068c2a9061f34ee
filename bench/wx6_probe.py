#!/usr/bin/env python3
"""bf16x6 Winograd (wino_x6.hip) vs the fp32-MFMA Winograd (winograd.hip) on
the ResNet-50 3x3 stride-1 shapes at one batch: forward with the BN-statistics
epilogue, grad-input (flipped filter) with the BN-backward epilogue; ms per
call (median of 20 after warm-up) and the speedup.  Prints one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

CL = torch.channels_last


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--mb", type=int, default=0)
    a = ap.parse_args()
    from gaussiank_sgd_amd import ops
    assert ops.load(), ops._load_error
    g = torch.ops.gksgd
    out = {}
    for (H, C) in ((56, 64), (28, 128), (14, 256), (7, 512)):
        N, K = a.batch, C
        x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=CL)
        w = (torch.randn(K, C, 3, 3, device="cuda") * (9 * C) ** -0.5).contiguous(memory_format=CL)
        y = torch.empty(N, K, H, H, device="cuda").contiguous(memory_format=CL)
        st = torch.empty(2, 1280, K, device="cuda")
        u = torch.empty(16 * K * C, device="cuda")
        u3 = torch.empty(48 * K * C, device="cuda", dtype=torch.bfloat16)
        g.wino_weights(w, u, False)
        g.wino_x6_weights(w, u3, False)
        t32 = timeit(lambda: g.wino_conv(x, u, y, a.mb, st))
        t6 = timeit(lambda: g.wino_x6_conv(x, u3, y, a.mb, st))
        h = torch.randn_like(x)
        mask = torch.randint(0, 16, (N * H * H * C // 4,), device="cuda", dtype=torch.uint8)
        dz = torch.empty_like(x)
        g.wino_weights(w, u, True)
        g.wino_x6_weights(w, u3, True)
        b32 = timeit(lambda: g.wino_conv(y, u, dz, a.mb, st, h, None, mask))
        b6 = timeit(lambda: g.wino_x6_conv(y, u3, dz, a.mb, st, h, None, mask))
        tag = "%dx%dx%d" % (H, H, C)
        out[tag] = {"fwd_f32_ms": round(t32, 4), "fwd_x6_ms": round(t6, 4), "fwd_speedup": round(t32 / t6, 3),
                    "dgrad_bn_f32_ms": round(b32, 4), "dgrad_bn_x6_ms": round(b6, 4),
                    "dgrad_speedup": round(b32 / b6, 3)}
        print(tag, out[tag], flush=True)
    print(json.dumps({"batch": a.batch, "shapes": out}))


if __name__ == "__main__":
    main()
