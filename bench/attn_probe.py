"""Fused self-attention (ops/attention.py) vs torch SDPA on BERT-base's shape
(B 32, heads 12, T 512, d 64, dropout 0.1): forward and forward+backward
times per call and the achieved MFMA rate (fwd 4*B*H*T^2*d FLOPs, bwd 2.5x).

    python bench/attn_probe.py [--B 32] [--T 512] [--heads 12] [--p 0.1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussiank_sgd_amd import ops  # noqa: E402
from gaussiank_sgd_amd.ops import attention  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=512)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    assert ops.load(), ops._load_error
    B, T, Hh, p = a.B, a.T, a.heads, a.p
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3 * Hh * 64, device="cuda").to(torch.bfloat16).requires_grad_(True)
    dout = torch.randn(B, T, Hh * 64, device="cuda").to(torch.bfloat16)
    flops = 4.0 * B * Hh * T * T * 64
    res = {"shape": [B, Hh, T, 64], "p": p}

    def ours_f():
        with torch.no_grad():
            attention._FlashAttnFn.apply(qkv, Hh, p, 1)

    def ours_fb():
        o = attention._FlashAttnFn.apply(qkv, Hh, p, 1)
        o.backward(dout)

    def sdpa_f():
        with torch.no_grad():
            attention._sdpa(qkv, Hh, p)

    def sdpa_fb():
        o = attention._sdpa(qkv, Hh, p)
        o.backward(dout)

    for name, f, fb in [("ours", ours_f, ours_fb), ("sdpa", sdpa_f, sdpa_fb)]:
        tf = timeit(f)
        tfb = timeit(fb)
        res[name] = {"fwd_us": round(tf, 1), "fwd_bwd_us": round(tfb, 1), "bwd_us": round(tfb - tf, 1),
                     "fwd_tflops": round(flops / tf / 1e6, 1), "bwd_tflops": round(2.5 * flops / max(tfb - tf, 1e-3) / 1e6, 1)}
    print(json.dumps(res))
    if a.json_out:
        with open(a.json_out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
