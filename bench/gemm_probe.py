#!/usr/bin/env python3
"""Run ONE gemm.hip kernel configuration repeatedly (for rocprofv3 counter
passes): python bench/gemm_probe.py --op conv|gemm|gemm_bnb|wgrad3|lwgrad|cwgrad --cfg N [--iters 20]
[--dtype bf16|f32] [--k 3] [--stride 1]

``--sweep 1,2,3``: time every listed cfg with HIP events instead and print
one JSON line per cfg (us per call, TFLOP/s, % of the dtype's dense MFMA
peak: 2.5 PF bf16, 157 TF fp32).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PEAK = {"bf16": 2.5e15, "f32": 157.3e12}


def make(a, cfg):
    g = torch.ops.gksgd
    dt = torch.float32 if a.dtype == "f32" else torch.bfloat16
    cl = torch.channels_last
    K = a.K or a.C
    k, s = a.k, a.stride
    p = k // 2
    if a.op == "lwgrad":   # linear grad-weight (BERT ffn): W[N, K] += G[M, N]^T X[M, K]
        M = a.batch * a.H
        G = torch.randn(M, K, device="cuda", dtype=dt)
        X = torch.randn(M, a.C, device="cuda", dtype=dt)
        out = torch.zeros(K, a.C, device="cuda")
        return (lambda: g.gemm_tn_acc(G, X, out, cfg, a.splits)), 2.0 * M * K * a.C
    x = torch.randn(a.batch, a.C, a.H, a.H, device="cuda", dtype=dt).contiguous(memory_format=cl)
    OH = (a.H + 2 * p - k) // s + 1
    z = torch.zeros(256, device="cuda", dtype=torch.bfloat16)
    if a.op in ("wgrad3", "cwgrad"):
        dy = torch.randn(a.batch, K, OH, OH, device="cuda", dtype=dt).contiguous(memory_format=cl)
        out = torch.zeros(K, a.C, k, k, device="cuda").contiguous(memory_format=cl)
        return (lambda: g.conv_tn_acc(dy, x, out, z, s, p, cfg, a.splits)), 2.0 * a.batch * OH * OH * K * a.C * k * k
    if a.op == "conv":
        w = torch.randn(K, a.C, k, k, device="cuda", dtype=dt).contiguous(memory_format=cl)
        y = torch.empty(a.batch, K, OH, OH, device="cuda", dtype=dt).contiguous(memory_format=cl)
        return (lambda: g.conv_nt(x, w, y, z, s, p, cfg, a.mb)), 2.0 * a.batch * OH * OH * K * a.C * k * k
    X = x.permute(0, 2, 3, 1).reshape(-1, a.C)
    W = torch.randn(K, a.C, device="cuda", dtype=dt)
    Y = torch.empty(X.shape[0], K, device="cuda", dtype=dt)
    if a.op == "gemm_bnb":   # grad-input GEMM with the BN-backward epilogue (dz = mask ? acc + dy2 : 0, stats)
        M = X.shape[0]
        h = torch.randn(M, K, device="cuda", dtype=dt)
        d2 = torch.randn(M, K, device="cuda", dtype=dt)
        mask = torch.randint(0, 16, (M, K // 4), device="cuda", dtype=torch.uint8)
        st = torch.empty(2, 1280, K, device="cuda")
        return (lambda: g.gemm_nt(X, W, Y, cfg, a.mb, st, None, h, d2, mask)), 2.0 * M * K * a.C
    return (lambda: g.gemm_nt(X, W, Y, cfg, a.mb)), 2.0 * X.shape[0] * K * a.C


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="conv")
    ap.add_argument("--cfg", type=int, default=124)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--H", type=int, default=14)
    ap.add_argument("--K", type=int, default=0)
    ap.add_argument("--k", type=int, default=3, help="conv kernel size (conv / cwgrad)")
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--mb", type=int, default=0, help="NT max blocks (0: persistent default)")
    ap.add_argument("--splits", type=int, default=0, help="TN splits (0: default)")
    ap.add_argument("--sweep", default="", help="comma-separated cfgs to time with events")
    a = ap.parse_args()
    from gaussiank_sgd_amd import ops
    assert ops.load()
    if a.sweep:
        for cfg in [int(c) for c in a.sweep.split(",") if c]:
            fn, flop = make(a, cfg)
            try:
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                print(json.dumps({"op": a.op, "dtype": a.dtype, "C": a.C, "K": a.K or a.C, "H": a.H, "k": a.k,
                                  "stride": a.stride, "cfg": cfg, "mb": a.mb, "splits": a.splits,
                                  "us": round(us, 1), "tflops": round(flop / us * 1e-6, 1),
                                  "pct_peak": round(100 * flop / (us * 1e-6) / PEAK[a.dtype], 1)}), flush=True)
            except RuntimeError as e:
                print(json.dumps({"cfg": cfg, "error": str(e)[:200]}), flush=True)
        return
    fn, _ = make(a, a.cfg)
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
