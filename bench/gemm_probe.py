#!/usr/bin/env python3
"""Run ONE gemm.hip kernel configuration repeatedly (for rocprofv3 counter
passes): python bench/gemm_probe.py --op conv|gemm --cfg N [--iters 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="conv")
    ap.add_argument("--cfg", type=int, default=124)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--H", type=int, default=14)
    ap.add_argument("--K", type=int, default=0)
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    from gaussiank_sgd_amd import ops
    assert ops.load()
    g = torch.ops.gksgd
    K = a.K or a.C
    x = torch.randn(a.batch, a.C, a.H, a.H, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    if a.op == "lwgrad":   # linear grad-weight (BERT ffn): W[N, K] += G[M, N]^T X[M, K]
        M = a.batch * a.H
        G = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        X = torch.randn(M, a.C, device="cuda", dtype=torch.bfloat16)
        out = torch.zeros(K, a.C, device="cuda")
        fn = lambda: g.gemm_tn_acc(G, X, out, a.cfg, 0)  # noqa: E731
    elif a.op == "wgrad3":
        dy = torch.randn(a.batch, K, a.H, a.H, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        out = torch.zeros(K, a.C, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
        z = torch.zeros(256, device="cuda", dtype=torch.bfloat16)
        fn = lambda: g.conv_tn_acc(dy, x, out, z, 1, 1, a.cfg, 0)  # noqa: E731
    elif a.op == "conv":
        w = torch.randn(K, a.C, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.empty(a.batch, K, a.H, a.H, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        z = torch.zeros(256, device="cuda", dtype=torch.bfloat16)
        fn = lambda: g.conv_nt(x, w, y, z, 1, 1, a.cfg, 0)  # noqa: E731
    else:
        X = x.permute(0, 2, 3, 1).reshape(-1, a.C)
        W = torch.randn(K, a.C, device="cuda", dtype=torch.bfloat16)
        Y = torch.empty(X.shape[0], K, device="cuda", dtype=torch.bfloat16)
        fn = lambda: g.gemm_nt(X, W, Y, a.cfg, 0)  # noqa: E731
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
