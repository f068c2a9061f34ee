#!/usr/bin/env python3
"""Grad-weight (TN) GEMM configurations vs hipBLASLt / MIOpen on the shapes
that dominate BERT-base (M = 32 x 512 tokens) and ResNet-50 bs512.

For each shape: every gemm_tn / conv_tn config of ops/conv1x1._TN_CFGS,
hipBLASLt bf16 -> fp32 with beta = 1 (``torch.addmm(out_dtype=float32)``)
for the linears, MIOpen for the convolutions; achieved TFLOP/s and % of the
2.5 PFLOP/s dense bf16 peak.

Usage (GPU): python bench/tn_probe.py [--json-out FILE]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PEAK = 2.5e15


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
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.ops import conv1x1 as cv
    assert ops.load()
    g = torch.ops.gksgd
    dev = torch.device("cuda", 0)
    rows = []
    lin = [(16384, 768, 768), (16384, 2304, 768), (16384, 3072, 768), (16384, 768, 3072)]
    for M, N, K in lin:
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        out = torch.zeros(N, K, device=dev)
        flops = 2.0 * M * N * K
        res = {}
        for c, sp in cv._TN_CFGS:
            try:
                res["hip %d/%d" % (c, sp)] = timeit(lambda c=c, sp=sp: g.gemm_tn_acc(dy, x, out, c, sp))
            except RuntimeError as e:
                res["hip %d/%d" % (c, sp)] = None
        res["hipblaslt fp32-out"] = timeit(lambda: torch.addmm(out, dy.t(), x, out_dtype=torch.float32, out=out))
        best = min((t, k) for k, t in res.items() if t)
        r = {"shape": "linear wgrad M=%d N=%d K=%d" % (M, N, K), "best": best[1], "best_us": round(best[0] * 1e6, 1),
             "best_pct_peak": round(100 * flops / best[0] / PEAK, 1),
             "hipblaslt_us": round(res["hipblaslt fp32-out"] * 1e6, 1),
             "all_us": {k: (round(t * 1e6, 1) if t else None) for k, t in res.items()}}
        rows.append(r)
        print(json.dumps({k: v for k, v in r.items() if k != "all_us"}), flush=True)
    convs = [(512, 64, 56, 64, 3, 1), (512, 128, 28, 128, 3, 1), (512, 256, 14, 256, 3, 1), (512, 512, 7, 512, 3, 1),
             (512, 256, 56, 64, 1, 1), (512, 1024, 14, 256, 1, 1)]
    for N, C, H, K, k, s in convs:
        x = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(K, C, k, k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        OH = (H + 2 * (k // 2) - k) // s + 1
        dy = torch.randn(N, K, OH, OH, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        out = torch.zeros(K, C, k, k, device=dev).contiguous(memory_format=torch.channels_last)
        z = torch.zeros(256, dtype=torch.bfloat16, device=dev)
        flops = 2.0 * N * OH * OH * K * C * k * k
        res = {}
        for c, sp in cv._TN_CFGS:
            try:
                if k == 1 and s == 1:
                    DY, X = cv._rows(dy), cv._rows(x)
                    fn = lambda c=c, sp=sp: g.gemm_tn_acc(DY, X, out.view(K, C), c, sp)  # noqa: E731
                else:
                    fn = lambda c=c, sp=sp: g.conv_tn_acc(dy, x, out, z, s, k // 2, c, sp)  # noqa: E731
                res["hip %d/%d" % (c, sp)] = timeit(fn)
            except RuntimeError:
                res["hip %d/%d" % (c, sp)] = None
        if k == 3 and s == 1 and g.wgrad3_supported(H, H, C, K):
            part = torch.empty(int(g.wgrad3_ws(N, H, H, C, K)), device=dev)
            res["w3 tap-parallel"] = timeit(lambda: g.conv3_wgrad(dy, x, out, part, torch.zeros(256, dtype=torch.bfloat16, device=x.device)))
        res["miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [k // 2, k // 2], [1, 1], False, [0, 0], 1, [False, True, False]))
        best = min((t, kk) for kk, t in res.items() if t)
        r = {"shape": "conv wgrad N=%d C=%d H=%d K=%d k=%d s=%d" % (N, C, H, K, k, s), "best": best[1],
             "w3_us": round(res["w3 tap-parallel"] * 1e6, 1) if "w3 tap-parallel" in res else None,
             "best_us": round(best[0] * 1e6, 1), "best_pct_peak": round(100 * flops / best[0] / PEAK, 1),
             "miopen_us": round(res["miopen"] * 1e6, 1),
             "all_us": {kk: (round(t * 1e6, 1) if t else None) for kk, t in res.items()}}
        rows.append(r)
        print(json.dumps({kk: v for kk, v in r.items() if kk != "all_us"}), flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
