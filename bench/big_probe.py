#!/usr/bin/env python3
"""BERT-base linear shapes (M = 32 x 512 rows): the large-tile bf16 GEMM
(csrc/kernels/gemm_big.hip, cfg 0-2) vs hipBLASLt (torch.mm / addmm) vs
gemm.hip's gemm_nt (best of a few configurations).  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussiank_sgd_amd import ops  # noqa: E402


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
    return a.elapsed_time(b) / iters * 1e3


def main():
    assert ops.load()
    g = torch.ops.gksgd
    M = 16384
    for K, N in ((768, 2304), (768, 768), (768, 3072), (3072, 768), (2304, 768)):
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        b16 = bias.to(torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        row = {"M": M, "K": K, "N": N}
        row["blas_us"] = round(timeit(lambda: torch.addmm(b16, A, B.t())), 1)
        for c in (0, 1, 2):
            if g.gemm_big_supported(M, N, K, c):
                row["big%d_us" % c] = round(timeit(lambda c=c: g.gemm_big(A, B, C, c, bias)), 1)
        best = None
        for c in (124, 125, 25, 5):
            try:
                t = timeit(lambda c=c: g.gemm_nt(A, B, C, c, 0, None, bias))
            except RuntimeError:
                continue
            best = t if best is None or t < best else best
        row["gemm_nt_us"] = round(best, 1) if best else None
        row["tflops_big_best"] = round(2.0 * M * N * K / min(v for k, v in row.items() if k.startswith("big")) * 1e-6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
