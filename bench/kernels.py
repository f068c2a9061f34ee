#!/usr/bin/env python3
"""Kernel micro-benchmarks: achieved HBM bandwidth of every hot HIP kernel.

Each line reports time per call and the effective bandwidth of the bytes the
kernel MUST move (compulsory traffic), against MI355X's ~6.3 TB/s achievable
(8 TB/s spec) HBM3E bandwidth.  Shapes are the ResNet-50 / bs512 training
step's: 25.56 M gradients (one bucket), k = 0.1 %, BN layer1 [512*56*56, 256].

Usage (GPU): python bench/kernels.py [--json-out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gaussiank_sgd_amd import ops  # noqa: E402
from gaussiank_sgd_amd.utils.stats import gaussian_z  # noqa: E402

HBM_ACHIEVABLE = 6.3e12


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=25_557_032)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    if not torch.cuda.is_available() or not ops.load():
        print("needs a GPU and the native extension", file=sys.stderr)
        return 2
    dev = torch.device("cuda", 0)
    n = (args.n + 63) // 64 * 64
    rows = []

    def report(name, sec, nbytes, extra=""):
        bw = nbytes / sec
        rows.append({"kernel": name, "us": round(sec * 1e6, 1), "GB": round(nbytes / 1e9, 3),
                     "TB_s": round(bw / 1e12, 2), "pct_achievable": round(100 * bw / HBM_ACHIEVABLE, 1),
                     "note": extra})
        print("%-34s %9.1f us  %7.3f GB  %5.2f TB/s  %5.1f%%  %s" % (name, sec * 1e6, nbytes / 1e9, bw / 1e12,
                                                                   100 * bw / HBM_ACHIEVABLE, extra), flush=True)

    # ---------------- compression pipeline ----------------
    g0 = torch.randn(n, device=dev) * 1e-3
    r = torch.zeros(n, device=dev)
    density = 0.001
    k = max(int(args.n * density), 1)
    for name, mode, kcap in (("compress gaussian (EC)", ops.MODE_GAUSSIAN, 2 * k),
                             ("compress topk exact (EC)", ops.MODE_TOPK, k),
                             ("compress randomk (EC)", ops.MODE_RANDOMK, k),
                             ("compress dgcsampling (EC)", ops.MODE_DGC, 2 * k)):
        bufs = ops.CompressBuffers(kcap, dev)
        g = g0.clone()

        def run(mode=mode, bufs=bufs, g=g, kcap=kcap):
            g.copy_(g0)  # included below as 2 passes
            ops.compress_(g, r, bufs, mode, ec=True, zero_g=True, loops=3, z=gaussian_z(density), k=k, k_cap=kcap,
                          seed=7, n_stats=args.n)
        t_copy = timeit(lambda g=g: g.copy_(g0))
        t = timeit(run) - t_copy
        # compulsory: read g, r; write r (new residual), zero g  -> 4 passes of fp32
        report(name, t, 4 * 4 * n, "k=%d, pipeline incl. stats/count/select" % k)

    # ---------------- decompress ----------------
    for P in (1, 8):
        bufs = ops.CompressBuffers(2 * k, dev)
        g = g0.clone()
        ops.compress_(g, r, bufs, ops.MODE_TOPK, ec=False, zero_g=False, k=k, k_cap=2 * k, n_stats=args.n)
        recs = bufs.record.repeat(P)
        dst = torch.zeros(n, device=dev)
        t = timeit(lambda: ops.scatter_add_records_(dst, recs, P, 2 * k, 1.0 / P))
        report("scatter_add_records P=%d" % P, t, P * k * 8 * 2, "atomic fp32, %d pairs" % (P * k))

    # ---------------- fused optimizer ----------------
    w = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    gr = torch.randn(n, device=dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    chunks = ops.make_chunk_table([(0, n, 0, 0)], dev)
    hp = [dict(lr=0.1, momentum=0.9, weight_decay=5e-5, dampening=0.0, nesterov=False, first_step=False)]
    t = timeit(lambda: ops.fused_sgd_(w, m, gr, chunks, hp, zero_grad=False))
    report("fused_sgd (w,m,g)", t, 5 * 4 * n)
    t = timeit(lambda: ops.fused_sgd_(w, m, gr, chunks, hp, zero_grad=True, w_bf16=sh))
    report("fused_sgd + zero g + bf16 shadow", t, 6 * 4 * n + 2 * n)
    u = torch.zeros(n, device=dev)
    t = timeit(lambda: ops.momentum_correct_(u, gr, w, chunks, 0, chunks.numel() // 2, hp))
    report("momentum_correct (u,g,w)", t, 5 * 4 * n)
    gb = torch.randn(n, device=dev).to(torch.bfloat16)
    t = timeit(lambda: ops.accum_grad_(gr, gb))
    report("accum_grad bf16->fp32", t, 4 * n * 2 + 2 * n)

    # ---------------- fused BN (layer1 shape, bs512) ----------------
    from gaussiank_sgd_amd.ops.bn import BNAct
    N, C, H, W = 512, 256, 56, 56
    x = torch.randn(N, C, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x)
    bn = BNAct(C, act="relu").to(dev)
    xe = x.numel() * 2
    t = timeit(lambda: bn(x, res), iters=10)
    report("BN+add+ReLU fwd [%dx%d]" % (N * H * W, C), t, xe * 4 + xe / 16, "stats + apply (x twice, res, y)")
    xg = x.clone().requires_grad_(True)
    rg = res.clone().requires_grad_(True)
    y = bn(xg, rg)
    dy = torch.randn_like(y)
    t = timeit(lambda: torch.autograd.grad(y, (xg, rg), dy, retain_graph=True), iters=10)
    report("BN+add+ReLU bwd", t, xe * 6 + xe / 8, "reduce + apply (dy,x twice; dx,dres)")
    # stem BN + ReLU + maxpool
    xs = torch.randn(N, 64, 112, 112, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bns = BNAct(64, act="relu", pool=(3, 2, 1)).to(dev)
    xse = xs.numel() * 2
    t = timeit(lambda: bns(xs), iters=10)
    report("stem BN+ReLU+maxpool fwd", t, xse * 2 + xse / 4 + xse / 8, "stats + pooled apply")
    xsg = xs.clone().requires_grad_(True)
    ys = bns(xsg)
    dys = torch.randn_like(ys)
    t = timeit(lambda: torch.autograd.grad(ys, xsg, dys, retain_graph=True), iters=10)
    report("stem BN+ReLU+maxpool bwd", t, xse * 3 + xse / 4, "gathered pool grad in reduce + apply")

    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
