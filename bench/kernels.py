#!/usr/bin/env python3
"""Kernel micro-benchmarks: achieved HBM bandwidth of every hot HIP kernel.

Each line reports time per call and the effective bandwidth of the bytes the
kernel MUST move (compulsory traffic), against MI355X's ~6.3 TB/s achievable
(8 TB/s spec) HBM3E bandwidth.  Shapes are the ResNet-50 / bs512 training
step's: 25.56 M gradients (one bucket), k = 0.1 %, BN layer1 [512*56*56, 256].

Usage (GPU): python bench/kernels.py [--json-out FILE] [--fit-out tuning/perf_model_mi355x.json]

--fit-out: times the production compression pipeline (Gaussian-k with DGC
momentum correction fused into its statistics pass, as DistributedOptimizer
runs it) at several bucket sizes, fits t = c0 + c1 * n and writes the
``compress`` entry of the planners' perf-model JSON with its provenance
(utils/perf_model.py).
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
    ap.add_argument("--fit-out", default=None)
    ap.add_argument("--only", default=None, help="comma list of sections: compress,round2,decompress,optim,bn,fit")
    args = ap.parse_args()
    only = set(args.only.split(",")) if args.only else None

    def want(sec):
        return only is None or sec in only
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
    for name, mode, kcap in () if not want("compress") else (("compress gaussian (EC)", ops.MODE_GAUSSIAN, 2 * k),
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

    # ---------------- round 2: calibrated Gaussian-k, fused MC, rank-ordered reduce ----------------
    chunks_all = ops.make_chunk_table([(0, n, 0, 0)], dev)
    hp1 = [dict(lr=0.1, momentum=0.875, weight_decay=6.1e-5, dampening=0.0, nesterov=False, first_step=False)]
    if want("round2"):
        kc = (4 * k + 2) // 3
        pipe = {}
        # training-like input: a fresh gradient every call (pool of 4), residual
        # carried over (EC), so the residual distribution is stationary
        pool = [torch.randn(n, device=dev) * 1e-3 * (1 + 0.1 * i) for i in range(4)]
        for name, mode in (("gaussian", ops.MODE_GAUSSIAN), ("gaussian_cal", ops.MODE_GAUSSIAN_CAL)):
            bufs = ops.CompressBuffers(kc, dev)
            g = g0.clone()
            rr = torch.zeros(n, device=dev)
            it = [0]

            def run(mode=mode, bufs=bufs, g=g, rr=rr, it=it):
                g.copy_(pool[it[0] % 4])
                it[0] += 1
                ops.compress_(g, rr, bufs, mode, ec=True, zero_g=True, loops=3, z=gaussian_z(density), k=k, k_cap=kc,
                              seed=7, n_stats=args.n)
            for _ in range(30):          # let the residual (and the calibrated ladder) settle
                run()
            t = timeit(run) - timeit(lambda g=g: g.copy_(pool[0]))
            pipe[name] = t
            fb, sel = 0, []
            for _ in range(40):
                run()
                hdr = bufs.record[:4].cpu()
                fb += int(hdr[2]) == ops.CAL_FALLBACK
                sel.append(int(hdr[1]) / k)
            report("compress %s k_cap=4k/3" % name, t, 4 * 4 * n,
                   "sel/k %.2f..%.2f, exact fallbacks %d/40" % (min(sel), max(sel), fb))
        rows.append({"kernel": "gaussian_cal overhead vs gaussian", "pct": round(100 * (pipe["gaussian_cal"] /
                                                                                       pipe["gaussian"] - 1), 1)})
        print("gaussian_cal overhead vs gaussian: %+.1f%%" % (100 * (pipe["gaussian_cal"] / pipe["gaussian"] - 1)))
        # DGC momentum correction: separate passes vs fused into the statistics pass
        u = torch.zeros(n, device=dev)
        wv = torch.randn(n, device=dev)
        g = g0.clone()
        bufs = ops.CompressBuffers(kc, dev)
        nch = chunks_all.numel() // 2

        def sep():
            g.copy_(g0)
            ops.momentum_correct_(u, g, wv, chunks_all, 0, nch, hp1)
            ops.compress_(g, r, bufs, ops.MODE_GAUSSIAN, ec=True, zero_g=True, z=gaussian_z(density), k=k, k_cap=kc,
                          n_stats=args.n)
            ops.mask_records_(u, bufs.record, kc)

        mc = {"u": u, "w": wv, "chunks": chunks_all, "begin": 0, "count": nch, "base": 0, "groups": hp1}

        def fused():
            g.copy_(g0)
            ops.compress_(g, r, bufs, ops.MODE_GAUSSIAN, ec=True, zero_g=True, z=gaussian_z(density), k=k, k_cap=kc,
                          n_stats=args.n, mc=mc)
        tc = timeit(lambda: g.copy_(g0))
        report("MC + compress, separate passes", timeit(sep) - tc, 9 * 4 * n, "momentum_correct + stats + mask")
        report("MC fused into compress stats", timeit(fused) - tc, 7 * 4 * n, "u,g,w,r -> u,r,g")
        # sparse aggregation / apply (P records of k_cap entries)
        for P in (1, 8):
            recs = bufs.record.repeat(P)
            dst = torch.zeros(n, device=dev)
            t = timeit(lambda: ops.scatter_add_records_(dst, recs, P, kc, 1.0 / P, True))
            report("reduce_records P=%d (rank order)" % P, t, P * kc * 8 + kc * 8, "deterministic, no atomics")
            sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
            t = timeit(lambda: ops.apply_records_sgd_(wv, sh, recs, P, kc, 1.0 / P, 0.1))
            report("apply_records_sgd P=%d" % P, t, P * kc * 8 + kc * 10, "sparse SGD + bf16 shadow")

    if args.fit_out or want("fit") and only is not None:
        from gaussiank_sgd_amd.utils import perf_model
        sizes, times = [], []
        for nn in (1 << 20, 1 << 22, 1 << 24, 25_557_056, 1 << 26):
            gg = torch.randn(nn, device=dev) * 1e-3
            g2, r2 = gg.clone(), torch.zeros(nn, device=dev)
            u2, w2 = torch.zeros(nn, device=dev), torch.randn(nn, device=dev)
            ch = ops.make_chunk_table([(0, nn, 0, 0)], dev)
            kk = max(int(nn * density), 1)
            kc2 = (4 * kk + 2) // 3
            bf = ops.CompressBuffers(kc2, dev)
            mc2 = {"u": u2, "w": w2, "chunks": ch, "begin": 0, "count": ch.numel() // 2, "base": 0, "groups": hp1}

            def run2():
                g2.copy_(gg)
                ops.compress_(g2, r2, bf, ops.MODE_GAUSSIAN, ec=True, zero_g=True, z=gaussian_z(density), k=kk,
                              k_cap=kc2, n_stats=nn, mc=mc2)
            t = timeit(run2) - timeit(lambda: g2.copy_(gg))
            sizes.append(nn)
            times.append(t)
            print("fit compress n=%d: %.1f us" % (nn, t * 1e6), flush=True)
            del gg, g2, r2, u2, w2
        c0, c1 = perf_model.fit_alpha_beta(sizes, times)
        entry = {"c0_s": c0, "c1_s_per_elem": c1, "measured": True,
                 "source": "bench/kernels.py --fit-out on %s: fused MC + Gaussian-k pipeline, density %g, "
                           "n in %s, times_us %s" % (torch.cuda.get_device_name(0), density, sizes,
                                                     [round(x * 1e6, 1) for x in times])}
        print("compress fit: c0 = %.1f us, c1 = %.3g s/elem (%.2f TB/s equivalent at 7 fp32 streams)" % (
            c0 * 1e6, c1, 28 / c1 / 1e12 if c1 > 0 else 0.0))
        if args.fit_out:
            perf_model.update(args.fit_out, "compress", entry)
        rows.append({"kernel": "compress fit", **entry})

    # ---------------- decompress ----------------
    for P in (1, 8) if want("decompress") else ():
        bufs = ops.CompressBuffers(2 * k, dev)
        g = g0.clone()
        ops.compress_(g, r, bufs, ops.MODE_TOPK, ec=False, zero_g=False, k=k, k_cap=2 * k, n_stats=args.n)
        recs = bufs.record.repeat(P)
        dst = torch.zeros(n, device=dev)
        t = timeit(lambda: ops.scatter_add_records_(dst, recs, P, 2 * k, 1.0 / P))
        report("scatter_add_records P=%d" % P, t, P * k * 8 * 2, "atomic fp32, %d pairs" % (P * k))

    # ---------------- fused optimizer ----------------
    if not want("optim") and not want("bn"):
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(rows, f, indent=1)
        return 0
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
