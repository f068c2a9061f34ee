"""Compression pipeline on the 25.6 M bucket (bench/kernels.py round2 shape),
looped for a kernel trace: ``rocprofv3 --kernel-trace --stats --output-format
csv -d DIR -o p -- python3 scripts/debug/compress_prof.py``, then
``python3 scripts/debug/compress_prof.py --summarize DIR`` prints per-kernel
times, the launch gaps and the first-to-last span of every pipeline call.
"""
import argparse
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(args):
    import torch
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.utils.stats import gaussian_z
    dev = torch.device("cuda", 0)
    n = (args.n + 63) // 64 * 64
    k = max(int(args.n * 0.001), 1)
    kc = (4 * k + 2) // 3
    pool = [torch.randn(n, device=dev) * 1e-3 * (1 + 0.1 * i) for i in range(4)]
    g = pool[0].clone()
    rr = torch.zeros(n, device=dev)
    bufs = ops.CompressBuffers(kc, dev)
    mode = {"gaussian": ops.MODE_GAUSSIAN, "gaussian_cal": ops.MODE_GAUSSIAN_CAL}[args.mode]
    for it in range(args.warmup + args.iters):
        g.copy_(pool[it % 4])
        ops.compress_(g, rr, bufs, mode, ec=True, zero_g=True, loops=3, z=gaussian_z(0.001), k=k, k_cap=kc,
                      seed=7, n_stats=args.n)
    torch.cuda.synchronize()
    print("done", args.mode, n, k, kc, flush=True)


def summarize(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not f:
        print("no kernel_trace.csv under", d)
        return 1
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one pipeline call = the kernels between two copies (elementwise copy kernels)
    calls, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if "copy" in name.lower() or "elementwise" in name.lower():
            if cur:
                calls.append(cur)
            cur = []
            continue
        if "gk::" in name:
            cur.append(r)
    if cur:
        calls.append(cur)
    calls = calls[len(calls) // 2:]   # steady state
    per = {}
    gaps, spans = [], []
    for c in calls:
        spans.append((int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3)
        for i, r in enumerate(c):
            nm = r["Kernel_Name"].split("(")[0][-70:]
            per.setdefault((i, nm), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            if i:
                gaps.append((int(r["Start_Timestamp"]) - int(c[i - 1]["End_Timestamp"])) / 1e3)
    print("calls %d, pipeline span median %.1f us (min %.1f)" % (len(calls), statistics.median(spans), min(spans)))
    print("launch gaps: %d per call, median %.2f us" % (len(gaps) // max(len(calls), 1), statistics.median(gaps)))
    for (i, nm), ts in sorted(per.items()):
        print("  %2d %-72s %8.2f us" % (i, nm, statistics.median(ts)))
    return 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=25_557_032)
    ap.add_argument("--mode", default="gaussian")
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        sys.exit(summarize(a.summarize))
    run(a)
