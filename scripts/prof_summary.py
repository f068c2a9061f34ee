#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/*.csv.

usage: python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv OUT.csv --steps 8 --title "..."
"""
import argparse
import collections
import csv
import re


def category(n: str) -> str:
    if "gk::" in n and ("add_ln" in n or "ln_param" in n):
        return "gk fused add+LayerNorm"
    if "gk::" in n and ("rec_gemm" in n or "lstm_" in n):
        return "gk LSTM (split-K step GEMM + fused cells)"
    if "gk::" in n and "colsum" in n:
        return "gk linear bias-grad column sums"
    if "gk::" in n and "weight_prep" in n:
        return "gk per-step weight re-layouts (prep.hip)"
    if "gk::" in n and ("gemm_nt" in n or "gemm_tn" in n or "stem_" in n or "wgrad3" in n or "wino_" in n or
                        "splitk_reduce" in n):
        return "gk HIP conv GEMMs (1x1 / implicit-GEMM 3x3 / Winograd, MFMA)"
    if "gk::" in n and "attn_" in n:
        return "gk fused attention (flash fwd / dQ / dK-dV, MFMA)"
    if "gk::" in n:
        if "bn_" in n:
            return "gk fused BN (+ReLU/residual/pool)"
        return "gk compression/exchange/optimizer"
    if "igemm_fwd" in n or "conv_fwd" in n:
        return "MIOpen conv fwd"
    if "igemm_bwd" in n or "bwd_data" in n:
        return "MIOpen conv bwd-data"
    if "igemm_wrw" in n or "bwd_weight" in n:
        return "MIOpen conv bwd-weight"
    if "attn_fwd" in n or "bwd_kernel_d" in n or "bwd_preprocess" in n:
        return "attention (torch SDPA flash kernels)"
    if "batched_gemm" in n or "Cijk" in n:
        return "GEMM (CK / hipBLASLt)"
    if "SubTensor" in n or "fillBuffer" in n:
        return "MIOpen/runtime zero-fill"
    if "copy" in n.lower():
        return "copies"
    return "other torch elementwise/reduce"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    cats = collections.Counter()
    for r in rows:
        cats[category(r["Name"])] += float(r["TotalDurationNs"])
    with open(a.out, "w") as f:
        f.write("# %s\n" % a.title)
        f.write("# total kernel time %.1f ms over %d steps = %.2f ms/step\n" % (tot / 1e6, a.steps,
                                                                              tot / 1e6 / a.steps))
        for c, v in cats.most_common():
            f.write("# category,%s,%.3f ms/step,%.1f%%\n" % (c, v / 1e6 / a.steps, 100 * v / tot))
        w = csv.writer(f)
        w.writerow(["name", "calls", "avg_us", "pct", "ms_per_step"])
        for r in rows[:a.top]:
            name = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", ""))[:160]
            t = float(r["TotalDurationNs"])
            w.writerow([name, r["Calls"], "%.1f" % (float(r["AverageNs"]) / 1e3), "%.2f" % (100 * t / tot),
                        "%.3f" % (t / 1e6 / a.steps)])


if __name__ == "__main__":
    main()
