#!/usr/bin/env python3
"""Gradient-distribution plots from dumped gradients (reference logs/plot_cdf.py).

Reads ``r<rank>_gradients_iter_<n>.npy`` dumps (numpy, ``allow_pickle=False``)
and draws a histogram-based density of each, overlaid with the normal fit
N(mean, std) that Gaussian-k assumes, plus the empirical CDF of |g| with the
Gaussian-k threshold for a given density.

    python tools/plot_cdf.py --filename r0_gradients_iter_100.npy --legend resnet20 --density 0.001
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summarize(x: np.ndarray, density: float) -> dict:
    from gaussiank_sgd_amd.utils.stats import gaussian_z
    mean, std = float(x.mean()), float(x.std(ddof=1))
    thr = mean + gaussian_z(density) * std
    k = max(int(x.size * density), 1)
    exact = float(np.sort(np.abs(x))[-k]) if x.size else 0.0
    return {"n": int(x.size), "mean": mean, "std": std, "gaussian_thr": thr, "topk_thr": exact,
            "selected_at_gaussian_thr": int((np.abs(x) > thr).sum()), "k": k}


def main(argv=None):
    ap = argparse.ArgumentParser(description="CDF PDF Plotting Script")
    ap.add_argument("--filename", nargs="+", required=True)
    ap.add_argument("--legend", nargs="+", default=None)
    ap.add_argument("--density", type=float, default=0.001)
    ap.add_argument("--output", default="plot.png")
    a = ap.parse_args(argv)
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    legends = a.legend or [os.path.basename(f) for f in a.filename]
    fig, (ax0, ax1) = plt.subplots(1, 2, figsize=(11, 4.5))
    for f, lab in zip(a.filename, legends):
        x = np.load(f, allow_pickle=False).astype(np.float64).ravel()
        s = summarize(x, a.density)
        print("Name: %s Min: %s Max: %s %s" % (os.path.basename(f), x.min(), x.max(), s))
        hist, edges = np.histogram(x, bins=400, density=True)
        c = 0.5 * (edges[1:] + edges[:-1])
        ax0.plot(c, hist, label=lab)
        g = np.exp(-0.5 * ((c - s["mean"]) / s["std"]) ** 2) / (s["std"] * math.sqrt(2 * math.pi))
        ax0.plot(c, g, "--", alpha=0.6, label=lab + " normal fit")
        ax0.set_yscale("log")
        ax = np.sort(np.abs(x))
        ax1.plot(ax, np.arange(1, ax.size + 1) / ax.size, label=lab)
        ax1.axvline(s["gaussian_thr"], ls="--", color="k", alpha=0.5)
    ax0.set_xlabel("Gradients")
    ax0.legend()
    ax1.set_xlabel("|g|")
    ax1.set_ylabel("CDF")
    ax1.set_xscale("log")
    fig.tight_layout()
    fig.savefig(a.output)
    print(a.output)


if __name__ == "__main__":
    main()
