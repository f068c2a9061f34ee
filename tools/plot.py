#!/usr/bin/env python3
"""Training-curve plots from trainer logs (reference logs/plot.py).

Parses the log lines written by ``DLTrainer``/``dist_trainer``:
  ``... Epoch %d, lr: %f, val loss: %f, val top-1 acc: %f, top-5 acc: %f``
  ``... Time per iteration including communication: %f, Speed: %f images/s``
and plots accuracy / loss / lr per epoch or throughput per display window.

    python tools/plot.py --network resnet20 --plot-type acc \
        --logfile-names logs/.../host-0.log logs/.../host-0.log --legends topk gaussian
"""
from __future__ import annotations

import argparse
import re
from typing import Dict, List

EPOCH_RE = re.compile(r"Epoch (\d+), lr: ([0-9.eE+-]+), val loss: ([0-9.eE+-naif]+), val top-1 acc: "
                      r"([0-9.eE+-naif]+), top-5 acc: ([0-9.eE+-naif]+)")
SPEED_RE = re.compile(r"Time per iteration including communication: ([0-9.eE+-]+), Speed: ([0-9.eE+-]+)")
SELECT_RE = re.compile(r"Average number of selected gradients: ([0-9.eE+-]+), exact k: (\d+)")


def read_log(path: str) -> Dict[str, List[float]]:
    out: Dict[str, List[float]] = {"epoch": [], "lr": [], "loss": [], "acc": [], "acc5": [], "iter_time": [],
                                   "speed": [], "selected": [], "k": []}
    with open(path) as f:
        for line in f:
            m = EPOCH_RE.search(line)
            if m:
                out["epoch"].append(int(m.group(1)))
                out["lr"].append(float(m.group(2)))
                out["loss"].append(float(m.group(3)))
                out["acc"].append(float(m.group(4)))
                out["acc5"].append(float(m.group(5)))
                continue
            m = SPEED_RE.search(line)
            if m:
                out["iter_time"].append(float(m.group(1)))
                out["speed"].append(float(m.group(2)))
                continue
            m = SELECT_RE.search(line)
            if m:
                out["selected"].append(float(m.group(1)))
                out["k"].append(int(m.group(2)))
    return out


def plot_graph(network: str, plot_type: str, logfile_names: List[str], legends: List[str], output: str):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots(figsize=(7, 4.5))
    key = {"acc": "acc", "loss": "loss", "lr": "lr", "speed": "speed", "acc5": "acc5", "selected": "selected"}[plot_type]
    for path, label in zip(logfile_names, legends):
        d = read_log(path)
        ys = d[key]
        xs = d["epoch"] if key in ("acc", "loss", "lr", "acc5") else list(range(1, len(ys) + 1))
        ax.plot(xs[: len(ys)], ys, label=label)
    ax.set_title(network)
    ax.set_xlabel("epoch" if key in ("acc", "loss", "lr", "acc5") else "display window")
    ax.set_ylabel({"acc": "top-1 accuracy (%)", "acc5": "top-5 accuracy (%)", "loss": "validation loss",
                   "lr": "learning rate", "speed": "images/s per worker", "selected": "selected gradients"}[key])
    ax.grid(alpha=0.3)
    ax.legend()
    fig.tight_layout()
    fig.savefig(output)
    return output


def main(argv=None):
    ap = argparse.ArgumentParser(description="Plotting Script")
    ap.add_argument("--network", type=str, default="resnet20")
    ap.add_argument("--plot-type", type=str, default="acc", choices=["acc", "acc5", "loss", "lr", "speed", "selected"])
    ap.add_argument("--logfile-names", nargs="+", required=True)
    ap.add_argument("--legends", nargs="+", required=True)
    ap.add_argument("--output", default=None)
    a = ap.parse_args(argv)
    out = a.output or "%s_%s.png" % (a.network, a.plot_type)
    print(plot_graph(a.network, a.plot_type, a.logfile_names, a.legends, out))


if __name__ == "__main__":
    main()
