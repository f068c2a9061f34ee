"""Checkpoint save/load.

Layout (reference dl_trainer.py:649-661,836-837): ``{'iter', 'epoch',
'state'}`` saved to ``weights/<prefix>/<dnn>-n<P>-bs<B>-lr<lr>/
<dnn>-rank<r>-epoch<e>.pth``; ``evaluate.py``-style loaders only need those
three keys.  Added (reference resume is lossy): ``optimizer`` (momentum),
``compression`` (per-rank residuals + density epoch), ``rng``.  Loads use
``weights_only=True`` -- nothing in a checkpoint is executed.
"""
from __future__ import annotations

import os

import torch


def save_checkpoint(state: dict, filename: str) -> None:
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = filename + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, filename)


def load_checkpoint(filename: str, map_location="cpu") -> dict:
    return torch.load(filename, map_location=map_location, weights_only=True)
