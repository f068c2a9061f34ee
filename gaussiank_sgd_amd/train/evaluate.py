"""Evaluate saved checkpoints epoch by epoch (reference evaluate.py:10-73).

For i in 1..N loads ``<dnn>-rank0-epoch<i>.pth`` from the checkpoint
directory, runs ``DLTrainer.test`` and tracks the best accuracy (or the
lowest perplexity for the LSTM).  Checkpoints are read with
``weights_only=True``.

    python -m gaussiank_sgd_amd.train.evaluate --dnn resnet20 --dataset cifar10 \
        --path weights/allreduce/resnet20-n2-bs32-lr0.1000 --epochs 10
"""
from __future__ import annotations

import argparse
import os

import torch

from ..settings import logger
from .trainer import DLTrainer, _support_datasets, _support_dnns


def evaluate(dnn, dataset, path, epochs, batch_size=64, device=None, num_batches=4):
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    trainer = DLTrainer(0, 1, dist=False, batch_size=batch_size, dataset=dataset, dnn=dnn, device=device)
    best, best_epoch = None, -1
    lower_is_better = dnn in ("lstm", "lstman4") or dnn.startswith("bert")
    results = {}
    for i in range(1, epochs + 1):
        fn = os.path.join(path, "%s-rank0-epoch%d.pth" % (dnn, i))
        if not os.path.isfile(fn):
            continue
        trainer.load_model_from_file(fn)
        acc = trainer.test(i, num_batches=num_batches)
        results[i] = acc
        better = best is None or (acc < best if lower_is_better else acc > best)
        if better:
            best, best_epoch = acc, i
    logger.info("Best accuracy/perplexity: %s at epoch %d", best, best_epoch)
    return best, best_epoch, results


def main(argv=None):
    ap = argparse.ArgumentParser(description="Evaluate checkpoints")
    ap.add_argument("--dnn", default="resnet20", choices=_support_dnns)
    ap.add_argument("--dataset", default="cifar10", choices=_support_datasets)
    ap.add_argument("--path", required=True)
    ap.add_argument("--epochs", type=int, default=140)
    ap.add_argument("--batch-size", type=int, default=64)
    args = ap.parse_args(argv)
    return evaluate(args.dnn, args.dataset, args.path, args.epochs, args.batch_size)


if __name__ == "__main__":
    main()
