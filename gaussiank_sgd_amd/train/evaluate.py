"""Evaluate saved checkpoints epoch by epoch (reference evaluate.py:10-73).

Same command line as the reference:

    python -m gaussiank_sgd_amd.train.evaluate --model-path weights/allreduce/resnet20-n2-bs32-lr0.1000 \
        --dnn resnet20 --dataset cifar10 --data-dir ./data --nepochs 140

* the model name, per-worker batch size and learning rate are parsed from the
  checkpoint directory name ``<dnn>-n<P>-bs<B>-lr<lr>`` (reference :21-24;
  ``DLTrainer.checkpoint_dir`` writes that layout);
* for i in 1..nepochs ``<dnn>-rank0-epoch<i>.pth`` is loaded and
  ``DLTrainer.test`` scores it on the WHOLE test split of ``--data-dir``
  (synthetic batches when the directory holds no data);
* the best accuracy (lowest perplexity / WER for lstm / lstman4, and
  perplexity for BERT) is logged after every epoch, and everything goes to
  ``<model-path>/evaluate.log`` as well (reference :68-71).

Checkpoints are read with ``weights_only=True``; a missing epoch file is
skipped (the reference would raise).  ``--path`` / ``--epochs`` are accepted
as aliases of ``--model-path`` / ``--nepochs``.
"""
from __future__ import annotations

import argparse
import logging
import os
from typing import Optional, Tuple

import torch

from ..settings import formatter, logger
from .trainer import DLTrainer, _support_datasets, _support_dnns


def parse_model_path(model_path: str) -> Tuple[Optional[str], Optional[int], Optional[float]]:
    """(dnn, batch_size, lr) from ``<dnn>-n<P>-bs<B>-lr<lr>`` (reference
    evaluate.py:21-24: items[0], items[2][2:], items[-1][2:]); None for a part
    that does not parse."""
    items = os.path.basename(os.path.normpath(model_path)).split("-")
    dnn = items[0] if items and items[0] else None
    bs = lr = None
    if len(items) >= 3 and items[2].startswith("bs"):
        try:
            bs = int(items[2][2:])
        except ValueError:
            bs = None
    if len(items) >= 2 and items[-1].startswith("lr"):
        try:
            lr = float(items[-1][2:])
        except ValueError:
            lr = None
    return dnn, bs, lr


def evaluate(model_path, dnn, dataset, data_dir="./data", nepochs=90, batch_size=None, lr=None, device=None,
             num_batches: Optional[int] = None):
    p_dnn, p_bs, p_lr = parse_model_path(model_path)
    if p_dnn in _support_dnns:
        dnn = p_dnn                        # the reference takes the model from the path
    batch_size = batch_size or p_bs or 64
    lr = lr if lr is not None else (p_lr if p_lr is not None else 0.1)
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    trainer = DLTrainer(0, 1, dist=False, ngpus=1, batch_size=batch_size, is_weak_scaling=True, dataset=dataset,
                        dnn=dnn, data_dir=data_dir, lr=lr, nworkers=1, device=device)
    lower_is_better = dnn in ("lstm", "lstman4") or dnn.startswith("bert")
    best, best_epoch = None, -1
    results = {}
    for i in range(1, nepochs + 1):
        fn = os.path.join(model_path, "%s-rank%d-epoch%d.pth" % (dnn, 0, i))
        if not os.path.isfile(fn):
            continue
        trainer.load_model_from_file(fn)
        acc = trainer.test(i, num_batches=num_batches)
        results[i] = acc
        if best is None or (acc < best if lower_is_better else acc > best):
            best, best_epoch = acc, i
        logger.info("Best validation accuracy or perprexity: %f", best)
    return best, best_epoch, results


def main(argv=None):
    ap = argparse.ArgumentParser(description="Evaluate checkpoints (reference evaluate.py)")
    ap.add_argument("--model-path", "--path", dest="model_path", required=True, help="saved model directory")
    ap.add_argument("--dnn", default="resnet20", choices=_support_dnns)
    ap.add_argument("--dataset", default="cifar10", choices=_support_datasets)
    ap.add_argument("--data-dir", default="./data", help="data root (test split)")
    ap.add_argument("--nepochs", "--epochs", dest="nepochs", type=int, default=90,
                    help="number of epochs to evaluate")
    ap.add_argument("--batch-size", type=int, default=None, help="default: parsed from the model path")
    ap.add_argument("--num-batches", type=int, default=None,
                    help="score only this many batches (default: the whole test split)")
    args = ap.parse_args(argv)
    hdlr = logging.FileHandler(os.path.join(args.model_path, "evaluate.log"))
    hdlr.setFormatter(formatter)
    logger.addHandler(hdlr)
    try:
        return evaluate(args.model_path, args.dnn, args.dataset, args.data_dir, args.nepochs, args.batch_size,
                        num_batches=args.num_batches)
    finally:
        logger.removeHandler(hdlr)
        hdlr.close()


if __name__ == "__main__":
    main()
