"""Single-GPU training entry (``train_with_single``) with the reference's CLI.

Parity: reference dl_trainer.py:879-927 -- ``train_with_single(dnn, dataset,
data_dir, nworkers, lr, batch_size, nsteps_update, max_epochs, num_steps)``
builds a ``DLTrainer`` with ``prefix='singlegpu'`` and runs the same
epoch / iteration loop as ``ssgd`` without any communication or compression;
``__main__`` logs to ``./logs/singlegpu-<PREFIX>/<dnn>-n1-bs<B>-lr<lr>-ns<n>/
<host>.log`` and prints ``Time per iteration including communication: %f.
Speed: %f images/s`` every ``display`` iterations.

MI355X: the update is the fused one-launch SGD over the flat parameter arena
(the ``DistributedOptimizer`` in a world of one: no hooks, no exchange) and,
on the GPU, the convolution / linear weight gradients go straight into that
arena; ``--plain-sgd`` keeps ``torch.optim.SGD`` as the reference did.
Run: ``python -m gaussiank_sgd_amd.train.single --dnn resnet20 --dataset
cifar10`` (or ``python -m gaussiank_sgd_amd.train.trainer``).
"""
from __future__ import annotations

import argparse
import logging
import os
import time

import numpy as np
import torch

from .. import settings, utils
from ..settings import formatter, logger
from .trainer import DLTrainer, _support_datasets, _support_dnns


def train_with_single(dnn, dataset, data_dir, nworkers, lr, batch_size, nsteps_update, max_epochs, num_steps=1,
                      amp=None, channels_last=False, max_iters=None, train_samples=None, fused=True,
                      f32_matmul=None, saved_dir="."):
    device = "cpu"
    if torch.cuda.is_available():
        torch.cuda.set_device(0)
        device = "cuda"
    if f32_matmul is not None:
        from ..ops import conv1x1
        conv1x1.set_f32_matmul(f32_matmul)
    trainer = DLTrainer(0, nworkers, dist=False, batch_size=batch_size, is_weak_scaling=True, ngpus=1,
                        data_dir=data_dir, dataset=dataset, dnn=dnn, lr=lr, nworkers=nworkers, prefix="singlegpu",
                        num_steps=num_steps, device=device, amp=amp, channels_last=channels_last,
                        weights_dir=os.path.join(saved_dir, "weights"), train_samples=train_samples)
    if fused:
        from ..compression import compressors
        from ..parallel.distributed_optimizer import DistributedOptimizer
        opt = DistributedOptimizer(trainer.optimizer, named_parameters=trainer.net.named_parameters(),
                                   compression=compressors["none"], is_sparse=False, density=1.0,
                                   threshold=524288000, density_warmup=False)
        if trainer.is_cuda:
            from ..parallel import install_bf16_shadow, install_direct_grads
            if trainer.amp == "bf16":
                install_bf16_shadow(trainer.net, opt)
            else:
                install_direct_grads(trainer.net, opt)
        trainer.update_optimizer(opt)
    iters_per_epoch = max(1, trainer.get_num_of_training_samples() // (nworkers * batch_size * nsteps_update))
    times = []
    display = 40 if iters_per_epoch > 40 else max(1, iters_per_epoch - 1)
    done = 0
    for epoch in range(max_epochs):
        hidden = None
        if dnn == "lstm":
            hidden = trainer.net.init_hidden()
        for i in range(iters_per_epoch):
            s = time.time()
            trainer.optimizer.zero_grad()
            for _ in range(nsteps_update):
                if dnn == "lstm":
                    _, hidden = trainer.train(1, hidden=hidden)
                else:
                    trainer.train(1)
            trainer.update_model()
            times.append(time.time() - s)
            if i % display == 0 and i > 0:
                if trainer.is_cuda:
                    torch.cuda.synchronize()
                time_per_iter = float(np.mean(times))
                logger.info("Time per iteration including communication: %f. Speed: %f images/s", time_per_iter,
                            batch_size * nsteps_update / time_per_iter)
                times = []
            done += 1
            if max_iters is not None and done >= max_iters:
                return trainer
    return trainer


def build_parser():
    p = argparse.ArgumentParser(description="Single trainer")
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--nsteps-update", type=int, default=1)
    p.add_argument("--dataset", type=str, default="imagenet", choices=_support_datasets,
                   help="Specify the dataset for training")
    p.add_argument("--dnn", type=str, default="resnet50", choices=_support_dnns,
                   help="Specify the neural network for training")
    p.add_argument("--data-dir", type=str, default="./data", help="Specify the data root path")
    p.add_argument("--lr", type=float, default=0.1, help="Default learning rate")
    p.add_argument("--max-epochs", type=int, default=settings.MAX_EPOCHS, help="Default maximum epochs to train")
    p.add_argument("--num-steps", type=int, default=35)
    # MI355X build additions
    p.add_argument("--amp", type=str, default=None, choices=[None, "bf16"])
    p.add_argument("--channels-last", action="store_true")
    p.add_argument("--max-iters", type=int, default=None)
    p.add_argument("--train-samples", type=int, default=None,
                   help="synthetic epoch length in samples (default: the dataset's real size)")
    p.add_argument("--plain-sgd", action="store_true", help="torch.optim.SGD instead of the fused arena update")
    p.add_argument("--f32-matmul", type=str, default=os.environ.get("GKSGD_F32_MATMUL", "bf16x6"),
                   choices=["native", "bf16x6"], help="fp32 GEMM algorithm (default: %(default)s, as bench.py)")
    p.add_argument("--saved-dir", type=str, default=".")
    p.add_argument("--logdir-root", type=str, default="./logs")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    batch_size = args.batch_size * args.nsteps_update
    relative_path = os.path.join(args.logdir_root, "singlegpu-%s/%s-n%d-bs%d-lr%.4f-ns%d" % (
        settings.PREFIX, args.dnn, 1, batch_size, args.lr, args.nsteps_update))
    utils.create_path(relative_path)
    logfile = os.path.join(relative_path, settings.hostname + ".log")
    hdlr = logging.FileHandler(logfile)
    hdlr.setFormatter(formatter)
    logger.addHandler(hdlr)
    logger.info("Configurations: %s", args)
    return train_with_single(args.dnn, args.dataset, args.data_dir, 1, args.lr, args.batch_size, args.nsteps_update,
                             args.max_epochs, args.num_steps, amp=args.amp, channels_last=args.channels_last,
                             max_iters=args.max_iters, train_samples=args.train_samples, fused=not args.plain_sgd,
                             f32_matmul=args.f32_matmul, saved_dir=args.saved_dir)


if __name__ == "__main__":
    main()
