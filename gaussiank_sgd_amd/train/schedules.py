"""Learning-rate schedules (called every iteration, like the reference).

Parity: dl_trainer.py:541-605 --
  * general: linear warm-up over 5 epochs from base/(5*iters) (when
    settings.WARMUP), then x0.1 steps at 81/122/155 (CIFAR/MNIST),
    30/60/80 (ImageNet) or 24/60/80 (PTB via the general path);
  * PTB LSTM: base until 63, then x0.1/x0.01/x0.001 at 63/60/80 (sic: the
    second boundary is below the first, so 0.1x is never used);
  * AN4: divide by 1.01 each epoch.
"""
from __future__ import annotations


def general_lr(base_lr: float, progress_epoch: int, train_iter: int, num_batches_per_epoch: int, dataset: str,
               warmup: bool = True, warmup_epochs: int = 5) -> float:
    if warmup and progress_epoch < warmup_epochs:
        total = max(1, num_batches_per_epoch * warmup_epochs)
        min_lr = base_lr / total
        return min_lr + (base_lr - min_lr) / total * train_iter
    first, second, third = 81, 81 + 41, 81 + 41 + 33
    if dataset == "imagenet":
        first, second, third = 30, 60, 80
    elif dataset == "ptb":
        first, second, third = 24, 60, 80
    if progress_epoch < first:
        return base_lr
    if progress_epoch < second:
        return base_lr * 0.1
    if progress_epoch < third:
        return base_lr * 0.01
    return base_lr * 0.001


def lstm_ptb_lr(base_lr: float, progress_epoch: int) -> float:
    first, second, third = 23 + 40, 60, 80
    if progress_epoch < first:
        return base_lr
    if progress_epoch < second:
        return base_lr * 0.1
    if progress_epoch < third:
        return base_lr * 0.01
    return base_lr * 0.001


class AN4Schedule:
    """lr /= 1.01 whenever the epoch index changes (dl_trainer.py:541-546)."""

    def __init__(self, base_lr: float):
        self.lr = base_lr
        self.tag = 0

    def __call__(self, epoch: int) -> float:
        if epoch != self.tag:
            self.tag = epoch
            self.lr = self.lr / 1.01
        return self.lr
