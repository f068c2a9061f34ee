"""Data pipelines.

The reference reads ImageNet-HDF5 / CIFAR-10 / MNIST through torchvision and
PTB through ptb_reader with single-threaded loaders (dl_trainer.py:295-502;
its IO is ~30% of an iteration).  There is no network here and
no torchvision, so the default pipeline is *synthetic, shape-exact and
generated on the device*: no host->device copies inside the timed loop.
``data/real.py`` reads real datasets (CIFAR / MNIST / PTB files, .npz /
.npy arrays, ImageNet image folders) when a user has them on disk.
"""
from .synthetic import DATASETS, SyntheticData, make_data

__all__ = ["DATASETS", "SyntheticData", "make_data"]
