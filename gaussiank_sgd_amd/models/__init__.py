"""Model zoo and the ``create_net`` factory.

Parity: reference ``dl_trainer.create_net`` (dl_trainer.py:84-120) and
``models/__init__.py:16-30``.  torchvision is not available on this image, so
every network the reference takes from torchvision (resnet50, vgg16i,
alexnet, inception_v3) is implemented here.
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import torch.nn as nn

from .bert import BertForMaskedLM, MaskedLMLoss, bert_base, bert_tiny
from .lstm_ptb import PTBLSTM, lstm, repackage_hidden
from .mlp import FCN5Net, LeNet, LinearRegression, MnistNet
from .resnet_cifar import (CifarPreResNet, CifarResNet, preresnet20, preresnet56, preresnet110, resnet20, resnet32,
                           resnet44, resnet56, resnet110)
from .resnet_imagenet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152, resnext50_32x4d
from .vgg import VGG, VGGImageNet, vgg16i

# dnn name -> (constructor(num_classes, **kw), default dataset)
_REGISTRY: Dict[str, Tuple[Callable[..., nn.Module], str]] = {
    "lr": (lambda nc, **kw: LinearRegression(nc), "mnist"),
    "fcn5net": (lambda nc, **kw: FCN5Net(nc), "mnist"),
    "lenet": (lambda nc, **kw: LeNet(nc), "mnist"),
    "mnistnet": (lambda nc, **kw: MnistNet(nc), "mnist"),
    "resnet20": (lambda nc, **kw: resnet20(nc), "cifar10"),
    "resnet32": (lambda nc, **kw: resnet32(nc), "cifar10"),
    "resnet44": (lambda nc, **kw: resnet44(nc), "cifar10"),
    "resnet56": (lambda nc, **kw: resnet56(nc), "cifar10"),
    "resnet110": (lambda nc, **kw: resnet110(nc), "cifar10"),
    "preresnet20": (lambda nc, **kw: preresnet20(nc), "cifar10"),
    "preresnet56": (lambda nc, **kw: preresnet56(nc), "cifar10"),
    "preresnet110": (lambda nc, **kw: preresnet110(nc), "cifar10"),
    "vgg11": (lambda nc, **kw: VGG("VGG11", nc), "cifar10"),
    "vgg13": (lambda nc, **kw: VGG("VGG13", nc), "cifar10"),
    "vgg16": (lambda nc, **kw: VGG("VGG16", nc), "cifar10"),
    "vgg19": (lambda nc, **kw: VGG("VGG19", nc), "cifar10"),
    "resnet18": (lambda nc, **kw: resnet18(nc), "imagenet"),
    "resnet34": (lambda nc, **kw: resnet34(nc), "imagenet"),
    "resnet50": (lambda nc, **kw: resnet50(nc, **{k: v for k, v in kw.items() if k == "zero_init_residual"}),
                 "imagenet"),
    "resnet101": (lambda nc, **kw: resnet101(nc), "imagenet"),
    "resnet152": (lambda nc, **kw: resnet152(nc), "imagenet"),
    "resnext50": (lambda nc, **kw: resnext50_32x4d(nc), "imagenet"),
    "vgg16i": (lambda nc, **kw: vgg16i(nc), "imagenet"),
    "lstm": (lambda nc, **kw: lstm(vocab_size=kw.get("vocab_size", 10000), batch_size=kw.get("batch_size", 20),
                                   num_steps=kw.get("num_steps", 35)), "ptb"),
    "bert": (lambda nc, **kw: bert_base(), "wikipedia"),
    "bert_tiny": (lambda nc, **kw: bert_tiny(), "wikipedia"),
}


def register(name: str, ctor: Callable[..., nn.Module], dataset: str) -> None:
    _REGISTRY[name] = (ctor, dataset)


def available() -> list:
    return sorted(_REGISTRY)


def default_dataset(dnn: str) -> str:
    return _REGISTRY[dnn][1]


def create_net(num_classes: int, dnn: str = "resnet20", **kwargs):
    """Return ``(net, ext)`` like the reference (ext is model-specific extras or None)."""
    if dnn not in _REGISTRY:
        raise ValueError("Unsupport neural network %s" % dnn)
    net = _REGISTRY[dnn][0](num_classes, **kwargs)
    if not hasattr(net, "name"):
        net.name = dnn
    return net, None


def _late_imports():
    # larger / less common zoo members register themselves on import
    from . import extra  # noqa: F401


try:
    _late_imports()
except ImportError:  # pragma: no cover
    pass
