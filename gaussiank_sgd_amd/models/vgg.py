"""VGG networks.

* ``VGG('VGG16')``: CIFAR VGG with batch-norm and a 512->10 classifier
  (reference models/vgg.py:6-38; 14,728,266 parameters for VGG16) -- the
  BASELINE config "VGG-16 on CIFAR-shaped synthetic".
* ``vgg16i``: ImageNet VGG-16 (reference uses torchvision.models.vgg16,
  dl_trainer.py:93-96), re-implemented here.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.bn import BNAct
from ..ops.conv1x1 import FastConv2d

cfg = {
    "VGG11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "VGG19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512,
              "M"],
}


def _features(spec, batch_norm: bool) -> nn.Sequential:
    """conv -> [BN] -> ReLU [-> MaxPool], the reference's layer order and
    state_dict indices.  MI355X: convolutions are FastConv2d (autotuned MFMA
    implicit GEMM vs MIOpen); with batch norm, BN + ReLU (+ the following 2x2
    max-pool) run as ONE fused BNAct pass and the ReLU / pool slots hold
    nn.Identity (no parameters, so the indices and keys are unchanged)."""
    layers = []
    c = 3
    for i, v in enumerate(spec):
        if v == "M":
            fused = batch_norm and i > 0 and spec[i - 1] != "M"
            layers.append(nn.Identity() if fused else nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers.append(FastConv2d(c, v, kernel_size=3, padding=1))
            if batch_norm:
                pool = (2, 2, 0) if i + 1 < len(spec) and spec[i + 1] == "M" else None
                layers.append(BNAct(v, act="relu", pool=pool))
                layers.append(nn.Identity())
            else:
                layers.append(nn.ReLU(inplace=True))
            c = v
    return nn.Sequential(*layers)


class VGG(nn.Module):
    """CIFAR VGG (32x32 inputs)."""

    def __init__(self, vgg_name: str = "VGG16", num_classes: int = 10):
        super().__init__()
        self.features = _features(cfg[vgg_name.upper()], batch_norm=True)
        self.fc = nn.Linear(512, num_classes)
        self.name = vgg_name.lower()

    def forward(self, x):
        out = self.features(x)
        return self.fc(out.reshape(out.shape[0], -1))


class VGGImageNet(nn.Module):
    """ImageNet VGG (224x224 inputs), torchvision layout."""

    def __init__(self, vgg_name: str = "VGG16", num_classes: int = 1000, batch_norm: bool = False):
        super().__init__()
        self.features = _features(cfg[vgg_name.upper()], batch_norm)
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(
            nn.Linear(512 * 7 * 7, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, num_classes))
        self.name = vgg_name.lower() + "i"
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


def vgg16i(num_classes=1000):
    return VGGImageNet("VGG16", num_classes)
