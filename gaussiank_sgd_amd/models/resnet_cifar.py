"""CIFAR ResNets (20/32/44/56/110) and pre-activation ResNets.

Parity: reference models/resnet.py:40-147 (option-A shortcut
``DownsampleA`` = stride-2 subsample + zero channel padding,
models/res_utils.py:4-13; uniform(-1/sqrt(n), 1/sqrt(n)) conv init) and
models/preresnet.py.  ResNet-20 has 269,722 parameters in 59 tensors
(the configuration of every published reference log).

MI355X: every BatchNorm is a ``BNAct`` (ops/bn.py) -- BN + ReLU (+ the
residual add of the block output) run as fused channels-last kernels, and a
block output that feeds both the next block and its shortcut hands out two
handles whose gradients are summed inside the BN backward (``twin``).  Same
parameters and state_dict keys as nn.BatchNorm2d.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import init

from ..ops.bn import BNAct


class DownsampleA(nn.Module):
    """Parameter-free shortcut: spatial subsample + zero-padded channels."""

    def __init__(self, nIn: int, nOut: int, stride: int):
        super().__init__()
        assert stride == 2
        self.pad = nOut - nIn

    def forward(self, x):
        x = x[:, :, ::2, ::2]
        return F.pad(x, (0, 0, 0, 0, 0, self.pad))


class ResNetBasicblock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv_a = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn_a = BNAct(planes, act="relu")
        self.conv_b = nn.Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn_b = BNAct(planes, act="relu")       # relu(bn_b(conv_b) + residual), fused
        self.downsample = downsample

    def forward(self, x):
        x, xs = x if isinstance(x, tuple) else (x, x)   # (main, shortcut) handles of a twin BN output
        residual = xs if self.downsample is None else self.downsample(xs)
        out = self.bn_a(self.conv_a(x))
        return self.bn_b(self.conv_b(out), residual)


class CifarResNet(nn.Module):
    def __init__(self, depth: int, num_classes: int = 10):
        super().__init__()
        assert (depth - 2) % 6 == 0, "depth should be one of 20, 32, 44, 56, 110"
        self.name = "resnet%d" % depth
        n = (depth - 2) // 6
        self.num_classes = num_classes
        self.conv_1_3x3 = nn.Conv2d(3, 16, 3, stride=1, padding=1, bias=False)
        self.bn_1 = BNAct(16, act="relu")
        self.inplanes = 16
        self.stage_1 = self._make_layer(16, n, 1)
        self.stage_2 = self._make_layer(32, n, 2)
        self.stage_3 = self._make_layer(64, n, 2)
        self.avgpool = nn.AvgPool2d(8)
        self.classifier = nn.Linear(64, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                stdv = 1.0 / math.sqrt(fan)
                m.weight.data.uniform_(-stdv, stdv)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                init.kaiming_normal_(m.weight)
                m.bias.data.zero_()
        blocks = [b for st in (self.stage_1, self.stage_2, self.stage_3) for b in st]
        self.bn_1.twin = True
        for b in blocks[:-1]:
            b.bn_b.twin = True

    def _make_layer(self, planes, blocks, stride):
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = DownsampleA(self.inplanes, planes, stride)
        layers = [ResNetBasicblock(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(ResNetBasicblock(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.bn_1(self.conv_1_3x3(x))
        x = self.stage_3(self.stage_2(self.stage_1(x)))
        x = self.avgpool(x)
        return self.classifier(x.reshape(x.shape[0], -1))


def resnet20(num_classes=10):
    return CifarResNet(20, num_classes)


def resnet32(num_classes=10):
    return CifarResNet(32, num_classes)


def resnet44(num_classes=10):
    return CifarResNet(44, num_classes)


def resnet56(num_classes=10):
    return CifarResNet(56, num_classes)


def resnet110(num_classes=10):
    return CifarResNet(110, num_classes)


class PreActBlock(nn.Module):
    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.bn_a = BNAct(inplanes, act="relu")
        self.conv_a = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn_b = BNAct(planes, act="relu")
        self.conv_b = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.downsample = downsample

    def forward(self, x):
        out = self.bn_a(x)
        residual = x if self.downsample is None else self.downsample(out)
        out = self.conv_a(out)
        out = self.conv_b(self.bn_b(out))
        return out + residual


class CifarPreResNet(nn.Module):
    """Pre-activation ResNet for CIFAR (reference models/preresnet.py)."""

    def __init__(self, depth: int, num_classes: int = 10):
        super().__init__()
        assert (depth - 2) % 6 == 0
        self.name = "preresnet%d" % depth
        n = (depth - 2) // 6
        self.conv_3x3 = nn.Conv2d(3, 16, 3, padding=1, bias=False)
        self.inplanes = 16
        self.stage_1 = self._make_layer(16, n, 1)
        self.stage_2 = self._make_layer(32, n, 2)
        self.stage_3 = self._make_layer(64, n, 2)
        self.lastact = nn.Sequential(BNAct(64, act="relu"), nn.Identity())
        self.avgpool = nn.AvgPool2d(8)
        self.classifier = nn.Linear(64, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / fan))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                init.kaiming_normal_(m.weight)
                m.bias.data.zero_()

    def _make_layer(self, planes, blocks, stride):
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = DownsampleA(self.inplanes, planes, stride)
        layers = [PreActBlock(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(PreActBlock(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.conv_3x3(x)
        x = self.stage_3(self.stage_2(self.stage_1(x)))
        x = self.avgpool(self.lastact(x))
        return self.classifier(x.reshape(x.shape[0], -1))


def preresnet20(num_classes=10):
    return CifarPreResNet(20, num_classes)


def preresnet56(num_classes=10):
    return CifarPreResNet(56, num_classes)


def preresnet110(num_classes=10):
    return CifarPreResNet(110, num_classes)
