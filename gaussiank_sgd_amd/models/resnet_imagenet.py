"""ImageNet ResNets (18/34/50/101/152), torchvision-equivalent architecture.

Parity: the reference builds ``torchvision.models.resnet50`` (dl_trainer.py:
88-90) and ships a local twin (models/imagenet_resnet.py:163-171);
torchvision is not available here, so this is an independent implementation
of the same network (25,557,032 parameters / 161 tensors for ResNet-50).

MI355X notes: run with ``memory_format=torch.channels_last`` and bf16
autocast so MIOpen picks its NHWC implicit-GEMM (MFMA) convolutions; the
final BN of every bottleneck is zero-initialised (``zero_init_residual``) as
is standard for large-batch data-parallel training (off by default for
parity).  Every BatchNorm is a ``BNAct`` (ops/bn.py): BN + residual add +
ReLU run as fused gfx950 kernels in training (same parameters/state_dict
keys as nn.BatchNorm2d; plain torch ops on CPU / in eval).
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from ..ops.bn import BNAct, global_avg_pool
from ..ops.conv1x1 import Conv1x1, Conv3x3, conv_stats
from ..ops.stem import StemConv


def conv3x3(inp: int, out: int, stride: int = 1, groups: int = 1, dilation: int = 1) -> nn.Conv2d:
    # nn.Conv2d subclass: training runs the autotuned implicit-GEMM MFMA kernels (ops/conv1x1.py)
    return Conv3x3(inp, out, stride, groups, dilation)


def conv1x1(inp: int, out: int, stride: int = 1) -> nn.Conv2d:
    # nn.Conv2d subclass: training runs the autotuned MFMA GEMMs (ops/conv1x1.py)
    return Conv1x1(inp, out, stride)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = BNAct(planes, act="relu")
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = BNAct(planes, act="relu")
        self.downsample = downsample

    def forward(self, x):
        x, xs = x if isinstance(x, tuple) else (x, x)   # (main, shortcut) handles, see BNAct twin
        identity = xs if self.downsample is None else _shortcut(self.downsample, xs, self.bn2)
        y, st = conv_stats(self.conv1, x)   # BN statistics from the conv epilogue when fused
        out = self.bn1(y, stats=st)
        y, st = conv_stats(self.conv2, out)
        return self.bn2(y, identity, stats=st)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = BNAct(width, act="relu")
        self.conv2 = conv3x3(width, width, stride, groups)
        self.bn2 = BNAct(width, act="relu")
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = BNAct(planes * self.expansion, act="relu")
        self.downsample = downsample

    def forward(self, x):
        x, xs = x if isinstance(x, tuple) else (x, x)   # (main, shortcut) handles, see BNAct twin
        identity = xs if self.downsample is None else _shortcut(self.downsample, xs, self.bn3)
        y, st = conv_stats(self.conv1, x)   # BN statistics from the conv epilogue when fused
        out = self.bn1(y, stats=st)
        y, st = conv_stats(self.conv2, out)
        out = self.bn2(y, stats=st)
        y, st = conv_stats(self.conv3, out)
        return self.bn3(y, identity, stats=st)


class ConvBN(nn.Sequential):
    """``Sequential(conv, BNAct)`` (state_dict keys ``0.*``, ``1.*`` as
    torchvision's downsample) passing the conv's fused BN statistics on."""

    def forward(self, x):
        y, st = conv_stats(self[0], x)
        return self[1](y, stats=st)

    def forward_deferred(self, x, consumer: BNAct):
        """The shortcut with its BN apply deferred into ``consumer`` (the block's
        last BN, which adds it as its residual): the pending handle of
        ``BNAct.deferred``, or the plain output when either BN is not fused."""
        y, st = conv_stats(self[0], x)
        if consumer.fused_ok(y):
            h = self[1].deferred(y, stats=st)
            if h is not None:
                return h
        return self[1](y, stats=st)


def _shortcut(ds: nn.Module, xs: torch.Tensor, consumer: BNAct) -> torch.Tensor:
    if isinstance(ds, ConvBN):
        return ds.forward_deferred(xs, consumer)
    return ds(xs)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False, groups: int = 1, width_per_group: int = 64,
                 name: Optional[str] = None):
        super().__init__()
        self.inplanes = 64
        self.groups = groups
        self.base_width = width_per_group
        # nn.Conv2d(3, 64, 7, 2, 3, bias=False) running the gfx950 stem kernels (ops/stem.py)
        self.conv1 = StemConv(3, 64)
        # stem BN + ReLU + 3x3/s2 max-pool run as one fused kernel pass (BNAct pool=...);
        # ``maxpool`` stays as an attribute (no parameters) for module-path compatibility.
        self.bn1 = BNAct(64, act="relu", pool=(3, 2, 1))
        self.maxpool = nn.Identity()
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        self.name = name or "resnet"
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # includes BNAct
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        # Every block output except the last feeds the next block twice (conv1 and
        # shortcut): let the producing BN hand out two handles so the backward
        # sums the two gradients inside the fused BN passes (no add kernel).
        blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
        self.bn1.twin = True
        for b in blocks[:-1]:
            (b.bn3 if isinstance(b, Bottleneck) else b.bn2).twin = True
        # Backward fusion (ops/bn.py BnLink): a BN whose output has exactly one
        # convolution consumer lets that conv's grad-input GEMM produce the
        # ReLU-masked gradient and the BN's reduction partials.  Inside a block
        # that is bn1 -> conv2 (and bn2 -> conv3); a block output feeds the next
        # block's conv1 and, through the shortcut, the next block's last BN, which
        # hands its residual gradient over -- not a downsample conv, whose
        # gradient would only arrive after conv1's backward.
        for i, b in enumerate(blocks):
            b.bn1.bwd_link = True
            if isinstance(b, Bottleneck):
                b.bn2.bwd_link = True
            if i + 1 < len(blocks) and blocks[i + 1].downsample is None:
                (b.bn3 if isinstance(b, Bottleneck) else b.bn2).bwd_link = True
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = ConvBN(conv1x1(self.inplanes, planes * block.expansion, stride),
                                BNAct(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width))
        return nn.Sequential(*layers)

    def forward(self, x):
        y, st = conv_stats(self.conv1, x)   # BN statistics from the stem kernel's epilogue
        x = self.maxpool(self.bn1(y, stats=st))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(global_avg_pool(x))   # == flatten(avgpool(x)), channels-last backward


def resnet18(num_classes=1000, **kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, name="resnet18", **kw)


def resnet34(num_classes=1000, **kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, name="resnet34", **kw)


def resnet50(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, name="resnet50", **kw)


def resnet101(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, name="resnet101", **kw)


def resnet152(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, name="resnet152", **kw)


def resnext50_32x4d(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, groups=32, width_per_group=4, name="resnext50", **kw)
