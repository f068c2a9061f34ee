"""Remaining zoo members of the reference (registered into ``create_net``).

Parity (reference files): AlexNet with LRN (models/alexnet.py), GoogLeNet
without aux heads (models/googlenet.py), Inception-v4 (models/inceptionv4.py),
Inception-v3 (torchvision in dl_trainer.py:93-96), DenseNet-100-12 for CIFAR
(models/densenet.py), CIFAR ResNeXt-29 (models/resnext.py), CaffeNet-CIFAR
(models/caffe_cifar.py), ResNet-mod (models/resnet_mod.py: CIFAR ResNet whose
forward also returns the pooled features) and the AN4 DeepSpeech network
(models/lstman4.py + lstm_models.py: 2 conv + 5 x LSTM-800 + lookahead).
Independent implementations, written against the architectures, not the files.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import register
from .resnet_cifar import CifarResNet


# ----------------------------------------------------------------------------
# AlexNet (LRN)
# ----------------------------------------------------------------------------
class LRN(nn.Module):
    """Local response normalisation across channels: x / (1 + alpha*avg(x^2))^beta."""

    def __init__(self, local_size=5, alpha=1e-4, beta=0.75):
        super().__init__()
        self.size, self.alpha, self.beta = local_size, alpha, beta

    def forward(self, x):
        div = F.avg_pool3d(x.pow(2).unsqueeze(1), (self.size, 1, 1), stride=1,
                           padding=((self.size - 1) // 2, 0, 0)).squeeze(1)
        return x / div.mul(self.alpha).add(1.0).pow(self.beta)


class AlexNet(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 96, 11, stride=4), nn.ReLU(inplace=True), LRN(5, 1e-4, 0.75), nn.MaxPool2d(3, 2),
            nn.Conv2d(96, 256, 5, padding=2, groups=2), nn.ReLU(inplace=True), LRN(5, 1e-4, 0.75),
            nn.MaxPool2d(3, 2),
            nn.Conv2d(256, 384, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 384, 3, padding=1, groups=2), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, 3, padding=1, groups=2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2))
        self.classifier = nn.Sequential(
            nn.Linear(256 * 6 * 6, 4096), nn.ReLU(inplace=True), nn.Dropout(),
            nn.Linear(4096, 4096), nn.ReLU(inplace=True), nn.Dropout(), nn.Linear(4096, num_classes))
        self.name = "alexnet"

    def forward(self, x):
        x = F.adaptive_avg_pool2d(self.features(x), (6, 6))
        return self.classifier(x.reshape(x.shape[0], 256 * 6 * 6))


# ----------------------------------------------------------------------------
# GoogLeNet / Inception building blocks
# ----------------------------------------------------------------------------
class BasicConv2d(nn.Module):
    def __init__(self, inp, out, eps=1e-3, **kw):
        super().__init__()
        self.conv = nn.Conv2d(inp, out, bias=False, **kw)
        self.bn = nn.BatchNorm2d(out, eps=eps)

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)), inplace=True)


class InceptionV1Block(nn.Module):
    def __init__(self, inp, c1, c3r, c3, c5r, c5, pool):
        super().__init__()
        self.branch1 = BasicConv2d(inp, c1, kernel_size=1)
        self.branch2 = nn.Sequential(BasicConv2d(inp, c3r, kernel_size=1), BasicConv2d(c3r, c3, kernel_size=3,
                                                                                         padding=1))
        self.branch3 = nn.Sequential(BasicConv2d(inp, c5r, kernel_size=1), BasicConv2d(c5r, c5, kernel_size=3,
                                                                                         padding=1))
        self.branch4 = nn.Sequential(nn.MaxPool2d(3, stride=1, padding=1, ceil_mode=True),
                                     BasicConv2d(inp, pool, kernel_size=1))

    def forward(self, x):
        return torch.cat([self.branch1(x), self.branch2(x), self.branch3(x), self.branch4(x)], 1)


class GoogLeNet(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1 = BasicConv2d(3, 64, kernel_size=7, stride=2, padding=3)
        self.maxpool1 = nn.MaxPool2d(3, stride=2, ceil_mode=True)
        self.conv2 = BasicConv2d(64, 64, kernel_size=1)
        self.conv3 = BasicConv2d(64, 192, kernel_size=3, padding=1)
        self.maxpool2 = nn.MaxPool2d(3, stride=2, ceil_mode=True)
        self.inception3a = InceptionV1Block(192, 64, 96, 128, 16, 32, 32)
        self.inception3b = InceptionV1Block(256, 128, 128, 192, 32, 96, 64)
        self.maxpool3 = nn.MaxPool2d(3, stride=2, ceil_mode=True)
        self.inception4a = InceptionV1Block(480, 192, 96, 208, 16, 48, 64)
        self.inception4b = InceptionV1Block(512, 160, 112, 224, 24, 64, 64)
        self.inception4c = InceptionV1Block(512, 128, 128, 256, 24, 64, 64)
        self.inception4d = InceptionV1Block(512, 112, 144, 288, 32, 64, 64)
        self.inception4e = InceptionV1Block(528, 256, 160, 320, 32, 128, 128)
        self.maxpool4 = nn.MaxPool2d(2, stride=2, ceil_mode=True)
        self.inception5a = InceptionV1Block(832, 256, 160, 320, 32, 128, 128)
        self.inception5b = InceptionV1Block(832, 384, 192, 384, 48, 128, 128)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.dropout = nn.Dropout(0.2)
        self.fc = nn.Linear(1024, num_classes)
        self.name = "googlenet"

    def forward(self, x):
        x = self.maxpool1(self.conv1(x))
        x = self.maxpool2(self.conv3(self.conv2(x)))
        x = self.maxpool3(self.inception3b(self.inception3a(x)))
        x = self.inception4e(self.inception4d(self.inception4c(self.inception4b(self.inception4a(x)))))
        x = self.inception5b(self.inception5a(self.maxpool4(x)))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(self.dropout(x))


# ---- Inception-v4 ----------------------------------------------------------
def _bc(i, o, k, s=1, p=0):
    return BasicConv2d(i, o, kernel_size=k, stride=s, padding=p)


class _Cat(nn.Module):
    def __init__(self, *branches):
        super().__init__()
        self.branches = nn.ModuleList(branches)

    def forward(self, x):
        return torch.cat([b(x) for b in self.branches], 1)


class InceptionV4(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        seq = nn.Sequential
        stem = [_bc(3, 32, 3, 2), _bc(32, 32, 3), _bc(32, 64, 3, 1, 1),
                _Cat(nn.MaxPool2d(3, 2), _bc(64, 96, 3, 2)),
                _Cat(seq(_bc(160, 64, 1), _bc(64, 96, 3)),
                     seq(_bc(160, 64, 1), _bc(64, 64, (1, 7), 1, (0, 3)), _bc(64, 64, (7, 1), 1, (3, 0)),
                         _bc(64, 96, 3))),
                _Cat(_bc(192, 192, 3, 2), nn.MaxPool2d(3, 2))]
        blocks = []
        for _ in range(4):
            blocks.append(_Cat(_bc(384, 96, 1), seq(_bc(384, 64, 1), _bc(64, 96, 3, 1, 1)),
                               seq(_bc(384, 64, 1), _bc(64, 96, 3, 1, 1), _bc(96, 96, 3, 1, 1)),
                               seq(nn.AvgPool2d(3, 1, 1, count_include_pad=False), _bc(384, 96, 1))))
        blocks.append(_Cat(_bc(384, 384, 3, 2), seq(_bc(384, 192, 1), _bc(192, 224, 3, 1, 1), _bc(224, 256, 3, 2)),
                           nn.MaxPool2d(3, 2)))
        for _ in range(7):
            blocks.append(_Cat(_bc(1024, 384, 1),
                               seq(_bc(1024, 192, 1), _bc(192, 224, (1, 7), 1, (0, 3)), _bc(224, 256, (7, 1), 1, (3, 0))),
                               seq(_bc(1024, 192, 1), _bc(192, 192, (7, 1), 1, (3, 0)), _bc(192, 224, (1, 7), 1, (0, 3)),
                                   _bc(224, 224, (7, 1), 1, (3, 0)), _bc(224, 256, (1, 7), 1, (0, 3))),
                               seq(nn.AvgPool2d(3, 1, 1, count_include_pad=False), _bc(1024, 128, 1))))
        blocks.append(_Cat(seq(_bc(1024, 192, 1), _bc(192, 192, 3, 2)),
                           seq(_bc(1024, 256, 1), _bc(256, 256, (1, 7), 1, (0, 3)), _bc(256, 320, (7, 1), 1, (3, 0)),
                               _bc(320, 320, 3, 2)),
                           nn.MaxPool2d(3, 2)))
        for _ in range(3):
            blocks.append(InceptionC())
        self.features = nn.Sequential(*stem, *blocks)
        self.last_linear = nn.Linear(1536, num_classes)
        self.name = "inceptionv4"

    def forward(self, x):
        x = self.features(x)
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.last_linear(x)


class InceptionC(nn.Module):
    def __init__(self):
        super().__init__()
        self.b0 = _bc(1536, 256, 1)
        self.b1_0 = _bc(1536, 384, 1)
        self.b1_1a = _bc(384, 256, (1, 3), 1, (0, 1))
        self.b1_1b = _bc(384, 256, (3, 1), 1, (1, 0))
        self.b2_0 = _bc(1536, 384, 1)
        self.b2_1 = _bc(384, 448, (3, 1), 1, (1, 0))
        self.b2_2 = _bc(448, 512, (1, 3), 1, (0, 1))
        self.b2_3a = _bc(512, 256, (1, 3), 1, (0, 1))
        self.b2_3b = _bc(512, 256, (3, 1), 1, (1, 0))
        self.b3 = nn.Sequential(nn.AvgPool2d(3, 1, 1, count_include_pad=False), _bc(1536, 256, 1))

    def forward(self, x):
        x1 = self.b1_0(x)
        x2 = self.b2_2(self.b2_1(self.b2_0(x)))
        return torch.cat([self.b0(x), self.b1_1a(x1), self.b1_1b(x1), self.b2_3a(x2), self.b2_3b(x2), self.b3(x)], 1)


# ---- Inception-v3 (torchvision layout, no aux head) -------------------------
class _IncA(nn.Module):
    def __init__(self, c, pool):
        super().__init__()
        self.b1 = _bc(c, 64, 1)
        self.b5 = nn.Sequential(_bc(c, 48, 1), _bc(48, 64, 5, 1, 2))
        self.b3 = nn.Sequential(_bc(c, 64, 1), _bc(64, 96, 3, 1, 1), _bc(96, 96, 3, 1, 1))
        self.bp = _bc(c, pool, 1)

    def forward(self, x):
        return torch.cat([self.b1(x), self.b5(x), self.b3(x), self.bp(F.avg_pool2d(x, 3, 1, 1))], 1)


class _IncB(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.b3 = _bc(c, 384, 3, 2)
        self.bd = nn.Sequential(_bc(c, 64, 1), _bc(64, 96, 3, 1, 1), _bc(96, 96, 3, 2))

    def forward(self, x):
        return torch.cat([self.b3(x), self.bd(x), F.max_pool2d(x, 3, 2)], 1)


class _IncC(nn.Module):
    def __init__(self, c, c7):
        super().__init__()
        self.b1 = _bc(c, 192, 1)
        self.b7 = nn.Sequential(_bc(c, c7, 1), _bc(c7, c7, (1, 7), 1, (0, 3)), _bc(c7, 192, (7, 1), 1, (3, 0)))
        self.bd = nn.Sequential(_bc(c, c7, 1), _bc(c7, c7, (7, 1), 1, (3, 0)), _bc(c7, c7, (1, 7), 1, (0, 3)),
                                _bc(c7, c7, (7, 1), 1, (3, 0)), _bc(c7, 192, (1, 7), 1, (0, 3)))
        self.bp = _bc(c, 192, 1)

    def forward(self, x):
        return torch.cat([self.b1(x), self.b7(x), self.bd(x), self.bp(F.avg_pool2d(x, 3, 1, 1))], 1)


class _IncD(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.b3 = nn.Sequential(_bc(c, 192, 1), _bc(192, 320, 3, 2))
        self.b7 = nn.Sequential(_bc(c, 192, 1), _bc(192, 192, (1, 7), 1, (0, 3)), _bc(192, 192, (7, 1), 1, (3, 0)),
                                _bc(192, 192, 3, 2))

    def forward(self, x):
        return torch.cat([self.b3(x), self.b7(x), F.max_pool2d(x, 3, 2)], 1)


class _IncE(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.b1 = _bc(c, 320, 1)
        self.b3 = _bc(c, 384, 1)
        self.b3a = _bc(384, 384, (1, 3), 1, (0, 1))
        self.b3b = _bc(384, 384, (3, 1), 1, (1, 0))
        self.bd1 = _bc(c, 448, 1)
        self.bd2 = _bc(448, 384, 3, 1, 1)
        self.bd3a = _bc(384, 384, (1, 3), 1, (0, 1))
        self.bd3b = _bc(384, 384, (3, 1), 1, (1, 0))
        self.bp = _bc(c, 192, 1)

    def forward(self, x):
        b3 = self.b3(x)
        bd = self.bd2(self.bd1(x))
        return torch.cat([self.b1(x), self.b3a(b3), self.b3b(b3), self.bd3a(bd), self.bd3b(bd),
                          self.bp(F.avg_pool2d(x, 3, 1, 1))], 1)


class InceptionV3(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(_bc(3, 32, 3, 2), _bc(32, 32, 3), _bc(32, 64, 3, 1, 1), nn.MaxPool2d(3, 2),
                                  _bc(64, 80, 1), _bc(80, 192, 3), nn.MaxPool2d(3, 2))
        self.blocks = nn.Sequential(_IncA(192, 32), _IncA(256, 64), _IncA(288, 64), _IncB(288),
                                    _IncC(768, 128), _IncC(768, 160), _IncC(768, 160), _IncC(768, 192),
                                    _IncD(768), _IncE(1280), _IncE(2048))
        self.dropout = nn.Dropout(0.5)
        self.fc = nn.Linear(2048, num_classes)
        self.name = "inceptionv3"

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return self.fc(self.dropout(F.adaptive_avg_pool2d(x, 1).flatten(1)))


# ----------------------------------------------------------------------------
# CIFAR DenseNet / ResNeXt / CaffeNet / ResNet-mod
# ----------------------------------------------------------------------------
class _DenseLayer(nn.Module):
    def __init__(self, c, growth, bottleneck):
        super().__init__()
        self.bottleneck = bottleneck
        self.bn1 = nn.BatchNorm2d(c)
        if bottleneck:
            self.conv1 = nn.Conv2d(c, 4 * growth, 1, bias=False)
            self.bn2 = nn.BatchNorm2d(4 * growth)
            self.conv2 = nn.Conv2d(4 * growth, growth, 3, padding=1, bias=False)
        else:
            self.conv1 = nn.Conv2d(c, growth, 3, padding=1, bias=False)

    def forward(self, x):
        out = self.conv1(F.relu(self.bn1(x)))
        if self.bottleneck:
            out = self.conv2(F.relu(self.bn2(out)))
        return torch.cat((x, out), 1)


class _Transition(nn.Module):
    def __init__(self, c, o):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(c)
        self.conv1 = nn.Conv2d(c, o, 1, bias=False)

    def forward(self, x):
        return F.avg_pool2d(self.conv1(F.relu(self.bn1(x))), 2)


class DenseNet(nn.Module):
    def __init__(self, growth=12, depth=100, reduction=0.5, num_classes=10, bottleneck=False):
        super().__init__()
        n = (depth - 4) // (6 if bottleneck else 3)
        c = 2 * growth
        self.conv1 = nn.Conv2d(3, c, 3, padding=1, bias=False)
        stages = []
        for s in range(3):
            layers = []
            for _ in range(n):
                layers.append(_DenseLayer(c, growth, bottleneck))
                c += growth
            stages.append(nn.Sequential(*layers))
            if s < 2:
                o = int(math.floor(c * reduction))
                stages.append(_Transition(c, o))
                c = o
        self.blocks = nn.Sequential(*stages)
        self.bn1 = nn.BatchNorm2d(c)
        self.fc = nn.Linear(c, num_classes)
        self.name = "densenet%d" % depth
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / fan))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.bias.data.zero_()

    def forward(self, x):
        out = self.blocks(self.conv1(x))
        out = F.adaptive_avg_pool2d(F.relu(self.bn1(out)), 1).flatten(1)
        return F.log_softmax(self.fc(out), dim=1)


class _ResNeXtBlock(nn.Module):
    def __init__(self, inp, planes, card, base_width, stride, downsample):
        super().__init__()
        D = int(math.floor(planes * (base_width / 64.0)))
        self.conv_reduce = nn.Conv2d(inp, D * card, 1, bias=False)
        self.bn_reduce = nn.BatchNorm2d(D * card)
        self.conv_conv = nn.Conv2d(D * card, D * card, 3, stride=stride, padding=1, groups=card, bias=False)
        self.bn = nn.BatchNorm2d(D * card)
        self.conv_expand = nn.Conv2d(D * card, planes * 4, 1, bias=False)
        self.bn_expand = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample

    def forward(self, x):
        r = x if self.downsample is None else self.downsample(x)
        b = F.relu(self.bn_reduce(self.conv_reduce(x)), inplace=True)
        b = F.relu(self.bn(self.conv_conv(b)), inplace=True)
        b = self.bn_expand(self.conv_expand(b))
        return F.relu(r + b, inplace=True)


class CifarResNeXt(nn.Module):
    def __init__(self, depth=29, cardinality=8, base_width=64, num_classes=10):
        super().__init__()
        assert (depth - 2) % 9 == 0
        n = (depth - 2) // 9
        self.conv_1_3x3 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn_1 = nn.BatchNorm2d(64)
        self.inplanes = 64
        self.stage_1 = self._stage(64, n, 1, cardinality, base_width)
        self.stage_2 = self._stage(128, n, 2, cardinality, base_width)
        self.stage_3 = self._stage(256, n, 2, cardinality, base_width)
        self.classifier = nn.Linear(1024, num_classes)
        self.name = "resnext%d_%d_%d" % (depth, cardinality, base_width)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / fan))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                nn.init.kaiming_normal_(m.weight)
                m.bias.data.zero_()

    def _stage(self, planes, blocks, stride, card, bw):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes * 4))
        layers = [_ResNeXtBlock(self.inplanes, planes, card, bw, stride, down)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(_ResNeXtBlock(self.inplanes, planes, card, bw, 1, None))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = F.relu(self.bn_1(self.conv_1_3x3(x)), inplace=True)
        x = self.stage_3(self.stage_2(self.stage_1(x)))
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.classifier(x)


class CifarCaffeNet(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.block_1 = nn.Sequential(nn.Conv2d(3, 32, 3, 1, 1), nn.MaxPool2d(3, 2), nn.ReLU(), nn.BatchNorm2d(32))
        self.block_2 = nn.Sequential(nn.Conv2d(32, 32, 3, 1, 1), nn.Conv2d(32, 64, 3, 1, 1), nn.ReLU(),
                                     nn.AvgPool2d(3, 2), nn.BatchNorm2d(64))
        self.block_3 = nn.Sequential(nn.Conv2d(64, 64, 3, 1, 1), nn.Conv2d(64, 128, 3, 1, 1), nn.ReLU(),
                                     nn.AvgPool2d(3, 2), nn.BatchNorm2d(128))
        self.classifier = nn.Linear(128 * 9, num_classes)
        self.name = "caffe_cifar"

    def forward(self, x):
        x = self.block_3(self.block_2(self.block_1(x)))
        return self.classifier(x.reshape(x.shape[0], -1))


class ResNetMod(CifarResNet):
    """CIFAR ResNet that also returns the pooled features (reference resnet_mod.py)."""

    def forward(self, x):
        x = F.relu(self.bn_1(self.conv_1_3x3(x)), inplace=True)
        x = self.stage_3(self.stage_2(self.stage_1(x)))
        feat = self.avgpool(x).reshape(x.shape[0], -1)
        return self.classifier(feat), feat


# ----------------------------------------------------------------------------
# DeepSpeech (AN4): 2 conv + 5 x LSTM + lookahead + linear, CTC
# ----------------------------------------------------------------------------
class _BatchRNN(nn.Module):
    def __init__(self, inp, hidden, batch_norm=True):
        super().__init__()
        self.bn = nn.BatchNorm1d(inp) if batch_norm else None
        self.rnn = nn.LSTM(inp, hidden, bias=True)

    def forward(self, x):  # x: T x N x H
        if self.bn is not None:
            T, N, H = x.shape
            x = self.bn(x.reshape(T * N, H)).reshape(T, N, H)
        return self.rnn(x)[0]


class Lookahead(nn.Module):
    def __init__(self, n_features, context):
        super().__init__()
        self.context = context
        self.conv = nn.Conv1d(n_features, n_features, kernel_size=context + 1, groups=n_features, bias=False)

    def forward(self, x):  # T x N x H
        x = x.permute(1, 2, 0)
        x = F.pad(x, (0, self.context))
        return self.conv(x).permute(2, 0, 1)


class DeepSpeech(nn.Module):
    def __init__(self, num_classes=29, hidden=800, layers=5, sample_rate=16000, window_size=0.02, context=20):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(1, 32, kernel_size=(41, 11), stride=(2, 2), padding=(20, 5)), nn.BatchNorm2d(32),
            nn.Hardtanh(0, 20, inplace=True),
            nn.Conv2d(32, 32, kernel_size=(21, 11), stride=(2, 1), padding=(10, 5)), nn.BatchNorm2d(32),
            nn.Hardtanh(0, 20, inplace=True))
        freq = int(math.floor(sample_rate * window_size / 2) + 1)
        freq = int(math.floor(freq + 2 * 20 - 41) / 2 + 1)
        freq = int(math.floor(freq + 2 * 10 - 21) / 2 + 1)
        rnn_in = freq * 32
        rnns = [_BatchRNN(rnn_in, hidden, batch_norm=False)]
        for _ in range(layers - 1):
            rnns.append(_BatchRNN(hidden, hidden))
        self.rnns = nn.Sequential(*rnns)
        self.lookahead = nn.Sequential(Lookahead(hidden, context), nn.Hardtanh(0, 20, inplace=True))
        self.fc = nn.Sequential(nn.BatchNorm1d(hidden), nn.Linear(hidden, num_classes, bias=False))
        self.name = "lstman4"
        self.freq_bins = int(math.floor(sample_rate * window_size / 2) + 1)

    def forward(self, x, lengths=None):  # x: N x 1 x F x T
        x = self.conv(x)
        N, C, Fq, T = x.shape
        x = x.reshape(N, C * Fq, T).permute(2, 0, 1).contiguous()  # T x N x H
        x = self.lookahead(self.rnns(x))
        T, N, H = x.shape
        out = self.fc(x.reshape(T * N, H)).reshape(T, N, -1)
        out_lengths = None
        if lengths is not None:
            out_lengths = torch.div(lengths + 1, 2, rounding_mode="floor")
        return out.transpose(0, 1), out_lengths  # N x T x classes


register("alexnet", lambda nc, **kw: AlexNet(nc), "imagenet")
register("googlenet", lambda nc, **kw: GoogLeNet(nc), "imagenet")
register("inceptionv4", lambda nc, **kw: InceptionV4(nc), "imagenet")
register("inceptionv3", lambda nc, **kw: InceptionV3(nc), "imagenet")
register("densenet100", lambda nc, **kw: DenseNet(12, 100, 0.5, nc, False), "cifar10")
register("resnext29", lambda nc, **kw: CifarResNeXt(29, 8, 64, nc), "cifar10")
register("resnext29_16", lambda nc, **kw: CifarResNeXt(29, 16, 64, nc), "cifar10")
register("caffe_cifar", lambda nc, **kw: CifarCaffeNet(nc), "cifar10")
register("resnet_mod20", lambda nc, **kw: ResNetMod(20, nc), "cifar10")
register("lstman4", lambda nc, **kw: DeepSpeech(29), "an4")
