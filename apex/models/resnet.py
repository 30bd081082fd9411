"""ResNet-50 (and 18/34/101/152) from scratch — BASELINE.json config 2 ("ResNet-50 amp O2 bf16 +
FusedSGD + SyncBatchNorm") and the model of the reference's ImageNet examples
(examples/imagenet/main.py:114-119 took it from torchvision, which is not installed here).

Convolutions run on MIOpen through PyTorch (library GEMM-class work); BatchNorm can be
swapped for apex.parallel.SyncBatchNorm with ``convert_syncbn_model`` (HIP Welford
kernels + one RCCL all-gather per layer); ``fuse_bn_relu`` then folds the ReLUs and each block's
residual add into the SyncBatchNorm kernels. ``channels_last`` keeps activations NHWC,
the layout MIOpen's fastest bf16 kernels use.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _bn_relu(bn, x, z=None):
    """relu(bn(x) (+ z)) — one fused HIP kernel each way when ``bn`` is an apex SyncBatchNorm with
    ``fuse_relu`` set (``fuse_bn_relu``), else BatchNorm, add and ReLU as separate ops."""
    if getattr(bn, "fuse_relu", False):
        return bn(x, z) if z is not None else bn(x)
    y = bn(x)
    if z is not None:
        y = y + z
    return F.relu(y, inplace=True)


def conv3x3(i, o, stride=1, groups=1, dilation=1):
    return nn.Conv2d(i, o, 3, stride=stride, padding=dilation, groups=groups, bias=False, dilation=dilation)


def conv1x1(i, o, stride=1):
    return nn.Conv2d(i, o, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = _bn_relu(self.bn1, self.conv1(x))
        return _bn_relu(self.bn2, self.conv2(out), idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * 4)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = _bn_relu(self.bn1, self.conv1(x))
        out = _bn_relu(self.bn2, self.conv2(out))
        return _bn_relu(self.bn3, self.conv3(out), idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, zero_init_residual=True):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.modules.batchnorm._BatchNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                 nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(_bn_relu(self.bn1, self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def fuse_bn_relu(model):
    """Set ``fuse_relu`` on every apex SyncBatchNorm that a ReLU follows (the stem, each block's
    inner norms and its output norm, whose residual add is fused too — not the downsample norms):
    BN + add + ReLU become one HIP kernel each way. Run after ``convert_syncbn_model``."""
    from ..parallel.sync_batchnorm import SyncBatchNorm

    bns = [model.bn1] if hasattr(model, "bn1") else []
    for m in model.modules():
        if isinstance(m, (BasicBlock, Bottleneck)):
            bns += [m.bn1, m.bn2] + ([m.bn3] if isinstance(m, Bottleneck) else [])
    for bn in bns:
        if isinstance(bn, SyncBatchNorm):
            bn.fuse_relu = True
    return model


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)


def synthetic_batch(batch, image_size=224, num_classes=1000, device="cpu", dtype=torch.float32,
                    channels_last=False, generator=None):
    x = torch.randn(batch, 3, image_size, image_size, device=device, dtype=dtype, generator=generator)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, num_classes, (batch,), device=device, generator=generator)
    return x, y
