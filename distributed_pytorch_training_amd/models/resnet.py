"""ResNet-18 / ResNet-50 with torchvision-identical architecture, parameter names and init.

The reference builds its model with ``torchvision.models.resnet18(num_classes=10)``
(reference ``train_ddp.py:153-156``).  torchvision is not part of this stack, so the
network lives here.  Parameter/buffer names (``conv1.weight``, ``layer1.0.bn1.running_mean``,
``fc.weight`` ...) and counts match torchvision exactly (ResNet-18/10 classes:
11,181,642 params; ResNet-50/1000 classes: 25,557,032), so checkpoints written by
``utils/checkpoint.py`` are interchangeable with torchvision state dicts.

MI355X notes
------------
* The stem is the ImageNet stem (7x7/2 conv + 3x3/2 max-pool) even for 32x32 CIFAR input,
  because that is what the reference trains.
* ``memory_format=torch.channels_last`` is applied by the trainer, not here: MIOpen's NHWC
  bf16 convolutions are the fast path on gfx950 and the choice is a runtime flag.
* BN -> (+identity) -> ReLU goes through ``layers.bn_act``: the torchvision composition
  (in-place add and ReLU) with stock ``nn.BatchNorm2d``, or one fused gfx950 kernel chain
  once ``layers.fuse_batchnorm`` has installed ``FusedBatchNorm2d`` (the native engine
  does this for channels_last GPU runs).
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from .layers import bn_act, bn_act_block_out, bn_relu_maxpool, downsample_branch, split_block_input


def _conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def _conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, width: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.conv1 = _conv3x3(cin, width, stride)
        self.bn1 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(width, width)
        self.bn2 = nn.BatchNorm2d(width)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        xc, xi = split_block_input(x)
        out = bn_act(self.bn1, self.conv1(xc))
        # downsample after conv1 (same values): autograd then runs its backward before conv1's,
        # so conv1's backward-data sees the whole identity-path gradient (ops/bn.py block tails)
        identity = xi if self.downsample is None else downsample_branch(self.downsample, xi, self.bn2)
        return bn_act_block_out(self.bn2, self.conv2(out), identity)


class Bottleneck(nn.Module):
    """ResNet v1.5 bottleneck: the stride sits on the 3x3 conv (torchvision layout)."""

    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.conv1 = _conv1x1(cin, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv1x1(width, width * self.expansion)
        self.bn3 = nn.BatchNorm2d(width * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        xc, xi = split_block_input(x)
        out = bn_act(self.bn1, self.conv1(xc))
        # downsample after conv1 (same values): autograd then runs its backward before conv1's,
        # so conv1's backward-data sees the whole identity-path gradient (ops/bn.py block tails)
        identity = xi if self.downsample is None else downsample_branch(self.downsample, xi, self.bn3)
        out = bn_act(self.bn2, self.conv2(out))
        return bn_act_block_out(self.bn3, self.conv3(out), identity)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int],
                 num_classes: int = 1000, zero_init_residual: bool = False) -> None:
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)

        # torchvision init: Kaiming-normal(fan_out) convs, BN gamma=1 / beta=0,
        # Linear keeps PyTorch's default (kaiming-uniform a=sqrt(5)).
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, width: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != width * block.expansion:
            downsample = nn.Sequential(
                _conv1x1(self.inplanes, width * block.expansion, stride),
                nn.BatchNorm2d(width * block.expansion),
            )
        layers = [block(self.inplanes, width, stride, downsample)]
        self.inplanes = width * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, width))
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = bn_relu_maxpool(self.bn1, self.maxpool, self.conv1(x))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if isinstance(x, tuple):  # fused block tails hand (conv-path, identity-path) aliases along
            x = x[0]
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes=num_classes, **kw)
