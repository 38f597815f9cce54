"""Normalisation + activation building block shared by the model zoo.

``bn_act(bn, x, relu, residual)`` computes ``relu(bn(x) + residual)``.  With a stock
``nn.BatchNorm2d`` it runs the unfused torchvision composition (BN, in-place add, in-place
ReLU).  With a ``FusedBatchNorm2d`` (installed by ``fuse_batchnorm``) and a channels_last
GPU activation it runs ONE fused gfx950 kernel chain (ops/bn.py) instead of three HBM
passes through MIOpen/ATen.  ``FusedBatchNorm2d`` subclasses ``nn.BatchNorm2d`` and keeps
its parameters and buffers, so state_dict keys, DDP buffer broadcast and checkpoints are
unchanged.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import bn as fused_bn


class FusedBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` that can also run fused with ReLU / residual add on gfx950."""

    def can_fuse(self, x: torch.Tensor) -> bool:
        if not (self.affine and self.track_running_stats and self.momentum is not None):
            return False
        if not self.training and torch.is_grad_enabled() and x.requires_grad:
            return False
        return fused_bn.bn_act_supported(x, self.num_features)

    def act(self, x: torch.Tensor, relu: bool, residual: Optional[torch.Tensor], pair: bool = False):
        if self.training:
            return fused_bn.bn_act_train(x, residual, self.weight, self.bias, self.running_mean,
                                         self.running_var, self.num_batches_tracked, self.momentum,
                                         self.eps, relu, pair)
        y = fused_bn.bn_act_eval(x, residual, self.weight, self.bias, self.running_mean,
                                 self.running_var, self.eps, relu)
        return (y, y) if pair else y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.can_fuse(x):
            return self.act(x, False, None)
        return super().forward(x)


def bn_act(bn: nn.Module, x: torch.Tensor, relu: bool = True,
           residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    if isinstance(bn, FusedBatchNorm2d) and bn.can_fuse(x):
        return bn.act(x, relu, residual)
    out = bn(x)
    if residual is not None:
        out += residual
    return F.relu(out, inplace=True) if relu else out


def bn_act_block_out(bn: nn.Module, x: torch.Tensor, residual: torch.Tensor):
    """Residual-block tail ``relu(bn(x) + residual)``.

    With a fused BN it returns ``(y_conv, y_identity)``: two aliases of the output whose
    gradients reach the fused backward separately (see ops/bn.py ``_BNActTrainPair``); the
    next block feeds the first to its conv path and the second to its identity path.
    Otherwise it returns the plain tensor.
    """
    if isinstance(bn, FusedBatchNorm2d) and bn.can_fuse(x):
        return bn.act(x, True, residual, pair=True)
    return bn_act(bn, x, True, residual)


def split_block_input(x):
    """(conv-path input, identity-path input) of a residual block."""
    return x if isinstance(x, tuple) else (x, x)


def fuse_batchnorm(model: nn.Module) -> int:
    """Swap every ``nn.BatchNorm2d`` for a ``FusedBatchNorm2d`` sharing its tensors."""
    n = 0
    for parent in model.modules():
        for name, child in list(parent.named_children()):
            if type(child) is nn.BatchNorm2d:
                new = FusedBatchNorm2d.__new__(FusedBatchNorm2d)
                new.__dict__ = child.__dict__  # same Parameters / buffers / hooks / flags
                setattr(parent, name, new)
                n += 1
    return n
