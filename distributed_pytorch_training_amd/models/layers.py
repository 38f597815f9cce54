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

import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import bn as fused_bn
from ..ops.conv_f32 import NativeConv2d
from ..ops import pool as fused_pool


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


class DeferredBN:
    """A downsample branch whose BatchNorm is not applied yet: ``bn(x)`` is folded into the block
    tail by ``bn_act_block_out`` (ops/bn.py ``_BN2AddReLUPair``) and never materialised."""

    __slots__ = ("bn", "x")

    def __init__(self, bn: nn.Module, x: torch.Tensor) -> None:
        self.bn, self.x = bn, x

    def materialize(self) -> torch.Tensor:
        return self.bn(self.x)


# 0 disables folding the downsample BatchNorm into the block tail (A/B)
DS_FUSE = os.environ.get("DPT_DS_FUSE", "1") != "0"


def downsample_branch(ds: nn.Module, x: torch.Tensor, tail_bn: nn.Module):
    """``ds(x)`` for a (conv, BatchNorm) downsample; a ``DeferredBN`` when the block tail can
    apply that BatchNorm itself (both fused BNs, training)."""
    if (DS_FUSE and isinstance(ds, nn.Sequential) and len(ds) == 2 and isinstance(ds[1], FusedBatchNorm2d)
            and isinstance(tail_bn, FusedBatchNorm2d) and ds[1].training and tail_bn.training
            and torch.is_grad_enabled()):
        h = ds[0](x)
        return DeferredBN(ds[1], h) if ds[1].can_fuse(h) else ds[1](h)
    return ds(x)


def bn_act_block_out(bn: nn.Module, x: torch.Tensor, residual):
    """Residual-block tail ``relu(bn(x) + residual)``.

    With a fused BN it returns ``(y_conv, y_identity)``: two aliases of the output whose
    gradients reach the fused backward separately (see ops/bn.py ``_BNActTrainPair``); the
    next block feeds the first to its conv path and the second to its identity path.
    Otherwise it returns the plain tensor.  ``residual`` may be a ``DeferredBN`` (downsample
    branch): both BatchNorms then run as one fused op.
    """
    if isinstance(residual, DeferredBN):
        if (isinstance(bn, FusedBatchNorm2d) and bn.can_fuse(x) and bn.training
                and residual.x.shape == x.shape and residual.x.dtype == x.dtype):
            return fused_bn.bn2_add_relu_train(x, bn, residual.x, residual.bn)
        residual = residual.materialize()
    if isinstance(bn, FusedBatchNorm2d) and bn.can_fuse(x):
        return bn.act(x, True, residual, pair=True)
    return bn_act(bn, x, True, residual)


# 0 keeps the stem BN apply as its own pass (A/B)
STEM_FUSE = os.environ.get("DPT_STEM_FUSE", "1") != "0"


def bn_relu_maxpool(bn: nn.Module, pool: nn.Module, x: torch.Tensor):
    """``pool(relu(bn(x)))`` - the ResNet stem.  With a fused BN and the stem's pair pool in
    training it is one op whose BN output is never materialised (ops/pool.py
    ``_BNReLUMaxPoolPair``); otherwise the plain composition."""
    if (STEM_FUSE and isinstance(bn, FusedBatchNorm2d) and isinstance(pool, FusedMaxPool2d) and pool.dpt_pair
            and bn.training and torch.is_grad_enabled() and bn.can_fuse(x)
            and fused_pool.bn_relu_maxpool_supported(x, bn, pool)):
        return fused_pool.bn_relu_maxpool_train(x, bn)
    return pool(bn_act(bn, x))


def split_block_input(x):
    """(conv-path input, identity-path input) of a residual block."""
    return x if isinstance(x, tuple) else (x, x)


class FusedMaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` that runs the gfx950 channels-last kernels when it can.  With
    ``dpt_pair`` (ResNet's stem pool, set by ``fuse_native_layers``) it returns
    ``(y_conv, y_identity)`` aliases for the first residual block, whose two gradients the
    backward sums while gathering."""

    dpt_pair = False

    def forward(self, x: torch.Tensor):
        if not self.return_indices and fused_pool.maxpool_supported(
                x, self.kernel_size, self.stride, self.padding, self.dilation, self.ceil_mode):
            as_int = lambda v: v if isinstance(v, int) else v[0]
            pair = self.dpt_pair and self.training and torch.is_grad_enabled()
            return fused_pool.max_pool2d_nhwc(x, as_int(self.kernel_size), as_int(self.stride),
                                              as_int(self.padding), pair)
        return super().forward(x)


class FusedAdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    """``nn.AdaptiveAvgPool2d((1, 1))`` whose backward is the gfx950 broadcast kernel."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if fused_pool.gap_supported(x) and torch.is_grad_enabled() and x.requires_grad:
            return fused_pool.global_avg_pool_nhwc(x)
        return super().forward(x)


class GemmConv1x1(nn.Conv2d):
    """1x1 / stride-1 / unpadded conv routed to a GEMM on channels_last activations.

    In channels_last memory the activation is a row-major [N*H*W, Cin] matrix, so the conv is
    ``x @ W^T`` with no data movement (hipBLASLt on gfx950, bf16 under autocast); autograd's
    matmul backward gives dgrad and wgrad as GEMMs as well.  Parameters and state-dict keys
    are the Conv2d's.
    """

    def gemm_ok(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dim() == 4 and self.groups == 1 and self.bias is None
                and self.kernel_size == (1, 1) and self.stride == (1, 1) and self.padding == (0, 0)
                and self.dilation == (1, 1) and x.is_contiguous(memory_format=torch.channels_last))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.gemm_ok(x):
            return super().forward(x)
        n, c, h, w = x.shape
        y = F.linear(x.permute(0, 2, 3, 1), self.weight.view(self.out_channels, c))
        return y.permute(0, 3, 1, 2)


def set_conv_routing(model: nn.Module, native_conv: bool = True, min_pixels=None, native_f32=None) -> None:
    """Per-model conv routing: MFMA kernels (ops/conv.py, ops/conv_f32.py) or MIOpen, stored on
    each conv; plain ``nn.Conv2d`` modules become ``NativeConv2d`` (same parameters).
    ``native_f32``: fp32 (no autocast) convs on the fp32 MFMA kernels for this model (None: the
    process default, ops/conv_f32.py ``ENABLED``)."""
    for m in model.modules():
        if type(m) is nn.Conv2d:
            m.__class__ = NativeConv2d
        if isinstance(m, nn.Conv2d):
            m.dpt_native_conv = bool(native_conv)
            m.dpt_min_pixels = min_pixels
            m.dpt_native_conv_f32 = None if native_f32 is None else bool(native_f32)


def fuse_native_layers(model: nn.Module, gemm_1x1: bool = False, native_conv: bool = True,
                       min_pixels=None, native_f32=None) -> int:
    """Install the gfx950 fused layers: BatchNorm2d -> FusedBatchNorm2d (fused with ReLU /
    residual add by the model's ``bn_act`` calls) and MaxPool2d -> FusedMaxPool2d.  Modules
    keep their parameters/buffers, so state dicts and checkpoints are unchanged.

    ``native_conv`` / ``min_pixels``: this model's conv routing (MFMA kernels or MIOpen; convs
    with fewer output pixels than ``min_pixels`` stay on MIOpen), stored on each conv module so
    two models in one process never share it."""
    set_conv_routing(model, native_conv, min_pixels, native_f32)
    n = fuse_batchnorm(model)
    for parent in model.modules():
        for name, child in list(parent.named_children()):
            new_cls = None
            if type(child) is nn.MaxPool2d:
                new_cls = FusedMaxPool2d
            elif type(child) is nn.AdaptiveAvgPool2d and child.output_size in (1, (1, 1)):
                new_cls = FusedAdaptiveAvgPool2d
            elif gemm_1x1 and type(child) is nn.Conv2d and child.kernel_size == (1, 1) \
                    and child.stride == (1, 1) and child.groups == 1 and child.bias is None:
                new_cls = GemmConv1x1
            if new_cls is not None:
                new = new_cls.__new__(new_cls)
                new.__dict__ = child.__dict__
                if new_cls is FusedMaxPool2d and name == "maxpool" and hasattr(parent, "layer1"):
                    new.dpt_pair = True  # ResNet stem: feeds layer1's conv and identity paths
                setattr(parent, name, new)
                n += 1
    tag_conv_bn_pairs(model)
    return n


def tag_conv_bn_pairs(model: nn.Module) -> int:
    """Mark convs whose output goes straight into a fused BatchNorm (``convK`` -> ``bnK`` in a
    block, ``(Conv2d, BatchNorm2d)`` consecutive in a Sequential): the native conv's epilogue
    then emits that BN's statistics (ops/conv.py) and the BN skips its statistics pass."""
    n = 0
    for parent in model.modules():
        kids = dict(parent.named_children())
        pairs = []
        if isinstance(parent, nn.Sequential):
            seq = list(parent)
            pairs = [(a, b) for a, b in zip(seq, seq[1:])]
        else:
            for name, child in kids.items():
                if name.startswith("conv") and ("bn" + name[4:]) in kids:
                    pairs.append((child, kids["bn" + name[4:]]))
        for conv, bn in pairs:
            if isinstance(conv, nn.Conv2d) and isinstance(bn, FusedBatchNorm2d) and conv.bias is None:
                conv.dpt_bn_stats = True
                n += 1
    return n


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
