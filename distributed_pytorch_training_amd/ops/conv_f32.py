"""Channels-last fp32 convolution autograd op on the gfx950 fp32 matrix cores
(csrc/kernels/conv_f32_kernels.hip, ``v_mfma_f32_32x32x2_f32``).

The reference's default precision is fp32 (reference ``train_ddp.py:210-214``: the FP32 branch of
the step, no ``--amp``), and its convolutions are torchvision's cuDNN convs (SURVEY.md §2.5
K2/K5/K10).  On MI355X those ran on MIOpen, whose fp32 NHWC solvers are non-deterministic in the
forward (split-K atomics), partly wrong under hipGraph replay, and a quarter of the fp32 MFMA
peak.  These kernels are exact fp32 (one rounding per product, like the MFMA itself), bitwise
deterministic run to run, replay-safe, and route every fp32 convolution of the native engine:

forward   implicit GEMM over (r, s, c) taps of x;
backward  input gradient as the transposed-conv gather of dy against the [C][R][S][Co] weight,
          weight gradient as dy^T X over pixels; split-K partials are summed in a fixed order.

Channels must be multiples of 4 (16-byte loads of one tap); a narrower input (the 3-channel
stem) is zero-padded to 4 channels, which autograd maps back.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import native, native_available

# Opt-in (``--native-conv-fp32`` or DPT_NATIVE_CONV_F32=1): bitwise deterministic, replay-safe and
# exact, but on ResNet-50 / 224 / batch 256 the step is 108.6 ms against 79.4 ms on MIOpen's fp32
# solvers (which use Winograd for the 3x3s), and the fp32 ResNet-18 / 32x32 replay 41k against 66k
# samples/s (profiles/conv_f32_r5.md) - so MIOpen stays the default fp32 path.
ENABLED = os.environ.get("DPT_NATIVE_CONV_F32", "0") == "1"
# Which convs the enabled path takes (A/B, DPT_NATIVE_CONV_F32_SCOPE): "all", "1x1" (one-tap,
# stride 1), "1x1s" (one-tap, any stride), "kxk" (multi-tap convs only); the rest stay on MIOpen.
SCOPE = os.environ.get("DPT_NATIVE_CONV_F32_SCOPE", "all")
_CL = torch.channels_last


def _in_scope(r: int, s: int, stride: int) -> bool:
    if SCOPE == "1x1":
        return r == 1 and s == 1 and stride == 1
    if SCOPE == "1x1s":
        return r == 1 and s == 1
    if SCOPE == "kxk":
        return r * s > 1
    return True


def supported(x: torch.Tensor, w: torch.Tensor, bias, stride, padding, dilation, groups,
              enabled: bool | None = None) -> bool:
    """``enabled``: the conv module's own routing (``dpt_native_conv_f32``); None = ``ENABLED``."""
    if not ((ENABLED if enabled is None else enabled) and x.is_cuda and native_available() and x.dtype == torch.float32 and w.dtype == torch.float32
            and x.dim() == 4 and groups == 1 and bias is None):
        return False
    if torch.is_autocast_enabled("cuda"):
        return False
    if tuple(dilation) != (1, 1) or stride[0] != stride[1] or padding[0] != padding[1]:
        return False
    cout, cin, r, s = w.shape
    if not _in_scope(r, s, stride[0]):
        return False
    return (cout % 4 == 0 and x.shape[1] == cin and x.is_contiguous(memory_format=_CL)
            and (x.shape[2] + 2 * padding[0] - r) // stride[0] + 1 > 0
            and (x.shape[3] + 2 * padding[1] - s) // stride[1] + 1 > 0)


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous(memory_format=_CL) else t.contiguous(memory_format=_CL)


class _ConvF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int):
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad = stride, pad
        return native().conv_f32_fwd(x, w, stride, pad)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = _cl(dy.float())
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = native().conv_f32_dgrad(dy, w, ctx.stride, ctx.pad, x.shape[2], x.shape[3])
        if ctx.needs_input_grad[1]:
            dw = native().conv_f32_wgrad(dy, x, list(w.shape), ctx.stride, ctx.pad)
        return dx, dw, None, None


def conv2d(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    """y = conv2d(x, w, stride, pad), fp32, channels_last, on the fp32 MFMA kernels."""
    cin = w.shape[1]
    if cin % 4:
        extra = 4 - cin % 4     # zero channels: the same products, autograd drops their gradients
        x = F.pad(x, (0, 0, 0, 0, 0, extra))
        w = F.pad(w, (0, 0, 0, 0, 0, extra))
    return _ConvF32.apply(_cl(x), _cl(w), int(stride), int(pad))


class NativeConv2d(nn.Conv2d):
    """``nn.Conv2d`` whose fp32 (no autocast) channels_last forward runs the fp32 MFMA kernels
    when the model's routing allows it (``dpt_native_conv`` and ``dpt_native_conv_f32``, set per
    model by models/layers.py ``set_conv_routing``); anything else is ``nn.Conv2d``'s own path.  Under autocast the shadow
    subclass (parallel/shadow.py ``ShadowConv2d``) takes the bf16 / fp16 MFMA kernels instead.
    Parameters and state-dict keys are the Conv2d's."""

    dpt_native_conv = True
    dpt_min_pixels = None
    dpt_native_conv_f32 = None    # per-model fp32 routing (set_conv_routing); None = ENABLED (env)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.dpt_native_conv and supported(x, self.weight, self.bias, self.stride, self.padding,
                                              self.dilation, self.groups, self.dpt_native_conv_f32):
            return conv2d(x, self.weight, self.stride[0], self.padding[0])
        return super().forward(x)
