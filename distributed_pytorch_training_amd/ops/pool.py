"""Channels-last max-pool on the gfx950 kernels (pool_kernels.hip).

Forward keeps a uint8 window-local argmax per output element (1 byte vs ATen's int64 flat
index); backward is a gather over the windows covering each input pixel - no atomics, no
zero-fill pass.  Same values, same tie-breaking (first max) and NaN propagation as
``torch.nn.functional.max_pool2d``.
"""
from __future__ import annotations

import torch

from . import native, native_available


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad):
        y, idx = native().maxpool_fwd(x, k, stride, pad)
        ctx.save_for_backward(idx)
        ctx.cfg = (x.shape[2], x.shape[3], k, stride, pad)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.cfg
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        return native().maxpool_bwd(dy, idx, H, W, k, s, p), None, None, None


def maxpool_supported(x: torch.Tensor, k, stride, pad, dilation, ceil_mode) -> bool:
    k, stride, pad, dilation = (v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else None)
                                for v in (k, stride, pad, dilation))
    return (x.is_cuda and native_available() and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last)
            and None not in (k, stride, pad, dilation) and dilation == 1 and not ceil_mode
            and k * k <= 255 and pad <= k // 2)


def max_pool2d_nhwc(x: torch.Tensor, k: int, stride: int, pad: int) -> torch.Tensor:
    return _MaxPoolNHWC.apply(x, int(k), int(stride), int(pad))
