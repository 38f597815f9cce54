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
        return native().maxpool_bwd(dy, idx, H, W, k, s, p)[0], None, None, None


class _MaxPoolNHWCPair(torch.autograd.Function):
    """Same op with two aliased outputs (ResNet's stem pool feeds layer1's conv path and its
    downsample identity path): autograd hands the two gradients over separately and the
    backward gather sums them while reading - no autograd add kernel (a full pass over the
    [B, 56, 56, 64] activation gradient, twice read once written)."""

    @staticmethod
    def forward(ctx, x, k, stride, pad, bn_src):
        y, idx = native().maxpool_fwd(x, k, stride, pad)
        ctx.save_for_backward(idx)
        ctx.cfg = (x.shape[2], x.shape[3], k, stride, pad)
        # (BN input, mean, coef) of the fused BN+ReLU that produced x (the ResNet stem): the
        # backward gather also sums that BN's backward statistics (ops/bn.py picks them up)
        ctx.bn_src = bn_src if (bn_src is not None and (k, stride, pad) == (3, 2, 1)) else None
        ctx.mark_non_differentiable(idx)
        ctx.set_materialize_grads(False)
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, dy, dy2):
        from .conv import BN_BWD_FUSE, register_bnb_partials

        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.cfg
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return None, None, None, None, None
        dy = _cl(dy)
        if dy2 is not None:
            dy2 = _cl(dy2.to(dy.dtype))
        src = ctx.bn_src if BN_BWD_FUSE else None
        if src is not None and src[0].dtype == dy.dtype:
            dx, p1, p2 = native().maxpool_bwd(dy, idx, H, W, k, s, p, dy2, src[0], src[1], src[2])
            register_bnb_partials(dx, p1, p2)
        else:
            dx = native().maxpool_bwd(dy, idx, H, W, k, s, p, dy2)[0]
        return dx, None, None, None, None


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def maxpool_supported(x: torch.Tensor, k, stride, pad, dilation, ceil_mode) -> bool:
    k, stride, pad, dilation = (v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else None)
                                for v in (k, stride, pad, dilation))
    return (x.is_cuda and native_available() and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last)
            and None not in (k, stride, pad, dilation) and dilation == 1 and not ceil_mode
            and k * k <= 255 and pad <= k // 2)


def max_pool2d_nhwc(x: torch.Tensor, k: int, stride: int, pad: int, pair: bool = False):
    """``pair``: return (y, y_alias) for a conv path and an identity path (see _MaxPoolNHWCPair)."""
    if pair:
        return _MaxPoolNHWCPair.apply(x, int(k), int(stride), int(pad), x.__dict__.get("_dpt_bn_src"))
    return _MaxPoolNHWC.apply(x, int(k), int(stride), int(pad))


class _GlobalAvgPoolNHWC(torch.autograd.Function):
    """adaptive_avg_pool2d(x, 1) on a channels_last activation; the backward broadcast
    g / (H*W) is one vectorised HIP kernel (pool_kernels.hip gap_bwd) instead of ATen's
    expand + strided copy."""

    @staticmethod
    def forward(ctx, x):
        ctx.cfg = (x.shape[2], x.shape[3], x.dtype)
        # x is the output of the network's last fused block tail (ops/bn.py: (BN input, mean,
        # slot), no downsample BN folded in): the backward also forms that tail's masked
        # gradient and sums its BN statistics (gap_bwd_bnr), as a conv's backward-data epilogue
        # does for every other tail - the BN backward then skips its statistics pass
        src = x.__dict__.get("_dpt_bn_src")
        from .conv import BN_BWD_FUSE
        ctx.bn_src = None
        if (BN_BWD_FUSE and src is not None and len(src) == 3 and isinstance(src[2], dict)
                and x.dtype in (torch.bfloat16, torch.float16) and 256 % (x.shape[1] // 8) == 0):
            ctx.bn_src = src
            ctx.save_for_backward(x)
        return torch.nn.functional.adaptive_avg_pool2d(x, 1)

    @staticmethod
    def backward(ctx, g):
        H, W, dt = ctx.cfg
        g2 = g.reshape(g.shape[0], g.shape[1]).contiguous()
        if ctx.bn_src is not None:
            from .conv import register_bnb_partials
            (y,) = ctx.saved_tensors
            dz, p1, p2 = native().gap_bwd_bnr(g2, y, ctx.bn_src[0], ctx.bn_src[1])
            register_bnb_partials(dz, p1, p2, masked=True)
            return dz
        return native().gap_bwd(g2, H, W, dt)


def gap_supported(x: torch.Tensor) -> bool:
    return (x.is_cuda and native_available() and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last))


def global_avg_pool_nhwc(x: torch.Tensor) -> torch.Tensor:
    return _GlobalAvgPoolNHWC.apply(x)


class _BNReLUMaxPoolPair(torch.autograd.Function):
    """ResNet stem ``maxpool3x3/2(relu(bn(x)))`` in training mode as ONE op, pair outputs.

    Forward: the BN's statistics (from the stem conv's epilogue partials), running-stat update
    and coefficients, then the pool reads x and applies the BN+ReLU to every loaded element with
    the apply pass's exact arithmetic and rounding (pool_kernels.hip AFF) - the 112x112 BN
    output is never written.  Backward: the pool's gather sums the two output gradients and the
    BN's backward statistics (BNS), then the BN backward applies from those partials; the ReLU
    mask is recomputed from x, so nothing of the BN output is needed there either."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, num_batches, momentum, eps, partials):
        C = native()
        ps, pq = partials if partials is not None else (None, None)
        _, mean, invstd, coef = C.bn_fwd_train(x, None, weight, bias, running_mean, running_var, num_batches,
                                               float(momentum), float(eps), True, ps, pq, False)
        y, idx = C.maxpool_fwd(x, 3, 2, 1, coef)
        ctx.save_for_backward(x, weight, mean, invstd, coef, idx)
        ctx.mark_non_differentiable(idx)
        ctx.set_materialize_grads(False)
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, dy, dy2):
        x, weight, mean, invstd, coef, idx = ctx.saved_tensors
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return (None,) * 9
        dy = _cl(dy)
        if dy2 is not None:
            dy2 = _cl(dy2.to(dy.dtype))
        C = native()
        dz, p1, p2 = C.maxpool_bwd(dy, idx, x.shape[2], x.shape[3], 3, 2, 1, dy2, x, mean, coef)
        want = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        dx, dg, db = C.bn_bwd_partials(dz, x, weight, mean, invstd, coef, p1, p2, bool(want))
        return (dx, dg if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None) + (None,) * 6


def bn_relu_maxpool_supported(x: torch.Tensor, bn, pool) -> bool:
    as_int = lambda v: v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else None)
    C = x.shape[1] if x.dim() == 4 else 0
    return (maxpool_supported(x, pool.kernel_size, pool.stride, pool.padding, pool.dilation, pool.ceil_mode)
            and (as_int(pool.kernel_size), as_int(pool.stride), as_int(pool.padding)) == (3, 2, 1)
            and not pool.return_indices and C <= 512 and (C & (C - 1)) == 0
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32))


def bn_relu_maxpool_train(x: torch.Tensor, bn) -> tuple:
    partials = x.__dict__.pop("_dpt_bn_partials", None)
    return _BNReLUMaxPoolPair.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                                    bn.momentum, bn.eps, partials)

