"""Fused BatchNorm(+ReLU)(+residual add) autograd op on the gfx950 kernels (bn_kernels.hip).

Semantics are exactly ``relu(batch_norm(x) + residual)`` in training mode (batch
statistics, biased variance for normalisation, unbiased for the running variance,
``momentum`` update, ``num_batches_tracked += 1``) and ``relu(x*a + b + residual)`` with
the running statistics in eval mode - the composition the reference's ResNet blocks run as
separate MIOpen/ATen kernels (BN, in-place add, in-place ReLU).

Saved for backward: the BN input ``x`` and, for BN+add+ReLU, the output ``y`` - tensors the
unfused graph keeps alive anyway (BN saves its input, ReLU its output, and ``y`` is the next
convolution's saved input), so the fusion costs no extra activation memory.  A block tail whose
output feeds a native conv also writes its ReLU mask as 1 bit per element (1/16 of ``y``), which
that conv's backward-data epilogue reads instead of ``y``.  For BN+ReLU
without a residual the ReLU mask is recomputed from ``x`` and the forward's per-channel
coefficients (``fma(x, a, b) > 0``, bit-identical to the forward's decision), so the backward
passes never read ``y``: 2 of 7 activation passes saved per such layer.
"""
from __future__ import annotations

from typing import Optional

import torch

import os

from . import native, native_available
from .conv import MASKED_NO_RES, take_bnb_partials

# Block-tail BN+add+ReLU backward statistics in the consuming conv's dgrad epilogue (see _bwd)
BNR_FUSE = os.environ.get("DPT_BNR_FUSE", "1") != "0"


def _cl(t: torch.Tensor) -> torch.Tensor:
    if t.dim() == 4 and not t.is_contiguous(memory_format=torch.channels_last):
        return t.contiguous(memory_format=torch.channels_last)
    return t


def _relu_mask(x: torch.Tensor) -> torch.Tensor:
    """uint8 [N*H*W, C/8]: bit k of byte (m, g) = (y[m, 8g + k] > 0), written by the forward apply."""
    c = x.shape[1]
    return torch.empty((x.numel() // c, c // 8), dtype=torch.uint8, device=x.device)


class _BNActTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, num_batches, momentum, eps, relu,
                partials, links):
        y = _fwd(ctx, x, residual, weight, bias, running_mean, running_var, num_batches, momentum, eps, relu,
                 partials=partials, links=links)
        return y

    @staticmethod
    def backward(ctx, dy):
        return _bwd(ctx, dy, None) + (None,) * 8


class _BNActTrainPair(torch.autograd.Function):
    """Same op with two aliased outputs: one for the next block's conv path, one for its
    identity path.  Autograd then hands their gradients to ``backward`` separately and the
    stats kernel sums them while it reads them - no autograd add kernel, and the summed,
    masked gradient it writes IS the residual-path gradient (SURVEY-era ResNet-50 profile:
    the residual-gradient adds were ~1.3 ms of a 33 ms step)."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, num_batches, momentum, eps, relu,
                partials, links):
        y = _fwd(ctx, x, residual, weight, bias, running_mean, running_var, num_batches, momentum, eps, relu,
                 pair=True, partials=partials, links=links)
        ctx.set_materialize_grads(False)  # an unused alias (last block) gives None, not zeros
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, dy, dy2):
        return _bwd(ctx, dy, dy2) + (None,) * 8


def _fwd(ctx, x, residual, weight, bias, running_mean, running_var, num_batches, momentum, eps, relu,
         pair=False, partials=None, links=(None, None)):
    ps, pq = partials if partials is not None else (None, None)
    own_slot, res_slot = links
    # block tail whose output feeds a native conv: the 1-bit ReLU mask that conv's dgrad epilogue
    # reads instead of y (1/16 of y's bytes; ops/conv.py BNR)
    mask = _relu_mask(x) if (own_slot is not None and relu and residual is not None) else None
    y, mean, invstd, coef = native().bn_fwd_train(x, residual, weight, bias, running_mean, running_var,
                                                  num_batches, float(momentum), float(eps), bool(relu), ps, pq,
                                                  mask_out=mask)
    ctx.relu = bool(relu)
    ctx.has_res = residual is not None
    mask_from_x = ctx.relu and not ctx.has_res and not pair   # pair outputs always write dz
    ctx.save_for_backward(x, y if (relu and not mask_from_x) else None, weight, mean, invstd,
                          coef if mask_from_x else None)
    if mask_from_x:
        # a native conv consuming y sums this BN's backward statistics in its dgrad epilogue
        y._dpt_bn_src = (x, mean, coef)
    ctx.res_slot = res_slot  # our residual input is the identity alias of an earlier block tail
    if own_slot is not None:
        if mask is not None:
            own_slot["mask"] = mask
        # block tail: the conv consuming y sums the statistics (and folds in the identity-path
        # gradient the next block's tail leaves in own_slot, see _bwd) in its dgrad epilogue
        y._dpt_bn_src = (x, mean, own_slot)
    return y


def _bwd(ctx, dy, dy2):
    x, y, weight, mean, invstd, coef = ctx.saved_tensors
    if dy is None:
        dy, dy2 = dy2, None
    if dy is None:
        return (None, None, None, None)
    want_params = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
    want_dz = ctx.has_res and ctx.needs_input_grad[1]
    if coef is not None and dy2 is None:
        part = take_bnb_partials(dy)
        if part is not None:  # statistics already summed by the consuming conv's dgrad epilogue
            dx, dg, db = native().bn_bwd_partials(dy, x, weight, mean, invstd, coef, part[0], part[1],
                                                  bool(want_params))
            return (dx, None, dg if want_params else None, db if want_params else None)
    if dy2 is not None and ctx.relu and ctx.has_res:
        part = take_bnb_partials(dy)
        if part is not None and part[3] is not None:
            raise RuntimeError("fused block-tail backward: unexpected downsample statistic")
        if part is not None:
            # the consuming conv's dgrad epilogue already formed dz = (dy + dy2) * (y > 0) in dy's
            # storage and summed its statistics (ops/conv.py); dz is also the residual gradient
            if part[2] != dy2.data_ptr():
                raise RuntimeError("fused block-tail backward: the identity-path gradient folded into the "
                                   "conv's dgrad is not the one autograd delivered (alias used twice?)")
            dx, dg, db = native().bn_bwd_partials(dy, x, weight, mean, invstd, None, part[0], part[1],
                                                  bool(want_params), True)
            if ctx.res_slot is not None:
                ctx.res_slot["dres"] = dy
            return (dx, dy if want_dz else None, dg if want_params else None, db if want_params else None)
    if dy2 is None and ctx.relu and ctx.has_res:
        part = take_bnb_partials(dy)
        if part is not None and part[2] == MASKED_NO_RES:
            # the last block tail: the average-pool backward formed dz = dy * (y > 0) and summed
            # the statistics (ops/pool.py gap_bwd_bnr); dz is also the residual gradient
            dx, dg, db = native().bn_bwd_partials(dy, x, weight, mean, invstd, None, part[0], part[1],
                                                  bool(want_params), True)
            if ctx.res_slot is not None:
                ctx.res_slot["dres"] = dy
            return (dx, dy if want_dz else None, dg if want_params else None, db if want_params else None)
    dx, dg, db, dz = native().bn_bwd(_cl(dy), None if dy2 is None else _cl(dy2), y, x, weight, mean, invstd,
                                     ctx.relu, bool(want_dz), bool(want_params), coef)
    if want_dz and ctx.res_slot is not None:
        ctx.res_slot["dres"] = dz  # picked up by the dgrad of the conv that consumed that alias
    return (dx, dz if want_dz else None, dg if want_params else None, db if want_params else None)


class _BN2AddReLUPair(torch.autograd.Function):
    """Residual-block tail whose identity path is a downsample BatchNorm:
    ``relu(bn(x) + bn2(x2))`` with both BNs in training mode, as ONE op.

    Forward: both BNs' statistics (from the producing convs' epilogue partials), running-stat
    updates and coefficients, then one apply pass ``relu(x*a + b + x2*a2 + b2)`` - the
    downsample BN's output is never written (the unfused chain writes it and reads it back).
    Backward: both BNs see the same masked gradient dz = (dy + dy2) * (y > 0).  When the
    consuming conv's dgrad epilogue formed dz (ops/conv.py BNR) it also summed
    s3 = sum dz*(x2 - mean2), so the downsample BN needs no statistics pass either, and one
    apply pass reads dz once and writes both input gradients.  Pair outputs as
    ``_BNActTrainPair``."""

    @staticmethod
    def forward(ctx, x, x2, w, b, rm, rv, nb, w2, b2, rm2, rv2, nb2, momentum, eps, momentum2, eps2,
                partials, partials2, own_slot):
        C = native()
        ps, pq = partials if partials is not None else (None, None)
        ps2, pq2 = partials2 if partials2 is not None else (None, None)
        _, mean, invstd, coef = C.bn_fwd_train(x, None, w, b, rm, rv, nb, float(momentum), float(eps), True,
                                               ps, pq, False)
        _, mean2, invstd2, coef2 = C.bn_fwd_train(x2, None, w2, b2, rm2, rv2, nb2, float(momentum2), float(eps2),
                                                  False, ps2, pq2, False)
        mask = _relu_mask(x) if own_slot is not None else None
        y = C.bn_apply_aff(x, x2, coef, coef2, mask_out=mask)
        ctx.save_for_backward(x, x2, y, w, w2, mean, invstd, mean2, invstd2)
        ctx.set_materialize_grads(False)
        if own_slot is not None:
            own_slot["mask"] = mask
            y._dpt_bn_src = (x, mean, own_slot, x2, mean2)
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, dy, dy2):
        x, x2, y, w, w2, mean, invstd, mean2, invstd2 = ctx.saved_tensors
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return (None,) * 19
        want = [ctx.needs_input_grad[i] for i in (2, 3, 7, 8)]
        want_params = any(want)
        C = native()
        part = take_bnb_partials(dy) if dy2 is not None else None
        if part is not None and part[3] is not None:
            if part[2] != dy2.data_ptr():
                raise RuntimeError("fused block-tail backward: the identity-path gradient folded into the "
                                   "conv's dgrad is not the one autograd delivered (alias used twice?)")
            dx, dx2, dg, db, dg2, db2 = C.bn2_bwd_partials(dy, x, x2, w, w2, mean, invstd, mean2, invstd2,
                                                           part[0], part[1], part[3], bool(want_params))
        else:
            if part is not None:
                raise RuntimeError("fused block-tail backward: partials without the downsample statistic")
            dx, dg, db, dz = C.bn_bwd(_cl(dy), None if dy2 is None else _cl(dy2), y, x, w, mean, invstd,
                                      True, True, bool(want_params), None)
            dx2, dg2, db2, _ = C.bn_bwd(dz, None, None, x2, w2, mean2, invstd2, False, False,
                                        bool(want_params), None)
        g = [dg, db, dg2, db2]
        g = [t if (want_params and want[i]) else None for i, t in enumerate(g)]
        return (dx, dx2, g[0], g[1], None, None, None, g[2], g[3]) + (None,) * 10


def bn2_add_relu_train(x, bn, x2, bn2):
    """Block tail ``relu(bn(x) + bn2(x2))`` in training mode (both ``FusedBatchNorm2d``), pair
    outputs (conv path, identity path) - see _BN2AddReLUPair."""
    x2 = _cl(x2.to(x.dtype))
    partials = x.__dict__.pop("_dpt_bn_partials", None)
    partials2 = x2.__dict__.pop("_dpt_bn_partials", None)
    own_slot = {} if (BNR_FUSE and x.dtype in (torch.bfloat16, torch.float16)) else None
    out = _BN2AddReLUPair.apply(x, x2, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                                bn2.weight, bn2.bias, bn2.running_mean, bn2.running_var, bn2.num_batches_tracked,
                                bn.momentum, bn.eps, bn2.momentum, bn2.eps, partials, partials2, own_slot)
    if own_slot is not None:
        out[1]._dpt_res_slot = own_slot
    return out


def bn_act_supported(x: torch.Tensor, num_features: int) -> bool:
    return (x.is_cuda and native_available() and x.dim() == 4
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last)
            and native().bn_supported(num_features))


def bn_act_train(x: torch.Tensor, residual: Optional[torch.Tensor], weight, bias, running_mean, running_var,
                 num_batches, momentum: float, eps: float, relu: bool, pair: bool = False):
    res_slot = None
    if residual is not None:
        if residual.dtype == x.dtype and residual.is_contiguous(memory_format=torch.channels_last):
            # the identity alias of an earlier fused block tail (see below)
            res_slot = residual.__dict__.get("_dpt_res_slot")
        residual = _cl(residual.to(x.dtype))
    # statistics already summed by the producing native conv's epilogue (ops/conv.py)
    partials = x.__dict__.pop("_dpt_bn_partials", None)
    # block tails: own_slot receives the identity-path gradient from the next block's tail
    # backward (which runs before the backward of the conv consuming our conv-path output)
    own_slot = {} if (pair and relu and residual is not None and BNR_FUSE
                      and x.dtype in (torch.bfloat16, torch.float16)) else None
    fn = _BNActTrainPair if pair else _BNActTrain
    out = fn.apply(x, residual, weight, bias, running_mean, running_var, num_batches, momentum, eps, relu,
                   partials, (own_slot, res_slot))
    if own_slot is not None:
        out[1]._dpt_res_slot = own_slot
    return out


@torch.no_grad()
def bn_act_eval(x: torch.Tensor, residual: Optional[torch.Tensor], weight, bias, running_mean, running_var,
                eps: float, relu: bool) -> torch.Tensor:
    a = torch.rsqrt(running_var.float() + eps)
    if weight is not None:
        a = a * weight.float()
    b = -running_mean.float() * a
    if bias is not None:
        b = b + bias.float()
    if residual is not None:
        residual = _cl(residual.to(x.dtype))
    return native().bn_apply(x, residual, a.contiguous(), b.contiguous(), bool(relu))


def reference_bn_act(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, relu):
    """Unfused PyTorch composition (CPU path and test oracle)."""
    y = torch.nn.functional.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y
