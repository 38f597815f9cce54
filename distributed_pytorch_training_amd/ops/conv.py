"""Channels-last bf16 / fp16 convolution autograd op on the hand-written MFMA kernels
(csrc/kernels/conv_kernels.hip).

forward   implicit-GEMM conv; with ``bn_stats`` its epilogue also emits the per-channel
          (sum, sum of squares) partials of the bf16 output, which the following fused
          BatchNorm consumes instead of re-reading the activation (ops/bn.py picks them up
          from the output tensor's ``_dpt_bn_partials`` attribute).
backward  input gradient: the same kernel on dy reading the weight as [co][ci] with flipped taps
          through transposing LDS reads (stride 1), or, stride 2, four parity-class convs whose
          outputs are scattered onto the even/odd rows and columns of dx; weight gradient: split-K MFMA kernel
          with transposing LDS reads, bf16 (the shadow weight's dtype).

Replaces the reference's cuDNN convolutions (reference
``train_ddp.py:205,207`` -> torchvision ``resnet18`` convs); measured per shape against MIOpen
in ``profiles/conv_kernels_vs_miopen_v1.md``.
"""
from __future__ import annotations

import os

import torch

from . import native, native_available

_CL = torch.channels_last
# element types of the MFMA kernels (bf16 and fp16 operands, fp32 accumulation)
_DT16 = (torch.bfloat16, torch.float16)
# process-wide kill switch (environment); per-model routing lives on the conv modules
ENABLED = os.environ.get("DPT_NATIVE_CONV", "1") != "0"
# Backward-data of a conv fed by a fused BN+ReLU also sums that BN's backward statistics in its
# epilogue (the BN backward then skips its statistics pass).
BN_BWD_FUSE = os.environ.get("DPT_BN_BWD_FUSE", "1") != "0"
# dx.data_ptr() -> (generation, dx._version, p1, p2, shape, dres_ptr, p3): handed from a conv's
# backward to the BN backward that receives dx as its output gradient (ops/bn.py), consumed once.
# An entry is only honoured in the step generation that made it and while dx is unmodified (its
# version counter unchanged: autograd accumulating a second gradient into dx in place would
# invalidate the statistics); begin_step()/reset_side_channels() drop everything left over (an
# aborted backward), so a reused allocation can never pick up stale statistics.
_BNB_PARTIALS = {}
_GEN = [0]
# Stride-2 backward-data on the MFMA kernels (four parity-class convs); 0 = MIOpen
S2_DGRAD = os.environ.get("DPT_S2_DGRAD", "1") != "0"
# Backward-weight before backward-data, its split-K reduce run by extra blocks in the
# backward-data launch's tail (conv_wgrad_deferred / wgrad_reduce=): no reduce launch of its own
WGRAD_REDUCE_FUSE = os.environ.get("DPT_WGRAD_REDUCE_FUSE", "1") != "0"
# The im2col stem path is correct but measured slower than MIOpen on ResNet-50's 7x7/2 stem at
# batch 256 (the [3.2M x 192] bf16 patch matrix is 1.2 GB written and read twice): opt-in only.
STEM_ENABLED = os.environ.get("DPT_NATIVE_STEM", "0") == "1"


# Convs with fewer output pixels than this go to MIOpen (default: none; a model can override it
# per conv through models.layers.fuse_native_layers(min_pixels=...)).  Small tile grids used to
# lose to MIOpen's small-shape kernels under hipGraph (ResNet-18 on 32x32: 128-2048 output
# pixels in layer2-4 at batch 128); the kernels now split the K loop over blocks there
# (conv_fwd_splits), which beats MIOpen at every size (BASELINE.md ResNet-18 table).
MIN_PIXELS = int(os.environ.get("DPT_CONV_MIN_PIXELS", "0"))


def supported(x: torch.Tensor, w: torch.Tensor, stride, padding, dilation, groups, min_pixels=None) -> bool:
    if not (ENABLED and x.is_cuda and native_available() and x.dtype in _DT16
            and w.dtype == x.dtype and x.dim() == 4 and groups == 1):
        return False
    if tuple(dilation) != (1, 1) or stride[0] != stride[1] or padding[0] != padding[1]:
        return False
    cout, cin, r, s = w.shape
    ho = (x.shape[2] + 2 * padding[0] - r) // stride[0] + 1
    wo = (x.shape[3] + 2 * padding[1] - s) // stride[1] + 1
    return (cin % 64 == 0 and cout % 64 == 0 and r == s and x.shape[1] == cin
            and x.shape[0] * ho * wo >= (MIN_PIXELS if min_pixels is None else min_pixels)
            and x.is_contiguous(memory_format=_CL))


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous(memory_format=_CL) else t.contiguous(memory_format=_CL)


# In-step attribution (bench/conv_instep.py): when a list, every conv pass records a timing event
# on the current stream before and after its launches, tagged (pass, shape, epilogue variant).
# Off (None) in training: no event, no Python work.
_CALLS = None


def profile_calls(on: bool) -> None:
    global _CALLS
    _CALLS = [] if on else None


def take_profile():
    """[(pass, shape, variant, start_event, end_event)] recorded since profile_calls(True)."""
    out = list(_CALLS or [])
    if _CALLS is not None:
        _CALLS.clear()
    return out


def _mark():
    if _CALLS is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _note(kind, x, w, stride, pad, variant, e0, out_hw=(0, 0)):
    if _CALLS is None or e0 is None:
        return
    co, ci, r, _ = w.shape
    key = (ci, x.shape[2], x.shape[3], co, r, int(stride), int(pad), tuple(int(v) for v in out_hw))
    _CALLS.append((kind, key, variant, e0, _mark()))


def _backward(ctx, dy):
    x, w = ctx.saved_tensors
    dy = _cl(dy.to(x.dtype))
    s, p = ctx.stride, ctx.pad
    dx = dw = red = None
    e0 = _mark()
    if ctx.needs_input_grad[1]:
        if ctx.needs_input_grad[0] and WGRAD_REDUCE_FUSE:
            dw, red = native().conv_wgrad_deferred(dy, x, list(w.shape), s, p)
        else:
            dw = native().conv_wgrad(dy, x, list(w.shape), s, p, False)
        _note("wgrad", x, w, s, p, "deferred-reduce" if red is not None else "reduce", e0)
        e0 = _mark()
    variant = None
    if ctx.needs_input_grad[0]:
        src = ctx.bn_src if (s == 1 and BN_BWD_FUSE) else None
        dres = None
        wt = _flipped(w) if s == 1 else None
        if src is not None and not isinstance(src[2], dict):  # BN+ReLU: (x, mean, coef)
            bn_x, bn_mean, bn_coef = src
            dx, p1, p2, _ = native().conv_dgrad_bnstats(dy, w, p, bn_x, bn_mean, bn_coef, w_flipped=wt,
                                                        wgrad_reduce=red)
            _put_bnb(dx, p1, p2, None, None)
            variant = "bnrelu-stats"
        elif src is not None and _dres_ok(dres := src[2].pop("dres", None), x):  # (x, mean, slot)
            # block-tail BN+add+ReLU (ops/bn.py pair outputs): the next block's tail already
            # produced the identity-path gradient dres; dx becomes the tail's masked total
            # gradient, the conv's input x is the tail's output y (the ReLU mask)
            bn_x, bn_mean = src[0], src[1]
            # (x, mean, slot, x2, mean2): the tail's identity path was a downsample BatchNorm
            # folded into it (ops/bn.py _BN2AddReLUPair) - also sum that BN's statistic
            x2, mean2 = (src[3], src[4]) if len(src) > 3 else (None, None)
            # the tail's 1-bit ReLU mask (ops/bn.py) is read instead of its output x when present
            dx, p1, p2, p3 = native().conv_dgrad_bnstats(dy, w, p, bn_x, bn_mean, None, x, dres, wt, x2, mean2,
                                                         wgrad_reduce=red, bn_mask=src[2].get("mask"))
            _put_bnb(dx, p1, p2, dres.data_ptr(), p3 if x2 is not None else None)
            variant = "tail+ds-stats" if x2 is not None else "tail-stats"
        elif s == 1:
            dx = (native().conv_dgrad_flip(dy, w, p, wgrad_reduce=red)[0] if wt is None
                  else native().conv_dgrad_preflipped(dy, wt, p, wgrad_reduce=red))
            variant = "plain"
        elif s == 2 and S2_DGRAD and x.dim() == 4:
            src = ctx.bn_src if BN_BWD_FUSE else None
            if src is not None and not isinstance(src[2], dict) and w.shape[2] > 1:
                # BN+ReLU input: its backward statistics from the parity-class epilogues too
                dx, p1, p2 = native().conv_dgrad_s2(dy, w, p, x.shape[2], x.shape[3], src[0], src[1], src[2],
                                                    wgrad_reduce=red)
                _put_bnb(dx, p1, p2, None, None)
                variant = "s2-bnrelu-stats"
            else:
                dx = native().conv_dgrad_s2(dy, w, p, x.shape[2], x.shape[3], wgrad_reduce=red)[0]
                variant = "s2"
        else:
            dx = torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                                     (True, False, False))[0]
    if red is not None and not red.done:
        native().conv_reduce_flush(red)   # no native backward-data launch took it
    if variant is not None:
        _note("dgrad", x, w, s, p, variant + ("+reduce" if red is not None else ""), e0)
    if dx is not None and ctx.res_slot is not None:
        # x is the identity alias of a fused block tail and this conv its downsample: hand the
        # identity-path gradient to the tail's conv-path consumer (see ops/bn.py)
        ctx.res_slot["dres"] = dx
    return dx, dw


# Per-step flip cache: the stride-1 backward-data reads a flipped/transposed weight copy
# wt[ci][R-1-r][S-1-s][co].  With the cache on (the trainer calls begin_step() each step) the
# forward registers every such weight and the first backward-data of the step flips them all
# in ONE launch (46 launches per ResNet-50 step otherwise).
_FLIP = {"on": False, "pending": {}, "done": {}}


def reset_side_channels() -> None:
    """New step generation: forget every BN-backward hand-over not consumed so far."""
    _GEN[0] += 1
    _BNB_PARTIALS.clear()


def _put_bnb(dx, p1, p2, dres_ptr, p3) -> None:
    _BNB_PARTIALS[dx.data_ptr()] = (_GEN[0], dx._version, p1, p2, tuple(dx.shape), dres_ptr, p3)


def begin_step() -> None:
    reset_side_channels()
    _FLIP["on"] = True
    _FLIP["pending"].clear()
    _FLIP["done"].clear()


def end_caching() -> None:
    _FLIP["on"] = False
    _FLIP["pending"].clear()
    _FLIP["done"].clear()


def _flipped(w: torch.Tensor):
    if not _FLIP["on"]:
        return None
    key = (w.data_ptr(), tuple(w.shape))
    wt = _FLIP["done"].get(key)
    if wt is None:
        pend = _FLIP["pending"]
        pend.setdefault(key, w)
        keys = list(pend.keys())
        for k, t in zip(keys, native().conv_wt_flip_multi([pend[k] for k in keys])):
            _FLIP["done"][k] = t
        pend.clear()
        wt = _FLIP["done"][key]
    return wt


def _dres_ok(dres, x) -> bool:
    return (dres is not None and dres.dtype == x.dtype and dres.shape == x.shape
            and dres.is_contiguous(memory_format=_CL))


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int, out_hw, bn_src, res_slot):
        e0 = _mark()
        y = native().conv_fwd(x, w, stride, pad, False, *out_hw)[0]
        _note("fwd", x, w, stride, pad, "plain", e0, out_hw)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad, ctx.bn_src, ctx.res_slot = stride, pad, bn_src, res_slot
        return y

    @staticmethod
    def backward(ctx, dy):
        return _backward(ctx, dy) + (None,) * 5


class _ConvStats(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int, out_hw, bn_src, res_slot):
        e0 = _mark()
        y, ps, pq = native().conv_fwd(x, w, stride, pad, True, *out_hw)
        _note("fwd", x, w, stride, pad, "stats", e0, out_hw)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad, ctx.bn_src, ctx.res_slot = stride, pad, bn_src, res_slot
        ctx.mark_non_differentiable(ps, pq)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the statistics outputs
        return y, ps, pq

    @staticmethod
    def backward(ctx, dy, _dps, _dpq):
        return _backward(ctx, dy) + (None,) * 5


def conv2d(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, bn_stats: bool = False,
           out_hw=(0, 0)) -> torch.Tensor:
    """y = conv2d(x, w, stride, pad) on the MFMA kernels; ``bn_stats`` attaches the output's
    BatchNorm partial sums as ``y._dpt_bn_partials`` (consumed by ops/bn.py).  ``out_hw``:
    explicit output size (asymmetric padding: top/left ``pad``, bottom/right what fits)."""
    w = _cl(w)
    if _FLIP["on"] and int(stride) == 1 and x.requires_grad:
        _FLIP["pending"].setdefault((w.data_ptr(), tuple(w.shape)), w)
    # (BN input, mean, coef) of the fused BN+ReLU that produced x, if any (ops/bn.py)
    bn_src = x.__dict__.get("_dpt_bn_src")
    # x is the identity alias of a fused block tail (this conv is a downsample)
    res_slot = x.__dict__.get("_dpt_res_slot")
    if not bn_stats:
        return _Conv.apply(x, w, int(stride), int(pad), tuple(out_hw), bn_src, res_slot)
    y, ps, pq = _ConvStats.apply(x, w, int(stride), int(pad), tuple(out_hw), bn_src, res_slot)
    y._dpt_bn_partials = (ps, pq)
    return y


# dres_ptr of an entry whose gradient is a block tail's already-masked gradient with no
# identity-path gradient folded in (the last tail, whose output only fed the average pool)
MASKED_NO_RES = -1


def register_bnb_partials(dx: torch.Tensor, p1: torch.Tensor, p2: torch.Tensor, masked: bool = False) -> None:
    """Hand BN backward-statistics partials summed by dx's producer to the BN backward that
    receives dx as its output gradient (other producers than convs: the stem pool for BN+ReLU;
    the average-pool backward for the last block tail, ``masked``: dx is already dz)."""
    _put_bnb(dx, p1, p2, MASKED_NO_RES if masked else None, None)


def take_bnb_partials(dy: torch.Tensor):
    """(p1, p2, dres_ptr, p3) the backward of the conv that consumed a BN output summed for
    ``dy``, once; dres_ptr is None for BN+ReLU, else the data pointer of the identity-path
    gradient that was folded into ``dy`` (block tails); p3: the folded downsample BN's statistic
    (tails with a downsample branch), else None."""
    if not _BNB_PARTIALS:
        return None
    ent = _BNB_PARTIALS.pop(dy.data_ptr(), None)
    if ent is None:
        return None
    gen, ver, p1, p2, shape, dres_ptr, p3 = ent
    if gen != _GEN[0] or ver != dy._version or shape != tuple(dy.shape):
        return None
    return p1, p2, dres_ptr, p3


def take_bn_partials(x: torch.Tensor):
    """The (psum, psq) partials a native conv attached to ``x``, once (None otherwise)."""
    part = x.__dict__.pop("_dpt_bn_partials", None)
    return part


def s2d_stem_supported(x: torch.Tensor, w: torch.Tensor, stride, padding, dilation, groups) -> bool:
    """ResNet's 7x7/2 pad-3 stem on <= 4 input channels: space-to-depth + 4x4 MFMA conv."""
    if not (ENABLED and x.is_cuda and native_available() and x.dim() == 4 and groups == 1
            and x.dtype in (torch.float32, torch.bfloat16) and w.dtype in _DT16):
        return False
    cout, cin, r, s = w.shape
    return (cin <= 4 and cout % 64 == 0 and (r, s) == (7, 7) and tuple(stride) == (2, 2)
            and tuple(padding) == (3, 3) and tuple(dilation) == (1, 1) and not x.requires_grad
            and x.shape[1] == cin and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0
            and x.is_contiguous(memory_format=_CL))


def s2d_stem_conv2d(x: torch.Tensor, w: torch.Tensor, bn_stats: bool = False) -> torch.Tensor:
    """7x7 / stride 2 / pad 3 conv as a 4x4 / stride 1 conv on the 2x2 space-to-depth image.

    With r = 2r' + a - 1 and s = 2s' + b - 1 (r', s' in 0..3, a, b in {0, 1}; tap -1 has zero
    weight) the input row 2*ho - 3 + r is 2*(ho - 2 + r') + a, so
    y[ho, wo] = sum_{r', s'} X2[ho - 2 + r', wo - 2 + s'] . W2[r', s']  with
    X2[i, j, (a*2 + b)*4 + c] = x[2i + a, 2j + b, c] and W2[r', s', (a*2+b)*4 + c] = w[2r'+a-1, 2s'+b-1, c]:
    K = 4*4*16 = 256, each 64-wide K-step four consecutive pixels of one row (the kernels' narrow-
    input path), top/left padding 2, output H/2 x W/2.  The weight re-indexing is plain torch ops,
    so autograd maps the 4x4 weight gradient back onto the 7x7 one."""
    cout, cin = w.shape[0], w.shape[1]
    x2 = native().space_to_depth2(x, w.dtype == torch.float16)
    wk = torch.nn.functional.pad(w.permute(0, 2, 3, 1), (0, 4 - cin, 1, 0, 1, 0))       # [Co, 8, 8, 4]
    w2 = wk.reshape(cout, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(cout, 4, 4, 16)
    w2 = w2.permute(0, 3, 1, 2)                                                         # [Co, 16, 4, 4] cl
    return conv2d(x2, w2, 1, 2, bn_stats, out_hw=(x.shape[2] // 2, x.shape[3] // 2))


def stem_supported(x: torch.Tensor, w: torch.Tensor, stride, padding, dilation, groups) -> bool:
    """Narrow-input conv (any kernel/stride) on the im2col + MFMA GEMM path."""
    if not (ENABLED and x.is_cuda and native_available() and x.dim() == 4 and groups == 1
            and x.dtype in (torch.float32, torch.bfloat16) and w.dtype == torch.bfloat16):
        return False
    cout, cin, r, s = w.shape
    return (cin < 64 and cout % 64 == 0 and not x.requires_grad and tuple(dilation) == (1, 1)
            and stride[0] == stride[1] and padding[0] == padding[1] and x.shape[1] == cin
            and x.is_contiguous(memory_format=_CL))


def stem_conv2d(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, bn_stats: bool = False) -> torch.Tensor:
    """conv2d for a narrow input that needs no input gradient: one im2col kernel writes the
    [pixels, Kp] bf16 patch matrix (Kp = R*S*Cin rounded up to 64, zero-padded), then the 1x1
    MFMA conv (GEMM) with the weight flattened to [Cout, R*S*Cin] (KRSC order) and zero-padded
    - its backward-weight is the 1x1 split-K kernel on the saved patch matrix."""
    cout, cin, r, s = w.shape
    k = r * s * cin
    kp = (k + 63) // 64 * 64
    a = native().im2col(x, r, s, int(stride), int(pad), kp)
    wf = torch.nn.functional.pad(w.permute(0, 2, 3, 1).reshape(cout, k), (0, kp - k))
    return conv2d(a, wf.view(cout, kp, 1, 1), 1, 0, bn_stats)
