"""16-bit weight shadows for mixed-precision training.

Under ``torch.autocast`` every convolution / linear layer casts its fp32 weight to bf16 on
every forward (one cast kernel per weight: 57 launches per ResNet-50 step) and autograd casts
the bf16 weight gradient back to fp32 (another 56).  Here the fused optimizer keeps a bf16
copy of the whole parameter arena up to date in the same pass that updates the fp32 master
weights (2 extra bytes per parameter), the layers read that copy directly, and the C++
reducer converts their bf16 gradients to fp32 while it gathers them into the arena.  The
values are bit-identical to autocast's (the same fp32->bf16 rounding of the same master
weight), so this is a pure data-movement optimisation.

Shadows are leaf tensors (views into ``shadow_flat``, laid out exactly like the fp32 arena)
that require grad; the master parameters stay the module's registered ``Parameter``s, so
``state_dict`` / checkpoints are unchanged.  Only used while autocast is active with the
shadow dtype; otherwise layers fall back to their fp32 weights.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.conv_f32 import NativeConv2d
from ..ops import conv as native_conv

SHADOW_ATTR = "_dpt_shadow"


def active_shadow(mod: nn.Module, x: torch.Tensor):
    sh = mod.__dict__.get(SHADOW_ATTR)
    if not sh or not x.is_cuda or not torch.is_autocast_enabled("cuda"):
        return None
    if torch.get_autocast_dtype("cuda") != next(iter(sh.values())).dtype:
        return None
    return sh


class ShadowConv2d(NativeConv2d):
    # set by fuse_native_layers on convs that feed a fused BatchNorm: the native conv's
    # epilogue then also emits the BN statistics partials
    dpt_bn_stats = False
    # per-model conv routing, set by models.layers.fuse_native_layers (None: ops/conv.py defaults)
    dpt_native_conv = True
    dpt_min_pixels = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        sh = active_shadow(self, x)
        if sh is None:
            return super().forward(x)          # NativeConv2d: the fp32 MFMA path, or nn.Conv2d
        w, b = sh["weight"], sh.get("bias", self.bias)
        if not self.dpt_native_conv:
            return nn.Conv2d._conv_forward(self, x, w, b)
        if b is None and native_conv.supported(x, w, self.stride, self.padding, self.dilation, self.groups,
                                               self.dpt_min_pixels):
            return native_conv.conv2d(x, w, self.stride[0], self.padding[0], self.dpt_bn_stats)
        if b is None and native_conv.s2d_stem_supported(x, w, self.stride, self.padding, self.dilation, self.groups):
            return native_conv.s2d_stem_conv2d(x, w, self.dpt_bn_stats)
        if (b is None and native_conv.STEM_ENABLED
                and native_conv.stem_supported(x, w, self.stride, self.padding, self.dilation, self.groups)):
            return native_conv.stem_conv2d(x, w, self.stride[0], self.padding[0], self.dpt_bn_stats)
        return self._conv_forward(x, w, b)


class ShadowLinear(nn.Linear):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        sh = active_shadow(self, x)
        if sh is None:
            return super().forward(x)
        return F.linear(x, sh["weight"], sh.get("bias", self.bias))


def shadow_param(mod: nn.Module, name: str, x: torch.Tensor) -> torch.Tensor:
    """For modules that use raw Parameters in F.* calls (ViT's fused in-projection)."""
    sh = active_shadow(mod, x)
    if sh is not None and name in sh:
        return sh[name]
    return getattr(mod, name)


_SWAP = {nn.Conv2d: ShadowConv2d, NativeConv2d: ShadowConv2d, nn.Linear: ShadowLinear}


def install_shadows(module: nn.Module, arena, dtype: torch.dtype) -> Tuple[torch.Tensor, Dict[int, torch.Tensor]]:
    """Create the shadow arena for ``arena`` and point every conv/linear at its shadows.

    Returns (shadow_flat, {arena parameter index: shadow leaf}).
    """
    index = {id(p): i for i, p in enumerate(arena.params)}
    shadow_flat = arena.param_flat.detach().to(dtype)
    leaves: Dict[int, torch.Tensor] = {}
    for mod in module.modules():
        cls = type(mod)
        if cls in _SWAP or cls in _SWAP.values():
            names = ("weight", "bias")
        else:
            names = getattr(mod, "dpt_shadow_names", ())
        d = {}
        for n in names:
            p = mod._parameters.get(n)
            if p is None or id(p) not in index:
                continue
            i = index[id(p)]
            off = arena.offsets[i]
            leaf = torch.as_strided(shadow_flat, p.shape, p.stride(), off).detach().requires_grad_(True)
            leaves[i] = leaf
            d[n] = leaf
        if d:
            mod.__dict__[SHADOW_ATTR] = d
            if cls in _SWAP:
                mod.__class__ = _SWAP[cls]
    return shadow_flat, leaves
