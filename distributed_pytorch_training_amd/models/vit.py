"""ViT-B/16 with torchvision-identical parameter names, shapes and init (86,567,656 params).

BASELINE.json config 5 trains ViT-B/16 under DDP to stress large-parameter bucket sizing
(330 MiB of fp32 gradients).  The reference itself only trains ResNet-18
(reference ``train_ddp.py:154``); this module is the model-zoo extension the baseline names.

MI355X notes
------------
* Self-attention runs the fused MFMA kernels of ops/attention.py (csrc/kernels/attn_kernels.hip:
  one workgroup per (image, head), Q/K/V read straight from the QKV projection output, context
  written straight into the out-projection input) for bf16 GPU runs; elsewhere it uses
  ``F.scaled_dot_product_attention`` instead of ``nn.MultiheadAttention``'s unfused path.  The parameters keep ``nn.MultiheadAttention``'s names (``in_proj_weight``,
  ``in_proj_bias``, ``out_proj.*``) so state dicts load into torchvision unchanged.
* 197 tokens (14x14 patches + CLS): no sequence sharding is needed.
* Under bf16/fp16 autocast on the GPU the encoder runs a fused path (ops/vit.py,
  csrc/kernels/vit_kernels.hip): each residual add + branch bias + LayerNorm is one kernel
  that writes the 16-bit GEMM operand directly, fc1's bias + GELU is one kernel, and the
  backward passes fold the bias-gradient column sums and residual-gradient adds into the
  same passes.  The branch GEMMs run bias-free; parameter names/shapes are unchanged.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.vit import (add_bias_layer_norm16, gelu_linear16, layer_norm16, linear16, ln_fusable, merge_heads,
                       split_heads)
from ..ops import attention as fused_attn
from ..parallel.shadow import shadow_param


class SelfAttention(nn.Module):
    dpt_shadow_names = ("in_proj_weight", "in_proj_bias")  # 16-bit weight shadows (parallel/shadow.py)
    # False: stock PyTorch ops (F.linear, scaled_dot_product_attention) - what torchvision's
    # nn.MultiheadAttention runs, and what the stock engine (--impl torch) must measure.  The
    # native engine turns it on (set_native): split-K linear backward, the gfx950 attention kernels.
    dpt_native = False
    native_patch = os.environ.get("DPT_VIT_NATIVE_PATCH", "1") != "0"   # A/B knob

    def __init__(self, dim: int, heads: int, dropout: float = 0.0) -> None:
        super().__init__()
        self.dim, self.heads, self.dropout = dim, heads, dropout
        self.in_proj_weight = nn.Parameter(torch.empty(3 * dim, dim))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * dim))
        self.out_proj = nn.Linear(dim, dim)
        # nn.MultiheadAttention._reset_parameters
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def _context(self, x: torch.Tensor) -> torch.Tensor:
        b, s, d = x.shape
        if not self.dpt_native:
            qkv = F.linear(x, self.in_proj_weight, self.in_proj_bias)
            q, k, v = qkv.view(b, s, 3, self.heads, d // self.heads).permute(2, 0, 3, 1, 4).unbind(0)
            y = F.scaled_dot_product_attention(q, k, v, dropout_p=self.dropout if self.training else 0.0)
            return y.transpose(1, 2).reshape(b, s, d)
        qkv = linear16(x, shadow_param(self, "in_proj_weight", x), shadow_param(self, "in_proj_bias", x))
        if (not self.training or self.dropout == 0.0) and fused_attn.supported(qkv, self.heads):
            return fused_attn.attention(qkv, self.heads)  # heads split/merged inside the kernels
        q, k, v = split_heads(qkv, self.heads)
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=self.dropout if self.training else 0.0)
        return merge_heads(y)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.out_proj(self._context(x))

    def attend_nobias(self, x: torch.Tensor):
        """(out_proj(context) without its bias, the bias) - the fused path adds the bias in
        the following add+LayerNorm kernel."""
        y = self._context(x)
        return linear16(y, shadow_param(self.out_proj, "weight", y)), _bias16(self.out_proj, "bias", y)


def _bias16(mod: nn.Module, name: str, like: torch.Tensor) -> torch.Tensor:
    """A bias the fused kernels add to a 16-bit GEMM output: the bf16 weight shadow, or (no
    shadows) the fp32 master rounded the way autocast's cast of nn.Linear's bias rounds it - the
    two engines then compute the same values (tests/test_engine_gpu.py weight-shadow test)."""
    b = shadow_param(mod, name, like)
    if (b.dtype != like.dtype and like.dtype in (torch.bfloat16, torch.float16)
            and torch.is_autocast_enabled(like.device.type)):
        b = b.to(like.dtype)
    return b


class MLPBlock(nn.Sequential):
    """Linear(0) - GELU(1) - Dropout(2) - Linear(3) - Dropout(4), torchvision key layout."""

    def __init__(self, dim: int, mlp_dim: int, dropout: float) -> None:
        super().__init__(nn.Linear(dim, mlp_dim), nn.GELU(), nn.Dropout(dropout),
                         nn.Linear(mlp_dim, dim), nn.Dropout(dropout))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.normal_(m.bias, std=1e-6)


class EncoderBlock(nn.Module):
    def __init__(self, heads: int, dim: int, mlp_dim: int, dropout: float, attn_dropout: float) -> None:
        super().__init__()
        self.ln_1 = nn.LayerNorm(dim, eps=1e-6)
        self.self_attention = SelfAttention(dim, heads, attn_dropout)
        self.dropout = nn.Dropout(dropout)
        self.ln_2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = MLPBlock(dim, mlp_dim, dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x + self.dropout(self.self_attention(self.ln_1(x)))
        return x + self.mlp(self.ln_2(x))


class Encoder(nn.Module):
    dpt_native = False   # the fused encoder path (set_native); stock module-by-module otherwise

    def __init__(self, seq_len: int, layers: int, heads: int, dim: int, mlp_dim: int,
                 dropout: float, attn_dropout: float) -> None:
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_len, dim).normal_(std=0.02))
        self.dropout = nn.Dropout(dropout)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", EncoderBlock(heads, dim, mlp_dim, dropout, attn_dropout))
            for i in range(layers)))
        self.ln = nn.LayerNorm(dim, eps=1e-6)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._fused_ok(x):
            return self._forward_fused(x)
        return self.ln(self.layers(self.dropout(x + self.pos_embedding)))

    def _fused_ok(self, x: torch.Tensor) -> bool:
        if not self.dpt_native:
            return False
        if not (x.is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") in (torch.bfloat16, torch.float16)):
            return False
        if not ln_fusable(x, x.shape[-1]):
            return False
        if self.training and any(isinstance(m, nn.Dropout) and m.p > 0 for m in self.modules()):
            return False
        blk = self.layers[0]
        return (blk.mlp[0].out_features % 8 == 0 and not (self.training and blk.self_attention.dropout > 0))

    def _forward_fused(self, x: torch.Tensor) -> torch.Tensor:
        dt = torch.get_autocast_dtype("cuda")
        x = (x + self.pos_embedding).float().contiguous()
        pending = None                    # (branch GEMM output without bias, its bias)
        for blk in self.layers:
            if pending is None:
                h = layer_norm16(x, blk.ln_1, dt)
            else:
                x, h = add_bias_layer_norm16(x, pending[0], pending[1], blk.ln_1)
            a, ab = blk.self_attention.attend_nobias(h)
            x, h2 = add_bias_layer_norm16(x, a, ab, blk.ln_2)
            fc1, fc2 = blk.mlp[0], blk.mlp[3]
            u = linear16(h2, shadow_param(fc1, "weight", h2))
            z = gelu_linear16(u, _bias16(fc1, "bias", h2), shadow_param(fc2, "weight", h2))
            pending = (z, _bias16(fc2, "bias", h2))
        return add_bias_layer_norm16(x, pending[0], pending[1], self.ln)[1]


class VisionTransformer(nn.Module):
    # native path (set_native): the patch embedding as one GEMM over the patch rows.  The conv
    # has stride == kernel, so its im2col is a pure reshape; MIOpen runs it as an implicit-GEMM
    # conv in both directions (~0.29 ms per B128 step, plus a find-mode search over naive
    # solvers on the first step); here a patch copy, a hipBLASLt forward GEMM and the native
    # split-K weight gradient of linear16.
    dpt_native = False
    native_patch = os.environ.get("DPT_VIT_NATIVE_PATCH", "1") != "0"   # A/B knob

    def __init__(self, image_size: int = 224, patch_size: int = 16, layers: int = 12,
                 heads: int = 12, dim: int = 768, mlp_dim: int = 3072, num_classes: int = 1000,
                 dropout: float = 0.0, attn_dropout: float = 0.0) -> None:
        super().__init__()
        if image_size % patch_size:
            raise ValueError(f"image_size {image_size} not divisible by patch_size {patch_size}")
        self.image_size, self.patch_size, self.dim = image_size, patch_size, dim
        self.conv_proj = nn.Conv2d(3, dim, kernel_size=patch_size, stride=patch_size)
        seq_len = (image_size // patch_size) ** 2 + 1
        self.class_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.encoder = Encoder(seq_len, layers, heads, dim, mlp_dim, dropout, attn_dropout)
        self.heads = nn.Sequential(OrderedDict(head=nn.Linear(dim, num_classes)))

        fan_in = 3 * patch_size * patch_size
        nn.init.trunc_normal_(self.conv_proj.weight, std=math.sqrt(1 / fan_in))
        nn.init.zeros_(self.conv_proj.bias)
        nn.init.zeros_(self.heads.head.weight)
        nn.init.zeros_(self.heads.head.bias)

    def patch_embed(self, x: torch.Tensor) -> torch.Tensor:
        """[N, 3, H, W] images -> [N, patches, dim] tokens (conv_proj's output, row-major)."""
        if not (self.dpt_native and self.native_patch):
            return self.conv_proj(x).flatten(2).transpose(1, 2)
        n, c, hh, ww = x.shape
        p = self.patch_size
        if torch.is_autocast_enabled(x.device.type):
            x = x.to(torch.get_autocast_dtype(x.device.type))   # cast before the patch copy
        rows = (x.reshape(n, c, hh // p, p, ww // p, p).permute(0, 2, 4, 1, 3, 5)
                .reshape(n * (hh // p) * (ww // p), c * p * p))    # (c, kh, kw): the weight's order
        w = shadow_param(self.conv_proj, "weight", rows)
        # linear16: split-K / native weight gradient (K = patch rows, 25,088 at B128)
        y = linear16(rows, w.reshape(self.dim, -1), shadow_param(self.conv_proj, "bias", rows))
        return y.view(n, (hh // p) * (ww // p), self.dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        n = x.shape[0]
        x = self.patch_embed(x)                                    # [N, 196, 768]
        x = torch.cat([self.class_token.expand(n, -1, -1), x], dim=1)
        x = self.encoder(x)
        return self.heads(x[:, 0])


def set_native(model: nn.Module, on: bool = True) -> int:
    """Route a ViT's encoder through the native fused path (on) or stock PyTorch ops (off, the
    default of a freshly built model); returns how many modules were switched."""
    n = 0
    for m in model.modules():
        if isinstance(m, (SelfAttention, Encoder, VisionTransformer)):
            m.dpt_native = bool(on)
            n += 1
    return n


def vit_b_16(num_classes: int = 1000, image_size: int = 224, **kw) -> VisionTransformer:
    return VisionTransformer(image_size=image_size, patch_size=16, layers=12, heads=12,
                             dim=768, mlp_dim=3072, num_classes=num_classes, **kw)
