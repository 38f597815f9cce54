"""Fused self-attention autograd op on the gfx950 MFMA kernels (csrc/kernels/attn_kernels.hip).

``attention(qkv, heads)`` takes the QKV projection output ``[B, S, 3*H*64]`` (bf16) and returns
the merged context ``[B, S, H*64]``: softmax(Q K^T / sqrt(64)) V per head, computed by one
workgroup per (image, head) with the whole head on chip.  It replaces head split + SDPA + head
merge of the unfused path (``F.scaled_dot_product_attention`` -> aotriton flash kernels plus
two strided copies), and its backward writes dQ/dK/dV straight into the QKV projection's
gradient layout.  Dropout-free (ViT-B/16 trains with attention dropout 0).
"""
from __future__ import annotations

import math
import os

import torch

from . import native, native_available

ENABLED = os.environ.get("DPT_NATIVE_ATTN", "1") != "0"


def supported(qkv: torch.Tensor, heads: int) -> bool:
    if not (ENABLED and qkv.is_cuda and native_available() and qkv.dtype == torch.bfloat16 and qkv.dim() == 3):
        return False
    b, s, d3 = qkv.shape
    return d3 == 3 * heads * 64 and 1 <= s <= 256


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads: int):
        qkv = qkv.contiguous()
        scale = 1.0 / math.sqrt(64)
        out, lse = native().attn_fwd(qkv, heads, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads, ctx.scale = heads, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dqkv = native().attn_bwd(qkv, out, dout.contiguous().to(torch.bfloat16), lse, ctx.heads, ctx.scale)
        return dqkv, None


def attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    return _Attention.apply(qkv, heads)


def reference_attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    """fp32 PyTorch composition of the same op (test oracle / CPU path)."""
    b, s, d3 = qkv.shape
    dh = d3 // 3 // heads
    q, k, v = qkv.float().view(b, s, 3, heads, dh).permute(2, 0, 3, 1, 4).unbind(0)
    p = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(dh), dim=-1)
    return (p @ v).transpose(1, 2).reshape(b, s, heads * dh)
