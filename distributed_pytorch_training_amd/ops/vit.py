"""Fused transformer-block ops for ViT on the gfx950 kernels (csrc/kernels/vit_kernels.hip).

* ``layer_norm16(x, ln)``               h = LayerNorm(x) written directly in 16 bits
* ``add_bias_layer_norm16(x, a, b, ln)`` s = x + a + b (fp32 residual stream), h = LayerNorm(s)
                                        in 16 bits; backward gives the residual gradient,
                                        the branch gradient (16-bit) and the branch bias
                                        gradient in one pass
* ``bias_gelu16(u, b)``                 gelu(u + b) (exact erf), backward with the bias-gradient
                                        column sums fused
* ``split_heads(qkv, h)`` / ``merge_heads(y)``  attention head layout changes: the backward of
                                        the split writes dq/dk/dv straight into one [b, s, 3D]
                                        gradient (no stack + transpose copy), the merge is one
                                        vectorised strided copy

``a`` / ``u`` are the outputs of bias-free GEMMs (``F.linear(h, W)``): the bias add moves into
these kernels so the bias gradient falls out of the pass that already reads the gradient
(no separate column-sum kernel per Linear).  Semantics equal the unfused PyTorch composition
under autocast up to rounding order (the fused path adds the bias in fp32 before rounding,
PyTorch rounds the GEMM+bias output to bf16 first); tests compare both against fp32.

CPU tensors run the PyTorch composition (same function signatures) so the model code has
one path.
"""
from __future__ import annotations

import os

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import native, native_available

_KIND = {torch.bfloat16: 1, torch.float16: 2}
_PKIND = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def ln_fusable(x: torch.Tensor, dim: int) -> bool:
    return x.is_cuda and native_available() and native().ln_supported(dim)


def _c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else t.contiguous()


class _LayerNorm16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, kind):
        _, h, mean, rstd = native().ln_fwd(x, None, None, weight, bias, float(eps), int(kind))
        ctx.save_for_backward(x, weight, mean, rstd)
        return h

    @staticmethod
    def backward(ctx, gh):
        x, weight, mean, rstd = ctx.saved_tensors
        want_p = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        gx, _, dg, db, _ = native().ln_bwd(None, gh.contiguous(), x, mean, rstd, weight, False, None, want_p)
        return gx, (dg if want_p else None), (db if want_p else None), None, None


class _AddBiasLayerNorm16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a, abias, weight, bias, eps):
        s, h, mean, rstd = native().ln_fwd(x, a, abias, weight, bias, float(eps), 1)
        ctx.save_for_backward(s, weight, mean, rstd, abias)
        ctx.a_dtype = a.dtype
        ctx.set_materialize_grads(False)
        return s, h

    @staticmethod
    def backward(ctx, gs, gh):
        s, weight, mean, rstd, abias = ctx.saved_tensors
        if gh is None:  # only the residual stream is used downstream: LN contributes nothing
            ga = None if gs is None else gs.to(ctx.a_dtype)
            return gs, ga, (None if gs is None or abias is None else gs.flatten(0, -2).sum(0).to(abias.dtype)), \
                None, None, None
        want_p = ctx.needs_input_grad[3] or ctx.needs_input_grad[4]
        gx, ga, dg, db, dab = native().ln_bwd(_c(gs), gh.contiguous(), s, mean, rstd, weight, True,
                                              abias, want_p)
        return (gx, ga, dab if abias is not None else None, dg if want_p else None,
                db if want_p else None, None)


class _BiasGELU16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, bias):
        ctx.save_for_backward(u, bias)
        return native().gelu_fwd(u, bias)

    @staticmethod
    def backward(ctx, gh):
        u, bias = ctx.saved_tensors
        gu, db = native().gelu_bwd(gh.contiguous(), u, bias, bias is not None and ctx.needs_input_grad[1])
        return gu, (db if bias is not None and ctx.needs_input_grad[1] else None)


class _SplitHeads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads):
        b, s, d3 = qkv.shape
        dh = d3 // 3 // heads
        ctx.shape = (b, s, heads, dh)
        v5 = qkv.view(b, s, 3, heads, dh).permute(2, 0, 3, 1, 4)
        return v5[0], v5[1], v5[2]

    @staticmethod
    def backward(ctx, dq, dk, dv):
        b, s, h, dh = ctx.shape
        ref = next(g for g in (dq, dk, dv) if g is not None)
        out = torch.empty(b, s, 3, h, dh, dtype=ref.dtype, device=ref.device)
        o5 = out.permute(2, 0, 3, 1, 4)
        C = native()
        for i, g in enumerate((dq, dk, dv)):
            if g is None:
                o5[i].zero_()
            else:
                C.copy_rows16(g if g.stride(-1) == 1 else g.contiguous(), o5[i])
        return out.view(b, s, 3 * h * dh), None


class _MergeHeads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y):
        b, h, s, dh = y.shape
        ctx.shape = (b, h, s, dh)
        out = torch.empty(b, s, h, dh, dtype=y.dtype, device=y.device)
        native().copy_rows16(y if y.stride(-1) == 1 else y.contiguous(), out.permute(0, 2, 1, 3))
        return out.view(b, s, h * dh)

    @staticmethod
    def backward(ctx, g):
        b, h, s, dh = ctx.shape
        return g.view(b, s, h, dh).permute(0, 2, 1, 3)


def heads_fusable(t: torch.Tensor, head_dim: int) -> bool:
    return (t.is_cuda and t.dtype in _KIND and head_dim % 8 == 0 and native_available())


def split_heads(qkv: torch.Tensor, heads: int):
    """[b, s, 3*D] -> q, k, v [b, heads, s, D/heads] (views)."""
    if heads_fusable(qkv, qkv.shape[-1] // 3 // heads):
        return _SplitHeads.apply(qkv, heads)
    b, s, d3 = qkv.shape
    return qkv.view(b, s, 3, heads, d3 // 3 // heads).permute(2, 0, 3, 1, 4).unbind(0)


def merge_heads(y: torch.Tensor) -> torch.Tensor:
    """[b, h, s, dh] -> [b, s, h*dh] contiguous."""
    b, h, s, dh = y.shape
    if heads_fusable(y, dh):
        return _MergeHeads.apply(y)
    return y.transpose(1, 2).reshape(b, s, h * dh)


# ---------------------------------------------------------------------------------------------
def layer_norm16(x: torch.Tensor, ln: torch.nn.LayerNorm, dtype: torch.dtype) -> torch.Tensor:
    """LayerNorm(x) (x fp32) returned in ``dtype`` (bf16/fp16)."""
    if x.is_cuda:
        return _LayerNorm16.apply(x.contiguous(), ln.weight, ln.bias, ln.eps, _KIND[dtype])
    return F.layer_norm(x, ln.normalized_shape, ln.weight, ln.bias, ln.eps).to(dtype)


def add_bias_layer_norm16(x: torch.Tensor, a: torch.Tensor, abias: Optional[torch.Tensor],
                          ln: torch.nn.LayerNorm) -> Tuple[torch.Tensor, torch.Tensor]:
    """(s, h) with s = x + a + abias (fp32) and h = LayerNorm(s) in a's dtype."""
    if x.is_cuda:
        return _AddBiasLayerNorm16.apply(x.contiguous(), a.contiguous(), abias, ln.weight, ln.bias, ln.eps)
    s = x + a.float() + (abias.float() if abias is not None else 0.0)
    return s, F.layer_norm(s, ln.normalized_shape, ln.weight, ln.bias, ln.eps).to(a.dtype)


def bias_gelu16(u: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    if u.is_cuda:
        return _BiasGELU16.apply(u.contiguous(), bias)
    z = u.float() + (bias.float() if bias is not None else 0.0)
    return F.gelu(z).to(u.dtype)


# ---- Linear with split-K weight gradient ------------------------------------------------------
def _wgrad_splits(n_out: int, n_in: int, T: int) -> int:
    """Batch-split count for dW = dY^T X with K = T tokens.  One [n_out x n_in] output has only
    ceil(n_out/256)*ceil(n_in/256) macro tiles (9..36 for ViT-B) for 256 CUs; splitting K into
    S batched GEMMs multiplies the tile count.  Measured on MI355X (bench/wgrad_splitk.py,
    T = 25,216): best S = 4 for 36 tiles, 8 for 27, 16 for 9."""
    tiles = -(-n_out // 256) * -(-n_in // 256)
    s = 4 if tiles >= 32 else (8 if tiles >= 16 else 16)
    while s > 1 and (T % s or T // s < 1024):
        s //= 2
    return s


# dW = dY^T X on the native MFMA backward-weight kernel of the 1x1 convolutions (a [1, 1, T, C]
# channels-last "image"; split-K with fp32 partials and a fixed-order reduce, deterministic) for
# inputs up to this many features; hipBLASLt's split-K batched GEMM above it.  ViT-B/16 at batch
# 128 (bench/vit_wgrad_ab.py, profiles/vit_wgrad_ab_r5.md): qkv 126 vs 138 us, proj 53 vs 64, fc1
# 150 vs 153, fc2 155 vs 141; step 23.65 vs 23.88 ms.  0 disables.  NATIVE_WGRAD_BLOCKS > 0 aims
# the split-K at that many blocks instead of the 1x1-conv policy's 512: 768 is 2-15 % faster per
# product in isolation but level in the step (profiles/vit_wgrad_ab_r5.md), so it stays 0.
NATIVE_WGRAD_MAX_IN = int(os.environ.get("DPT_VIT_NATIVE_WGRAD_MAX_IN", "1024"))
NATIVE_WGRAD_BLOCKS = 0


def _native_wgrad_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    n_out, n_in = dy.shape[1], x.shape[1]
    return (dy.is_cuda and native_available() and dy.dtype == x.dtype and dy.dtype in _KIND
            and n_in <= NATIVE_WGRAD_MAX_IN and n_out % 64 == 0 and n_in % 64 == 0 and dy.shape[0] < (1 << 31))


def wgrad_splitk(dy: torch.Tensor, x: torch.Tensor, out_dtype: torch.dtype) -> torch.Tensor:
    """dY^T X ([T, n_out], [T, n_in] -> [n_out, n_in]) as split-K with fp32 partials."""
    T, n_out = dy.shape
    n_in = x.shape[1]
    if _native_wgrad_ok(dy, x) and out_dtype in (torch.float32, dy.dtype):
        cl = torch.channels_last
        dy4 = dy.view(1, 1, T, n_out).permute(0, 3, 1, 2)      # [1, n_out, 1, T], channels_last
        x4 = x.view(1, 1, T, n_in).permute(0, 3, 1, 2)
        if dy4.is_contiguous(memory_format=cl) and x4.is_contiguous(memory_format=cl):
            dw = native().conv_wgrad(dy4, x4, [n_out, n_in, 1, 1], 1, 0, out_dtype == torch.float32,
                                     NATIVE_WGRAD_BLOCKS)
            return dw.view(n_out, n_in)
    s = _wgrad_splits(n_out, n_in, T)
    if s == 1:
        return (dy.t() @ x).to(out_dtype)
    part = torch.bmm(dy.view(s, T // s, n_out).transpose(1, 2), x.view(s, T // s, n_in),
                     out_dtype=torch.float32)
    if native_available() and (n_out * n_in) % 4 == 0:
        return native().sum_partials(part, _PKIND[out_dtype])   # sum + cast in one pass
    return part.sum(0).to(out_dtype)


def _to(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    return t if t.dtype == dtype else t.to(dtype)


class _Linear16(torch.autograd.Function):
    """y = x W^T (+ b) on 16-bit operands; backward computes dW as a split-K batched GEMM
    (hipBLASLt's single-GEMM choice leaves most CUs idle on these long-K shapes)."""

    @staticmethod
    def forward(ctx, x, w, b):
        w16 = w if w.dtype == x.dtype else w.to(x.dtype)
        b16 = None if b is None else (b if b.dtype == x.dtype else b.to(x.dtype))
        ctx.save_for_backward(x, w16)
        ctx.w_dtype = w.dtype
        ctx.b_dtype = None if b is None else b.dtype
        return F.linear(x, w16, b16)

    @staticmethod
    def backward(ctx, dy):
        x, w16 = ctx.saved_tensors
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dx = (dy2 @ w16).view(shp) if ctx.needs_input_grad[0] else None
        # autocast semantics for fp32 masters (no weight shadows): the gradient of the 16-bit
        # weight / bias copy, rounded once, then cast back - what F.linear on autocast's casts gives
        dw = _to(wgrad_splitk(dy2, x2, w16.dtype), ctx.w_dtype) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.b_dtype is not None and ctx.needs_input_grad[2]:
            if dy2.shape[1] % 8 == 0 and dy2.dtype in _KIND:
                db = _to(native().bias_grad16(dy2, _PKIND[dy2.dtype]), ctx.b_dtype)
            else:
                db = dy2.sum(0, dtype=torch.float32).to(dy2.dtype).to(ctx.b_dtype)
        return dx, dw, db


# fc2's backward-data and GELU's backward in one launch (conv_fwd_kernel's DGELU epilogue):
# gu = (dz W2) * gelu'(u + b1) with the bias-gradient column sums, instead of a hipBLASLt GEMM
# writing gh and a GELU pass re-reading it.  DPT_VIT_FUSED_DGELU=0 keeps the two launches (A/B).
FUSED_DGELU = os.environ.get("DPT_VIT_FUSED_DGELU", "1") != "0"


class _GeluLinear16(torch.autograd.Function):
    """z = gelu(u + b1) W2^T on 16-bit operands (ViT's MLP after fc1), with the fused backward."""

    @staticmethod
    def forward(ctx, u, b1, w2):
        w16 = w2 if w2.dtype == u.dtype else w2.to(u.dtype)
        h = native().gelu_fwd(u, b1)
        ctx.save_for_backward(u, b1, h, w16)
        ctx.w_dtype = w2.dtype
        return F.linear(h, w16)

    @staticmethod
    def backward(ctx, gz):
        u, b1, h, w16 = ctx.saved_tensors
        n_in, n_out = u.shape[-1], gz.shape[-1]
        gz2 = gz.reshape(-1, n_out).contiguous()
        u2 = u.reshape(-1, n_in)
        dw2 = _to(wgrad_splitk(gz2, h.reshape(-1, n_in), w16.dtype), ctx.w_dtype) if ctx.needs_input_grad[2] else None
        gu = db1 = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            bk = b1 if b1.dtype in (u.dtype, torch.float32) else b1.float()    # 16-bit: read as is
            gu, part = native().linear_dgrad_dgelu(gz2, _transpose16(w16), u2, bk.contiguous())
            gu = gu.view(u.shape)
            if ctx.needs_input_grad[1]:
                # sum over tiles + cast in one pass (16-bit like autocast's bias copy, then b1's dtype)
                db1 = _to(native().colsum_rows(part, _PKIND[u.dtype]), b1.dtype)
        return gu, db1, dw2


def _transpose16(w: torch.Tensor) -> torch.Tensor:
    """W^T of a contiguous 16-bit [n_out, n_in] weight through the tiled weight-flip kernel (a 1x1
    conv weight's [Cout, C] -> [C, Cout]): ~3x faster than the strided copy of .t().contiguous()."""
    n_out, n_in = w.shape
    if w.is_contiguous() and w.data_ptr() % 16 == 0 and n_out % 8 == 0:
        return native().conv_wt_flip_multi([w.view(n_out, n_in, 1, 1)])[0].view(n_in, n_out)
    return w.t().contiguous()


def gelu_linear16(u: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """linear16(bias_gelu16(u, b1), w2) with fc2's backward-data and GELU's backward fused."""
    n_in, n_out = u.shape[-1], w2.shape[0]
    if (FUSED_DGELU and u.is_cuda and native_available() and u.dtype in _KIND and u.is_contiguous()
            and b1 is not None and n_in % 128 == 0 and n_out % 64 == 0):
        return _GeluLinear16.apply(u, b1, w2)
    return linear16(bias_gelu16(u, b1), w2)


def linear16(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """F.linear for 16-bit activations (autocast region) with the split-K weight gradient."""
    if x.is_cuda and x.dtype in _KIND and x.is_contiguous():
        return _Linear16.apply(x, w, b)
    return F.linear(x, w, b)
