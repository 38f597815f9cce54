"""Fused MFMA self-attention (csrc/kernels/attn_kernels.hip) vs an fp32 PyTorch reference."""
import math

import pytest
import torch

from distributed_pytorch_training_amd import ops
from distributed_pytorch_training_amd.ops import attention as fa

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,S,H", [(2, 197, 12), (3, 64, 2), (1, 33, 4), (2, 256, 3), (4, 5, 1)])
def test_attention_fwd_bwd_matches_fp32(cuda, B, S, H):
    g = torch.Generator(device=cuda).manual_seed(S + H)
    qkv = (torch.randn(B, S, 3 * H * 64, device=cuda, generator=g) * 1.5).to(torch.bfloat16)
    qkv.requires_grad_(True)
    out = fa.attention(qkv, H)
    ref_in = qkv.detach().float().requires_grad_(True)
    ref = fa.reference_attention(ref_in, H)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    # lse2 matches log2-sum-exp of the scaled scores
    _, lse = ops.native().attn_fwd(qkv.detach(), H, 1 / 8)
    q, k, _ = ref_in.detach().view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    want = torch.logsumexp(q @ k.transpose(-1, -2) / 8, dim=-1) / math.log(2)
    torch.testing.assert_close(lse.view(B * H, -1)[:, :S], want.reshape(B * H, S), rtol=1e-3, atol=2e-2)
    dout = torch.randn(B, S, H * 64, device=cuda, generator=g).to(torch.bfloat16)
    out.backward(dout)
    ref.backward(dout.float())
    gq, gr = qkv.grad.float(), ref_in.grad
    scale = gr.abs().max().item()
    torch.testing.assert_close(gq, gr, rtol=3e-2, atol=2e-2 * scale)
    assert ((gq - gr).norm() / gr.norm()).item() < 2e-2


def test_vit_uses_fused_attention(cuda):
    from distributed_pytorch_training_amd.models import build_model

    from distributed_pytorch_training_amd.models.vit import set_native

    m = build_model("vit_b_16", 10, cuda, image_size=32).train()
    assert set_native(m) > 0
    x = torch.randn(2, 3, 32, 32, device=cuda)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = m(x)
    fa.ENABLED = False
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y2 = m(x)
    finally:
        fa.ENABLED = True
    torch.testing.assert_close(y1.float(), y2.float(), rtol=5e-2, atol=5e-2)


def test_attention_bwd_phase_split_is_bitwise_identical(cuda):
    """The backward as two phase kernels (dK/dV over Q and dO images, dQ over K and V images,
    the ViT-B/16 default) computes exactly what the one two-phase kernel does."""
    C = ops.native()
    g = torch.Generator(device=cuda).manual_seed(5)
    B, S, H = 3, 197, 4
    qkv = (torch.randn(B, S, 3 * H * 64, device=cuda, generator=g) * 1.5).to(torch.bfloat16)
    dout = torch.randn(B, S, H * 64, device=cuda, generator=g).to(torch.bfloat16)
    out, lse = C.attn_fwd(qkv, H, 0.125)
    try:
        C.attn_set_bwd_split(0)
        one = C.attn_bwd(qkv, out, dout, lse, H, 0.125)
        C.attn_set_bwd_split(1)
        split = C.attn_bwd(qkv, out, dout, lse, H, 0.125)
    finally:
        C.attn_set_bwd_split(1)
    assert torch.equal(one, split)
