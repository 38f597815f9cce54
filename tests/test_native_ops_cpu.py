"""CPU-side checks of the MFMA conv / attention integration (no GPU needed): the conv->BN
tagging, the space-to-depth stem algebra, the attention oracle, and that the native ops never
claim CPU tensors."""
import torch
import torch.nn.functional as F

from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.models.layers import FusedBatchNorm2d, fuse_native_layers
from distributed_pytorch_training_amd.ops import attention as fa
from distributed_pytorch_training_amd.ops import conv as nc


def test_every_resnet50_conv_feeds_a_fused_bn():
    m = build_model("resnet50", 1000)
    fuse_native_layers(m)
    convs = [mod for mod in m.modules() if isinstance(mod, torch.nn.Conv2d)]
    assert len(convs) == 53
    assert all(getattr(c, "dpt_bn_stats", False) for c in convs)
    assert sum(isinstance(mod, FusedBatchNorm2d) for mod in m.modules()) == 53


def _space_to_depth2(x):
    n, c, h, w = x.shape
    xc = x.permute(0, 2, 3, 1)
    out = torch.zeros(n, h // 2, w // 2, 16, dtype=x.dtype)
    for a in range(2):
        for b in range(2):
            out[..., (a * 2 + b) * 4:(a * 2 + b) * 4 + c] = xc[:, a::2, b::2, :]
    return out.permute(0, 3, 1, 2)


def test_space_to_depth_stem_algebra():
    """The 7x7/2 pad-3 conv equals the 4x4/1 top-left-pad-2 conv on the 2x2 space-to-depth
    image with the weight re-indexed exactly as ops/conv.py s2d_stem_conv2d does."""
    torch.manual_seed(0)
    x = torch.randn(2, 3, 34, 30, dtype=torch.float64)
    w = torch.randn(64, 3, 7, 7, dtype=torch.float64)
    ref = F.conv2d(x, w, stride=2, padding=3)
    wk = F.pad(w.permute(0, 2, 3, 1), (0, 1, 1, 0, 1, 0))
    w2 = wk.reshape(64, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(64, 4, 4, 16).permute(0, 3, 1, 2)
    y = F.conv2d(_space_to_depth2(x), w2, padding=2)[:, :, :17, :15]
    torch.testing.assert_close(y, ref, rtol=1e-10, atol=1e-10)


def test_attention_oracle_matches_sdpa():
    torch.manual_seed(1)
    qkv = torch.randn(2, 197, 3 * 4 * 64)
    q, k, v = qkv.view(2, 197, 3, 4, 64).permute(2, 0, 3, 1, 4).unbind(0)
    want = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(2, 197, 256)
    torch.testing.assert_close(fa.reference_attention(qkv, 4), want, rtol=1e-5, atol=1e-5)


def test_native_ops_never_claim_cpu_tensors():
    x = torch.randn(2, 64, 8, 8).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 64, 3, 3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not nc.supported(x, w, (1, 1), (1, 1), (1, 1), 1)
    assert not nc.s2d_stem_supported(torch.randn(2, 3, 32, 32), w[:, :3, :1, :1], (2, 2), (3, 3), (1, 1), 1)
    assert not fa.supported(torch.randn(2, 5, 3 * 64).to(torch.bfloat16), 1)
