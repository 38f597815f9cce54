"""CPU composition of the fused ViT ops (ops/vit.py): same math the GPU kernels implement."""
import torch
import torch.nn.functional as F

from distributed_pytorch_training_amd.ops.vit import add_bias_layer_norm16, bias_gelu16, layer_norm16


def test_cpu_compositions():
    torch.manual_seed(0)
    ln = torch.nn.LayerNorm(256, eps=1e-6)
    x = torch.randn(2, 5, 256)
    a = torch.randn(2, 5, 256).to(torch.bfloat16)
    b = torch.randn(256)
    h = layer_norm16(x, ln, torch.bfloat16)
    assert h.dtype == torch.bfloat16
    torch.testing.assert_close(h.float(), F.layer_norm(x, (256,), ln.weight, ln.bias, 1e-6), rtol=1e-2, atol=2e-2)
    s, h2 = add_bias_layer_norm16(x, a, b, ln)
    torch.testing.assert_close(s, x + a.float() + b)
    assert h2.dtype == torch.bfloat16
    u = torch.randn(10, 64).to(torch.bfloat16)
    g = bias_gelu16(u, torch.zeros(64))
    torch.testing.assert_close(g.float(), F.gelu(u.float()), rtol=1e-2, atol=1e-2)


def test_vit_cpu_forward_unchanged_by_fused_hooks():
    """On CPU (no autocast) the encoder takes the module path: output equals a plain composition."""
    from distributed_pytorch_training_amd.models import build_model

    torch.manual_seed(0)
    m = build_model("vit_b_16", 10, torch.device("cpu"), image_size=32)
    x = torch.randn(2, 3, 32, 32)
    enc = m.encoder
    assert not enc._fused_ok(torch.randn(2, 5, 768))
    out = m(x)
    assert out.shape == (2, 10) and torch.isfinite(out).all()


def test_wgrad_split_choice():
    from distributed_pytorch_training_amd.ops.vit import _wgrad_splits

    T = 128 * 197
    assert _wgrad_splits(3072, 768, T) == 4
    assert _wgrad_splits(2304, 768, T) == 8
    assert _wgrad_splits(768, 768, T) == 16
    assert _wgrad_splits(768, 768, 1000) == 1          # too few rows per split
    assert _wgrad_splits(768, 768, 197 * 3) == 1       # odd token count: no even split


def test_native_patch_embed_matches_conv():
    """set_native's patch embedding (patch rows x one GEMM) against conv_proj: values and the
    conv weight / bias gradients."""
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.models.vit import set_native

    torch.manual_seed(0)
    m = build_model("vit_b_16", 10, torch.device("cpu"), image_size=64)
    with torch.no_grad():
        m.conv_proj.bias.normal_()
    x = torch.randn(3, 3, 64, 64)
    ref = m.patch_embed(x)
    gw = torch.randn_like(ref)
    ref.backward(gw)
    g_ref = (m.conv_proj.weight.grad.clone(), m.conv_proj.bias.grad.clone())
    m.zero_grad()
    assert set_native(m) > 0 and m.dpt_native
    out = m.patch_embed(x)
    assert out.shape == (3, 16, 768)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    out.backward(gw)
    torch.testing.assert_close(m.conv_proj.weight.grad, g_ref[0], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.conv_proj.bias.grad, g_ref[1], rtol=1e-4, atol=1e-4)
