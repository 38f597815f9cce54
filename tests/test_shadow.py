"""CPU mechanics of 16-bit weight shadows (parallel/shadow.py); numerics are GPU-tested in
test_engine_gpu.py::test_weight_shadow_matches_autocast_casts."""
import torch
import torch.nn as nn

from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.parallel.flat import FlatArena
from distributed_pytorch_training_amd.parallel.shadow import (SHADOW_ATTR, ShadowConv2d, ShadowLinear,
                                                              install_shadows, shadow_param)


def test_install_shadows_resnet_layout_and_fallback():
    torch.manual_seed(0)
    m = build_model("resnet18", 10, torch.device("cpu"), image_size=32, channels_last=True)
    keys = list(m.state_dict().keys())
    x = torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    want = m(x)
    arena = FlatArena(list(reversed(list(m.parameters()))))
    flat, leaves = install_shadows(m, arena, torch.bfloat16)
    assert flat.dtype == torch.bfloat16 and flat.numel() == arena.numel
    convs = [mod for mod in m.modules() if isinstance(mod, nn.Conv2d)]
    assert convs and all(type(c) is ShadowConv2d for c in convs)
    assert type(m.fc) is ShadowLinear
    n_shadowed = sum(len(mod.__dict__.get(SHADOW_ATTR, {})) for mod in m.modules())
    assert n_shadowed == len(leaves) == len(convs) + 2      # every conv weight + fc weight/bias
    for i, leaf in leaves.items():
        p = arena.params[i]
        assert leaf.is_leaf and leaf.requires_grad and leaf.shape == p.shape and leaf.stride() == p.stride()
        assert leaf.data_ptr() == flat.data_ptr() + arena.offsets[i] * 2
        assert torch.equal(leaf, p.detach().to(torch.bfloat16))
    assert list(m.state_dict().keys()) == keys               # masters stay the registered params
    torch.testing.assert_close(m(x), want)                   # CPU / no autocast: fp32 weights


def test_vit_in_proj_shadow_names():
    torch.manual_seed(0)
    m = build_model("vit_b_16", 10, torch.device("cpu"), image_size=32)
    arena = FlatArena(list(m.parameters()))
    _, leaves = install_shadows(m, arena, torch.bfloat16)
    attn = m.encoder.layers[0].self_attention
    assert set(attn.__dict__[SHADOW_ATTR]) == {"in_proj_weight", "in_proj_bias"}
    x = torch.randn(1, 4, 768)
    assert shadow_param(attn, "in_proj_weight", x) is attn.in_proj_weight   # CPU: master
    # LayerNorm / pos_embedding / class_token stay fp32-only
    assert len(leaves) == sum(1 for mod in m.modules() for n in mod.__dict__.get(SHADOW_ATTR, {}))
    assert not hasattr(m.encoder.ln, SHADOW_ATTR)
