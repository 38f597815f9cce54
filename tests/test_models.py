"""Model zoo parity with torchvision architectures (param counts/keys/shapes)."""
import pytest
import torch

from distributed_pytorch_training_amd.models import PARAM_COUNTS, build_model, count_params


@pytest.mark.parametrize("key", list(PARAM_COUNTS))
def test_param_counts(key):
    name, classes = key
    assert count_params(build_model(name, classes)) == PARAM_COUNTS[key]


def test_resnet18_keys_and_tensor_count():
    m = build_model("resnet18", 10)
    sd = m.state_dict()
    assert len(list(m.parameters())) == 62
    for k in ["conv1.weight", "bn1.running_mean", "layer1.0.bn1.running_mean", "layer2.0.downsample.0.weight",
              "layer4.1.conv2.weight", "fc.weight", "fc.bias", "bn1.num_batches_tracked"]:
        assert k in sd, k
    assert sum(v.numel() for k, v in sd.items() if "running_" in k) == 9600


def test_resnet50_buffers():
    m = build_model("resnet50", 1000)
    assert len(list(m.parameters())) == 161
    assert sum(b.numel() for n, b in m.named_buffers() if "running_" in n) == 53120


def test_vit_keys_and_forward():
    m = build_model("vit_b_16", 1000)
    sd = m.state_dict()
    for k in ["class_token", "conv_proj.weight", "encoder.pos_embedding",
              "encoder.layers.encoder_layer_11.self_attention.in_proj_weight",
              "encoder.layers.encoder_layer_0.mlp.0.weight", "encoder.layers.encoder_layer_0.mlp.3.bias",
              "encoder.ln.weight", "heads.head.weight"]:
        assert k in sd, k
    assert len(list(m.buffers())) == 0
    m.eval()
    with torch.no_grad():
        assert m(torch.randn(1, 3, 224, 224)).shape == (1, 1000)


def test_vit_attention_matches_nn_multihead():
    from distributed_pytorch_training_amd.models.vit import SelfAttention

    torch.manual_seed(0)
    ours = SelfAttention(64, 4)
    ref = torch.nn.MultiheadAttention(64, 4, batch_first=True)
    ref.load_state_dict(ours.state_dict())
    x = torch.randn(2, 7, 64)
    torch.testing.assert_close(ours(x), ref(x, x, x, need_weights=False)[0], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name,size,classes", [("resnet18", 32, 10), ("resnet50", 64, 1000)])
def test_forward_backward_channels_last(name, size, classes):
    m = build_model(name, classes, channels_last=True)
    x = torch.randn(2, 3, size, size).contiguous(memory_format=torch.channels_last)
    y = m(x)
    assert y.shape == (2, classes)
    y.sum().backward()
    assert all(p.grad is not None for p in m.parameters())
