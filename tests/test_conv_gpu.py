"""Hand-written MFMA implicit-GEMM convolutions (csrc/kernels/conv_kernels.hip) vs an fp32
PyTorch reference of the same op on the same bf16-rounded operands."""
import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_training_amd import ops

pytestmark = pytest.mark.gpu

CL = torch.channels_last

SHAPES = [
    # N, C, H, W, Cout, k, stride, pad
    (2, 64, 8, 8, 64, 1, 1, 0),
    (3, 64, 7, 7, 128, 1, 1, 0),      # M = 147: partial M tile
    (2, 128, 9, 9, 256, 3, 1, 1),
    (2, 64, 10, 10, 64, 3, 1, 1),
    (2, 256, 14, 14, 128, 1, 2, 0),   # strided 1x1 (downsample)
    (2, 64, 15, 15, 128, 3, 2, 1),    # strided 3x3
    (4, 512, 7, 7, 2048, 1, 1, 0),
    (1, 192, 5, 6, 64, 3, 1, 1),      # non-square image
]


def _operands(cuda, N, C, H, W, Cout, k, seed=0):
    g = torch.Generator(device=cuda).manual_seed(seed)
    x = torch.randn(N, C, H, W, device=cuda, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, C, k, k, device=cuda, generator=g) / (C * k * k) ** 0.5).to(torch.bfloat16)
    return x, w.contiguous(memory_format=CL)


@pytest.fixture(params=[1, 2, 3, 4], ids=["2stage-ldsepi", "2stage-regepi", "1stage-regepi", "1stage-ldsepi"])
def variant(request):
    ops.native().conv_set_variant(request.param)
    yield request.param
    ops.native().conv_set_variant(0)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd_matches_fp32(cuda, variant, shape):
    N, C, H, W, Cout, k, s, p = shape
    x, w = _operands(cuda, N, C, H, W, Cout, k)
    y, ps, pq = ops.native().conv_fwd(x, w, s, p, True)
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=p)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=CL)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    yf = y.float()
    torch.testing.assert_close(ps.sum(1), yf.sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(pq.sum(1), (yf * yf).sum((0, 2, 3)), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[6] == 1])
def test_conv_dgrad_matches_fp32(cuda, shape):
    N, C, H, W, Cout, k, s, p = shape
    x, w = _operands(cuda, N, C, H, W, Cout, k, seed=1)
    Ho, Wo = H + 2 * p - k + 1, W + 2 * p - k + 1
    gy = torch.randn(N, Cout, Ho, Wo, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    dx, wt = ops.native().conv_dgrad(gy, w, p)
    ref = torch.nn.grad.conv2d_input(x.shape, w.float(), gy.float(), stride=1, padding=p)
    torch.testing.assert_close(dx.float(), ref, rtol=1e-2, atol=2e-2)
    assert torch.equal(wt, w.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL))


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("fp32_out", [True, False])
@pytest.mark.parametrize("wvariant", [0, 1], ids=["1stage", "2stage"])
def test_conv_wgrad_matches_fp32(cuda, shape, fp32_out, wvariant):
    ops.native().conv_set_variant(wvariant)
    N, C, H, W, Cout, k, s, p = shape
    x, w = _operands(cuda, N, C, H, W, Cout, k, seed=2)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    gy = torch.randn(N, Cout, Ho, Wo, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    dw = ops.native().conv_wgrad(gy, x, list(w.shape), s, p, fp32_out)
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, gy.float(), stride=s, padding=p)
    assert dw.dtype == (torch.float32 if fp32_out else torch.bfloat16)
    assert dw.is_contiguous(memory_format=CL)
    ops.native().conv_set_variant(0)
    scale = ref.abs().max().item()
    torch.testing.assert_close(dw.float(), ref, rtol=1e-2, atol=1e-3 * scale + 1e-3)


def test_conv_wgrad_large_split(cuda):
    """Many split-K partials (1x1, 64->64 over 56x56: the layer1 shape at a small batch)."""
    x, w = _operands(cuda, 8, 64, 56, 56, 64, 1, seed=3)
    gy = torch.randn(8, 64, 56, 56, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    dw = ops.native().conv_wgrad(gy, x, list(w.shape), 1, 0, True)
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, gy.float())
    torch.testing.assert_close(dw, ref, rtol=1e-3, atol=1e-2)
