"""Fused channels_last BN(+add)(+ReLU) HIP kernels vs the unfused PyTorch fp32 composition."""
import pytest
import torch

from distributed_pytorch_training_amd.models.layers import FusedBatchNorm2d, bn_act
from distributed_pytorch_training_amd.ops.bn import reference_bn_act

pytestmark = pytest.mark.gpu

TOL = {torch.float32: (1e-4, 1e-4), torch.bfloat16: (2e-2, 2e-2), torch.float16: (3e-3, 3e-3)}


def _mk(shape, dtype, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    t = torch.randn(shape, device=dev, generator=g) * 1.7 + 0.3
    return t.to(dtype).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape", [(4, 64, 7, 9), (32, 256, 14, 14), (8, 2048, 7, 7), (2, 8, 3, 3)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False), (False, True)])
def test_fused_bn_train_matches_reference(cuda, dtype, shape, relu, res):
    C = shape[1]
    x = _mk(shape, dtype, cuda, 1).requires_grad_()
    r = _mk(shape, dtype, cuda, 2).requires_grad_() if res else None
    bn = FusedBatchNorm2d(C).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
    ref_rm, ref_rv = bn.running_mean.clone(), bn.running_var.clone()
    w = bn.weight.detach().clone().requires_grad_()
    b = bn.bias.detach().clone().requires_grad_()
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    y = bn_act(bn, x, relu=relu, residual=r)
    zr = reference_bn_act(xr, rr, w, b, ref_rm, ref_rv, True, bn.momentum, bn.eps, False)
    rt, at = TOL[dtype]
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), torch.relu(zr) if relu else zr, rtol=rt, atol=at)
    # Backward oracle through OUR ReLU mask: at z ~ 0 the two roundings of z may disagree on
    # the sign, which flips one gradient element between pass-through and zero (a tie, not
    # an error).
    yr = zr * (y.detach() > 0).float() if relu else zr
    torch.testing.assert_close(bn.running_mean, ref_rm, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref_rv, rtol=1e-4, atol=1e-5)
    assert bn.num_batches_tracked.item() == 1
    gy = _mk(shape, dtype, cuda, 3)
    y.backward(gy)
    # reference backward through the same (rounded) output mask
    yr.backward(gy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=rt * 4, atol=at * 4)
    torch.testing.assert_close(bn.weight.grad, w.grad, rtol=rt * 4, atol=at * 20 * (shape[0] * shape[2] * shape[3]) ** 0.5)
    torch.testing.assert_close(bn.bias.grad, b.grad, rtol=rt * 4, atol=at * 20 * (shape[0] * shape[2] * shape[3]) ** 0.5)
    if res:
        torch.testing.assert_close(r.grad.float(), rr.grad, rtol=rt, atol=at)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_fused_bn_eval(cuda, dtype):
    bn = FusedBatchNorm2d(128).to(cuda).eval()
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = _mk((4, 128, 5, 5), dtype, cuda, 4)
    r = _mk((4, 128, 5, 5), dtype, cuda, 5)
    with torch.no_grad():
        y = bn_act(bn, x, relu=True, residual=r)
        yr = reference_bn_act(x.float(), r.float(), bn.weight, bn.bias, bn.running_mean, bn.running_var,
                              False, 0.1, bn.eps, True)
    rt, at = TOL[dtype]
    torch.testing.assert_close(y.float(), yr, rtol=rt, atol=at)


def test_fused_bn_large_batch_statistics(cuda):
    """ResNet-50 stem-sized reduction (M = 64*112*112): fp64 finalize keeps the variance exact."""
    x = (torch.randn(64, 64, 112, 112, device=cuda) * 0.05 + 3.0).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    bn = FusedBatchNorm2d(64).to(cuda)
    y = bn_act(bn, x, relu=False)
    xf = x.float()
    mean = xf.mean(dim=(0, 2, 3))
    var = xf.var(dim=(0, 2, 3), unbiased=True)
    torch.testing.assert_close(bn.running_mean, 0.1 * mean, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(bn.running_var, 0.9 + 0.1 * var, rtol=1e-4, atol=1e-6)
    yf = y.float()
    assert abs(yf.mean().item()) < 2e-2 and abs(yf.std().item() - 1) < 2e-2


def test_resnet_fused_matches_unfused_step(cuda):
    import copy

    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.models.layers import fuse_batchnorm

    torch.manual_seed(0)
    ref = build_model("resnet50", 100, cuda, image_size=64, channels_last=True)
    fused = copy.deepcopy(ref)
    assert fuse_batchnorm(fused) == 53
    x = torch.randn(8, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        a = ref(x)
        b = fused(x)
    torch.testing.assert_close(b.float(), a.float(), rtol=5e-2, atol=5e-2)
    a.float().sum().backward()
    b.float().sum().backward()
    for (n, p), q in zip(ref.named_parameters(), fused.parameters()):
        scale = p.grad.abs().max().item() + 1e-6
        assert (p.grad - q.grad).abs().max().item() / scale < 0.1, n
    for (n, p), q in zip(ref.named_buffers(), fused.buffers()):
        torch.testing.assert_close(p.float(), q.float(), rtol=1e-2, atol=1e-2, msg=n)
