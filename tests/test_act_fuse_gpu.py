"""conv(relu(bn(x))) as one op (ops/conv.py ``_BNReLUConv``; conv_kernels.hip ACT).

The fused op applies the BatchNorm+ReLU to the conv's staged input instead of running the BN's
forward apply pass, and stores the activation once for the backward-weight.  It must be
bit-identical to the unfused composition (``FusedBatchNorm2d`` relu apply -> native conv): the
same fp32 fma / clamp / round-to-nearest-even of every activation element and the same MFMA
summation order, so the conv output, its BatchNorm partials, the stored activation, every input
gradient and the running statistics agree exactly.  Shapes: 1x1 and 3x3 / stride 1 (the fused
kernel, both output-tile widths, several output-channel tiles so only tile 0 writes the
activation), plus shapes that take the op's fallback (stride 2; a grid small enough to split K).
The whole ResNet-50 step with the fusion on and off is compared too.  Against fp32 PyTorch:
``F.batch_norm -> relu -> conv2d``.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_training_amd.models.layers import FusedBatchNorm2d, bn_act
from distributed_pytorch_training_amd.ops import conv as native_conv

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def _mk(shape, dtype, dev, seed, scale=1.0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.randn(shape, device=dev, generator=g) * scale).to(dtype).contiguous(memory_format=CL)


def _bn(C, dev, seed):
    bn = FusedBatchNorm2d(C).to(dev)
    g = torch.Generator(device="cpu").manual_seed(seed)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.rand(C, generator=g) - 0.5)
        bn.running_mean.copy_(torch.rand(C, generator=g) * 0.2 - 0.1)
    return bn


CASES = [  # (N, C, H, W, Cout, k, stride, pad)
    (8, 64, 14, 14, 256, 1, 1, 0),     # 1x1, 128-wide tiles, two output-channel tiles
    (8, 128, 14, 14, 64, 1, 1, 0),     # 1x1, 64-wide tile, two K-steps
    (8, 64, 14, 14, 64, 3, 1, 1),      # 3x3 HALO, 64-wide tile
    (4, 128, 28, 28, 128, 3, 1, 1),    # 3x3 HALO, 128-wide tile, several m-tiles
    (8, 64, 28, 28, 512, 1, 1, 0),     # 1x1, four output-channel tiles
    (8, 64, 14, 14, 64, 3, 2, 1),      # stride 2: fallback (apply pass + plain conv)
    (2, 512, 4, 4, 512, 3, 1, 1),      # tiny grid: split-K fallback
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES, ids=[f"{c[1]}x{c[2]}->{c[4]}k{c[5]}s{c[6]}" for c in CASES])
def test_fused_op_is_bitwise_the_unfused_pair(cuda, monkeypatch, dtype, case):
    N, C, H, W, Co, k, s, p = case
    monkeypatch.setattr(native_conv, "ACT_FUSE", True)
    x0 = _mk((N, C, H, W), dtype, cuda, 1, 1.5)
    w0 = _mk((Co, C, k, k), dtype, cuda, 2, 0.05)
    g0 = _mk((N, Co, (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1), dtype, cuda, 3)
    outs = {}
    for mode in ("fused", "unfused"):
        bn = _bn(C, cuda, 4)
        x = x0.clone().requires_grad_()
        w = w0.clone().requires_grad_()
        assert native_conv.act_supported(x, w, (s, s), (p, p), (1, 1), 1)
        if mode == "fused":
            y = native_conv.bn_relu_conv2d(x, bn, w, s, p, bn_stats=True)
        else:
            y = native_conv.conv2d(bn_act(bn, x), w, s, p, bn_stats=True)
        ps, pq = y._dpt_bn_partials
        y.backward(g0)
        torch.cuda.synchronize()
        outs[mode] = dict(y=y.detach(), ps=ps, pq=pq, dx=x.grad, dw=w.grad, dg=bn.weight.grad, db=bn.bias.grad,
                          rm=bn.running_mean.detach().clone(), rv=bn.running_var.detach().clone(),
                          nb=bn.num_batches_tracked.clone())
    a, b = outs["fused"], outs["unfused"]
    for key in a:
        assert torch.equal(a[key], b[key]), (key, (a[key].float() - b[key].float()).abs().max().item())


@pytest.mark.parametrize("case", CASES[:4], ids=[f"{c[1]}x{c[2]}->{c[4]}k{c[5]}" for c in CASES[:4]])
def test_fused_op_matches_fp32_torch(cuda, monkeypatch, case):
    N, C, H, W, Co, k, s, p = case
    monkeypatch.setattr(native_conv, "ACT_FUSE", True)
    x = _mk((N, C, H, W), torch.bfloat16, cuda, 1, 1.5).requires_grad_()
    w = _mk((Co, C, k, k), torch.bfloat16, cuda, 2, 0.05).requires_grad_()
    bn = _bn(C, cuda, 4)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    gw, gb = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    y = native_conv.bn_relu_conv2d(x, bn, w, s, p)
    yr = F.conv2d(torch.relu(F.batch_norm(xr, rm, rv, gw, gb, True, bn.momentum, bn.eps)), wr, None, s, p)
    torch.testing.assert_close(y.float(), yr, rtol=3e-2, atol=3e-2)
    g = torch.randn_like(yr)
    y.backward(g.to(y.dtype).contiguous(memory_format=CL))
    yr.backward(g)
    for got, want, tol in ((x.grad, xr.grad, 6e-2), (w.grad, wr.grad, 6e-2), (bn.weight.grad, gw.grad, 6e-2),
                           (bn.bias.grad, gb.grad, 6e-2)):
        err = ((got.float() - want).norm() / want.norm().clamp_min(1e-12)).item()
        assert err < tol, err
    torch.testing.assert_close(bn.running_mean, rm, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, rv, rtol=1e-4, atol=1e-5)


def test_resnet50_step_identical_with_and_without_fusion(cuda, monkeypatch):
    """Two native ResNet-50 training steps (bf16, 64 px, batch 16) from the same weights: with the
    fused op (every bottleneck's bn1 -> conv2 and bn2 -> conv3) and without, bit-identical
    parameters, BN buffers and loss."""
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model

    torch.manual_seed(0)
    base = build_model("resnet50", 100, cuda, image_size=64, channels_last=True)
    args = parse_args(["--model", "resnet50", "--dataset", "synthetic", "--amp", "--amp-dtype", "bf16",
                       "--channels-last", "--no-cuda-graph", "--image-size", "64", "--num-classes", "100"])
    g = torch.Generator(device=cuda).manual_seed(7)
    batches = [(torch.randn(16, 3, 64, 64, device=cuda, generator=g).contiguous(memory_format=CL),
                torch.randint(0, 100, (16,), device=cuda, generator=g)) for _ in range(2)]
    res = {}
    for on in (True, False):
        monkeypatch.setattr(native_conv, "ACT_FUSE", on)
        tr = Trainer(copy.deepcopy(base), args, 0, 1, cuda, log=lambda s: None)
        calls = []
        if on:
            real = native_conv._BNReLUConv.apply
            monkeypatch.setattr(native_conv._BNReLUConv, "apply", lambda *a: calls.append(1) or real(*a))
        losses = [tr.train_step(x, y)[1].detach().clone() for x, y in batches]
        torch.cuda.synchronize()
        if on:
            assert len(calls) == 2 * 32, len(calls)      # 16 bottlenecks x (bn1->conv2, bn2->conv3) x 2 steps
        res[on] = (tr.ddp.arena.param_flat.clone(), [b.clone() for b in tr.module.buffers()], losses)
        monkeypatch.undo()
    assert torch.equal(res[True][0], res[False][0])
    assert all(torch.equal(a, b) for a, b in zip(res[True][1], res[False][1]))
    assert all(torch.equal(a, b) for a, b in zip(res[True][2], res[False][2]))
